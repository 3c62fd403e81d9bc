"""Eigensolver convergence probe (development): replicate-iterations of the
factored C3 bootstrap (T=500 N=2000 r=8, B=4000) against the eigenvalue
(Kato-Temple) tolerance and the strict eigenvector-residual tolerance.

    python tools/conv_probe.py          # on a GPU box
"""
import sys, time, numpy as np
sys.path.insert(0, '/root/repo')
import torch; torch.cuda.init()
import dfm_pkg
D = dfm_pkg.load()
ctx = D.Context(0)
T, N, R, B = 500, 2000, 8, 4000
rng = np.random.default_rng(20261015 + 3)
y, x, *_ = D.factor_model_DGP(T, N, R, rng=rng)
x = D.normalize(x); w = np.ones((T, 1))
m = D.DynamicFactorModel(y, w, x, R, "ICp2", ctx=ctx)
print("eig", m.eigenvalues[:R], "trace", m.trace_G)
idx, eta = D.draw_wild_fast(5, B, T)
for tol in [1e-6, 1e-8, 1e-10, 1e-12, 1e-14]:
    ctx.set_value_tol(tol); ctx.reset_timing()
    t0 = time.time(); out = D.wild_bootstrap(m, B, [D.Stat.V(), D.Stat.eigenvalue(8)], idx=idx, eta=eta); el = time.time() - t0
    st = ctx.eig_stats()
    print(f"value tol {tol:g}: rep-iters/rep {st['replicate_iterations']/B:.2f} max {st['max_iterations']} time {el:.3f}s  ev8 med {np.median(out[:,1]):.6g}")
ctx.set_value_tol(0.0)
for tol in [1e-12, 1e-10, 1e-8]:
    ctx.set_eig_params(tol=tol); ctx.reset_timing()
    out = D.wild_bootstrap(m, B, [D.Stat.V()], idx=idx, eta=eta)
    st = ctx.eig_stats()
    print(f"strict residual tol {tol:g}: rep-iters/rep {st['replicate_iterations']/B:.2f} max {st['max_iterations']}")
