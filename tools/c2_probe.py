import sys, time, numpy as np
sys.path.insert(0, '/root/repo')
import torch; torch.cuda.init()
import dfm_pkg
D = dfm_pkg.load()
ctx = D.Context(0)
rng = np.random.default_rng(20261015 + 2)
T, N, B, bp = 600, 130, 999, 300
y, x, *_ = D.factor_model_DGP(T, N, 3, model="Breitung_Eickmeier_2011", b=0.5, rng=rng)
x = D.normalize(x); w = np.ones((T, 1))
m = D.DynamicFactorModel(y, w, x, "ICp2", kmax=8, ctx=ctx)
print("r", m.number_of_factors, "eig", m.eigenvalues[:8])
S = D.Stat
idx, eta = D.draw_wild_fast(7, B, T)
for blk in [16, 20, 24, 32]:
    ctx.set_eig_params(block=blk); ctx.reset_timing()
    for rep in range(2):
        t0 = time.perf_counter()
        out = D.wild_bootstrap(m, B, [S.V(), S.LR_all(bp), S.LM_all(bp), S.Wald_all(bp)], idx=idx, eta=eta)
        el = time.perf_counter() - t0
    st = ctx.eig_stats()
    print(f"block {blk}: {el*1e3:.1f} ms (host incl.), iters/batch {st['iterations']/max(1,st['batches']):.1f} rep-iters/rep {st['replicate_iterations']/B/2:.1f}")
