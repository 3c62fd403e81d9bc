"""C3 convergence probe: iterations per replicate vs the eigenvalue stopping
tolerance, and vs the block width p (values-only rule)."""
import sys, time
import numpy as np
sys.path.insert(0, "."); sys.path.insert(0, "oracle")
import torch
torch.cuda.init()
import dfm_pkg
D = dfm_pkg.load()
T, N, R = 500, 2000, 8
rng = np.random.default_rng(20261015 + 3)
y, x, *_ = D.factor_model_DGP(T, N, R, rng=rng)
x = D.normalize(x)
B = 2000
idx, eta = D.draw_wild_fast(7, B, T)
for block in [0, 12, 20, 24]:
    for vt in [1e-12, 1e-10, 1e-8]:
        ctx = D.Context(0)
        ctx.set_value_tol(vt)
        if block:
            ctx.set_eig_params(block=block)
        m = D.DynamicFactorModel(y, np.ones((T, 1)), x, R, "ICp2", ctx=ctx)
        out = D.wild_bootstrap(m, B, [D.Stat.V(), D.Stat.criterion()], idx=idx, eta=eta)
        t0 = time.perf_counter()
        out = D.wild_bootstrap(m, B, [D.Stat.V(), D.Stat.criterion()], idx=idx, eta=eta)
        dt = time.perf_counter() - t0
        it = ctx.eig_stats() if hasattr(ctx, "eig_stats") else None
        print(f"block={block or 16} value_tol={vt:g}: {B/dt:9.0f} rep/s  iters={it}  V[0]={out[0,0]:.15e}", flush=True)
