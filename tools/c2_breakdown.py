"""C2 (T=600 N=130, B=999, Chow all variables) per-kernel-class breakdown."""
import sys
import numpy as np
sys.path.insert(0, ".")
import torch
torch.cuda.init()
import dfm_pkg
D = dfm_pkg.load()
sys.argv += []
ctx = D.Context(0)
rng = np.random.default_rng(20261015 + 2)
T, N, B, bp = 600, 130, 999, 300
y, x, *_ = D.factor_model_DGP(T, N, 3, model="Breitung_Eickmeier_2011", b=0.5, rng=rng)
x = D.normalize(x)
w = np.ones((T, 1))
model = D.DynamicFactorModel(y, w, x, "ICp2", kmax=8, ctx=ctx)
S = D.Stat
for name, stats in [("V+ICp2", [S.V(), S.criterion()]),
                    ("V+ICp2+Chow", [S.V(), S.criterion(), S.LR_all(bp), S.LM_all(bp), S.Wald_all(bp)])]:
    idx, eta = D.draw_wild_fast(7, B, T)
    D.wild_bootstrap(model, B, stats, idx=idx, eta=eta)
    ctx.enable_timing(True)
    ctx.reset_timing() if hasattr(ctx, "reset_timing") else None
    import time
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        D.wild_bootstrap(model, B, stats, idx=idx, eta=eta)
    dt = (time.perf_counter() - t0) / 3
    tm = ctx.read_timing() if hasattr(ctx, "read_timing") else None
    ctx.enable_timing(False)
    print(name, f"r={model.number_of_factors} {B/dt:.0f} rep/s ({dt*1e3:.2f} ms incl. host copies)", tm, ctx.eig_stats(),
          flush=True)
