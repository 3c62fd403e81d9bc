"""C2 eigen-phase A/B: the batched subspace solver (default block p = 16) vs the
dense batched top-k path (tridiagonalisation + bisection + inverse iteration,
forced with block > 32), same draws; prints per-job ms, the kernel split and
the max relative difference of the statistic rows."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import dfm_pkg
D = dfm_pkg.load()
rng = np.random.default_rng(20261015 + 2)
T, N, B, bp = 600, 130, 999, 300
y, x, *_ = D.factor_model_DGP(T, N, 3, model="Breitung_Eickmeier_2011", b=0.5, rng=rng)
x = D.normalize(x)
w = np.ones((T, 1))
res = {}
for block in (0, 64):
    ctx = D.Context(0)
    if block:
        ctx.set_eig_params(block=block)
    model = D.DynamicFactorModel(y, w, x, "ICp2", kmax=8, ctx=ctx)
    S = D.Stat
    stats = [S.V(), S.criterion(), S.LR_all(bp), S.LM_all(bp), S.Wald_all(bp)]
    arr = D.api._stat_array(stats)
    width = int(ctx.lib.dfm_stats_width(model.handle, arr, len(stats)))
    idx, eta = D.draw_wild_fast(7, B, T)
    dev = torch.device("cuda", 0)
    di, de = torch.from_numpy(idx).to(dev), torch.from_numpy(eta).to(dev)
    out = torch.empty((B, width), dtype=torch.float64, device=dev)
    run = lambda: ctx.check(ctx.lib.dfm_bootstrap_dev(model.handle, 0, B, di.data_ptr(), de.data_ptr(), arr,
                                                      len(stats), out.data_ptr()))
    run(); ctx.synchronize()
    ctx.reset_timing(); ctx.enable_timing(True)
    t0 = time.perf_counter()
    for _ in range(5):
        run()
    ctx.synchronize()
    ms = (time.perf_counter() - t0) / 5 * 1e3
    ctx.enable_timing(False)
    tm = ctx.read_timing()
    res[block] = out.cpu().numpy()
    print(f"block {block}: {ms:.3f} ms/job", {k: round(v[0] / 5, 3) for k, v in tm.items() if v[1]}, flush=True)
a, b = res[0], res[64]
print("max rel diff", float(np.max(np.abs(a - b) / np.maximum(np.abs(a), 1e-300))))
