"""C5 (T=2000 N=20000, 200 windows, kmax 8) per-kernel-class breakdown."""
import sys, time
import numpy as np
sys.path.insert(0, ".")
import torch
torch.cuda.init()
import dfm_pkg
D = dfm_pkg.load()
ctx = D.Context(0)
rng = np.random.default_rng(20261015 + 5)
T, N, P = 2000, 20000, 200
y, x, *_ = D.factor_model_DGP(T, N, 8, rng=rng)
x = np.asfortranarray(D.normalize(x))
w = np.ones((T, 1))
D.pseudo_out_of_sample_refits(y, w, x, "ICp2", num_predictions=P, kmax=8, ctx=ctx)
ctx.enable_timing(True)
ctx.reset_timing()
t0 = time.perf_counter()
out = D.pseudo_out_of_sample_refits(y, w, x, "ICp2", num_predictions=P, kmax=8, ctx=ctx)
dt = time.perf_counter() - t0
print(f"{dt*1e3:.1f} ms total", {k: (round(v[0], 2), v[1]) for k, v in ctx.read_timing().items() if v[1]},
      ctx.eig_stats(), flush=True)
xc = np.asfortranarray(x)
t0 = time.perf_counter(); xt = torch.from_numpy(xc.ravel(order="F")).to("cuda"); torch.cuda.synchronize()
print(f"H2D of the panel alone: {(time.perf_counter()-t0)*1e3:.1f} ms ({x.nbytes/1e6:.0f} MB)")
