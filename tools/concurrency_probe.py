"""Development probe: does running two replicate halves concurrently (two
contexts = two HIP streams, two host threads) beat one full-size call?
C3 shape (T=500 N=2000 r=8), B = 9999, stats V + ICp2.
    python tools/concurrency_probe.py     # on a GPU box
"""
import sys, time, threading
import numpy as np
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch
torch.cuda.init()
import dfm_pkg
D = dfm_pkg.load()
T, N, R, B = 500, 2000, 8, 9999
rng = np.random.default_rng(20261015 + 3)
y, x, *_ = D.factor_model_DGP(T, N, R, rng=rng)
x = D.normalize(x); w = np.ones((T, 1))
ctxs = [D.Context(0), D.Context(0)]
models = [D.DynamicFactorModel(y, w, x, R, "ICp2", ctx=c) for c in ctxs]
stats = [D.Stat.V(), D.Stat.criterion()]
arr = D.api._stat_array(stats)
idx, eta = D.draw_wild_fast(3, B, T)
dev = torch.device("cuda", 0)
di, de = torch.from_numpy(idx).to(dev), torch.from_numpy(eta).to(dev)
out = torch.empty((B, 2), dtype=torch.float64, device=dev)
torch.cuda.synchronize()
h = B // 2

def run(k, b0, n):
    c = ctxs[k]
    c.check(c.lib.dfm_bootstrap_dev(models[k].handle, 0, n, di.data_ptr() + b0 * T * 4,
                                    de.data_ptr() + b0 * T * 8, arr, 2, out.data_ptr() + b0 * 16))
    c.synchronize()

for rep in range(3):
    t0 = time.perf_counter(); run(0, 0, B); t1 = time.perf_counter()
    ref = out.cpu().numpy().copy()
    t2 = time.perf_counter(); run(0, 0, h); run(0, h, B - h); t3 = time.perf_counter()
    th = [threading.Thread(target=run, args=(0, 0, h)), threading.Thread(target=run, args=(1, h, B - h))]
    t4 = time.perf_counter()
    for t in th: t.start()
    for t in th: t.join()
    t5 = time.perf_counter()
    same = np.array_equal(out.cpu().numpy(), ref)
    print(f"full {1e3*(t1-t0):.1f} ms | halves sequential {1e3*(t3-t2):.1f} ms | halves concurrent {1e3*(t5-t4):.1f} ms | identical {same}", flush=True)
