"""Timings of the any-r / full-spectrum paths (single fits) on the GPU."""
import sys, time, math
import numpy as np
sys.path.insert(0, ".")
import torch
torch.cuda.init()
import dfm_pkg
dfm = dfm_pkg.load()
sys.path.insert(0, "oracle")
import dfm_oracle as O

def panel(T, N, r, seed):
    rng = np.random.default_rng(seed)
    y, x, *_ = O.factor_model_DGP(T, N, r, rng)
    return y, O.normalize(x), np.ones((T, 1))

def tm(f, reps=3):
    f()
    t0 = time.perf_counter()
    for _ in range(reps): f()
    return (time.perf_counter() - t0) / reps

for (T, N) in [(200, 100), (200, 130), (500, 2000), (2000, 1500), (1000, 3000)]:
    y, x, w = panel(T, N, 8, 1)
    m = min(T, N)
    t_def = tm(lambda: dfm.DynamicFactorModel(y, w, x))
    t_pcp = tm(lambda: dfm.DynamicFactorModel(y, w, x, 8, "PCp2"))
    t_spec = tm(lambda: dfm.gram_spectrum(x))
    print(f"T={T} N={N} m={m}: default r={math.ceil(m/2)} fit {t_def*1e3:.1f} ms | PCp2 r=8 fit {t_pcp*1e3:.1f} ms | "
          f"gram_spectrum {t_spec*1e3:.1f} ms", flush=True)
