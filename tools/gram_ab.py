#!/usr/bin/env python3
"""A/B of the plain-panel Gram kernels (DFM_GRAM_DMA=1: LDS-DMA SYRK,
DFM_GRAM_DMA=0: register-staged gram_kernel): digests of dfm_pca outputs at
shapes covering m % 64 != 0, K % 16 != 0 and split-K, plus the eigenvalue error
against numpy, and the C5 prefix-Gram launch time.  Run once per setting."""
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dfm_pkg  # noqa: E402

D = dfm_pkg.load()
ctx = D.Context(0)
mode = os.environ.get("DFM_GRAM_DMA", "1")
for (T, N) in [(64, 300), (65, 301), (300, 5000), (1000, 4100), (257, 9001), (2000, 20000)]:
    x = np.random.default_rng(T * 7 + N).standard_normal((T, N))
    ctx.reset_timing()
    ctx.enable_timing(True)
    ev, F, L, tr = D.principal_components(x, 4, ctx=ctx)
    t0 = time.perf_counter()
    ev, F, L, tr = D.principal_components(x, 4, ctx=ctx)
    el = time.perf_counter() - t0
    ctx.enable_timing(False)
    tm = ctx.read_timing().get("gram", (0.0, 0))
    h = hashlib.sha1(np.concatenate([ev, F.ravel(), L.ravel(), [tr]]).tobytes()).hexdigest()[:16]
    if T * N <= 4_000_000:
        g = x @ x.T
        ref = np.sort(np.linalg.eigvalsh(g))[::-1][:4]
        err = float(np.max(np.abs(ev - ref) / ref))
        terr = abs(tr - np.trace(g)) / np.trace(g)
    else:
        err = terr = float("nan")
    print(f"DMA={mode} T={T} N={N} digest={h} ev_rel_err={err:.2e} tr_rel_err={terr:.2e} "
          f"gram_ms={tm[0] / max(tm[1], 1):.3f} pca_ms={el * 1e3:.1f}", flush=True)
