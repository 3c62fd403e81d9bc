"""Explicit-Gram eigensolver (eig_run) time vs Gram size m: dfm_pca on N > T
panels of T = m rows (3 strong factors), per-kernel-class HIP-event times."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import dfm_pkg
D = dfm_pkg.load()
ctx = D.default_context()
for T in [int(a) for a in sys.argv[1:]] or [512, 1024, 2048, 3072, 4000]:
    N = T + 100
    rng = np.random.default_rng(T)
    f = rng.standard_normal((T, 3))
    x = f @ rng.standard_normal((3, N)) * 2.0 + rng.standard_normal((T, N))
    ctx.reset_timing(); ctx.enable_timing(True)
    t0 = time.perf_counter()
    ev, F, L, tr = D.principal_components(x, 3)
    el = time.perf_counter() - t0
    ctx.enable_timing(False)
    tm = {k: (round(v[0], 2), v[1]) for k, v in ctx.read_timing().items() if v[1]}
    print("T", T, "pca s", round(el, 3), tm, ctx.eig_stats(), flush=True)
