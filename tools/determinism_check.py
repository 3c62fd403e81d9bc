#!/usr/bin/env python3
"""Run-to-run bit reproducibility of the dense-spectrum path (tridiag_kernel +
bisection + inverse iteration + back-transform): the same principal_components
call repeated in one process must return identical bits."""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dfm_pkg  # noqa: E402

D = dfm_pkg.load()
ctx = D.Context(0)
for T, N, k in [(300, 180, 60), (150, 500, 60), (900, 1100, 40)]:
    x = np.random.default_rng(T + N).standard_normal((T, N))
    hs = set()
    for _ in range(4):
        ev, F, L, tr = D.principal_components(x, k, ctx=ctx)
        hs.add(hashlib.sha1(np.concatenate([ev, F.ravel(), L.ravel()]).tobytes()).hexdigest()[:16])
    print(f"T={T} N={N} k={k} distinct_digests={len(hs)}", flush=True)
