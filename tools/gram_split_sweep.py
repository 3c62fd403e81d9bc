#!/usr/bin/env python3
"""Time the C5 prefix Gram (T=2000, N=20000, plain row-major panel) at one
split-K setting (DFM_GRAM_SPLIT=S in the environment); 5 timed launches."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dfm_pkg  # noqa: E402

D = dfm_pkg.load()
ctx = D.Context(0)
T, N = int(os.environ.get("GS_T", 2000)), int(os.environ.get("GS_N", 20000))
x = np.random.default_rng(5).standard_normal((T, N))
ev, tr = None, None
D.principal_components(x, 2, ctx=ctx)
ctx.reset_timing()
ctx.enable_timing(True)
for _ in range(5):
    D.principal_components(x, 2, ctx=ctx)
ctx.enable_timing(False)
ms, n = ctx.read_timing().get("gram", (0.0, 0))
per = ms / max(n, 1)
print(f"S={os.environ.get('DFM_GRAM_SPLIT', 'auto')} T={T} N={N} gram_ms={per:.3f} "
      f"TF/s={T * (T + 1) * N / per / 1e9:.1f}", flush=True)
