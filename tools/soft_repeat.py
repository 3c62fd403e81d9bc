"""Repeat the soft-threshold selection of tests/test_gpu_soft.py's first
oracle case (T=200, N=40, q=2: p = 42, one helper per problem) in one process
and report each call's wall time and the lasso launch record
(``lasso_stats``: every timed-out leader/helper spin, relaunches, the
workgroups' entry spread); the library describes each timeout on stderr."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import dfm_pkg  # noqa: E402
import dfm_oracle as O  # noqa: E402
from test_gpu_parity import panel  # noqa: E402

D = dfm_pkg.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
T, N = 200, 40
y, x, w = panel(O, T, N, 3, 70 + T)
w = np.hstack([w, np.r_[0.0, y[:-1]][:, None]])
folds = O.glmnet_default_folds(T, np.random.default_rng(T))
ref = None
times = []
D.lasso_stats(reset=True)
last = D.lasso_stats()
for i in range(n):
    t0 = time.perf_counter()
    mask, path = D.targeted_predictors(y, w, x, "soft", folds=folds, nlambda=100, return_path=True)
    times.append(time.perf_counter() - t0)
    st = D.lasso_stats()
    if i < 3 or i % 50 == 0 or times[-1] > 0.1 or st["timeouts"] != last["timeouts"]:
        print(f"call {i}: {times[-1] * 1e3:.1f} ms  timeouts {st['timeouts']} relaunches {st['relaunches']}",
              flush=True)
    last = st
    if ref is None:
        ref = mask.copy()
    assert np.array_equal(mask, ref)
print(f"{n} calls: median {np.median(times) * 1e3:.1f} ms, max {max(times) * 1e3:.1f} ms "
      f"(max after call 0: {max(times[1:] or [0]) * 1e3:.1f} ms)")
print("lasso_stats", D.lasso_stats())
