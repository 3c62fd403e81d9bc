"""Diagnostic (variant library built with -DDFM_DIAG_X, loaded through
DFM_LIB_PATH): for one C3 bootstrap job (the bench's model and draws), how far
each replicate's eigenvalue-bound convergence test is from passing at
Rayleigh-Ritz steps 1..4 (x <= 1 passes).  Under the current schedule
(degree-2 Chebyshev filter between Rayleigh-Ritz steps) a degree-3 first filter
would divide step 3's excess by (T3/T2)^2 ~ 574, two degree-3 filters by ~3.3e5."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dfm_pkg  # noqa: E402

D = dfm_pkg.load()
ctx = D.Context(0)
T, N, R, B = 500, 2000, 8, int(os.environ.get("B", "9999"))
rng = np.random.default_rng(20261015 + 3)
y, x, *_ = D.factor_model_DGP(T, N, R, rng=rng)
x = D.normalize(x)
m = D.DynamicFactorModel(y, np.ones((T, 1)), x, R, "ICp2", ctx=ctx)
idx, eta = D.draw_wild_fast(1_000_003, B, T)
st = D.wild_bootstrap(m, B, [D.Stat.V(), D.Stat.criterion(), D.Stat.iterations()], idx=idx, eta=eta)
out = np.zeros((4, 16384))
ctx.lib.dfm_diag_read_x.argtypes = [C.c_void_p]
assert ctx.lib.dfm_diag_read_x(out.ctypes.data) == 0
it = st[:, 2]
print("iterations histogram", {int(k): int(v) for k, v in zip(*np.unique(it, return_counts=True))})
for s in range(4):
    xs = out[s, :B]
    q = np.quantile(xs, [0.0, 0.1, 0.5, 0.9, 0.99, 1.0])
    print(f"RR step {s + 1}: excess quantiles 0/10/50/90/99/100% = " + " ".join(f"{v:.3g}" for v in q))
x3 = out[2, :B]
for f in (1.0, 574.0, 574.0 ** 2, 8.2e4):
    print(f"step 3 excess <= {f:.3g}: {np.mean(x3 <= f) * 100:.2f}% of replicates")
