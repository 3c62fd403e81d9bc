"""The C4 full-fit lasso path alone (one problem: 1 leader + up to 64
helpers) vs inside glmnetcv (11 concurrent problems): separates the helpers'
per-task latency from the chip-wide bandwidth the 11 problems share.
Run with DFM_LASSO_PROF=1 for the leader's phase split."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
import numpy as np
import dfm_pkg
import make_golden
import dfm_oracle as O
D = dfm_pkg.load()
y, w, x, folds = make_golden.c4_inputs()
Z = np.hstack([w, x])
mu, sd, ju, yb, ys, G, c = O._glmnet_standardize(Z, y)
lam_max = float(np.max(np.abs(c[ju])))
alms = O.glmnet_lambdas(lam_max, 100, 0.01 if Z.shape[0] < Z.shape[1] else 1e-4)
ctx = D.Context(0)
for rep in range(3):
    t0 = time.perf_counter()
    b, r = D.lasso_path(G, c, ju, alms, early=True, ctx=ctx)
    print(f"single problem: {1e3 * (time.perf_counter() - t0):.1f} ms, L {len(r)}, |A| {int((b[-1] != 0).sum())}",
          flush=True)
