"""C4 soft-threshold timing with the lasso leaders' phase profile
(DFM_LASSO_PROF=1 prints per-problem phase times to stderr)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
import numpy as np
import dfm_pkg
import make_golden
D = dfm_pkg.load()
y, w, x, folds = make_golden.c4_inputs()
ctx = D.Context(0)
for rep in range(3):
    t0 = time.perf_counter()
    m = D.targeted_predictors(y, w, x, "soft", folds=folds, ctx=ctx)
    print(f"soft {1e3 * (time.perf_counter() - t0):.1f} ms, selected {int(m.sum())}", flush=True)
