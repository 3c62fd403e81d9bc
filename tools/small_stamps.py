"""Dev aid: phase stamps (shader cycles) of eig_small_kernel for replicate 0
of a C3 factored bootstrap, uncontended (B=1) and in a full batch.
Run with DFM_SMALL_STAMPS=1."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import dfm_pkg
D = dfm_pkg.load()
T, N, R = 500, 2000, 8
y, x, *_ = D.factor_model_DGP(T, N, R, rng=np.random.default_rng(20261015 + 3))
x = D.normalize(x)
g = D.DynamicFactorModel(y, np.ones((T, 1)), x, R, "ICp2")
for B in (1, int(sys.argv[1]) if len(sys.argv) > 1 else 2000):
    idx, eta = D.draw_wild_fast(5, B, T)
    print(f"--- B={B}", file=sys.stderr, flush=True)
    D.wild_bootstrap(g, B, [D.Stat.V()], idx=idx, eta=eta)
