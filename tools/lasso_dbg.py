import sys, os
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/oracle')
import numpy as np
import dfm_pkg, dfm_oracle as O
D = dfm_pkg.load()
rng = np.random.default_rng(1)
y, x, *_ = O.factor_model_DGP(80, 40, 3, rng)
x = O.normalize(x); w = np.ones((80, 1))
mu, sd, ju, yb, ys, G, c = O._glmnet_standardize(np.hstack([w, x]), y)
alms = O.glmnet_lambdas(float(np.max(np.abs(c[ju]))), 5, 1e-2)
try:
    b, r = D.lasso_path(G, c, ju, alms)
    print("ok", b.shape)
except Exception as e:
    print("ERR", e)
