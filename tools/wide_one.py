"""One default-constructor fit (r = ceil(m/2)) for kernel profiling."""
import sys
import numpy as np
sys.path.insert(0, "."); sys.path.insert(0, "oracle")
import torch
torch.cuda.init()
import dfm_pkg
import dfm_oracle as O
dfm = dfm_pkg.load()
T, N = int(sys.argv[1]), int(sys.argv[2])
rng = np.random.default_rng(1)
y, x, *_ = O.factor_model_DGP(T, N, 8, rng)
x = O.normalize(x)
d = dfm.DynamicFactorModel(y, np.ones((T, 1)), x)
print("r =", d.number_of_factors, "V =", d.V)
