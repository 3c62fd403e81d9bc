"""C2: per-replicate Rayleigh-Ritz step counts of the direct eigensolver
(Stat.iterations) — how long the straggler tail of a 999-replicate job is."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import dfm_pkg
D = dfm_pkg.load()
rng = np.random.default_rng(20261015 + 2)
T, N, B, bp = 600, 130, 999, 300
y, x, *_ = D.factor_model_DGP(T, N, 3, model="Breitung_Eickmeier_2011", b=0.5, rng=rng)
x = D.normalize(x)
w = np.ones((T, 1))
model = D.DynamicFactorModel(y, w, x, "ICp2", kmax=8)
idx, eta = D.draw_wild_fast(7, B, T)
S = D.Stat
out = D.wild_bootstrap(model, B, [S.iterations(), S.LR(bp, 1)], idx=idx, eta=eta)
it = out[:, 0].astype(int)
print("r", model.number_of_factors, "iterations histogram", dict(zip(*np.unique(it, return_counts=True))))
out2 = D.wild_bootstrap(model, B, [S.iterations(), S.V()], idx=idx, eta=eta)
it2 = out2[:, 0].astype(int)
print("value-only stats:", dict(zip(*np.unique(it2, return_counts=True))))
