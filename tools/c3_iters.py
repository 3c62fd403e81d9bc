"""C3: per-replicate Rayleigh-Ritz step counts of the factored eigensolver
(Stat.iterations), eigenvalue-only stats (the bench's V + ICp2: Kato-Temple
rule) and with a coefficient stat (strict eigenvector rule)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import dfm_pkg
D = dfm_pkg.load()
rng = np.random.default_rng(20261015 + 3)
T, N, B = 500, 2000, int(sys.argv[1]) if len(sys.argv) > 1 else 2000
y, x, *_ = D.factor_model_DGP(T, N, 8, rng=rng)
x = D.normalize(x)
w = np.ones((T, 1))
model = D.DynamicFactorModel(y, w, x, 8, "ICp2")
idx, eta = D.draw_wild_fast(1_000_003, B, T)
S = D.Stat
ctx = model._ctx
for name, tol, stats in (("value-only (V, ICp2) tol 1e-12", 1e-12, [S.iterations(), S.V(), S.criterion()]),
                         ("value-only (V, ICp2) tol 1e-11", 1e-11, [S.iterations(), S.V(), S.criterion()]),
                         ("value-only (V, ICp2) tol 3e-12", 3e-12, [S.iterations(), S.V(), S.criterion()]),
                         ("strict (t-stat)", 1e-12, [S.iterations(), S.t_stat(2)])):
    ctx.set_value_tol(tol)
    out = D.wild_bootstrap(model, B, stats, idx=idx, eta=eta)
    it = out[:, 0].astype(int)
    print(name, "iterations histogram", {int(k): int(v) for k, v in zip(*np.unique(it, return_counts=True))},
          "mean", float(it.mean()), flush=True)
