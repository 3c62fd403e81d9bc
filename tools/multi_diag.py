"""Diagnose multi-context bootstrap bit-identity (reproduces the C harness
call sequence through the Python binding)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import dfm_pkg
D = dfm_pkg.load()
T, N, B = 96, 150, 6
rng = np.random.default_rng(11)
y = rng.standard_normal(T)
f = rng.standard_normal((T, 3))
X = f @ rng.standard_normal((3, N)) + rng.standard_normal((T, N))
X = (X - X.mean(0)) / X.std(0, ddof=1)
idx = rng.integers(0, T, size=(B, T), dtype=np.int32)
eta = rng.standard_normal((B, T))
w = np.ones((T, 1))
S = D.Stat
stats = [S.V(), S.criterion(), S.LR_all(T // 2)]
for variant in ("plain", "residual_first"):
    g = D.DynamicFactorModel(y, w, X, "ICp2", kmax=8)
    print("r =", g.number_of_factors)
    one = D.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
    if variant == "residual_first":
        D.residual_bootstrap(g, B, S.V(), idx=idx)
    c = D.clone_model(g, D.Context(0))
    many = D.wild_bootstrap([g, c], B, stats, idx=idx, eta=eta)
    again = D.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
    onc = D.wild_bootstrap(c, B, stats, idx=idx, eta=eta)
    for name, arr in (("multi", many), ("again", again), ("clone_single", onc)):
        d = np.abs(arr - one)
        bad = np.argwhere(d > 0)
        print(variant, name, "max abs diff", d.max(), "n diff", len(bad), "rows", sorted(set(bad[:, 0].tolist()))[:10],
              "cols", sorted(set(bad[:, 1].tolist()))[:10])
