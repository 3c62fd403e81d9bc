"""Determinism probe for the two-lane bootstrap (tests/test_gpu_multi.py::
test_two_lanes_are_bit_identical, direct case): K two-lane runs and K one-lane
runs of the same job in one process; prints the replicates whose rows differ
from the first one-lane run."""
import os, sys
import numpy as np
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
for d in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, d)
import dfm_pkg, dfm_oracle as oracle
from test_gpu_parity import panel

T, N, r, mode, B = [int(a) if a.isdigit() else a for a in (sys.argv[1:6] or ["96", "150", "3", "direct", "600"])]
K = int(sys.argv[6]) if len(sys.argv) > 6 else 8
dfm = dfm_pkg.load()
y, x, w = panel(oracle, T, N, r, 700 + T)
g = dfm.DynamicFactorModel(y, w, x, r, "ICp2")
g.set_bootstrap_mode(mode)
idx, eta = dfm.draw_wild_fast(77, B, T)
S = dfm.Stat
stats = [S.V(), S.criterion(), S.eigenvalue(1), S.coefficient(1), S.t_stat(2), S.LR_all(T // 2),
         S.LM(T // 2, 1), S.iterations()]
lanes = [dfm.wild_bootstrap(g, B, stats, idx=idx, eta=eta) for _ in range(K)]
g.set_batch(B)
ones = [dfm.wild_bootstrap(g, B, stats, idx=idx, eta=eta) for _ in range(K)]
ref = ones[0]
bad = 0
for name, runs in (("lanes", lanes), ("one", ones)):
    for i, a in enumerate(runs):
        rows = np.where(~np.all((a == ref) | (np.isnan(a) & np.isnan(ref)), axis=1))[0]
        if len(rows):
            bad += 1
            print(f"{name} run {i}: {len(rows)} rows differ, first {rows[:8].tolist()}; "
                  f"eig {a[rows[0], 2]:.6g} vs {ref[rows[0], 2]:.6g}, steps {a[rows[0], -1]:.0f} vs {ref[rows[0], -1]:.0f}",
                  flush=True)
print(f"T={T} N={N} r={r} {mode} B={B}: {bad} of {2 * K} runs differ from one-lane run 0", flush=True)
