"""Determinism probe 2: the test order of tests/test_gpu_multi.py's two-lane
test — a fresh model per case, the factored case before the direct one, the
models dropped between rounds — repeated; prints direct-case rows that differ
from the first round's one-lane result."""
import gc, os, sys
import numpy as np
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
for d in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, d)
import dfm_pkg, dfm_oracle as oracle
from test_gpu_parity import panel

K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
dfm = dfm_pkg.load()
S = dfm.Stat


def job(T, N, r, mode, B):
    y, x, w = panel(oracle, T, N, r, 700 + T)
    g = dfm.DynamicFactorModel(y, w, x, r, "ICp2")
    g.set_bootstrap_mode(mode)
    idx, eta = dfm.draw_wild_fast(77, B, T)
    stats = [S.V(), S.criterion(), S.eigenvalue(1), S.coefficient(1), S.t_stat(2), S.LR_all(T // 2),
             S.LM(T // 2, 1), S.iterations()]
    lanes = dfm.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
    g.set_batch(B)
    one = dfm.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
    return lanes, one


ref = None
bad = 0
for k in range(K):
    job(200, 400, 4, "factored", 700)
    gc.collect()
    lanes, one = job(96, 150, 3, "direct", 600)
    gc.collect()
    if ref is None:
        ref = one
    for name, a in (("lanes", lanes), ("one", one)):
        rows = np.where(~np.all((a == ref) | (np.isnan(a) & np.isnan(ref)), axis=1))[0]
        if len(rows):
            bad += 1
            print(f"round {k} {name}: {len(rows)} rows differ, first {rows[:8].tolist()}; eig {a[rows[0], 2]:.6g} vs "
                  f"{ref[rows[0], 2]:.6g}, steps {a[rows[0], -1]:.0f} vs {ref[rows[0], -1]:.0f}", flush=True)
    print(f"round {k} done", flush=True)
print(f"{bad} of {2 * K} direct-case results differ from round 0's one-lane result", flush=True)
