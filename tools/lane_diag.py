"""Deterministic diagnosis of the two-lane bootstrap defect (VERDICT r04 Weak #1).

Runs the failing case of tests/test_gpu_multi.py::test_two_lanes_are_bit_identical
([96-150-3-direct-600], preceded by its factored case as in the suite) once per
lane skew, on the DEBUG build of libdfm (csrc Makefile EXTRA=-DDFM_DEBUG_MEM:
fresh allocations NaN-poisoned, the draws and output rows inside guard bands
and checked against the host draws after the call, DFM_LANE_SKEW_US holding
one lane back on the device).  For every run it prints which rows of the
two-lane result differ from the one-lane result, by how much, and whether any
is NaN.  Not a repetition probe: each skew runs once.

usage: DFM_LIB_PATH=variants/dbg/libdfm.so python tools/lane_diag.py [skew_us ...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import dfm_pkg  # noqa: E402
import dfm_oracle as O  # noqa: E402


def panel(T, N, r, seed):
    rng = np.random.default_rng(seed)
    out = O.factor_model_DGP(T, N, r, rng)
    return out[0], O.normalize(out[1]), np.ones((T, 1))


def case(D, T, N, r, mode, B, first_only=False):
    y, x, w = panel(T, N, r, 700 + T)
    g = D.DynamicFactorModel(y, w, x, r, "ICp2")
    g.set_bootstrap_mode(mode)
    idx, eta = D.draw_wild_fast(77, B, T)
    S = D.Stat
    stats = [S.V(), S.criterion(), S.eigenvalue(1), S.coefficient(1), S.t_stat(2), S.LR_all(T // 2),
             S.LM(T // 2, 1), S.iterations()]
    lanes = D.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
    lanes2 = None if first_only else D.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
    g.set_batch(B)
    one = D.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
    return lanes, lanes2, one


def report(tag, a, b):
    diff = np.where(~np.all((a == b) | (np.isnan(a) & np.isnan(b)), axis=1))[0]
    nan_rows = np.where(np.any(np.isnan(a), axis=1))[0]
    print(f"  {tag}: {len(diff)} rows differ", end="")
    if len(diff):
        rel = np.max(np.abs(a[diff] - b[diff]) / np.maximum(np.abs(b[diff]), 1e-300), axis=1)
        print(f" (rows {diff[:12].tolist()}{' ...' if len(diff) > 12 else ''}; max rel {rel.max():.3e};"
              f" eigenvalue(1) {a[diff[-1], 2]:.6e} vs {b[diff[-1], 2]:.6e};"
              f" steps {a[diff[-1], -1]:.0f} vs {b[diff[-1], -1]:.0f})", end="")
    print(f"; NaN rows {len(nan_rows)}", flush=True)
    return len(diff)


def main():
    D = dfm_pkg.load()
    skews = [int(s) for s in sys.argv[1:]] or [0]
    print("lib:", os.environ.get("DFM_LIB_PATH", "production"), flush=True)
    bad = 0
    for sk in skews:
        os.environ["DFM_LANE_SKEW_US"] = str(sk)
        print(f"skew {sk} us", flush=True)
        try:
            la, _, on = case(D, 200, 400, 4, "factored", 700, first_only=True)
            bad += report("factored 200x400 B=700 first call", la, on)
            la, la2, on = case(D, 96, 150, 3, "direct", 600)
            bad += report("direct 96x150 B=600 first call", la, on)
            bad += report("direct 96x150 B=600 second call", la2, on)
        except Exception as e:   # a debug-build guard violation surfaces as DFMError 9001
            print("  ERROR:", e, flush=True)
            bad += 1
    print("TOTAL differing rows / errors:", bad, flush=True)


if __name__ == "__main__":
    main()
