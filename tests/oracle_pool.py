"""Whole-batch oracle checks on a CPU process pool (test infrastructure only).

The benched jobs (C3: 9 999 replicates, C2: 999 replicates with Chow tests of
every variable) are checked replicate by replicate against the
reference-faithful oracle (oracle/dfm_oracle.py: the replicate loop of
src/bootstrap.jl:41-51 and the Chow tests of src/chowtest.jl:19-42 as
written).  The children are `spawn`-context processes that import only the
oracle (NumPy / SciPy, one BLAS thread each) — never torch or libdfm — so they
never touch the GPU; the parent hands them the draws and gets the oracle's
values back, and the test compares.

Each child rebuilds the base fit itself (from the panel the parent passes),
so only the draws travel."""
from __future__ import annotations

import os
import sys

import numpy as np

_S: dict = {}
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _oracle():
    p = os.path.join(ROOT, "oracle")
    if p not in sys.path:
        sys.path.insert(0, p)
    import dfm_oracle
    return dfm_oracle


def _init(y, w, x, r, crit):
    O = _oracle()
    base = O.DynamicFactorModel(y, w, x, r, crit)
    _S.update(O=O, y=y, w=w, r=r, crit=crit, C=base.common_component, E=base.factor_residuals)


def _refit(i, e):
    O = _S["O"]
    return O.DynamicFactorModel(_S["y"], _S["w"], _S["C"] + e[:, None] * _S["E"][i], _S["r"], _S["crit"])


def _c3_chunk(args):
    """(idx, eta) rows -> (n, 3 + r): V (src/criteria.jl:5), the criterion,
    trace(X*X*') = |X*|_F^2 and the top-r eigenvalues of each refit."""
    idx, eta = args
    O, r = _S["O"], _S["r"]
    out = np.empty((len(idx), 3 + r))
    for k in range(len(idx)):
        d = _refit(idx[k], eta[k])
        xs = d.x
        out[k, 0] = O.factor_residual_variance(d)
        out[k, 1] = d.number_of_factors_criterion_value
        out[k, 2] = np.sum(xs * xs)
        out[k, 3:] = d.eigenvalues[0][:r]
    return out


def _c2_chunk(args):
    """(idx, eta, bp, vs) -> (n, 2 + 3 len(vs)): V, the criterion, and per
    variable of vs the oracle's Wald, LR and LM (src/chowtest.jl:19-42)."""
    idx, eta, bp, vs = args
    O = _S["O"]
    nv = len(vs)
    out = np.empty((len(idx), 2 + 3 * nv))
    for k in range(len(idx)):
        d = _refit(idx[k], eta[k])
        out[k, 0] = O.factor_residual_variance(d)
        out[k, 1] = d.number_of_factors_criterion_value
        for j, i in enumerate(vs):
            out[k, 2 + j] = O.Wald_test(d, bp, i)
            out[k, 2 + nv + j] = O.LR_test(d, bp, i)
            out[k, 2 + 2 * nv + j] = O.LM_test(d, bp, i)
    return out


def _c2_referee(args):
    """(idx, eta, bp, vs) for ONE replicate -> (len(vs), 2): the double-double
    referee's LR and LM (oracle/dfm_xp.py) of the oracle's refit — the
    exact values that set the LR / LM bars where the fp64 oracle itself is
    further than 1e-10 from them."""
    idx, eta, bp, vs = args
    import dfm_xp
    d = _refit(idx[0], eta[0])
    out = np.empty((len(vs), 2))
    for j, i in enumerate(vs):
        out[j, 0] = dfm_xp.lr_referee(d.F, d.x[:, i], d.factor_residuals[:, i], bp)
        out[j, 1] = dfm_xp.lm_referee(d.F, d.factor_residuals[:, i], bp)
    return out


def workers() -> int:
    """This process's CPU share (affinity mask capped by the cgroup quota:
    bench.cpu_share, 16 on the GPU box)."""
    sys.path.insert(0, ROOT)
    from bench import cpu_share
    return cpu_share()[0]


def run(kind: str, y, w, x, r, crit, idx, eta, extra=(), chunk: int = 32, nproc: int = 0, jobs=None):
    """Oracle rows for every replicate of (idx, eta), in replicate order, on a
    spawn pool of `nproc` (default: this process's CPU share) one-BLAS-thread
    children.  kind "c2ref" takes explicit `jobs` (one replicate each) and
    returns the list of their results."""
    import multiprocessing as mp
    fn = {"c3": _c3_chunk, "c2": _c2_chunk, "c2ref": _c2_referee}[kind]
    nproc = nproc or workers()
    if jobs is None:
        jobs = [(idx[a:a + chunk], eta[a:a + chunk]) + tuple(extra) for a in range(0, len(idx), chunk)]
    if not jobs:
        return []
    saved = {k: os.environ.get(k) for k in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS", "MKL_NUM_THREADS")}
    for k in saved:
        os.environ[k] = "1"
    try:
        with mp.get_context("spawn").Pool(nproc, initializer=_init, initargs=(y, w, x, r, crit)) as pool:
            parts = pool.map(fn, jobs, chunksize=1)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return parts if kind == "c2ref" else np.concatenate(parts, axis=0)
