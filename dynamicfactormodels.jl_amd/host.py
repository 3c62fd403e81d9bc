"""Host-side pieces of the reference API that are not device work: input
generators and preprocessing (``src/utils.jl``), the host RNG contract for the
bootstrap draws, and the t-quantile used as the targeted-predictor critical
value.  These run on the CPU by design — as the reference's own callers do —
and feed device-resident panels to libdfm; none of them computes a hot-path
result.
"""
from __future__ import annotations

import math
from typing import Sequence

import numpy as np


def normalize(A, by=None) -> np.ndarray:
    """``src/utils.jl:33-34``: (A .- mean) ./ std (sample std, n-1), or by a
    given (mean, std) tuple."""
    A = np.asarray(A, dtype=np.float64)
    if by is not None:
        return (A - by[0]) / by[1]
    return (A - A.mean(axis=0)) / A.std(axis=0, ddof=1)


def factor_model_DGP(T: int, N: int, r: int, model: str = "Bai_Ng_2002", b: float = 0.0,
                     rng: np.random.Generator | None = None):
    """``src/utils.jl:76-105`` (Bai_Ng_2002 :93-103, Breitung_Eickmeier_2011
    :80-91) on a NumPy generator (the reference's Julia RNG stream cannot be
    reproduced; the draw order follows the reference)."""
    rng = rng or np.random.default_rng()
    if model == "Bai_Ng_2002":
        f = rng.standard_normal((T, r))
        lam = rng.standard_normal((N, r))
        eps_x = math.sqrt(r) * rng.standard_normal((T, N))
        x = f @ lam.T + eps_x
        beta = rng.uniform(size=r)
        eps_y = rng.standard_normal(T)
        return f @ beta + eps_y, x, f, lam, eps_x, eps_y
    if model == "Breitung_Eickmeier_2011":
        bp = T // 2 if T % 2 == 0 else int(math.ceil(T / 2))
        sigma = rng.uniform(0.5, 1.5, size=N)
        f = rng.standard_normal((T, r))
        Lam = rng.standard_normal((N, r)) + 1.0
        eps = rng.standard_normal((T, N)) * sigma[None, :]
        pre = np.arange(1, T + 1) < bp
        x = np.empty((T, N))
        x[pre] = f[pre] @ Lam.T
        x[~pre] = f[~pre] @ (Lam + b).T
        x += eps
        return rng.uniform(size=T), x, f, Lam, eps
    raise ValueError(f"unknown DGP model {model!r}")


def draw_wild(rng: np.random.Generator, B: int, T: int):
    """Host RNG contract of the wild bootstrap (``src/bootstrap.jl:44-45``):
    per replicate T row indices (0-based) then T N(0,1) multipliers."""
    idx = np.empty((B, T), dtype=np.int32)
    eta = np.empty((B, T))
    for b in range(B):
        idx[b] = rng.integers(0, T, size=T)
        eta[b] = rng.standard_normal(T)
    return idx, eta


def draw_wild_fast(seed: int, B: int, T: int):
    """Vectorised draws for large B (bench inputs): same distributions,
    different (documented) stream order — all rows' indices, then all eta."""
    rng = np.random.default_rng(seed)
    idx = rng.integers(0, T, size=(B, T), dtype=np.int32)
    eta = rng.standard_normal((B, T))
    return idx, eta


def draw_residual(rng: np.random.Generator, B: int, T: int, break_indices: Sequence[int] = ()):
    """Block-wise U{a..b} draws of ``src/bootstrap.jl:23-28`` (0-based)."""
    bp = [1] + list(break_indices) + [T + 1]
    idx = np.empty((B, T), dtype=np.int32)
    for b in range(B):
        for i in range(1, len(bp)):
            a, e = bp[i - 1] - 1, bp[i] - 1
            idx[b, a:e] = rng.integers(a, e, size=e - a)
    return idx


def glmnet_default_folds(n: int, rng: np.random.Generator, nfolds: int | None = None) -> np.ndarray:
    """GLMNet.jl's default fold assignment for glmnetcv (used by
    ``src/targeted_predictors.jl:33``): nfolds = min(10, n ÷ 3),
    shuffle([repeat(1:nfolds, outer=n ÷ nfolds); 1:(n % nfolds)]) — 1-based
    ids, drawn on the host like the bootstrap indices."""
    k = nfolds or min(10, n // 3)
    q, rem = divmod(n, k)
    f = np.concatenate([np.tile(np.arange(1, k + 1), q), np.arange(1, rem + 1)]).astype(np.int32)
    rng.shuffle(f)
    return f


def t_quantile(p: float, df: float) -> float:
    """``quantile(TDist(df), p)`` (``src/targeted_predictors.jl:27``)."""
    from scipy import stats
    return float(stats.t.ppf(p, df))
