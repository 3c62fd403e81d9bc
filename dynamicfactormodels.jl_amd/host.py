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


# --------------------------------------------------------------- data input
def lag_vector(vec) -> np.ma.MaskedArray:
    """``src/utils.jl:5-10``: the one-period lag [0, vec[1:end-1]] with the
    first entry missing (a DataArray NA there; a masked entry here).  A masked
    input keeps its mask shifted along."""
    v = np.ma.asarray(vec, dtype=np.float64)
    out = np.ma.empty(v.shape, dtype=np.float64)
    out[0] = 0.0
    out[1:] = v[:-1]
    mask = np.zeros(v.shape, dtype=bool)
    mask[0] = True
    mask[1:] = np.ma.getmaskarray(v)[:-1]
    out.mask = mask
    return out


def lag_matrix(matr) -> np.ma.MaskedArray:
    """``src/utils.jl:11-16``: lag_vector applied to every column."""
    m = np.ma.asarray(matr, dtype=np.float64)
    return np.ma.column_stack([lag_vector(m[:, c]) for c in range(m.shape[1])])


def norm_vector(vec) -> np.ndarray:
    """``src/utils.jl:43``: vec ./ norm(vec)."""
    v = np.asarray(vec, dtype=np.float64)
    return v / np.linalg.norm(v)


def norm_matrix(mat) -> np.ndarray:
    """``src/utils.jl:44``: mapslices(norm_vector, mat, 2) — every ROW scaled to
    unit norm (slices along dimension 2, as the code does; its comment says
    columns)."""
    m = np.asarray(mat, dtype=np.float64)
    return m / np.linalg.norm(m, axis=1, keepdims=True)


def possemidef(x) -> bool:
    """``src/utils.jl:46-51``: whether the Cholesky factorisation succeeds."""
    try:
        np.linalg.cholesky(np.asarray(x, dtype=np.float64))
        return True
    except np.linalg.LinAlgError:
        return False


def read_panel_csv(path: str):
    """The data load of ``test/DynamicFactorModel.jl:6-7``: ``readtable`` of a
    CSV whose first column is the date / id and whose other columns are the
    series; returns (series names, T x (columns-1) float64 matrix).  Missing
    values raise, as ``convert(Array{Float64}, col)`` does on an NA."""
    import csv
    with open(path, newline="") as fh:
        rows = list(csv.reader(fh))
    header, body = rows[0], [r for r in rows[1:] if r]
    names = [h.strip() for h in header[1:]]
    data = np.empty((len(body), len(names)))
    for t, row in enumerate(body):
        if len(row) != len(header):
            raise ValueError(f"row {t + 2}: {len(row)} fields, expected {len(header)}")
        for c, cell in enumerate(row[1:]):
            cell = cell.strip()
            if cell in ("", "NA", "NaN", "nan"):
                raise ValueError(f"missing value in column {names[c]!r}, row {t + 2}")
            data[t, c] = float(cell)
    return names, data


def reference_test_design(data_matrix, nlags: int = 4):
    """``test/DynamicFactorModel.jl:8-20``: y = the first series, x = the
    others, w = [1, y_{t-1}, ..., y_{t-nlags}] built with lag_vector, and the
    first nlags rows (whose lags are missing) dropped.  Returns (y, w, x)."""
    d = np.asarray(data_matrix, dtype=np.float64)
    T = d.shape[0] - nlags
    y_full, x_full = d[:, 0], d[:, 1:]
    lags, cur = [], y_full
    for _ in range(nlags):
        cur = lag_vector(cur)
        lags.append(cur)
    w = np.column_stack([np.ones(T)] + [np.ma.getdata(l)[nlags:] for l in lags])
    return y_full[nlags:].copy(), w, x_full[nlags:].copy()
