"""Host logic of the stat::Function escape (src/bootstrap.jl:21, :41) — CPU.

``api._bootstrap_closure`` turns the device's per-replicate rows (V, the
criterion, eigenvalues, coefficients, t-statistics, DFM_STAT_FACTORS,
DFM_STAT_LOADINGS per block) into one ``ReplicateFit`` record per replicate
and runs the closure on it.  Here the rows are synthesised from the oracle's
own replicate fits in the device's layout, so the unpacking, the replicate
panel X*_b = C + diag(eta_b) E[idx_b], the blockwise factor residuals and
the chunking are checked without a GPU: a closure of oracle functions on the
rebuilt records must return the oracle's loop values exactly (the same fp64
operations on the same arrays) or to rounding where the record recomputes
a field."""
import numpy as np
import pytest


class _Base:
    """The fields of a fitted model that the closure path reads."""

    def __init__(self, o):
        self.x, self.y, self.w = o.x, o.y, o.w
        r = o.number_of_factors
        self.number_of_factors = r
        self.number_of_factors_criterion = o.number_of_factors_criterion
        self.break_indices = list(o.break_indices)
        self.factor_type = "principal components"
        self.factors = [F[:, :r] for F in o.factors]
        self.factor_residuals = o.factor_residuals
        self.targeted_predictors = np.ones(o.x.shape[1], dtype=bool)


def _rows(oracle, o, fits, stats_order=True):
    """Device-layout rows: V, crit?, eig 1..r, coef 1..d, t 1..d, F (T r), L_j (N r) per block."""
    r, q = o.number_of_factors, o.w.shape[1]
    rows = []
    for d in fits:
        row = [oracle.factor_residual_variance(d)]
        if o.number_of_factors_criterion:
            row.append(d.number_of_factors_criterion_value)
        row += list(d.eigenvalues[0][:r])
        row += list(d.coefficients[:q + r]) + list(d.t_stats[:q + r])
        row += list(d.F.ravel())
        for L in d.loadings:
            row += list(L[:, :r].ravel())
        rows.append(row)
    return np.array(rows)


@pytest.mark.parametrize("T,N,breaks,kind", [(60, 40, [], 0), (50, 70, [26], 0), (60, 40, [], 1)])
def test_closure_records_match_oracle_loop(dfm, oracle, T, N, breaks, kind):
    rng = np.random.default_rng(5)
    y, x, *_ = oracle.factor_model_DGP(T, N, 2, rng, model="Breitung_Eickmeier_2011", b=0.5)
    x = oracle.normalize(x)
    w = np.ones((T, 1))
    o = oracle.DynamicFactorModel(y, w, x, 2, "ICp2", breaks)
    B = 5
    if kind == 0:
        idx, eta = oracle.draw_wild(np.random.default_rng(1), B, T)
        xs = [o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]] for b in range(B)]
    else:
        idx, eta = oracle.draw_residual(np.random.default_rng(1), B, T, breaks), None
        xs = [o.common_component + o.factor_residuals[idx[b]] for b in range(B)]
    fits = [oracle.DynamicFactorModel(y, w, xb, 2, "ICp2", breaks) for xb in xs]
    rows = _rows(oracle, o, fits)
    calls = []

    def run_rows(stats, c0, c1):
        calls.append((c0, c1))
        return rows[c0:c1]

    from dfm_amd import api
    bp = T // 2 + 2
    base = _Base(o)
    lr = api._bootstrap_closure(base, kind, B, lambda d: oracle.LR_test(d, bp, 3), np.asarray(idx, np.int32),
                                eta, run_rows)
    V = api._bootstrap_closure(base, kind, B, oracle.factor_residual_variance, np.asarray(idx, np.int32), eta,
                               run_rows)
    recs = []
    api._bootstrap_closure(base, kind, B, lambda d: recs.append(d) or 0.0, np.asarray(idx, np.int32), eta, run_rows)
    for b, d in enumerate(fits):
        rec = recs[b]
        assert np.max(np.abs(rec.x - d.x)) <= 4e-15 * np.max(np.abs(d.x))        # the replicate panel
        assert np.max(np.abs(rec.factor_residuals - d.factor_residuals)) <= 1e-13 * np.max(np.abs(d.x))
        assert np.array_equal(rec.F, d.F) and len(rec.factors) == len(breaks) + 1
        assert np.array_equal(rec.coefficients, d.coefficients) and np.array_equal(rec.t_stats, d.t_stats)
        assert np.max(np.abs(rec.residuals - d.residuals)) <= 1e-12 * np.max(np.abs(d.residuals))
        assert rec.V == oracle.factor_residual_variance(d)
        # the HC2 sandwich of src/DynamicFactorModel.jl:43-46 rebuilt on the host
        cov = d.coefficient_covariance
        assert np.max(np.abs(rec.coefficient_covariance - cov)) <= 1e-10 * np.max(np.abs(cov))
        assert np.array_equal(rec.targeted_predictors, base.targeted_predictors)
        assert np.array_equal(rec.eigenvalues, d.eigenvalues[0][:2]) if len(breaks) == 0 else True
        assert (rec.block_eigenvalues is None) == (len(breaks) > 0)
        assert abs(lr[b] - oracle.LR_test(d, bp, 3)) <= 1e-9 * abs(oracle.LR_test(d, bp, 3))
        assert abs(V[b] - oracle.factor_residual_variance(d)) <= 1e-12 * oracle.factor_residual_variance(d)


def test_closure_is_chunked_in_replicate_order(dfm, oracle, monkeypatch):
    """Rows come in bounded chunks (the device returns T r + N r values per
    replicate) and the closure runs in replicate order."""
    rng = np.random.default_rng(2)
    T, N = 40, 30
    y, x, *_ = oracle.factor_model_DGP(T, N, 2, rng)
    x = oracle.normalize(x)
    w = np.ones((T, 1))
    o = oracle.DynamicFactorModel(y, w, x, 2, "")
    B = 7
    idx, eta = oracle.draw_wild(np.random.default_rng(3), B, T)
    fits = [oracle.DynamicFactorModel(y, w, o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]], 2, "")
            for b in range(B)]
    rows = _rows(oracle, o, fits)
    from dfm_amd import api
    width = rows.shape[1]
    monkeypatch.setattr(api, "_CLOSURE_CHUNK_BYTES", 3 * 8 * width)   # three replicates per chunk
    calls = []

    def run_rows(stats, c0, c1):
        calls.append((c0, c1))
        return rows[c0:c1]
    order = []
    api._bootstrap_closure(_Base(o), 0, B, lambda d: order.append(d.V) or 0.0, np.asarray(idx, np.int32), eta,
                           run_rows)
    assert calls == [(0, 3), (3, 6), (6, 7)]
    assert order == [oracle.factor_residual_variance(d) for d in fits]
