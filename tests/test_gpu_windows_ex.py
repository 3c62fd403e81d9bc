"""GPU parity for the generic window driver (dfm_windows_ex) and the fitted
model's predict / get_factors / per-variable Chow / criterion entry points.

pseudo_out_of_sample_forecasts(model, y, w, x, model_args...) (src/utils.jl
:54-72) refits `model(y[1:t-1], w[1:t-1,:], x[1:t-1,:], model_args...)` per
window: model_args may name an IC criterion (the sweep constructor,
src/DynamicFactorModel.jl:53), a fixed r with a criterion (the workhorse,
:28), nothing (the 3-arg default r = ceil(m/2), D2) or break_indices (:73).
Rolling windows (BASELINE.json configs[4]) refit on the last L rows instead.
Each window is compared with the oracle's fit of the same rows; forecasts go
through predict with get_factors repaired (D4)."""
import numpy as np
import pytest

from test_gpu_parity import STAT_RTOL, panel, rel

pytestmark = pytest.mark.gpu


def check_windows(out, fits, q=1):
    for j, o in enumerate(fits):
        r = o.number_of_factors
        assert out["number_of_factors"][j] == r, j
        assert abs(out["V"][j] - o.V_) <= STAT_RTOL * o.V_, j
        if o.number_of_factors_criterion:
            cv = o.number_of_factors_criterion_value
            assert abs(out["criterion_value"][j] - cv) <= STAT_RTOL * abs(cv), j
        else:
            assert np.isnan(out["criterion_value"][j])
        assert rel(out["eigenvalues"][j][:r], o.eigenvalues[0][:r]) < STAT_RTOL, j
        assert rel(out["t_stats"][j][:q], o.t_stats[:q]) < STAT_RTOL, j          # w columns: sign-invariant
        assert rel(out["coefficients"][j][:q], o.coefficients[:q]) < STAT_RTOL, j
        assert rel(np.abs(out["t_stats"][j][q:q + r]), np.abs(o.t_stats[q:])) < STAT_RTOL, j


def annotate(oracle, fits):
    for o in fits:
        o.V_ = oracle.factor_residual_variance(o)
    return fits


@pytest.mark.parametrize("T,N,P,L,crit", [(90, 160, 6, 40, "ICp2"), (140, 30, 6, 60, "BIC"),
                                          (120, 70, 5, 50, "PCp2"), (100, 40, 4, 30, "ICp1")])
def test_rolling_windows_ic_sweep(dfm, oracle, T, N, P, L, crit):
    """Rolling windows of L rows (N > L: diagonal blocks of the one prefix
    Gram, factored solver; L >= N: per-window Grams), IC sweep kmax 5."""
    y, x, w = panel(oracle, T, N, 3, 6000 + T + L)
    out = dfm.pseudo_out_of_sample_windows(y, w, x, crit, num_predictions=P, kmax=5, rolling=L, forecast=True)
    po, to, fits = oracle.rolling_window_forecasts(
        lambda yy, ww, xx: oracle.DynamicFactorModel_ic(yy, ww, xx, crit, kmax=5), y, w, x, P, L)
    check_windows(out, annotate(oracle, fits))
    assert np.array_equal(out["true_values"], to)
    assert np.max(np.abs(out["predictions"] - po)) <= STAT_RTOL * np.max(np.abs(po))


@pytest.mark.parametrize("T,N,P,r,crit,rolling", [(80, 150, 5, 3, "BIC", None), (120, 40, 6, 2, "ICp2", None),
                                                  (80, 150, 5, 4, "", 50), (120, 40, 5, 3, "PCp1", 60)])
def test_fixed_r_windows(dfm, oracle, T, N, P, r, crit, rolling):
    """model_args = (r, criterion): the workhorse constructor per window."""
    y, x, w = panel(oracle, T, N, 3, 6100 + T + r)
    args = (r, crit) if crit else (r,)
    out = dfm.pseudo_out_of_sample_windows(y, w, x, *args, num_predictions=P, rolling=rolling, forecast=True)
    fit = lambda yy, ww, xx: oracle.DynamicFactorModel(yy, ww, xx, r, crit)   # noqa: E731
    if rolling:
        po, to, fits = oracle.rolling_window_forecasts(fit, y, w, x, P, rolling)
    else:
        po, to, fits = oracle.pseudo_out_of_sample_forecasts(fit, y, w, x, P)
    check_windows(out, annotate(oracle, fits))
    assert np.max(np.abs(out["predictions"] - po)) <= STAT_RTOL * np.max(np.abs(po))
    pred, true = dfm.pseudo_out_of_sample_forecasts(dfm.DynamicFactorModel, y, w, x, *args, num_predictions=P,
                                                    rolling=rolling)
    assert np.array_equal(pred, out["predictions"]) and np.array_equal(true, to)


@pytest.mark.parametrize("T,N,P", [(40, 16, 4), (30, 60, 4)])
def test_default_r_windows(dfm, oracle, T, N, P):
    """No model_args: the 3-arg constructor, r_w = ceil(min(t-1, N)/2) (D2)."""
    y, x, w = panel(oracle, T, N, 2, 6200 + T)
    out = dfm.pseudo_out_of_sample_windows(y, w, x, num_predictions=P, forecast=True)
    po, to, fits = oracle.pseudo_out_of_sample_forecasts(lambda yy, ww, xx: oracle.DynamicFactorModel(yy, ww, xx),
                                                         y, w, x, P)
    check_windows(out, annotate(oracle, fits))
    assert np.max(np.abs(out["predictions"] - po)) <= STAT_RTOL * np.max(np.abs(po))


@pytest.mark.parametrize("T,N,P,crit", [(120, 40, 5, "ICp2"), (90, 150, 4, "BIC")])
def test_break_windows(dfm, oracle, T, N, P, crit):
    """model_args with break_indices: every window is a break-aware fit (per
    block PCA with the window's T, N, D7), forecasts by predict."""
    y, x, w = panel(oracle, T, N, 2, 6300 + T, model="Breitung_Eickmeier_2011", b=0.5)
    bp = 50
    out = dfm.pseudo_out_of_sample_windows(y, w, x, crit, "principal components", None, 0, [bp],
                                           num_predictions=P, kmax=4, forecast=True)
    po, to, fits = oracle.pseudo_out_of_sample_forecasts(
        lambda yy, ww, xx: oracle.DynamicFactorModel_ic(yy, ww, xx, crit, kmax=4, break_indices=[bp]), y, w, x, P)
    for j, o in enumerate(fits):
        r = o.number_of_factors
        assert out["number_of_factors"][j] == r
        V = oracle.factor_residual_variance(o)
        assert abs(out["V"][j] - V) <= STAT_RTOL * V
        assert abs(out["criterion_value"][j] - o.number_of_factors_criterion_value) <= \
            STAT_RTOL * abs(o.number_of_factors_criterion_value)
        assert rel(out["t_stats"][j][:1], o.t_stats[:1]) < STAT_RTOL
    assert np.array_equal(out["true_values"], to)
    assert np.max(np.abs(out["predictions"] - po)) <= STAT_RTOL * np.max(np.abs(po))


def test_windows_dev_inputs_match_host(dfm, oracle):
    """The same generic windows from device-resident (column-major) inputs."""
    import torch
    y, x, w = panel(oracle, 100, 160, 3, 6400)
    host = dfm.pseudo_out_of_sample_windows(y, w, x, 3, "ICp2", num_predictions=5, rolling=45, forecast=True)
    dev = torch.device("cuda", 0)
    yd = torch.from_numpy(y.copy()).to(dev)
    wd = torch.from_numpy(np.ascontiguousarray(w.T)).to(dev).t()
    xd = torch.from_numpy(np.ascontiguousarray(x.T)).to(dev).t()
    got = dfm.pseudo_out_of_sample_windows(yd, wd, xd, 3, "ICp2", num_predictions=5, rolling=45, forecast=True)
    for k in ("number_of_factors", "V", "criterion_value", "eigenvalues", "t_stats", "predictions"):
        assert np.array_equal(np.nan_to_num(got[k]), np.nan_to_num(host[k])), k


def test_windows_beyond_factored_T(dfm, oracle):
    """N > T windows with T above the factored solver's 4096 rows: masked
    explicit window Grams (diagonal blocks of the prefix Gram) on the explicit
    Gram solver; eigenvalues and V against LAPACK on the windows' rows."""
    import scipy.linalg as sla
    T, N, P, k = 4200, 4300, 1, 3
    rng = np.random.default_rng(77)
    f = rng.standard_normal((T, 3))
    x = f @ rng.standard_normal((3, N)) * 2.0 + rng.standard_normal((T, N))
    y = f @ np.ones(3) + rng.standard_normal(T)
    w = np.ones((T, 1))
    out = dfm.pseudo_out_of_sample_windows(y, w, x, k, num_predictions=P)
    for j in range(P):
        n = T - P + j
        xs = x[:n]
        G = xs @ xs.T
        ev = sla.eigh(G, eigvals_only=True, subset_by_index=[n - k, n - 1], driver="evr")[::-1]
        assert rel(out["eigenvalues"][j][:k], ev) < STAT_RTOL
        V = (np.trace(G) - ev.sum()) / (n * N)
        assert abs(out["V"][j] - V) <= 1e-9 * V


# ------------------------------------------------ fitted-model entry points
@pytest.mark.parametrize("T,N,breaks", [(150, 60, ()), (60, 150, ()), (150, 60, (70,)), (80, 140, (40,))])
def test_predict_and_get_factors(dfm, oracle, T, N, breaks):
    """get_factors / predict (src/DynamicFactorModel.jl:125-128, :152-155, D4)
    on new rows, against the oracle's repaired restatement."""
    y, x, w = panel(oracle, T + 3, N, 3, 6500 + T)
    g = dfm.DynamicFactorModel(y[:T], w[:T], x[:T], 3, "ICp2", break_indices=list(breaks))
    o = oracle.DynamicFactorModel(y[:T], w[:T], x[:T], 3, "ICp2", list(breaks))
    s = np.sign(np.sum(g.loadings[0] * o.loadings[0][:, :3], axis=0))
    Fg = dfm.get_factors(g, x[T:])
    Fo = oracle.get_factors(o, x[T:])
    assert np.max(np.abs(Fg * s - Fo)) <= STAT_RTOL * np.max(np.abs(Fo))
    pg = dfm.predict(g, w[T:], x[T:])
    po = oracle.predict(o, w[T:], x[T:])
    assert np.max(np.abs(pg - po)) <= STAT_RTOL * np.max(np.abs(po))


def test_per_variable_chow_and_model_criteria(dfm, oracle):
    """LR_test / LM_test / Wald_test of one variable (dfm_chow: the model
    keeps the all-variables result) and criterion_<name>(dfm) for every name
    on a model fitted with another criterion (dfm_model_criterion)."""
    y, x, w = panel(oracle, 200, 80, 3, 6600, model="Breitung_Eickmeier_2011", b=0.5)
    g = dfm.DynamicFactorModel(y, w, x, 3, "ICp2")
    o = oracle.DynamicFactorModel(y, w, x, 3, "ICp2")
    LR, LM, W = dfm.chow_all(g, 100)
    for i in (1, 17, 80):
        assert dfm.LR_test(g, 100, i) == LR[i - 1] and dfm.LM_test(g, 100, i) == LM[i - 1]
        assert dfm.Wald_test(g, 100, i) == W[i - 1]
        assert abs(dfm.LR_test(g, 100, i) - oracle.LR_test(o, 100, i - 1)) <= STAT_RTOL * abs(LR[i - 1])
    assert abs(dfm.LM_test(g, 90, 5) - oracle.LM_test(o, 90, 4)) <= STAT_RTOL * abs(oracle.LM_test(o, 90, 4))
    for name in dfm.CRITERIA:
        ref = oracle.criterion_value(name, o)
        got = getattr(dfm.api, f"criterion_{name}")(g)
        assert abs(got - ref) <= STAT_RTOL * abs(ref), name
