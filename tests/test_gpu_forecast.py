"""GPU parity for the forecast step of pseudo_out_of_sample_forecasts
(src/utils.jl:54-72): per window, the IC-sweep refit on rows 1..date_index-1
and predict (src/DynamicFactorModel.jl:152-155) through get_factors with
defect D4 repaired (the local rotation of :126), against the oracle's
restatement.  The forecast is sign-invariant (F_new and the factor
coefficients flip together), so it is compared directly."""
import numpy as np
import pytest

from test_gpu_parity import panel

pytestmark = pytest.mark.gpu
FCST_RTOL = 1e-10


@pytest.mark.parametrize("T,N,P,crit", [(90, 160, 8, "ICp2"), (140, 40, 10, "BIC"), (120, 300, 6, "ICp1"),
                                        (90, 160, 8, "PCp2"), (140, 40, 10, "PCp1"), (260, 400, 5, "PCp3")])
def test_forecasts_match_oracle(dfm, oracle, T, N, P, crit):
    y, x, w = panel(oracle, T, N, 3, 4000 + T)
    kmax = 6
    pred, true = dfm.pseudo_out_of_sample_forecasts(dfm.DynamicFactorModel, y, w, x, crit,
                                                    num_predictions=P, kmax=kmax)
    po, to, fits = oracle.pseudo_out_of_sample_forecasts(
        lambda yy, ww, xx: oracle.DynamicFactorModel_ic(yy, ww, xx, crit, kmax=kmax), y, w, x, P)
    assert np.array_equal(true, to)
    assert np.max(np.abs(pred - po)) <= FCST_RTOL * np.max(np.abs(po))
    assert abs(dfm.MSE(true, pred) - oracle.MSE(to, po)) <= FCST_RTOL * oracle.MSE(to, po)


def test_forecast_with_extra_regressor(dfm, oracle):
    T, N, P = 100, 150, 5
    y, x, w = panel(oracle, T, N, 2, 4444)
    w = np.hstack([w, np.r_[0.0, y[:-1]][:, None]])     # a lag of y, as test/DynamicFactorModel.jl:13-18
    pred, true = dfm.pseudo_out_of_sample_forecasts(dfm.DynamicFactorModel, y, w, x, "ICp2",
                                                    num_predictions=P, kmax=5)
    po, to, _ = oracle.pseudo_out_of_sample_forecasts(
        lambda yy, ww, xx: oracle.DynamicFactorModel_ic(yy, ww, xx, "ICp2", kmax=5), y, w, x, P)
    assert np.max(np.abs(pred - po)) <= FCST_RTOL * np.max(np.abs(po))


@pytest.mark.parametrize("T,N,P,crit", [(70, 160, 4, "ICp2"), (150, 60, 5, "PCp2")])
def test_forecasts_default_kmax(dfm, oracle, T, N, P, crit):
    """model_args = (criterion,) only: every window sweeps to its own ceil(m_w/2)."""
    y, x, w = panel(oracle, T, N, 3, 4500 + T)
    pred, true = dfm.pseudo_out_of_sample_forecasts(dfm.DynamicFactorModel, y, w, x, crit, num_predictions=P)
    po, to, _ = oracle.pseudo_out_of_sample_forecasts(
        lambda yy, ww, xx: oracle.DynamicFactorModel_ic(yy, ww, xx, crit), y, w, x, P)
    assert np.array_equal(true, to)
    assert np.max(np.abs(pred - po)) <= FCST_RTOL * np.max(np.abs(po))
