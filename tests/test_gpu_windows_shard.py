"""Expanding windows (src/utils.jl:54-72) with the panel resident in HBM
(dfm_windows_dev) and the multi-GPU window shard: windows [w0, w1) of (T, P)
are the (T - P + w1, w1 - w0) windows problem on the leading rows (a
zero-copy view of the column-major device panel).  Shards are run one after
another on the one GPU here; tests/test_parallel.py covers the gather."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

STAT_RTOL = 1e-10


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300))) if a.size else 0.0


def _dev_panel(y, w, x):
    import torch
    d = torch.device("cuda", 0)
    yd = torch.from_numpy(np.ascontiguousarray(y)).to(d)
    wd = torch.from_numpy(np.ascontiguousarray(w.T)).to(d).t()     # column-major (1, T)
    xd = torch.from_numpy(np.ascontiguousarray(x.T)).to(d).t()
    return yd, wd, xd


def _panel(oracle, T, N, seed):
    rng = np.random.default_rng(seed)
    y, x, *_ = oracle.factor_model_DGP(T, N, 3, rng)
    return y, np.ones((T, 1)), oracle.normalize(x)


@pytest.mark.parametrize("T,N,P,crit,kmax", [(120, 400, 12, "ICp2", 8), (90, 30, 6, "BIC", 6),
                                             (80, 200, 8, "PCp2", 6), (70, 160, 7, "ICp2", None)])
def test_dev_path_matches_host_and_oracle(dfm, oracle, T, N, P, crit, kmax):
    y, w, x = _panel(oracle, T, N, 700 + T)
    host = dfm.pseudo_out_of_sample_refits(y, w, x, crit, num_predictions=P, kmax=kmax)
    dev = dfm.pseudo_out_of_sample_refits_dev(*_dev_panel(y, w, x), crit, num_predictions=P, kmax=kmax)
    assert np.array_equal(host["number_of_factors"], dev["number_of_factors"])
    for f in ("V", "criterion_value", "eigenvalues"):
        assert rel(dev[f], host[f]) < STAT_RTOL, f
    assert np.array_equal(np.isnan(host["coefficients"]), np.isnan(dev["coefficients"]))
    fits = oracle.expanding_window_refits(y, w, x, P, lambda yy, ww, xx: oracle.DynamicFactorModel_ic(
        yy, ww, xx, crit, kmax=kmax))
    for j, o in enumerate(fits):
        assert dev["number_of_factors"][j] == o.number_of_factors
        assert abs(dev["V"][j] - oracle.factor_residual_variance(o)) <= STAT_RTOL * oracle.factor_residual_variance(o)


@pytest.mark.parametrize("T,N,P,world,kmax", [(120, 400, 12, 3, 8), (90, 30, 6, 4, 6), (2000, 20000, 16, 2, 8),
                                              (70, 160, 7, 2, None)])
def test_window_shards_reassemble(dfm, T, N, P, world, kmax, oracle):
    from dfm_amd.parallel import window_shard, _pack_windows, _unpack_windows
    from dfm_amd.api import _window_kmax
    y, w, x = _panel(oracle, T, N, 900 + T)
    yd, wd, xd = _dev_panel(y, w, x)
    full = dfm.pseudo_out_of_sample_refits_dev(yd, wd, xd, "ICp2", num_predictions=P, kmax=kmax)
    K, q = _window_kmax(T, N, kmax), 1
    blocks = []
    for rank in range(world):
        w0, w1, rows = window_shard(T, P, world, rank)
        res = dfm.pseudo_out_of_sample_refits_dev(yd, wd, xd, "ICp2", num_predictions=w1 - w0, kmax=kmax,
                                                  rows=rows) if w1 > w0 else {}
        blocks.append(_pack_windows(res, w1 - w0, K, q))
    got = _unpack_windows(np.concatenate(blocks), T, P, K, q)
    assert np.array_equal(got["number_of_factors"], full["number_of_factors"])
    assert rel(got["V"], full["V"]) < STAT_RTOL
    assert rel(got["criterion_value"], full["criterion_value"]) < STAT_RTOL
    for j in range(P):
        kw = min(kmax or 10**9, -(-min(T - P + j, N) // 2))
        assert rel(got["eigenvalues"][j, :kw], full["eigenvalues"][j, :kw]) < STAT_RTOL
        assert rel(got["t_stats"][j, :1], full["t_stats"][j, :1]) < STAT_RTOL     # intercept: sign-invariant
