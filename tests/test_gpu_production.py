"""Production-size parity: the exact batch paths the benchmarks time, checked
against the reference-faithful oracle (not only against themselves).

* C3 (BASELINE.json configs[2]): B = 9999 replicates of T=500 N=2000 r=8 in ONE
  device batch through dfm_bootstrap_dev — the 16 GB factored workspace, the
  straggler phase with column compaction, the eigenvalue (Kato-Temple)
  stopping rule of the bench's V + ICp2 stats — with sampled replicates
  (first, last, the slowest stragglers by eigensolver steps, two random)
  refit by the oracle (src/bootstrap.jl:41-51) at 1e-10.
* C5 (configs[4]): T=2000 N=20000, P=200 expanding windows through
  dfm_windows_dev (the bench's path), windows 0 / 100 / 199 against the
  oracle's DynamicFactorModel_ic(kmax=8) refits (src/utils.jl:54-72), frozen
  in tests/golden/c5_windows.npz by make_golden.py (an oracle window costs
  ~40 s of CPU there); the panel is regenerated from its seed and its digest
  checked first.
* C5 rolling (configs[4], `--rolling 1000`): windows 0 / 100 / 199 of the
  1000-row rolling refits, frozen in tests/golden/c5_rolling.npz.
* C2 (configs[1]): B = 999 wild-bootstrap replicates of T=600 N=130 with V,
  ICp2 and LR/LM/Wald of every variable — the bench's job, which runs as two
  lanes (two streams) — sampled replicates (first, last, the slowest, two
  random) against the oracle's Chow tests (src/chowtest.jl:19-42).
* C4 (configs[3]): hard PER_CANDIDATE thresholding on the full T=400
  N=5000 panel against the oracle (src/targeted_predictors.jl:9-30, D8)."""
import os

import numpy as np
import pytest

from test_gpu_parity import STAT_RTOL, lm_within, lr_within, rel

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_c3_full_batch_sampled_replicates_match_oracle(dfm, oracle):
    import torch
    T, N, r, B = 500, 2000, 8, 9999
    rng = np.random.default_rng(20261015 + 3)
    y, x, *_ = oracle.factor_model_DGP(T, N, r, rng)
    x = oracle.normalize(x)
    w = np.ones((T, 1))
    ctx = dfm.Context(0)
    g = dfm.DynamicFactorModel(y, w, x, r, "ICp2", ctx=ctx)
    S = dfm.Stat
    stats = [S.V(), S.criterion(), S.trace(), S.iterations()] + [S.eigenvalue(j) for j in range(1, r + 1)]
    arr = dfm.api._stat_array(stats)
    width = int(ctx.lib.dfm_stats_width(g.handle, arr, len(stats)))
    idx, eta = dfm.draw_wild_fast(1_000_003, B, T)          # the bench's first step draws
    dev = torch.device("cuda", 0)
    idx_d, eta_d = torch.from_numpy(idx).to(dev), torch.from_numpy(eta).to(dev)
    out = torch.empty((B, width), dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    ctx.reset_timing()
    ctx.check(ctx.lib.dfm_bootstrap_dev(g.handle, 0, B, idx_d.data_ptr(), eta_d.data_ptr(), arr, len(stats),
                                        out.data_ptr()))
    ctx.synchronize()
    es = ctx.eig_stats()
    assert es["batches"] == 1                                # the whole job in one device batch
    res = out.cpu().numpy()
    assert np.all(np.isfinite(res))
    its = res[:, 3]
    assert np.all(its >= 1)
    order = np.argsort(-its, kind="stable")
    sample = sorted(set([0, B - 1] + list(order[:6]) + list(np.random.default_rng(1).integers(1, B - 1, 2))))
    assert its[order[0]] > np.median(its)                    # the stragglers are in the sample
    o = oracle.DynamicFactorModel(y, w, x, r, "ICp2")
    common, E = o.common_component, o.factor_residuals
    for b in sample:
        xs = common + eta[b][:, None] * E[idx[b]]
        d = oracle.DynamicFactorModel(y, w, xs, r, "ICp2")
        ref = [oracle.factor_residual_variance(d), d.number_of_factors_criterion_value, np.sum(xs * xs)]
        ref += list(d.eigenvalues[0][:r])
        got = [res[b, 0], res[b, 1], res[b, 2]] + list(res[b, 4:])
        assert rel(got, ref) < STAT_RTOL, (b, its[b])


def test_c3_full_batch_coefficients_loadings_chow_match_oracle(dfm, oracle):
    """The B = 9999 C3 job with the fit's regression outputs requested (every
    OLS coefficient and HC2 t-statistic, src/DynamicFactorModel.jl:40-48) and
    the Chow LR of every variable (src/chowtest.jl:19-23, which reads each
    replicate's loadings through E* = X* - F* L*'): the strict eigenvector
    stopping rule, the factored loadings GEMM, OLS and Chow kernels at full
    size, sampled replicates against the oracle at 1e-10.  Factor columns'
    coefficients are compared in absolute value (eigenvector signs are
    arbitrary; both sides canonicalise them), the intercept's exactly."""
    import torch
    T, N, r, B = 500, 2000, 8, 9999
    rng = np.random.default_rng(20261015 + 3)
    y, x, *_ = oracle.factor_model_DGP(T, N, r, rng)
    x = oracle.normalize(x)
    w = np.ones((T, 1))
    ctx = dfm.Context(0)
    g = dfm.DynamicFactorModel(y, w, x, r, "ICp2", ctx=ctx)
    S = dfm.Stat
    d = 1 + r
    bp = 250
    stats = [S.coefficient(j) for j in range(1, d + 1)] + [S.t_stat(j) for j in range(1, d + 1)] + [S.LR_all(bp)]
    arr = dfm.api._stat_array(stats)
    width = int(ctx.lib.dfm_stats_width(g.handle, arr, len(stats)))
    assert width == 2 * d + N
    idx, eta = dfm.draw_wild_fast(1_000_004, B, T)
    dev = torch.device("cuda", 0)
    idx_d, eta_d = torch.from_numpy(idx).to(dev), torch.from_numpy(eta).to(dev)
    out = torch.empty((B, width), dtype=torch.float64, device=dev)
    ctx.check(ctx.lib.dfm_bootstrap_dev(g.handle, 0, B, idx_d.data_ptr(), eta_d.data_ptr(), arr, len(stats),
                                        out.data_ptr()))
    ctx.synchronize()
    res = out.cpu().numpy()
    del out
    assert np.all(np.isfinite(res))
    o = oracle.DynamicFactorModel(y, w, x, r, "ICp2")
    common, E = o.common_component, o.factor_residuals
    vs = [0, 1, 977, N - 1]
    for b in sorted(set([0, B - 1] + list(np.random.default_rng(2).integers(1, B - 1, 4)))):
        xs = common + eta[b][:, None] * E[idx[b]]
        dd = oracle.DynamicFactorModel(y, w, xs, r, "ICp2")
        assert rel(res[b, 0], dd.coefficients[0]) < STAT_RTOL and rel(res[b, d], dd.t_stats[0]) < STAT_RTOL, b
        assert rel(np.abs(res[b, 1:d]), np.abs(dd.coefficients[1:])) < STAT_RTOL, b
        assert rel(np.abs(res[b, d + 1:2 * d]), np.abs(dd.t_stats[1:])) < STAT_RTOL, b
        ref = [oracle.LR_test(dd, bp, i) for i in vs]
        assert rel(res[b, 2 * d + np.array(vs)], ref) < STAT_RTOL, b


def c5_panel(oracle):
    rng = np.random.default_rng(20261015 + 5)
    y, x, *_ = oracle.factor_model_DGP(2000, 20000, 8, rng)
    return y, oracle.normalize(x)


def test_c5_full_panel_windows_match_frozen_oracle(dfm, oracle):
    import torch
    g = np.load(os.path.join(GOLD, "c5_windows.npz"))
    y, x = c5_panel(oracle)
    # same panel as the fixture's (the column means are ~0, so the plain sum
    # is compared absolutely: NumPy's SIMD summation order differs by host)
    assert abs(x.sum() - g["digest"][0]) < 1e-6
    assert rel([np.abs(x).sum(), y.sum()], g["digest"][1:]) < 1e-12
    dev = torch.device("cuda", 0)
    yd = torch.from_numpy(np.ascontiguousarray(y)).to(dev)
    wd = torch.ones((2000, 1), dtype=torch.float64, device=dev)
    xd = torch.from_numpy(np.ascontiguousarray(x.T)).to(dev).t()     # column-major, as the bench
    del x
    out = dfm.pseudo_out_of_sample_refits_dev(yd, wd, xd, "ICp2", num_predictions=200, kmax=8)
    for k, wi in enumerate(g["windows"]):
        r = int(g["r"][k])
        assert out["number_of_factors"][wi] == r, wi
        assert abs(out["V"][wi] - g["V"][k]) <= STAT_RTOL * g["V"][k]
        assert abs(out["criterion_value"][wi] - g["crit"][k]) <= STAT_RTOL * abs(g["crit"][k])
        assert rel(out["eigenvalues"][wi][:8], g["eigvals"][k]) < STAT_RTOL
        assert rel(out["t_stats"][wi][:1], g["tstat"][k][:1]) < STAT_RTOL            # intercept: sign-free
        assert rel(out["coefficients"][wi][:1], g["coef"][k][:1]) < STAT_RTOL
        # factor columns in absolute value (eigenvector signs are arbitrary)
        assert rel(np.abs(out["coefficients"][wi][1:1 + r]), np.abs(g["coef"][k][1:1 + r])) < STAT_RTOL, wi
        assert rel(np.abs(out["t_stats"][wi][1:1 + r]), np.abs(g["tstat"][k][1:1 + r])) < STAT_RTOL, wi


def test_c2_b999_two_lane_job_sampled_replicates_match_oracle(dfm, oracle):
    """BASELINE configs[1] exactly as `tools/bench_configs.py c2` runs it:
    B = 999 in one dfm_bootstrap_dev call (two lanes), stats V + ICp2 +
    LR/LM/Wald of all 130 variables at bp = 300.  Sampled replicates against
    the oracle's refit of the same draw (src/bootstrap.jl:41-51,
    src/chowtest.jl:19-42): V and the criterion at 1e-10, Wald at 1e-10,
    LR / LM within the double-double referee bar of the oracle's fit."""
    import torch
    T, N, B, bp = 600, 130, 999, 300
    y, x, *_ = dfm.factor_model_DGP(T, N, 3, model="Breitung_Eickmeier_2011", b=0.5,
                                    rng=np.random.default_rng(20261015 + 2))
    x = dfm.normalize(x)
    w = np.ones((T, 1))
    ctx = dfm.Context(0)
    g = dfm.DynamicFactorModel(y, w, x, "ICp2", kmax=8, ctx=ctx)
    r = g.number_of_factors
    S = dfm.Stat
    stats = [S.V(), S.criterion(), S.LR_all(bp), S.LM_all(bp), S.Wald_all(bp), S.iterations()]
    arr = dfm.api._stat_array(stats)
    width = int(ctx.lib.dfm_stats_width(g.handle, arr, len(stats)))
    assert width == 3 + 3 * N
    idx, eta = dfm.draw_wild_fast(7, B, T)
    dev = torch.device("cuda", 0)
    di, de = torch.from_numpy(idx).to(dev), torch.from_numpy(eta).to(dev)
    out = torch.empty((B, width), dtype=torch.float64, device=dev)
    ctx.check(ctx.lib.dfm_bootstrap_dev(g.handle, 0, B, di.data_ptr(), de.data_ptr(), arr, len(stats),
                                        out.data_ptr()))
    ctx.synchronize()
    res = out.cpu().numpy()
    assert np.all(np.isfinite(res))
    o = oracle.DynamicFactorModel(y, w, x, r, "ICp2")
    common, E = o.common_component, o.factor_residuals
    slow = int(np.argmax(res[:, -1]))
    vs = np.array(list(range(8)) + list(range(N - 8, N)))
    picks = sorted(set([0, B - 1, slow, B // 2 - 1, B // 2] + list(np.random.default_rng(3).integers(1, B - 1, 2))))
    for b in picks:   # (B // 2 - 1, B // 2: the last of lane 0, the first of lane 1)
        d = oracle.DynamicFactorModel(y, w, common + eta[b][:, None] * E[idx[b]], r, "ICp2")
        assert rel(res[b, 0], oracle.factor_residual_variance(d)) < STAT_RTOL, b
        assert rel(res[b, 1], d.number_of_factors_criterion_value) < STAT_RTOL, b
        lr_within(res[b, 2 + vs], d, bp, vs, oracle)
        lm_within(res[b, 2 + N + vs], d, bp, vs, oracle)
        assert rel(res[b, 2 + 2 * N + vs], [oracle.Wald_test(d, bp, i) for i in vs]) < STAT_RTOL, b


def test_c5_full_panel_rolling_windows_match_frozen_oracle(dfm, oracle):
    """BASELINE configs[4] in its rolling form (`bench.py --workload c5
    --rolling 1000`): 200 windows of the 1000 rows before each forecast date
    of the full T=2000, N=20000 panel, resident in HBM; windows 0, 100, 199
    against the oracle's IC sweeps frozen in tests/golden/c5_rolling.npz."""
    import torch
    g = np.load(os.path.join(GOLD, "c5_rolling.npz"))
    y, x = c5_panel(oracle)
    assert abs(x.sum() - g["digest"][0]) < 1e-6
    assert rel([np.abs(x).sum(), y.sum()], g["digest"][1:]) < 1e-12
    dev = torch.device("cuda", 0)
    yd = torch.from_numpy(np.ascontiguousarray(y)).to(dev)
    wd = torch.ones((2000, 1), dtype=torch.float64, device=dev)
    xd = torch.from_numpy(np.ascontiguousarray(x.T)).to(dev).t()     # column-major, as the bench
    del x
    out = dfm.pseudo_out_of_sample_windows(yd, wd, xd, "ICp2", num_predictions=200, kmax=8, rolling=int(g["L"]))
    assert np.array_equal(out["window_first_row"][g["windows"]], 2000 - 200 - int(g["L"]) + g["windows"])
    for k, wi in enumerate(g["windows"]):
        r = int(g["r"][k])
        assert out["number_of_factors"][wi] == r, wi
        assert abs(out["V"][wi] - g["V"][k]) <= STAT_RTOL * g["V"][k]
        assert abs(out["criterion_value"][wi] - g["crit"][k]) <= STAT_RTOL * abs(g["crit"][k])
        assert rel(out["eigenvalues"][wi][:8], g["eigvals"][k]) < STAT_RTOL
        assert rel(out["t_stats"][wi][:1], g["tstat"][k][:1]) < STAT_RTOL            # intercept: sign-free
        assert rel(out["coefficients"][wi][:1], g["coef"][k][:1]) < STAT_RTOL
        # factor columns in absolute value (eigenvector signs are arbitrary)
        assert rel(np.abs(out["coefficients"][wi][1:1 + r]), np.abs(g["coef"][k][1:1 + r])) < STAT_RTOL, wi
        assert rel(np.abs(out["t_stats"][wi][1:1 + r]), np.abs(g["tstat"][k][1:1 + r])) < STAT_RTOL, wi


def test_c4_full_panel_per_candidate_matches_oracle(dfm, oracle):
    rng = np.random.default_rng(20261015 + 4)
    T, N = 400, 5000
    y, x, *_ = oracle.factor_model_DGP(T, N, 5, rng)
    x = oracle.normalize(x)
    w = np.ones((T, 1))
    mask, t = dfm.targeted_predictors(y, w, x, "hard", mode="per_candidate", return_tstats=True)
    to, mo = oracle.targeted_predictors_hard(y, w, x, "per_candidate")
    assert rel(t, to) < STAT_RTOL
    assert np.array_equal(mask, mo)
    assert 0 < mask.sum() < N
