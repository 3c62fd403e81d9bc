"""Production-size parity: the exact batch paths the benchmarks time, checked
against the reference-faithful oracle (not only against themselves).

* C3 (BASELINE.json configs[2]): B = 9999 replicates of T=500 N=2000 r=8 in ONE
  device batch through dfm_bootstrap_dev — the 16 GB factored workspace, the
  straggler phase with column compaction, the eigenvalue (Kato-Temple)
  stopping rule of the bench's V + ICp2 stats — EVERY replicate refit by the
  oracle (src/bootstrap.jl:41-51) at 1e-10 on a CPU process pool
  (tests/oracle_pool.py).
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
  lanes (two streams) — EVERY replicate and every variable against the
  oracle's Chow tests (src/chowtest.jl:19-42).
* C4 (configs[3]): hard PER_CANDIDATE thresholding on the full T=400
  N=5000 panel against the oracle (src/targeted_predictors.jl:9-30, D8)."""
import os

import numpy as np
import pytest

from test_gpu_parity import STAT_RTOL, rel

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_c3_full_batch_every_replicate_matches_oracle(dfm, oracle):
    """The bench's first timed step exactly (its draws, its one 9999-replicate
    device batch, its eigenvalue stopping rule) and EVERY replicate against
    the oracle's refit of the same draw (src/bootstrap.jl:41-51): V, ICp2,
    the trace and the top-8 eigenvalues at 1e-10.  The oracle side runs on a
    spawn pool of CPU children that never touch the GPU (tests/oracle_pool.py;
    ~20 s on the box's 16 cores)."""
    import torch
    import oracle_pool
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
    del out, idx_d, eta_d
    assert np.all(np.isfinite(res))
    its = res[:, 3]
    assert np.all(its >= 1) and its.max() > np.median(its)  # a straggler phase ran
    ref = oracle_pool.run("c3", y, w, x, r, "ICp2", idx, eta)
    got = np.concatenate([res[:, :3], res[:, 4:]], axis=1)
    err = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-300)
    worst = np.unravel_index(np.argmax(err), err.shape)
    assert err.max() < STAT_RTOL, (worst, err.max(), its[worst[0]])


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


def test_c2_b999_two_lane_job_every_replicate_matches_oracle(dfm, oracle):
    """BASELINE configs[1] exactly as `tools/bench_configs.py c2` runs it:
    B = 999 in one dfm_bootstrap_dev call (two lanes), stats V + ICp2 +
    LR/LM/Wald of all 130 variables at bp = 300.  EVERY replicate and EVERY
    variable against the oracle's refit of the same draw
    (src/bootstrap.jl:41-51, src/chowtest.jl:19-42; a spawn pool of CPU
    children, tests/oracle_pool.py): V, the criterion and Wald at 1e-10; LR
    and LM at 1e-10 of the oracle, and where the fp64 oracle is itself
    further off than that, within the double-double referee bar of the
    oracle's fit (lr_within / lm_within: the referee recomputed for those
    replicates only)."""
    import torch
    import oracle_pool
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
    vs = list(range(N))
    ref = oracle_pool.run("c2", y, w, x, r, "ICp2", idx, eta, extra=(bp, vs), chunk=8)
    assert rel(res[:, 0], ref[:, 0]) < STAT_RTOL and rel(res[:, 1], ref[:, 1]) < STAT_RTOL
    wald_g, wald_o = res[:, 2 + 2 * N:2 + 3 * N], ref[:, 2:2 + N]
    assert rel(wald_g, wald_o) < STAT_RTOL, np.unravel_index(np.argmax(np.abs(wald_g - wald_o) / np.abs(wald_o)),
                                                             wald_o.shape)
    lr_g, lr_o = res[:, 2:2 + N], ref[:, 2 + N:2 + 2 * N]
    lm_g, lm_o = res[:, 2 + N:2 + 2 * N], ref[:, 2 + 2 * N:2 + 3 * N]
    off = (np.abs(lr_g - lr_o) > STAT_RTOL * np.abs(lr_o)) | (np.abs(lm_g - lm_o) > STAT_RTOL * np.abs(lm_o))
    reps = sorted(set(np.nonzero(off)[0].tolist()))
    assert len(reps) <= B // 4, len(reps)                    # the referee is for the few ill-conditioned cases
    jobs = [(idx[b:b + 1], eta[b:b + 1], bp, [int(i) for i in np.nonzero(off[b])[0]]) for b in reps]
    exact = oracle_pool.run("c2ref", y, w, x, r, "ICp2", None, None, jobs=jobs)
    for (b, (_, _, _, ivs)), ex in zip(zip(reps, jobs), exact):
        for j, i in enumerate(ivs):
            lr_ref, lm_ref = ex[j]
            assert abs(lr_g[b, i] - lr_ref) <= max(STAT_RTOL * abs(lr_ref), abs(lr_o[b, i] - lr_ref),
                                                   T * 1e-14), (b, i, lr_g[b, i], lr_ref, lr_o[b, i])
            assert abs(lm_g[b, i] - lm_ref) <= max(STAT_RTOL * abs(lm_ref), abs(lm_o[b, i] - lm_ref)), \
                (b, i, lm_g[b, i], lm_ref, lm_o[b, i])


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
