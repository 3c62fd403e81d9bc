"""GPU parity for soft-threshold targeted predictors
(src/targeted_predictors.jl:31-36, GLMNet.glmnetcv on [w x]): libdfm's
dfm_targeted_soft against the CPU restatement of glmnet (oracle glmnetcv) and
the committed fixtures (tests/golden/tp_soft.npz, made by
tests/golden/make_golden.py).  PARITY UNPINNED against GLMNet itself (not
importable here, never imported by the reference: defect D5).

Bar: given the same standardised covariance the lasso path is bit-identical
(dfm_lasso_path vs the elnet1 restatement); through the whole glmnetcv (the
device forms its own Grams on MFMA) the selection mask is bit-exact, the CV
path length and the CV-optimal lambda index are equal, the lambda grid agrees
to 1e-12 relative, the hold-out mean losses to 1e-9 relative and the
coefficients at the optimum to 1e-8 of their largest magnitude (coordinate
descent stopped at glmnet's 1e-7 threshold on both sides, same loop order)."""
import os

import numpy as np
import pytest

from test_gpu_parity import ANGLE_TOL, GOLD, STAT_RTOL, max_sin_angle, panel, rel

pytestmark = pytest.mark.gpu
LAM_RTOL = 1e-12
LOSS_RTOL = 1e-9
BETA_TOL = 1e-8
CLEAN = ("relaunches", "timeouts", "task_timeouts", "done_timeouts", "pipe_timeouts", "budget_overruns",
         "late_entries", "slow_launches", "wave_splits")


@pytest.fixture(autouse=True)
def clean_launch_record(dfm):
    """Every lasso launch of every test completes with no timed-out
    leader/helper spin, no relaunch, every workgroup resident, every
    workgroup's waves leaving together and the host's wait no longer than the
    kernel (``lasso_stats``): a hand-off that only completed
    through its timeout, a relaunch that hid one, or waves left spinning after
    their workgroup's wave 0 exited (round 3's 2 s stalls) fail the test."""
    dfm.lasso_stats(reset=True)
    yield
    st = dfm.lasso_stats(reset=True)
    assert {k: st[k] for k in CLEAN} == {k: 0 for k in CLEAN}, st


def check(mask, path, mask_o, lam_o, loss_o, best_o, beta_o):
    assert path["best"] == best_o
    assert len(path["lambda"]) == len(lam_o)
    assert np.max(np.abs(path["lambda"] / lam_o - 1)) < LAM_RTOL
    assert np.max(np.abs(path["meanloss"] / loss_o - 1)) < LOSS_RTOL
    assert np.array_equal(mask, mask_o)
    assert np.max(np.abs(path["beta"] - beta_o)) <= BETA_TOL * np.max(np.abs(beta_o))


def test_golden_soft_small(dfm):
    g = np.load(os.path.join(GOLD, "tp_soft.npz"))
    mask, path = dfm.targeted_predictors(g["y"], g["w"], g["x"], "soft", folds=g["folds"], return_path=True)
    check(mask, path, g["mask"], g["lam"], g["meanloss"], int(g["best"]), g["beta"])
    assert abs(path["a0"] - float(g["a0"])) < 1e-8 * max(1.0, abs(float(g["a0"])))


@pytest.mark.parametrize("T,N,q,nlam,lmr", [
    (200, 40, 2, 100, None),     # T > q + N: lambda_min_ratio 1e-4
    (90, 150, 1, 50, 0.05),      # short grid
    (64, 500, 1, 100, None),     # p >> T
])
def test_soft_matches_oracle(dfm, oracle, T, N, q, nlam, lmr):
    y, x, w = panel(oracle, T, N, 3, 70 + T)
    if q == 2:   # a penalised, non-constant extra regressor (as lags of y would be)
        w = np.hstack([w, np.r_[0.0, y[:-1]][:, None]])
    folds = oracle.glmnet_default_folds(T, np.random.default_rng(T))
    mask_o, res = oracle.targeted_predictors_soft(y, w, x, folds, nlambda=nlam, lambda_min_ratio=lmr)
    mask, path = dfm.targeted_predictors(y, w, x, "soft", folds=folds, nlambda=nlam,
                                         lambda_min_ratio=lmr, return_path=True)
    b = res["best"]
    check(mask, path, mask_o, res["lambda"], res["meanloss"], b, res["betas"][b])


def test_c4_soft_full_size(dfm, oracle):
    """BASELINE configs[3]: T=400, N=5000 candidates (the CPU restatement
    takes ~80 s, so its outputs are the committed fixture; the inputs are
    regenerated from the seed and checked against a digest)."""
    import sys
    sys.path.insert(0, GOLD)
    import make_golden
    g = np.load(os.path.join(GOLD, "tp_soft.npz"))
    y, w, x, folds = make_golden.c4_inputs()
    assert np.allclose([x.sum(), np.abs(x).sum(), y.sum(), folds.sum()], g["c4_digest"], rtol=1e-12, atol=1e-9)
    mask, path = dfm.targeted_predictors(y, w, x, "soft", folds=folds, return_path=True)
    check(mask, path, g["c4_mask"], g["c4_lam"], g["c4_meanloss"], int(g["c4_best"]), g["c4_beta"])


def test_c4_chain_soft_then_pca(dfm, oracle):
    """BASELINE configs[3] as ONE chain, as tools/bench_configs.py c4 times it:
    the device's soft glmnetcv mask (src/targeted_predictors.jl:31-36; equal to
    the frozen fixture bit for bit) selects the columns, then the device PCA
    of the selected columns (src/DynamicFactorModel.jl:75-95, r = 5) against
    the oracle's principal_components of the same columns: eigenvalues and
    trace at the statistic bar, factors and loadings up to sign / principal
    angle.  (The reference's principal-components branch itself ignores the
    targeted_predictors argument, :96-100 — the selection is applied to x.)"""
    import sys
    sys.path.insert(0, GOLD)
    import make_golden
    g = np.load(os.path.join(GOLD, "tp_soft.npz"))
    y, w, x, folds = make_golden.c4_inputs()
    mask = dfm.targeted_predictors(y, w, x, "soft", folds=folds)
    assert np.array_equal(mask, g["c4_mask"]) and mask.sum() > 5
    xs = x[:, mask]
    T, Ns = xs.shape
    k = 5
    ev, F, L, tr = dfm.principal_components(xs, k)
    Fo, Lo, wo = oracle.principal_components(xs, T, Ns)
    assert rel(ev, wo[:k]) < STAT_RTOL
    assert abs(tr - float(np.sum(xs * xs))) <= 1e-12 * abs(tr)
    assert max_sin_angle(F, Fo[:, :k]) < ANGLE_TOL and max_sin_angle(L, Lo[:, :k]) < ANGLE_TOL


def _lasso_inputs(oracle, T, N, seed, lmr=None, nlam=100):
    y, x, w = panel(oracle, T, N, 3, seed)
    Z = np.hstack([w, x])
    mu, sd, ju, yb, ys, G, c = oracle._glmnet_standardize(Z, y)
    lam_max = float(np.max(np.abs(c[ju])))
    if lmr is None:
        lmr = 1e-2 if T < Z.shape[1] else 1e-4
    return G, c, ju, oracle.glmnet_lambdas(lam_max, nlam, lmr)


@pytest.mark.parametrize("T,N,early", [(80, 40, True), (120, 300, True), (60, 700, False), (200, 150, False)])
def test_lasso_path_bit_identical_to_elnet1_restatement(dfm, oracle, T, N, early):
    """Given the same standardised covariance G and c, the device path
    (cooperative leader/helper kernel) is bit-identical to the oracle's
    restatement of glmnet's elnet1: same loop order, same rounding (every
    product and difference rounded separately, sequential dot products)."""
    G, c, ju, alms = _lasso_inputs(oracle, T, N, 90 + N)
    cnt = {}
    bo, ro = oracle.lasso_path_cd(G, c, ju, alms, early, counters=cnt)
    bg, rg = dfm.lasso_path(G, c, ju, alms, early=early)
    assert bg.shape == bo.shape
    assert np.array_equal(bg, bo)
    assert np.array_equal(rg, ro)
    assert cnt["full_passes"] > len(alms) // 2 and np.count_nonzero(bo[-1]) > 10   # entries mid-pass exercised


def test_lasso_path_c4_full_fit_bit_identical(dfm, oracle):
    """BASELINE configs[3] full fit (T=400, p=5001: active set to ~380, ~220
    full passes with in-pass entries) on the oracle's G: bit-identical."""
    import sys
    sys.path.insert(0, GOLD)
    import make_golden
    y, w, x, folds = make_golden.c4_inputs()
    mu, sd, ju, yb, ys, G, c = oracle._glmnet_standardize(np.hstack([w, x]), y)
    alms = oracle.glmnet_lambdas(float(np.max(np.abs(c[ju]))), 100, 1e-2)
    bo, ro = oracle.lasso_path_cd(G, c, ju, alms, True)
    bg, rg = dfm.lasso_path(G, c, ju, alms, early=True)
    assert np.array_equal(bg, bo) and np.array_equal(rg, ro)


def test_lasso_with_another_context_bootstrapping(dfm, oracle):
    """The lasso grid fills the chip and needs every workgroup resident
    (leader/helper hand-offs); a second context's kernels holding CUs would
    leave hand-offs to their timeouts (VERDICT r04 Weak #9).  Here a second
    context bootstraps in another host thread (ctypes releases the GIL) while
    this thread runs the lasso path again and again: the device gate
    (dfm_common.h DeviceShare / DeviceSolo) keeps them apart — every path
    bit-identical to the solo one, the launch record clean (fixture above),
    the concurrent bootstrap rows equal to its solo rows."""
    import threading
    G, c, ju, alms = _lasso_inputs(oracle, 120, 300, 390)
    ref_b, ref_r = dfm.lasso_path(G, c, ju, alms, early=True)
    y, x, w = panel(oracle, 150, 900, 3, 5)
    m = dfm.DynamicFactorModel(y, w, x, 3, ctx=dfm.Context(0))
    idx, eta = dfm.draw_wild(np.random.default_rng(2), 700, 150)
    ref_rows = dfm.wild_bootstrap(m, 700, [dfm.Stat.V(), dfm.Stat.eigenvalue(1)], idx=idx, eta=eta)
    stop, rows, errs = threading.Event(), [], []

    def boot():
        try:
            while not stop.is_set():
                rows.append(dfm.wild_bootstrap(m, 700, [dfm.Stat.V(), dfm.Stat.eigenvalue(1)], idx=idx, eta=eta))
        except Exception as e:   # (reported below, on the test's thread)
            errs.append(e)

    th = threading.Thread(target=boot)
    th.start()
    try:
        for _ in range(12):
            bg, rg = dfm.lasso_path(G, c, ju, alms, early=True)
            assert np.array_equal(bg, ref_b) and np.array_equal(rg, ref_r)
    finally:
        stop.set()
        th.join(timeout=60)
    assert not errs, errs
    assert len(rows) >= 2
    for r in rows:
        assert np.array_equal(r, ref_rows)


def test_soft_rejects_bad_folds(dfm, oracle):
    y, x, w = panel(oracle, 60, 30, 2, 1)
    with pytest.raises(dfm.DFMError):
        dfm.targeted_predictors(y, w, x, "soft", folds=np.ones(60, dtype=np.int32))   # one fold
    f = oracle.glmnet_default_folds(60, np.random.default_rng(0))
    f[3] = 0
    with pytest.raises(dfm.DFMError):
        dfm.targeted_predictors(y, w, x, "soft", folds=f)


def test_soft_repeated_calls_are_clean_and_stable(dfm, oracle):
    """Round 3's intermittent 2 s stall (a fold leader's waves 1..7 spinning
    until the timeout after wave 0 had left) showed up in ~1 of
    6 back-to-back calls of this p = 42 case.  200 calls in one process: the
    same mask each time, no call slower than 20x the median, and the launch
    record (fixture above) clean."""
    import time
    T, N = 200, 40
    y, x, w = panel(oracle, T, N, 3, 70 + T)
    w = np.hstack([w, np.r_[0.0, y[:-1]][:, None]])
    folds = oracle.glmnet_default_folds(T, np.random.default_rng(T))
    ref = dfm.targeted_predictors(y, w, x, "soft", folds=folds)
    times = []
    for _ in range(200):
        t0 = time.perf_counter()
        mask = dfm.targeted_predictors(y, w, x, "soft", folds=folds)
        times.append(time.perf_counter() - t0)
        assert np.array_equal(mask, ref)
    assert max(times) < 20 * np.median(times), (max(times), np.median(times), dfm.lasso_stats())
