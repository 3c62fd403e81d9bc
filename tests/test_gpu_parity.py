"""GPU parity: libdfm (through its C ABI) vs the CPU oracle and the golden
fixtures.  Tolerances are the north star's (BASELINE.json): statistics and
criteria within 1e-10 relative in fp64; factors equal up to sign with max
principal angle < 1e-8; resample indices are host-generated and shared
(bit-exact by construction)."""
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
STAT_RTOL = 1e-10
ANGLE_TOL = 1e-8


def rel(a, b):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300)))


def lm_within(got, d, bp, vs, oracle):
    """LM_test values `got` (variables vs, 0-based) of the ORACLE's fit d
    against the double-double referee of that fit (oracle/dfm_xp.py
    lm_referee): within 1e-10 of it, or no further from it than the oracle's
    fp64 T (1 - |v|^2/|E_i|^2) form is (that form loses ~eps / R^2 relative
    when R^2 is small).  Only the oracle's fit enters the bar."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
    import dfm_xp
    for g, i in zip(np.atleast_1d(got), vs):
        ref = dfm_xp.lm_referee(d.F, d.factor_residuals[:, i], bp)
        orc = oracle.LM_test(d, bp, i)
        bar = max(STAT_RTOL * abs(ref), abs(orc - ref))
        assert abs(g - ref) <= bar, (i, g, ref, orc)


def lr_within(got, d, bp, vs, oracle):
    """LR_test values `got` (variables vs, 0-based) of the ORACLE's fit d
    against the double-double referee of that fit (oracle/dfm_xp.py
    lr_referee): within 1e-10 of it, or no further from it than the oracle's
    fp64 projections are, or within T * 1e-14 absolute — LR = T log(SSR_r /
    SSR_u) and an fp64 ratio carries a few ulps (~1e-15 relative) whatever
    computes it, so no fp64 evaluation of a near-zero LR can do better.  Only
    the oracle's fit enters the bar."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
    import dfm_xp
    for g, i in zip(np.atleast_1d(got), vs):
        ref = dfm_xp.lr_referee(d.F, d.x[:, i], d.factor_residuals[:, i], bp)
        orc = oracle.LR_test(d, bp, i)
        floor = d.F.shape[0] * 1e-14
        assert abs(g - ref) <= max(STAT_RTOL * abs(ref), abs(orc - ref), floor), (i, g, ref, orc)


def max_sin_angle(A, B):
    """sin of the largest principal angle between span(A) and span(B)."""
    Qa, _ = np.linalg.qr(A)
    Qb, _ = np.linalg.qr(B)
    return float(np.linalg.norm(Qa - Qb @ (Qb.T @ Qa), 2))


def column_angles(A, B):
    """Per-factor angles (columns matched in order, sign-free)."""
    out = []
    for j in range(A.shape[1]):
        a = A[:, j] / np.linalg.norm(A[:, j])
        b = B[:, j] / np.linalg.norm(B[:, j])
        b = b * np.sign(a @ b)
        out.append(float(np.linalg.norm(a - b)))
    return np.array(out)


def signs(F, Fo):
    s = np.sign(np.sum(F * Fo, axis=0))
    s[s == 0] = 1
    return s


def panel(oracle, T, N, r, seed, model="Bai_Ng_2002", **kw):
    rng = np.random.default_rng(seed)
    out = oracle.factor_model_DGP(T, N, r, rng, model=model, **kw)
    return out[0], oracle.normalize(out[1]), np.ones((T, 1))


def assert_fit_matches(g, o, oracle, q=1):
    r = o.number_of_factors
    assert g.number_of_factors == r
    assert rel(g.eigenvalues[:r], o.eigenvalues[0][:r]) < STAT_RTOL
    Fo = o.F
    assert max_sin_angle(g.factors[0], Fo) < ANGLE_TOL
    assert np.all(column_angles(g.factors[0], Fo) < ANGLE_TOL)
    s = signs(g.factors[0], Fo)
    assert rel(g.factors[0] * s, Fo) < 1e-8
    assert abs(g.V - oracle.factor_residual_variance(o)) < STAT_RTOL * oracle.factor_residual_variance(o)
    cg = g.coefficients.copy()
    cg[q:] *= s
    tg = g.t_stats.copy()
    tg[q:] *= s
    assert rel(cg, o.coefficients) < STAT_RTOL
    assert rel(tg, o.t_stats) < STAT_RTOL
    assert np.max(np.abs(g.factor_residuals - o.factor_residuals)) < 1e-9 * np.max(np.abs(o.factor_residuals))
    if o.number_of_factors_criterion:
        assert abs(g.number_of_factors_criterion_value - o.number_of_factors_criterion_value) <= \
            STAT_RTOL * abs(o.number_of_factors_criterion_value)


# ------------------------------------------------------------------ fixtures
def test_golden_c1_fit(dfm, oracle):
    g = np.load(os.path.join(GOLD, "c1_bai_ng_T200_N100_r3.npz"))
    d = dfm.DynamicFactorModel(g["y"], g["w"], g["x"], int(g["r"]), "ICp2")
    assert rel(d.eigenvalues[:3], g["eigvals"][:3]) < STAT_RTOL
    assert max_sin_angle(d.factors[0], g["F"]) < ANGLE_TOL
    s = signs(d.factors[0], g["F"])
    c = d.coefficients.copy(); c[1:] *= s
    t = d.t_stats.copy(); t[1:] *= s
    assert rel(c, g["coefficients"]) < STAT_RTOL and rel(t, g["t_stats"]) < STAT_RTOL
    assert abs(d.V - float(g["V"])) < STAT_RTOL * float(g["V"])
    assert abs(d.number_of_factors_criterion_value - float(g["crit_ICp2"])) < STAT_RTOL * abs(float(g["crit_ICp2"]))
    assert np.allclose(d.residuals, g["residuals"], rtol=0, atol=1e-10 * np.abs(g["residuals"]).max())


def test_golden_c1_ic_sweep(dfm):
    g = np.load(os.path.join(GOLD, "c1_bai_ng_T200_N100_r3.npz"))
    d = dfm.DynamicFactorModel(g["y"], g["w"], g["x"], "ICp2", kmax=8)
    assert d.number_of_factors == int(g["ic_best_r"]) == 3
    assert rel(d.ic_values, g["ic_values"]) < STAT_RTOL


@pytest.mark.parametrize("crit", ["PCp1", "PCp2", "PCp3", "ICp1", "ICp3", "BIC"])
def test_golden_c1_ic_sweep_every_criterion(dfm, crit):
    g = np.load(os.path.join(GOLD, "c1_bai_ng_T200_N100_r3.npz"))
    d = dfm.DynamicFactorModel(g["y"], g["w"], g["x"], crit, kmax=8)
    row = list(dfm.CRITERIA).index(crit)
    assert d.number_of_factors == int(np.argmin(g["ic_values"][row])) + 1
    assert abs(d.number_of_factors_criterion_value - g["ic_values"][row, d.number_of_factors - 1]) \
        <= STAT_RTOL * abs(g["ic_values"][row, d.number_of_factors - 1])


def test_golden_c2_base_and_chow(dfm):
    g = np.load(os.path.join(GOLD, "c2_breitung_eickmeier_T600_N130_B16.npz"))
    d = dfm.DynamicFactorModel(g["y"], g["w"], g["x"], "ICp2", kmax=8)
    assert d.number_of_factors == int(g["r"])
    assert abs(d.V - float(g["base_V"])) < STAT_RTOL * float(g["base_V"])
    LR, LM, W = dfm.chow_all(d, int(g["bp"]))
    assert rel(LR, g["base_chow"][:, 0]) < STAT_RTOL
    assert rel(LM, g["base_chow"][:, 1]) < STAT_RTOL
    assert rel(W, g["base_chow"][:, 2]) < STAT_RTOL
    assert abs(dfm.LR_test(d, int(g["bp"]), 5) - g["base_chow"][4, 0]) < STAT_RTOL * abs(g["base_chow"][4, 0])


def test_golden_c2_wild_bootstrap(dfm):
    g = np.load(os.path.join(GOLD, "c2_breitung_eickmeier_T600_N130_B16.npz"))
    d = dfm.DynamicFactorModel(g["y"], g["w"], g["x"], "ICp2", kmax=8)
    bp, nv = int(g["bp"]), int(g["nv"])
    S = dfm.Stat
    stats = [S.V(), S.criterion()] + [S.LR(bp, i + 1) for i in range(nv)] + \
        [S.LM(bp, i + 1) for i in range(nv)] + [S.Wald(bp, i + 1) for i in range(nv)]
    out = dfm.wild_bootstrap(d, 16, stats, idx=g["idx"], eta=g["eta"])
    assert rel(out[:, :2], g["boot"][:, :2]) < STAT_RTOL
    assert rel(out[:, 2:], g["boot"][:, 2:]) < STAT_RTOL
    # the all-variables form gives the same numbers
    allv = dfm.wild_bootstrap(d, 16, [S.LR_all(bp), S.LM_all(bp), S.Wald_all(bp)], idx=g["idx"], eta=g["eta"])
    N = g["x"].shape[1]
    assert np.array_equal(allv[:, :nv], out[:, 2:2 + nv])
    assert np.array_equal(allv[:, 2 * N:2 * N + nv], out[:, 2 + 2 * nv:])


def test_golden_targeted(dfm):
    g = np.load(os.path.join(GOLD, "tp_hard.npz"))
    m, t = dfm.targeted_predictors(g["y"], g["w"], g["x"], return_tstats=True)
    assert rel(t, g["t_joint"]) < STAT_RTOL and np.array_equal(m, g["m_joint"])
    m2, t2 = dfm.targeted_predictors(g["y2"], g["w2"], g["x2"], mode="per_candidate", return_tstats=True)
    assert rel(t2, g["t_cand"]) < STAT_RTOL and np.array_equal(m2, g["m_cand"])


# -------------------------------------------------- oracle on seeded inputs
@pytest.mark.parametrize("T,N,r,crit", [
    (200, 100, 3, "ICp2"),      # C1 shape, T >= N branch
    (120, 120, 2, "BIC"),       # T == N takes the T >= N branch (:77)
    (60, 150, 4, "ICp1"),       # N > T branch
    (500, 2000, 8, "ICp2"),     # C3 shape
    (12, 9, 2, "ICp3"),         # m < the eigensolver block (p = m)
    (10, 25, 1, ""),            # r = 1, no criterion (D3: NaN)
])
def test_fit_matches_oracle(dfm, oracle, T, N, r, crit):
    y, x, w = panel(oracle, T, N, r, 1000 + T + N)
    g = dfm.DynamicFactorModel(y, w, x, r, crit)
    o = oracle.DynamicFactorModel(y, w, x, r, crit)
    assert_fit_matches(g, o, oracle)
    if not crit:
        assert math.isnan(g.number_of_factors_criterion_value)


def test_fit_with_extra_regressors(dfm, oracle):
    """w = [1, y_{t-1..t-4}] as in test/DynamicFactorModel.jl:13-18."""
    rng = np.random.default_rng(11)
    y, x, *_ = oracle.factor_model_DGP(204, 80, 3, rng)
    x = oracle.normalize(x)[4:]
    yl = np.column_stack([y[4 - k:-k] for k in range(1, 5)])
    w = np.hstack([np.ones((200, 1)), yl])
    y = y[4:]
    g = dfm.DynamicFactorModel(y, w, x, 3, "ICp2")
    o = oracle.DynamicFactorModel(y, w, x, 3, "ICp2")
    assert_fit_matches(g, o, oracle, q=5)


def test_exact_rank_panel(dfm):
    rng = np.random.default_rng(12)
    T, N, r = 40, 20, 3
    x = rng.standard_normal((T, r)) @ rng.standard_normal((N, r)).T
    d = dfm.DynamicFactorModel(rng.standard_normal(T), np.ones((T, 1)), x, r)
    assert abs(d.V) < 1e-26 * np.sum(x * x)
    assert np.max(np.abs(d.factor_residuals)) < 1e-10


def test_r_clamped_to_half_min(dfm, oracle):
    """src/DynamicFactorModel.jl:116-119."""
    y, x, w = panel(oracle, 30, 8, 2, 13)
    d = dfm.DynamicFactorModel(y, w, x, 7)
    assert d.number_of_factors == 4


def test_principal_components_and_spectrum(dfm, oracle):
    for T, N in [(150, 60), (60, 150)]:
        _, x, _ = panel(oracle, T, N, 4, 14)
        ev, F, L, tr = dfm.principal_components(x, 5)
        Fo, Lo, wo = oracle.principal_components(x, T, N)
        assert rel(ev, wo[:5]) < STAT_RTOL
        assert max_sin_angle(F, Fo[:, :5]) < ANGLE_TOL
        assert rel(L * signs(F, Fo[:, :5]), Lo[:, :5]) < 1e-8
        full, tr2 = dfm.gram_spectrum(x)
        assert rel(full[:40], wo[:40]) < STAT_RTOL
        assert abs(tr - np.sum(x * x)) < 1e-12 * tr


def test_ic_sweep_default_kmax(dfm, oracle):
    """kmax = ceil(m/2) (src/DynamicFactorModel.jl:54) with m <= 140."""
    y, x, w = panel(oracle, 80, 30, 2, 15)
    d = dfm.DynamicFactorModel(y, w, x, "ICp2")
    o = oracle.DynamicFactorModel_ic(y, w, x, "ICp2")
    assert d.number_of_factors == o.number_of_factors
    assert abs(d.number_of_factors_criterion_value - o.number_of_factors_criterion_value) < \
        STAT_RTOL * abs(o.number_of_factors_criterion_value)


@pytest.mark.parametrize("T,N,r,mode", [(200, 100, 3, "auto"), (60, 150, 4, "direct"),
                                        (60, 150, 4, "factored"), (37, 101, 3, "factored")])
def test_wild_bootstrap_matches_oracle(dfm, oracle, T, N, r, mode):
    y, x, w = panel(oracle, T, N, r, 2000 + T)
    g = dfm.DynamicFactorModel(y, w, x, r, "ICp2")
    g.set_bootstrap_mode(mode)
    o = oracle.DynamicFactorModel(y, w, x, r, "ICp2")
    B = 6
    idx, eta = oracle.draw_wild(np.random.default_rng(3), B, T)
    S = dfm.Stat
    stats = [S.V(), S.criterion(), S.criterion("BIC"), S.eigenvalue(1), S.eigenvalue(r), S.trace(),
             S.coefficient(1), S.t_stat(1)]
    out = dfm.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
    for b in range(B):
        xs = o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]]
        d = oracle.DynamicFactorModel(y, w, xs, r, "ICp2")
        ref = [oracle.factor_residual_variance(d), d.number_of_factors_criterion_value,
               oracle.criterion_value("BIC", d), d.eigenvalues[0][0], d.eigenvalues[0][r - 1],
               np.sum(xs * xs), d.coefficients[0], d.t_stats[0]]
        assert rel(out[b, :6], ref[:6]) < STAT_RTOL
        assert rel(out[b, 6:], ref[6:]) < STAT_RTOL      # w-column coef/t: sign-invariant


@pytest.mark.parametrize("mode", ["factored", "direct"])
def test_wild_bootstrap_exact_rank_panel(dfm, oracle, mode):
    """Replicates of an exact rank-3 panel: the factor residuals vanish, so every
    replicate Gram has rank 3 and the Rayleigh-Ritz block (width > 3) runs
    on rank-deficient Q'Q — the dead-pivot path of the in-register Cholesky and
    its random refill.  Eigenvalues against the oracle; V at the rounding floor."""
    rng = np.random.default_rng(31)
    T, N, r = 60, 40, 3
    x = rng.standard_normal((T, r)) @ rng.standard_normal((N, r)).T
    y, w = rng.standard_normal(T), np.ones((T, 1))
    g = dfm.DynamicFactorModel(y, w, x, r)
    g.set_bootstrap_mode(mode)
    o = oracle.DynamicFactorModel(y, w, x, r)
    B = 4
    idx, eta = oracle.draw_wild(np.random.default_rng(6), B, T)
    S = dfm.Stat
    out = dfm.wild_bootstrap(g, B, [S.V(), S.eigenvalue(1), S.eigenvalue(r), S.trace()], idx=idx, eta=eta)
    assert np.all(np.isfinite(out))
    for b in range(B):
        xs = o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]]
        d = oracle.DynamicFactorModel(y, w, xs, r)
        tr = np.sum(xs * xs)
        assert abs(out[b, 0]) < 1e-12 * tr / (N * T)
        assert rel(out[b, 1:3], [d.eigenvalues[0][0], d.eigenvalues[0][r - 1]]) < STAT_RTOL
        assert rel(out[b, 3], tr) < 1e-12


@pytest.mark.parametrize("T,N", [(150, 70), (70, 150)])
def test_residual_bootstrap_matches_oracle(dfm, oracle, T, N):
    y, x, w = panel(oracle, T, N, 2, 16)
    g = dfm.DynamicFactorModel(y, w, x, 2, "ICp1")
    o = oracle.DynamicFactorModel(y, w, x, 2, "ICp1")
    idx = oracle.draw_residual(np.random.default_rng(4), 5, T)
    out = dfm.residual_bootstrap(g, 5, [dfm.Stat.V(), dfm.Stat.criterion()], idx=idx)
    ref = oracle.residual_bootstrap(o, 5, lambda d: oracle.factor_residual_variance(d), idx)
    assert rel(out[:, 0], ref) < STAT_RTOL


# N = 24: one thread per variable per replicate block; N = 90, 120: the flat
# (replicate, variable) mapping, blocks spanning up to 4 replicates (dfm_chow.hip)
@pytest.mark.parametrize("T,N", [(160, 24), (80, 120), (100, 90)])
def test_bootstrap_chow_all_matches_oracle(dfm, oracle, T, N):
    y, x, w = panel(oracle, T, N, 2, 17, model="Breitung_Eickmeier_2011", b=0.5)
    g = dfm.DynamicFactorModel(y, w, x, 2)
    o = oracle.DynamicFactorModel(y, w, x, 2)
    B = 6   # N = 90: the second 256-thread block spans replicates 2..5
    idx, eta = oracle.draw_wild(np.random.default_rng(5), B, T)
    S = dfm.Stat
    bp = T // 2
    out = dfm.wild_bootstrap(g, B, [S.LR_all(bp), S.LM_all(bp), S.Wald_all(bp)], idx=idx, eta=eta)
    vs = np.array(sorted(set(range(min(N, 12))) | set(range(max(0, N - 12), N))))   # both panel edges
    for b in range(B):
        d = oracle.DynamicFactorModel(y, w, o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]], 2)
        ref = np.array([[oracle.LR_test(d, bp, i), oracle.LM_test(d, bp, i), oracle.Wald_test(d, bp, i)]
                        for i in vs])
        assert rel(out[b, vs], ref[:, 0]) < STAT_RTOL
        lm_within(out[b, N + vs], d, bp, vs, oracle)
        assert rel(out[b, 2 * N + vs], ref[:, 2]) < STAT_RTOL


@pytest.mark.parametrize("T,N,breaks", [(80, 120, []), (160, 24, []), (120, 60, [61])])
def test_bootstrap_host_closure_matches_oracle_loop(dfm, oracle, T, N, breaks):
    """The reference's `stat::Function` (src/bootstrap.jl:21, :41) as a host
    closure: the device refits every replicate and returns its factors,
    loadings, eigenvalues, coefficients and t-statistics (DFM_STAT_FACTORS /
    LOADINGS); the closure then runs on the rebuilt record — here the
    oracle's own LR_test and factor_residual_variance, exactly as the
    reference's loop would call them — against the oracle's loop."""
    r = 2
    y, x, w = panel(oracle, T, N, r, 41, model="Breitung_Eickmeier_2011", b=0.5)
    g = dfm.DynamicFactorModel(y, w, x, r, "ICp2", break_indices=breaks)
    o = oracle.DynamicFactorModel(y, w, x, r, "ICp2", breaks)
    B, bp = 3, T // 2 + 3
    idx, eta = oracle.draw_wild(np.random.default_rng(8), B, T)
    lr = dfm.wild_bootstrap(g, B, lambda d: oracle.LR_test(d, bp, 2), idx=idx, eta=eta)
    V = dfm.wild_bootstrap(g, B, oracle.factor_residual_variance, idx=idx, eta=eta)
    reps = []
    dfm.wild_bootstrap(g, B, lambda d: reps.append(d) or 0.0, idx=idx, eta=eta)
    assert lr.shape == (B,) and V.shape == (B,)
    for b in range(B):
        d = oracle.DynamicFactorModel(y, w, o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]],
                                      r, "ICp2", breaks)
        lr_within([lr[b]], d, bp, [2], oracle)
        assert rel(V[b], oracle.factor_residual_variance(d)) < STAT_RTOL
        rep = reps[b]
        assert len(rep.factors) == len(d.factors) == len(breaks) + 1
        assert max_sin_angle(rep.F, d.F) < ANGLE_TOL
        assert np.max(np.abs(rep.x - d.x)) < 1e-12 * np.max(np.abs(d.x))
        s = signs(rep.F, d.F)
        assert rel(rep.coefficients[1:] * s, d.coefficients[1:]) < STAT_RTOL
        assert rel(rep.t_stats[1:] * s, d.t_stats[1:]) < STAT_RTOL
        cs = np.concatenate([[1.0], s])   # the HC2 covariance rebuilt on the host (:43-46), factor signs applied
        assert rel(rep.coefficient_covariance * np.outer(cs, cs), d.coefficient_covariance) < 1e-9


@pytest.mark.parametrize("T,N,breaks", [(120, 60, [61]), (90, 140, [40]), (80, 120, [])])
def test_residual_bootstrap_host_closure(dfm, oracle, T, N, breaks):
    """The residual bootstrap's closure path (src/bootstrap.jl:21-39): X*_b =
    C + E[idx_b] with idx_b drawn WITHIN each break block (:23-28), refit per
    block; every block's loadings (DFM_STAT_LOADINGS, copied per block out of
    the replicate's loadings slab) against the oracle's refit, up to sign and
    principal angle, and a closure statistic against the oracle's loop."""
    r = 2
    y, x, w = panel(oracle, T, N, r, 57, model="Breitung_Eickmeier_2011", b=0.5)
    g = dfm.DynamicFactorModel(y, w, x, r, "ICp2", break_indices=breaks)
    o = oracle.DynamicFactorModel(y, w, x, r, "ICp2", breaks)
    B = 3
    idx = oracle.draw_residual(np.random.default_rng(12), B, T, breaks)
    reps = []
    V = dfm.residual_bootstrap(g, B, lambda d: reps.append(d) or oracle.factor_residual_variance(d), idx=idx)
    for b in range(B):
        d = oracle.DynamicFactorModel(y, w, o.common_component + o.factor_residuals[idx[b]], r, "ICp2", breaks)
        rep = reps[b]
        assert rel(V[b], oracle.factor_residual_variance(d)) < STAT_RTOL
        assert np.max(np.abs(rep.x - d.x)) < 1e-12 * np.max(np.abs(d.x))
        assert len(rep.loadings) == len(d.loadings) == len(breaks) + 1
        for Lg, Lo in zip(rep.loadings, d.loadings):
            assert max_sin_angle(Lg, Lo[:, :r]) < ANGLE_TOL
            sj = signs(Lg, Lo[:, :r])
            assert rel(Lg * sj, Lo[:, :r]) < 1e-9
        for Fg, Fo in zip(rep.factors, d.factors):
            assert max_sin_angle(Fg, Fo[:, :r]) < ANGLE_TOL


@pytest.mark.parametrize("T,N", [(80, 120), (160, 24)])
def test_bootstrap_chow_with_block_equal_r(dfm, oracle, T, N):
    """A requested eigen block of r (dfm_ctx_set_eig_params block = r): the
    library raises it to r + 1 — with p == r the subspace convergence rule
    has no unwanted Ritz value to measure a gap against (it now falls back to
    the neighbour gaps) and the Chebyshev filter's interval reaches the r-th
    wanted eigenvalue, which then never converges.  A Chow-only call (the
    subspace rule) with the smallest block: replicates against the oracle at
    the usual bar."""
    r = 3   # (Bai-Ng strong factors: without guard vectors the block converges at lambda_4 / lambda_3 per step)
    y, x, w = panel(oracle, T, N, r, 23)
    ctx = dfm.Context(0)
    ctx.set_eig_params(block=r)
    g = dfm.DynamicFactorModel(y, w, x, r, ctx=ctx)
    o = oracle.DynamicFactorModel(y, w, x, r)
    B, bp = 4, T // 2 + 3
    idx, eta = oracle.draw_wild(np.random.default_rng(31), B, T)
    S = dfm.Stat
    out = dfm.wild_bootstrap(g, B, [S.LR_all(bp), S.Wald_all(bp)], idx=idx, eta=eta)
    vs = np.arange(min(N, 10))
    for b in range(B):
        d = oracle.DynamicFactorModel(y, w, o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]], r)
        lr_within(out[b, vs], d, bp, vs, oracle)
        assert rel(out[b, N + vs], [oracle.Wald_test(d, bp, i) for i in vs]) < STAT_RTOL


# -------------------------------------- full-size (C3) size-independent props
@pytest.mark.parametrize("mode", ["direct", "factored"])
def test_c3_identity_draw_reproduces_base(dfm, oracle, mode):
    """At T=500, N=2000, r=8: idx = identity, eta = 1 rebuilds X exactly, so
    every replicate must reproduce the base fit's V and eigenvalues."""
    y, x, w = panel(oracle, 500, 2000, 8, 18)
    g = dfm.DynamicFactorModel(y, w, x, 8, "ICp2")
    g.set_bootstrap_mode(mode)
    B = 32
    idx = np.tile(np.arange(500, dtype=np.int32), (B, 1))
    eta = np.ones((B, 500))
    out = dfm.wild_bootstrap(g, B, [dfm.Stat.V(), dfm.Stat.eigenvalue(1), dfm.Stat.eigenvalue(8)],
                             idx=idx, eta=eta)
    assert rel(out[:, 0], np.full(B, g.V)) < 1e-11
    assert rel(out[:, 1], np.full(B, g.eigenvalues[0])) < 1e-12
    assert rel(out[:, 2], np.full(B, g.eigenvalues[7])) < 1e-12


@pytest.mark.parametrize("mode", ["direct", "factored"])
def test_c3_replicates_match_oracle(dfm, oracle, mode):
    y, x, w = panel(oracle, 500, 2000, 8, 19)
    g = dfm.DynamicFactorModel(y, w, x, 8, "ICp2")
    g.set_bootstrap_mode(mode)
    o = oracle.DynamicFactorModel(y, w, x, 8, "ICp2")
    idx, eta = oracle.draw_wild(np.random.default_rng(6), 3, 500)
    out = dfm.wild_bootstrap(g, 3, [dfm.Stat.V(), dfm.Stat.criterion(), dfm.Stat.t_stat(1)],
                             idx=idx, eta=eta)
    ref = np.array([[oracle.factor_residual_variance(d), d.number_of_factors_criterion_value, d.t_stats[0]]
                    for d in [oracle.DynamicFactorModel(y, w, o.common_component + eta[b][:, None] *
                                                        o.factor_residuals[idx[b]], 8, "ICp2")
                              for b in range(3)]])
    assert rel(out[:, :2], ref[:, :2]) < STAT_RTOL
    assert rel(out[:, 2], ref[:, 2]) < STAT_RTOL


@pytest.mark.parametrize("mode", ["direct", "factored"])
def test_c3_value_only_stopping_rule(dfm, oracle, mode):
    """Eigenvalue-only statistics stop the eigensolver on the Kato-Temple
    eigenvalue bound (dfm_ctx_set_value_tol): V, criteria, eigenvalues and the
    trace must still match the oracle within STAT_RTOL at C3 size, and the
    strict (eigenvector-residual) rule within 1e-11."""
    y, x, w = panel(oracle, 500, 2000, 8, 23)
    g = dfm.DynamicFactorModel(y, w, x, 8, "ICp2")
    g.set_bootstrap_mode(mode)
    o = oracle.DynamicFactorModel(y, w, x, 8, "ICp2")
    B = 4
    idx, eta = oracle.draw_wild(np.random.default_rng(8), B, 500)
    S = dfm.Stat
    stats = [S.V(), S.criterion(), S.criterion("BIC"), S.trace()] + [S.eigenvalue(j) for j in range(1, 9)]
    out = dfm.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
    for b in range(B):
        xs = o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]]
        d = oracle.DynamicFactorModel(y, w, xs, 8, "ICp2")
        ref = [oracle.factor_residual_variance(d), d.number_of_factors_criterion_value,
               oracle.criterion_value("BIC", d), np.sum(xs * xs)] + list(d.eigenvalues[0][:8])
        assert rel(out[b], ref) < STAT_RTOL
    ctx = g._ctx
    ctx.set_value_tol(0.0)
    try:
        strict = dfm.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
    finally:
        ctx.set_value_tol(1e-12)
    assert rel(out, strict) < 1e-11


@pytest.mark.parametrize("mode", ["direct", "factored"])
def test_batching_is_bit_identical(dfm, oracle, mode):
    """Per-replicate results do not depend on batch composition — the property
    behind bit-identical 1-GPU vs 8-GPU sharding."""
    y, x, w = panel(oracle, 200, 300, 4, 20)
    g = dfm.DynamicFactorModel(y, w, x, 4, "ICp2")
    g.set_bootstrap_mode(mode)
    B = 24
    idx, eta = dfm.draw_wild_fast(7, B, 200)
    stats = [dfm.Stat.V(), dfm.Stat.criterion(), dfm.Stat.t_stat(2)]
    g.set_batch(24)
    a = dfm.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
    g.set_batch(5)
    b = dfm.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
    c = dfm.wild_bootstrap(g, 8, stats, idx=idx[16:], eta=eta[16:])
    assert np.array_equal(a, b)
    assert np.array_equal(a[16:], c)


# ----------------------------------------------------------- error behaviour
def test_direct_and_factored_agree(dfm, oracle):
    """The two N > T algorithms give the same replicates to rounding, incl.
    per-variable Chow statistics (which read the factored loadings)."""
    y, x, w = panel(oracle, 120, 400, 3, 22, model="Breitung_Eickmeier_2011", b=0.3)
    g = dfm.DynamicFactorModel(y, w, x, 3, "ICp2")
    idx, eta = dfm.draw_wild_fast(9, 40, 120)
    S = dfm.Stat
    stats = [S.V(), S.criterion(), S.eigenvalue(3), S.t_stat(1), S.LR_all(60), S.Wald_all(60)]
    g.set_bootstrap_mode("direct")
    a = dfm.wild_bootstrap(g, 40, stats, idx=idx, eta=eta)
    g.set_bootstrap_mode("factored")
    b = dfm.wild_bootstrap(g, 40, stats, idx=idx, eta=eta)
    assert rel(b[:, :4], a[:, :4]) < STAT_RTOL
    assert rel(b[:, 4:], a[:, 4:]) < STAT_RTOL


def test_direct_and_factored_agree_at_large_T(dfm, oracle):
    """T = 3300 (the factored solver's prep and last Horner step then need more
    than 64 KB of dynamic LDS: 24 T + 8 and 20 T + 4 bytes) against the direct
    (Gram-forming) path on the same draws (src/bootstrap.jl:41-51)."""
    y, x, w = panel(oracle, 3300, 3600, 3, 23)
    g = dfm.DynamicFactorModel(y, w, x, 3, "ICp2")
    idx, eta = dfm.draw_wild_fast(10, 6, 3300)
    stats = [dfm.Stat.V(), dfm.Stat.criterion(), dfm.Stat.eigenvalue(1), dfm.Stat.eigenvalue(3)]
    g.set_bootstrap_mode("direct")
    a = dfm.wild_bootstrap(g, 6, stats, idx=idx, eta=eta)
    g.set_bootstrap_mode("factored")
    assert g.fact_block()[0] > 0
    b = dfm.wild_bootstrap(g, 6, stats, idx=idx, eta=eta)
    assert np.all(np.isfinite(b)) and rel(b, a) < STAT_RTOL


@pytest.mark.parametrize("T,N,P,crit,kmax", [
    (60, 150, 6, "ICp2", 6), (90, 30, 5, "BIC", 6), (41, 300, 3, "ICp1", 6),
    (60, 150, 6, "PCp2", 6), (200, 160, 4, "PCp1", 6),
    # the constructor's default kmax_w = ceil(m_w/2) per window (:54): 28..30
    # for N > T (full spectra + dense eigenpairs), 20 / 35 for T >= N
    (60, 150, 5, "ICp2", None), (140, 40, 6, "BIC", None), (200, 70, 4, "PCp2", None)])
def test_expanding_window_refits(dfm, oracle, T, N, P, crit, kmax):
    """src/utils.jl:54-72 refit loop: each window = IC-sweep constructor on rows
    1..date_index-1 (N > T via the prefix-Gram identity)."""
    y, x, w = panel(oracle, T, N, 3, 3000 + T)
    out = dfm.pseudo_out_of_sample_refits(y, w, x, crit, num_predictions=P, kmax=kmax)
    fits = oracle.expanding_window_refits(y, w, x, P, lambda yy, ww, xx: oracle.DynamicFactorModel_ic(
        yy, ww, xx, crit, kmax=kmax))
    for j, o in enumerate(fits):
        assert out["number_of_factors"][j] == o.number_of_factors
        assert abs(out["criterion_value"][j] - o.number_of_factors_criterion_value) <= \
            STAT_RTOL * abs(o.number_of_factors_criterion_value)
        assert abs(out["V"][j] - oracle.factor_residual_variance(o)) <= STAT_RTOL * oracle.factor_residual_variance(o)
        r = o.number_of_factors
        assert rel(out["eigenvalues"][j][:r], o.eigenvalues[0][:r]) < STAT_RTOL
        assert rel(out["t_stats"][j][:1], o.t_stats[:1]) < STAT_RTOL       # intercept: sign-invariant


def test_errors_are_reported(dfm, oracle):
    y, x, w = panel(oracle, 50, 20, 2, 21)
    g = dfm.DynamicFactorModel(y, w, x, 2, "PCp2")
    idx, eta = oracle.draw_wild(np.random.default_rng(0), 2, 50)
    with pytest.raises(dfm.DFMError):      # break period leaves < r rows
        dfm.chow_all(g, 1)
    with pytest.raises(dfm.DFMError):      # D8: joint thresholding singular
        dfm.targeted_predictors(y, w, np.random.default_rng(0).standard_normal((50, 60)))
    with pytest.raises(dfm.DFMError):
        dfm.wild_bootstrap(g, 1, dfm.Stat.V(), idx=np.full((1, 50), 99, dtype=np.int32), eta=eta[:1])


@pytest.mark.parametrize("r,mode", [(11, "direct"), (11, "factored"), (12, "direct"), (12, "factored")])
def test_ols_width_boundary(dfm, oracle, r, mode):
    """OLS + HC2 (src/DynamicFactorModel.jl:40-48) at the boundary of the
    one-wave MFMA kernel: q + r = 15 (d + 1 = 16 columns with y: one wave)
    and q + r = 16 (the 256-thread LDS kernel), in the base fit and in
    bootstrap replicates — every coefficient and t-statistic."""
    T, N, q = 140, 90 if mode == "direct" else 260, 4
    rng = np.random.default_rng(40 + r)
    y, x, *_ = oracle.factor_model_DGP(T + 3, N, 12, rng)
    x = oracle.normalize(x)[3:]
    w = np.hstack([np.ones((T, 1)), np.column_stack([y[3 - k:len(y) - k] for k in range(1, 4)])])
    y = y[3:]
    g = dfm.DynamicFactorModel(y, w, x, r, "ICp2")
    g.set_bootstrap_mode(mode)
    o = oracle.DynamicFactorModel(y, w, x, r, "ICp2")
    assert_fit_matches(g, o, oracle, q=q)
    B = 3
    idx, eta = oracle.draw_wild(np.random.default_rng(5), B, T)
    S = dfm.Stat
    d = q + r
    out = dfm.wild_bootstrap(g, B, [S.coefficient(j) for j in range(1, d + 1)] +
                             [S.t_stat(j) for j in range(1, d + 1)], idx=idx, eta=eta)
    for b in range(B):
        xs = o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]]
        ob = oracle.DynamicFactorModel(y, w, xs, r, "ICp2")
        assert rel(out[b, :d], ob.coefficients) < STAT_RTOL
        assert rel(out[b, d:], ob.t_stats) < STAT_RTOL


@pytest.mark.parametrize("T", [1000, 3000])
def test_wild_bootstrap_long_panel(dfm, oracle, T):
    """T >= N replicate Grams at long T: T = 1000 takes the weighted-GEMM path
    (gram_wk, its prep kernel's LDS 52 KB), T = 3000 exceeds the 64 KB that
    path may stage and falls back to the fused-gather K1 Gram."""
    N, r, B = 60, 4, 3
    y, x, w = panel(oracle, T, N, r, 5000 + T)
    g = dfm.DynamicFactorModel(y, w, x, r, "ICp2")
    o = oracle.DynamicFactorModel(y, w, x, r, "ICp2")
    idx, eta = oracle.draw_wild(np.random.default_rng(12), B, T)
    S = dfm.Stat
    out = dfm.wild_bootstrap(g, B, [S.V(), S.criterion(), S.eigenvalue(1), S.eigenvalue(r), S.t_stat(1),
                                    S.LR_all(T // 2)], idx=idx, eta=eta)
    for b in range(B):
        d = oracle.DynamicFactorModel(y, w, o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]], r,
                                      "ICp2")
        ref = [oracle.factor_residual_variance(d), d.number_of_factors_criterion_value, d.eigenvalues[0][0],
               d.eigenvalues[0][r - 1], d.t_stats[0]] + [oracle.LR_test(d, T // 2, i) for i in range(4)]
        assert rel(out[b, :9], ref) < STAT_RTOL
