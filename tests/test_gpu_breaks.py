"""GPU parity for structural breaks: break-aware principal components
(src/DynamicFactorModel.jl:71-121 with break_indices — per-block PCA using the
full-sample T, N, defect D7), the workhorse fit on the stacked block factors
(:31-50, :130-133), the IC sweep and the bootstrap refits that pass
dfm.break_indices (src/bootstrap.jl:21-51, block-wise residual draws :23-28).
Tolerances as tests/test_gpu_parity.py (north star: 1e-10 relative for
statistics, principal angle < 1e-8 for factors)."""
import numpy as np
import pytest

from test_gpu_parity import ANGLE_TOL, STAT_RTOL, lm_within, lr_within, max_sin_angle, panel, rel

pytestmark = pytest.mark.gpu


def nrel(a, b):
    """Normwise relative difference (elementwise ratios blow up on the tiny
    entries of weak-gap noise factors; the angle bound is the north star's)."""
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def x_of(o):
    return o.x


def assert_block_fit(g, o, oracle):
    r = o.number_of_factors
    assert g.number_of_factors == r
    assert len(g.factors) == len(o.factors)
    for j, (Fg, Fo, Lg, Lo) in enumerate(zip(g.factors, o.factors, g.loadings, o.loadings)):
        assert Fg.shape == (Fo.shape[0], r)
        assert max_sin_angle(Fg, Fo[:, :r]) < ANGLE_TOL, j
        # both sides canonicalise signs (largest-|.| entry positive): equal columns
        assert nrel(Fg, Fo[:, :r]) < ANGLE_TOL, j
        assert nrel(Lg, Lo[:, :r]) < ANGLE_TOL, j
        assert rel(g.block_eigenvalues[j], o.eigenvalues[j][:r]) < STAT_RTOL, j
    V = oracle.factor_residual_variance(o)
    assert abs(g.V - V) < STAT_RTOL * V
    # E = X - F L' inherits the factor angle (< 1e-8) times |X|
    assert np.max(np.abs(g.factor_residuals - o.factor_residuals)) < ANGLE_TOL * np.max(np.abs(x_of(o)))
    # coefficients / t-stats of weak (noise-level) factors chosen by a sweep are
    # O(1e-3): compare on the vector's scale, as the factor angle bounds them
    assert np.max(np.abs(g.coefficients - o.coefficients)) < STAT_RTOL * np.max(np.abs(o.coefficients))
    assert np.max(np.abs(g.t_stats - o.t_stats)) < STAT_RTOL * np.max(np.abs(o.t_stats))
    if o.number_of_factors_criterion:
        assert abs(g.number_of_factors_criterion_value - o.number_of_factors_criterion_value) <= \
            STAT_RTOL * abs(o.number_of_factors_criterion_value)


@pytest.mark.parametrize("T,N,r,breaks,crit", [
    (120, 300, 3, [61], "ICp2"),           # N > T: block Grams X_j X_j', F_j = sqrt(T) U_j
    (150, 400, 2, [40, 101], "BIC"),       # three blocks, unequal lengths
    (200, 40, 3, [81], "ICp1"),            # T >= N: block Grams X_j' X_j, L_j = sqrt(N) V_j
    (240, 60, 2, [60, 120, 200], "ICp3"),  # four blocks, a short last block
])
def test_break_fit_matches_oracle(dfm, oracle, T, N, r, breaks, crit):
    y, x, w = panel(oracle, T, N, r, 31 + T, model="Breitung_Eickmeier_2011", b=0.8)
    g = dfm.DynamicFactorModel(y, w, x, r, crit, break_indices=breaks)
    o = oracle.DynamicFactorModel(y, w, x, r, crit, breaks)
    assert_block_fit(g, o, oracle)


@pytest.mark.parametrize("crit", ["PCp2", "ICp2", "BIC"])
@pytest.mark.parametrize("T,N,breaks", [(120, 200, [61]), (160, 50, [70])])
def test_break_ic_sweep_matches_oracle(dfm, oracle, T, N, breaks, crit):
    y, x, w = panel(oracle, T, N, 3, 47, model="Breitung_Eickmeier_2011", b=0.5)
    g = dfm.DynamicFactorModel(y, w, x, crit, kmax=8, break_indices=breaks)
    o = oracle.DynamicFactorModel_ic(y, w, x, crit, kmax=8, break_indices=breaks)
    assert_block_fit(g, o, oracle)


def test_break_calculate_factors(dfm, oracle):
    y, x, w = panel(oracle, 100, 250, 2, 5)
    Fg, Lg, r = dfm.calculate_factors(x, number_of_factors=2, break_indices=[40])
    Fo, Lo, _, ro = oracle.calculate_factors(x, 2, [40])
    assert r == ro == 2 and len(Fg) == 2
    for j in range(2):
        assert nrel(Fg[j], Fo[j][:, :2]) < ANGLE_TOL and nrel(Lg[j], Lo[j][:, :2]) < ANGLE_TOL


@pytest.mark.parametrize("T,N,breaks", [(120, 300, [61]), (200, 40, [81, 150])])
def test_break_wild_bootstrap_matches_oracle(dfm, oracle, T, N, breaks):
    y, x, w = panel(oracle, T, N, 2, 53, model="Breitung_Eickmeier_2011", b=0.5)
    g = dfm.DynamicFactorModel(y, w, x, 2, "ICp2", break_indices=breaks)
    o = oracle.DynamicFactorModel(y, w, x, 2, "ICp2", breaks)
    idx, eta = oracle.draw_wild(np.random.default_rng(8), 5, T)
    S = dfm.Stat
    out = dfm.wild_bootstrap(g, 5, [S.V(), S.criterion(), S.coefficient(1), S.t_stat(1), S.trace()],
                             idx=idx, eta=eta)
    for b in range(5):
        d = oracle.DynamicFactorModel(y, w, o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]],
                                      2, "ICp2", breaks)
        assert abs(out[b, 0] - oracle.factor_residual_variance(d)) < STAT_RTOL * oracle.factor_residual_variance(d)
        assert abs(out[b, 1] - d.number_of_factors_criterion_value) < STAT_RTOL * abs(d.number_of_factors_criterion_value)
        assert abs(out[b, 2] - d.coefficients[0]) < STAT_RTOL * abs(d.coefficients[0])
        assert abs(out[b, 3] - d.t_stats[0]) < STAT_RTOL * abs(d.t_stats[0])


def test_break_residual_bootstrap_block_draws(dfm, oracle):
    T, N, breaks = 140, 260, [71]
    y, x, w = panel(oracle, T, N, 3, 59, model="Breitung_Eickmeier_2011", b=1.0)
    g = dfm.DynamicFactorModel(y, w, x, 3, "ICp1", break_indices=breaks)
    o = oracle.DynamicFactorModel(y, w, x, 3, "ICp1", breaks)
    idx = oracle.draw_residual(np.random.default_rng(9), 4, T, breaks)
    assert np.all(idx[:, :70] < 70) and np.all(idx[:, 70:] >= 70)   # :23-28 block-wise U{a..b}
    out = dfm.residual_bootstrap(g, 4, [dfm.Stat.V(), dfm.Stat.criterion()], idx=idx)
    ref = oracle.residual_bootstrap(o, 4, lambda d: oracle.factor_residual_variance(d), idx)
    assert rel(out[:, 0], ref) < STAT_RTOL


def test_single_block_break_list_is_the_plain_fit(dfm, oracle):
    y, x, w = panel(oracle, 90, 200, 2, 3)
    a = dfm.DynamicFactorModel(y, w, x, 2, "ICp2")
    b = dfm.DynamicFactorModel(y, w, x, 2, "ICp2", break_indices=[])
    assert a.V == b.V and np.array_equal(a.coefficients, b.coefficients)


def test_break_errors(dfm, oracle):
    y, x, w = panel(oracle, 100, 200, 2, 2)
    with pytest.raises(dfm.DFMError):           # block of 2 rows cannot hold r = 3 factors (N > T)
        dfm.DynamicFactorModel(y, w, x, 3, break_indices=[99])
    with pytest.raises(dfm.DFMError):           # not increasing
        dfm.DynamicFactorModel(y, w, x, 2, break_indices=[60, 40])
    with pytest.raises(dfm.DFMError):           # outside 2..T
        dfm.DynamicFactorModel(y, w, x, 2, break_indices=[101])
    g = dfm.DynamicFactorModel(y, w, x, 2, break_indices=[50])
    with pytest.raises(dfm.DFMError):           # break period leaves < r rows
        dfm.chow_all(g, 1)


# ---------------------------------------------- Chow tests of break-fitted models
# src/chowtest.jl reads dfm.factors (F = vcat(F_j), D1), dfm.x and
# dfm.factor_residuals (E = X - vcat(F_j L_j')) — never one loadings matrix —
# so a model fitted with break_indices has well-defined LR / LM / Wald tests.
@pytest.mark.parametrize("T,N,r,breaks", [
    (120, 60, 2, [61]),                # T >= N: two blocks
    (96, 150, 3, [31, 70]),            # N > T: three blocks, bp inside block 2
    (200, 40, 2, [50, 101, 160]),      # four blocks
    (120, 160, 17, [61]),              # r > 16: the GEMM-built (explicit-residual) Chow
])
def test_break_chow_all_matches_oracle(dfm, oracle, T, N, r, breaks):
    y, x, w = panel(oracle, T, N, 2, 71 + T, model="Breitung_Eickmeier_2011", b=0.6)
    g = dfm.DynamicFactorModel(y, w, x, r, break_indices=breaks)
    o = oracle.DynamicFactorModel(y, w, x, r, "", breaks)
    # break periods off the blocks' boundaries (at a boundary the subperiod
    # SSRs equal ||E_i||^2 exactly — each block's loadings are its OLS
    # coefficients — and LR, LM vanish to rounding)
    for bp in (T // 2 + 7, breaks[0] + 3):
        LR, LM, W = dfm.chow_all(g, bp)
        nv = min(N, 30)
        ref = np.array([[oracle.LR_test(o, bp, i), oracle.LM_test(o, bp, i), oracle.Wald_test(o, bp, i)]
                        for i in range(nv)])
        lr_within(LR[:nv], o, bp, range(nv), oracle)
        lm_within(LM[:nv], o, bp, range(nv), oracle)
        assert rel(W[:nv], ref[:, 2]) < STAT_RTOL, bp
        assert dfm.LM_test(g, bp, 3) == LM[2]


@pytest.mark.parametrize("T,N,r,breaks", [(120, 60, 2, [61]), (96, 150, 3, [31, 70]), (120, 160, 17, [61])])
def test_break_bootstrap_chow_matches_oracle(dfm, oracle, T, N, r, breaks):
    y, x, w = panel(oracle, T, N, 2, 83 + T, model="Breitung_Eickmeier_2011", b=0.6)
    g = dfm.DynamicFactorModel(y, w, x, r, "ICp2", break_indices=breaks)
    o = oracle.DynamicFactorModel(y, w, x, r, "ICp2", breaks)
    B, bp = 3, T // 2 + 7
    idx, eta = oracle.draw_wild(np.random.default_rng(12), B, T)
    S = dfm.Stat
    out = dfm.wild_bootstrap(g, B, [S.LR_all(bp), S.LM_all(bp), S.Wald_all(bp), S.LR(bp, 2)], idx=idx, eta=eta)
    nv = min(N, 20)
    for b in range(B):
        d = oracle.DynamicFactorModel(y, w, o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]],
                                      r, "ICp2", breaks)
        ref = np.array([[oracle.LR_test(d, bp, i), oracle.LM_test(d, bp, i), oracle.Wald_test(d, bp, i)]
                        for i in range(nv)])
        assert rel(out[b, :nv], ref[:, 0]) < STAT_RTOL
        lm_within(out[b, N:N + nv], d, bp, range(nv), oracle)
        assert rel(out[b, 2 * N:2 * N + nv], ref[:, 2]) < STAT_RTOL
        assert out[b, 3 * N] == out[b, 1]      # single-variable LR(bp, 2) = row entry 2
    idx_r = oracle.draw_residual(np.random.default_rng(13), 2, T, breaks)
    outr = dfm.residual_bootstrap(g, 2, [S.LM_all(bp)], idx=idx_r)
    for b in range(2):
        d = oracle.DynamicFactorModel(y, w, o.common_component + o.factor_residuals[idx_r[b]], r, "ICp2", breaks)
        lm_within(outr[b, :nv], d, bp, range(nv), oracle)
