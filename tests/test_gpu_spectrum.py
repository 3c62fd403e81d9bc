"""GPU parity for the full spectrum of Grams of any size (dfm_spec.hip:
Householder tridiagonalisation + Sturm bisection above the Jacobi kernel's
140): the full `eig` of src/DynamicFactorModel.jl:78 / :87, read past the top
r by the PCp criteria's sigma^2 (src/criteria.jl:18, :23, :28) and by IC
sweeps with kmax > 24 (src/DynamicFactorModel.jl:54)."""
import numpy as np
import pytest
import scipy.linalg

from test_gpu_parity import panel, STAT_RTOL, assert_fit_matches, lm_within, max_sin_angle, signs, rel, ANGLE_TOL

pytestmark = pytest.mark.gpu


# (70, 5003), (700, 6001): the N > T plain-panel Gram on LDS-DMA (gram_dma_kernel)
# with m % 64 != 0, K % 16 != 0 and deep split-K (S = 19, 15)
@pytest.mark.parametrize("T,N", [(400, 300), (250, 900), (141, 500), (900, 141), (1100, 1300), (70, 5003),
                                 (700, 6001)])
def test_gram_spectrum_any_size(dfm, oracle, T, N):
    _, x, _ = panel(oracle, T, N, 4, 7000 + T)
    G = x.T @ x if T >= N else x @ x.T
    ref = scipy.linalg.eigh(G, eigvals_only=True, driver="evr")[::-1]
    ev, tr = dfm.gram_spectrum(x)
    assert ev.shape == (min(T, N),)
    assert np.all(np.diff(ev) <= 0)
    # backward stable: every eigenvalue to O(eps ||G||), tail sums to far better than STAT_RTOL
    assert np.max(np.abs(ev - ref)) <= 1e-12 * ref[0] * np.sqrt(min(T, N))
    h = -(-min(T, N) // 2)
    assert abs(ev[h:].sum() - ref[h:].sum()) <= 1e-11 * ref.sum()


def test_spectrum_of_exact_rank_gram(dfm):
    """Rank-deficient Gram: the zero eigenvalues come out at O(eps ||G||)."""
    rng = np.random.default_rng(5)
    x = rng.standard_normal((300, 6)) @ rng.standard_normal((6, 200))
    ev, _ = dfm.gram_spectrum(x)
    ref = np.linalg.eigvalsh(x.T @ x)[::-1]
    assert np.max(np.abs(ev - ref)) <= 1e-11 * ref[0]
    assert np.max(np.abs(ev[6:])) <= 1e-11 * ref[0]


@pytest.mark.parametrize("T,N,r,crit", [(300, 200, 3, "PCp2"), (180, 600, 4, "PCp1"), (500, 2000, 8, "PCp3")])
def test_pcp_fit_beyond_jacobi_size(dfm, oracle, T, N, r, crit):
    y, x, w = panel(oracle, T, N, r, 7100 + T)
    g = dfm.DynamicFactorModel(y, w, x, r, crit)
    o = oracle.DynamicFactorModel(y, w, x, r, crit)
    assert abs(g.number_of_factors_criterion_value - o.number_of_factors_criterion_value) <= \
        STAT_RTOL * abs(o.number_of_factors_criterion_value)


@pytest.mark.parametrize("T,N,crit", [(300, 200, "ICp2"), (160, 400, "PCp2")])
def test_default_kmax_sweep_beyond_jacobi_size(dfm, oracle, T, N, crit):
    """kmax = ceil(m/2) > 24: the sweep reads the full spectrum."""
    y, x, w = panel(oracle, T, N, 3, 7200 + T)
    d = dfm.DynamicFactorModel(y, w, x, crit)
    o = oracle.DynamicFactorModel_ic(y, w, x, crit)
    assert d.number_of_factors == o.number_of_factors
    assert abs(d.number_of_factors_criterion_value - o.number_of_factors_criterion_value) <= \
        STAT_RTOL * abs(o.number_of_factors_criterion_value)


def test_pcp_sweep_with_large_break_blocks(dfm, oracle):
    y, x, w = panel(oracle, 420, 180, 3, 7300)
    d = dfm.DynamicFactorModel(y, w, x, "PCp2", break_indices=[210], kmax=8)
    o = oracle.DynamicFactorModel_ic(y, w, x, "PCp2", kmax=8, break_indices=[210])
    assert d.number_of_factors == o.number_of_factors
    assert abs(d.number_of_factors_criterion_value - o.number_of_factors_criterion_value) <= \
        STAT_RTOL * abs(o.number_of_factors_criterion_value)


# ------------------------------------------- top-k eigenpairs with k > 24
@pytest.mark.parametrize("T,N,r,crit", [(200, 160, 30, "ICp2"), (120, 400, 41, "BIC"), (600, 2000, 36, "ICp1"),
                                        (70, 60, 30, "ICp3")])
def test_fit_with_many_factors(dfm, oracle, T, N, r, crit):
    """r beyond the subspace eigensolver's block: the dense path (reference
    allows any r <= ceil(m/2), src/DynamicFactorModel.jl:116-119)."""
    y, x, w = panel(oracle, T, N, 3, 7400 + T)
    g = dfm.DynamicFactorModel(y, w, x, r, crit)
    o = oracle.DynamicFactorModel(y, w, x, r, crit)
    assert_fit_matches(g, o, oracle)


def test_principal_components_many(dfm, oracle):
    for T, N in [(300, 180), (150, 500)]:
        _, x, _ = panel(oracle, T, N, 4, 7500 + T)
        ev, F, L, tr = dfm.principal_components(x, 60)
        Fo, Lo, wo = oracle.principal_components(x, T, N)
        assert rel(ev, wo[:60]) < STAT_RTOL
        assert max_sin_angle(F, Fo[:, :60]) < ANGLE_TOL
        assert rel(L * signs(F, Fo[:, :60]), Lo[:, :60]) < 1e-8
        assert np.allclose(F.T @ F / (T if N > T else 1.0), np.eye(60) if N > T else F.T @ F, atol=1e-10 * T)


def test_default_constructor_reference_test_shape(dfm, oracle):
    """The reference's own test (test/DynamicFactorModel.jl:6-24): w = [1, 4
    lags of y], the 3-argument constructor, r = ceil(min(T,N)/2) (D2) — here
    T = 200, N = 130 -> r = 65, q + r = 70 regressors."""
    rng = np.random.default_rng(77)
    y0, x0, *_ = oracle.factor_model_DGP(204, 130, 4, rng)
    x = oracle.normalize(x0)[4:]
    lags = np.column_stack([y0[4 - k:-k] for k in range(1, 5)])
    w = np.hstack([np.ones((200, 1)), lags])
    y = y0[4:]
    g = dfm.DynamicFactorModel(y, w, x)
    o = oracle.DynamicFactorModel(y, w, x)
    assert g.number_of_factors == o.number_of_factors == 65
    assert_fit_matches(g, o, oracle, q=5)
    # the reference test's quantity: sum(model.factor_residuals.^2)
    assert abs(np.sum(g.factor_residuals ** 2) - np.sum(o.factor_residuals ** 2)) <= \
        1e-10 * np.sum(o.factor_residuals ** 2)


def test_many_factors_with_breaks(dfm, oracle):
    """Per-block dense eigenpairs + wide factors + wide OLS (D7, D13 as in test_gpu_breaks)."""
    y, x, w = panel(oracle, 240, 90, 3, 7600)
    g = dfm.DynamicFactorModel(y, w, x, 35, "ICp2", break_indices=[121])
    o = oracle.DynamicFactorModel(y, w, x, 35, "ICp2", break_indices=[121])
    assert g.number_of_factors == o.number_of_factors == 35
    assert abs(g.V - oracle.factor_residual_variance(o)) <= STAT_RTOL * oracle.factor_residual_variance(o)
    assert rel(g.t_stats[:1], o.t_stats[:1]) < STAT_RTOL
    assert np.max(np.abs(g.factor_residuals - o.factor_residuals)) < 1e-9 * np.max(np.abs(o.factor_residuals))


# ------------------------------------------------ PCp inside the bootstrap
@pytest.mark.parametrize("T,N,r,crit,mode,breaks", [
    (120, 60, 3, "PCp2", "auto", ()),          # m = 60: Jacobi spectrum per replicate
    (60, 150, 2, "PCp1", "factored", ()),       # N > T: the PCp stat forces the direct Gram
    (300, 180, 3, "PCp3", "auto", ()),          # m = 180: tridiagonal + bisection per replicate
    (160, 70, 2, "PCp2", "auto", (81,)),        # break blocks: sigma^2 from the full-sample Gram
])
def test_pcp_criterion_in_replicates(dfm, oracle, T, N, r, crit, mode, breaks):
    y, x, w = panel(oracle, T, N, r, 7700 + T)
    g = dfm.DynamicFactorModel(y, w, x, r, crit, break_indices=breaks)
    g.set_bootstrap_mode(mode)
    o = oracle.DynamicFactorModel(y, w, x, r, crit, break_indices=breaks)
    B = 4
    idx, eta = oracle.draw_wild(np.random.default_rng(9), B, T)
    S = dfm.Stat
    out = dfm.wild_bootstrap(g, B, [S.criterion(), S.criterion("PCp1"), S.V()], idx=idx, eta=eta)
    for b in range(B):
        xs = o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]]
        d = oracle.DynamicFactorModel(y, w, xs, r, crit, break_indices=breaks)
        ref = [d.number_of_factors_criterion_value, oracle.criterion_value("PCp1", d),
               oracle.factor_residual_variance(d)]
        assert rel(out[b], ref) < STAT_RTOL


# ------------------------------------------- bootstrap at r > 24 (dense batch)
@pytest.mark.parametrize("T,N,r,crit,breaks", [
    (150, 70, 30, "ICp2", ()),        # T >= N: r <= 32 factor kernels, q + r <= 32 OLS
    (90, 200, 40, "BIC", ()),         # N > T: wide factors (materialised X*) and wide OLS
    (200, 130, 65, "PCp2", ()),       # the default r = ceil(m/2) of the reference's test shape, PCp
    (160, 60, 27, "ICp1", (81,)),     # break blocks, per-block dense eigenpairs
])
def test_bootstrap_many_factors(dfm, oracle, T, N, r, crit, breaks):
    y, x, w = panel(oracle, T, N, 3, 7800 + T)
    g = dfm.DynamicFactorModel(y, w, x, r, crit, break_indices=breaks)
    o = oracle.DynamicFactorModel(y, w, x, r, crit, break_indices=breaks)
    B = 3
    idx, eta = oracle.draw_wild(np.random.default_rng(21), B, T)
    S = dfm.Stat
    out = dfm.wild_bootstrap(g, B, [S.V(), S.criterion(), S.eigenvalue(1), S.eigenvalue(r), S.trace(),
                                    S.coefficient(1), S.t_stat(1)], idx=idx, eta=eta)
    for b in range(B):
        xs = o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]]
        d = oracle.DynamicFactorModel(y, w, xs, r, crit, break_indices=breaks)
        ref = [oracle.factor_residual_variance(d), d.number_of_factors_criterion_value,
               sum(e[0] for e in d.eigenvalues), sum(e[r - 1] for e in d.eigenvalues), np.sum(xs * xs),
               d.coefficients[0], d.t_stats[0]]
        assert rel(out[b, :5], ref[:5]) < STAT_RTOL
        assert rel(out[b, 5:], ref[5:]) < STAT_RTOL


# ------------------------------------------------ Chow tests at r > 16
@pytest.mark.parametrize("T,N,r", [(160, 40, 20), (90, 150, 18)])
def test_chow_all_many_factors(dfm, oracle, T, N, r):
    y, x, w = panel(oracle, T, N, 2, 7900 + T, model="Breitung_Eickmeier_2011", b=0.5)
    g = dfm.DynamicFactorModel(y, w, x, r)
    o = oracle.DynamicFactorModel(y, w, x, r)
    bp = T // 2
    LR, LM, WD = dfm.chow_all(g, bp)
    nv = min(N, 12)
    ref = np.array([[oracle.LR_test(o, bp, i), oracle.LM_test(o, bp, i), oracle.Wald_test(o, bp, i)]
                    for i in range(nv)])
    assert rel(LR[:nv], ref[:, 0]) < STAT_RTOL
    lm_within(LM[:nv], o, bp, range(nv), oracle)
    assert rel(WD[:nv], ref[:, 2]) < STAT_RTOL


@pytest.mark.parametrize("r", [2, 20])
def test_bootstrap_chow_batched(dfm, oracle, r):
    """r = 2 (fused Chow kernels) and r = 20 (GEMM-built Chow on materialised
    replicates), several batches with a short tail batch, all-variable and
    single-variable forms."""
    T, N = 150, 40
    y, x, w = panel(oracle, T, N, 2, 7950, model="Breitung_Eickmeier_2011", b=0.5)
    g = dfm.DynamicFactorModel(y, w, x, r)
    g.set_batch(2)
    o = oracle.DynamicFactorModel(y, w, x, r)
    B, bp, i0 = 5, 70, 3
    idx, eta = oracle.draw_wild(np.random.default_rng(6), B, T)
    S = dfm.Stat
    out = dfm.wild_bootstrap(g, B, [S.LR_all(bp), S.LM(bp, i0 + 1), S.Wald(bp, i0 + 1)], idx=idx, eta=eta)
    for b in range(B):
        d = oracle.DynamicFactorModel(y, w, o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]], r)
        assert rel(out[b, :8], [oracle.LR_test(d, bp, i) for i in range(8)]) < STAT_RTOL
        lm_within([out[b, N]], d, bp, [i0], oracle)
        assert rel(out[b, N + 1], oracle.Wald_test(d, bp, i0)) < STAT_RTOL


# ---------------------------------------- JOINT hard thresholding, q + N > 64
@pytest.mark.parametrize("T,N,q", [(400, 150, 3), (260, 200, 5)])
def test_targeted_joint_wide(dfm, oracle, T, N, q):
    rng = np.random.default_rng(8000 + N)
    y, x, *_ = oracle.factor_model_DGP(T, N, 4, rng)
    x = oracle.normalize(x)
    w = np.hstack([np.ones((T, 1)), rng.standard_normal((T, q - 1))])
    mask, t = dfm.targeted_predictors(y, w, x, return_tstats=True)
    to, mo = oracle.targeted_predictors_hard(y, w, x, mode="joint")
    assert rel(t, to) < STAT_RTOL
    # the mask may differ only where |t| sits within rounding of the critical value
    cv = oracle.sps.t.ppf(0.975, T - q - N) if hasattr(oracle, "sps") else None
    diff = np.flatnonzero(mask != mo)
    if cv is not None:
        assert np.all(np.abs(np.abs(to[diff]) - cv) < 1e-8 * cv)
    else:
        assert diff.size == 0


def test_reference_test_workflow_from_csv(dfm, oracle, tmp_path):
    """test/DynamicFactorModel.jl end to end: readtable of a panel CSV, y = the
    first series, 4 lags of y in w, the 3-argument constructor (r = ceil(m/2)),
    sum(model.factor_residuals.^2)."""
    rng = np.random.default_rng(88)
    _, x0, *_ = oracle.factor_model_DGP(160, 61, 3, rng)
    data = oracle.normalize(x0)
    p = tmp_path / "1959-2014_normalized.csv"
    with open(p, "w") as fh:
        fh.write("date," + ",".join(f"V{i}" for i in range(61)) + "\n")
        for t in range(160):
            fh.write(f"d{t}," + ",".join(repr(float(v)) for v in data[t]) + "\n")
    _, d = dfm.read_panel_csv(str(p))
    y, w, x = dfm.reference_test_design(d, 4)
    g = dfm.DynamicFactorModel(y, w, x)
    o = oracle.DynamicFactorModel(y, w, x)
    assert g.number_of_factors == o.number_of_factors == 30
    ssr_g, ssr_o = np.sum(g.factor_residuals ** 2), np.sum(o.factor_residuals ** 2)
    assert abs(ssr_g - ssr_o) <= 1e-10 * ssr_o
    assert rel(g.t_stats[:5], o.t_stats[:5]) < STAT_RTOL       # intercept and lags: sign-invariant


def test_dense_spectrum_bit_reproducible(dfm, oracle):
    """tridiag_kernel accumulates p = A v in a fixed order (no float atomics):
    repeated calls return identical bits, and the many-factor loadings stay
    within the parity bar of test_principal_components_many."""
    import hashlib
    T, N = 150, 500
    _, x, _ = panel(oracle, T, N, 4, 7500 + T)
    digests = set()
    for _ in range(3):
        ev, F, L, tr = dfm.principal_components(x, 60)
        digests.add(hashlib.sha1(np.concatenate([ev, F.ravel(), L.ravel()]).tobytes()).hexdigest())
    assert len(digests) == 1
