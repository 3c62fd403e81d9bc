"""CPU checks that pin the oracle (oracle/dfm_oracle.py).

The reference has no golden vectors or assertions and cannot run
here (§8(c)): the oracle is therefore pinned by analytic known answers,
invariants of the reference algebra, an independent SVD
cross-implementation, the Bai–Ng (2002) selection known answer that the
reference's MC script (src/Bai_Ng.jl) targets, and the committed fixtures
(tests/golden/, which freeze the oracle against drift).
"""
import math
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _panel(O, T, N, r, seed, model="Bai_Ng_2002", **kw):
    rng = np.random.default_rng(seed)
    out = O.factor_model_DGP(T, N, r, rng, model=model, **kw)
    return out[0], O.normalize(out[1]), np.ones((T, 1))


# ---------------------------------------------------------- analytic answers
@pytest.mark.parametrize("T,N", [(40, 20), (20, 40)])
def test_exact_rank_panel_has_zero_residual(oracle, T, N):
    rng = np.random.default_rng(0)
    r = 3
    x = rng.standard_normal((T, r)) @ rng.standard_normal((N, r)).T
    y = rng.standard_normal(T)
    d = oracle.DynamicFactorModel(y, np.ones((T, 1)), x, r)
    assert oracle.factor_residual_variance(d) < 1e-24 * np.sum(x ** 2)
    assert np.all(np.abs(d.eigenvalues[0][r:]) < 1e-10 * d.eigenvalues[0][0])


@pytest.mark.parametrize("T,N", [(120, 50), (50, 120), (60, 60)])
def test_normalisation_identities(oracle, T, N):
    """src/DynamicFactorModel.jl:80 (L'L/N = I for T >= N) and :89 (F'F/T = I)."""
    _, x, _ = _panel(oracle, T, N, 3, 1)
    F, L, _ = oracle.principal_components(x, T, N)
    if T >= N:
        assert np.allclose(L.T @ L / N, np.eye(N), atol=1e-12)
    else:
        assert np.allclose(F.T @ F / T, np.eye(T), atol=1e-12)
    assert np.allclose(F @ L.T, x, atol=1e-10)   # full width reproduces x


@pytest.mark.parametrize("T,N", [(150, 60), (60, 150)])
def test_pca_matches_svd(oracle, T, N):
    """Independent cross-implementation: eigenvalues = squared singular values,
    the factor space = leading left singular space."""
    _, x, _ = _panel(oracle, T, N, 4, 2)
    F, L, w = oracle.principal_components(x, T, N)
    U, s, Vt = np.linalg.svd(x, full_matrices=False)
    m = min(T, N)
    assert np.allclose(w[:m], s ** 2, rtol=1e-11, atol=1e-9 * s[0] ** 2)
    k = 4
    Fk = F[:, :k] / np.linalg.norm(F[:, :k], axis=0)
    cosines = np.linalg.svd(U[:, :k].T @ Fk, compute_uv=False)
    assert np.all(cosines > 1 - 1e-12)


def test_V_trace_identity(oracle):
    """||E_k||^2 = tr(G) - sum_{j<=k} lambda_j (both branches)."""
    for T, N in [(200, 100), (80, 160)]:
        y, x, w = _panel(oracle, T, N, 3, 3)
        for k in (1, 3, 5):
            d = oracle.DynamicFactorModel(y, w, x, k)
            lam = d.eigenvalues[0]
            V = (np.sum(x * x) - lam[:k].sum()) / (T * N)
            assert abs(V - oracle.factor_residual_variance(d)) <= 1e-12 * V


def test_hc2_matches_leverage_form(oracle):
    """:43-46 with the T x T hat matrix equals the leverage-vector form."""
    rng = np.random.default_rng(4)
    T = 80
    D = np.hstack([np.ones((T, 1)), rng.standard_normal((T, 3))])
    y = D @ np.array([1.0, -2, 0.5, 3]) + rng.standard_normal(T)
    b, cov, t, u = oracle._ols_hc2(D, y)
    Q, _ = np.linalg.qr(D)
    h = np.sum(Q * Q, axis=1)
    DtDi = np.linalg.inv(D.T @ D)
    cov2 = DtDi @ (D.T * (u ** 2 / (1 - h))) @ D @ DtDi
    assert np.allclose(cov, cov2, rtol=1e-12)
    assert np.allclose(b, np.linalg.lstsq(D, y, rcond=None)[0], rtol=1e-12)


def test_bai_ng_selects_true_r(oracle):
    """Known answer of Bai & Ng (2002) Table 2 for (T, N) = (200, 100), r = 3:
    ICp1/ICp2 select the true r (the MC script src/Bai_Ng.jl:12-39)."""
    hits = 0
    for seed in range(5):
        y, x, w = _panel(oracle, 200, 100, 3, 100 + seed)
        ic = oracle.ic_sweep_values(y, w, x, 8, criteria=("ICp1", "ICp2"))
        hits += int(np.argmin(ic[0]) + 1 == 3 and np.argmin(ic[1]) + 1 == 3)
    assert hits >= 4


def test_ic_sweep_constructor_is_first_argmin(oracle):
    y, x, w = _panel(oracle, 150, 80, 2, 5)
    best = oracle.DynamicFactorModel_ic(y, w, x, "BIC", kmax=6)
    vals = oracle.ic_sweep_values(y, w, x, 6, criteria=("BIC",))[0]
    assert best.number_of_factors == int(np.argmin(vals)) + 1


def test_chow_stats_sign_invariant(oracle):
    """LR/LM/Wald are invariant to factor sign flips."""
    y, x, w = _panel(oracle, 120, 30, 2, 6, model="Breitung_Eickmeier_2011", b=1.0)
    d = oracle.DynamicFactorModel(y, w, x, 2)
    s = [oracle.LR_test(d, 60, 3), oracle.LM_test(d, 60, 3), oracle.Wald_test(d, 60, 3)]
    d.factors = [d.factors[0] * np.r_[-1.0, 1.0, np.ones(d.factors[0].shape[1] - 2)]]
    d.loadings = [d.loadings[0] * np.r_[-1.0, 1.0, np.ones(d.loadings[0].shape[1] - 2)]]
    s2 = [oracle.LR_test(d, 60, 3), oracle.LM_test(d, 60, 3), oracle.Wald_test(d, 60, 3)]
    assert np.allclose(s, s2, rtol=1e-10)


def test_chow_detects_break(oracle):
    """A loading break of size b (src/utils.jl:80-91) inflates LR/Wald."""
    y, x, w = _panel(oracle, 400, 40, 1, 7, model="Breitung_Eickmeier_2011", b=1.5)
    d = oracle.DynamicFactorModel(y, w, x, 1)
    y0, x0, _ = _panel(oracle, 400, 40, 1, 7, model="Breitung_Eickmeier_2011", b=0.0)
    d0 = oracle.DynamicFactorModel(y0, w, x0, 1)
    lr = np.mean([oracle.LR_test(d, 200, i) for i in range(10)])
    lr0 = np.mean([oracle.LR_test(d0, 200, i) for i in range(10)])
    assert lr > 3 * lr0


def test_wild_bootstrap_identity_draw_reproduces_fit(oracle):
    """idx = identity and eta = 1 rebuild X exactly: the replicate is the fit."""
    y, x, w = _panel(oracle, 100, 50, 2, 8)
    d = oracle.DynamicFactorModel(y, w, x, 2, "ICp2")
    B, T = 2, 100
    idx = np.tile(np.arange(T, dtype=np.int32), (B, 1))
    eta = np.ones((B, T))
    st = oracle.wild_bootstrap(d, B, oracle.factor_residual_variance, idx, eta)
    assert np.allclose(st, oracle.factor_residual_variance(d), rtol=1e-10)


def test_targeted_per_candidate_matches_explicit_ols(oracle):
    """FWL form used by the engine == the explicit OLS [w x_i] with HC0."""
    rng = np.random.default_rng(9)
    T, N = 120, 6
    x = rng.standard_normal((T, N))
    w = np.hstack([np.ones((T, 1)), rng.standard_normal((T, 1))])
    y = x[:, 0] * 0.8 + rng.standard_normal(T)
    t, _ = oracle.targeted_predictors_hard(y, w, x, "per_candidate")
    for i in range(N):
        Z = np.hstack([w, x[:, i:i + 1]])
        Zi = np.linalg.inv(Z.T @ Z)
        b = Zi @ Z.T @ y
        u = y - Z @ b
        cov = Zi @ (Z.T @ np.diag(u ** 2) @ Z) @ Zi
        assert abs(t[i] - b[-1] / math.sqrt(cov[-1, -1])) < 1e-10 * abs(t[i])


def test_targeted_joint_critical_value(oracle):
    """:27 — quantile(TDist(T - q - N), 0.975)."""
    from scipy import stats
    y, x, w = _panel(oracle, 100, 10, 2, 10)
    t, m = oracle.targeted_predictors_hard(y, w, x, "joint")
    cv = stats.t.ppf(0.975, 100 - 1 - 10)
    assert np.array_equal(m, np.abs(t) > cv)


# ------------------------------------------------------------ golden fixtures
def test_golden_c1_reproduces(oracle):
    g = np.load(os.path.join(GOLD, "c1_bai_ng_T200_N100_r3.npz"))
    d = oracle.DynamicFactorModel(g["y"], g["w"], g["x"], int(g["r"]), "ICp2")
    assert np.allclose(d.eigenvalues[0][:16], g["eigvals"], rtol=1e-12)
    assert np.allclose(d.coefficients, g["coefficients"], rtol=1e-10)
    assert abs(oracle.factor_residual_variance(d) - float(g["V"])) < 1e-12
    ic = oracle.ic_sweep_values(g["y"], g["w"], g["x"], 8)
    assert np.allclose(ic, g["ic_values"], rtol=1e-12)
    assert int(np.argmin(ic[4])) + 1 == int(g["ic_best_r"]) == 3


def test_golden_c2_base_reproduces(oracle):
    g = np.load(os.path.join(GOLD, "c2_breitung_eickmeier_T600_N130_B16.npz"))
    base = oracle.DynamicFactorModel_ic(g["y"], g["w"], g["x"], "ICp2", kmax=8)
    assert base.number_of_factors == int(g["r"])
    for i in (0, 7, 129):
        assert abs(oracle.LR_test(base, 300, i) - g["base_chow"][i, 0]) < 1e-9 * max(1, abs(g["base_chow"][i, 0]))


# ------------------------------------------------------------- break blocks
@pytest.mark.parametrize("T,N,breaks", [(90, 200, [31, 61]), (160, 40, [81])])
def test_break_blocks_scaling_and_residual_identity(oracle, T, N, breaks):
    """src/DynamicFactorModel.jl:72-98 with break_indices: each block's PCA
    uses the FULL-sample T, N (D7): F_j'F_j/T = I (N > T) or L_j'L_j/N = I
    (T >= N); the block common component is the projection of X_j on its top-r
    eigenspace, so ||E||^2 = sum_j (trace G_j - sum_{i<=r} lambda_{j,i})."""
    y, x, w = _panel(oracle, T, N, 2, 11, model="Breitung_Eickmeier_2011", b=0.7)
    r = 2
    d = oracle.DynamicFactorModel(y, w, x, r, "", breaks)
    b = [1] + breaks + [T + 1]
    assert [F.shape[0] for F in d.factors] == [b[i] - b[i - 1] for i in range(1, len(b))]
    energy = 0.0
    for j, (F, L, ev) in enumerate(zip(d.factors, d.loadings, d.eigenvalues)):
        xj = x[b[j] - 1:b[j + 1] - 1]
        if N > T:
            assert np.allclose(F.T @ F / T, np.eye(F.shape[1]), atol=1e-11)
        else:
            assert np.allclose(L.T @ L / N, np.eye(N), atol=1e-11)
        P = F[:, :r] @ L[:, :r].T
        assert np.allclose(P, xj - d.factor_residuals[b[j] - 1:b[j + 1] - 1], atol=1e-10)
        energy += np.sum(xj ** 2) - np.sum(ev[:r])
    assert abs(np.sum(d.factor_residuals ** 2) - energy) < 1e-9 * np.sum(x ** 2)
    # the design matrix stacks the blocks' factors (:131)
    assert d.design_matrix.shape == (T, 1 + r)
    assert np.array_equal(d.design_matrix[:, 1:], np.vstack([F[:, :r] for F in d.factors]))


def test_break_residual_draws_stay_in_block(oracle):
    """src/bootstrap.jl:23-28: DiscreteUniform(from, to) per break block."""
    idx = oracle.draw_residual(np.random.default_rng(0), 50, 30, [11, 21])
    assert np.all((idx[:, :10] >= 0) & (idx[:, :10] < 10))
    assert np.all((idx[:, 10:20] >= 10) & (idx[:, 10:20] < 20))
    assert np.all((idx[:, 20:] >= 20) & (idx[:, 20:] < 30))


# ------------------------------------------------- soft thresholding (glmnet)
def test_glmnet_default_folds(oracle):
    """GLMNet.jl: nfolds = min(10, n ÷ 3), fold sizes differ by at most one."""
    f = oracle.glmnet_default_folds(103, np.random.default_rng(0))
    assert f.min() == 1 and f.max() == 10
    counts = np.bincount(f)[1:]
    assert counts.max() - counts.min() <= 1 and counts.sum() == 103
    assert oracle.glmnet_default_folds(12, np.random.default_rng(0)).max() == 4


def test_lasso_cd_fixed_point_matches_sklearn(oracle):
    """Independent cross-implementation: at a tight threshold the coordinate-
    descent path point is the lasso minimiser (1/2n)||y - Zb||^2 + lam|b|_1,
    which sklearn's Lasso (its own CD) also computes."""
    from sklearn.linear_model import Lasso
    y, x, w = _panel(oracle, 80, 150, 3, 21)
    Z = np.hstack([w, x])
    mu, sd, ju, yb, ys, G, c = oracle._glmnet_standardize(Z, y)
    Zs = np.where(ju, (Z - mu) / sd, 0.0)
    lam_max = float(np.max(np.abs(c[ju])))
    alms = [lam_max * 0.97 ** m for m in range(40)]
    betas, rsq = oracle.lasso_path_cd(G, c, ju, alms, early_exit=False, thresh=1e-26)
    assert np.all(betas[0] == 0.0)                       # lambda_max: nothing enters
    assert np.count_nonzero(betas[1]) == 1               # just below: the argmax enters
    for m in (5, 20, 39):
        sk = Lasso(alpha=alms[m], fit_intercept=False, tol=1e-14, max_iter=10 ** 6).fit(Zs, (y - yb) / ys)
        assert np.max(np.abs(sk.coef_ - betas[m])) < 1e-8
        assert np.array_equal(sk.coef_ != 0, betas[m] != 0)
        r = (y - yb) / ys - Zs @ betas[m]
        assert abs(rsq[m] - (1 - r @ r / len(y))) < 1e-10   # R^2 = b'(c + g)


def test_glmnetcv_loss_and_selection(oracle):
    """meanloss = fold-size-weighted hold-out MSE; the lambda grid is
    log-spaced from lambda_max with ratio lambda_min_ratio^(1/(nlambda-1))."""
    y, x, w = _panel(oracle, 90, 60, 3, 22)
    folds = oracle.glmnet_default_folds(90, np.random.default_rng(3))
    mask, res = oracle.targeted_predictors_soft(y, w, x, folds, nlambda=30, lambda_min_ratio=0.05)
    lam = res["lambda"]
    assert np.allclose(lam[1:] / lam[:-1], 0.05 ** (1 / 29), rtol=1e-12)
    assert res["best"] == int(np.argmin(res["meanloss"]))
    b = res["best"]
    assert np.array_equal(mask, res["betas"][b][1:] != 0)
    # refit fold 1 by hand at the best lambda and check its share of the loss
    ho = folds == 1
    mu, sd, ju, yb, ys, G, c = oracle._glmnet_standardize(np.hstack([w, x])[~ho], y[~ho])
    bf, _ = oracle.lasso_path_cd(G, c, ju, list(lam / ys), early_exit=False)
    assert bf.shape[0] == len(lam)
    assert np.all(res["meanloss"] > 0)


def test_golden_soft_reproduces(oracle):
    g = np.load(os.path.join(GOLD, "tp_soft.npz"))
    mask, res = oracle.targeted_predictors_soft(g["y"], g["w"], g["x"], g["folds"])
    assert np.array_equal(mask, g["mask"]) and res["best"] == int(g["best"])
    assert np.allclose(res["meanloss"], g["meanloss"], rtol=1e-10, atol=0)


# ----------------------------------------------------- forecasts (D4 repaired)
def test_repaired_get_factors_reproduces_in_sample_factors(oracle):
    """get_factors(dfm, x) of the training rows themselves, with the scalar
    normalisation undone, reproduces the fitted factors: rotation = L (L'L)^-1
    is the least-squares inverse of x = F L' on the factor space."""
    for T, N in [(80, 150), (150, 40)]:
        y, x, w = _panel(oracle, T, N, 3, 31)
        d = oracle.DynamicFactorModel(y, w, x, 3)
        L = d.loadings[0]
        rot = L @ np.linalg.inv(L.T @ L)
        assert np.allclose((x @ rot)[:, :3], d.F, atol=1e-8 * np.abs(d.F).max())
        xs_new = x[:2] * x.std(ddof=1) + x.mean()        # de-normalised by the scalar moments
        assert np.allclose(oracle.get_factors(d, xs_new), d.F[:2], atol=1e-8 * np.abs(d.F).max())


# ------------------------------------------------ extended-precision referee
def test_xp_referee_pins_the_oracle(oracle):
    """oracle/dfm_xp.py recomputes the fit, criteria and Chow statistics in
    double-double: on a small panel the fp64 oracle agrees with it to 1e-11
    (the referee's own arithmetic is checked by the identities below)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
    import dfm_xp as XP
    a = XP.DD(np.array([1.0, 3.0]))
    third = a / 3.0
    assert third.hi[0] == 1.0 / 3.0 and abs((third * 3.0 - 1.0).f64()[0]) < 1e-30
    assert abs((XP.DD(2.0).sqrt() * XP.DD(2.0).sqrt() - 2.0).f64()) < 1e-30
    for T, N in [(60, 25), (25, 60)]:
        y, x, w = _panel(oracle, T, N, 2, 77, model="Breitung_Eickmeier_2011", b=0.5)
        f = XP.XPFit(y, w, x, 2, "ICp1")
        o = oracle.DynamicFactorModel(y, w, x, 2, "ICp1")
        assert abs(f.V.f64() / oracle.factor_residual_variance(o) - 1) < 1e-12
        assert abs(f.criterion_value("ICp1") / o.number_of_factors_criterion_value - 1) < 1e-12
        s = np.sign(np.sum(f.F.f64() * o.F, axis=0))
        assert np.allclose(f.t_stats[1:] * s, o.t_stats[1:], rtol=1e-11, atol=0)
        LR, LM, W = f.chow_all(T // 2)
        ref = np.array([[oracle.LR_test(o, T // 2, i), oracle.LM_test(o, T // 2, i), oracle.Wald_test(o, T // 2, i)]
                        for i in range(N)])
        assert np.allclose(np.column_stack([LR, LM, W]), ref, rtol=1e-11, atol=0)
        lr1 = [XP.lr_referee(o.F, o.x[:, i], o.factor_residuals[:, i], T // 2) for i in range(N)]
        assert np.allclose(lr1, ref[:, 0], rtol=1e-11, atol=0)


def test_xp_fixture_agrees_with_golden():
    """The committed referee values and the oracle's golden values differ by
    less than 1e-10 relative (the C2 oracle's largest deviation is 4e-12)."""
    xp = np.load(os.path.join(GOLD, "xp_c1_c2.npz"))
    g2 = np.load(os.path.join(GOLD, "c2_breitung_eickmeier_T600_N130_B16.npz"))
    assert np.all(np.abs(xp["c2_base_chow"] - g2["base_chow"]) < 1e-10 * np.abs(xp["c2_base_chow"]))
    nv, N = int(g2["nv"]), g2["x"].shape[1]
    cols = [0, 1] + [2 + k * N + i for k in range(3) for i in range(nv)]
    assert np.all(np.abs(xp["c2_boot"][:, cols] - g2["boot"]) < 1e-10 * np.abs(xp["c2_boot"][:, cols]))
    assert np.all(xp["c2_boot_bar"] >= 1e-10 * np.abs(xp["c2_boot"]))
    g1 = np.load(os.path.join(GOLD, "c1_bai_ng_T200_N100_r3.npz"))
    assert np.all(np.abs(xp["c1_ic"] - g1["ic_values"]) < 1e-10 * np.abs(xp["c1_ic"]))


def test_oracle_pool_matches_serial_oracle(oracle):
    """tests/oracle_pool.py (the whole-batch checker of the -m gpu production
    tests) returns, in replicate order, exactly what the serial oracle loop
    gives for the same draws (src/bootstrap.jl:41-51, src/chowtest.jl:19-42)."""
    import oracle_pool
    T, N, r, B, bp = 60, 40, 2, 7, 30
    y, x, *_ = oracle.factor_model_DGP(T, N, r, np.random.default_rng(5))
    x = oracle.normalize(x)
    w = np.ones((T, 1))
    rng = np.random.default_rng(6)
    idx = rng.integers(0, T, (B, T)).astype(np.int32)
    eta = rng.standard_normal((B, T))
    c3 = oracle_pool.run("c3", y, w, x, r, "ICp2", idx, eta, chunk=3, nproc=2)
    vs = [0, 5, 39]
    c2 = oracle_pool.run("c2", y, w, x, r, "ICp2", idx, eta, extra=(bp, vs), chunk=2, nproc=2)
    ex = oracle_pool.run("c2ref", y, w, x, r, "ICp2", None, None, jobs=[(idx[3:4], eta[3:4], bp, vs)], nproc=2)
    base = oracle.DynamicFactorModel(y, w, x, r, "ICp2")
    for b in range(B):
        d = oracle.DynamicFactorModel(y, w, base.common_component + eta[b][:, None] * base.factor_residuals[idx[b]],
                                      r, "ICp2")
        want = [oracle.factor_residual_variance(d), d.number_of_factors_criterion_value, np.sum(d.x ** 2)]
        assert np.allclose(c3[b], want + list(d.eigenvalues[0][:r]), rtol=1e-13, atol=0)
        want2 = want[:2] + [oracle.Wald_test(d, bp, i) for i in vs] + [oracle.LR_test(d, bp, i) for i in vs] + \
            [oracle.LM_test(d, bp, i) for i in vs]
        assert np.allclose(c2[b], want2, rtol=1e-13, atol=0)
        if b == 3:
            assert np.allclose(ex[0][:, 0], want2[2 + 3:2 + 6], rtol=1e-9)
            assert np.allclose(ex[0][:, 1], want2[2 + 6:], rtol=1e-9)
