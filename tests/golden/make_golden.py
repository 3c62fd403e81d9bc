"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

The reference (Julia 0.3) cannot run here and ships no vectors of its own
(SURVEY §4, §8(c)), so these fixtures are produced by the reference-faithful
oracle (oracle/dfm_oracle.py) on the BASELINE configs' shapes at reduced B.
They freeze the oracle's outputs (so a later edit cannot drift silently) and
are the inputs/expected outputs of the GPU parity tests.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import dfm_oracle as O  # noqa: E402
import dfm_xp as XP  # noqa: E402


def c1():
    """C1: Bai–Ng DGP T=200 N=100 r=3, fit at r=3 + IC sweep k<=8, all criteria."""
    rng = np.random.default_rng(20261015 + 1)
    T, N, r = 200, 100, 3
    y, x, *_ = O.factor_model_DGP(T, N, r, rng)
    x = O.normalize(x)
    w = np.ones((T, 1))
    fit = O.DynamicFactorModel(y, w, x, r, "ICp2")
    ic = O.ic_sweep_values(y, w, x, 8)
    best = O.DynamicFactorModel_ic(y, w, x, "ICp2", kmax=8)
    np.savez_compressed(
        os.path.join(HERE, "c1_bai_ng_T200_N100_r3.npz"),
        y=y, w=w, x=x, r=r, eigvals=fit.eigenvalues[0][:16], F=fit.F, L=fit.loadings[0][:, :r],
        coefficients=fit.coefficients, t_stats=fit.t_stats, coef_cov=fit.coefficient_covariance,
        residuals=fit.residuals, V=O.factor_residual_variance(fit),
        crit_ICp2=fit.number_of_factors_criterion_value, ic_values=ic,
        ic_best_r=best.number_of_factors, factor_residuals=fit.factor_residuals)


def c2():
    """C2: Breitung–Eickmeier DGP T=600 N=130 b=0.5, r by ICp2 over 1..8, wild
    bootstrap B=16 with V, ICp2 and the Chow LR/LM/Wald of variables 1..6."""
    rng = np.random.default_rng(20261015 + 2)
    T, N = 600, 130
    y, x, *_ = O.factor_model_DGP(T, N, 3, rng, model="Breitung_Eickmeier_2011", b=0.5)
    x = O.normalize(x)
    w = np.ones((T, 1))
    base = O.DynamicFactorModel_ic(y, w, x, "ICp2", kmax=8)
    r = base.number_of_factors
    B, bp, nv = 16, 300, 6
    idx, eta = O.draw_wild(np.random.default_rng(99), B, T)
    common, E = base.common_component, base.factor_residuals
    rows = []
    for b in range(B):
        d = O.DynamicFactorModel(y, w, common + eta[b][:, None] * E[idx[b]], r, "ICp2")
        row = [O.factor_residual_variance(d), d.number_of_factors_criterion_value]
        row += [O.LR_test(d, bp, i) for i in range(nv)]
        row += [O.LM_test(d, bp, i) for i in range(nv)]
        row += [O.Wald_test(d, bp, i) for i in range(nv)]
        rows.append(row)
    base_chow = np.array([[O.LR_test(base, bp, i), O.LM_test(base, bp, i), O.Wald_test(base, bp, i)]
                          for i in range(N)])
    np.savez_compressed(
        os.path.join(HERE, "c2_breitung_eickmeier_T600_N130_B16.npz"),
        y=y, w=w, x=x, r=r, bp=bp, nv=nv, idx=idx, eta=eta, boot=np.array(rows),
        base_V=O.factor_residual_variance(base), base_crit=base.number_of_factors_criterion_value,
        base_chow=base_chow, base_eigvals=base.eigenvalues[0][:16])


def tp():
    """Targeted predictors (hard): JOINT at T=200, N=40 and PER_CANDIDATE at
    a C4-shaped T=400, N=250 slice."""
    rng = np.random.default_rng(20261015 + 4)
    y, x, *_ = O.factor_model_DGP(200, 40, 3, rng)
    x = O.normalize(x)
    w = np.ones((200, 1))
    tj, mj = O.targeted_predictors_hard(y, w, x, "joint")
    y2, x2, *_ = O.factor_model_DGP(400, 250, 5, rng)
    x2 = O.normalize(x2)
    w2 = np.ones((400, 1))
    tc, mc = O.targeted_predictors_hard(y2, w2, x2, "per_candidate")
    np.savez_compressed(os.path.join(HERE, "tp_hard.npz"), y=y, w=w, x=x, t_joint=tj, m_joint=mj,
                        y2=y2, w2=w2, x2=x2, t_cand=tc, m_cand=mc)


def c4_inputs():
    """C4 panel (regenerated, not stored: 16 MB): Bai-Ng DGP T=400, N=5000,
    r=5, y = f beta + eps, normalised x, w = 1, GLMNet.jl default folds."""
    rng = np.random.default_rng(20261015 + 4)
    T, N = 400, 5000
    y, x, *_ = O.factor_model_DGP(T, N, 5, rng)
    x = O.normalize(x)
    w = np.ones((T, 1))
    folds = O.glmnet_default_folds(T, np.random.default_rng(404))
    return y, w, x, folds


def soft():
    """Targeted predictors (soft, glmnetcv lasso): a small panel with its
    inputs, and the full C4 panel (T=400, N=5000) as outputs + input digest."""
    rng = np.random.default_rng(20261015 + 5)
    y, x, *_ = O.factor_model_DGP(120, 300, 3, rng)
    x = O.normalize(x)
    w = np.ones((120, 1))
    folds = O.glmnet_default_folds(120, np.random.default_rng(5))
    mask, res = O.targeted_predictors_soft(y, w, x, folds)
    y4, w4, x4, f4 = c4_inputs()
    mask4, res4 = O.targeted_predictors_soft(y4, w4, x4, f4)
    np.savez_compressed(
        os.path.join(HERE, "tp_soft.npz"), y=y, w=w, x=x, folds=folds, mask=mask,
        lam=res["lambda"], meanloss=res["meanloss"], best=res["best"], beta=res["betas"][res["best"]],
        a0=res["a0"][res["best"]],
        c4_digest=np.array([x4.sum(), np.abs(x4).sum(), y4.sum(), f4.sum()]), c4_mask=mask4,
        c4_lam=res4["lambda"], c4_meanloss=res4["meanloss"], c4_best=res4["best"],
        c4_beta=res4["betas"][res4["best"]])


def c5():
    """C5 (BASELINE.json configs[4]) at full size: Bai-Ng DGP T=2000 N=20000
    r=8, normalised, w = 1; the refits of pseudo_out_of_sample_forecasts
    (src/utils.jl:54-72, P = 200) for windows 0, 100, 199 — each the IC-sweep
    constructor DynamicFactorModel_ic(kmax=8) on rows 1..T-P+w — by the
    reference-faithful oracle.  The panel (320 MB) is not stored: its seed
    and a digest are."""
    rng = np.random.default_rng(20261015 + 5)
    T, N, P = 2000, 20000, 200
    y, x, *_ = O.factor_model_DGP(T, N, 8, rng)
    x = O.normalize(x)
    w = np.ones((T, 1))
    wins = [0, 100, 199]
    rows = {"r": [], "V": [], "crit": [], "eigvals": [], "coef": [], "tstat": []}
    for wi in wins:
        n = T - P + wi
        d = O.DynamicFactorModel_ic(y[:n], w[:n], x[:n], "ICp2", kmax=8)
        r = d.number_of_factors
        rows["r"].append(r)
        rows["V"].append(O.factor_residual_variance(d))
        rows["crit"].append(d.number_of_factors_criterion_value)
        rows["eigvals"].append(d.eigenvalues[0][:8])
        c = np.full(9, np.nan)
        t = np.full(9, np.nan)
        c[:1 + r] = d.coefficients
        t[:1 + r] = d.t_stats
        rows["coef"].append(c)
        rows["tstat"].append(t)
        print("c5 window", wi, "r", r, flush=True)
    np.savez_compressed(os.path.join(HERE, "c5_windows.npz"), windows=np.array(wins),
                        digest=np.array([x.sum(), np.abs(x).sum(), y.sum()]),
                        **{k: np.array(v) for k, v in rows.items()})


def c5_rolling():
    """C5's rolling form (BASELINE.json configs[4], `bench.py --workload c5
    --rolling 1000`) at full size: the same panel as c5(); window w is the
    IC-sweep constructor DynamicFactorModel_ic(kmax=8) on the L = 1000 rows
    before date_index = T-P+1+w (0-based rows T-P-L+w .. T-P+w-1), windows 0,
    100, 199, by the reference-faithful oracle."""
    rng = np.random.default_rng(20261015 + 5)
    T, N, P, L = 2000, 20000, 200, 1000
    y, x, *_ = O.factor_model_DGP(T, N, 8, rng)
    x = O.normalize(x)
    w = np.ones((T, 1))
    wins = [0, 100, 199]
    rows = {"r": [], "V": [], "crit": [], "eigvals": [], "coef": [], "tstat": []}
    for wi in wins:
        a = T - P - L + wi
        d = O.DynamicFactorModel_ic(y[a:a + L], w[a:a + L], x[a:a + L], "ICp2", kmax=8)
        r = d.number_of_factors
        rows["r"].append(r)
        rows["V"].append(O.factor_residual_variance(d))
        rows["crit"].append(d.number_of_factors_criterion_value)
        rows["eigvals"].append(d.eigenvalues[0][:8])
        c = np.full(9, np.nan)
        t = np.full(9, np.nan)
        c[:1 + r] = d.coefficients
        t[:1 + r] = d.t_stats
        rows["coef"].append(c)
        rows["tstat"].append(t)
        print("c5 rolling window", wi, "r", r, flush=True)
    np.savez_compressed(os.path.join(HERE, "c5_rolling.npz"), windows=np.array(wins), L=np.array(L),
                        digest=np.array([x.sum(), np.abs(x).sum(), y.sum()]),
                        **{k: np.array(v) for k, v in rows.items()})


def xp():
    """Extended-precision (double-double) referee values for golden C1 and C2
    (oracle/dfm_xp.py): the values the reference's algebra defines, to ~1e-28,
    and each one's parity bar max(1e-10 |exact|, |oracle - exact|) — the GPU
    must be within 1e-10 relative of the exact value, or no further from it
    than the fp64 oracle is.  C2: the base fit's Chow LR/LM/Wald of all 130
    variables, and V, ICp2 and all 3 x 130 Chow statistics of each of the 16
    wild-bootstrap replicates (same idx/eta as the C2 fixture)."""
    def bar(exact, orc):
        exact, orc = np.asarray(exact, float), np.asarray(orc, float)
        return np.maximum(1e-10 * np.abs(exact), np.abs(orc - exact))

    out = {}
    g = np.load(os.path.join(HERE, "c1_bai_ng_T200_N100_r3.npz"))
    f = XP.XPFit(g["y"], g["w"], g["x"], int(g["r"]), "ICp2")
    o = O.DynamicFactorModel(g["y"], g["w"], g["x"], int(g["r"]), "ICp2")
    s = np.sign(np.sum(f.F.f64() * o.F, axis=0))
    coef, t = f.coefficients.f64(), f.t_stats.copy()
    coef[1:] *= s
    t[1:] *= s
    out.update(c1_coef=coef, c1_coef_bar=bar(coef, o.coefficients), c1_t=t, c1_t_bar=bar(t, o.t_stats),
               c1_V=f.V.f64(), c1_eig=f.lam[:16].f64(), c1_ICp2=f.criterion_value("ICp2"))
    ic = np.empty((len(O.CRITERIA), 8))
    h = (100 + 1) // 2
    s2 = (f.trace - f.lam[:h].sum()) / float(200 * 100)
    for k in range(1, 9):
        fk = XP.XPFit(g["y"], g["w"], g["x"], k)
        for ci, name in enumerate(O.CRITERIA):
            ic[ci, k - 1] = fk.criterion_value(name, s2)
    out.update(c1_ic=ic, c1_ic_bar=bar(ic, g["ic_values"]))
    print("xp c1 done", flush=True)

    g = np.load(os.path.join(HERE, "c2_breitung_eickmeier_T600_N130_B16.npz"))
    r, bp = int(g["r"]), int(g["bp"])
    N = g["x"].shape[1]
    f = XP.XPFit(g["y"], g["w"], g["x"], r, "ICp2")
    base = np.column_stack(f.chow_all(bp))
    out.update(c2_base_chow=base, c2_base_chow_bar=bar(base, g["base_chow"]), c2_base_V=f.V.f64())
    o = O.DynamicFactorModel(g["y"], g["w"], g["x"], r, "ICp2")
    C, E = o.common_component, o.factor_residuals
    rows, bars = [], []
    for b in range(g["idx"].shape[0]):
        xs = f.replicate(g["idx"][b], g["eta"][b])
        fb = XP.XPFit(g["y"], g["w"], xs, r, "ICp2")
        ex = np.concatenate([[fb.V.f64(), fb.criterion_value("ICp2")], *fb.chow_all(bp)])
        d = O.DynamicFactorModel(g["y"], g["w"], C + g["eta"][b][:, None] * E[g["idx"][b]], r, "ICp2")
        orc = np.concatenate([[O.factor_residual_variance(d), d.number_of_factors_criterion_value],
                              [O.LR_test(d, bp, i) for i in range(N)], [O.LM_test(d, bp, i) for i in range(N)],
                              [O.Wald_test(d, bp, i) for i in range(N)]])
        rows.append(ex)
        bars.append(bar(ex, orc))
        print("xp c2 replicate", b, "oracle max rel dev", float(np.max(np.abs(orc - ex) / np.abs(ex))), flush=True)
    out.update(c2_boot=np.array(rows), c2_boot_bar=np.array(bars))
    np.savez_compressed(os.path.join(HERE, "xp_c1_c2.npz"), **out)


if __name__ == "__main__":
    import sys as _s
    if len(_s.argv) > 1:          # regenerate selected fixtures, e.g. `make_golden.py c5`
        for name in _s.argv[1:]:
            globals()[name]()
        raise SystemExit(0)
    c1()
    c2()
    tp()
    soft()
    c5()
    c5_rolling()
    print("golden fixtures written to", HERE)
