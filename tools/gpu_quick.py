"""Quick GPU-vs-oracle diff script (development aid; the real checks live in tests/)."""
import sys, os, time, math
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import dfm_pkg
sys.path.insert(0, os.path.join(dfm_pkg.ROOT, "oracle"))
import dfm_oracle as O
D = dfm_pkg.load()

def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))

def align(F, Fo):
    s = np.sign(np.sum(F * Fo, axis=0)); s[s == 0] = 1
    return F * s

def check_fit(T, N, r, seed, crit=""):
    rng = np.random.default_rng(seed)
    y, x, *_ = O.factor_model_DGP(T, N, r, rng)
    x = O.normalize(x)
    w = np.ones((T, 1))
    t0 = time.time()
    g = D.DynamicFactorModel(y, w, x, r, crit)
    t1 = time.time()
    o = O.DynamicFactorModel(y, w, x, r, crit)
    F, Fo = g.factors[0], o.F
    Fa = align(F, Fo)
    print(f"fit T={T} N={N} r={r}: gpu {t1-t0:.3f}s  eig rel {rel(g.eigenvalues[:r], o.eigenvalues[0][:r]):.2e}"
          f"  F rel {rel(Fa, Fo):.2e}  V rel {abs(g.V - O.factor_residual_variance(o))/O.factor_residual_variance(o):.2e}"
          f"  E rel {rel(g.factor_residuals, o.factor_residuals):.2e}")
    s = np.sign(np.sum(F * Fo, axis=0))
    cg = g.coefficients.copy(); cg[1:] *= s
    tg = g.t_stats.copy(); tg[1:] *= s
    print(f"   coef rel {rel(cg, o.coefficients):.2e}  t rel {rel(tg, o.t_stats):.2e}  crit {g.number_of_factors_criterion_value} vs {o.number_of_factors_criterion_value}")
    return g, o, y, w, x

g, o, y, w, x = check_fit(200, 100, 3, 1, "ICp2")
check_fit(60, 150, 4, 2, "ICp2")
check_fit(500, 2000, 8, 3, "ICp2")
# IC sweep C1
rng = np.random.default_rng(20261016)
y, x, *_ = O.factor_model_DGP(200, 100, 3, rng); x = O.normalize(x); w = np.ones((200, 1))
gs = D.DynamicFactorModel(y, w, x, "ICp2", kmax=8)
ic_o = O.ic_sweep_values(y, w, x, 8)
print("IC sweep r:", gs.number_of_factors, " ic rel", rel(gs.ic_values, ic_o))
# Chow
LR, LM, W = D.chow_all(g, 100)
print("chow LR", rel(LR[:5], [O.LR_test(o, 100, i) for i in range(5)]),
      "LM", rel(LM[:5], [O.LM_test(o, 100, i) for i in range(5)]),
      "Wald", rel(W[:5], [O.Wald_test(o, 100, i) for i in range(5)]))
# bootstrap
B = 8
idx, eta = O.draw_wild(np.random.default_rng(5), B, 200)
stats = [D.Stat.V(), D.Stat.criterion(), D.Stat.eigenvalue(1), D.Stat.t_stat(1)]
t0 = time.time()
sg = D.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
t1 = time.time()
so = np.array([[O.factor_residual_variance(d), d.number_of_factors_criterion_value, d.eigenvalues[0][0], d.t_stats[0]]
               for d in [O.DynamicFactorModel(o.y, o.w, o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]], 3, "ICp2") for b in range(B)]])
print(f"boot gpu {t1-t0:.3f}s rel per stat:", [rel(sg[:, j], so[:, j]) for j in range(4)])
sgc = D.wild_bootstrap(g, B, [D.Stat.LR_all(100), D.Stat.Wald(100, 3)], idx=idx, eta=eta)
ob = [O.DynamicFactorModel(o.y, o.w, o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]], 3, "ICp2") for b in range(B)]
print("boot chow LR rel", rel(sgc[:, :5], np.array([[O.LR_test(d, 100, i) for i in range(5)] for d in ob])),
      "Wald(3) rel", rel(sgc[:, 100], [O.Wald_test(d, 100, 2) for d in ob]))
# targeted
rng = np.random.default_rng(7)
y, x, *_ = O.factor_model_DGP(200, 30, 3, rng); x = O.normalize(x); w = np.ones((200, 1))
mg, tg = D.targeted_predictors(y, w, x, return_tstats=True)
to, mo = O.targeted_predictors_hard(y, w, x)
print("tp joint t rel", rel(tg, to), "mask eq", bool(np.all(mg == mo)))
mg, tg = D.targeted_predictors(y, w, x, mode="per_candidate", return_tstats=True)
to, mo = O.targeted_predictors_hard(y, w, x, mode="per_candidate")
print("tp cand t rel", rel(tg, to), "mask eq", bool(np.all(mg == mo)))
