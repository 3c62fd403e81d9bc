"""C2: accuracy of the Chow statistics against the double-double referee
(tests/golden/xp_c1_c2.npz) and Rayleigh-Ritz steps per replicate, as a
function of the eigenvector-residual tolerance (dfm_ctx_set_eig_params)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import dfm_pkg
D = dfm_pkg.load()
G = os.path.join(dfm_pkg.ROOT, "tests", "golden")
g = np.load(os.path.join(G, "c2_breitung_eickmeier_T600_N130_B16.npz"))
xp = np.load(os.path.join(G, "xp_c1_c2.npz"))
ctx = D.default_context()
d = D.DynamicFactorModel(g["y"], g["w"], g["x"], "ICp2", kmax=8, ctx=ctx)
bp = int(g["bp"])
S = D.Stat
rng = np.random.default_rng(20261015 + 2)
T, N, B = 600, 130, 999
y, x, *_ = D.factor_model_DGP(T, N, 3, model="Breitung_Eickmeier_2011", b=0.5, rng=rng)
x = D.normalize(x)
m2 = D.DynamicFactorModel(y, np.ones((T, 1)), x, "ICp2", kmax=8, ctx=ctx)
idx, eta = D.draw_wild_fast(7, B, T)
for tol in (1e-12, 3e-12, 1e-11, 3e-11):
    ctx.set_eig_params(tol=tol)
    out = D.wild_bootstrap(d, 16, [S.V(), S.criterion(), S.LR_all(bp), S.LM_all(bp), S.Wald_all(bp)],
                           idx=g["idx"], eta=g["eta"])
    ex, bar = xp["c2_boot"], xp["c2_boot_bar"]
    dev = np.abs(out - ex)
    rel = dev / np.abs(ex)
    it = D.wild_bootstrap(m2, B, [S.iterations(), S.LR(bp, 1)], idx=idx, eta=eta)[:, 0]
    print(f"tol {tol:.0e}: max rel dev vs exact {rel.max():.2e} (LR {rel[:, 2:2+N].max():.2e} "
          f"LM {rel[:, 2+N:2+2*N].max():.2e} Wald {rel[:, 2+2*N:].max():.2e}), max dev/bar "
          f"{(dev / bar).max():.3f}; C2 job RR steps mean {it.mean():.2f} max {it.max():.0f}", flush=True)
