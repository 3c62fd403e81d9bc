"""N > T windows past the factored solver's T range (T > 4096): time of the
masked explicit-Gram path of dfm_windows_ex, one window, and its eigenvalues
against LAPACK on the window's rows.  `pca` mode: the same rows through
dfm_pca (the explicit-Gram subspace solver on one T x T Gram) for comparison."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import dfm_pkg
D = dfm_pkg.load()
mode = sys.argv[1] if len(sys.argv) > 1 else "windows"
T = int(sys.argv[2]) if len(sys.argv) > 2 else 4200
N, P, k = 4300, 1, 3
rng = np.random.default_rng(77)
f = rng.standard_normal((T, 3))
x = f @ rng.standard_normal((3, N)) * 2.0 + rng.standard_normal((T, N))
y = f @ np.ones(3) + rng.standard_normal(T)
w = np.ones((T, 1))
ctx = D.default_context()
ctx.reset_timing(); ctx.enable_timing(True)
print("start", mode, T, flush=True)
t0 = time.perf_counter()
if mode == "pca":
    ev, F, L, tr = D.principal_components(x[:T - 1], k)
else:
    out = D.pseudo_out_of_sample_windows(y, w, x, k, num_predictions=P)
    ev = out["eigenvalues"][0][:k]
el = time.perf_counter() - t0
ctx.enable_timing(False)
print(mode, "T", T, "time", round(el, 3), "s", {kk: v for kk, v in ctx.read_timing().items() if v[1]},
      "eig_stats", ctx.eig_stats(), flush=True)
import scipy.linalg as sla
n = T - P
xs = x[:n]
ref = sla.eigh(xs @ xs.T, eigvals_only=True, subset_by_index=[n - k, n - 1], driver="evr")[::-1]
print("eigenvalue rel err", float(np.max(np.abs(np.asarray(ev) - ref) / ref)), flush=True)
