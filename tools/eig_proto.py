"""CPU prototype (NumPy) of the factored bootstrap's eigen-iteration at the C3
shape, to explore warm starts and filter schedules before touching kernels:
block p = 16, Rayleigh-Ritz with CholQR, Chebyshev filter on [0, theta_p],
the eigenvalue (Kato-Temple) stopping rule of decide_converged (1e-12).
Reports Rayleigh-Ritz steps and G-products per replicate.
  python tools/eig_proto.py [nrep] [schedule ...]   schedule e.g. "r8:2,2" "w16:2,2" "w16:3,2"
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dynamicfactormodels.jl_amd"))
import host  # noqa: E402

T, N, R = 500, 2000, 8
P = int(os.environ.get("P", "16"))


def shifted_cheb(d):
    t0, t1 = np.zeros(d + 1), np.zeros(d + 1)
    t0[0] = 1.0
    if d == 0:
        return t0
    t1[0], t1[1] = -1.0, 2.0
    for _ in range(1, d):
        t2 = -2.0 * t1 - t0
        t2[1:] += 4.0 * t1[:-1]
        t0, t1 = t1, t2
    return t1


def solve(G, Q0, degs, k=R, tol=1e-12, maxit=30, beta=0.0, strict=False):
    Q = Q0.copy()
    tr = np.trace(G)
    prods = 0
    for it in range(maxit):
        Y = G @ Q
        prods += 1
        L = np.linalg.cholesky(Q.T @ Q)
        Li = np.linalg.inv(L)
        Hm = Li @ (Q.T @ Y) @ Li.T
        Hm = 0.5 * (Hm + Hm.T)
        th, V = np.linalg.eigh(Hm)
        o = np.argsort(-th)
        th, V = th[o], V[:, o]
        A = Li.T @ V
        U = Q @ A
        Res = Y @ A - U * th
        res2 = np.sum(Res ** 2, axis=0)
        gap = np.full(P, np.inf)
        gap[1:] = np.minimum(gap[1:], np.abs(th[1:] - th[:-1]))
        gap[:-1] = np.minimum(gap[:-1], np.abs(th[:-1] - th[1:]))
        if strict:   # subspace rule: res_j <= tol |theta_j - theta_k|
            res = np.sqrt(res2[:k])
            if np.all((res <= tol * np.abs(th[:k] - th[k])) | (res <= 2e-14 * th[0])):
                return it + 1, prods
        else:
            bnd = res2[:k] / (0.5 * gap[:k])
            ok = np.all((bnd <= tol * np.abs(th[:k])) | (np.sqrt(res2[:k]) <= 2e-14 * th[0]))
            vnum = max(abs(tr - th[:k].sum()), 1e-6 * abs(tr))
            if ok and bnd.sum() <= tol * vnum:
                return it + 1, prods
        ZZ = A.T @ (Y.T @ Y) @ A
        L2 = np.linalg.cholesky(0.5 * (ZZ + ZZ.T))
        Bm = A @ np.linalg.inv(L2).T
        d = degs[min(it, len(degs) - 1)]
        b = th[P - 1]
        if it == 0 and beta > 0:   # first filter: interval end from the wanted Ritz values
            b = max(b, beta * th[k - 1])
        a = shifted_cheb(d)
        K = Q @ Bm                       # K_0
        X = a[0] * K
        Kn = Y @ Bm                      # K_1 = G K_0
        X = X + (a[1] / b) * Kn
        for s in range(2, d + 1):
            Kn = G @ Kn
            prods += 1
            X = X + (a[s] / b ** s) * Kn
        Q = X
    return maxit, prods


def main():
    nrep = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    scheds = sys.argv[2:] or ["r8:2", "w16:2", "w16:3,2", "w16:4,2", "w24:2"]
    global T, N, R
    c2 = os.environ.get("SHAPE") in ("c2", "c1")
    c1 = os.environ.get("SHAPE") == "c1"
    strict = c2 or os.environ.get("STRICT") == "1"
    if c1:   # tools/bench_configs.py c1: T = 200, N = 100, r = 3 (the fit itself: one Gram)
        T, N = 200, 100
        rng = np.random.default_rng(20261015 + 1)
        y, x, *_ = host.factor_model_DGP(T, N, 3, rng=rng)
        R = 3
    elif c2:   # tools/bench_configs.py c2: T = 600, N = 130, Breitung-Eickmeier DGP, r = 4 (ICp2)
        T, N = 600, 130
        rng = np.random.default_rng(20261015 + 2)
        y, x, *_ = host.factor_model_DGP(T, N, 3, model="Breitung_Eickmeier_2011", b=0.5, rng=rng)
        R = int(os.environ.get("R", "4"))
    else:
        rng = np.random.default_rng(20261015 + 3)
        y, x, *_ = host.factor_model_DGP(T, N, R, rng=rng)
    x = host.normalize(x)
    if c2:   # T >= N: the N x N Gram, eigenvectors = loadings directions
        x = x.T
        T, N = N, T
    G0 = x @ x.T
    lam, Uall = np.linalg.eigh(G0)
    Uall = Uall[:, ::-1]
    F = np.sqrt(T) * Uall[:, :R]
    Lb = x.T @ F / T
    C = F @ Lb.T
    E = x - C
    Tr = x.shape[1] if c2 else T   # rows resampled: the panel's time dimension
    idx, eta = host.draw_wild_fast(1_000_003, nrep, Tr)
    hrng = np.random.default_rng(5)
    rnd = hrng.uniform(-1, 1, size=(T, P))
    Gs = []
    for b in range(nrep):
        if c2:   # rows of the T x N panel are columns here
            Xs = C + eta[b][None, :] * E[:, idx[b]]
        else:
            Xs = C + eta[b][:, None] * E[idx[b]]
        Gs.append(Xs @ Xs.T)
    for sc in scheds:
        start, degs = sc.split(":")
        degs = [int(v) for v in degs.split(",")]
        beta = 0.0
        if "@" in start:
            start, beta = start.split("@")
            beta = float(beta)
        kw = int(start[1:])
        Q0 = np.hstack([Uall[:, :min(kw, P)], rnd[:, min(kw, P):]]) if start[0] in "rw" else None
        res = []
        for G in Gs:
            try:
                res.append(solve(G, Q0, degs, k=R, beta=beta, strict=strict,
                                 tol=float(os.environ.get("TOL", "1e-12"))))
            except np.linalg.LinAlgError:
                res.append((99, 99))
        its, prs = zip(*res)
        print(f"{sc:12s} RR steps mean {np.mean(its):.2f} max {max(its)}  products mean {np.mean(prs):.2f}"
              f"  hist {dict(zip(*np.unique(its, return_counts=True)))}")


if __name__ == "__main__":
    main()
