#!/usr/bin/env python3
"""Secondary measurements: the BASELINE.json configs other than the headline
C3 (bench.py).  One JSON line per config on stdout; the CPU column is the
reference-faithful oracle (oracle/dfm_oracle.py) on this host, bounded.

    python tools/bench_configs.py [--configs c1,c2,c4,c5] [--cpu] [--reps K]

c1  Simulated DFM T=200 N=100 r=3: fit + Bai-Ng IC sweep k<=8 (all 7 criteria)
c2  FRED-MD-shaped T=600 N=130, r by ICp2 over 1..8, wild bootstrap B=999 with
    LR/LM/Wald for all 130 variables at bp=300 (+ V, ICp2)      [replicates/s]
c4  Targeted predictors T=400 N=5000: hard per-candidate t-stats, soft
    glmnetcv lasso (100 lambdas x 10 folds), then PCA (r=5) on the soft
    selection                                                  [selections/s]
c5  T=2000 N=20000: P=200 expanding windows, IC sweep (ICp2, kmax 8) each
    (src/utils.jl:54-72 refit loop)                               [windows/s]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps, sync):
    fn()
    sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    sync()
    return (time.perf_counter() - t0) / reps


def oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import dfm_oracle as O
    return O


def cores():
    try:
        from threadpoolctl import threadpool_info
        return max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        return os.cpu_count()


def c1(D, ctx, args):
    rng = np.random.default_rng(20261015 + 1)
    y, x, *_ = D.factor_model_DGP(200, 100, 3, rng=rng)
    x = D.normalize(x)
    w = np.ones((200, 1))
    s = timed(lambda: D.DynamicFactorModel(y, w, x, "ICp2", kmax=8, ctx=ctx), args.reps, ctx.synchronize)
    rec = {"config": "c1", "workload": "fit + IC sweep k<=8, T=200 N=100 (host buffers in/out)",
           "value": round(1.0 / s, 3), "unit": "fits/s", "ms": round(s * 1e3, 3)}
    if args.cpu:
        O = oracle()
        t0 = time.perf_counter()
        O.DynamicFactorModel_ic(y, w, x, "ICp2", kmax=8)
        O.ic_sweep_values(y, w, x, 8)
        el = time.perf_counter() - t0
        rec["cpu_baseline"] = {"value": round(1 / el, 3), "unit": "fits/s", "cores": cores(), "kind": "port",
                               "sample": "1 oracle IC sweep (8 brute-force refits) + all-criteria table"}
    return rec


def c2_pmc_bytes(prefix):
    """DRAM bytes per launch of the C2 kernel named `prefix` from the latest
    committed C2 PMC passes (profiles/rNN_pmc_traffic_c2.json,
    tools/pmc_traffic.py; one launch = one 500-replicate lane); None when absent."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc_traffic_c2.json")))
    if not files:
        return None
    rec = json.load(open(files[-1]))
    for k, v in rec.items():
        if k.startswith(prefix):
            return {"hbm_bytes_per_launch": v.get("hbm_bytes_per_launch"), "source": os.path.basename(files[-1])}
    return None


def c2(D, ctx, args):
    import torch
    rng = np.random.default_rng(20261015 + 2)
    T, N, B, bp = 600, 130, 999, 300
    y, x, *_ = D.factor_model_DGP(T, N, 3, model="Breitung_Eickmeier_2011", b=0.5, rng=rng)
    x = D.normalize(x)
    w = np.ones((T, 1))
    model = D.DynamicFactorModel(y, w, x, "ICp2", kmax=8, ctx=ctx)
    S = D.Stat
    stats = [S.V(), S.criterion(), S.LR_all(bp), S.LM_all(bp), S.Wald_all(bp)]
    arr = D.api._stat_array(stats)
    width = int(ctx.lib.dfm_stats_width(model.handle, arr, len(stats)))
    idx, eta = D.draw_wild_fast(7, B, T)
    dev = torch.device("cuda", 0)
    di, de = torch.from_numpy(idx).to(dev), torch.from_numpy(eta).to(dev)
    out = torch.empty((B, width), dtype=torch.float64, device=dev)
    torch.cuda.synchronize()

    def run():
        ctx.check(ctx.lib.dfm_bootstrap_dev(model.handle, 0, B, di.data_ptr(), de.data_ptr(), arr, len(stats),
                                            out.data_ptr()))
    run()
    ctx.synchronize()
    ctx.reset_timing()
    ctx.enable_timing(True)
    s = timed(run, args.reps, ctx.synchronize)
    ctx.enable_timing(False)
    tm = ctx.read_timing()
    rec = {"config": "c2", "workload": f"wild bootstrap B={B}, T={T} N={N} r={model.number_of_factors}, "
                                       f"LR/LM/Wald all variables at bp={bp} + V + ICp2 (inputs resident)",
           "value": round(B / s, 1), "unit": "replicates/s", "ms_per_job": round(s * 1e3, 3),
           "kernels_ms_per_job": {k: round(v[0] / (args.reps + 1), 4) for k, v in tm.items() if v[1]}}
    es = ctx.eig_stats()
    rec["eig_iterations"] = dict(es, rayleigh_ritz_steps_per_replicate=round(
        es["replicate_iterations"] / (B * (args.reps + 1)), 3))
    # Gram roofline: the replicate Grams X*'X* (130 x 130 over T = 600), SYRK
    # count N (N + 1) T per replicate (the weighted GEMM Q = W K
    # of the gram_wk path does 2 T N (N + 1) / 2, the same count), over the
    # HIP-event time of the whole Gram phase (prep + GEMM + combine)
    gms, gn = tm.get("gram", (0.0, 0))
    if gn:
        flop = B * (args.reps + 1) * N * (N + 1) * T
        rec["roofline_gram"] = {"kernel": "gram_wk: prep (w, B = F'DPE) + ONE batch GEMM Q = W K on gemmh_kernel_t "
                                          "(v_mfma_f64_4x4x4_4b) + tiled symmetric combine",
                                "bound": "mfma", "achieved": round(flop / (gms * 1e-3) / 1e12, 3), "peak": 78.6,
                                "unit": "TFLOP/s", "frac": round(flop / (gms * 1e-3) / 1e12 / 78.6, 4),
                                "avg_launch_ms": round(gms / gn, 4), "flop_per_replicate": N * (N + 1) * T}
    # Chow pass, labelled by its measured bound: fp64 VALU.  Per
    # (replicate, variable) and row t, pass A forms e = x - F_t l (r FMA), ||e||^2
    # (1) and F_t'x (r); pass B the subperiod residuals u, rs (2 r), ssr (1),
    # u^2 z_t (r) and the HC0 block's r (r + 1) / 2 sums: 5 r + 2 + r (r + 1) / 2
    # FMA = 2 x that in flop.  Its DRAM traffic (PMC FETCH_SIZE / WRITE_SIZE,
    # profiles/*_pmc_traffic_c2.json) is far below HBM peak: the gathered x rows
    # come from the L2-resident C and E panels.
    # Fused direct eigensolver (eig_fused_kernel, class eig_gq): MFMA products
    # G S of the replicate's m x m Gram with the 16-column block, 2 m^2 16 flop
    # each; dfm_ctx_gemm_products counts them exactly (a[i] replicates at
    # Rayleigh-Ritz step i, dg(i) products each).  A per-replicate latency
    # chain (one workgroup per replicate): the frac says how far from the MFMA
    # peak that chain runs, the PMC bytes that it is not HBM-bound either.
    ems, en = tm.get("eig_gq", (0.0, 0))
    if en and es.get("gemm_products"):
        m = min(T, N)
        fl = 2.0 * m * m * 16 * es["gemm_products"]
        tf = fl / (ems * 1e-3) / 1e12
        rec["roofline_eig_fused"] = {"kernel": "eig_fused_kernel (one workgroup per replicate, Q and Y in LDS, "
                                               "G streamed from L2/MALL, v_mfma_f64_4x4x4_4b)",
                                     "bound": "mfma (latency chain)", "achieved": round(tf, 3), "peak": 78.6,
                                     "unit": "TFLOP/s", "frac": round(tf / 78.6, 4),
                                     "products_per_replicate": round(es["gemm_products"] / (B * (args.reps + 1)), 2),
                                     "flop_per_product": 2 * m * m * 16,
                                     "traffic": c2_pmc_bytes("eig_fused_kernel")}
    cms, cn = tm.get("chow", (0.0, 0))
    if cn:
        r = model.number_of_factors
        fl = B * (args.reps + 1) * N * T * 2 * (5 * r + 2 + r * (r + 1) // 2)
        tf = fl / (cms * 1e-3) / 1e12
        rec["roofline_chow"] = {"kernel": "chow_prep + chow_all_kernel", "bound": "valu (fp64)",
                                "achieved": round(tf, 3), "peak": 78.6, "unit": "TFLOP/s",
                                "frac": round(tf / 78.6, 4),
                                "flop_per_replicate": N * T * 2 * (5 * r + 2 + r * (r + 1) // 2),
                                "traffic": c2_pmc_bytes("chow_all_kernel")}
    if args.cpu:
        O = oracle()
        o = O.DynamicFactorModel_ic(y, w, x, "ICp2", kmax=8)
        C, E = o.common_component, o.factor_residuals
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_seconds or n < 1:
            d = O.DynamicFactorModel(y, w, C + eta[n][:, None] * E[idx[n]], o.number_of_factors, "ICp2")
            for i in range(N):
                O.LR_test(d, bp, i), O.LM_test(d, bp, i), O.Wald_test(d, bp, i)
            n += 1
        el = time.perf_counter() - t0
        rec["cpu_baseline"] = {"value": round(n / el, 4), "unit": "replicates/s", "cores": cores(), "kind": "port",
                               "sample": f"{n} oracle replicates (refit + 3 x {N} Chow tests) in {el:.1f} s"}
    return rec


def c4(D, ctx, args):
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    rng = np.random.default_rng(20261015 + 4)
    T, N = 400, 5000
    y, x, *_ = D.factor_model_DGP(T, N, 5, rng=rng)
    x = D.normalize(x)
    w = np.ones((T, 1))
    folds = D.glmnet_default_folds(T, np.random.default_rng(404))
    parts = {}

    def run():
        t0 = time.perf_counter()
        hard = D.targeted_predictors(y, w, x, "hard", "per_candidate", ctx=ctx)
        t1 = time.perf_counter()
        soft = D.targeted_predictors(y, w, x, "soft", folds=folds, ctx=ctx)
        t2 = time.perf_counter()
        D.principal_components(x[:, soft], 5, ctx=ctx)
        t3 = time.perf_counter()
        parts.update(hard_ms=(t1 - t0) * 1e3, soft_ms=(t2 - t1) * 1e3, pca_ms=(t3 - t2) * 1e3,
                     n_hard=int(hard.sum()), n_soft=int(soft.sum()))
    s = timed(run, args.reps, ctx.synchronize)
    rec = {"config": "c4", "workload": "hard per-candidate t-stats + soft glmnetcv (100 lambdas, 10 folds) "
                                       "+ PCA r=5 on the soft selection, T=400 N=5000 (host buffers in/out)",
           "value": round(1.0 / s, 3), "unit": "selections/s", "ms": round(s * 1e3, 2),
           "parts_ms": {k: round(v, 2) for k, v in parts.items() if k.endswith("ms")},
           "selected": {"hard": parts["n_hard"], "soft": parts["n_soft"]}}
    if args.cpu:
        O = oracle()
        t0 = time.perf_counter()
        O.targeted_predictors_hard(y, w, x, "per_candidate")
        t1 = time.perf_counter()
        m, _ = O.targeted_predictors_soft(y, w, x, folds)
        t2 = time.perf_counter()
        O.principal_components(x[:, m], T, int(m.sum()))
        el = time.perf_counter() - t0
        rec["cpu_baseline"] = {"value": round(1 / el, 5), "unit": "selections/s", "cores": cores(), "kind": "port",
                               "sample": f"1 oracle selection: hard {t1 - t0:.1f} s, soft {t2 - t1:.1f} s"}
    return rec


def c5(D, ctx, args):
    rng = np.random.default_rng(20261015 + 5)
    T, N, P = 2000, 20000, 200
    y, x, *_ = D.factor_model_DGP(T, N, 8, rng=rng)
    # column-major host panel, as a Julia caller hands it over (no harness
    # transpose inside the timed region; the PCIe upload stays in)
    x = np.asfortranarray(D.normalize(x))
    w = np.asfortranarray(np.ones((T, 1)))
    out = {}
    s = timed(lambda: out.update(D.pseudo_out_of_sample_refits(y, w, x, "ICp2", num_predictions=P, kmax=8,
                                                                ctx=ctx)), max(1, args.reps // 2), ctx.synchronize)
    rec = {"config": "c5", "workload": f"{P} expanding windows (rows 1..t-1, t = T-P+1..T) x IC sweep ICp2 "
                                       f"kmax 8, T={T} N={N} (host panel in, per-window results out)",
           "value": round(P / s, 2), "unit": "windows/s", "ms_per_job": round(s * 1e3, 1),
           "r_selected": sorted(set(int(v) for v in out["number_of_factors"]))}
    if args.cpu:
        O = oracle()
        t0 = time.perf_counter()
        O.DynamicFactorModel_ic(y[:T - 1], w[:T - 1], x[:T - 1], "ICp2", kmax=8)
        el = time.perf_counter() - t0
        rec["cpu_baseline"] = {"value": round(1 / el, 5), "unit": "windows/s", "cores": cores(), "kind": "port",
                               "sample": f"1 oracle window (T-1 rows, 8 brute-force refits) in {el:.1f} s"}
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c1,c2,c4,c5")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu", action="store_true", help="also time the CPU oracle (bounded samples)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--dump-maps", default="", help="copy /proc/self/maps here at interpreter exit (names the "
                                                      "libraries behind addresses in an exit-time stack trace)")
    args = ap.parse_args()
    if args.dump_maps:
        import atexit
        import shutil
        atexit.register(lambda: shutil.copyfile("/proc/self/maps", args.dump_maps))
    import torch  # noqa: F401  (before libdfm: one HIP runtime in the process, as bench.py)
    torch.cuda.init()
    import dfm_pkg
    D = dfm_pkg.load()
    ctx = D.Context(0)
    for name in args.configs.split(","):
        rec = globals()[name](D, ctx, args)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
