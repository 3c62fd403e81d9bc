#!/usr/bin/env python3
"""Headline benchmark: wild-bootstrap replicates/s at T=500, N=2000, r=8
(BASELINE.json configs[2], the metric's config), one process per GPU.

A step = one complete B=9999-replicate wild-bootstrap job on each GPU
(src/bootstrap.jl:41-51: per replicate resample X* = F_r L_r' + diag(eta)
E[idx,:], refit the DFM at r = 8 and evaluate the stats V(8) and ICp2),
followed by the RCCL all-gather of the per-replicate statistics (torchrun).
What the refit forms is demand-driven: V(8) and ICp2 read only the top-8
eigenvalues of X*X*' and its trace (src/criteria.jl:5, :35-46), so the timed
job runs the eigensolve (factored identity: H.Z GEMMs + per-replicate
Rayleigh-Ritz, Kato-Temple eigenvalue stopping rule) and does NOT form the
replicate factors F*, loadings L* or the OLS + HC2 regression.  The line's
`all_fields` extra (timed separately, after the headline region) is the rate
with the whole regression record per replicate — F*, L*, all OLS
coefficients and HC2 t-statistics (src/DynamicFactorModel.jl:28-51).  Replicates shard
across ranks (strong scaling, as BASELINE.json configs[2] states: the 9999
replicates of a step are sharded contiguously over the ranks, replicate b on
rank floor(b N / B); a weak-scaling extra field reruns with 9999 per rank).  Inputs (the fitted base model and every replicate's idx/eta) are
resident in HBM before the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

A plain `python bench.py --gpus N` with N > 1 (no torchrun environment) is a
launcher: before anything touches a GPU it starts `torch.distributed.run` with
N ranks as a CHILD process (never an exec), forwards its output and exits with
its status.  Under torchrun, --gpus must equal WORLD_SIZE.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

T, N, R, B = 500, 2000, 8, 9999
SYRK_FLOP = T * (T + 1) * N          # per replicate (5.01e8)
PEAK_F64_TFLOPS = 78.6               # MI355X fp64 matrix, spec (measured 75.1 for 4x4x4_4b)
PEAK_HBM_GBS = 8000.0


def _c3_oracle_setup():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import dfm_oracle as O
    rng = np.random.default_rng(20261015 + 3)
    y, x, *_ = O.factor_model_DGP(T, N, R, rng)
    x = O.normalize(x)
    w = np.ones((T, 1))
    base = O.DynamicFactorModel(y, w, x, R, "ICp2")
    return O, y, w, base.common_component, base.factor_residuals


def _c3_oracle_loop(seconds: float, seed: int):
    """The reference-faithful replicate loop (src/bootstrap.jl:43-48) for
    `seconds`: (replicates done, elapsed)."""
    O, y, w, common, E = _c3_oracle_setup()
    draw = np.random.default_rng(seed)
    n, t0 = 0, time.perf_counter()
    while True:
        idx = draw.integers(0, T, size=T)
        eta = draw.standard_normal(T)
        d = O.DynamicFactorModel(y, w, common + eta[:, None] * E[idx], R, "ICp2")
        _ = (O.factor_residual_variance(d), d.number_of_factors_criterion_value)
        n += 1
        el = time.perf_counter() - t0
        if (el > seconds and n >= 2) or el > 4 * seconds:
            return n, el


def _pool_worker(args):
    return _c3_oracle_loop(*args)


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share():
    """CPUs this process may use: the affinity mask, capped by the cgroup's
    cpu.max quota when one is set (cgroup v2; v1's cfs quota otherwise).
    Returns (count, how it was determined)."""
    n = len(os.sched_getaffinity(0))
    how = f"sched_getaffinity: {n}"
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(p)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                p = int(f.read())
            if q > 0:
                quota = q / p
        except (OSError, ValueError):
            pass
    if quota is not None:
        how += f", cgroup quota {quota:g}"
        n = max(1, min(n, int(quota)))
    return n, how


def cpu_baseline(seconds: float = 12.0):
    """Reference-faithful oracle (full eig, full loadings, T x T hat matrix,
    serial replicate loop: the algorithm of src/bootstrap.jl:41-51 as written)
    on this host's cores, bounded samples, in the two modes of BASELINE.md:
      1. one process, OpenBLAS threads = the host's BLAS pool (Julia's serial
         loop over threaded BLAS);
      2. a pool of processes x 1 BLAS thread, one per CPU of this process's
         share (affinity mask and cgroup quota: cpu_share()); best CPU
         throughput for independent replicates.
    `value` is the faster mode."""
    try:
        from threadpoolctl import threadpool_info
        blas = [i for i in threadpool_info() if i.get("user_api") == "blas"]
        threads = max([i.get("num_threads", 1) for i in blas] or [1])
        blas_info = ", ".join(f"{i.get('internal_api')} {i.get('version')} x{i.get('num_threads')}" for i in blas)
    except Exception:
        threads, blas_info = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)), "unknown"
    n1, el1 = _c3_oracle_loop(seconds, 1)
    mode1 = {"value": n1 / el1, "cores": int(threads), "sample": f"{n1} replicates in {el1:.1f} s"}
    workers, share_how = cpu_share()
    import multiprocessing as mp
    saved = {k: os.environ.get(k) for k in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS", "MKL_NUM_THREADS")}
    for k in saved:
        os.environ[k] = "1"
    try:
        with mp.get_context("spawn").Pool(workers) as pool:
            res = pool.map(_pool_worker, [(seconds, 100 + i) for i in range(workers)])
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    n2 = sum(n for n, _ in res)
    v2 = sum(n / el for n, el in res)
    mode2 = {"value": v2, "cores": workers,
             "sample": f"{n2} replicates over {workers} processes x 1 BLAS thread, ~{seconds:.0f} s each"}
    best = mode2 if v2 > mode1["value"] else mode1
    return {"value": best["value"], "unit": "replicates/s", "cores": best["cores"], "kind": "port",
            "sample": f"C3 wild bootstrap (T=500 N=2000 r=8, V + ICp2), oracle/dfm_oracle.py "
                      f"reference-faithful loop; {best['sample']}",
            "modes": {"1_threaded_blas": mode1, "2_process_pool": mode2},
            "cpu_model": _cpu_model(), "os_cpu_count": os.cpu_count(), "cpu_share": share_how,
            "blas": blas_info}


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC pass
    (profiles/*_pmc_traffic.json, written by tools/pmc_traffic.py from
    FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE); None when absent."""
    import glob
    # the headline bench's own pass (rNN_pmc_traffic.json), not the C2 one (rNN_pmc_traffic_c2.json)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc_traffic.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        rec = json.load(f).get(kernel)
    return None if rec is None else rec.get("hbm_bytes_per_launch")


def rocprof_avg_ms(kernel_prefix):
    """Average launch duration of `kernel_prefix` in the latest committed
    rocprofv3 --kernel-trace --stats summary of this bench
    (profiles/*_bench_kernel_stats.csv); (ms, file) or (None, None)."""
    import csv
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_bench_kernel_stats.csv")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        for row in csv.DictReader(f):
            if row["Name"].replace("void ", "").startswith(kernel_prefix):
                return float(row["AverageNs"]) * 1e-6, os.path.basename(files[-1])
    return None, None


def hbm_rooflines(timing, eig, Bn, steps, pz=16):
    """Achieved HBM bandwidth of the per-replicate gather/residual passes of
    the factored solver (HIP-event time of their kernel class over the timed
    region; algorithmic bytes per replicate-pass; P = pz
    columns per row of the per-replicate buffers Q, Y, S, V0, PV (compact rows
    since round 6; 16 before); pz = the solver's block, rounded up to even =
    the columns of Z and HZ):
      y2  (class eig_gq):    Y = G*Q rows from the gathered HZ rows, Q'Y / Y'Y / Q'Q:
                             reads Q and HZ[idx], writes Y = (2 P + pz) T 8 B per Rayleigh-Ritz step
      ap2 (class eig_apply): (4 P + pz) T 8 B per pass (Q, Y in; the filter's first Horner term S,
                             V0 = Q Bm and Z out); passes = Rayleigh-Ritz steps + one init per replicate
      last Horner step of a filter (boot_cheb_kernel, class eig_apply): (3 P + 2 pz) T 8 B per pass
                             (HZ[idx], V0 in; S written and re-read by the CSR gather, Z out);
                             passes = one per filter = Rayleigh-Ritz steps - replicates
      middle Horner steps (boot_cheb_mid_kernel, class eig_apply): (pz + P + r + 1) T 8 B in
                             (HZ, PV, PF, e2 rows) + T pz 8 B out (Z); passes = the other
                             GEMM products after the Rayleigh-Ritz ones
    Replicate-passes come from the library's own counters (eig_iterations)."""
    P = pz
    out = []
    rr = eig.get("replicate_iterations", 0)
    cheb = max(eig.get("gemm_products", 0) - rr, 0)
    last = max(min(rr - Bn * steps, cheb), 0)
    t8 = T * 8
    for cls, name, parts in (
            ("eig_gq", "boot_y2_kernel", (((2 * P + pz) * t8, rr),)),
            ("eig_apply", "boot_ap2_kernel + boot_cheb_kernel + boot_cheb_mid_kernel",
             (((4 * P + pz) * t8, rr + Bn * steps), ((3 * P + 2 * pz) * t8, last),
              ((2 * pz + P + R + 1) * t8, cheb - last)))):
        ms, n = timing.get(cls, (0.0, 0))
        units = sum(u for _, u in parts)
        if not n or not units:
            continue
        byts = sum(b * u for b, u in parts)
        gbs = byts / (ms * 1e-3) / 1e9
        out.append({"kernel": name, "bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS,
                    "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4),
                    "bytes_per_replicate_pass": [b for b, _ in parts], "replicate_passes": [int(u) for _, u in parts]})
    return out


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """`python bench.py --gpus N` (N > 1, no torchrun environment): run the
    same command as N ranks under torch.distributed.run in a child process.
    This process imports no torch and makes no HIP call, so it never holds
    the GPU; rank 0's JSON line comes through its stdout.  Returns the
    child's exit status (non-zero if any rank failed)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    print(f"bench.py: launching {n} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    for line in p.stdout:
        sys.stdout.write(line)
        sys.stdout.flush()
    rc = p.wait()
    if rc != 0:
        print(f"bench.py: torch.distributed.run exited with status {rc}", file=sys.stderr, flush=True)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 20 timed steps after 3 warm-up steps: a C3 step is ~15 ms, so the default
    # timed region is ~0.3 s (5 steps read 641-652 k on the same build)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0, help="replicates per device batch (0 = auto)")
    ap.add_argument("--replicates", type=int, default=B)
    ap.add_argument("--mode", default="auto", choices=["auto", "direct", "factored"])
    ap.add_argument("--eig-tol", type=float, default=-1.0, help="eigensolver gap tolerance (default 1e-12)")
    ap.add_argument("--value-tol", type=float, default=-1.0,
                    help="Kato-Temple eigenvalue tolerance of eigenvalue-only stats (default: the library's)")
    ap.add_argument("--strict", action="store_true",
                    help="eigenvector-residual stopping rule even for eigenvalue-only stats")
    ap.add_argument("--workload", default="c3", choices=["c3", "c5"],
                    help="c3 (default, the metric's config) or c5: 200 expanding windows x ICp2 sweep at "
                         "T=2000 N=20000, windows sharded over the ranks (strong scaling)")
    ap.add_argument("--rolling", type=int, default=0,
                    help="c5: rolling windows of this many rows instead of expanding windows")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-weak", action="store_true", help="skip the weak-scaling extra field (N > 1)")
    ap.add_argument("--no-all-fields", action="store_true",
                    help="skip the all_fields extra (the job with the whole regression record per replicate: F*, "
                         "L*, OLS formed) — for rocprofv3 runs whose trace must hold the headline launches only")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--dump-rows", default="",
                    help="rank 0 saves the last timed step's gathered per-replicate rows (.npy) here")
    ap.add_argument("--share-device", action="store_true",
                    help="TEST ONLY: every rank on cuda:0 with the gloo backend (a one-GPU box rehearses "
                         "N ranks; RCCL refuses two ranks on one GPU)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']} "
                 f"(launch with --nproc-per-node equal to --gpus)")

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.share_device else int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    backend = None
    # launched by torchrun (any N, N = 1 included): one rank per GPU over RCCL,
    # the per-replicate rows all-gathered on the device; a plain `python
    # bench.py` (the driver's N = 1 run) has no process group
    if "WORLD_SIZE" in os.environ:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if args.share_device:
            backend = "gloo"
            dist.init_process_group("gloo")
        else:
            backend = "nccl"
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    # where the exchanged rows and the max-over-ranks time live: the GPU for
    # RCCL, the host for gloo
    comm_dev = dev if backend == "nccl" else torch.device("cpu")

    import dfm_pkg
    D = dfm_pkg.load()
    ctx = D.Context(local)
    if args.workload == "c5":
        return bench_windows(args, D, ctx, torch, dist, world, rank, dev, comm_dev)
    if args.eig_tol > 0:
        ctx.set_eig_params(tol=args.eig_tol)
    if args.value_tol > 0:
        ctx.set_value_tol(args.value_tol)
    if args.strict:
        ctx.set_value_tol(0.0)
    Bn = args.replicates

    # ---- base model (identical on every rank), resident in HBM
    rng = np.random.default_rng(20261015 + 3)
    y, x, *_ = D.factor_model_DGP(T, N, R, rng=rng)
    x = D.normalize(x, ctx=ctx)
    w = np.ones((T, 1))
    model = D.DynamicFactorModel(y, w, x, R, "ICp2", ctx=ctx)
    if args.batch:
        model.set_batch(args.batch)
    model.set_bootstrap_mode(args.mode)
    stats = [D.Stat.V(), D.Stat.criterion()]
    arr = D.api._stat_array(stats)
    width = int(ctx.lib.dfm_stats_width(model.handle, arr, len(stats)))

    # ---- every step's draws (the same global B x T draws on every rank; a rank
    # uploads its contiguous shard, replicate b on rank floor(b * world / B)),
    # resident in HBM before timing
    from dfm_amd.parallel import shard_range, gather_rows
    b0, b1 = shard_range(Bn, world, rank)
    nloc = b1 - b0
    nsteps = args.warmup + args.steps
    idx_d, eta_d = [], []
    for s in range(nsteps):
        idx, eta = D.draw_wild_fast(1_000_003 + s, Bn, T)
        idx_d.append(torch.from_numpy(np.ascontiguousarray(idx[b0:b1])).to(dev))
        eta_d.append(torch.from_numpy(np.ascontiguousarray(eta[b0:b1])).to(dev))
        del idx, eta
    out = torch.empty((max(nloc, 1), width), dtype=torch.float64, device=dev)
    holder = {}
    torch.cuda.synchronize()

    def step(s):
        if nloc:
            ctx.check(ctx.lib.dfm_bootstrap_dev(model.handle, 0, nloc, idx_d[s].data_ptr(),
                                                eta_d[s].data_ptr(), arr, len(stats), out.data_ptr()))
        holder["rows"] = gather_rows(out[:nloc].to(comm_dev), Bn) if dist is not None else out

    def timed(fn, first, count):
        """Barrier + sync on both sides of `count` steps; max over ranks."""
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(first, first + count):
            fn(s)
        ctx.synchronize()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        el = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([el], dtype=torch.float64, device=comm_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    for s in range(args.warmup):
        step(s)
    torch.cuda.synchronize()
    ctx.synchronize()
    ctx.reset_timing()
    ctx.enable_timing(True)
    el = timed(step, args.warmup, args.steps)
    ctx.enable_timing(False)
    timing = ctx.read_timing()
    eig = ctx.eig_stats()
    weak = None
    if world > 1 and not args.no_weak:
        # weak scaling (extra field): every rank runs a full B-replicate job on
        # its own draws, K steps
        wi, we = [], []
        for s in range(args.steps):
            idx, eta = D.draw_wild_fast(7_000_003 * (rank + 1) + s, Bn, T)
            wi.append(torch.from_numpy(idx).to(dev))
            we.append(torch.from_numpy(eta).to(dev))
        wout = torch.empty((Bn, width), dtype=torch.float64, device=dev)

        def wstep(s):
            ctx.check(ctx.lib.dfm_bootstrap_dev(model.handle, 0, Bn, wi[s].data_ptr(), we[s].data_ptr(), arr,
                                                len(stats), wout.data_ptr()))

        wstep(0)
        wel = timed(wstep, 0, args.steps)
        weak = {"value": round(Bn * args.steps * world / wel, 2), "unit": "replicates/s",
                "ms_per_step": round(wel / args.steps * 1e3, 3), "replicates_per_gpu": Bn,
                "scaling": "weak"}
        del wi, we, wout
    # Extra field: the same job with the fit's whole regression record per
    # replicate (V, ICp2 and every OLS coefficient and HC2 t-statistic,
    # src/DynamicFactorModel.jl:40-48), so the replicate factors F*, loadings
    # L* and the OLS pass run too.  The headline stats (V + ICp2) read only
    # the eigenvalues and the trace, and the library forms only the fields the
    # requested statistics read (include/dfm.h).
    # Timed after the headline region (its own barrier-bracketed steps);
    # `--no-all-fields` leaves it out so a rocprofv3 trace holds only the
    # headline job's launches (its H.Z GEMM average then agrees with the
    # HIP-event roofline of the same run).
    full = None
    if not args.no_all_fields and world == 1 and nloc:
        fstats = stats + [D.Stat.coefficient(j) for j in range(1, R + 2)] + [D.Stat.t_stat(j) for j in range(1, R + 2)]
        farr = D.api._stat_array(fstats)
        fwidth = int(ctx.lib.dfm_stats_width(model.handle, farr, len(fstats)))
        fout = torch.empty((nloc, fwidth), dtype=torch.float64, device=dev)

        def fstep(s):
            ctx.check(ctx.lib.dfm_bootstrap_dev(model.handle, 0, nloc, idx_d[s].data_ptr(), eta_d[s].data_ptr(),
                                                farr, len(fstats), fout.data_ptr()))
        fstep(0)
        fk = min(args.steps, 3)
        fel = timed(fstep, args.warmup, fk)
        full = {"stats": "V + ICp2 + the 9 OLS coefficients + 9 HC2 t-statistics (F*, L* and OLS formed)",
                "value": round(nloc * fk / fel, 2), "unit": "replicates/s", "ms_per_step": round(fel / fk * 1e3, 3),
                "steps": fk}
        del fout
    res = holder["rows"].cpu().numpy()
    ok = bool(np.all(np.isfinite(res))) and res.shape[0] >= Bn if dist is not None else bool(np.all(np.isfinite(res)))
    if args.dump_rows and rank == 0:
        np.save(args.dump_rows, res[:Bn])

    total = Bn * args.steps
    value = total / el
    gram_ms, gram_n = timing.get("gram", (0.0, 0))
    gemm_ms, gemm_n = timing.get("gemm", (0.0, 0))
    roof = None
    if gemm_n:
        # factored path: every product of the eigen-iteration (two per
        # Rayleigh-Ritz step with the degree-2 Chebyshev filter) is one GEMM
        # H (T x T) . Z (T x nb*P).  Algorithmic flop = 2 T^2 P per replicate
        # still unconverged when the GEMM runs (converged replicates' column
        # blocks are skipped), summed by the library over the timed region.
        _, PZ = model.fact_block()   # columns per replicate in the GEMM (the solver's block, even)
        flop_total = 2.0 * T * T * PZ * eig["gemm_products"]
        per_launch_ms = gemm_ms / gemm_n
        achieved = flop_total / (gemm_ms * 1e-3) / 1e12
        roof = {"kernel": "gemmh_zrm_kernel (batched eigen-iteration H.Z: LDS-DMA 3-deep ring, running source "
                          "pointers over the replicate-major chunked Z, 3 workgroups/CU, v_mfma_f64_4x4x4_4b)",
                "bound": "mfma", "achieved": round(achieved, 3), "peak": PEAK_F64_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / PEAK_F64_TFLOPS, 4),
                "traffic": pmc_traffic("gemmh_zrm_kernel"),
                "avg_launch_ms": round(per_launch_ms, 4),
                "flop_per_launch": round(flop_total / gemm_n), "launches": gemm_n,
                "flop_per_replicate_product": 2 * T * T * PZ, "block_columns": PZ}
        rp_ms, rp_src = rocprof_avg_ms("dfm::gemmh_zrm_kernel")
        if rp_ms:   # the same algorithmic flop per launch over rocprof's average duration
            roof["rocprof"] = {"avg_launch_ms": round(rp_ms, 4), "source": f"profiles/{rp_src}",
                               "frac": round(flop_total / gemm_n / (rp_ms * 1e-3) / 1e12 / PEAK_F64_TFLOPS, 4)}
    elif gram_n:
        # direct mode (N > T, no breaks): the replicate Grams come from the
        # factored identity (gram_fact_kernel, 2 T^2 r flop), bound by writing
        # each T x T Gram (8 T^2 bytes per replicate) to HBM
        per_launch_ms = gram_ms / gram_n
        reps_per_launch = nloc * args.steps / gram_n
        gbytes = 8.0 * T * T
        achieved = gbytes * reps_per_launch / (per_launch_ms * 1e-3) / 1e9
        roof = {"kernel": "gram_fact_kernel (replicate Grams by the factored identity, T x T written per replicate)",
                "bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
                "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": None,
                "avg_launch_ms": round(per_launch_ms, 4), "replicates_per_launch": reps_per_launch,
                "bytes_per_replicate": gbytes}
    rec = {
        "metric": "bootstrap replicates/sec (node), T=500 N=2000 r=8; % fp64 MFMA peak",
        "value": round(value, 2), "unit": "replicates/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"C3: wild bootstrap, Bai-Ng DGP T={T} N={N} r={R}, "
                               f"B={Bn} replicates per step sharded over the GPUs, stats V(8)+ICp2",
                   "T": T, "N": N, "r": R, "replicates": Bn, "replicates_per_gpu": nloc,
                   "parallelism": f"replicate-sharded x{world}"},
        "roofline": roof,
        "kernels_ms": {k: round(v[0], 3) for k, v in timing.items() if v[1]},
        "kernel_launches": {k: int(v[1]) for k, v in timing.items() if v[1]},
        "outputs_finite": ok,
        "collective": ((f"RCCL all-gather of the per-replicate rows over {world} rank(s) ({backend})"
                        if backend == "nccl" else
                        f"gloo all-gather of the per-replicate rows over {world} rank(s) sharing cuda:0 (test mode)")
                       if dist is not None else "none (single process, no process group)"),
        "mode": args.mode,
        "stopping_rule": "eigenvector residual (strict)" if args.strict else
                         "eigenvalue Kato-Temple bound, 1e-12 relative (stats are eigenvalue-only)",
        "eig_iterations": eig,
        "eig_filter": ("Chebyshev filters in Horner form: degree 6 on [0, max(theta_p, 0.2 theta_k)] after the "
                       "first Rayleigh-Ritz step of the warm start (middle steps row-local), degree 2 on "
                       "[0, theta_p] after later ones"),
        "roofline_hbm": hbm_rooflines(timing, eig, nloc, args.steps, model.fact_block()[1] or 16),
        "fields_formed": "eigenvalues + trace: V and ICp2 read nothing else, so the replicate factors, loadings "
                         "and OLS are not formed (demand-driven); the all_fields extra is the rate with the whole "
                         "regression record (F*, L*, OLS + HC2) formed per replicate",
    }
    if full:
        rec["all_fields"] = full
    if weak:
        rec["weak_scaling"] = weak
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if dist is not None:
        dist.destroy_process_group()


C5_T, C5_N, C5_P, C5_KMAX = 2000, 20000, 200, 8


def bench_windows(args, D, ctx, torch, dist, world, rank, dev, comm_dev):
    """BASELINE.json configs[4]: the refits of pseudo_out_of_sample_forecasts
    (src/utils.jl:54-72), P = 200 expanding windows x ICp2 sweep k <= 8 on a
    T=2000 N=20000 panel.  The panel is resident in HBM (column-major, as Julia
    holds it); a step = all 200 windows, sharded over the ranks as contiguous
    window blocks (parallel.window_shard: a rank reads only the leading rows its
    windows reach) + one all-gather of the per-window rows.  Strong scaling."""
    from dfm_amd.parallel import window_rows, _pack_windows, gather_rows
    from dfm_amd.api import _window_kmax, _windows_K
    T5, N5, P5, km = C5_T, C5_N, C5_P, C5_KMAX
    L = int(args.rolling) or None
    rng = np.random.default_rng(20261015 + 5)
    y, x, *_ = D.factor_model_DGP(T5, N5, 8, rng=rng)
    x = D.normalize(x, ctx=ctx)
    yd = torch.from_numpy(np.ascontiguousarray(y)).to(dev)
    wd = torch.ones((T5, 1), dtype=torch.float64, device=dev)
    xd = torch.from_numpy(np.ascontiguousarray(x.T)).to(dev).t()     # column-major T x N in HBM
    del x
    w0, w1, a0, rows = window_rows(T5, P5, world, rank, L)
    K = _windows_K(T5, N5, P5, 0, km, L) if L else _window_kmax(T5, N5, km)
    holder = {}

    def step():
        if w1 <= w0:
            res = {}
        elif L:   # rolling: this rank's row slice [a0, rows), a zero-copy column-major view
            res = D.pseudo_out_of_sample_windows(yd[a0:rows], wd[a0:rows], xd[a0:rows], "ICp2",
                                                 num_predictions=w1 - w0, kmax=km, rolling=L, ctx=ctx)
        else:
            res = D.pseudo_out_of_sample_refits_dev(yd, wd, xd, "ICp2", num_predictions=w1 - w0, kmax=km,
                                                    rows=rows, ctx=ctx)
        loc = torch.from_numpy(_pack_windows(res, w1 - w0, K, 1)).to(comm_dev)
        holder["all"] = gather_rows(loc, P5) if dist is not None else loc

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ctx.reset_timing()
    ctx.enable_timing(True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.synchronize()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    ctx.enable_timing(False)
    timing = ctx.read_timing()
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device=comm_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    allrows = holder["all"].cpu().numpy()
    gram_ms, gram_n = timing.get("gram", (0.0, 0))
    roof = None
    if gram_n:   # rank-local prefix Gram of the rows its windows reach: m (m+1) N flop (SYRK count)
        per = gram_ms / gram_n
        m_rows = rows - a0
        ach = m_rows * (m_rows + 1) * N5 / (per * 1e-3) / 1e12
        roof = {"kernel": "gram_dma_kernel (prefix Gram X X' of the leading rows: LDS-DMA ring, v_mfma_f64_4x4x4_4b)",
                "bound": "mfma", "achieved": round(ach, 3), "peak": PEAK_F64_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / PEAK_F64_TFLOPS, 4), "traffic": None, "avg_launch_ms": round(per, 4),
                "flop_per_launch": m_rows * (m_rows + 1) * N5}
    kind = f"rolling ({L} rows)" if L else "expanding"
    rec = {
        "metric": f"{kind}-window refits/sec (node), T=2000 N=20000, 200 windows x ICp2 sweep kmax 8",
        "value": round(P5 * args.steps / el, 2), "unit": "windows/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": f"C5: pseudo_out_of_sample_forecasts refits, {kind} windows, Bai-Ng DGP "
                               f"T=2000 N=20000 r=8, P=200 windows per step (all ranks together), panel "
                               f"resident in HBM",
                   "T": T5, "N": N5, "P": P5, "kmax": km, "rolling": L, "parallelism": f"window-sharded x{world}"},
        "roofline": roof,
        "kernels_ms": {k: round(v[0], 3) for k, v in timing.items() if v[1]},
        "kernel_launches": {k: int(v[1]) for k, v in timing.items() if v[1]},
        "outputs_finite": bool(np.all(np.isfinite(allrows[:, :3]))),
        "r_selected": sorted(set(int(v) for v in allrows[:, 0])),
    }
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
