"""Multi-device paths through the C ABI, on one MI355X: several contexts on
device 0 stand in for several GPUs ("on a one-GPU box, emulate with
several contexts on one device").

* dfm_model_clone + dfm_bootstrap_multi: the replicate loop of
  src/bootstrap.jl:43 sharded over contexts (replicate b on context
  floor(b n / B)) must give rows bit-identical to one context.
* the torch.distributed path (parallel.wild_bootstrap_sharded): two processes,
  each with its own context on the GPU and the real engine, rows exchanged by
  a gloo all-gather, bit-identical to one process.
* normalize (src/utils.jl:33) on the device vs the oracle."""
import os
import socket

import numpy as np
import pytest

from test_gpu_parity import panel, rel

pytestmark = pytest.mark.gpu


def contexts(dfm, n):
    return [dfm.Context(0) for _ in range(n)]


@pytest.mark.parametrize("T,N,r,mode", [(200, 400, 4, "factored"), (96, 150, 3, "factored"), (150, 60, 3, "auto"),
                                        (120, 300, 3, "direct")])
@pytest.mark.parametrize("n", [2, 3])
def test_bootstrap_multi_is_bit_identical(dfm, oracle, T, N, r, mode, n):
    y, x, w = panel(oracle, T, N, r, 400 + T + n)
    g = dfm.DynamicFactorModel(y, w, x, r, "ICp2")
    g.set_bootstrap_mode(mode)
    copies = [g] + [dfm.clone_model(g, c) for c in contexts(dfm, n - 1)]
    for c in copies[1:]:
        c.set_bootstrap_mode(mode)
        assert c.V == g.V and np.array_equal(c.coefficients, g.coefficients)
    B = 23
    idx, eta = dfm.draw_wild_fast(31, B, T)
    S = dfm.Stat
    stats = [S.V(), S.criterion(), S.eigenvalue(r), S.t_stat(1), S.LR_all(T // 2)]
    one = dfm.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
    many = dfm.wild_bootstrap(copies, B, stats, idx=idx, eta=eta)
    assert np.array_equal(one, many)
    ridx = oracle.draw_residual(np.random.default_rng(2), B, T)
    assert np.array_equal(dfm.residual_bootstrap(g, B, S.V(), idx=ridx),
                          dfm.residual_bootstrap(copies, B, S.V(), idx=ridx))


@pytest.mark.parametrize("T,N,r,mode,B", [(200, 400, 4, "factored", 700), (96, 150, 3, "direct", 600),
                                          (150, 60, 3, "auto", 520), (80, 160, 2, "auto", 6000)])
def test_two_lanes_are_bit_identical(dfm, oracle, T, N, r, mode, B):
    """Jobs of 512..6000 replicates in automatic batching run as two lanes
    (the halves of the replicate range on two streams / host threads,
    dfm_bootstrap_dev); an explicit batch size keeps one lane.  Rows equal to
    the bit, with the Chow statistics, coefficients and iteration counts."""
    y, x, w = panel(oracle, T, N, r, 700 + T)
    g = dfm.DynamicFactorModel(y, w, x, r, "ICp2")
    g.set_bootstrap_mode(mode)
    idx, eta = dfm.draw_wild_fast(77, B, T)
    S = dfm.Stat
    stats = [S.V(), S.criterion(), S.eigenvalue(1), S.coefficient(1), S.t_stat(2), S.LR_all(T // 2),
             S.LM(T // 2, 1), S.iterations()]
    lanes = dfm.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
    g.set_batch(B)
    one = dfm.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
    assert np.array_equal(lanes, one)
    ridx = oracle.draw_residual(np.random.default_rng(3), B, T)
    one_r = dfm.residual_bootstrap(g, B, S.V(), idx=ridx)
    g.set_batch(0)
    assert np.array_equal(dfm.residual_bootstrap(g, B, S.V(), idx=ridx), one_r)


@pytest.mark.parametrize("mode", ["direct", "factored"])
def test_clone_is_complete_before_its_first_bootstrap(dfm, oracle, mode):
    """Root cause of round 4's intermittent two-lane wrong rows:
    ``dfm_model_clone`` copied the fit with ``hipMemcpyPeer`` — on the legacy
    null stream, returning before a device-to-device copy lands — while the
    copy's context stream is non-blocking, so the clone's first kernels
    (H = E E', EL = E L, F S F', the warm start) could read a partly copied
    E, L or U.  A large panel (three 96 MB panel copies ahead of L and U)
    turns that window from microseconds into ~0.1 ms: without the fix the
    clone's rows — and the second lane's, whose clone is made by the first
    two-lane call — differ from the original's on every run."""
    T, N, r = 200, 60000, 3
    rng = np.random.default_rng(61)
    y, x, *_ = oracle.factor_model_DGP(T, N, r, rng)
    x, w = oracle.normalize(x), np.ones((T, 1))
    S = dfm.Stat
    stats = [S.V(), S.criterion(), S.eigenvalue(1), S.coefficient(1), S.t_stat(2), S.LM(T // 2, 1),
             S.iterations()]
    g = dfm.DynamicFactorModel(y, w, x, r, "ICp2")
    g.set_bootstrap_mode(mode)
    c = dfm.clone_model(g, dfm.Context(0))      # and at once a bootstrap on the copy
    c.set_bootstrap_mode(mode)
    idx, eta = dfm.draw_wild_fast(3, 8, T)
    got = dfm.wild_bootstrap(c, 8, stats, idx=idx, eta=eta)
    assert np.array_equal(got, dfm.wild_bootstrap(g, 8, stats, idx=idx, eta=eta))
    # the two-lane job on a fresh fit: its first call makes the lane's clone
    h = dfm.DynamicFactorModel(y, w, x, r, "ICp2")
    h.set_bootstrap_mode(mode)
    B = 600
    idx, eta = dfm.draw_wild_fast(4, B, T)
    lanes = dfm.wild_bootstrap(h, B, stats, idx=idx, eta=eta)
    h.set_batch(B)
    one = dfm.wild_bootstrap(h, B, stats, idx=idx, eta=eta)
    bad = np.where(~np.all(lanes == one, axis=1))[0]
    assert len(bad) == 0, f"{len(bad)} two-lane rows differ from one lane (first {bad[:5]}, last {bad[-1:]})"


def test_clone_ignores_the_legacy_null_stream(dfm, oracle):
    """The same hazard made deterministic: the legacy null stream (PyTorch's
    default stream) is held busy with ~0.1 s of fp64 GEMMs when the fit is
    cloned.  Round 4's clone queued its copies behind that work (hipMemcpyPeer)
    and returned at once, and the copy's bootstrap — on the context's
    non-blocking stream — read buffers not yet copied.  The clone now copies
    on its own context's stream and waits for those copies only."""
    import torch
    T, N, r = 200, 4000, 3
    rng = np.random.default_rng(62)
    y, x, *_ = oracle.factor_model_DGP(T, N, r, rng)
    x, w = oracle.normalize(x), np.ones((T, 1))
    S = dfm.Stat
    stats = [S.V(), S.criterion(), S.eigenvalue(1), S.coefficient(1), S.t_stat(2), S.iterations()]
    g = dfm.DynamicFactorModel(y, w, x, r, "ICp2")
    idx, eta = dfm.draw_wild_fast(5, 8, T)
    ref = dfm.wild_bootstrap(g, 8, stats, idx=idx, eta=eta)
    a = torch.full((6144, 6144), 1e-4, device="cuda", dtype=torch.float64)
    torch.cuda.synchronize()
    assert torch.cuda.current_stream().cuda_stream == 0      # the legacy null stream
    for _ in range(6):
        a = a @ a
    c = dfm.clone_model(g, dfm.Context(0))
    got = dfm.wild_bootstrap(c, 8, stats, idx=idx, eta=eta)
    torch.cuda.synchronize()
    bad = np.where(~np.all(got == ref, axis=1))[0]
    assert len(bad) == 0, f"clone rows differ: {bad}"


def test_bootstrap_multi_break_model(dfm, oracle):
    y, x, w = panel(oracle, 120, 200, 2, 91, model="Breitung_Eickmeier_2011", b=0.5)
    g = dfm.DynamicFactorModel(y, w, x, 2, "ICp2", break_indices=[61])
    c = dfm.clone_model(g, dfm.Context(0))
    assert len(c.factors) == 2 and np.array_equal(c.loadings[1], g.loadings[1])
    idx, eta = dfm.draw_wild_fast(5, 9, 120)
    S = dfm.Stat
    stats = [S.V(), S.criterion(), S.LM_all(60)]
    assert np.array_equal(dfm.wild_bootstrap(g, 9, stats, idx=idx, eta=eta),
                          dfm.wild_bootstrap([g, c], 9, stats, idx=idx, eta=eta))


def test_bootstrap_multi_errors(dfm, oracle):
    y, x, w = panel(oracle, 80, 120, 2, 7)
    g = dfm.DynamicFactorModel(y, w, x, 2, "ICp2")
    idx, eta = dfm.draw_wild_fast(1, 4, 80)
    with pytest.raises(dfm.DFMError):     # the same context twice: one host thread per context
        dfm.wild_bootstrap([g, g], 4, dfm.Stat.V(), idx=idx, eta=eta)
    h = dfm.DynamicFactorModel(y, w, x, 3, "ICp2", ctx=dfm.Context(0))
    with pytest.raises(dfm.DFMError):     # not a copy of the same fit
        dfm.wild_bootstrap([g, h], 4, dfm.Stat.V(), idx=idx, eta=eta)
    bad = idx.copy()
    bad[3, 5] = 80
    c = dfm.clone_model(g, dfm.Context(0))
    with pytest.raises(dfm.DFMError):     # out-of-range index inside the second shard
        dfm.wild_bootstrap([g, c], 4, dfm.Stat.V(), idx=bad, eta=eta)


def test_stat_indices_are_one_based(dfm, oracle):
    with pytest.raises(ValueError):
        dfm.Stat.eigenvalue(0)
    with pytest.raises(ValueError):
        dfm.Stat.t_stat(0)
    y, x, w = panel(oracle, 80, 120, 2, 8)
    g = dfm.DynamicFactorModel(y, w, x, 2, "ICp2")
    idx, eta = dfm.draw_wild_fast(1, 2, 80)
    import dfm_amd.api as A
    for bad in (A.Stat(2, -1), A.Stat(3, -1), A.Stat(4, 3), A.Stat(2, 2)):   # raw 0-based: out of range
        with pytest.raises(dfm.DFMError):
            dfm.wild_bootstrap(g, 2, bad, idx=idx, eta=eta)


@pytest.mark.parametrize("T,N", [(200, 100), (37, 1001), (500, 2000)])
def test_normalize_matches_oracle(dfm, oracle, T, N):
    x = np.random.default_rng(T).standard_normal((T, N)) * np.linspace(0.5, 4.0, N) + np.linspace(-3, 3, N)
    got = dfm.normalize(x)
    ref = oracle.normalize(x)
    assert np.max(np.abs(got - ref)) < 1e-13 * np.max(np.abs(ref))


def test_normalize_dev_in_place(dfm, oracle):
    import torch
    x = np.random.default_rng(3).standard_normal((300, 700)) * 3.0 + 1.0
    xd = torch.from_numpy(np.ascontiguousarray(x.T)).cuda().t()       # column-major in HBM
    dfm.normalize_dev(xd, xd)
    torch.cuda.synchronize()
    dfm.default_context().synchronize()
    assert np.max(np.abs(xd.cpu().numpy() - oracle.normalize(x))) < 1e-13 * 10


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _engine_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch.distributed as dist
    import dfm_pkg
    import dfm_oracle as O
    D = dfm_pkg.load()
    from dfm_amd.parallel import wild_bootstrap_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    y, x, *_ = O.factor_model_DGP(150, 300, 3, np.random.default_rng(44))
    x, w = O.normalize(x), np.ones((150, 1))
    g = D.DynamicFactorModel(y, w, x, 3, "ICp2", ctx=D.Context(0))
    idx, eta = D.draw_wild_fast(12, 17, 150)
    stats = [D.Stat.V(), D.Stat.criterion(), D.Stat.Wald_all(75)]
    got = wild_bootstrap_sharded(g, 17, stats, idx, eta)
    q.put((rank, got))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_real_engine(dfm, oracle):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_engine_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    y, x, *_ = oracle.factor_model_DGP(150, 300, 3, np.random.default_rng(44))
    x, w = oracle.normalize(x), np.ones((150, 1))
    g = dfm.DynamicFactorModel(y, w, x, 3, "ICp2")
    idx, eta = dfm.draw_wild_fast(12, 17, 150)
    ref = dfm.wild_bootstrap(g, 17, [dfm.Stat.V(), dfm.Stat.criterion(), dfm.Stat.Wald_all(75)], idx=idx, eta=eta)
    for r in (0, 1):
        assert np.array_equal(res[r], ref)


def test_rccl_world1_device_gather(dfm, oracle):
    """The nccl (= RCCL) branch of parallel._comm_device / gather_rows with
    device tensors, at world size 1 on cuda:0 (an 8-GPU node is the driver's;
    this runs the same code path on the one-GPU box): the rows of
    wild_bootstrap_sharded through RCCL equal the unsharded rows
    (src/bootstrap.jl:43's loop, replicate b on rank floor(b world / B))."""
    import torch
    import torch.distributed as dist
    from dfm_amd.parallel import _comm_device, gather_rows, wild_bootstrap_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        assert _comm_device(None, None) == torch.device("cuda", 0)
        loc = torch.arange(15, dtype=torch.float64, device="cuda").reshape(5, 3)
        got = gather_rows(loc, 5)
        assert got.is_cuda and torch.equal(got, loc)
        y, x, w = panel(oracle, 150, 300, 3, 45)
        g = dfm.DynamicFactorModel(y, w, x, 3, "ICp2")
        idx, eta = dfm.draw_wild_fast(13, 17, 150)
        stats = [dfm.Stat.V(), dfm.Stat.criterion(), dfm.Stat.Wald_all(75)]
        rows = wild_bootstrap_sharded(g, 17, stats, idx, eta)
        assert np.array_equal(rows, dfm.wild_bootstrap(g, 17, stats, idx=idx, eta=eta))
    finally:
        dist.destroy_process_group()


def test_bench_under_torchrun_world1():
    """bench.py under torchrun at --nproc-per-node 1 takes the RCCL path (the
    process group, the device all-gather of the rows, barriers and the
    max-over-ranks time) — the code the driver's N = 2..8 runs execute."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "1", "--steps", "1", "--warmup", "1", "--replicates", "600", "--no-cpu-baseline",
           "--no-all-fields"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=root)
    assert p.returncode == 0, p.stderr[-2000:]
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["n_gpus"] == 1 and rec["outputs_finite"] and rec["value"] > 0
    assert rec["collective"].startswith("RCCL all-gather") and "nccl" in rec["collective"]



def _bench(root, tmp_path, gpus, tag, extra=()):
    import json
    import subprocess
    import sys
    dump = str(tmp_path / f"rows_{tag}.npy")
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", str(gpus), "--steps", "1", "--warmup", "1",
           "--no-cpu-baseline", "--no-all-fields", "--no-weak", "--dump-rows", dump] + list(extra)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=root, env=env)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    return rec, np.load(dump)


@pytest.mark.timeout(600)
def test_bench_gpus2_launches_two_ranks(tmp_path):
    """`python3 bench.py --gpus 2` — the driver's command form — starts two
    ranks itself (a torch.distributed.run child; the parent never touches the
    GPU).  On the one-GPU box both ranks share cuda:0 over gloo
    (`--share-device`, test only: RCCL refuses two ranks on one GPU).  The
    C3 job's 9999 replicates split 5000 / 4999 (replicate b on rank
    floor(2 b / B), src/bootstrap.jl:43) and the gathered rows are
    bit-identical to the one-process run's."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    one, rows1 = _bench(root, tmp_path, 1, "n1")
    two, rows2 = _bench(root, tmp_path, 2, "n2", ["--share-device"])
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["config"]["replicates_per_gpu"] == 5000 and two["config"]["replicates"] == 9999
    assert "over 2 rank(s)" in two["collective"] and two["outputs_finite"]
    assert rows1.shape == rows2.shape == (9999, rows1.shape[1])
    assert np.array_equal(rows1, rows2)


def test_two_contexts_on_one_external_stream(dfm, oracle):
    """two contexts bound to the same external stream
    (dfm_ctx_set_stream) draw their stream-ordered scratch from the device's
    default pool, not from whichever context registered last — so one of
    them can be destroyed while the other keeps running jobs on the stream.
    Every row equals a private context's row (src/bootstrap.jl:41-51)."""
    import torch
    y, x, w = panel(oracle, 200, 400, 4, 611)
    idx, eta = dfm.draw_wild_fast(612, 40, 200)
    stats = [dfm.Stat.V(), dfm.Stat.criterion(), dfm.Stat.t_stat(2)]
    ref = dfm.wild_bootstrap(dfm.DynamicFactorModel(y, w, x, 4, "ICp2", ctx=dfm.Context(0)), 40, stats, idx=idx, eta=eta)
    s = torch.cuda.Stream()
    a, b = dfm.Context(0), dfm.Context(0)
    a.set_stream(s.cuda_stream)
    b.set_stream(s.cuda_stream)
    ga = dfm.DynamicFactorModel(y, w, x, 4, "ICp2", ctx=a)
    gb = dfm.DynamicFactorModel(y, w, x, 4, "ICp2", ctx=b)
    assert np.array_equal(dfm.wild_bootstrap(ga, 40, stats, idx=idx, eta=eta), ref)
    assert np.array_equal(dfm.wild_bootstrap(gb, 40, stats, idx=idx, eta=eta), ref)
    del ga
    a.close()
    for _ in range(3):
        assert np.array_equal(dfm.wild_bootstrap(gb, 40, stats, idx=idx, eta=eta), ref)
    torch.cuda.synchronize()
