"""Multi-process (world_size 2, gloo, CPU) checks of the replicate-sharding
path: shard boundaries and the ordered all-gather of per-replicate rows."""
import os
import socket

import numpy as np
import pytest


def test_shard_range_partitions(dfm):
    from dfm_amd.parallel import shard_range
    for B in (1, 7, 9999, 10000):
        for world in (1, 2, 3, 8):
            covered = []
            for r in range(world):
                b0, b1 = shard_range(B, world, r)
                assert 0 <= b0 <= b1 <= B
                covered.extend(range(b0, b1))
            assert covered == list(range(B))
            sizes = [shard_range(B, world, r)[1] - shard_range(B, world, r)[0] for r in range(world)]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch.distributed as dist
    import dfm_pkg
    D = dfm_pkg.load()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dfm_amd.parallel import sharded_bootstrap

    # stand-in for the per-replicate engine call: a deterministic function of
    # the GLOBAL replicate index, so misordering or dropped rows are detected
    def run_local(b0, b1):
        b = np.arange(b0, b1, dtype=np.float64)
        return np.stack([b, b * b + 0.5, np.sin(b)], axis=1)

    full = sharded_bootstrap(run_local, B)
    q.put((rank, full))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("B", [9, 10])
def test_gloo_world2_gather_order(dfm, B):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, B, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    b = np.arange(B, dtype=np.float64)
    ref = np.stack([b, b * b + 0.5, np.sin(b)], axis=1)
    for r in (0, 1):
        assert np.array_equal(res[r], ref)


def test_window_shard_ranges(dfm):
    from dfm_amd.parallel import window_shard
    for T, P in ((2000, 200), (30, 7), (50, 3)):
        for world in (1, 2, 3, 8):
            got = []
            for r in range(world):
                w0, w1, rows = window_shard(T, P, world, r)
                assert rows == T - P + w1 and rows <= T
                got.extend(range(w0, w1))
            assert got == list(range(P))


def _oracle_windows(O, y, w, x, P, kmax):
    """pseudo_out_of_sample_refits' dict from the oracle's serial refit loop
    (src/utils.jl:54-72) on the given rows."""
    T, N = x.shape
    from dfm_amd.api import _window_kmax
    K = _window_kmax(T, N, kmax)
    fits = O.expanding_window_refits(y, w, x, P, lambda yy, ww, xx: O.DynamicFactorModel_ic(
        yy, ww, xx, "ICp2", kmax=kmax))
    out = {"number_of_factors": np.array([o.number_of_factors for o in fits], dtype=np.int64),
           "V": np.array([O.factor_residual_variance(o) for o in fits]),
           "criterion_value": np.array([o.number_of_factors_criterion_value for o in fits]),
           "eigenvalues": np.full((P, K), np.nan), "coefficients": np.full((P, 1 + K), np.nan),
           "t_stats": np.full((P, 1 + K), np.nan)}
    for j, o in enumerate(fits):
        ev = o.eigenvalues[0][:K]
        out["eigenvalues"][j, :ev.size] = ev
        out["coefficients"][j, :o.coefficients.size] = o.coefficients
        out["t_stats"][j, :o.t_stats.size] = o.t_stats
    return out


def _window_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch.distributed as dist
    import dfm_pkg
    import dfm_oracle as O
    dfm_pkg.load()
    from dfm_amd.parallel import windows_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    T, N, P, kmax = 40, 90, 5, 4
    rng = np.random.default_rng(5)
    y, x, *_ = O.factor_model_DGP(T, N, 2, rng)
    x, w = O.normalize(x), np.ones((T, 1))
    # stand-in for the per-rank GPU call: the oracle on the shard's leading rows
    got = windows_sharded(lambda rows, n: _oracle_windows(O, y[:rows], w[:rows], x[:rows], n, kmax),
                          T, N, 1, P, kmax)
    q.put((rank, got, _oracle_windows(O, y, w, x, P, kmax) if rank == 0 else None))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_windows_sharded(dfm):
    """Windows sharded over 2 ranks by leading-row truncation and gathered in
    window order equal the unsharded serial refit loop exactly."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_window_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, got, ref = q.get(timeout=180)
        res[r] = (got, ref)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = res[0][1]
    for r in (0, 1):
        got = res[r][0]
        for f in ("number_of_factors", "V", "criterion_value", "eigenvalues", "coefficients", "t_stats"):
            assert np.array_equal(got[f], ref[f], equal_nan=True), f


def test_rolling_window_rows_cover_each_window():
    """Rolling windows (L rows before each forecast date) shard by row slices:
    rank's slice [a, b) holds exactly the rows its windows read, and window
    w0 + j of the full problem is window j of the (b - a, w1 - w0) problem."""
    from dfm_amd.parallel import window_rows
    T, P, L = 2000, 200, 700
    for world in (1, 2, 3, 8):
        seen = []
        for rank in range(world):
            w0, w1, a, b = window_rows(T, P, world, rank, L)
            Tl, Pl = b - a, w1 - w0
            for j in range(Pl):
                g_lo, g_hi = T - P + w0 + j - L, T - P + w0 + j          # full problem's window rows
                l_lo, l_hi = Tl - Pl + j - L, Tl - Pl + j                 # the slice problem's
                assert (a + l_lo, a + l_hi) == (g_lo, g_hi)
                assert 0 <= l_lo and l_hi <= Tl
                seen.append(w0 + j)
        assert seen == list(range(P))
    assert window_rows(T, P, 4, 1, None)[2] == 0                          # expanding: from row 0


def test_bench_gpus_must_match_world_size():
    """Under torchrun, bench.py --gpus N with WORLD_SIZE != N fails loudly
    before importing torch (no silent one-GPU line for an N-GPU request)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4"], capture_output=True,
                       text=True, timeout=60, cwd=root, env=env)
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr


def test_bench_launcher_propagates_rank_failure():
    """`python bench.py --gpus 2` without torchrun launches two ranks in a
    child torch.distributed.run; here (no GPU) the ranks fail, and the
    launcher must exit non-zero instead of printing a line."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--no-cpu-baseline"], capture_output=True, text=True, timeout=180,
                       cwd=root, env=env)
    assert p.returncode != 0
    assert "launching 2 ranks" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
