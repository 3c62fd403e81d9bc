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
