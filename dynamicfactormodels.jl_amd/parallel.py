"""Replicate sharding across GPUs (one process per GPU, torch.distributed).

Bootstrap replicates are independent given (idx_b, eta_b) (src/bootstrap.jl:43
is a serial loop with no carried state), so B replicates shard as contiguous
blocks over the ranks with no data-path collective.  The only exchange is the
final all-gather of the per-replicate statistic rows (RCCL over xGMI on GPUs,
gloo in the CPU tests) so that every rank can form quantiles / p-values.
Per-replicate results are bit-identical to a 1-GPU run because every kernel
reduces in a fixed order and the eigensolver's start vectors do not depend on
the replicate's position (tests/test_gpu_parity.py::test_batching_is_bit_identical).
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np


def shard_range(B: int, world: int, rank: int) -> Tuple[int, int]:
    """Replicate b goes to rank floor(b * world / B): contiguous
    blocks whose sizes differ by at most one."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    return (rank * B) // world, ((rank + 1) * B) // world


def gather_rows(local, B: int, group=None, device=None):
    """All-gather each rank's (b1-b0, W) block into the full (B, W) array, in
    replicate order.  `local` is a torch tensor (on the GPU for RCCL)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    width = local.shape[1]
    mx = max(shard_range(B, world, r)[1] - shard_range(B, world, r)[0] for r in range(world))
    pad = torch.zeros((mx, width), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    parts = []
    for r in range(world):
        b0, b1 = shard_range(B, world, r)
        parts.append(bufs[r][: b1 - b0])
    return torch.cat(parts, dim=0)


def sharded_bootstrap(run_local: Callable[[int, int], np.ndarray], B: int, group=None,
                      device=None) -> np.ndarray:
    """Run replicates [b0, b1) of this rank through `run_local(b0, b1)` (which
    returns a (b1-b0, W) array from the engine) and all-gather the rows."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    b0, b1 = shard_range(B, world, rank)
    loc = np.asarray(run_local(b0, b1), dtype=np.float64)
    if loc.ndim == 1:
        loc = loc[:, None]
    t = torch.from_numpy(np.ascontiguousarray(loc))
    if device is not None:
        t = t.to(device)
    return gather_rows(t, B, group).cpu().numpy()


def wild_bootstrap_sharded(dfm, B: int, stat, idx: np.ndarray, eta: np.ndarray, group=None,
                           device=None) -> np.ndarray:
    """`wild_bootstrap` over all ranks: each rank runs its shard on its own
    GPU (its default context), then the rows are all-gathered."""
    from .api import wild_bootstrap

    def run(b0, b1):
        out = wild_bootstrap(dfm, b1 - b0, stat, idx=idx[b0:b1], eta=eta[b0:b1])
        return out if out.ndim == 2 else out[:, None]

    return sharded_bootstrap(run, B, group, device)
