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
    return (rank * B + world - 1) // world, ((rank + 1) * B + world - 1) // world


def _comm_device(group, device):
    """Where the exchanged rows must live: RCCL ("nccl") moves device tensors
    only, so with that backend and no explicit device the rows go to this
    rank's GPU (LOCAL_RANK); gloo takes host tensors."""
    import os
    import torch
    import torch.distributed as dist
    if device is not None:
        return device
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    return None


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
    device = _comm_device(group, device)
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


# ---------------------------------------------------------------- windows
# Expanding windows (pseudo_out_of_sample_forecasts, src/utils.jl:54-72) are
# independent given the panel: window w refits on rows 0..T-P+w-1 only.  A
# contiguous shard [w0, w1) of the P windows is therefore exactly the
# (T - P + w1, w1 - w0) windows problem on the panel's leading T - P + w1 rows
# (a zero-copy view: same pointer, same leading dimension).  With N > T every
# window's Gram is a leading block of the one prefix Gram, so
# a rank forms only the Gram of the rows its windows reach.

WINDOW_FIELDS = ("number_of_factors", "V", "criterion_value", "eigenvalues", "coefficients", "t_stats")


def window_shard(T: int, P: int, world: int, rank: int) -> Tuple[int, int, int]:
    """(w0, w1, rows): this rank's windows [w0, w1) and the leading rows of the
    panel they read (window w reads rows < T - P + w)."""
    w0, w1 = shard_range(P, world, rank)
    return w0, w1, T - P + w1


def window_rows(T: int, P: int, world: int, rank: int, rolling: Optional[int] = None) -> Tuple[int, int, int, int]:
    """(w0, w1, a, b): this rank's windows [w0, w1) and the panel rows [a, b)
    they read.  Expanding windows read from row 0 (a = 0); rolling windows of
    L rows (window w = rows T-P+w-L .. T-P+w-1) read only [T-P+w0-L, T-P+w1),
    so a rank runs the (b - a, w1 - w0) rolling problem on that row slice (a
    zero-copy view of a column-major panel: pointer + a, same leading
    dimension) — its own diagonal block of the prefix Gram, no exchange."""
    w0, w1 = shard_range(P, world, rank)
    b = T - P + w1
    a = T - P + w0 - int(rolling) if rolling else 0
    return w0, w1, a, b


def _pack_windows(res: dict, n: int, K: int, q: int) -> np.ndarray:
    """One (n, 3 + K + 2 (q + K)) float64 row block per shard; columns past the
    shard's own sweep bound are NaN."""
    out = np.full((n, 3 + K + 2 * (q + K)), np.nan)
    if n == 0:
        return out
    out[:, 0] = res["number_of_factors"]
    out[:, 1] = res["V"]
    out[:, 2] = res["criterion_value"]
    ev = res["eigenvalues"]
    out[:, 3:3 + ev.shape[1]] = ev
    c0 = 3 + K
    for f in ("coefficients", "t_stats"):
        a = res[f]
        out[:, c0:c0 + a.shape[1]] = a
        c0 += q + K
    return out


def _unpack_windows(rows: np.ndarray, T: int, P: int, K: int, q: int) -> dict:
    c0 = 3 + K
    return {"window_rows": np.arange(T - P, T), "number_of_factors": rows[:, 0].astype(np.int64),
            "V": rows[:, 1].copy(), "criterion_value": rows[:, 2].copy(),
            "eigenvalues": rows[:, 3:3 + K].copy(), "coefficients": rows[:, c0:c0 + q + K].copy(),
            "t_stats": rows[:, c0 + q + K:c0 + 2 * (q + K)].copy()}


def windows_sharded(run_local: Callable[[int, int], dict], T: int, N: int, q: int, P: int,
                    kmax: Optional[int] = None, group=None, device=None) -> dict:
    """All P windows over all ranks: this rank runs its shard through
    ``run_local(rows, n)`` (the windows problem on the leading ``rows`` rows with
    ``n`` windows; returns ``pseudo_out_of_sample_refits``' dict), then one
    all-gather of the packed per-window rows.  The eigenvalue / coefficient
    columns keep the unsharded width K = min(kmax, ceil(min(T-1, N)/2)); with
    kmax unset a shard whose widest window sweeps fewer than K factors fills
    the rest with NaN (its windows' own sweep bounds are unchanged)."""
    import torch
    import torch.distributed as dist
    from .api import _window_kmax
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    K = _window_kmax(T, N, kmax)
    w0, w1, rows = window_shard(T, P, world, rank)
    res = run_local(rows, w1 - w0) if w1 > w0 else {}
    loc = torch.from_numpy(_pack_windows(res, w1 - w0, K, q))
    device = _comm_device(group, device)
    if device is not None:
        loc = loc.to(device)
    return _unpack_windows(gather_rows(loc, P, group).cpu().numpy(), T, P, K, q)
