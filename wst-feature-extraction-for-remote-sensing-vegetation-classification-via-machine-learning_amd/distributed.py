"""Patch sharding across the GPUs of one node.

The reference extracts features serially, one image and one channel at a time
(src/training/train_and_save_model.py:486-488).  Patches are independent, so here each rank (one process per
GPU, launched by ``torch.distributed.run``) transforms a contiguous range of patches with its own replicated
plan.  The data path has no collective.  The only exchange is an optional all-gather that reassembles the
per-patch outputs.  Over RCCL/xGMI (backend "nccl") the buffers are device tensors; with "gloo" the same code
runs on host tensors, which is how the CPU tests exercise the N>1 path.
"""
from __future__ import annotations

from typing import Callable, Optional


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [start, stop) of ``n`` items for ``rank``; shard sizes differ by at most one and
    the lower ranks take the remainder."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    if n < 0:
        raise ValueError("n < 0")
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def gather_shards(local, n_total: int, group=None):
    """All-gather per-rank shards (first dim = this rank's patches, ranges from ``shard_range``)
    into the full ``(n_total, ...)`` tensor on every rank.  Shards are padded to the largest shard
    so a single ``all_gather_into_tensor`` (one RCCL call, per-link bound on xGMI) moves them."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    cap = shard_range(n_total, 0, world)[1]            # rank 0 holds the largest shard
    pad = torch.zeros((cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    full = torch.empty((world * cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "gloo":
        parts = list(full.chunk(world))
        dist.all_gather(parts, pad, group=group)
    else:
        dist.all_gather_into_tensor(full, pad, group=group)
    keep = []
    for r in range(world):
        a, b = shard_range(n_total, r, world)
        keep.append(full[r * cap: r * cap + (b - a)])
    return torch.cat(keep, 0)


def extract_sharded(images, J: int = 2, L: int = 8, max_order: int = 2, pooled: bool = True,
                    gather: bool = True, group=None,
                    compute: Optional[Callable] = None):
    """Transform ``images`` (N, C, H, W), each rank handling its ``shard_range``.

    Returns the gathered (N, C, 2K) pooled features [or (N, C, K, Mo, No)] on every rank when
    ``gather``, else this rank's shard.  ``compute(x_shard) -> tensor`` defaults to the HIP path
    on this rank's current device; it is injectable so the sharding/gather logic is testable on
    CPU ranks."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    n = images.shape[0]
    a, b = shard_range(n, rank, world)
    shard = images[a:b]
    if compute is None:
        from .frontend import scatter_device

        def compute(xs):
            dev = torch.device("cuda", torch.cuda.current_device())
            x = torch.as_tensor(xs, dtype=torch.float32).to(dev).contiguous()
            C, H, W = x.shape[1:]
            y = scatter_device(x.reshape(-1, H, W), H, W, J, L, max_order, False, pooled=pooled)
            return y.reshape((x.shape[0], C) + tuple(y.shape[1:]))
    local = compute(shard)
    if not gather or world == 1:
        return local
    return gather_shards(local, n, group)
