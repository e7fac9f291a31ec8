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


class ShardGather:
    """All-gather of per-rank shards into preallocated buffers (SURVEY.md §8(e) exchange step).

    ``local`` holds this rank's shard (rows = its patches, ``shard_range`` order), padded to the
    largest shard, so compute writes straight into it and one ``all_gather_into_tensor`` (one RCCL
    call; ``all_gather`` of chunks under gloo) moves every shard with no staging copy.  ``gather``
    returns the ``(n_total, ...)`` result: a view of the receive buffer when the shards are equal
    (n_total % world == 0, e.g. BASELINE c3's 10^6 patches over 1/2/4/8 GPUs), else a compacted
    copy.  ``to_root`` gathers to rank ``root`` only (the others receive nothing).  Buffers are
    allocated once, outside any timed region."""

    def __init__(self, n_total: int, row_shape, dtype, device, group=None, root_only: bool = False):
        import torch
        import torch.distributed as dist

        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.n_total = n_total
        self.lo, self.hi = shard_range(n_total, self.rank, self.world)
        self.cap = shard_range(n_total, 0, self.world)[1]     # rank 0 holds the largest shard
        self.root_only = root_only
        row_shape = tuple(row_shape)
        self.local = torch.zeros((self.cap,) + row_shape, dtype=dtype, device=device)
        self.full = None
        if self.world > 1 and (not root_only or self.rank == 0):
            self.full = torch.empty((self.world * self.cap,) + row_shape, dtype=dtype, device=device)
        self.equal = n_total % self.world == 0

    @property
    def mine(self) -> int:
        return self.hi - self.lo

    def bytes_moved(self) -> int:
        """Payload bytes of one gather (all shards, padding included)."""
        return 0 if self.world == 1 else self.world * self.local.numel() * self.local.element_size()

    def gather(self):
        import torch
        import torch.distributed as dist

        if self.world == 1:
            return self.local[: self.mine]
        gloo = dist.get_backend(self.group) == "gloo"
        if self.root_only:
            parts = list(self.full.chunk(self.world)) if self.rank == 0 else None
            dist.gather(self.local, parts, dst=0, group=self.group)
            if self.rank != 0:
                return None
        elif gloo:
            dist.all_gather(list(self.full.chunk(self.world)), self.local, group=self.group)
        else:
            dist.all_gather_into_tensor(self.full, self.local, group=self.group)
        if self.equal:
            return self.full
        keep = []
        for r in range(self.world):
            a, b = shard_range(self.n_total, r, self.world)
            keep.append(self.full[r * self.cap: r * self.cap + (b - a)])
        return torch.cat(keep, 0)


def run_sharded_job(sg: "ShardGather", batch: int, generate: Callable, compute: Callable, gather: bool = True):
    """One pass of a patch-sharded job (BASELINE c3; bench.py --config c3 runs exactly this): this
    rank's patches [lo, hi) in batches of ``batch``, ``generate(first_global_index, n)`` makes them
    (keyed by global index, so no rank needs another's inputs), ``compute(x, n, out_rows)`` writes
    their outputs into this rank's rows of ``sg.local``; then the all-gather (when ``gather``)."""
    for b0 in range(0, sg.mine, batch):
        nb = min(batch, sg.mine - b0)
        x = generate(sg.lo + b0, nb)
        compute(x, nb, sg.local[b0: b0 + nb])
    return sg.gather() if gather else sg.local[: sg.mine]


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
