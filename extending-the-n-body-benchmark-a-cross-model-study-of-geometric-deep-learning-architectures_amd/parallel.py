"""Data-parallel sharding of independent N-body systems.

Systems never interact, so a batch of B systems splits into contiguous blocks,
one per rank (one process per GPU), with no collective on the data path; the
only exchange is one all-gather of the per-rank results (final states or whole
trajectories) over RCCL/xGMI.  The same code runs on ``gloo`` for CPU tests.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

__all__ = ["init_from_env", "shard_range", "all_gather_shards", "max_over_ranks", "barrier", "world", "rank",
           "allreduce_gradients"]


def world(group=None) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def init_from_env(backend=None):
    """One process per GPU under torch.distributed.run: reads RANK / WORLD_SIZE /
    LOCAL_RANK, binds the local device, initialises the process group (``nccl`` =
    RCCL on ROCm when a GPU is present, else ``gloo``).  Returns
    ``(rank, world, device)``."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rk = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (several ranks on one GPU): NBX_LOCAL_DEVICE pins every rank to one device,
    # NBX_DIST_BACKEND overrides the backend (gloo: RCCL refuses two ranks on one device)
    if os.environ.get("NBX_LOCAL_DEVICE") is not None:
        local = int(os.environ["NBX_LOCAL_DEVICE"])
    backend = backend or os.environ.get("NBX_DIST_BACKEND") or None
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if ws > 1 and not dist.is_initialized():
        dist.init_process_group(backend or ("nccl" if device.type == "cuda" else "gloo"))
    return rk, ws, device


def shard_range(total: int, rank: int, world: int):
    """Contiguous block of ``total`` systems owned by ``rank``: (start, count); the
    first ``total % world`` ranks take one extra system."""
    base, extra = divmod(total, world)
    count = base + (1 if rank < extra else 0)
    start = rank * base + min(rank, extra)
    return start, count


def all_gather_shards(local: torch.Tensor, total: int | None = None) -> torch.Tensor:
    """Concatenate every rank's ``local`` [count_r, ...] along dim 0 in rank order
    (uneven counts allowed: shards are padded to the largest for the collective)."""
    ws = world()
    if ws == 1:
        return local
    counts = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    all_counts = [torch.zeros_like(counts) for _ in range(ws)]
    dist.all_gather(all_counts, counts)
    all_counts = [int(c.item()) for c in all_counts]
    mx = max(all_counts)
    pad = local
    if local.shape[0] < mx:
        pad = torch.cat([local, local.new_zeros((mx - local.shape[0],) + tuple(local.shape[1:]))], 0)
    bufs = [torch.empty_like(pad) for _ in range(ws)]
    dist.all_gather(bufs, pad.contiguous())
    out = torch.cat([b[:c] for b, c in zip(bufs, all_counts)], 0)
    if total is not None and out.shape[0] != total:
        raise RuntimeError(f"gathered {out.shape[0]} systems, expected {total}")
    return out


def max_over_ranks(x: float, device=None) -> float:
    if world() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier():
    if world() > 1:
        dist.barrier()


def allreduce_gradients(params, group=None, bucket_bytes: int = 64 << 20) -> None:
    """Data-parallel training (one process per GPU, each on its own batch): average every
    parameter gradient over the ranks in place.  Gradients are flattened into buckets of at most
    ``bucket_bytes`` (one all-reduce per bucket; the EGNN-MC C1 model's 3.5 MB is one bucket), so
    the ring collective runs on few large messages (xGMI links are point-to-point: per-message
    latency, not bandwidth, bounds small all-reduces).  No-op on one rank.  The reference trains
    on one device (trainer.py:233-358); this is the multi-GPU form of its optimizer step."""
    if world() == 1:
        return
    n = world(group) if group is not None else world()
    # buckets hold one gradient dtype each (the reference trains in float64 by default,
    # config.yaml precision_mode: double) and are sized by that dtype's element size
    by_dtype = {}
    for q in params:
        if q.grad is not None:
            by_dtype.setdefault((q.grad.dtype, q.grad.device), []).append(q)
    for plist in by_dtype.values():
        esz = plist[0].grad.element_size()
        i = 0
        while i < len(plist):
            bucket, size = [], 0
            while i < len(plist) and (not bucket or size + plist[i].grad.numel() * esz <= bucket_bytes):
                bucket.append(plist[i])
                size += plist[i].grad.numel() * esz
                i += 1
            flat = torch.cat([q.grad.reshape(-1) for q in bucket])
            dist.all_reduce(flat, group=group)
            flat /= n
            o = 0
            for q in bucket:
                q.grad.copy_(flat[o:o + q.numel()].view_as(q.grad))
                o += q.numel()
