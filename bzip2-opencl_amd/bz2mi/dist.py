"""Multi-GPU sharding of bz2mi work (one process per GPU, torch.distributed).

The unit of sharding is an independent object: every rank compresses its own
input to a complete .bz2 stream (bzip2 streams concatenate into a valid
multi-stream file), so the data path needs no collective (weak scaling).  The
only exchange is the optional ordered gather of the finished streams to one
rank -- sizes first, then the padded payloads -- which over RCCL/xGMI is one
all_gather of about the compressed size.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def object_seed(base: int, rank: int) -> int:
    """Seed of the synthetic object a rank compresses (bench / tests)."""
    return base + rank


def gather_streams(local: torch.Tensor, dst: int = 0) -> list[torch.Tensor] | None:
    """Ordered gather of variable-length uint8 streams (one per rank).

    `local` is a 1-D uint8 tensor on this rank's device (CUDA with nccl,
    CPU with gloo).  Returns the list of per-rank streams on `dst`, None
    elsewhere."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    n = torch.tensor([local.numel()], dtype=torch.int64, device=local.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    cap = max(sizes) if sizes else 0
    buf = torch.zeros(cap, dtype=torch.uint8, device=local.device)
    buf[: local.numel()] = local
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    if rank != dst:
        return None
    return [p[:s] for p, s in zip(parts, sizes)]


def concat_streams(streams: list[torch.Tensor]) -> bytes:
    """Rank-ordered multi-stream .bz2 file."""
    return b"".join(bytes(s.cpu().numpy().tobytes()) for s in streams)
