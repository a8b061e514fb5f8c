"""Data-parallel sharding of independent 30-s clips across ranks (SURVEY.md §8 e).

One process per GPU; rank r owns clips [r*n, (r+1)*n) (weights replicated, no
collective on the data path). The only exchange is the final gather of every
rank's fixed-size token records to rank 0 — an all-gather over RCCL/xGMI on
the GPU box (backend "nccl"), over gloo in the CPU tests.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np

RECORD_FIELDS = 4  # id, t0, t1, p (as raw f32 bits) per token


def clip_ids(rank: int, clips_per_rank: int) -> List[int]:
    """Global ids (synthetic-clip seeds) of the clips rank `rank` processes."""
    return list(range(rank * clips_per_rank, (rank + 1) * clips_per_rank))


def pack_tokens(per_clip: Sequence[Sequence[int]], max_tokens: int) -> np.ndarray:
    """Fixed-size int32 [clips][max_tokens + 1] block: column 0 = token count,
    then the ids (zero padded), so ranks gather equal-sized tensors."""
    out = np.zeros((len(per_clip), max_tokens + 1), np.int32)
    for c, ids in enumerate(per_clip):
        ids = list(ids)[:max_tokens]
        out[c, 0] = len(ids)
        out[c, 1:1 + len(ids)] = ids
    return out


def unpack_tokens(block: np.ndarray) -> List[List[int]]:
    return [list(map(int, row[1:1 + int(row[0])])) for row in block]


def gather_to_rank0(dist, block: np.ndarray, device: Optional[str] = None) -> Optional[np.ndarray]:
    """All-gather each rank's [clips][W] int32 block; rank 0 returns the
    [world*clips][W] concatenation in rank order, other ranks None. `dist` is
    torch.distributed (initialised) or None for a single process."""
    import torch
    t = torch.from_numpy(np.ascontiguousarray(block))
    if device:
        t = t.to(device)
    if dist is None:
        return t.cpu().numpy()
    world, rank = dist.get_world_size(), dist.get_rank()
    out = torch.empty((world * block.shape[0], block.shape[1]), dtype=t.dtype, device=t.device)
    if dist.get_backend() == "gloo":
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        out = torch.cat(parts, 0)
    else:
        dist.all_gather_into_tensor(out, t)
    return out.cpu().numpy() if rank == 0 else None
