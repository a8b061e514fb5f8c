"""Data-parallel sharding of independent 30-s clips across ranks (SURVEY.md §8 e).

One process per GPU; rank r owns clips [r*n, (r+1)*n) (weights replicated, no
collective on the data path). The only exchange is the final gather of every
rank's fixed-size token records to rank 0 — an all-gather over RCCL/xGMI on
the GPU box (backend "nccl"), over gloo in the CPU tests.

Record layout (int32, one row per clip): column 0 = token count, then
RECORD_FIELDS words per token: id, t0, t1 (10-ms ticks) and p (the raw f32
bits) — the fields SttEngine reads from whisper_token_data
(src/stt_engine.cpp:288-296).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

RECORD_FIELDS = 4  # id, t0, t1, p (as raw f32 bits) per token

Record = Tuple[int, int, int, float]


def clip_ids(rank: int, clips_per_rank: int) -> List[int]:
    """Global ids (synthetic-clip seeds) of the clips rank `rank` processes."""
    return list(range(rank * clips_per_rank, (rank + 1) * clips_per_rank))


def pack_records(per_clip: Sequence[Sequence[Record]], max_tokens: int) -> np.ndarray:
    """Fixed-size int32 [clips][1 + RECORD_FIELDS * max_tokens] block so every
    rank gathers an equal-sized tensor. A clip with more than max_tokens
    tokens raises: a truncated gather would silently drop transcript."""
    out = np.zeros((len(per_clip), 1 + RECORD_FIELDS * max_tokens), np.int32)
    for c, recs in enumerate(per_clip):
        recs = list(recs)
        if len(recs) > max_tokens:
            raise ValueError(f"clip {c}: {len(recs)} tokens exceed the record capacity {max_tokens}")
        out[c, 0] = len(recs)
        if recs:
            a = np.array([(i, t0, t1, 0) for i, t0, t1, _ in recs], np.int64).astype(np.int32)
            a[:, 3] = np.array([p for *_, p in recs], np.float32).view(np.int32)
            out[c, 1:1 + RECORD_FIELDS * len(recs)] = a.reshape(-1)
    return out


def unpack_records(block: np.ndarray) -> List[List[Record]]:
    out = []
    for row in np.asarray(block, np.int32):
        n = int(row[0])
        a = row[1:1 + RECORD_FIELDS * n].reshape(n, RECORD_FIELDS)
        p = a[:, 3].copy().view(np.float32)
        out.append([(int(a[j, 0]), int(a[j, 1]), int(a[j, 2]), float(p[j])) for j in range(n)])
    return out


def pack_tokens(per_clip: Sequence[Sequence[int]], max_tokens: int) -> np.ndarray:
    """Token ids only (t0 = t1 = -1, p = 0): pack_records of bare ids."""
    return pack_records([[(int(i), -1, -1, 0.0) for i in ids] for ids in per_clip], max_tokens)


def unpack_tokens(block: np.ndarray) -> List[List[int]]:
    return [[r[0] for r in recs] for recs in unpack_records(block)]


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
