"""World-size-2 gloo test of the data-parallel path (SURVEY.md §8 e): clip
sharding is disjoint and complete, and the token gather delivers every rank's
records to rank 0 in rank order (the same shard.gather_to_rank0 bench.py runs
over RCCL on the GPU box)."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sentiric-stt-whisper-service_amd"))

import shard  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_tokens(clip_id, n):
    rng = np.random.default_rng(clip_id)
    return list(rng.integers(0, 51864, size=int(rng.integers(0, n + 1))))


def _worker(rank, world, port, clips, max_tok, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids = shard.clip_ids(rank, clips)
    block = shard.pack_tokens([_fake_tokens(c, max_tok) for c in ids], max_tok)
    g = shard.gather_to_rank0(dist, block)
    q.put((rank, ids, None if g is None else g.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_clip_sharding_disjoint_and_complete():
    world, n = 8, 32
    all_ids = [c for r in range(world) for c in shard.clip_ids(r, n)]
    assert sorted(all_ids) == list(range(world * n))


def test_pack_unpack_roundtrip():
    toks = [[1, 2, 3], [], list(range(300))]
    b = shard.pack_tokens(toks, 220)
    assert b.shape == (3, 221)
    assert shard.unpack_tokens(b) == [[1, 2, 3], [], list(range(220))]


@pytest.mark.timeout(120)
def test_gloo_world2_gather_to_rank0():
    import torch.multiprocessing as mp
    world, clips, max_tok = 2, 5, 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, clips, max_tok, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (ids, g)) for r, ids, g in (q.get(timeout=100) for _ in range(world)))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert res[1][1] is None
    got = shard.unpack_tokens(np.array(res[0][1], np.int32))
    want = [_fake_tokens(c, max_tok) for r in range(world) for c in shard.clip_ids(r, clips)]
    assert got == want
