"""World-size-2 gloo test of the data-parallel path (SURVEY.md §8 e): clip
sharding is disjoint and complete, and the token gather delivers every rank's
records to rank 0 in rank order (the same shard.gather_to_rank0 bench.py runs
over RCCL on the GPU box)."""
import json
import os
import socket
import subprocess
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
    toks = [[1, 2, 3], [], list(range(220))]
    b = shard.pack_tokens(toks, 220)
    assert b.shape == (3, 1 + shard.RECORD_FIELDS * 220)
    assert shard.unpack_tokens(b) == toks
    recs = [[(50365, 0, 12, 0.5), (7, 12, 40, 0.123456789)], []]
    got = shard.unpack_records(shard.pack_records(recs, 4))
    assert got[1] == [] and [r[:3] for r in got[0]] == [r[:3] for r in recs[0]]
    assert [r[3] for r in got[0]] == [float(np.float32(r[3])) for r in recs[0]]
    with pytest.raises(ValueError):  # truncation fails loudly
        shard.pack_records([[(1, 0, 0, 0.0)] * 5], 4)


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


def _oracle_records(model_path, clip_id):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import mwx
    import orc
    o = orc.Oracle(model_path, threads=2)
    opt = orc.FullOptions.service_defaults()
    opt.temperature_inc = 0.0
    opt.language = "en"
    pcm = mwx.pcm16_to_f32(mwx.synth_pcm16(clip_id, 8 * 16000))
    _, segs, _, _ = o.full(pcm, opt)
    o.close()
    return [(t.id, t.t0, t.t1, t.p) for sg in segs for t in sg.tokens]


def _oracle_worker(rank, world, port, clips, max_tok, model_path, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    block = shard.pack_records([_oracle_records(model_path, c) for c in shard.clip_ids(rank, clips)],
                               max_tok)
    g = shard.gather_to_rank0(dist, block)
    q.put((rank, None if g is None else g.tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_gathers_transcription_records(make_model):
    """Each rank transcribes its own clips (the CPU oracle standing in for the
    engine: no GPU here) and gathers full token records (id, t0, t1, p) to
    rank 0, which receives every clip's records in rank order, bit for bit."""
    import torch.multiprocessing as mp
    path = make_model("micro-rich")
    world, clips, max_tok = 2, 2, 448
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_oracle_worker, args=(r, world, port, clips, max_tok, path, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=280) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert res[1] is None
    got = shard.unpack_records(np.array(res[0], np.int32))
    want = [_oracle_records(path, c) for r in range(world) for c in shard.clip_ids(r, clips)]
    assert got == [[(i, a, b, float(np.float32(p))) for i, a, b, p in w] for w in want]
    assert all(len(w) > 0 for w in want)


@pytest.mark.timeout(300)
def test_bench_gpus2_launches_two_ranks():
    """`bench.py --gpus 2` without torch.distributed.run starts two rank
    processes itself (RANK / WORLD_SIZE / MASTER_* set before any GPU call in
    the parent); here, with no GPU, over gloo and with synthetic records."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                        "--clips", "3", "--decode-steps", "20"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    line = lines[0]
    assert line["n_gpus"] == 2 and line["gathered_clips"] == 6 and line["gather_rank_order_ok"]


@pytest.mark.gpu
def test_two_engine_ranks_gather_equals_single(tmp_path):
    """The data-parallel path with real engine ranks:
    `bench.py --gpus 2` starts two rank processes, each transcribing its own
    shard of clips with the engine, and gathers every rank's token records
    to rank 0. On the one-GPU box both ranks share GPU 0 and the gather runs
    over gloo (MWX_BENCH_ONE_DEVICE=1; RCCL needs a GPU per rank). Rank 0's
    gathered block holds rank 0's clips then rank 1's, and every clip's
    records (id, t0, t1, p) equal that clip decoded alone."""
    out = tmp_path / "gathered.npy"
    env = dict(os.environ, MWX_BENCH_ONE_DEVICE="1", TMPDIR=str(tmp_path))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--arch", "micro",
           "--wtype", "f16", "--clips", "3", "--steps", "1", "--warmup", "0", "--lanes", "1",
           "--decode-steps", "24", "--no-cpu-baseline", "--no-one-lane", "--dump-gather", str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["gathered"]["complete"], line["gathered"]
    got = shard.unpack_records(np.load(out))
    assert len(got) == 6
    import mwx
    path = str(tmp_path / "mwx_bench_micro_f16.bin")  # the model file the run wrote
    with mwx.Context.open(path) as ctx:
        p = ctx.default_params(mwx.SAMPLING_GREEDY)  # (bench.py main(), same fields)
        p.language = b"en"
        p.temperature = 0.0
        p.temperature_inc = 0.0
        p.token_timestamps = True
        p.suppress_nst = True
        p.bench_fixed_steps = 24
        for c in range(6):  # global clip id c = rank * 3 + i (shard.clip_ids)
            pcm = mwx.pcm16_to_f32(mwx.synth_pcm16(c, 30 * 16000))
            assert ctx.full(pcm, p, state_index=c) == 0
            assert ctx.token_records(c) == got[c], c
    print(f"two engine ranks: {sum(len(g) for g in got)} tokens of 6 clips gathered to rank 0, "
          f"each clip equal to its single-engine run")
