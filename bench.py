#!/usr/bin/env python3
"""bench.py — throughput of the MI355X Whisper hot path (BASELINE.json metric).

One step = one mwx_full_batch pass over a batch of synthetic 30-s clips per GPU
(device log-mel -> conv stem -> 32-layer encoder -> cross K/V -> KV-cached greedy
decode with on-device logits processing -> segments) followed by the RCCL gather
of every rank's token streams to rank 0. Workload (configs[2] of BASELINE.json):
Whisper-large-v3 shapes, bf16 weights (synthetic, seeded), 32 clips x 30 s per
GPU, decode length fixed at the upstream cap of 220 steps per clip (EOT and
timestamps suppressed via bench_fixed_steps so every clip costs the same).

Lanes (default 2 = the reference's parallel_requests default, src/config.h:41):
two batches are in flight per GPU, each driven by its own host thread on its
own states and HIP stream, as the SttEngine's batchers run them; a lane takes
the next of the K timed batches when its previous one is done. Every batch is still 32 clips; one lane's
encoder / host work overlaps the other's decode. --lanes 1 times one batch at
a time (the PCIe-inclusive --host-input legs always do).

Multi-GPU: launched with torch.distributed.run, one process per GPU; clips are
sharded (weak scaling, 32 per GPU); RCCL is used only for the final token-stream
gather. value = audio seconds processed by all ranks / max-over-ranks time.

Also reported: a roofline object for the dominant kernel (HIP events recorded
by the engine on its own stream during the timed region) and a CPU baseline
(the oracle — a CPU restatement of the reference path — timed on a bounded
sample on this host).
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sentiric-stt-whisper-service_amd"))

METRIC = "audio-sec/s/GPU + RTF, Whisper-large-v3 30s chunks at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
MFMA_PEAK_TFLOPS = 2500.0  # dense bf16/f16 MFMA (spec)

ARCH = {  # n_mels, d, heads, enc layers, dec layers, vocab
    "large-v3": (128, 1280, 20, 32, 32, 51866),
    "medium": (80, 1024, 16, 24, 24, 51865),
    "base": (80, 512, 8, 6, 6, 51865),
    "tiny.en": (80, 384, 6, 4, 4, 51864),
    "micro": (80, 128, 2, 2, 3, 51864),
}


def kernel_model(arch, kclass, clips, rows, launches, prompt_len, steps, windows=1, kv8=False):
    """Algorithmic work of one launch of `kclass`, averaged over the launches of
    one step: (bound, per-launch bytes or flops, description). kv8: the cross
    K/V cache is MX-fp8 (--fp8: one e4m3 byte per element + one E8M0 scale
    byte per 32)."""
    n_mels, d, H, Le, Ld, V = ARCH[arch]
    L, T = 1500, 3000
    if kclass == "dec_attn_cross":
        # every clip's cross K and V for one layer is read once per launch
        # (greedy: one row per clip; beam / best-of: the clip's decoders share
        # it), plus q in / o out per row
        per = (1 + 1 / 32) if kv8 else 2
        b = clips * L * d * 2 * per + rows * d * 2 * 2
        kind = "MX-fp8 (e4m3 + E8M0 per 32)" if kv8 else "f16"
        return "hbm", b, f"{clips:g} clips x K+V 1500x{d} {kind} + {rows:g} rows x q/o per launch"
    if kclass == "dec_attn_self":
        # every row reads its history K and V (f16, 64 per head) for one
        # layer: positions 1..(prompt_len + steps - 1) averaged over the steps,
        # plus the QKV slab reads and the o write
        n_avg = (prompt_len + (prompt_len + steps - 1)) / 2.0
        b = rows * (n_avg * d * 2 * 2 + 3 * d * 4 * 2 + d * 2)
        return "hbm", b, f"{rows:g} rows x mean {n_avg:.0f} positions x K+V {d} f16 per launch"
    if kclass == "enc_gemm":
        conv = 2 * T * d * 3 * n_mels + 2 * L * d * 3 * d
        layer = 2 * L * d * (3 * d + d + 4 * d + 4 * d)
        flops = clips * windows * (conv + Le * layer)  # every 30-s window is encoded
        return "mfma", flops / max(1, launches), "conv1/conv2/QKV/out/FC1/FC2 FLOPs per launch"
    if kclass == "cross_gemm":
        return "mfma", 2 * clips * L * d * 2 * d * Ld, "all-layer cross K/V GEMM"
    if kclass == "enc_attn":
        return "mfma", clips * H * 4 * L * L * 64, "QK^T + PV FLOPs per layer launch"
    if kclass == "dec_gemm":
        # six weight GEMMs per layer and decode step
        w = 2 * (3 * d * d + d * d + d * d + d * d + 8 * d * d)
        return "hbm", w / 6, "decoder weight bytes per launch (mean of the 6 GEMMs of a layer)"
    if kclass == "logits_gemm":
        return "hbm", V * d * 2 + rows * V * 4, "tied embedding bf16 + f32 logits"
    raise ValueError(kclass)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def oracle_stt_transcribe(o, pcm16, steps):
    """SttEngine::transcribe_pcm16 restated on the CPU oracle: int16 / 32768
    (src/stt_engine.cpp:117-125), whisper_full with the service's parameters
    (:204-243; greedy, language en, decode length fixed like the GPU leg) and
    the post-filters of :258-311 (oracle/service_filters.py). Returns the kept
    segments."""
    import mwx
    import orc
    import service_filters as sf
    opt = orc.FullOptions.service_defaults()
    opt.language = "en"
    opt.temperature_inc = 0.0
    opt.bench_fixed_steps = steps
    _, segs, _, _ = o.full(mwx.pcm16_to_f32(pcm16), opt)
    return sf.postprocess([(s.raw, s.t0, s.t1, [(t.id, t.p, t.t0, t.t1) for t in s.tokens])
                           for s in segs], o.eot, o.token_bytes)


CPU_DEC_STEPS = 8  # (cpu_large_sample: a bounded decode sample when asked for; both bench legs decode the whole window)


def cpu_large_sample(model_path, arch, threads, prompt_len, steps, dec_steps=None):
    """The oracle (scalar C++ + OpenMP) on ONE clip of the benched model:
    full log-mel, conv stem + ALL encoder layers, the all-layer cross K/V and
    the prompt + dec_steps decode positions (KV-cached, on the clip's own
    cross K/V) measured; dec_steps None = every decode step of the window
    (nothing extrapolated), else the remaining steps are extrapolated at the
    measured mean time per step."""
    import mwx
    import orc
    o = orc.Oracle(model_path, threads=threads)
    pcm = mwx.pcm16_to_f32(mwx.synth_pcm16(0))
    t0 = time.perf_counter()
    mel, _ = o.mel(pcm)
    t_mel = time.perf_counter() - t0
    t0 = time.perf_counter()
    enc = o.encode(mel)
    t_enc = time.perf_counter() - t0
    t0 = time.perf_counter()
    k, v = o.cross(enc)
    t_cross = time.perf_counter() - t0
    n_meas = prompt_len + (steps if dec_steps is None else min(dec_steps, steps))
    toks = [o.sot] + [300 + i for i in range(n_meas - 1)]
    t0 = time.perf_counter()
    o.decode_seq(k, v, toks)
    t_dec_meas = time.perf_counter() - t0
    t_step = t_dec_meas / n_meas
    n_total = prompt_len + steps
    t_clip = t_mel + t_enc + t_cross + t_dec_meas + (n_total - n_meas) * t_step
    o.close()
    measured = t_mel + t_enc + t_cross + t_dec_meas
    return 30.0 / t_clip, measured, t_clip, n_meas, n_total


def granted_cpus():
    """CPUs this job may use: the affinity mask, capped by OMP_NUM_THREADS when
    the host sets it (the GPU box grants 16 CPUs per GPU and exports
    OMP_NUM_THREADS=16 while os.cpu_count() reports the whole machine)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    return min(aff, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else aff, aff


def cpu_baseline(model_path, arch, threads, prompt_len, steps):
    """Reported CPU baseline (BASELINE.md "CPU-baseline plan"): the CPU
    restatement of the reference path (oracle/, whisper.cpp v1.8.2 semantics)
    on this host, at the reference's n_threads = 4 (src/config.h:40) and at
    all granted cores. value: the benched model (bounded sample, see
    cpu_large_sample); c1: config C1 (tiny.en greedy, one 30-s clip) measured
    end to end through the SttEngine steps (oracle_stt_transcribe)."""
    import mwx
    import orc
    granted, aff = granted_cpus()
    out = {"unit": "audio-sec/s", "kind": "port", "cpu_model": cpu_model(),
           "host_cpus": os.cpu_count(), "affinity_cpus": aff, "granted_cpus": granted,
           "label": "CPU restatement of the reference path (whisper.cpp v1.8.2 semantics)"}
    legs = {}
    for th in sorted({4, threads}):
        # both legs -- all granted cores (reported) and the reference's
        # n_threads = 4 default (src/config.h:40) -- decode the whole window
        # (the 4-thread leg takes about a minute)
        v, measured, t_clip, n_meas, n_total = cpu_large_sample(
            model_path, arch, th, prompt_len, steps, None)
        if n_meas == n_total:
            what = (f"{n_total} of {n_total} decode positions: the whole window measured, "
                    f"{t_clip:.1f} s/clip")
        else:
            what = (f"{n_meas} of {n_total} decode positions measured ({measured:.1f} s); the "
                    f"other {n_total - n_meas} decode steps extrapolated at the measured mean: "
                    f"{t_clip:.1f} s/clip")
        legs[th] = {"value": round(v, 4), "cores": th,
                    "sample": (f"1 clip of 30 s, {arch}: log-mel + conv + all {ARCH[arch][3]} "
                               f"encoder layers + all-layer cross K/V + {what}")}
    out.update(legs[threads])
    out["threads4"] = legs[4]
    tiny = os.path.join(os.environ.get("TMPDIR", "/tmp"), "mwx_bench_tiny.en_f16.bin")
    if not os.path.exists(tiny):
        tmp = tiny + f".tmp{os.getpid()}"
        mwx.write_synthetic_model(tmp, "tiny.en", mwx.GGML_F16, 0)
        os.replace(tmp, tiny)
    c1 = {}
    for th in sorted({4, threads}):
        o = orc.Oracle(tiny, threads=th)
        t0 = time.perf_counter()
        res = oracle_stt_transcribe(o, mwx.synth_pcm16(0), steps)
        el = time.perf_counter() - t0
        o.close()
        c1[f"threads{th}"] = {"value": round(30.0 / el, 3), "seconds": round(el, 3),
                              "segments": len(res)}
    out["c1_tiny_en"] = dict(c1, config="C1: tiny.en greedy, one 30-s 16 kHz clip, "
                                        f"{steps} decode steps, end to end (mel, encoder, "
                                        "decode, post-filters), measured")
    return out


def prosody_segments(n_samp, seed):
    """Whisper-like segmentation of one clip: consecutive 1-8 s segments."""
    rng = np.random.default_rng(seed)
    starts, lens, s = [], [], 0
    while s < n_samp:
        n = min(int(rng.integers(16000, 8 * 16000)), n_samp - s)
        starts.append(s)
        lens.append(n)
        s += n
    return starts, lens


def prosody_bench(args):
    """Segment prosody (k_prosody.hip through mwx_prosody_batch_device) over
    the segments of --clips clips per GPU (default 256 x 30 s), PCM and
    segment table resident in HBM; one launch per step, one workgroup per
    segment. CPU baseline: the reference's own extract_prosody
    (oracle/_ref) on a bounded sample of the same segments."""
    import ctypes
    import torch
    import mwx
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = init_dist(world, local)
    import shard
    clips = args.clips if args.clips != 32 else 256
    n_samp = int(args.clip_seconds * 16000)
    ids = shard.clip_ids(rank, clips)
    pcm = np.concatenate([mwx.pcm16_to_f32(mwx.synth_pcm16(k, n_samp)) for k in ids])
    desc, frames = [], 0
    for c, k in enumerate(ids):
        st, ln = prosody_segments(n_samp, k)
        for s0, n in zip(st, ln):
            desc.append((c * n_samp + s0, n, frames))
            frames += n // 160 if n >= 160 else 0
    desc = np.array(desc, np.int64)
    n_seg = len(desc)
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "mwx_bench_prosody_micro.bin")
    if local == 0 and not os.path.exists(path):
        tmp = path + f".tmp{os.getpid()}"
        mwx.write_synthetic_model(tmp, "micro", mwx.GGML_F16, 0)
        os.replace(tmp, path)
    if dist is not None:
        dist.barrier()
    ctx = mwx.Context.open(path, device=local)
    L = mwx.lib()
    d_pcm = torch.from_numpy(pcm).to(f"cuda:{local}")
    d_desc = torch.from_numpy(desc.reshape(-1)).to(f"cuda:{local}")
    d_out = torch.empty(n_seg * ctypes.sizeof(mwx.Prosody), dtype=torch.uint8, device=f"cuda:{local}")
    prm = L.mwx_prosody_default_params()
    st0 = ctx.state(0)

    def step():
        rc = L.mwx_prosody_batch_device(ctx.ctx, st0, d_pcm.data_ptr(), d_desc.data_ptr(), n_seg,
                                        frames, 16000, ctypes.byref(prm), d_out.data_ptr())
        if rc != 0:
            raise RuntimeError(f"mwx_prosody_batch_device rc={rc}")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()  # the state's stream: mwx_perf_read below syncs it too
    L.mwx_perf_read(st0, None, None)
    L.mwx_perf_enable(st0, b"prosody")
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    tot_ms, nl = ctypes.c_double(), ctypes.c_int()
    L.mwx_perf_read(st0, ctypes.byref(tot_ms), ctypes.byref(nl))  # synchronizes the stream
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    L.mwx_perf_enable(st0, None)
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    audio_s = world * clips * args.clip_seconds * args.steps
    if rank == 0:
        avg_s = tot_ms.value / 1e3 / max(1, nl.value)
        work = 4 * int(desc[:, 1].sum())  # algorithmic: every sample read once
        achieved = work / avg_s / 1e9
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = prosody_cpu_baseline(pcm, desc)
        line = {
            "metric": "segment_prosody_audio_seconds_per_second",
            "value": round(audio_s / elapsed, 1),
            "unit": "audio-sec/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded 16 kHz PCM16 clips resident in HBM)",
            "config": {"workload": f"extract_prosody over {n_seg} segments (1-8 s) of {clips} x "
                                   f"{args.clip_seconds:g} s clips per GPU, one launch per step",
                       "global_batch": world * n_seg, "seq_len": n_samp,
                       "parallelism": f"dp{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None, "kernel": "prosody",
                         "avg_launch_us": round(avg_s * 1e6, 2), "launches": nl.value,
                         "work_per_launch": work,
                         "work_desc": "4 B per PCM sample of every segment (read once)"},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def is_headline_config(args):
    """The full default C3 run (BASELINE.json configs[1]) - the one the driver's bench line is."""
    return (not args.no_service_leg and not args.no_cpu_baseline and not args.service_defaults
            and args.arch == "large-v3"
            and args.beam <= 1 and not args.fp8 and not args.rich and args.decode_steps == 220
            and args.clip_seconds == 30.0 and not args.host_input)


def service_leg():
    """What DEFAULT requests of the service cost, reported beside the headline (VERDICT r05
    weak 9): batches of 32 x 30-s clips at --service-defaults (language auto, beam 5, the
    temperature ladder, token timestamps, '-rich' weights decoded to the model's stop), two
    lanes as the headline (the service's parallel_requests = 2, src/config.h:41): one batch per
    lane timed after one warm-up batch per lane. Run as a child process once this process has
    released its context; its failure is reported, never fatal to the headline."""
    cmd = [sys.executable, "-u", os.path.abspath(__file__), "--service-defaults", "--lanes", "2",
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-one-lane"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
        rec = None
        for ln in r.stdout.splitlines():
            if ln.startswith("{"):
                rec = json.loads(ln)
        if r.returncode != 0 or rec is None:
            return {"error": f"exit {r.returncode}: {r.stderr[-400:]}"}
    except Exception as ex:
        return {"error": str(ex)}
    return {"value": rec["value"], "unit": rec["unit"], "ms_per_step": rec["ms_per_step"],
            "steps": rec["steps"], "warmup": rec["warmup"], "lanes": 2,
            "workload": rec["config"]["workload"], "decode_work": rec.get("decode_work"),
            "cmd": "python bench.py --service-defaults --lanes 2 --steps 2 --warmup 1"}


def prosody_cpu_baseline(pcm, desc, budget_s=10.0):
    """The reference's extract_prosody (oracle/_ref, compiled from its own
    sources) — or, where that was not built, the oracle restatement — on one
    core over the first segments until ~budget_s of CPU time."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    kind, fn = "port", None
    ref = os.path.join(ROOT, "oracle", "_ref", "libref_prosody.so")
    if os.path.exists(ref):
        import make_prosody_golden as mpg
        L = mpg.load_ref()
        kind = "reference"
        fn = lambda x: mpg.ref_prosody(L, x, 16000, (0.07, 170.0, 60.0, 500.0))  # noqa: E731
    else:
        import orc
        fn = lambda x: orc.prosody(x)  # noqa: E731
    done_s, t0, i = 0.0, time.perf_counter(), 0
    while time.perf_counter() - t0 < budget_s and i < len(desc):
        s0, n = int(desc[i, 0]), int(desc[i, 1])
        fn(pcm[s0:s0 + n])
        done_s += n / 16000.0
        i += 1
    el = time.perf_counter() - t0
    return {"value": round(done_s / el, 1), "unit": "audio-sec/s", "cores": 1, "kind": kind,
            "sample": f"first {i} segments ({done_s:.0f} s of audio), one thread"}


def gather_summary(block, clips, per_clip):
    """Rank 0's view of the last step's record gather: clips received and
    whether every clip carries its full fixed-length token record (per_clip
    None: decoding until the model stops, every clip has some tokens)."""
    import shard
    if block is None:
        return None
    import zlib
    recs = shard.unpack_records(block)
    full = (lambda r: len(r) == per_clip) if per_clip else (lambda r: len(r) > 0)
    # crc32 of the records (id, t0, t1, p bits): equal across runs and boxes
    # for the same build and workload (the decode is deterministic)
    crc = zlib.crc32(repr(recs).encode())
    return {"clips": len(recs), "tokens": sum(len(r) for r in recs),
            "complete": len(recs) == clips and all(full(r) for r in recs),
            "records_crc32": f"{crc:08x}"}


def launch_ranks(n):
    """`bench.py --gpus N` outside torch.distributed.run: start N fresh rank
    processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one GPU each)
    before this process touches the GPU, wait for all of them and return the
    first failing exit status (0 if all succeeded). Rank 0 prints the line."""
    import signal
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in live:  # a failed rank leaves its peers blocked in a collective
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return rc


def one_device():
    """MWX_BENCH_ONE_DEVICE=1: every rank on GPU 0 and the record gather over
    gloo (RCCL needs one GPU per rank) -- the N-rank path exercised on a
    1-GPU box (tests/test_multi_rank.py); never for a timed line."""
    return os.environ.get("MWX_BENCH_ONE_DEVICE") == "1"


def init_dist(world, local):
    """torch.distributed over RCCL (backend "nccl") when the rank has a GPU,
    gloo otherwise (the CPU tests of the launcher / gather path, and
    MWX_BENCH_ONE_DEVICE)."""
    if world <= 1:
        return None
    import torch
    import torch.distributed as dist
    if torch.cuda.is_available() and not one_device():
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    else:
        dist.init_process_group("gloo")
    return dist


def dry_run(args, world, rank, local):
    """--dry-run: the launcher, process group and rank-ordered record gather
    of the real run with the transcription replaced by deterministic
    synthetic records (no engine, no GPU needed); rank 0 checks that the
    gathered records are every rank's, in rank order."""
    import shard
    dist = init_dist(world, local)
    dev = "cuda" if dist is not None and dist.get_backend() == "nccl" else None

    def recs(c):
        rng = np.random.default_rng(1000 + c)
        n = int(rng.integers(1, args.decode_steps + 1))
        return [(int(rng.integers(0, 51866)), 2 * j, 2 * j + 2, float(rng.random())) for j in range(n)]

    ids = shard.clip_ids(rank, args.clips)
    block = shard.pack_records([recs(c) for c in ids], args.decode_steps)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    g = shard.gather_to_rank0(dist, block, device=dev)
    elapsed = time.perf_counter() - t0
    if rank == 0:
        got = shard.unpack_records(g)
        want = [recs(c) for r in range(world) for c in shard.clip_ids(r, args.clips)]
        ok = len(got) == len(want) and all(
            [(a, b, c) for a, b, c, _ in x] == [(a, b, c) for a, b, c, _ in y] and
            np.allclose([p for *_, p in x], [p for *_, p in y], rtol=0, atol=1e-7)
            for x, y in zip(got, want))
        print(json.dumps({"metric": METRIC, "dry_run": True, "n_gpus": world,
                          "backend": dist.get_backend() if dist is not None else None,
                          "gathered_clips": len(got), "gather_rank_order_ok": bool(ok),
                          "gather_ms": round(elapsed * 1e3, 3)}), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


def stream_bench(args):
    """Streaming re-transcription latency: one live stream
    through the service path (SttEngine + StreamSession over libmwx_stt.so,
    the reference's gRPC loop without the transport) fed 0.5-s chunks of a
    synthetic 16 kHz PCM16 stream; every chunk triggers a re-transcription of
    the whole growing buffer (up to the 30-s cap), as the reference does.
    Reports the wall time of each partial (chunk in -> events out).
    MWX_NO_MEL_CACHE=1 disables the incremental log-mel for an A/B."""
    import ctypes as C
    import mwx
    local = int(os.environ.get("LOCAL_RANK", "0"))
    wt = mwx.GGML_BF16 if args.wtype == "bf16" else mwx.GGML_F16
    d = os.environ.get("TMPDIR", "/tmp")
    march = args.arch + ("-rich" if args.rich else "")
    name = f"mwx_bench_{march}_{args.wtype}.bin"
    path = os.path.join(d, name)
    if not os.path.exists(path):
        tmp = path + f".tmp{os.getpid()}"
        mwx.write_synthetic_model(tmp, march, wt, 0)
        os.replace(tmp, path)
    L = C.CDLL(os.path.join(ROOT, "sentiric-stt-whisper-service_amd", "libmwx_stt.so"))
    L.mwx_stt_new_ex.restype = C.c_void_p
    L.mwx_stt_new_ex.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_char_p,
                                 C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    L.mwx_stt_stream_new.restype = C.c_void_p
    L.mwx_stt_stream_new.argtypes = [C.c_void_p]
    L.mwx_stt_stream_free.argtypes = [C.c_void_p]
    L.mwx_stt_stream_feed.restype = C.c_int
    L.mwx_stt_stream_feed.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_char_p, C.c_int]
    L.mwx_stt_free.argtypes = [C.c_void_p]
    beam = max(1, args.beam)
    eng = L.mwx_stt_new_ex(d.encode(), name.encode(), 1, 20000, beam, b"en", 500, local, 1, 2000,
                           8000)
    if not eng:
        raise RuntimeError("SttEngine init failed")
    cap = 1 << 22
    out = C.create_string_buffer(cap)
    lat = []
    for rep in range(args.warmup + args.steps):
        raw = mwx.synth_pcm16(100 + rep, 30 * 16000).tobytes()
        s = L.mwx_stt_stream_new(eng)
        for p in range(0, len(raw), 16000):  # 0.5-s chunks = stream_buffer_samples
            t0 = time.perf_counter()
            r = L.mwx_stt_stream_feed(s, raw[p:p + 16000], len(raw[p:p + 16000]), out, cap)
            t1 = time.perf_counter()
            if r < 0:
                raise RuntimeError(f"stream feed rc={r}")
            if rep >= args.warmup:
                lat.append((t1 - t0) * 1e3)
        L.mwx_stt_stream_feed(s, b"", 0, out, cap)  # end of speech (final, not timed)
        L.mwx_stt_stream_free(s)
        part = lat[-60:] if rep >= args.warmup else []
        print(f"stream {rep}: {len(part)} timed partials, p50 "
              f"{np.percentile(part, 50) if len(part) else float('nan'):.2f} ms", file=sys.stderr,
              flush=True)
    L.mwx_stt_free(eng)
    lat = np.array(lat)
    line = {"metric": "streaming partial latency (0.5-s cadence, re-transcription of the growing "
                      "buffer)", "value": round(float(np.percentile(lat, 50)), 2), "unit": "ms",
            "higher_is_better": False, "p95_ms": round(float(np.percentile(lat, 95)), 2),
            "max_ms": round(float(lat.max()), 2), "mean_ms": round(float(lat.mean()), 2),
            "partials": int(len(lat)), "streams": args.steps, "n_gpus": 1,
            "dtype": args.wtype, "data": "synthetic (seeded 16 kHz PCM16 stream, seeded weights)",
            "mel_cache": os.environ.get("MWX_NO_MEL_CACHE") is None,
            "config": {"workload": f"whisper-{march} {args.wtype}: one 30-s stream in 0.5-s "
                                   f"chunks through SttEngine/StreamSession, "
                                   f"{'beam-%d' % beam if beam > 1 else 'greedy'} decode until "
                                   f"the model stops"}}
    print(json.dumps(line), flush=True)
    return 0


def run_lanes(n, lanes, step, stagger=0.0):
    """Runs n batches over `lanes` host threads and returns their results in
    batch order. Each lane drives its own states and HIP stream (the
    SttEngine's parallel_requests batchers) and takes the next batch when its
    previous one is done, so one lane's encoder / host work overlaps another
    lane's decode; step(lane) runs one batch on that lane. The first error
    stops every lane and is re-raised."""
    if lanes <= 1:
        return [step(0) for _ in range(n)]
    import threading
    out = {}
    errs = []
    nxt = [0]
    lock = threading.Lock()

    def lane_loop(lane):
        try:
            if stagger > 0:  # (inside the caller's timed region)
                time.sleep(lane * stagger)
            while True:
                with lock:
                    i = nxt[0]
                    nxt[0] += 1
                if i >= n or errs:
                    return
                out[i] = step(lane)
        except Exception as ex:  # re-raised in the calling thread
            errs.append(ex)

    th = [threading.Thread(target=lane_loop, args=(i,)) for i in range(lanes)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    return [out[i] for i in range(n)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one GPU each); without torch.distributed.run, bench.py starts "
                         "them itself")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher + record gather only, synthetic records (no GPU needed)")
    ap.add_argument("--steps", type=int, default=6,
                    help="timed batches (a multiple of --lanes keeps the lanes evenly loaded)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--arch", default="large-v3")
    ap.add_argument("--wtype", default="bf16", choices=["bf16", "f16"])
    ap.add_argument("--clips", type=int, default=32, help="30-s clips per GPU")
    ap.add_argument("--decode-steps", type=int, default=220,
                    help="fixed decode steps per 30-s window (bench_fixed_steps); 0 = decode "
                         "until the model stops (EOT / timestamps), carrying each window's text "
                         "into the next window's prompt")
    ap.add_argument("--rich", action="store_true",
                    help="'-rich' synthetic weights (timestamps, EOT and segment splits in the "
                         "token stream; use with --decode-steps 0)")
    ap.add_argument("--prompt-leg", action="store_true",
                    help="long-form leg with real previous-window text in every prompt: "
                         "--rich --decode-steps 0 --clip-seconds 600")
    ap.add_argument("--service-defaults", action="store_true",
                    help="what a default request of the service costs (src/config.h:47,52, "
                         "src/stt_engine.cpp:204-243): language auto (window-0 detect), beam 5, "
                         "the temperature-fallback ladder (temperature_inc 0.2), token "
                         "timestamps, '-rich' weights decoded to the model's stop")
    ap.add_argument("--no-service-leg", action="store_true",
                    help="skip the service-default leg the full default (C3) run reports beside its "
                         "headline (one batch at --service-defaults, one lane, in a child process; "
                         "--no-cpu-baseline quick runs skip it too)")
    ap.add_argument("--beam", type=int, default=0,
                    help="beam size (0: greedy; the service default is 5)")
    ap.add_argument("--clip-seconds", type=float, default=30.0,
                    help="clip length (> 30: long-form, windows decoded one after another)")
    ap.add_argument("--perf-class", default="dec_attn_cross")
    ap.add_argument("--lanes", type=int, default=2,
                    help="concurrent batches (host threads, each with its own states and HIP "
                         "stream), as the SttEngine's parallel_requests batchers run them")
    ap.add_argument("--lane-stagger", type=float, default=0.0,
                    help="seconds lane i waits (x i) before its first timed batch")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-token-timestamps", action="store_true",
                    help="token_timestamps off (A/B only: the service sets it on)")
    ap.add_argument("--timing", choices=["span", "events"], default="span",
                    help="live kernel timing: device-clock launch spans (default) or HIP event "
                         "brackets")
    ap.add_argument("--no-one-lane", action="store_true",
                    help="skip the one-lane pass after the timed region (a kernel trace of the "
                         "run then holds the multi-lane launches only)")
    ap.add_argument("--fp8", action="store_true",
                    help="MX-fp8 compute (C5): encoder, cross-K/V and decoder weight GEMMs, cross K/V cache")
    ap.add_argument("--host-input", action="store_true",
                    help="PCM in host memory, uploaded inside each step (PCIe-inclusive rate)")
    ap.add_argument("--pcm16", action="store_true",
                    help="with --host-input: upload int16 PCM, converted on the device")
    ap.add_argument("--dump-gather", default=None,
                    help="rank 0 saves the last gathered record block (int32 .npy) here")
    ap.add_argument("--stream", action="store_true",
                    help="streaming partial-latency leg (SURVEY.md §8 f3) instead of transcription")
    ap.add_argument("--prosody", action="store_true",
                    help="segment-prosody leg (SURVEY.md §8 f4) instead of transcription")
    args = ap.parse_args()
    if args.prompt_leg:
        args.rich, args.decode_steps, args.clip_seconds = True, 0, 600.0
    if args.service_defaults:
        args.rich, args.decode_steps = True, 0
        args.beam = args.beam or 5
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    if args.dry_run:
        return dry_run(args, world, rank, local)
    if args.prosody:
        return prosody_bench(args)
    if args.stream:
        return stream_bench(args)

    import torch
    if one_device():
        local = 0
    dist = init_dist(world, local)

    def barrier():
        if dist is not None:
            dist.barrier()

    import mwx
    wt = mwx.GGML_BF16 if args.wtype == "bf16" else mwx.GGML_F16
    march = args.arch + ("-rich" if args.rich else "")
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"mwx_bench_{march}_{args.wtype}.bin")
    if local == 0 and not os.path.exists(path):
        tmp = path + f".tmp{os.getpid()}"
        mwx.write_synthetic_model(tmp, march, wt, 0)
        os.replace(tmp, path)
    barrier()
    ctx = mwx.Context.open(path, device=local,
                           compute=mwx.COMPUTE_MXFP8 if args.fp8 else mwx.COMPUTE_MODEL)
    import shard
    n_samp = int(args.clip_seconds * 16000)
    pcms = [mwx.pcm16_to_f32(mwx.synth_pcm16(k, n_samp)) for k in shard.clip_ids(rank, args.clips)]
    p = ctx.default_params(mwx.SAMPLING_BEAM_SEARCH if args.beam > 1 else mwx.SAMPLING_GREEDY)
    if args.beam > 1:
        p.beam_search.beam_size = args.beam
    p.language = b"auto" if args.service_defaults else b"en"
    p.temperature = 0.0
    p.temperature_inc = 0.2 if args.service_defaults else 0.0
    p.token_timestamps = not args.no_token_timestamps  # on, as the service sets it (src/stt_engine.cpp:225)
    p.suppress_nst = True
    p.bench_fixed_steps = args.decode_steps
    prompt_len = 3 if ARCH[args.arch][5] >= 51865 else 1
    n_windows = max(1, int(np.ceil(args.clip_seconds / 30.0 - 1e-9)))
    # record capacity per clip: a fixed-step window emits decode_steps tokens;
    # decoding to the model's stop, long-form windows advance to the last
    # timestamp (not a fixed 30 s), so a clip can take several times
    # n_windows windows of up to n_text_ctx (448) tokens each
    max_tok = args.decode_steps * n_windows if args.decode_steps else 448 * n_windows * 4
    gathered = {}

    # inputs resident in HBM before the timed region (the PCIe-inclusive rate,
    # host buffers uploaded inside the step, is --host-input)
    lanes = max(1, args.lanes)
    if args.host_input:
        lanes = 1  # (the PCIe-inclusive legs time one batch at a time)
    for i in range(lanes * args.clips):  # all states exist before any lane thread runs
        ctx.state(i)
    if args.host_input and args.pcm16:
        p16s = [mwx.synth_pcm16(k, n_samp) for k in shard.clip_ids(rank, args.clips)]
        run_batch = lambda lane: ctx.full_batch_pcm16(p16s, p)  # noqa: E731
    elif args.host_input:
        run_batch = lambda lane: ctx.full_batch(pcms, p)  # noqa: E731
    else:
        dev = [ctx.upload(x) for x in pcms]
        run_batch = lambda lane: ctx.full_batch_device(dev, p, lane * args.clips)  # noqa: E731

    def step(lane):
        """One batch of `clips` clips on lane `lane` (states lane*clips ..):
        mel -> encoder -> cross K/V -> decode; returns the packed token records."""
        rc = run_batch(lane)
        if rc != 0:
            raise RuntimeError(f"mwx_full_batch rc={rc}")
        print(f"bench.py: lane {lane}: batch done", file=sys.stderr, flush=True)  # (progress)
        s0 = lane * args.clips
        recs = [ctx.token_records(s0 + c) for c in range(args.clips)]
        tok_count.append(sum(len(r) for r in recs))
        return shard.pack_records(recs, max_tok)

    tok_count = []  # tokens generated per batch (list.append: thread-safe)

    gdev = None if dist is not None and dist.get_backend() == "gloo" else "cuda"

    def gather(block):
        # RCCL over xGMI: every rank's token records (id, t0, t1, p) to rank 0
        g = shard.gather_to_rank0(dist, block, device=gdev)
        if g is not None:
            gathered["tokens"] = g

    def run_steps(n):
        for block in run_lanes(n, lanes, step, args.lane_stagger):
            gather(block)

    for lane in range(lanes):
        for _ in range(args.warmup):
            gather(step(lane))
    L = mwx.lib()
    owners = [ctx.state(lane * args.clips) for lane in range(lanes)]  # workspace / stream owners
    # the dominant kernel's class, plus the encoder GEMMs (MFMA fraction,
    # SURVEY.md §8 d asks for both bounds), timed in the same steps
    # (+ event_bracket: the timing events around an empty kernel at the same
    # point of the decode chain, whose average is the events' own cost)
    # Timing (--timing span, the default): launch spans, device clock stamps of
    # the first workgroup start and the last workgroup end (kcommon.h
    # span_start) -- the duration a kernel trace measures, without the
    # dispatch queueing behind the other lane's kernels that a HIP event
    # bracket includes (and without event-record nodes in the graph: they
    # perturbed the other lane). --timing events: event brackets, corrected by
    # an empty kernel's bracket at the same point of the chain (event_bracket)
    kinds = [args.perf_class] + (["enc_gemm"] if args.perf_class != "enc_gemm" else [])
    if args.timing == "span":
        classes = [c + ".span" for c in kinds]
    else:
        classes = kinds + (["event_bracket"] if args.perf_class.startswith("dec_attn") else [])
    for so in owners:
        L.mwx_perf_read(so, None, None)
        L.mwx_perf_enable(so, ",".join(classes).encode())
    for lane in range(lanes):
        ctx.decode_counters(lane * args.clips, reset=True)
        ctx.window_counters(lane * args.clips, reset=True)
        ctx.runahead_fallbacks(lane * args.clips, reset=True)
    del tok_count[:]
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(args.steps)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    import ctypes

    def read_timed(states):
        out = {}
        for cls in classes:
            tot, cnt = 0.0, 0
            for so in states:  # summed over the lanes' states
                tms, nlc = ctypes.c_double(), ctypes.c_int()
                L.mwx_perf_read_class(so, cls.encode(), ctypes.byref(tms), ctypes.byref(nlc))
                tot, cnt = tot + tms.value, cnt + nlc.value
            out[cls] = (tot, cnt)
        for so in states:
            L.mwx_perf_enable(so, None)
        return out

    timed = read_timed(owners)
    # decode work of the timed batches: steps launched (one per token position
    # of the longest row), prompt positions run by the batched prefill, tokens
    # windows decoded and decode attempts (a temperature-fallback re-run is
    # an attempt beyond the window's first), run-ahead attempts redone on the
    # host loop (0 unless device and host disagree)
    dsteps = dpre = nwin = natt = nra = ncs = 0
    for lane in range(lanes):
        a, b = ctx.decode_counters(lane * args.clips, reset=True)
        w, at, cs = ctx.window_counters(lane * args.clips, reset=True)
        dsteps, dpre, nwin, natt, ncs = dsteps + a, dpre + b, nwin + w, natt + at, ncs + cs
        nra += ctx.runahead_fallbacks(lane * args.clips, reset=True)
    n_batches = args.steps
    win_per_clip = nwin / n_batches / args.clips
    decode_work = {"decode_steps_per_batch": round(dsteps / args.steps, 1),
                   "prefill_positions_per_batch": round(dpre / args.steps, 1),
                   "tokens_per_clip": round(sum(tok_count) / args.steps / args.clips, 1),
                   "windows_per_clip": round(win_per_clip, 3),
                   "fallback_reruns_per_clip": round((natt - nwin) / n_batches / args.clips, 3),
                   "runahead_host_redos": nra,
                   "live_clips_per_step": round(ncs / max(1, dsteps), 2)}
    if not args.decode_steps:
        n_windows = win_per_clip  # (encoder work: every decoded window is encoded)
    timed_1lane, steps_1lane, elapsed_1lane = None, 0, None
    if lanes > 1 and not args.no_one_lane:
        # after the timed region (not part of `value`): the same batches on one
        # lane (B = 32 strictly one batch at a time), timed and with the
        # kernels' rooflines measured without another lane's kernels sharing
        # HBM and CUs with them
        steps_1lane = min(2 if args.clip_seconds <= 30 else 1, args.steps)
        L.mwx_perf_read(owners[0], None, None)
        L.mwx_perf_enable(owners[0], ",".join(classes).encode())
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(steps_1lane):
            gather(step(0))
        torch.cuda.synchronize()
        elapsed_1lane = time.perf_counter() - t1
        timed_1lane = read_timed(owners[:1])
    if args.dump_gather and rank == 0 and gathered.get("tokens") is not None:
        np.save(args.dump_gather, gathered["tokens"])
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64, device=gdev or "cpu")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    audio_s = world * args.clips * args.clip_seconds * args.steps
    value = audio_s / elapsed

    def make_roofs(tm, nsteps):
        """(dominant-kernel roofline, encoder-GEMM roofline) from live timings"""
        span = args.timing == "span"
        tot, launches = tm[args.perf_class + (".span" if span else "")]
        if launches == 0 or tot <= 0.0:
            # (a class without span stamps: --timing events times it)
            return ({"kernel": args.perf_class, "error": f"no {args.timing} timings for this class"},
                    None)
        avg_raw = tot / 1e3 / launches
        ev_s = None
        if not span and tm.get("event_bracket", (0, 0))[1] > 0:
            # the bracket of an empty kernel at the same point of the chain:
            # the two event nodes' own cost (+ the empty kernel)
            ev_s = tm["event_bracket"][0] / 1e3 / tm["event_bracket"][1]
        avg_s = avg_raw - ev_s if ev_s is not None and ev_s < 0.5 * avg_raw else avg_raw
        # the engine times every 8th decode step's launches (MWX_PERF_PERIOD),
        # all inside the timed region
        # clips whose cross K/V one launch reads: all of them at fixed steps;
        # decoding to the model's stop, the timed steps' measured average of
        # clips with a live row (clips finish their windows at different steps)
        clips_per_launch = args.clips if args.decode_steps else max(
            1e-9, decode_work["live_clips_per_step"])
        rows = clips_per_launch * max(1, args.beam)
        bound, work, desc = kernel_model(args.arch, args.perf_class, clips_per_launch, rows,
                                         launches // max(1, nsteps), prompt_len,
                                         args.decode_steps, n_windows, kv8=args.fp8)
        traffic = None
        tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(tf):
            try:
                key = f"{args.arch}:{args.perf_class}:{args.clips}" + (":fp8" if args.fp8 else "")
                traffic = json.load(open(tf)).get(key) if args.beam <= 1 else None
            except Exception:
                traffic = None
        if bound == "hbm":
            achieved = work / avg_s / 1e9
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": traffic}
        else:
            achieved = work / avg_s / 1e12
            roof = {"bound": "mfma", "achieved": round(achieved, 1), "peak": MFMA_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(achieved / MFMA_PEAK_TFLOPS, 4),
                    "traffic": traffic}
        roof.update({"kernel": args.perf_class, "avg_launch_us": round(avg_s * 1e6, 2),
                     "timing": ("launch span (device clock: first workgroup start to last "
                                "workgroup end, every 8th decode step)") if span
                               else "event bracket - event cost",
                     "launches": launches, "work_per_launch": work, "work_desc": desc})
        if not span:
            roof.update({"avg_bracket_us": round(avg_raw * 1e6, 2),
                         "event_bracket_us": round(ev_s * 1e6, 2) if ev_s is not None else None})
        roof_enc = None
        ecls = "enc_gemm" + (".span" if span else "")
        if ecls in tm and args.perf_class != "enc_gemm" and tm[ecls][1] > 0:
            ems, en = tm[ecls]
            _, ework, edesc = kernel_model(args.arch, "enc_gemm", args.clips, rows,
                                           en // max(1, nsteps), prompt_len, args.decode_steps,
                                           n_windows)
            eavg = ems / 1e3 / en
            epeak = 2 * MFMA_PEAK_TFLOPS if args.fp8 else MFMA_PEAK_TFLOPS
            each = ework / eavg / 1e12
            roof_enc = {"bound": "mfma", "achieved": round(each, 1), "peak": epeak,
                        "unit": "TFLOP/s", "frac": round(each / epeak, 4), "kernel": "enc_gemm",
                        "avg_launch_us": round(eavg * 1e6, 2), "launches": en,
                        "timing": "launch span (device clock)" if span else "event bracket",
                        "work_per_launch": ework, "work_desc": edesc}
        return roof, roof_enc

    if rank == 0:
        roof, roof_enc = make_roofs(timed, args.steps)
        if roof_enc is not None and lanes > 1:
            roof_enc["note"] = ("spans of the encoder GEMMs while the other lanes' decode "
                                "kernels share the CUs (the encoder runs on a low-priority "
                                "stream); one_lane.roofline_encoder is the uncontended rate")
        roof_1lane = None
        if timed_1lane is not None:
            r1, e1 = make_roofs(timed_1lane, steps_1lane)
            v1 = args.clips * args.clip_seconds * steps_1lane / elapsed_1lane
            roof_1lane = {"note": f"{steps_1lane} batches on one lane after the timed region "
                                  f"(one batch of {args.clips} clips at a time)",
                          "value": round(v1, 2), "unit": "audio-sec/s",
                          "ms_per_step": round(elapsed_1lane / steps_1lane * 1e3, 2),
                          "roofline": r1, "roofline_encoder": e1}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            # all cores granted to this job (the GPU box: 16 per GPU, OMP_NUM_THREADS)
            threads = granted_cpus()[0]
            try:
                sys.path.insert(0, os.path.join(ROOT, "oracle"))
                cpu = cpu_baseline(path, args.arch, threads, prompt_len, args.decode_steps)
            except Exception as ex:  # reported, never fatal to the GPU number
                cpu = {"error": str(ex)}
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "audio-sec/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": (f"mxfp8 (encoder/cross/decoder weight GEMMs, cross K/V cache) + {args.wtype}"
                      if args.fp8 else args.wtype),
            "data": ("synthetic (seeded 16 kHz PCM16 clips, "
                     + (("host int16, uploaded and converted per step" if args.pcm16 else
                         "host memory, uploaded per step") if args.host_input else "resident in HBM")
                     + "; seeded weights in the ggml .bin layout)"),
            "config": {
                "workload": (f"whisper-{args.arch}{' (-rich weights)' if args.rich else ''} "
                             f"{'MX-fp8 compute (from the ' + args.wtype + ' file)' if args.fp8 else args.wtype}"
                             f": batches of {args.clips} x "
                             f"{args.clip_seconds:g} s clips per GPU ({lanes} in flight), "
                             f"{'service defaults (language auto: window-0 detect; temperature ladder 0.0/0.2/../1.0), ' if args.service_defaults else ''}mel + "
                             f"encoder + cross-KV + {args.decode_steps or 'until-EOT'} "
                             f"{'beam-%d' % args.beam if args.beam > 1 else 'greedy'} KV-cached "
                             f"decode steps per 30-s window, token timestamps "
                             f"{'OFF (A/B)' if args.no_token_timestamps else 'on (as the service)'}, RCCL "
                             f"token gather to rank 0"),
                "global_batch": world * args.clips,
                "seq_len": 1500,
                "parallelism": f"dp{world}",
                "lanes": lanes,
            },
            "audio_sec_per_s_per_gpu": round(value / world, 2),
            "rtf": round(elapsed / audio_s * world, 6),
            "x_realtime_per_gpu": round(value / world, 1),
            "gathered": gather_summary(gathered.get("tokens"), world * args.clips,
                                       max_tok if args.decode_steps else None),
            "decode_work": decode_work,
            "roofline": roof,
            "roofline_encoder": roof_enc,
            "one_lane": roof_1lane,
            "cpu_baseline": cpu,
        }
    ctx.close()
    if rank == 0:
        if world == 1 and is_headline_config(args):
            line["service_defaults"] = service_leg()
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
