"""Diagnostic (GPU): the two-engine-rank bench gather vs single-clip runs,
repeated, to locate a nondeterministic record (r06aa). Measurement probe."""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sentiric-stt-whisper-service_amd")]
import mwx  # noqa: E402
import shard  # noqa: E402

gathers = []
for trial in range(3):
    d = tempfile.mkdtemp(prefix=f"mrdiag{trial}_")
    out = os.path.join(d, "gathered.npy")
    env = dict(os.environ, MWX_BENCH_ONE_DEVICE="1", TMPDIR=d)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--arch", "micro",
           "--wtype", "f16", "--clips", "3", "--steps", "1", "--warmup", "0", "--lanes", "1",
           "--decode-steps", "24", "--no-cpu-baseline", "--no-one-lane", "--dump-gather", out]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    print("trial", trial, "rc", r.returncode, flush=True)
    if r.returncode != 0:
        print(r.stderr[-3000:])
        sys.exit(1)
    gathers.append((d, shard.unpack_records(np.load(out))))
base = gathers[0][1]
for t, (_, g) in enumerate(gathers):
    print("gather", t, "== gather 0 per clip:", [g[c] == base[c] for c in range(6)], flush=True)
path = os.path.join(gathers[0][0], "mwx_bench_micro_f16.bin")
singles = {}
with mwx.Context.open(path) as ctx:
    p = ctx.default_params(mwx.SAMPLING_GREEDY)
    p.language = b"en"
    p.temperature = 0.0
    p.temperature_inc = 0.0
    p.token_timestamps = True
    p.suppress_nst = True
    p.bench_fixed_steps = 24
    idx = 0
    for fold in (True, False, True):
        mwx.set_ln_fold(fold)
        recs = []
        for c in range(6):
            pcm = mwx.pcm16_to_f32(mwx.synth_pcm16(c, 30 * 16000))
            assert ctx.full(pcm, p, state_index=idx) == 0
            recs.append(ctx.token_records(idx))
            idx += 1
        singles.setdefault(fold, []).append(recs)
        print("fold", fold, "single == gather 0 per clip:", [recs[c] == base[c] for c in range(6)],
              flush=True)
    # batch of 3 in this process (no fold: R = 3), both shards
    for r0 in (0, 3):
        pcms = [mwx.pcm16_to_f32(mwx.synth_pcm16(c, 30 * 16000)) for c in range(r0, r0 + 3)]
        st = list(range(idx, idx + 3))
        for s in st:
            ctx.state(s)
        assert ctx.full_batch_states(pcms, p, st) == 0
        recs = [ctx.token_records(s) for s in st]
        idx += 3
        print("batch", r0, "== gather 0:", [recs[i] == base[r0 + i] for i in range(3)],
              "== single fold:", [recs[i] == singles[True][0][r0 + i] for i in range(3)], flush=True)
    mwx.set_ln_fold(None)
for c in range(6):
    a, b = singles[True][0][c], base[c]
    if a != b:
        i = next(i for i, (x, y) in enumerate(zip(a, b)) if x != y)
        print("clip", c, "first diff at token", i, a[i], b[i])
