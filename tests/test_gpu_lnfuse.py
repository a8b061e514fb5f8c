"""Decode LayerNorm folded into the consumer GEMMs for <= 4 rows (the
single-request / streaming case, config C2; kernels.h LnFuse): every
workgroup of the consumer recomputes the rows' LayerNorm exactly as the
separate ln_dec launch does, so the results with MWX_LN_FUSE=1 must be the same
bits as with the default separate LayerNorm launches (MWX_LN_FUSE=0)."""
import json
import os
import subprocess
import sys

import pytest

import mwx

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_RUN = r'''
import json, sys
sys.path.insert(0, "sentiric-stt-whisper-service_amd")
import mwx
path, n, inc = sys.argv[1], int(sys.argv[2]), float(sys.argv[3])
ctx = mwx.Context.open(path)
p = ctx.default_params(mwx.SAMPLING_GREEDY)
p.token_timestamps = True
p.suppress_nst = True
p.no_speech_thold = 0.85
p.entropy_thold = 2.40
p.logprob_thold = -0.7
p.temperature_inc = inc
p.greedy.best_of = 5
p.language = b"en"
pcms = [mwx.pcm16_to_f32(mwx.synth_pcm16(20 + k, int((45.0 - 7.5 * k) * 16000))) for k in range(n)]
assert ctx.full_batch(pcms, p) == 0
out = [[[s.t0, s.t1, s.text, [(t.id, t.tid, t.p, t.plog, t.pt, t.t0, t.t1) for t in s.tokens]]
        for s in ctx.segments(i)] for i in range(n)]
print(json.dumps(out))
'''


def run(path, n, inc, fuse):
    env = dict(os.environ, MWX_LN_FUSE="1" if fuse else "0")
    r = subprocess.run([sys.executable, "-c", _RUN, path, str(n), str(inc)], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("arch,wtype,n,inc", [
    ("micro-rich", mwx.GGML_F16, 1, 0.2),     # d 128, fallback (best_of 5 rows > 4: unfused)
    ("tiny.en-rich", mwx.GGML_F16, 3, 0.0),   # d 384, split-K 3 slabs, 3 rows
    ("base-rich", mwx.GGML_F16, 2, 0.0),      # d 512 (config C2 shapes), two rows
    ("large-v3-l2-rich", mwx.GGML_BF16, 2, 0.0),  # d 1280, bf16, 2 rows
])
def test_ln_fused_equals_separate(make_model, arch, wtype, n, inc):
    path = make_model(arch, wtype)
    a = run(path, n, inc, True)
    b = run(path, n, inc, False)
    assert a == b
    assert sum(len(s[3]) for c in a for s in c) > 3 * n
