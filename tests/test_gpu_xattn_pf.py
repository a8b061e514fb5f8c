"""L2-prefetch helper workgroups in the cross-attention of small grids
(MWX_XATTN_PF=7, k_attn.hip dec_attn_kernel PF): the helpers only load K / V
rows into L2; the attending workgroups' arithmetic is unchanged, so the
results must be the same bits as without them (base geometry: 8 heads, one
and two requests)."""
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


def run(path, n, inc, pf):
    env = dict(os.environ, MWX_XATTN_PF="7" if pf else "0")
    r = subprocess.run([sys.executable, "-c", _RUN, path, str(n), str(inc)], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("n", [1, 2])
def test_xattn_prefetch_helpers_bit_identical(make_model, n):
    path = make_model("base-rich", mwx.GGML_F16)
    a = run(path, n, 0.0, True)
    b = run(path, n, 0.0, False)
    assert a == b
    assert sum(len(s[3]) for c in a for s in c) > 3 * n
