"""Paired decode (MWX_DECODE_PAIR=1, engine.cpp decode_group_pair): a step's
rows split into two sets whose layer chains run on two streams with their
cross-attentions interleaved. Every set runs the kernels of a decode step of
that set alone and every kernel is row-blocked, so the results must be the
same bits as the unpaired step (greedy run-ahead, temperature fallback with
best_of rows, beam search groups, bf16 at v3 geometry)."""
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
path, n, inc, beam = sys.argv[1], int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4])
ctx = mwx.Context.open(path)
p = ctx.default_params(mwx.SAMPLING_BEAM_SEARCH if beam else mwx.SAMPLING_GREEDY)
if beam:
    p.beam_search.beam_size = beam
p.token_timestamps = True
p.suppress_nst = True
p.no_speech_thold = 0.85
p.entropy_thold = 2.40
p.logprob_thold = -0.7
p.temperature_inc = inc
p.greedy.best_of = 5
p.language = b"en"
pcms = [mwx.pcm16_to_f32(mwx.synth_pcm16(40 + k, int((45.0 - 5.0 * k) * 16000))) for k in range(n)]
assert ctx.full_batch(pcms, p) == 0
out = [[[s.t0, s.t1, s.text, [(t.id, t.tid, t.p, t.plog, t.pt, t.t0, t.t1) for t in s.tokens]]
        for s in ctx.segments(i)] for i in range(n)]
print(json.dumps(out))
'''


def run(path, n, inc, beam, pair):
    env = dict(os.environ, MWX_DECODE_PAIR="1" if pair else "0", MWX_PAIR_MIN="2")
    r = subprocess.run([sys.executable, "-c", _RUN, path, str(n), str(inc), str(beam)], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("arch,wtype,n,inc,beam", [
    ("micro-rich", mwx.GGML_F16, 6, 0.0, 0),          # greedy, run-ahead loop
    ("micro-rich", mwx.GGML_F16, 4, 0.2, 0),          # fallback: best_of 5 rows per clip
    ("tiny.en-rich", mwx.GGML_F16, 4, 0.0, 5),        # beam 5 groups (split at a clip boundary)
    ("large-v3-l2-rich", mwx.GGML_BF16, 5, 0.0, 0),   # bf16, d 1280, odd row count
])
def test_paired_decode_equals_single_chain(make_model, arch, wtype, n, inc, beam):
    path = make_model(arch, wtype)
    a = run(path, n, inc, beam, True)
    b = run(path, n, inc, beam, False)
    assert a == b
    assert sum(len(s[3]) for c in a for s in c) > 3 * n
