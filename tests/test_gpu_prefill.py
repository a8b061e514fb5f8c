"""Batched prompt prefill (SURVEY.md §3.5 "prefill").

whisper.cpp decodes a window's prompt — [SOT_PREV, prompt_past..., SOT,
lang, task] — in one whisper_decode call; the service passes
`initial_prompt` (/root/reference/src/stt_engine.cpp:233) and long-form
transcription carries the previous windows' text as `prompt_past`. mwx runs
positions 0 .. P-2 of the prompt as virtual rows of one pass of the decoder
layer stack (engine.cpp Driver::prefill) and starts the decode loop at the
prompt's last position. Every virtual row's arithmetic is a decode step's,
so the results must be bit-identical to stepping through the prompt
(MWX_PREFILL_MIN=0) and token-exact against the oracle."""
import json
import os
import subprocess
import sys

import pytest

import mwx
import orc
from test_gpu_parity import assert_same, pcm_clip, service_params

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROMPT = b" the quick brown fox jumps over the lazy dog"

_RUN = r'''
import json, sys
sys.path.insert(0, "sentiric-stt-whisper-service_amd")
import mwx
path, beam, inc, secs, prompt = sys.argv[1], int(sys.argv[2]), float(sys.argv[3]), float(sys.argv[4]), sys.argv[5]
ctx = mwx.Context.open(path)
p = ctx.default_params(mwx.SAMPLING_BEAM_SEARCH if beam > 1 else mwx.SAMPLING_GREEDY)
if beam > 1:
    p.beam_search.beam_size = beam
p.token_timestamps = True
p.suppress_nst = True
p.no_speech_thold = 0.85
p.entropy_thold = 2.40
p.logprob_thold = -0.7
p.temperature_inc = inc
p.greedy.best_of = 5
p.language = b"en"
if prompt:
    p.initial_prompt = prompt.encode()
pcms = [mwx.pcm16_to_f32(mwx.synth_pcm16(k, int((secs - 9.5 * k) * 16000))) for k in range(3)]
assert ctx.full_batch(pcms, p) == 0
steps, pf = ctx.decode_counters(0)
out = [[[s.t0, s.t1, s.text, [(t.id, t.tid, t.p, t.plog, t.t0, t.t1) for t in s.tokens]]
        for s in ctx.segments(i)] for i in range(len(pcms))]
print(json.dumps({"out": out, "steps": steps, "prefill": pf}))
'''


def run(path, beam, inc, secs, prompt, prefill_min):
    env = dict(os.environ, MWX_PREFILL_MIN=str(prefill_min))
    r = subprocess.run([sys.executable, "-c", _RUN, path, str(beam), str(inc), str(secs),
                        prompt.decode()], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=400)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("arch,wtype,fp8", [("micro", mwx.GGML_F16, False),
                                            ("tiny.en", mwx.GGML_F16, False),
                                            ("large-v3-l2", mwx.GGML_BF16, False),
                                            ("large-v3-l2", mwx.GGML_BF16, True)])
def test_prefill_logits_equal_stepwise(make_model, arch, wtype, fp8):
    """Teacher-forced: tokens 0 .. n-2 through the prefill (one pass, virtual
    rows in 16- / 32-row GEMM blocks, cross-attention in groups of q = min(8,
    n - 1): q = 2 .. 8, every grouped-kernel instantiation a short prompt
    takes) and the last as a decode step (the chained seams) give the
    stepwise logits bit for bit, for prompts of 3 .. 226 positions (chunks of
    up to MWX_PREFILL_ROWS rows); also in the MX-fp8 compute mode, whose
    cross-attention is the MFMA-score grouped kernel for every group size."""
    path = make_model(arch, wtype)
    import numpy as np
    with mwx.Context.open(path, compute=mwx.COMPUTE_MXFP8 if fp8 else mwx.COMPUTE_MODEL) as ctx:
        ctx.test_encode(pcm_clip(1), cross=False, state_index=0)
        ctx.test_encode(pcm_clip(1), cross=False, state_index=1)
        rng = np.random.default_rng(7)
        for n in (3, 4, 5, 6, 7, 8, 9, 70, 226):
            toks = [int(t) for t in rng.integers(0, 50000, n)]
            a = ctx.test_decode_last(toks, state_index=0)
            b = ctx.test_decode_last_prefill(toks, state_index=1)
            assert np.array_equal(a, b), (n, np.abs(a - b).max())


@pytest.mark.parametrize("arch,wtype,beam,inc", [
    ("micro-rich", mwx.GGML_F16, 1, 0.2),
    ("large-v3-l2-rich", mwx.GGML_BF16, 1, 0.0),
    ("large-v3-l2-rich", mwx.GGML_BF16, 5, 0.0),
])
def test_prefill_equals_stepwise(make_model, arch, wtype, beam, inc):
    """Three long-form clips (70 / 60.5 / 51 s) with an initial prompt, one
    batch: prefill on (default) and off give the same token ids, timestamps
    and probabilities bit for bit (greedy with fallback, beam 5 at large-v3
    geometry), and the prefill removes the prompt's positions from the decode
    steps."""
    path = make_model(arch, wtype)
    on = run(path, beam, inc, 70.0, PROMPT, 2)
    off = run(path, beam, inc, 70.0, PROMPT, 0)
    assert on["out"] == off["out"]
    assert sum(len(s[3]) for c in on["out"] for s in c) > 30
    assert off["prefill"] == 0 and on["prefill"] > 0
    assert on["steps"] + on["prefill"] // 3 <= off["steps"], (on["steps"], on["prefill"], off["steps"])
    print(f"{arch} beam {beam}: decode steps {off['steps']} -> {on['steps']} "
          f"(+{on['prefill']} prompt positions prefilled)")


@pytest.mark.parametrize("arch,wtype", [("micro-rich", mwx.GGML_F16),
                                        ("large-v3-l2-rich", mwx.GGML_BF16)])
def test_prefill_long_form_initial_prompt_matches_oracle(make_model, arch, wtype):
    """70-s long-form clip, initial prompt, the service's greedy parameters:
    window after window the prompt (previous text + init) is prefilled; token
    ids, segments and token timestamps exactly the oracle's."""
    path = make_model(arch, wtype)
    pcm = pcm_clip(4, 70.0)
    with mwx.Context.open(path) as ctx:
        p = service_params(ctx, temperature_inc=0.0, language=b"en")
        p.initial_prompt = PROMPT
        assert ctx.full(pcm, p, state_index=0) == 0
        segs = ctx.segments(0)
        steps, pf = ctx.decode_counters(0)
    opt = orc.FullOptions.service_defaults()
    opt.temperature_inc = 0.0
    opt.language = "en"
    opt.initial_prompt = PROMPT.decode()
    _, osegs, _, windows = orc.Oracle(path).full(pcm, opt)
    assert len(windows) >= 2 and len(segs) >= 2
    # (bf16 at v3 geometry: the diagnostic `tid` of a text token can be a
    # timestamp tie within rounding noise, seen pt 0.4272 / 0.4253)
    assert_same(segs, osegs, p_tol=2e-2, tid_tie_tol=2e-2)
    # every window's prompt but its last position went through the prefill
    # (the step counts with and without it: test_prefill_equals_stepwise)
    assert pf >= len(PROMPT.split()) * len(windows), (steps, pf)
    print(f"{arch}: {len(windows)} windows, {steps} decode steps, {pf} prompt positions prefilled")
