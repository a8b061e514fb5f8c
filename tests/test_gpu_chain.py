"""Chained decode seams (k_chain.hip): out-proj -> LN2 ->
cross-Q, cross-out -> LN3 -> FFN1 and FFN2 -> LN1 -> QKV each run as ONE
launch whose three block roles hand off through counters, instead of three
launches. Every block's arithmetic is that of the separate kernels
(gemm_splitk_partials, layer_norm_dec, the 4-wave FFN1 gemm_decode), so the
results must be the same bits with the chain on (the default for decode steps
of <= 64 rows) and off (mwx_test_set_chain(0)), on every path the chain
takes: greedy run-ahead, the sampling fallback (best_of 5 rows), beam search
with few clips (<= 64 rows), one request (C2 shapes), and the widths of
micro / tiny / base / large-v3."""
import numpy as np
import pytest

import mwx
from test_gpu_parity import service_params

pytestmark = pytest.mark.gpu


def transcribe(path, n, secs, inc=0.0, beam=0, chain=True):
    prev = mwx.set_chain(chain)
    try:
        with mwx.Context.open(path) as ctx:
            p = service_params(ctx, beam=beam or 1, temperature_inc=inc, language=b"en")
            pcms = [mwx.pcm16_to_f32(mwx.synth_pcm16(30 + k, int((secs - 6.5 * k) * 16000)))
                    for k in range(n)]
            rc = ctx.full_batch(pcms, p)
            assert rc == 0, rc
            return [[(s.t0, s.t1, s.text, [(t.id, t.tid, t.p, t.plog, t.pt, t.ptsum, t.t0, t.t1)
                                           for t in s.tokens]) for s in ctx.segments(i)]
                    for i in range(n)]
    finally:
        mwx.set_chain(None if prev < 0 else bool(prev))


@pytest.mark.parametrize("arch,wtype,n,secs,inc,beam", [
    ("micro-rich", mwx.GGML_F16, 2, 45.0, 0.2, 0),       # d 128, fallback: best_of 5 rows
    ("tiny.en-rich", mwx.GGML_F16, 3, 40.0, 0.0, 0),     # d 384, split-K 3 slabs
    ("base-rich", mwx.GGML_F16, 1, 30.0, 0.0, 0),        # d 512, one request (C2)
    ("large-v3-l2-rich", mwx.GGML_BF16, 4, 35.0, 0.0, 0),  # d 1280 bf16 (C3 widths)
    ("large-v3-l2-rich", mwx.GGML_BF16, 2, 30.0, 0.0, 5),  # beam 5: 10 rows
    ("micro-rich", mwx.GGML_F16, 12, 30.0, 0.0, 5),      # beam 5: 60 rows, 4 row blocks
])
def test_chained_seams_equal_separate_launches(make_model, arch, wtype, n, secs, inc, beam):
    path = make_model(arch, wtype)
    on = transcribe(path, n, secs, inc, beam, chain=True)
    off = transcribe(path, n, secs, inc, beam, chain=False)
    assert on == off
    assert sum(len(s[3]) for c in on for s in c) > 3 * n


def test_chained_teacher_forced_logits_equal(make_model):
    """Teacher-forced logits of a decode-step path (chain) against the same
    steps with the chain off, bit for bit, at large-v3 width."""
    path = make_model("large-v3-l2", mwx.GGML_BF16)
    rng = np.random.default_rng(3)
    toks = [int(t) for t in rng.integers(0, 50000, 24)]
    out = {}
    for chain in (True, False):
        prev = mwx.set_chain(chain)
        try:
            with mwx.Context.open(path) as ctx:
                ctx.test_encode(mwx.pcm16_to_f32(mwx.synth_pcm16(5, 20 * 16000)), cross=False)
                out[chain] = ctx.test_decode_last(toks)
        finally:
            mwx.set_chain(None if prev < 0 else bool(prev))
    assert np.array_equal(out[True].view(np.uint32), out[False].view(np.uint32))
