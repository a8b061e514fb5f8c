"""GPU parity on the benchmarked model itself: large-v3 at full depth (32 + 32
layers, bf16, the seed-0 synthetic weights bench.py runs), plus plain-weight
greedy decoding at large-v3 geometry with the oracle's top-1 margin reported
at every step.

North star: token-id-exact greedy decode against the CPU reference path
(BASELINE.json configs[2]). The other large-v3 tests run 2 + 2 layers
(test_gpu_shapes.py); these check that bf16 rounding noise accumulated over 32
encoder and 32 decoder layers still leaves the device's greedy tokens equal to
the oracle's, on the exact workload the bench times (bench_fixed_steps: EOT and
timestamp tokens masked, every step a text token)."""
import numpy as np
import pytest

import mwx
import orc
from test_gpu_parity import assert_same, pcm_clip, service_params

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

STEPS = 32  # decode steps per window (the bench runs 220; the oracle pays ~0.1 s per step)


@pytest.fixture(scope="module")
def v3full(make_model):
    path = make_model("large-v3", mwx.GGML_BF16)
    ctx = mwx.Context.open(path)
    yield ctx, path
    ctx.close()


def bench_params(ctx, steps=STEPS):
    p = service_params(ctx, temperature_inc=0.0, language=b"en")
    p.bench_fixed_steps = steps
    return p


def greedy_opt(steps=0):
    opt = orc.FullOptions.service_defaults()
    opt.temperature_inc = 0.0
    opt.language = "en"
    opt.bench_fixed_steps = steps
    return opt


def text_margins(o, pcm, prompt, toks, n_text):
    """The oracle's own top-1 minus top-2 logit, over the first n_text
    vocabulary entries (the text tokens), at every generated step of window 0:
    how far each greedy choice is from a tie in the reference arithmetic."""
    mel, _ = o.mel(pcm)
    k, v = o.cross(o.encode(mel))
    lg = o.decode_seq(k, v, list(prompt) + list(toks[:-1]))
    lg = lg[len(prompt) - 1:, :n_text]
    s = np.sort(lg, axis=1)
    return s[:, -1] - s[:, -2]


def test_full_depth_large_v3_greedy_matches_oracle(v3full):
    """The benched model end to end (mel, 32 encoder layers, cross K/V, 32
    decoder layers, logits processing): greedy token ids exactly the oracle's,
    probabilities within bf16 noise; the oracle's margins are printed."""
    ctx, path = v3full
    pcm = pcm_clip(0)
    assert ctx.full(pcm, bench_params(ctx), state_index=0) == 0
    segs = ctx.segments(0)
    o = orc.Oracle(path)
    _, osegs, _, _ = o.full(pcm, greedy_opt(STEPS))
    ids = [t.id for s in segs for t in s.tokens]
    oids = [t.id for s in osegs for t in s.tokens]
    m = text_margins(o, pcm, [o.sot, o.sot + 1, o.transcribe], oids, o.eot)
    print(f"full-depth large-v3: {len(oids)} tokens, oracle top-1 margin min {m.min():.4f} "
          f"median {np.median(m):.4f}")
    assert len(oids) == STEPS
    assert ids == oids, next(((i, a, b, float(m[i])) for i, (a, b) in enumerate(zip(ids, oids))
                              if a != b), None)
    p = np.array([t.p for s in segs for t in s.tokens])
    op = np.array([t.p for s in osegs for t in s.tokens])
    assert np.abs(p - op).max() < 3e-2, np.abs(p - op).max()


def test_full_depth_large_v3_batch_equals_single(v3full):
    """4 clips of the benched model in one mwx_full_batch == each alone, token
    for token and probability for probability (rows in 16-row blocks, 4 of
    them active; the bench runs 32)."""
    ctx, _ = v3full
    p = bench_params(ctx)
    pcms = [pcm_clip(k, 30.0 - 2.5 * k) for k in range(4)]
    assert ctx.full_batch_states(pcms, p, range(1, 5)) == 0
    batched = [[(t.id, t.p) for s in ctx.segments(1 + i) for t in s.tokens] for i in range(4)]
    for i, pcm in enumerate(pcms):
        assert ctx.full(pcm, p, state_index=5) == 0
        assert [(t.id, t.p) for s in ctx.segments(5) for t in s.tokens] == batched[i], i
    assert all(len(b) == STEPS for b in batched)


def test_v3_geometry_plain_weights_greedy_matches_oracle(make_model):
    """Plain (non -rich) synthetic weights at large-v3 geometry (d 1280, 20
    heads, 128 mels, vocab 51866; 2 + 2 layers), the service's greedy
    parameters, no fixed step count: the logits carry no engineered
    separation, so this is the strict case. Token ids / segments exactly the
    oracle's; the oracle's top-1 margin at every step is printed."""
    path = make_model("large-v3-l2", mwx.GGML_BF16)
    o = orc.Oracle(path)
    with mwx.Context.open(path) as ctx:
        for k in (0, 1):
            pcm = pcm_clip(k)
            assert ctx.full(pcm, service_params(ctx, temperature_inc=0.0, language=b"en"),
                            state_index=k) == 0
            segs = ctx.segments(k)
            _, osegs, _, windows = o.full(pcm, greedy_opt())
            oids = [t.id for s in osegs for t in s.tokens]
            m = text_margins(o, pcm, [o.sot, o.sot + 1, o.transcribe], windows[0], o.n_vocab)
            print(f"plain large-v3-l2 clip {k}: {len(oids)} tokens in {len(windows)} window(s), "
                  f"oracle top-1 margin min {m.min():.4f} median {np.median(m):.4f}")
            assert len(oids) > 10
            # (plain weights carry no timestamp signal: the timestamp argmax
            # behind the diagnostic `tid` field is a tie within bf16 noise —
            # seen: pt 0.3441 / 0.3416 on the same text token, equal t0 / t1)
            assert_same(segs, osegs, p_tol=3e-2, tid_tie_tol=1e-2)
