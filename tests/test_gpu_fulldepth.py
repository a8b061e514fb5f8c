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

STEPS = 32  # decode steps per window of the cheaper tests (the oracle pays ~0.1 s per step)
BENCH_STEPS = 220  # bench.py's bench_fixed_steps (n_text_ctx / 2 - 4)


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
    decoder layers, logits processing) on the bench's own window: 220 fixed
    greedy steps (bench.py's bench_fixed_steps). Checks, along the oracle's
    token stream: the device's teacher-forced logits within bf16 noise of the
    oracle's (err printed); the device's argmax of the processed logits equal
    to the oracle's token at every step whose oracle top-1 margin exceeds 2 x
    err; and the free-running token ids equal to the oracle's up to the first
    step whose margin is inside that noise (all 220 where there is none)."""
    ctx, path = v3full
    pcm = pcm_clip(0)
    assert ctx.full(pcm, bench_params(ctx, BENCH_STEPS), state_index=0) == 0
    segs = ctx.segments(0)
    o = orc.Oracle(path)
    _, osegs, _, _ = o.full(pcm, greedy_opt(BENCH_STEPS))
    ids = [t.id for s in segs for t in s.tokens]
    oids = [t.id for s in osegs for t in s.tokens]
    assert len(oids) == BENCH_STEPS and len(ids) == BENCH_STEPS
    prompt = [o.sot, o.sot + 1, o.transcribe]
    mel, _ = o.mel(pcm)
    k, v = o.cross(o.encode(mel))
    lg_o = o.decode_seq(k, v, prompt + oids[:-1])[len(prompt) - 1:]
    ctx.test_encode(pcm, cross=False)
    lg_d = ctx.test_decode(prompt + oids[:-1])[len(prompt) - 1:]
    n_text = o.eot
    err = float(np.abs(lg_d[:, :n_text] - lg_o[:, :n_text]).max())
    so = np.sort(lg_o[:, :n_text], axis=1)
    m = so[:, -1] - so[:, -2]
    # the argmax of the processed logits (bench_fixed_steps: EOT and
    # timestamps masked, suppress_nst) on both sides
    agree = 0
    for i in range(BENCH_STEPS):
        pre, _, _, rec = o.process_logits(lg_o[i], oids[:i], False, 3000, suppress_nst=True,
                                          bench_fixed_steps=BENCH_STEPS)
        assert rec[0] == oids[i]
        dmask = np.where(np.isneginf(pre), -np.inf, lg_d[i])
        if m[i] > 2 * err:
            assert int(np.argmax(dmask)) == oids[i], (i, float(m[i]), err)
            agree += 1
    first = next((i for i, (a, b) in enumerate(zip(ids, oids)) if a != b), None)
    print(f"full-depth large-v3, {BENCH_STEPS} steps: logits err {err:.4f}; oracle top-1 margin "
          f"min {m.min():.4f} median {np.median(m):.4f}; teacher-forced argmax checked at "
          f"{agree} steps; free-running ids equal up to step "
          f"{BENCH_STEPS if first is None else first}")
    assert err < 0.25, err
    if first is not None:
        # a divergence is allowed only at a step the reference arithmetic
        # itself cannot separate from a tie at bf16 noise
        assert m[first] <= 2 * err, (first, ids[first], oids[first], float(m[first]), err)
    p = np.array([t.p for s in segs for t in s.tokens])[: first or BENCH_STEPS]
    op = np.array([t.p for s in osegs for t in s.tokens])[: first or BENCH_STEPS]
    assert np.abs(p - op).max() < 3e-2, np.abs(p - op).max()


def test_bench_workload_each_clip_equals_single(v3full):
    """bench.py's own timed call at full size: large-v3 bf16, 32 clips per
    batch from device-resident PCM, two batches in flight on two host threads
    (lanes, each on its own 32 states and HIP stream), bench_fixed_steps 220,
    token_timestamps on. Every clip's token records (id, t0, t1, p) equal that
    clip decoded alone (batch == single and lane independence, at the
    benched size)."""
    import threading
    ctx, _ = v3full
    n = 32
    p = ctx.default_params(mwx.SAMPLING_GREEDY)  # (bench.py main(), same fields)
    p.language = b"en"
    p.temperature = 0.0
    p.temperature_inc = 0.0
    p.token_timestamps = True
    p.suppress_nst = True
    p.bench_fixed_steps = BENCH_STEPS
    pcms = [mwx.pcm16_to_f32(mwx.synth_pcm16(k, 30 * 16000)) for k in range(n)]
    base = len(ctx.states)
    for i in range(2 * n + 1):
        ctx.state(base + i)
    dev = [ctx.upload(x) for x in pcms]
    rcs = [None, None]

    def lane(j):
        rcs[j] = ctx.full_batch_device(dev, p, base + j * n)

    th = [threading.Thread(target=lane, args=(j,)) for j in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert rcs == [0, 0], rcs
    recs = [[ctx.token_records(base + j * n + c) for c in range(n)] for j in range(2)]
    single = base + 2 * n
    for c in range(n):
        assert ctx.full(pcms[c], p, state_index=single) == 0
        want = ctx.token_records(single)
        assert len(want) == BENCH_STEPS
        assert recs[0][c] == want, c
        assert recs[1][c] == want, c
    for b in dev:
        b.free()


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


def test_full_depth_large_v3_language_auto_matches_oracle(v3full):
    """The service's default language = "auto" (/root/reference/src/config.h:47)
    on the benched model at full depth: the window-0 detect (encode, one
    decode of <|startoftranscript|>, argmax over the language tokens) and the
    greedy window that follows (STEPS fixed steps) against the oracle. The
    detected language must equal the oracle's wherever the oracle's top-1 /
    top-2 language-logit margin exceeds 2 x the measured logits error, and the
    token ids must equal the oracle's up to the first step inside that noise."""
    ctx, path = v3full
    pcm = pcm_clip(0)
    idx = len(ctx.states)
    p = service_params(ctx, temperature_inc=0.0, language=b"auto")
    p.bench_fixed_steps = STEPS
    assert ctx.full(pcm, p, state_index=idx) == 0
    ids = [t.id for s in ctx.segments(idx) for t in s.tokens]
    o = orc.Oracle(path)
    opt = greedy_opt(STEPS)
    opt.language = "auto"
    _, osegs, lang, _ = o.full(pcm, opt)
    oids = [t.id for s in osegs for t in s.tokens]
    n_lang = o.translate - o.sot - 1
    mel, _ = o.mel(pcm)
    k, v = o.cross(o.encode(mel))
    lg_o = o.decode_seq(k, v, [o.sot])[0, o.sot + 1:o.sot + 1 + n_lang]
    ctx.test_encode(pcm, cross=False)  # (mwx_test_decode runs on state 0)
    lg_d = ctx.test_decode([o.sot])[0, o.sot + 1:o.sot + 1 + n_lang]
    lerr = float(np.abs(lg_d - lg_o).max())
    s = np.sort(lg_o)
    lmargin = float(s[-1] - s[-2])
    dlang = ctx.lang_id(idx)
    print(f"full-depth large-v3 language auto: oracle language {lang}, device {dlang}; "
          f"language-logit margin {lmargin:.4f}, err {lerr:.4f}")
    assert lerr < 0.25, lerr
    if lmargin > 2 * lerr:
        assert dlang == lang, (dlang, lang, lmargin, lerr)
    if dlang != lang:
        return  # a near-tie language pick: the windows decode different prompts
    prompt = [o.sot, o.sot + 1 + lang, o.transcribe]
    m = text_margins(o, pcm, prompt, oids, o.eot)
    lg_t = ctx.test_decode(prompt + oids[:-1])[len(prompt) - 1:, :o.eot]
    ref = o.decode_seq(k, v, prompt + oids[:-1])[len(prompt) - 1:, :o.eot]
    err = float(np.abs(lg_t - ref).max())
    first = next((i for i, (a, b) in enumerate(zip(ids, oids)) if a != b), None)
    print(f"  window 0 ({STEPS} steps): logits err {err:.4f}, oracle top-1 margin min "
          f"{m.min():.4f}; ids equal up to step {STEPS if first is None else first}")
    assert len(ids) == len(oids) == STEPS
    if first is not None:
        assert m[first] <= 2 * err, (first, float(m[first]), err)
