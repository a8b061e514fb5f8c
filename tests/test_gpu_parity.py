"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the
same seeded weights and inputs. Tolerances are stated per stage; the full
pipeline is compared token-id for token-id."""
import numpy as np
import pytest

import mwx
import orc

pytestmark = pytest.mark.gpu


def pcm_clip(k=0, seconds=30.0):
    n = int(seconds * 16000)
    return mwx.pcm16_to_f32(mwx.synth_pcm16(k, n))


@pytest.fixture(scope="module")
def micro(make_model):
    path = make_model("micro")
    ctx = mwx.Context.open(path)
    yield ctx, orc.Oracle(path), path
    ctx.close()


# ---------------------------------------------------------------- mel
@pytest.mark.parametrize("arch,seconds", [("micro", 30.0), ("micro-v3", 30.0), ("micro", 2.5),
                                          ("micro", 75.3)])
def test_mel_parity(make_model, arch, seconds):
    path = make_model(arch)
    with mwx.Context.open(path) as ctx:
        pcm = pcm_clip(1, seconds)
        dev = ctx.test_mel(pcm)
    ref, _ = orc.Oracle(path).mel(pcm)
    assert dev.shape == ref.shape
    np.testing.assert_allclose(dev, ref, atol=1e-4, rtol=0)  # north-star tolerance


def test_incremental_mel_equals_fresh(make_model):
    """Streaming re-transcription: a state that saw a
    buffer reuses the raw log-mel of every frame tile whose samples are
    unchanged. A growing 0.5-s-cadence buffer, an edit in the middle, a
    shorter buffer (new stream) and a long one, each bit-identical to the
    log-mel computed on a fresh state, and to the oracle within 1e-4."""
    path = make_model("micro-v3")
    full = pcm_clip(6, 36.0)
    edited = full[:9 * 16000].copy()
    edited[4 * 16000 + 77] += 0.25
    seq = [full[:k * 8000] for k in (1, 2, 3, 4, 9, 10, 11)] + [edited, full[:9 * 16000],
                                                                full[:30 * 16000],
                                                                full[:30 * 16000 + 160 * 7 + 3],
                                                                full[:2 * 16000], full]
    o = orc.Oracle(path)
    with mwx.Context.open(path) as ctx:
        for j, pcm in enumerate(seq):
            inc = ctx.test_mel(pcm, state_index=0)
            fresh = ctx.test_mel(pcm, state_index=1 + j)
            assert np.array_equal(inc, fresh), (j, len(pcm))
            if j in (3, 7, 11):
                ref, _ = o.mel(pcm)
                np.testing.assert_allclose(inc, ref, atol=1e-4, rtol=0)


# ---------------------------------------------------------------- encoder
def test_encoder_and_cross_kv_parity(micro):
    ctx, o, _ = micro
    pcm = pcm_clip(0)
    enc, k, v = ctx.test_encode(pcm)
    mel, _ = o.mel(pcm)
    enc_ref = o.encode(mel)
    k_ref, v_ref = o.cross(enc_ref)
    # encoder output is stored in the weight type (f16): compare at f16 resolution
    err = np.abs(enc - enc_ref).max()
    assert err < 2e-2, err
    assert np.abs(enc - enc_ref).mean() < 1e-3
    assert np.abs(k - k_ref).max() < 3e-2 and np.abs(v - v_ref).max() < 3e-2


def test_decoder_logits_parity(micro):
    ctx, o, _ = micro
    pcm = pcm_clip(0)
    enc, k, v = ctx.test_encode(pcm)
    toks = [o.sot, 300, 1234, o.beg, 777, 40000, 220, o.beg + 37]
    dev = ctx.test_decode(toks)
    ref = o.decode_seq(k, v, toks)  # same cross K/V as the device -> decoder-only comparison
    assert np.abs(dev - ref).max() < 2e-2, np.abs(dev - ref).max()
    assert (dev.argmax(1) == ref.argmax(1)).all()


# ---------------------------------------------------------------- full pipeline
def run_both(ctx, o, pcm, opt: orc.FullOptions, p: mwx.FullParams):
    rc = ctx.full(pcm, p)
    assert rc == 0
    segs = ctx.segments()
    orc_rc, osegs, lang, _ = o.full(pcm, opt)
    assert orc_rc == 0
    return segs, osegs, lang


def service_params(ctx, beam=1, temperature_inc=0.2, language=b"auto"):
    p = ctx.default_params(mwx.SAMPLING_BEAM_SEARCH if beam > 1 else mwx.SAMPLING_GREEDY)
    if beam > 1:
        p.beam_search.beam_size = beam
    p.token_timestamps = True
    p.suppress_nst = True
    p.no_speech_thold = 0.85
    p.entropy_thold = 2.40
    p.logprob_thold = -0.7
    p.temperature = 0.0
    p.temperature_inc = temperature_inc
    # (the service sets best_of for greedy only, src/stt_engine.cpp:235-238)
    p.greedy.best_of = 5 if beam <= 1 else -1
    p.language = language
    return p


def assert_same(segs, osegs, p_tol=5e-3, tid_tie_tol=0.0):
    """Token ids, segment text/times and token timestamps must match exactly;
    token probabilities within p_tol (logits agree to ~1e-2 abs for f16: the
    activations are rounded to 16 bits at the same points, only the f32
    summation order differs; bf16 rounding is 8x coarser).

    `tid` (the most likely timestamp token of each text token, a diagnostic
    field of whisper_token_data the service never reads — it consumes id, p,
    t0, t1: src/stt_engine.cpp:288-296) must match too, except, with
    tid_tie_tol > 0, where both sides picked a timestamp token at the same
    probability within tid_tie_tol: two timestamp tokens tied within the
    logits' rounding noise (weights whose timestamp logits carry no signal)."""
    ids = [t.id for s in segs for t in s.tokens]
    oids = [t.id for s in osegs for t in s.tokens]
    assert ids == oids, next(((i, a, b) for i, (a, b) in enumerate(zip(ids, oids)) if a != b), None)
    assert [(s.t0, s.t1, s.text) for s in segs] == [(s.t0, s.t1, s.text) for s in osegs]
    i = 0
    for sg, osg in zip(segs, osegs):
        # a timestamp tie inside the segment (two timestamp tokens within the
        # rounding noise of the logits: the argmax `tid` differs) feeds
        # whisper_exp_compute_token_level_timestamps a different timestamp
        # anchor, which moves that segment's word times; they are compared
        # only for segments without a tie
        tie = any(t.tid != to.tid for t, to in zip(sg.tokens, osg.tokens))
        for t, to in zip(sg.tokens, osg.tokens):
            assert t.tid == to.tid or abs(t.pt - to.pt) < tid_tie_tol, (i, t, to)
            assert tie or (t.t0, t.t1) == (to.t0, to.t1), (
                f"token {i}: dev t0/t1 {t.t0}/{t.t1} pt {t.pt:.6f} ptsum {t.ptsum:.6f} tid {t.tid} | "
                f"oracle {to.t0}/{to.t1} pt {to.pt:.6f} ptsum {to.ptsum:.6f} tid {to.tid}")
            assert abs(t.p - to.p) < p_tol and abs(t.plog - to.plog) < 2 * p_tol, (i, t, to)
            i += 1


def test_greedy_tokens_match_oracle(micro):
    ctx, o, _ = micro
    pcm = pcm_clip(0)
    opt = orc.FullOptions.service_defaults()
    opt.temperature_inc = 0.0
    segs, osegs, _ = run_both(ctx, o, pcm, opt, service_params(ctx, temperature_inc=0.0))
    assert len(segs) > 0
    assert_same(segs, osegs)


def test_temperature_fallback_matches_oracle(micro):
    """Service defaults: greedy at t=0, then best_of=5 sampled decoders at
    t=0.2, 0.4, ... (std::mt19937 + std::discrete_distribution)."""
    ctx, o, _ = micro
    pcm = pcm_clip(2)
    segs, osegs, _ = run_both(ctx, o, pcm, orc.FullOptions.service_defaults(), service_params(ctx))
    assert_same(segs, osegs)


def test_batch_equals_single(micro):
    ctx, o, _ = micro
    p = service_params(ctx, temperature_inc=0.0, language=b"en")
    pcms = [pcm_clip(k, 30.0 - 4 * k) for k in range(4)]
    singles = []
    for pcm in pcms:
        assert ctx.full(pcm, p) == 0
        singles.append(mwx.token_ids(ctx.segments()))
    assert ctx.full_batch(pcms, p) == 0
    batched = [mwx.token_ids(ctx.segments(i)) for i in range(4)]
    assert batched == singles


def test_multilingual_language_detection(make_model):
    path = make_model("micro-ml")
    o = orc.Oracle(path)
    with mwx.Context.open(path) as ctx:
        pcm = pcm_clip(3)
        opt = orc.FullOptions.service_defaults()
        opt.temperature_inc = 0.0
        segs, osegs, lang = run_both(ctx, o, pcm, opt, service_params(ctx, temperature_inc=0.0))
        assert ctx.lang_id() == lang
        assert_same(segs, osegs)


def test_long_form_multi_window(micro):
    ctx, o, _ = micro
    pcm = pcm_clip(4, 70.0)
    opt = orc.FullOptions.service_defaults()
    opt.temperature_inc = 0.0
    segs, osegs, _ = run_both(ctx, o, pcm, opt, service_params(ctx, temperature_inc=0.0))
    assert_same(segs, osegs)


def test_bf16_model(make_model):
    path = make_model("micro", mwx.GGML_BF16)
    o = orc.Oracle(path)
    with mwx.Context.open(path) as ctx:
        assert ctx.hparam("model_wtype") == mwx.GGML_BF16
        opt = orc.FullOptions.service_defaults()
        opt.temperature_inc = 0.0
        segs, osegs, _ = run_both(ctx, o, pcm_clip(5), opt, service_params(ctx, temperature_inc=0.0))
        assert_same(segs, osegs, p_tol=2e-2)


def test_tiny_en_greedy(make_model):
    path = make_model("tiny.en")
    o = orc.Oracle(path)
    with mwx.Context.open(path) as ctx:
        opt = orc.FullOptions.service_defaults()
        opt.temperature_inc = 0.0
        segs, osegs, _ = run_both(ctx, o, pcm_clip(6), opt, service_params(ctx, temperature_inc=0.0))
        assert_same(segs, osegs)


def test_bench_fixed_steps_workload(micro):
    ctx, o, _ = micro
    p = service_params(ctx, temperature_inc=0.0, language=b"en")
    p.bench_fixed_steps = 40
    assert ctx.full(pcm_clip(0), p) == 0
    assert sum(len(s.tokens) for s in ctx.segments()) == 40


def test_device_resident_input_equals_host_input(micro):
    """mwx_full_batch over PCM already in HBM (mwx_device_buffer) gives the
    same transcripts as over host PCM."""
    ctx, o, _ = micro
    p = service_params(ctx, temperature_inc=0.0, language=b"en")
    pcms = [pcm_clip(30 + k, 6.0 + 3 * k) for k in range(3)]
    assert ctx.full_batch(pcms, p) == 0
    host = [mwx.token_ids(ctx.segments(i)) for i in range(3)]
    bufs = [ctx.upload(x) for x in pcms]
    try:
        assert ctx.full_batch_device(bufs, p) == 0
        dev = [mwx.token_ids(ctx.segments(i)) for i in range(3)]
    finally:
        for b in bufs:
            b.free()
    assert dev == host and all(len(t) > 0 for t in host)


def test_pcm16_input_equals_f32_input(micro):
    """mwx_full_batch_pcm16 (int16 PCM converted on the device, x / 32768)
    gives the transcripts of mwx_full_batch over the host-converted f32 PCM;
    clip lengths not a multiple of 4 exercise the staging offsets."""
    ctx, o, _ = micro
    p = service_params(ctx, temperature_inc=0.0, language=b"en")
    p16 = [mwx.synth_pcm16(40 + k, n=int(16000 * (5.0 + 2.5 * k)) + k) for k in range(3)]
    def toks():
        return [[(t.id, t.p) for s in ctx.segments(i) for t in s.tokens] for i in range(3)]
    assert ctx.full_batch([mwx.pcm16_to_f32(x) for x in p16], p) == 0
    want = toks()
    assert ctx.full_batch_pcm16(p16, p) == 0
    assert toks() == want and all(len(t) > 0 for t in want)


def test_bench_fixed_steps_long_form(micro):
    """Benchmark workload on a long clip: every 30-s window decodes the fixed
    step count, then the clip advances by a whole window (oracle: same rule)."""
    ctx, o, _ = micro
    pcm = pcm_clip(4, 75.0)
    p = service_params(ctx, temperature_inc=0.0, language=b"en")
    p.bench_fixed_steps = 20
    assert ctx.full(pcm, p) == 0
    got = mwx.token_ids(ctx.segments())
    assert len(got) == 3 * 20
    opt = orc.FullOptions.service_defaults()
    opt.temperature_inc = 0.0
    opt.language = "en"
    opt.bench_fixed_steps = 20
    _, osegs, _, _ = o.full(pcm, opt)
    assert got == [t.id for sg in osegs for t in sg.tokens]


def test_fallback_batch_over_64_rows_equals_single(micro):
    """Temperature fallback on 14 clips at once runs 14 x best_of(5) = 70
    decoder rows (row blocks > 64 in every split-K GEMM); each clip must decode
    exactly as when it runs alone (5 rows)."""
    ctx, o, _ = micro
    # decoder 0's std::mt19937 lives in the state (whisper_init_state) and
    # advances with every sampled token, so batch and singles use fresh states
    p = service_params(ctx, language=b"en")
    pcms = [pcm_clip(20 + k, 8.0 + k) for k in range(14)]
    base = len(ctx.states)
    assert ctx.full_batch_states(pcms, p, range(base, base + 14)) == 0
    batched = [mwx.token_ids(ctx.segments(base + i)) for i in range(14)]
    singles = []
    for i, pcm in enumerate(pcms):
        assert ctx.full(pcm, p, state_index=base + 14 + i) == 0
        singles.append(mwx.token_ids(ctx.segments(base + 14 + i)))
    assert batched == singles


# ---------------------------------------------------------------- beam search
def run_fresh(ctx, pcm, p):
    """Run on a state never used before (decoder 0's RNG lives in the state)."""
    idx = len(ctx.states)
    assert ctx.full(pcm, p, state_index=idx) == 0
    return ctx.segments(idx)


@pytest.fixture(scope="module")
def rich(make_model):
    """micro weights whose token loop emits timestamps, segment splits, EOT and
    window seeks (the plain micro model repeats one token for 220 steps)."""
    path = make_model("micro-rich")
    ctx = mwx.Context.open(path)
    yield ctx, orc.Oracle(path), path
    ctx.close()


def test_rich_greedy_matches_oracle(rich):
    ctx, o, _ = rich
    for k in (0, 2):
        pcm = pcm_clip(k)
        opt = orc.FullOptions.service_defaults()
        opt.temperature_inc = 0.0
        opt.language = "en"
        segs = run_fresh(ctx, pcm, service_params(ctx, temperature_inc=0.0, language=b"en"))
        _, osegs, _, windows = o.full(pcm, opt)
        assert len(segs) > 3 and len(windows) > 1  # the token loop is exercised
        assert_same(segs, osegs)


def test_rich_fallback_matches_oracle(rich):
    """Temperature fallback (best_of 5 sampled decoders, std::mt19937 +
    std::discrete_distribution): token for token identical to the oracle's
    whisper_full run on the device's logits (replay); against the oracle's own
    arithmetic the stream agrees until a draw lands within f32 noise of a
    cumulative-probability boundary (the two f32 dot-product orders differ)."""
    ctx, o, _ = rich
    pcm = pcm_clip(3)
    opt = orc.FullOptions.service_defaults()
    opt.language = "en"
    segs = run_fresh(ctx, pcm, service_params(ctx, language=b"en"))
    osegs = replay(ctx, o, pcm, opt)
    assert_same(segs, osegs, p_tol=1e-4)
    _, own, _, _ = o.full(pcm, opt)
    ids = [t.id for sg in segs for t in sg.tokens]
    oids = [t.id for sg in own for t in sg.tokens]
    assert ids[:12] == oids[:12]


@pytest.mark.parametrize("k", [3, 50])
def test_rich_greedy_ladder_matches_oracle_replay(rich, k):
    """Every window walks the whole temperature ladder (logprob_thold above
    any average log-probability): greedy at t = 0, then best_of 5 sampled
    decoders at t = 0.2 .. 1.0, all run ahead on the device since round 6, and
    the window's result kept by whisper.cpp's best_decoder_id rule across the
    attempts. Token for token identical to the oracle's loop on the device's
    logits."""
    ctx, o, _ = rich
    pcm = pcm_clip(k, 14.0)  # (the oracle replays every attempt: 6 per window)
    opt = orc.FullOptions.service_defaults()
    opt.language = "en"
    opt.logprob_thold = 0.5
    p = service_params(ctx, language=b"en")
    p.logprob_thold = 0.5
    idx = len(ctx.states)
    ctx.state(idx)
    ctx.window_counters(idx)
    ctx.runahead_fallbacks(idx)
    assert ctx.full(pcm, p, state_index=idx) == 0
    segs = ctx.segments(idx)
    windows, attempts, _ = ctx.window_counters(idx)
    assert attempts == 6 * windows and ctx.runahead_fallbacks(idx) == 0, (windows, attempts)
    osegs = replay(ctx, o, pcm, opt)
    assert_same(segs, osegs, p_tol=1e-4)
    print(f"clip {k}: {windows} windows x 6 attempts, "
          f"{sum(len(sg.tokens) for sg in segs)} tokens")


def beam_params(ctx, temperature_inc):
    return service_params(ctx, beam=5, temperature_inc=temperature_inc, language=b"en")


def beam_opt(temperature_inc):
    opt = orc.FullOptions.service_defaults(beam_size=5)
    opt.temperature_inc = temperature_inc
    opt.language = "en"
    return opt


def replay(ctx, o, pcm, opt):
    """The oracle's whisper_full logic (logits rules, draws, beam ranking,
    fallback, segments) run on logits the device computes for each prefix
    (teacher-forced through the C ABI): isolates the token-loop logic from the
    f16 noise of the logits, which can reorder beam hypotheses whose summed
    log-probs differ by less than ~1e-2."""
    idx = len(ctx.states)
    ctx.state(idx)

    def enc(seek):
        ctx.test_encode(pcm, seek=seek, cross=False, state_index=idx)

    def logits(tokens):
        return ctx.test_decode_last(tokens, state_index=idx)

    _, segs, _, _ = o.full_external(pcm, opt, enc, logits)
    return segs


@pytest.mark.parametrize("temperature_inc", [0.0, 0.2])
def test_beam_search_replay_exact(rich, temperature_inc):
    """The service default (src/config.h:52): beam_size 5 -> whisper.cpp beam
    search (beam_size draws per decoder, candidates sorted by
    sum_logprobs_all, de-duplicated, KV caches handed over between decoders),
    with and without temperature fallback: token for token identical to the
    oracle's beam search run on the device's logits."""
    ctx, o, _ = rich
    pcm = pcm_clip(0, 14.0)
    segs = run_fresh(ctx, pcm, beam_params(ctx, temperature_inc))
    osegs = replay(ctx, o, pcm, beam_opt(temperature_inc))
    assert len(segs) > 1
    assert_same(segs, osegs, p_tol=1e-4)


def test_beam_search_replay_exact_split_k(make_model):
    """As above on tiny.en shapes (d 384: the decoder projections run split-K
    with 3 slabs, so the grouped cross-attention / remapped self-attention
    reduce multi-slab queries)."""
    path = make_model("tiny.en-rich")
    o = orc.Oracle(path)
    with mwx.Context.open(path) as ctx:
        pcm = pcm_clip(2, 30.0)  # (oracle: 5 segments, 4 windows)
        segs = run_fresh(ctx, pcm, beam_params(ctx, 0.0))
        osegs = replay(ctx, o, pcm, beam_opt(0.0))
        assert len(segs) >= 3
        assert_same(segs, osegs, p_tol=1e-4)


def test_beam_search_tracks_oracle(rich):
    """Against the oracle's own arithmetic: the first tokens agree until two
    hypotheses come within float noise of each other."""
    ctx, o, _ = rich
    pcm = pcm_clip(0)
    segs = run_fresh(ctx, pcm, beam_params(ctx, 0.0))
    _, osegs, _, _ = o.full(pcm, beam_opt(0.0))
    ids = [t.id for s in segs for t in s.tokens]
    oids = [t.id for s in osegs for t in s.tokens]
    assert ids[:12] == oids[:12]


def test_beam_search_batch_equals_single(rich):
    ctx, o, _ = rich
    p = service_params(ctx, beam=5, language=b"en")
    pcms = [pcm_clip(30 + k, 12.0 + 5 * k) for k in range(3)]
    base = len(ctx.states)
    assert ctx.full_batch_states(pcms, p, range(base, base + 3)) == 0
    batched = [mwx.token_ids(ctx.segments(base + i)) for i in range(3)]
    singles = [mwx.token_ids(run_fresh(ctx, pcm, p)) for pcm in pcms]
    assert batched == singles


# ---------------------------------------------------------------- quantized files
@pytest.mark.parametrize("qname", ["q5_0", "q8_0", "q4_1"])
def test_quantized_model_greedy_matches_oracle(make_model, qname):
    """whisper.cpp quantize-tool files (block formats dequantized at load, f16
    compute): tokens, timestamps and probabilities against the oracle reading
    the same file."""
    path = make_model("micro-rich", mwx.GGML_QUANT_TYPES[qname])
    o = orc.Oracle(path)
    with mwx.Context.open(path) as ctx:
        pcm = pcm_clip(0)
        opt = orc.FullOptions.service_defaults()
        opt.temperature_inc = 0.0
        opt.language = "en"
        segs = run_fresh(ctx, pcm, service_params(ctx, temperature_inc=0.0, language=b"en"))
        _, osegs, _, windows = o.full(pcm, opt)
        assert len(segs) > 3 and len(windows) > 1
        assert_same(segs, osegs)


def decision_margins(lg, eot, beg):
    """per position: the smaller of |log-sum-exp of the timestamp log-probs -
    max text log-prob| (whisper.cpp's timestamp-vs-text rule) and the top-2
    logit gap over text and timestamp tokens (the argmax); a decision whose
    margin is within the logits' rounding noise may go either way"""
    x = lg.astype(np.float64)
    m = x.max(axis=1, keepdims=True)
    lp = x - (m + np.log(np.exp(x - m).sum(axis=1, keepdims=True)))
    ts = np.logaddexp.reduce(lp[:, beg:], axis=1)
    tx = lp[:, :eot].max(axis=1)
    cand = np.concatenate([x[:, :eot], x[:, beg:]], axis=1)
    top2 = np.sort(cand, axis=1)[:, -2:]
    return np.minimum(np.abs(ts - tx), top2[:, 1] - top2[:, 0])


@pytest.mark.parametrize("qname", ["q2_k", "q3_k", "q4_k", "q5_k", "q6_k"])
def test_k_quantized_model_greedy_matches_oracle(make_model, qname):
    """256-element K super-block files (q2_K .. q6_K; micro256: rows of 256,
    the smallest geometry ggml can K-quantize), dequantized at load and
    computed in f16, against the oracle reading the same file (its own
    per-element restatement of the blocks). The coarse K codes leave the
    -rich weights' timestamp and text logits close (q3_K on this clip: a
    timestamp-vs-text decision 0.0019 apart, oracle-computed), so the check is
    the chain: (1) the device's token loop is token-for-token the oracle's
    loop run on the device's logits; (2) the device's teacher-forced logits
    over the oracle's first window agree with the oracle's within err; (3) the
    oracle's own window tokens equal those of its loop on the device's logits
    up to the first decision whose oracle margin is within 2 err (everything
    after it follows a tie)."""
    path = make_model("micro256-rich", mwx.GGML_QUANT_TYPES[qname])
    o = orc.Oracle(path)
    with mwx.Context.open(path) as ctx:
        pcm = pcm_clip(0)
        opt = orc.FullOptions.service_defaults()
        opt.temperature_inc = 0.0
        opt.language = "en"
        segs = run_fresh(ctx, pcm, service_params(ctx, temperature_inc=0.0, language=b"en"))
        _, osegs, _, owin = o.full(pcm, opt)
        # (q2_K's 2-bit codes leave the -rich weights little to say: 2 segments)
        assert len(segs) >= (2 if qname == "q2_k" else 20) and len(owin) > 1
        idx = 1
        ctx.state(idx)
        calls = []

        def enc(seek):
            ctx.test_encode(pcm, seek=seek, cross=False, state_index=idx)

        def logits(tokens):
            calls.append(list(tokens))
            return ctx.test_decode_last(tokens, state_index=idx)

        _, rsegs, _, rwin = o.full_external(pcm, opt, enc, logits)
        assert_same(segs, rsegs, p_tol=1e-4)                          # (1)
        if rwin == owin:
            assert_same(segs, osegs)
            return
        prompt = calls[0]  # window 0's prompt (sot, language, task)
        seq = prompt + owin[0]
        mel, _ = o.mel(pcm)
        k, v = o.cross(o.encode(mel, 0))
        lo = o.decode_seq(k, v, seq)[len(prompt) - 1:-1]  # logits that chose owin[0]
        ctx.test_encode(pcm, seek=0, cross=False)
        ld = ctx.test_decode(seq)[len(prompt) - 1:-1]
        err = float(np.abs(ld - lo).max())
        assert err < 5e-2, err                                         # (2)
        tie = decision_margins(lo, ctx.token("eot"), ctx.token("beg")) < 2 * err
        assert tie.any(), "window tokens differ without a near-tie in window 0"
        t = int(np.argmax(tie))
        assert rwin[0][:t] == owin[0][:t], (t, rwin[0][:t + 2], owin[0][:t + 2])  # (3)


def np_discrete_draws(probs, u, ndraw):
    """libstdc++ std::discrete_distribution<int>(w.begin(), w.end()) then
    operator()(rng) with generate_canonical value u: S = sequential double sum,
    p_i = w_i / S, cp = sequential partial sums, cp[-1] = 1, lower_bound."""
    out = np.zeros(u.shape, np.int32)
    for r in range(probs.shape[0]):
        w = probs[r].astype(np.float64)
        S = np.cumsum(w)[-1]
        cp = np.cumsum(w / S)
        cp[-1] = 1.0
        out[r, :ndraw[r]] = np.searchsorted(cp, u[r, :ndraw[r]], side="left")
    return out


def test_sample_draws_kernels_match_libstdcxx_rule(micro):
    """Both draw kernels (fast parallel path with its margin fallback, and the
    sequential one) against a numpy restatement of libstdc++'s
    discrete_distribution, on flat and peaked rows at the large-v3 vocabulary
    size; u values placed exactly on cumulative values hit the fallback."""
    ctx, _, _ = micro
    rng = np.random.default_rng(5)
    R, V, KD = 96, 51866, 5
    logits = rng.normal(0, 1, (R, V)) * np.linspace(0.5, 12.0, R)[:, None]
    pr = np.exp(logits - logits.max(axis=1, keepdims=True))
    pr = (pr / pr.sum(axis=1, keepdims=True)).astype(np.float32)
    lp = np.log(np.maximum(pr, 1e-30)).astype(np.float32)
    u = rng.random((R, KD))
    for r in range(0, R, 7):  # on a cumulative value: the margin test must defer
        w = pr[r].astype(np.float64)
        cp = np.cumsum(w / np.cumsum(w)[-1])
        u[r, 0] = cp[rng.integers(V - 1)]
    nd = rng.integers(0, KD + 1, R).astype(np.int32)
    nd[:4] = KD
    want = np_discrete_draws(pr, u, nd)
    mask = np.arange(KD)[None, :] < nd[:, None]
    for exact in (False, True):
        ids, us = ctx.test_sample_draws(pr, lp, u, nd, exact=exact, reps=20)
        np.testing.assert_array_equal(np.where(mask, ids, 0), want)
        print(f"draws exact={exact}: {us:.1f} us per launch ({R} rows x {V})")


def test_draws_fast_path_equals_sequential(rich, monkeypatch):
    """The parallel draw kernel (margin-checked) and the sequential
    libstdc++-order kernel give identical beam search / fallback results."""
    import subprocess, sys, os, json
    code = r'''
import json, sys
sys.path.insert(0, "sentiric-stt-whisper-service_amd")
import mwx
path = sys.argv[1]
ctx = mwx.Context.open(path)
out = []
for k, beam in ((0, True), (3, False)):
    pcm = mwx.pcm16_to_f32(mwx.synth_pcm16(k, 30 * 16000))
    p = ctx.default_params(mwx.SAMPLING_BEAM_SEARCH if beam else mwx.SAMPLING_GREEDY)
    p.language = b"en"
    if not beam:
        p.temperature = 0.4
    assert ctx.full(pcm, p, state_index=len(ctx.states)) == 0
    out.append(mwx.token_ids(ctx.segments(len(ctx.states) - 1)))
print(json.dumps(out))
'''
    _, _, path = rich
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = []
    for exact in (False, True):
        env = dict(os.environ)
        env.pop("MWX_DRAW_EXACT", None)
        if exact:
            env["MWX_DRAW_EXACT"] = "1"
        r = subprocess.run([sys.executable, "-c", code, path], cwd=root, env=env,
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        res.append(json.loads(r.stdout.strip().splitlines()[-1]))
    assert res[0] == res[1]
    assert all(len(t) > 0 for t in res[0])


# ---------------------------------------------------------------- MX-fp8 compute mode
def _bf16(x):
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16 << 16
    return u.astype(np.uint32).view(np.float32)


def test_mx_gemm_exact(micro):
    """One block-scaled fp8 MFMA GEMM (device activation quantizer, host
    weight quantizer, v_mfma_scale_f32_16x16x128_f8f6f4 operand / scale
    layout) against float64 products of the same MX-rounded operands: only
    f32 accumulation error remains. Shapes cover partial 256-row/column tiles."""
    from test_quant_format import np_mx_round
    ctx, _, _ = micro
    rng = np.random.default_rng(5)
    for M, N, K in ((300, 260, 256), (64, 512, 1280)):
        a = rng.standard_normal((M, K)).astype(np.float32) * rng.uniform(0.01, 10, (M, 1)).astype(np.float32)
        w = rng.standard_normal((N, K)).astype(np.float32) * 0.05
        c = ctx.test_gemm_mx(a, w)
        aq = np_mx_round(_bf16(a)).reshape(M, K).astype(np.float64)
        wq = np_mx_round(_bf16(w)).reshape(N, K).astype(np.float64)
        ref = aq @ wq.T
        scale = np.abs(aq) @ np.abs(wq).T
        err = np.abs(c - ref) / (scale + 1e-30)
        # (observed <= 1.4e-5: the block-scaled MFMA's internal accumulation
        # is not a plain f32 fma chain)
        assert err.max() < 5e-5, (M, N, K, err.max())
        assert err.mean() < 2e-6, (M, N, K, err.mean())


def test_gemm_gelu_table_equals_tanhf(micro):
    """The encoder FFN1 GEMM's GELU epilogue by the f16 table in LDS (the
    engine's path) gives exactly the outputs of evaluating gelu_ggml (tanhf)
    per output, for f16 and bf16 operands; pre-activations spread over
    [-14, 14] cover the +-10 saturation edges and every f16 exponent in between.
    Partial 256-row tiles included. A float64 GELU of the float64 product
    bounds both (16-bit output rounding + the f16 input rounding)."""
    ctx, _, _ = micro
    rng = np.random.default_rng(11)
    M, N, K = 300, 512, 256
    a = rng.standard_normal((M, K)).astype(np.float32) * rng.uniform(0.001, 1.0, (M, 1)).astype(np.float32)
    w = rng.standard_normal((N, K)).astype(np.float32) * 0.06
    bias = rng.uniform(-12, 12, N).astype(np.float32)
    for bf16 in (False, True):
        t = ctx.test_gemm_gelu(a, w, bias, bf16, True)
        d = ctx.test_gemm_gelu(a, w, bias, bf16, False)
        assert np.array_equal(t.view(np.uint32), d.view(np.uint32)), (bf16, np.abs(t - d).max())
        rnd = _bf16 if bf16 else (lambda x: x.astype(np.float16).astype(np.float32))
        x = rnd(a).astype(np.float64) @ rnd(w).astype(np.float64).T + bias
        g = 0.5 * x * (1 + np.tanh(np.sqrt(2 / np.pi) * x * (1 + 0.044715 * x * x)))
        g = np.where(x <= -10, 0.0, np.where(x >= 10, x, g))
        assert (np.abs(x) > 10).mean() > 0.05 and (np.abs(x) < 1).mean() > 0.05
        err = np.abs(t - g) / np.maximum(np.abs(g), 1e-3)
        assert err.max() < 2e-2, (bf16, err.max())


def test_mxfp8_encoder_matches_mx_oracle(make_model):
    """MWX_COMPUTE_MXFP8: encoder and cross-K/V GEMMs on block-scaled fp8 MFMA.
    The oracle's ORC_MXFP8 mode applies the same MX rounding to the same
    operands. fp8 re-rounding amplifies tiny differences: the oracle itself
    moves by 0.016 mean abs when its mel input is perturbed by 1e-5 (0.0015 in
    16-bit mode), so the bar is that noise level, and the device must be
    clearly closer to the MX oracle than to the 16-bit one."""
    path = make_model("micro", mwx.GGML_BF16)
    pcm = pcm_clip(0)
    with mwx.Context.open(path, compute=mwx.COMPUTE_MXFP8) as ctx:
        enc, k, v = ctx.test_encode(pcm)
    omx, o16 = orc.Oracle(path, mxfp8=True), orc.Oracle(path)
    mel, _ = omx.mel(pcm)
    ref = omx.encode(mel)
    ref16 = o16.encode(mel)
    k_ref, v_ref = omx.cross(ref)
    d_mx = np.abs(enc - ref)
    d_16 = np.abs(enc - ref16)
    assert d_mx.mean() < 0.6 * d_16.mean(), (d_mx.mean(), d_16.mean())
    assert d_mx.mean() < 0.03 and d_mx.max() < 0.5, (d_mx.mean(), d_mx.max())
    k16, v16 = o16.cross(ref16)
    for got, want, want16 in ((k, k_ref, k16), (v, v_ref, v16)):
        assert np.abs(got - want).mean() < 0.6 * np.abs(got - want16).mean()


def test_mxfp8_greedy_tokens_track_mx_oracle(make_model):
    """fp8 mode end to end: the token stream agrees with the MX oracle's until
    fp8 re-rounding noise (see above) first reorders two close logits."""
    path = make_model("micro-rich", mwx.GGML_BF16)
    o = orc.Oracle(path, mxfp8=True)
    with mwx.Context.open(path, compute=mwx.COMPUTE_MXFP8) as ctx:
        pcm = pcm_clip(0)
        opt = orc.FullOptions.service_defaults()
        opt.temperature_inc = 0.0
        opt.language = "en"
        segs = run_fresh(ctx, pcm, service_params(ctx, temperature_inc=0.0, language=b"en"))
        _, osegs, _, windows = o.full(pcm, opt)
        assert len(segs) > 3 and len(windows) > 1
        ids = [t.id for sg in segs for t in sg.tokens]
        oids = [t.id for sg in osegs for t in sg.tokens]
        assert ids[:16] == oids[:16]


def test_mxfp8_decoder_logits_match_mx_oracle(make_model):
    """MWX_COMPUTE_MXFP8 decoder: MX-fp8 decoder weights and tied embedding
    (dequantized in registers, bf16 MFMA) over the MX-fp8 cross K/V cache.
    Teacher-forced logits against the oracle's ORC_MXFP8 decoder on the same
    (device) cross K/V — a decoder-only comparison — and the device cache
    against the MX oracle's cross K/V."""
    path = make_model("micro-rich", mwx.GGML_BF16)
    pcm = pcm_clip(0)
    with mwx.Context.open(path, compute=mwx.COMPUTE_MXFP8) as ctx:
        enc, k, v = ctx.test_encode(pcm)
        omx = orc.Oracle(path, mxfp8=True)
        toks = [omx.sot, 300, 1234, omx.beg, 777, 40000, 220, omx.beg + 37]
        dev = ctx.test_decode(toks)
    ref = omx.decode_seq(k, v, toks)
    o16 = orc.Oracle(path)
    ref16 = o16.decode_seq(k, v, toks)  # 16-bit decoder weights on the same K/V
    err, err16 = np.abs(dev - ref).max(), np.abs(dev - ref16).max()
    assert err < 0.15, err
    assert err < 0.5 * err16, (err, err16)  # the device runs the fp8 weights
    assert (dev.argmax(1) == ref.argmax(1)).all()
    # cache: every value is an MX-fp8 value (code x 2^e, e per 32-block) and
    # tracks the MX oracle's rounding of its own K/V
    mel, _ = omx.mel(pcm)
    k_ref, v_ref = omx.cross(omx.encode(mel))
    for got, want in ((k, k_ref), (v, v_ref)):
        d = np.abs(got - want)
        assert d.mean() < 0.05 * np.abs(want).mean(), (d.mean(), np.abs(want).mean())


def test_mxfp8_batch_equals_single(make_model):
    """fp8 mode (fp8 decoder weights, fp8 cross cache read by the grouped
    kernel at one row per clip): a batch decodes each clip as alone."""
    path = make_model("micro-rich", mwx.GGML_BF16)
    with mwx.Context.open(path, compute=mwx.COMPUTE_MXFP8) as ctx:
        p = service_params(ctx, temperature_inc=0.0, language=b"en")
        pcms = [pcm_clip(50 + k, 10.0 + 4 * k) for k in range(5)]
        assert ctx.full_batch_states(pcms, p, range(5)) == 0
        batched = [mwx.token_ids(ctx.segments(i)) for i in range(5)]
        singles = [mwx.token_ids(run_fresh(ctx, pcm, p)) for pcm in pcms]
    assert batched == singles and all(len(t) > 0 for t in batched)


_RUN_MODES = r'''
import json, sys
sys.path.insert(0, "sentiric-stt-whisper-service_amd")
import mwx
path, max_tokens, inc = sys.argv[1], int(sys.argv[2]), float(sys.argv[3])
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
p.max_tokens = max_tokens
secs = [30.0, 75.3, 12.5, 48.0, 3.0, 30.0]
pcms = [mwx.pcm16_to_f32(mwx.synth_pcm16(k, int(s * 16000))) for k, s in enumerate(secs)]
assert ctx.full_batch(pcms, p) == 0
out = [[[s.t0, s.t1, s.text, [(t.id, t.tid, t.p, t.t0, t.t1) for t in s.tokens]]
        for s in ctx.segments(i)] for i in range(len(pcms))]
print(json.dumps([out, ctx.window_counters(0)[:2], ctx.runahead_fallbacks(0)]))
'''


@pytest.mark.parametrize("max_tokens,inc", [(0, 0.0), (0, 0.2), (7, 0.0)])
def test_runahead_decode_equals_synchronous_loop(make_model, max_tokens, inc):
    """Run-ahead greedy decoding (the device applies the token loop's stop and
    next-input rules after each step, the host reads step k while step k+1
    runs) gives exactly the host-driven loop's results (MWX_NO_RUNAHEAD=1):
    six clips of 3-75 s (long-form seeks, timestamps, EOT), the fallback
    re-decodes (best-of-5 temperature sampling, run ahead too since round 6:
    each row's token is its device draw, its uniforms come from the ring the
    host fills from a copy of its RNG), and the max_tokens stop."""
    import json
    import os
    import subprocess
    import sys
    path = make_model("micro-rich")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = []
    for extra in ({}, {"MWX_NO_RUNAHEAD": "1"}):
        env = dict(os.environ)
        env.update(extra)
        r = subprocess.run([sys.executable, "-c", _RUN_MODES, path, str(max_tokens), str(inc)],
                           cwd=root, env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        res.append(json.loads(r.stdout.strip().splitlines()[-1]))
    (out_ra, (windows, attempts), redos), (out_host, _, _) = res
    print("windows", windows, "attempts", attempts, "run-ahead redos", redos)
    assert redos == 0  # (a redo would run the host loop: the comparison would be vacuous)
    assert inc == 0.0 or attempts > windows  # temperature fallback attempts ran
    assert out_ra == out_host
    assert sum(len(s[3]) for c in out_ra for s in c) > 40


@pytest.mark.parametrize("temperature_inc,best_of", [(0.0, 5), (0.2, 5), (0.2, -1)])
def test_beam_runahead_equals_host_loop(rich, temperature_inc, best_of, monkeypatch):
    """Beam search run ahead on the device (beam_advance_kernel: ranking,
    dedup, decoder hand-over and KV maps, the next step's inputs and uniforms)
    == the host loop (MWX_NO_RUNAHEAD: beam_step on the host, one round trip
    per step): every clip's token records bit for bit, 4 clips in one batch.
    With fallback, the attempts at t > 0 (beam search over best_of decoders
    drawing from the temperature-scaled probs; run ahead since round 6) draw
    from RNG streams the earlier attempts consumed from their uniform rings.
    best_of = -1 is what the service runs (src/stt_engine.cpp:235-238 sets
    best_of for greedy only: one decoder at t > 0). These clips pass at t = 0,
    so the t > 0 cases raise logprob_thold above any average log-probability:
    every window walks the whole ladder 0.0 -> 1.0."""
    ctx, _, _ = rich
    p = beam_params(ctx, temperature_inc)
    p.greedy.best_of = best_of
    if temperature_inc > 0.0:
        p.logprob_thold = 0.5
    pcms = [pcm_clip(40 + k, 10.0 + 7 * k) for k in range(4)]

    def run():
        base = len(ctx.states)
        for i in range(4):
            ctx.state(base + i)
        ctx.window_counters(base)
        ctx.runahead_fallbacks(base)
        assert ctx.full_batch_states(pcms, p, range(base, base + 4)) == 0
        return ([ctx.token_records(base + i) for i in range(4)], ctx.window_counters(base)[:2],
                ctx.runahead_fallbacks(base))

    ra, (windows, attempts), redos = run()
    monkeypatch.setenv("MWX_NO_RUNAHEAD", "1")
    host, _, _ = run()
    print("tokens per clip:", [len(x) for x in ra], "windows", windows, "attempts", attempts)
    assert redos == 0
    assert temperature_inc == 0.0 or attempts > windows
    assert sum(len(x) for x in ra) > 20
    assert ra == host


@pytest.mark.parametrize("beam,fault_step,ladder", [(5, 0, False), (5, 3, False), (1, 2, False),
                                                    (5, 2, True), (1, 2, True)])
def test_runahead_mismatch_falls_back_to_host_loop(rich, beam, fault_step, ladder, monkeypatch):
    """A disagreement between the device's run-ahead advance and the host's
    replay (forced at run-ahead step `fault_step` by mwx_test_set_ra_mismatch)
    does not fail the request: the attempt is redone on the host-driven loop
    and the batch's token records equal a run on the host loop throughout
    (beam 5, the service default, and greedy). `ladder`: every window walks
    the whole temperature ladder (logprob_thold raised), so the faulted
    attempts include the sampling ones, whose redo must draw the uniforms the
    run-ahead did not consume (the rows' RNGs advance only once an attempt's
    loop has finished)."""
    ctx, _, _ = rich
    p = service_params(ctx, beam=beam, temperature_inc=0.2 if ladder else 0.0, language=b"en")
    if ladder:
        p.logprob_thold = 0.5
    pcms = [pcm_clip(60 + k, 11.0 + 6 * k) for k in range(3)]

    def run():
        base = len(ctx.states)
        for i in range(3):
            ctx.state(base + i)
        ctx.runahead_fallbacks(base)
        assert ctx.full_batch_states(pcms, p, range(base, base + 3)) == 0
        return [ctx.token_records(base + i) for i in range(3)], ctx.runahead_fallbacks(base)

    monkeypatch.setenv("MWX_NO_RUNAHEAD", "1")
    host, n0 = run()
    monkeypatch.delenv("MWX_NO_RUNAHEAD")
    mwx.set_ra_mismatch(fault_step)
    try:
        redone, n1 = run()
    finally:
        mwx.set_ra_mismatch(-1)
    print(f"beam {beam}, fault at step {fault_step}: {n1} attempt(s) redone on the host loop, "
          f"{sum(len(x) for x in host)} tokens")
    assert n0 == 0 and n1 >= 1
    assert redone == host


def _e4m3_encode(v):
    """e4m3fn codes (nearest even; |v| <= 448) of float64 values."""
    a = np.abs(v)
    sub = a < 2.0 ** -6
    e = np.floor(np.log2(np.where(sub, 1.0, a))).astype(np.int64)
    m = np.where(sub, np.rint(a / 2.0 ** -9), np.rint(a / np.ldexp(1.0, e - 3)) - 8)
    # rounding up to the next binade
    up = ~sub & (m == 8)
    e = np.where(up, e + 1, e)
    m = np.where(up, 0, m)
    sub_to_norm = sub & (m == 8)
    code = np.where(sub & ~sub_to_norm, m, 0) + np.where(sub_to_norm, 1 << 3, 0)
    code = np.where(sub, code, ((e + 7) << 3) + m)
    return (code.astype(np.int64) | np.where(v < 0, 0x80, 0)).astype(np.uint8)


def _e4m3_decode(c):
    c = c.astype(np.int64)
    s = np.where(c & 0x80, -1.0, 1.0)
    e, m = (c >> 3) & 15, c & 7
    return s * np.where(e == 0, m / 8.0 * 2.0 ** -6, (1.0 + m / 8.0) * np.ldexp(1.0, e - 7))


def _mx_rows(x):
    """x [..., 64] -> (codes uint8 [..., 64], E8M0 scales uint8 [..., 2], the
    dequantized float64 values): one power-of-two scale per 32-element half,
    the smallest 2^E with max |x| <= 448 * 2^E."""
    h = x.reshape(*x.shape[:-1], 2, 32).astype(np.float64)
    amax = np.abs(h).max(axis=-1, keepdims=True)
    E = np.ceil(np.log2(np.maximum(amax, 1e-30) / 448.0))
    codes = _e4m3_encode(h / np.ldexp(1.0, E.astype(np.int64)))
    deq = _e4m3_decode(codes) * np.ldexp(1.0, E.astype(np.int64))
    return (codes.reshape(x.shape), (E[..., 0] + 127).astype(np.uint8),
            deq.reshape(x.shape))


@pytest.mark.parametrize("sharp", [False, True])
def test_mx_cross_attention_kernel_vs_f64(micro, sharp):
    """The MX-fp8 grouped cross-attention kernel (the C5 cross-attention) on
    K / V with large-v3-like MX scale ranges (per-row magnitudes spread over
    2^-12 .. 2^-2 scales) and 1500 keys, against float64 attention over the
    same dequantized values and f16-rounded queries. Diffuse softmax (weights
    ~1/1500: the case where folding the V scale into an f16 P underflowed) and
    peaked softmax. Bound: max |o - o64| <= 3e-3 x max |o64| per row, for both
    the MFMA (default) and the v_dot2 path, and MFMA error <= 1.5 x v_dot2's +
    1e-4 x max |o64|."""
    ctx, _, _ = micro
    rng = np.random.default_rng(7 if sharp else 3)
    H, n, nq, G = 2, 1500, 5, 2
    R = G * nq
    rowscale = np.exp2(rng.uniform(-5, 3, size=(G, H, n, 1)))
    k = rng.standard_normal((G, H, n, 64)) * 0.35 * rowscale
    v = rng.standard_normal((G, H, n, 64)) * rowscale
    k8, ks, kd = _mx_rows(k)
    v8, vs, vd = _mx_rows(v)
    q = (rng.standard_normal((R, H * 64)) * (3.0 if sharp else 0.02)).astype(np.float32)
    qh = q.astype(np.float16).astype(np.float64)
    scale = 64.0 ** -0.25
    ref = np.empty((R, H * 64))
    for r in range(R):
        g = r // nq
        for h in range(H):
            s = kd[g, h] @ qh[r, h * 64:(h + 1) * 64] * scale
            p = np.exp(s - s.max())
            p /= p.sum()
            ref[r, h * 64:(h + 1) * 64] = p @ vd[g, h]
    errs = {}
    prev = mwx.set_xattn_mfs(True)
    try:
        for mfs in (True, False):
            mwx.set_xattn_mfs(mfs)
            o = ctx.test_xattn_mx(q, k8, ks, v8, vs, nq)
            scale_r = np.abs(ref).max(axis=1, keepdims=True)
            errs[mfs] = float((np.abs(o - ref) / scale_r).max())
    finally:
        mwx.set_xattn_mfs(None if prev < 0 else bool(prev))
    print(f"MX cross-attention vs f64 ({'peaked' if sharp else 'diffuse'}): "
          f"MFMA {errs[True]:.2e}, v_dot2 {errs[False]:.2e} (of max |o| per row)")
    assert errs[True] <= 3e-3 and errs[False] <= 3e-3, errs
    assert errs[True] <= 1.5 * errs[False] + 1e-4, errs



def test_mx_cache_widening_pinned(micro):
    """The MX-fp8 cross K/V cache's widening to f16 (v_cvt_scalef32_pk_f16_fp8,
    both cross-attention paths) for every finite e4m3 code under E8M0
    exponents 2^-37 .. 2^13: equal to code x 2^E rounded to f16 with
    round-to-nearest-even wherever that is within f16's range (normal or
    subnormal, flushed nowhere: r06c measured 12630 values, 5678 of them
    subnormal, 2942 rounding to 0), and +-inf beyond it (no saturation). Pins
    what 'exact while code x scale is f16-representable' means."""
    ctx, _, _ = micro
    codes = np.array([c for c in range(256) if (c & 0x7F) != 0x7F], np.uint8)  # finite codes
    vals = _e4m3_decode(codes.astype(np.int64))
    exps = np.arange(127 - 37, 127 + 14)
    n = len(codes)
    pad = (-n) % 8
    cg = np.concatenate([codes, np.zeros(pad, np.uint8)])
    allc = np.tile(cg, len(exps))
    alle = np.repeat(exps.astype(np.uint8), len(cg) // 8)
    dev = ctx.test_mx_widen(allc, alle).astype(np.float64).reshape(len(exps), -1)[:, :n]
    want = (vals[None, :] * np.exp2(exps[:, None] - 127.0))
    rne = want.astype(np.float16).astype(np.float64)
    ok = np.abs(want) <= 65504.0
    assert np.array_equal(dev[ok], rne[ok]), np.argwhere((dev != rne) & ok)[:8]
    sub = ok & (np.abs(want) < 2.0 ** -14) & (want != 0)
    big = ~ok
    assert np.all(np.isinf(dev[big])) and np.array_equal(np.sign(dev[big]), np.sign(want[big]))
    print(f"MX widening: {int(ok.sum())} representable values equal to f16 RNE "
          f"({int(sub.sum())} of them f16 subnormals, {int((sub & (rne == 0)).sum())} rounding to 0); "
          f"beyond f16's range: {sorted(set(np.abs(dev[big]).tolist()))[:4]}")


def test_mx_cross_attention_kernel_extreme_scales(micro):
    """Block scales at the edge of f16's range: V rows whose
    code x scale values fall into f16's subnormal range (row magnitudes
    2^-22 .. 2^-14). Both kernel paths widen the codes to f16 before the
    arithmetic, so the pinned behaviour is attention over the f16-ROUNDED
    dequantized values with f16 subnormals kept (a flush to zero would lose
    whole rows): for the MFMA and the v_dot2 path alike, max |o - o64| per row
    within one f16 subnormal step (2^-24, the output is f16 here and lies in
    that range itself) + 3e-3 x max |o64|, o64 = float64 attention over
    np.float16(values); the distance to the unrounded values is printed.
    (Measured first at a relative bound alone: 1.3e-2, the output's own f16
    subnormal rounding.)"""
    ctx, _, _ = micro
    rng = np.random.default_rng(11)
    H, n, nq, G = 2, 1500, 5, 2
    R = G * nq
    k = rng.standard_normal((G, H, n, 64)) * 0.35 * np.exp2(rng.uniform(-5, 3, size=(G, H, n, 1)))
    v = rng.standard_normal((G, H, n, 64)) * np.exp2(rng.uniform(-22, -14, size=(G, H, n, 1)))
    k8, ks, kd = _mx_rows(k)
    v8, vs, vd = _mx_rows(v)
    vd16 = vd.astype(np.float16).astype(np.float64)
    assert (np.abs(vd) < 2.0 ** -14).mean() > 0.5  # mostly f16 subnormals
    q = (rng.standard_normal((R, H * 64)) * 0.5).astype(np.float32)
    qh = q.astype(np.float16).astype(np.float64)
    scale = 64.0 ** -0.25
    ref, ref_exact = np.empty((R, H * 64)), np.empty((R, H * 64))
    for r in range(R):
        g = r // nq
        for h in range(H):
            sc = kd[g, h] @ qh[r, h * 64:(h + 1) * 64] * scale
            p = np.exp(sc - sc.max())
            p /= p.sum()
            ref[r, h * 64:(h + 1) * 64] = p @ vd16[g, h]
            ref_exact[r, h * 64:(h + 1) * 64] = p @ vd[g, h]
    errs, exact = {}, {}
    prev = mwx.set_xattn_mfs(True)
    try:
        for mfs in (True, False):
            mwx.set_xattn_mfs(mfs)
            o = ctx.test_xattn_mx(q, k8, ks, v8, vs, nq)
            bound = 2.0 ** -24 + 3e-3 * np.abs(ref).max(axis=1, keepdims=True)
            errs[mfs] = float((np.abs(o - ref) / bound).max())
            exact[mfs] = float((np.abs(o - ref_exact) / bound).max())
    finally:
        mwx.set_xattn_mfs(None if prev < 0 else bool(prev))
    print(f"MX cross-attention, V in f16's subnormal range: max |o - o64| / (2^-24 + 3e-3 max|o64|) "
          f"vs f16-rounded values MFMA {errs[True]:.3f} / v_dot2 {errs[False]:.3f}; vs unrounded "
          f"MFMA {exact[True]:.3f} / v_dot2 {exact[False]:.3f}")
    assert errs[True] <= 1.0 and errs[False] <= 1.0, (errs, exact)


@pytest.mark.parametrize("M,N,K", [(300, 512, 64), (300, 512, 128), (513, 256, 192),
                                   (256, 768, 1280), (1500, 1280, 5120)])
def test_gemm_8phase_equals_2stage(micro, M, N, K):
    """The encoder GEMM's 8-phase main loop (mwx_test_set_gemm_8ph) against the
    2-stage loop (the default) on the same operands: bit-identical outputs
    (every output fragment accumulates its K in the same order), for f16 and
    bf16, K of 1 / 2 / 3 / 20 / 80 tiles (the prologue and the drained tail of
    the stage pipeline) and partial 256-row tiles."""
    ctx, _, _ = micro
    rng = np.random.default_rng(M + K)
    a = rng.standard_normal((M, K)).astype(np.float32)
    w = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float32)
    bias = rng.uniform(-2, 2, N).astype(np.float32)
    for bf16 in (False, True):
        try:
            mwx.set_gemm_8ph(False)
            ref = ctx.test_gemm_gelu(a, w, bias, bf16, True)
            mwx.set_gemm_8ph(True)
            out = ctx.test_gemm_gelu(a, w, bias, bf16, True)
        finally:
            mwx.set_gemm_8ph(None)
        assert np.array_equal(ref.view(np.uint32), out.view(np.uint32)), (bf16, np.abs(ref - out).max())


@pytest.mark.parametrize("arch,wt", [("micro", mwx.GGML_F16), ("large-v3-l2", mwx.GGML_BF16),
                                     ("base", mwx.GGML_F16)])
def test_encoder_8phase_gemm_bit_identical(make_model, arch, wt):
    """Whole encoder (conv stem, every layer's QKV / out / FFN GEMMs with their
    epilogues) and the all-layer cross-K/V GEMM: 8-phase == 2-stage, bit for bit."""
    path = make_model(arch, wt)
    pcm = pcm_clip(4, 30.0)
    with mwx.Context.open(path) as ctx:
        try:
            mwx.set_gemm_8ph(False)
            e0, k0, v0 = ctx.test_encode(pcm, state_index=0)
            mwx.set_gemm_8ph(True)
            e1, k1, v1 = ctx.test_encode(pcm, state_index=1)
        finally:
            mwx.set_gemm_8ph(None)
    for x, y in ((e0, e1), (k0, k1), (v0, v1)):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), float(np.abs(x - y).max())


@pytest.mark.parametrize("arch,wt,mx", [("micro-rich", mwx.GGML_F16, False),
                                        ("base", mwx.GGML_F16, False),
                                        ("large-v3-l2", mwx.GGML_BF16, False),
                                        ("large-v3-l2", mwx.GGML_BF16, True)])
def test_ln_fold_bit_identical(make_model, arch, wt, mx):
    """The decode LayerNorms before the QKV and cross-Q projections folded
    into those split-K GEMMs at one row (gemm_splitk_ln, the default for
    single-row steps: C2 and the replays' test decodes) against the separate
    LayerNorm launches (ln_dec_kernel): the logits of every position of a
    48-token prefix bit for bit, and a whole single-clip service-default run
    (greedy, temperature fallback, token timestamps) record for record. mx:
    MX-fp8 compute (the fold's fp8-weight GEMM variants)."""
    path = make_model(arch, wt)
    pcm = pcm_clip(5, 30.0)
    toks = [int(t) for t in np.random.default_rng(7).integers(0, 50000, 48)]
    with mwx.Context.open(path, compute=mwx.COMPUTE_MXFP8 if mx else mwx.COMPUTE_MODEL) as ctx:
        logits, recs = [], []
        try:
            for fold in (False, True):
                mwx.set_ln_fold(fold)
                ctx.test_encode(pcm, cross=False, state_index=0)
                logits.append(ctx.test_decode(toks))
                idx = len(ctx.states)
                assert ctx.full(pcm, service_params(ctx, language=b"en"), state_index=idx) == 0
                recs.append(ctx.token_records(idx))
        finally:
            mwx.set_ln_fold(None)
    assert np.array_equal(logits[0].view(np.uint32), logits[1].view(np.uint32)), \
        float(np.abs(logits[0] - logits[1]).max())
    assert recs[0] == recs[1] and len(recs[0]) > 0
