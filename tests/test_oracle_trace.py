"""The oracle's decision trace (mwx_oracle.cpp TraceKind), which the GPU
beam-vs-oracle tests (test_gpu_beam_oracle.py) compare across two runs: CPU
checks that it is a faithful record of full()'s decisions."""
import numpy as np
import pytest

import mwx
import orc


@pytest.fixture(scope="module")
def rich(tmp_path_factory):
    path = str(tmp_path_factory.mktemp("tr") / "rich.bin")
    mwx.write_synthetic_model(path, "micro-rich", mwx.GGML_F16, 0)
    return orc.Oracle(path)


def beam_opt():
    opt = orc.FullOptions.service_defaults(beam_size=5)
    opt.temperature_inc = 0.0
    opt.language = "en"
    return opt


def test_trace_replay_of_own_logits_is_identical(rich):
    """full_external fed the oracle's own logits for every prefix takes the
    same decisions, with the same margins, as full() (so a divergence between
    the oracle's own run and a replay of device logits comes from the logits
    alone), and the trace is deterministic."""
    o = rich
    pcm = mwx.pcm16_to_f32(mwx.synth_pcm16(50, 6 * 16000))
    (_, segs, _, _), ta = o.traced(o.full, pcm, beam_opt())
    (_, segs2, _, _), ta2 = o.traced(o.full, pcm, beam_opt())
    assert [e.key() for e in ta] == [e.key() for e in ta2]
    mel, _ = o.mel(pcm)
    cur = {}

    def enc(seek):
        cur["kv"] = o.cross(o.encode(mel, seek=seek))

    def logits(toks):
        return o.decode_seq(*cur["kv"], toks)[-1]

    (_, rsegs, _, _), tb = o.traced(o.full_external, pcm, beam_opt(), enc, logits)
    assert orc.first_divergence(ta, tb) is None
    assert [e.margin for e in ta] == [e.margin for e in tb]
    assert [(t.id, t.p) for s in segs for t in s.tokens] == \
        [(t.id, t.p) for s in rsegs for t in s.tokens]
    kinds = {e.kind for e in ta}
    assert {"draw", "assign", "ts_mass", "status", "best"} <= kinds
    assert "exact_tie" not in kinds


def test_trace_draw_margin_matches_discrete_distribution(rich):
    """The first step's draws of decoder 0, rebuilt independently: the
    uniforms of std::mt19937(0) through generate_canonical<double, 53> (two
    32-bit outputs per draw; numpy's MT19937 with the legacy init_genrand
    seeding), the probabilities from the oracle's prompt logits through its
    process_logits, the id as libstdc++ std::discrete_distribution picks it
    (lower_bound over the normalised partial sums), and the margin as the
    distance of the uniform to the nearest boundary of that id's interval."""
    o = rich
    pcm = mwx.pcm16_to_f32(mwx.synth_pcm16(51, 4 * 16000))
    _, tr = o.traced(o.full, pcm, beam_opt())
    draws = [e for e in tr if e.kind == "draw" and e.seek == 0 and e.it == 0 and e.step == 0
             and e.dec == 0]
    assert [e.a for e in draws] == [0, 1, 2, 3, 4]
    bg = np.random.MT19937()
    bg._legacy_seeding(0)
    raw = bg.random_raw(10).astype(np.float64)
    u = (raw[0::2] + raw[1::2] * 2.0 ** 32) / 2.0 ** 64
    mel, _ = o.mel(pcm)
    k, v = o.cross(o.encode(mel))
    prompt = [o.sot, o.sot + 1, o.transcribe] if o.n_vocab >= 51865 else [o.sot]
    raw_lg = o.decode_seq(k, v, prompt)[-1]
    _, _, pr, _ = o.process_logits(raw_lg, [], False, 3000, suppress_nst=True)
    cp = np.cumsum(pr.astype(np.float64) / pr.astype(np.float64).sum())
    for e, uk in zip(draws, u):
        assert e.v == uk
        i = int(np.searchsorted(cp, uk, side="left"))
        assert e.b == i
        lo = cp[i - 1] if i else 0.0
        assert abs(e.margin - min(uk - lo, cp[i] - uk)) < 1e-9
    assert len([e for e in tr if e.kind == "draw"]) >= 50


def test_first_divergence():
    ev = lambda k, b: orc.TraceEv(k, 0, 0, 0, 0, 0, b, 1.0, 0.0)  # noqa: E731
    a = [ev("draw", 1), ev("draw", 2), ev("assign", 3)]
    assert orc.first_divergence(a, list(a)) is None
    assert orc.first_divergence(a, [ev("draw", 1), ev("draw", 5), ev("assign", 3)]) == 1
    assert orc.first_divergence(a, a[:2]) == 2
    assert np.isfinite(a[0].margin)


def perturbed_guide(o, pcm, opt, amp):
    """The oracle's loop replayed on its own logits plus seeded noise of
    amplitude `amp` per prefix (a stand-in for the device's rounding): its
    trace and the rows it decoded."""
    mel, _ = o.mel(pcm)
    cur = {}
    rows = {}

    def enc(seek):
        cur["seek"] = seek
        cur["kv"] = o.cross(o.encode(mel, seek=seek))

    def logits(toks):
        lg = o.decode_seq(*cur["kv"], toks)[-1]
        rng = np.random.default_rng(abs(hash((cur["seek"],) + tuple(toks))) % 2 ** 32)
        lg = lg + rng.uniform(-amp, amp, lg.shape).astype(np.float32)
        rows[(cur["seek"], tuple(toks))] = lg
        return lg

    (_, segs, _, _), tb = o.traced(o.full_external, pcm, opt, enc, logits)
    return segs, tb, rows


@pytest.mark.parametrize("temperature_inc", [0.0, 0.2])
def test_follow_mode_checks_every_decision(rich, temperature_inc):
    """Follow mode (the whole-window beam comparison of
    test_gpu_beam_oracle.py) on CPU: the guide is the oracle's loop on its own
    logits perturbed by seeded noise, so near-tie draws flip as they do on the
    device. The oracle on its own logits, following the guide, takes every
    decision the guide took (forced where its own arithmetic differs, each
    within the bound of the measured noise) and ends on the guide's tokens."""
    from beam_follow import follow_compare

    o = rich
    opt = beam_opt()
    opt.temperature_inc = temperature_inc
    n_forced = 0
    for k in range(2):
        pcm = mwx.pcm16_to_f32(mwx.synth_pcm16(50 + k, (10 + 4 * k) * 16000))
        gsegs, tb, rows = perturbed_guide(o, pcm, opt, 0.03)
        r = follow_compare(o, pcm, opt, tb, rows)
        assert r.tokens == [t.id for s in gsegs for t in s.tokens]
        assert 0.0 < r.eps_max <= 0.03 + 1e-6
        n_forced += len(r.forced)
        print(r.summary(f"clip {k}"))
    assert n_forced > 0  # the noise did flip near-tie decisions, and they were followed


def test_follow_mode_stops_at_a_structural_difference(rich):
    """A guide whose decoder status differs from the oracle's (a changed rule,
    not a near-tie) is not followed past that event."""
    o = rich
    pcm = mwx.pcm16_to_f32(mwx.synth_pcm16(50, 6 * 16000))
    _, tr = o.traced(o.full, pcm, beam_opt())
    i = next(i for i, e in enumerate(tr) if e.kind == "status")
    bad = list(tr)
    e = bad[i]
    bad[i] = orc.TraceEv(e.kind, e.seek, e.it, e.step, e.dec, e.a ^ 2, e.b, e.margin, e.v)
    _, _, brk = o.traced_follow(bad, pcm, beam_opt())
    assert brk == i
    _, tr2, brk2 = o.traced_follow(tr, pcm, beam_opt())  # its own trace: followed to the end
    assert brk2 is None and not [x for x in tr2 if x.forced]
    assert [x.key() for x in tr2] == [x.key() for x in tr]


def test_best_decoder_id_persists_across_attempts(rich):
    """whisper.cpp v1.8.2 declares best_decoder_id before the temperature loop
    and resets only the decoders an attempt runs: beam search's fallbacks run
    one decoder (best_of = -1, src/stt_engine.cpp:235-238), and when it fails
    the window's best stays the earlier attempt's decoder — whose state that
    attempt left. The oracle keeps that (the engine's driver does too, checked
    on the GPU by test_beam5_temperature_ladder_vs_oracle_arithmetic): on this
    clip, with every window walking the ladder, the t > 0 attempts' BEST events
    name decoder 2 of the t = 0 beam pass although only decoder 0 ran."""
    o = rich
    pcm = mwx.pcm16_to_f32(mwx.synth_pcm16(50, 14 * 16000))
    opt = beam_opt()
    opt.temperature_inc = 0.2
    opt.logprob_thold = 0.5
    assert opt.best_of == -1
    (_, segs, _, _), tr = o.traced(o.full, pcm, opt)
    best = [(e.seek, e.it, e.a) for e in tr if e.kind == "best"]
    stale = [b for b in best if b[1] > 0 and b[2] > 0]
    assert stale, best
