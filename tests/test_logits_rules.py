"""Pins the oracle's token-loop rules (whisper_process_logits + the greedy
whisper_sample_token record) against an INDEPENDENT
implementation of the same OpenAI rule set: HF transformers'
SuppressTokensLogitsProcessor, SuppressTokensAtBeginLogitsProcessor and
WhisperTimeStampLogitsProcessor (transformers 5.x, importable in this image).

The reference service sets these rules through whisper_full_params
(/root/reference/src/stt_engine.cpp:221-243: suppress_nst, suppress_blank by
default, token_timestamps, the thresholds); whisper.cpp v1.8.2 implements
them in whisper_process_logits. Where whisper.cpp deliberately differs from
the OpenAI / HF rules, the difference is predicted here by a named rule and
checked to be exactly that (DESIGN.md §2 lists them):

  D1  initial step: OpenAI / HF suppress every non-timestamp token at
      sample_begin ("suppress generating non-timestamp tokens at the
      beginning"); whisper_process_logits applies only the max_initial_ts cap.
  D2  monotonic timestamps: HF forbids timestamps < the last one when the last
      two tokens are (text, timestamp), and <= the last one otherwise;
      whisper.cpp keeps decoder.seek_delta (2 x the last sampled timestamp
      index, set only for ids > token_beg) and suppresses [beg, beg +
      seek_delta/2): an equal timestamp stays allowed, and <|0.00|> never
      starts the rule.
  D3  temperature: whisper.cpp divides the logits by the temperature before
      every rule, so the timestamp-mass rule sees the tempered logits; HF
      applies TemperatureLogitsWarper after the processors (checked: with the
      tempered logits fed to HF the masks agree).
  D4  suppress_nst's token list: whisper.cpp suppresses the vocabulary entries
      that equal a non_speech_tokens string (or " " + it) plus " -" and " '";
      OpenAI encodes each symbol with the BPE tokenizer (first token of a
      multi-token musical symbol too). No whisper tokenizer is in the image,
      so the list itself is whisper.cpp's (the mask it produces is pinned).

Three checks per case: (A) the masks before the timestamp-mass rule equal
HF's up to the predicted D1 / D2 ids; (B) HF's timestamp-mass rule applied to
the oracle's pre-rule logits gives the oracle's final logits bit for bit;
(C) logprobs / probs and the greedy record (id, tid, p, plog, pt, ptsum)
against a float64 log-softmax (whisper.cpp's order: log-softmax, then the
timestamp-mass rule masks text logprobs without renormalising).
"""
import numpy as np
import pytest

import orc

torch = pytest.importorskip("torch")
lp_mod = pytest.importorskip("transformers.generation.logits_process")

# whisper.cpp v1.8.2 non_speech_tokens (whisper.cpp: whisper_process_logits)
NST = ["\"", "#", "(", ")", "*", "+", "/", ":", ";", "<", "=", ">", "@", "[", "\\", "]", "^",
       "_", "`", "{", "|", "}", "~", "「", "」", "『", "』", "<<", ">>", "<<<", ">>>", "--",
       "---", "-(", "-[", "('", "(\"", "((", "))", "(((", ")))", "[[", "]]", "{{", "}}", "♪♪",
       "♪♪♪", "♩", "♪", "♫", "♬", "♭", "♮", "♯"]
N_LANG = 100


class GenCfg:
    """The fields WhisperTimeStampLogitsProcessor reads from a generation config."""

    def __init__(self, no_ts, eot, max_initial_index):
        self.no_timestamps_token_id = no_ts
        self.eos_token_id = eot
        self.bos_token_id = eot
        self.max_initial_timestamp_index = max_initial_index
        self._detect_timestamp_from_logprob = True


@pytest.fixture(scope="module", params=["micro-v3", "micro"])
def vocab(request, make_model):
    o = orc.Oracle(make_model(request.param))
    tok2id = {}
    for i in range(o.eot):
        tok2id.setdefault(o.token_bytes(i), i)
    return o, tok2id


def static_suppress(o, tok2id, suppress_nst, tdrz=False):
    """whisper_process_logits' unconditional suppressions (sot, nosp, solm,
    task tokens, prev, language tokens) and the suppress_nst list (D4)."""
    s = {o.sot, o.nosp, o.translate, o.transcribe, o.prev}
    if not tdrz:
        s.add(o.solm)
    s.update(o.sot + 1 + i for i in range(N_LANG))
    if suppress_nst:
        for t in NST:
            for w in (t, " " + t):
                i = tok2id.get(w.encode())
                if i is not None:
                    s.add(i)
        for w in (" -", " '"):
            i = tok2id.get(w.encode())
            if i is not None:
                s.add(i)
    return sorted(s)


def hf_chain(o, tok2id, prompt_len, suppress_blank, suppress_nst, max_initial_ts, detect):
    procs = [lp_mod.SuppressTokensLogitsProcessor(static_suppress(o, tok2id, suppress_nst))]
    if suppress_blank:
        procs.append(lp_mod.SuppressTokensAtBeginLogitsProcessor([tok2id[b" "], o.eot], prompt_len))
    mi = int(round(max_initial_ts / 0.02)) if max_initial_ts > 0 else None
    procs.append(lp_mod.WhisperTimeStampLogitsProcessor(GenCfg(o.not_, o.eot, mi), prompt_len,
                                                        _detect_timestamp_from_logprob=detect))
    return procs


def run_hf(procs, ids, scores):
    ids_t = torch.tensor([ids], dtype=torch.long)
    s = torch.tensor(scores[None, :], dtype=torch.float32)
    for p in procs:
        s = p(ids_t, s)
    return s[0].numpy()


def loop_state(o, hist):
    """decoder.has_ts / seek_delta as the whisper_full token loop keeps them
    (set by sampled ids > token_beg; full() in the oracle)."""
    has_ts, sd = False, 3000
    for t in hist:
        if t > o.beg:
            has_ts, sd = True, 2 * (t - o.beg)
    return has_ts, sd


def predicted_dev(o, hist, V):
    """Ids HF masks and whisper.cpp does not, before the timestamp-mass rule
    (D1, D2)."""
    dev = np.zeros(V, bool)
    if not hist:  # D1
        dev[:o.beg] = True
        return dev
    last_ts = hist[-1] >= o.beg
    pen_ts = len(hist) < 2 or hist[-2] >= o.beg
    ts = [t for t in hist if t >= o.beg]
    if ts:  # D2
        hf_end = ts[-1] if (last_ts and not pen_ts) else ts[-1] + 1
        has_ts, sd = loop_state(o, hist)
        cpp_end = o.beg + sd // 2 if has_ts else o.beg
        dev[cpp_end:hf_end] = True
    return dev


def cases(o, V, rng):
    """(history, raw logits): initial steps, text runs, every timestamp-pair
    state, <|0.00|>, repeated timestamps, timestamp-heavy and text-heavy rows."""
    beg, eot = o.beg, o.eot
    text = lambda: int(rng.integers(0, eot))  # noqa: E731
    ts = lambda lo=0, hi=1500: int(beg + rng.integers(lo, hi))  # noqa: E731
    hists = [[], [], [text()], [text(), text(), text()]]
    for _ in range(3):
        a = ts(0, 200)
        b = a + int(rng.integers(1, 300))
        hists += [[a], [a, text()], [a, text(), text(), b], [a, text(), b, b], [a, text(), b, b, text()],
                  [a, text(), b], [a, text(), b, b, text(), text()]]
    hists += [[beg], [beg, text()], [beg, text(), beg + 50], [beg, beg], [beg, beg, text()],
              [beg + 7, text(), beg + 7], [beg + 7, text(), beg + 7, beg + 7, text()]]
    out = []
    for h in hists:
        for mode in ("flat", "ts", "text"):
            x = rng.normal(0.0, 3.0, V).astype(np.float32)
            if mode == "ts":
                x[beg:] += 4.0
            elif mode == "text":
                x[:eot] += 2.0
                x[int(rng.integers(0, eot))] += 12.0
            out.append((h, x))
    return out


@pytest.mark.parametrize("suppress_blank,suppress_nst,max_initial_ts,temperature",
                         [(True, True, 1.0, 0.0), (True, False, 0.0, 0.0),
                          (False, True, 1.0, 0.0), (True, True, 1.0, 0.6)])
def test_process_logits_matches_hf_processors(vocab, suppress_blank, suppress_nst, max_initial_ts,
                                             temperature):
    o, tok2id = vocab
    V = o.n_vocab
    rng = np.random.default_rng(11)
    prompt = [o.sot, o.sot + 1, o.transcribe] if V >= 51865 else [o.sot]
    n_dev = 0
    for hist, raw in cases(o, V, rng):
        has_ts, sd = loop_state(o, hist)
        kw = dict(suppress_blank=suppress_blank, suppress_nst=suppress_nst,
                  max_initial_ts=max_initial_ts, temperature=temperature)
        pre, _, _, _ = o.process_logits(raw, hist, has_ts, sd, ts_mass_rule=False, **kw)
        lg, lp, pr, rec = o.process_logits(raw, hist, has_ts, sd, **kw)
        # D3: HF sees the tempered logits (whisper.cpp divides first)
        x = raw / np.float32(temperature) if temperature > 0 else raw
        ids = prompt + list(hist)
        # (A) masks before the timestamp-mass rule, up to the predicted deviations
        hf_pre = run_hf(hf_chain(o, tok2id, len(prompt), suppress_blank, suppress_nst,
                                 max_initial_ts, False), ids, x)
        dev = predicted_dev(o, hist, V)
        m_cpp, m_hf = np.isneginf(pre), np.isneginf(hf_pre)
        assert not (m_cpp & ~m_hf).any(), (hist, np.nonzero(m_cpp & ~m_hf)[0][:8])
        assert ((m_hf & ~m_cpp) == (dev & ~m_cpp)).all(), (hist, np.nonzero((m_hf & ~m_cpp) ^ (dev & ~m_cpp))[0][:8])
        n_dev += int((dev & ~m_cpp).any())
        fin = ~m_cpp
        np.testing.assert_array_equal(pre[fin], x[fin])
        # (B) HF's timestamp-mass rule on the oracle's pre-rule logits: a
        # history past the prompt with no timestamp, so only that rule (and
        # the <|notimestamps|> suppression, already applied) can fire
        ts_rule = lp_mod.WhisperTimeStampLogitsProcessor(GenCfg(o.not_, o.eot, None), len(prompt),
                                                         _detect_timestamp_from_logprob=True)
        hf_fin = run_hf([ts_rule], prompt + [0], pre)
        np.testing.assert_array_equal(np.isneginf(lg), np.isneginf(hf_fin))
        np.testing.assert_array_equal(lg[~np.isneginf(lg)], hf_fin[~np.isneginf(hf_fin)])
        # (C) logprobs / probs / the greedy record against float64. whisper.cpp
        # takes the log-softmax BEFORE the timestamp-mass rule and then only
        # sets the suppressed text entries to -inf (the timestamps' logprobs
        # are not renormalised); it sums exp() in float over the vocabulary
        # (~1e-4 of drift)
        f = ~np.isneginf(lg)
        fp = ~np.isneginf(pre)
        l64 = lg.astype(np.float64)
        p64_ = pre.astype(np.float64)
        lse = np.log(np.exp(p64_[fp] - p64_[fp].max()).sum()) + p64_[fp].max()
        np.testing.assert_allclose(lp[f], l64[f] - lse, atol=5e-4, rtol=0)
        assert np.isneginf(lp[~f]).all() and (pr[~f] == 0).all()
        p64 = np.where(f, np.exp(np.where(f, l64 - lse, 0.0)), 0.0)
        np.testing.assert_allclose(pr, p64, atol=1e-6, rtol=5e-4)
        rid, rtid, rp, rplog, rpt, rptsum = rec
        assert rid == int(np.argmax(pr)) and rp == pr[rid] and rplog == lp[rid]
        if rid >= o.beg:
            assert rtid == rid and rpt == rp
        else:
            tsp = pr[o.beg:].astype(np.float64)
            assert rtid == o.beg + int(np.argmax(tsp)) or tsp.max() == 0
            assert abs(rpt - tsp.max() / (tsp.sum() + 1e-10)) < 1e-6
            assert abs(rptsum - tsp.sum()) < 1e-6
    assert n_dev > 0  # the deviation rules were exercised, not vacuous


def test_forced_timestamp_rule_fires(vocab):
    """The timestamp-mass rule (sum p(timestamps) > max p(text) -> only
    timestamps) fires on timestamp-heavy rows and not on text-heavy rows, on
    both implementations."""
    o, tok2id = vocab
    V = o.n_vocab
    rng = np.random.default_rng(5)
    prompt = [o.sot]
    fired = kept = 0
    for mode in ("ts", "text") * 6:
        x = rng.normal(0, 1.0, V).astype(np.float32)
        if mode == "ts":
            x[o.beg:] += 3.0
        else:
            x[int(rng.integers(0, o.eot))] += 30.0
        hist = [int(rng.integers(0, o.eot))]
        lg, _, _, rec = o.process_logits(x, hist, False, 3000, suppress_nst=True)
        hf = run_hf(hf_chain(o, tok2id, 1, True, True, 1.0, True), prompt + hist, x)
        np.testing.assert_array_equal(np.isneginf(lg), np.isneginf(hf))
        if np.isneginf(lg[:o.beg]).all():
            fired += 1
            assert rec[0] >= o.beg
        else:
            kept += 1
    assert fired == 6 and kept == 6
