"""SttEngine host mirror (sentiric-stt-whisper-service_amd/host/, over the C ABI):
the service-level filters against their restatement in oracle/service_filters.py
(CPU), and transcribe_pcm16 end to end on the GPU against the oracle's full
pipeline + the same post-filters (mirrors how the reference's HTTP/gRPC
handlers call SttEngine::transcribe_pcm16, src/http_server.cpp:165-166)."""
import ctypes as C
import json
import os
import random
import sys
import threading

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "sentiric-stt-whisper-service_amd"))
import service_filters as sf  # noqa: E402

LIB = os.path.join(ROOT, "sentiric-stt-whisper-service_amd", "libmwx_stt.so")


def lib():
    L = C.CDLL(LIB)
    L.mwx_stt_is_hallucination.argtypes = [C.c_char_p]
    L.mwx_stt_new.restype = C.c_void_p
    L.mwx_stt_new.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_char_p,
                              C.c_int, C.c_int]
    L.mwx_stt_free.argtypes = [C.c_void_p]
    L.mwx_stt_new_batched.restype = C.c_void_p
    L.mwx_stt_new_batched.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int,
                                      C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int]
    L.mwx_stt_batches.restype = C.c_long
    L.mwx_stt_batches.argtypes = [C.c_void_p]
    L.mwx_stt_transcribe_pcm16.argtypes = [C.c_void_p, C.POINTER(C.c_int16), C.c_int, C.c_int,
                                           C.c_char_p, C.c_int, C.c_float, C.c_char_p, C.c_int,
                                           C.POINTER(C.c_double)]
    return L


CASES = [
    "", " ", "a", " a ", "...", " ?! ", "[Music]", "(laughs)", "[ok", "Thank you.",
    "thank you for coming", "THANK YOU", "Thanks for watching!", "www.example.org", "x.com",
    "Hmm", "hmm...", "...Hmm!", "Hmm hmm", "Okay.", "okay.", "Okay", "Bye.", "bye", "Ahem",
    "Umarım", "umarım.", "Altyazı M.K.", "ALTYAZI", "Teşekkürler.", "teşekkür ederim",
    "Abone ol!", "2分", "ご視聴ありがとう", "Eh", "eh?", "Oh!", "oh no", "Hıhı", "Pffft.",
    "Hello world.", "I'm going to go home", "transcription: x", "subtitle: y", "Aa",
    "Merhaba dünya", "devam edecek...", "\tHello\n", "A.", "OK",
]


def test_is_hallucination_matches_restatement():
    L = lib()
    rng = random.Random(7)
    pieces = ["Hmm", "ok", "Thank you", ".", "!", "?", " ", "[", "]", "(", ")", "www.", "a",
              "Okay.", "Eh", "ı", "İ", "分", "\t", "-", "'"]
    cases = list(CASES) + ["".join(rng.choice(pieces) for _ in range(rng.randint(0, 5)))
                           for _ in range(2000)]
    for t in cases:
        b = t.encode()
        assert bool(L.mwx_stt_is_hallucination(b)) == sf.is_hallucination(b), repr(t)


def test_library_exports():
    L = lib()
    for name in ("mwx_stt_is_hallucination", "mwx_stt_new", "mwx_stt_free",
                 "mwx_stt_transcribe_pcm16", "mwx_stt_new_batched", "mwx_stt_batches",
                 "mwx_stt_cluster_ids"):
        assert hasattr(L, name)


def _transcribe(L, eng, pcm16, lang=b"en", beam=1, temp=-1.0):
    cap = 1 << 20
    buf = C.create_string_buffer(cap)
    m = (C.c_double * 3)()
    p = np.ascontiguousarray(pcm16, np.int16)
    r = L.mwx_stt_transcribe_pcm16(eng, p.ctypes.data_as(C.POINTER(C.c_int16)), len(p), 16000,
                                   lang, beam, temp, buf, cap, m)
    if r < 0:
        return r, None, list(m)
    return r, json.loads(buf.value.decode()), list(m)


def check_prosody(res, pcm):
    """Segment affect fields and speaker ids (src/stt_engine.cpp:313-337):
    bit-exact against the oracle's prosody of each segment's sample range and
    its clusterer run over the kept segments in order."""
    import orc
    clus = orc.Clusterer(0.88)
    for g in res:
        s0 = max(0, min(int((g["t0"] / 100.0) * 16000.0), len(pcm)))
        s1 = max(s0, min(int((g["t1"] / 100.0) * 16000.0), len(pcm)))
        w = orc.prosody(pcm[s0:s1] if s1 - s0 >= 160 else None)
        assert g["gender"] == ("?", "M", "F")[w.gender]
        assert g["emotion"] == ("neutral", "excited", "angry", "sad")[w.emotion]
        for n in orc.PROSODY_FLOATS:
            assert np.float32(g[n]) == np.float32(getattr(w, n)), n
        assert np.array_equal(np.array(g["speaker_vec"], np.float32),
                              np.array(list(w.speaker_vec), np.float32))
        want_spk = clus.assign(np.array(list(w.speaker_vec), np.float32)) if s1 - s0 >= 160 else "?"
        assert g["speaker"] == want_spk


@pytest.mark.gpu
def test_transcribe_pcm16_matches_oracle(tmp_path):
    import mwx
    import orc
    path = str(tmp_path / "ggml-micro.bin")
    mwx.write_synthetic_model(path, "micro-rich", mwx.GGML_F16, 0)
    L = lib()
    o = orc.Oracle(path)
    try:
        for seed, secs in ((1, 10), (2, 30), (3, 45)):
            # a fresh engine per request: the fallback sampler's std::mt19937
            # lives in the state and advances across requests (as in
            # whisper.cpp), while each oracle run starts from a fresh state
            eng = L.mwx_stt_new(str(tmp_path).encode(), b"ggml-micro.bin", 2, 5000, 1, b"auto",
                                500, 0)
            assert eng
            pcm16 = mwx.synth_pcm16(seed, n=secs * 16000)
            rc, res, metrics = _transcribe(L, eng, pcm16)
            L.mwx_stt_free(eng)
            assert rc >= 0
            opt = orc.FullOptions.service_defaults(beam_size=1)
            opt.language = "en"
            _, segs, _, _ = o.full(mwx.pcm16_to_f32(pcm16), opt)
            want = sf.postprocess(
                [(s.raw, s.t0, s.t1, [(t.id, t.p, t.t0, t.t1) for t in s.tokens]) for s in segs],
                o.eot, o.token_bytes)
            assert len(res) == len(want)
            for g, w in zip(res, want):
                assert bytes.fromhex(g["text"]) == w["text"]
                assert (g["t0"], g["t1"]) == (w["t0"], w["t1"])
                assert len(g["tokens"]) == len(w["tokens"]) == g["n"]
                for gt, wt in zip(g["tokens"], w["tokens"]):
                    assert bytes.fromhex(gt["text"]) == wt[0]
                    assert abs(gt["p"] - wt[1]) < 5e-3
                    assert (gt["t0"], gt["t1"]) == (wt[2], wt[3])
                assert abs(g["prob"] - w["prob"]) < 5e-3
                assert bytes.fromhex(g["language"]) == b"en"
            check_prosody(res, mwx.pcm16_to_f32(pcm16))
            assert metrics[2] >= sum(len(w["tokens"]) for w in want)
        # too-short audio gate (src/stt_engine.cpp:153-167): < 500 ms -> no results
        eng = L.mwx_stt_new(str(tmp_path).encode(), b"ggml-micro.bin", 1, 5000, 1, b"auto", 500, 0)
        rc, res, metrics = _transcribe(L, eng, mwx.synth_pcm16(4, n=4800))
        L.mwx_stt_free(eng)
        assert rc >= 0 and res == [] and metrics == [0.0, 0.0, 0.0]
    finally:
        o.close()


@pytest.mark.gpu
def test_engine_busy_when_pool_exhausted(tmp_path):
    import mwx
    path = str(tmp_path / "ggml-micro.bin")
    mwx.write_synthetic_model(path, "micro", mwx.GGML_F16, 12)
    L = lib()
    # one state, 1 ms queue timeout: concurrent requests must see EngineBusy
    eng = L.mwx_stt_new(str(tmp_path).encode(), b"ggml-micro.bin", 1, 1, 1, b"en", 500, 0)
    assert eng
    pcm16 = mwx.synth_pcm16(5)
    codes = []

    def run():
        codes.append(_transcribe(L, eng, pcm16)[0])

    try:
        ts = [threading.Thread(target=run) for _ in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert -2 in codes and any(c >= 0 for c in codes), codes
    finally:
        L.mwx_stt_free(eng)


@pytest.mark.gpu
def test_dynamic_batching_equals_single_requests(tmp_path):
    """Concurrent transcribe_pcm16 calls on an engine with max_batch 8 are
    served as shared mwx_full_batch runs; every caller gets exactly the
    result a one-request engine gives for its clip (fresh states on both
    sides, so the fallback sampler's RNG streams match)."""
    import mwx
    path = str(tmp_path / "ggml-micro.bin")
    mwx.write_synthetic_model(path, "micro-rich", mwx.GGML_F16, 0)
    L = lib()
    d = str(tmp_path).encode()
    clips = [mwx.synth_pcm16(40 + k, n=(6 + 3 * k) * 16000) for k in range(8)]
    singles = []
    for pcm in clips:
        eng = L.mwx_stt_new(d, b"ggml-micro.bin", 1, 5000, 1, b"en", 500, 0)
        rc, res, _ = _transcribe(L, eng, pcm)
        L.mwx_stt_free(eng)
        assert rc >= 0
        singles.append(res)
    eng = L.mwx_stt_new_batched(d, b"ggml-micro.bin", 1, 20000, 1, b"en", 500, 0, 8, 200000)
    assert eng
    out = [None] * len(clips)

    def run(i):
        out[i] = _transcribe(L, eng, clips[i])

    try:
        ts = [threading.Thread(target=run, args=(i,)) for i in range(len(clips))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        batches = L.mwx_stt_batches(eng)
    finally:
        L.mwx_stt_free(eng)
    assert all(o[0] >= 0 for o in out)
    assert [o[1] for o in out] == singles
    assert batches < len(clips), batches  # requests were actually batched


def test_missing_model_raises_in_constructor(tmp_path):
    # SttEngine's constructor throws on a model that fails to load
    # (src/stt_engine.cpp:34); the C shim reports it as NULL
    L = lib()
    eng = L.mwx_stt_new(str(tmp_path).encode(), b"nope.bin", 1, 10, 1, b"en", 500, 0)
    assert not eng
