"""Streaming re-transcription sessions (host/stt_stream.h,
the reference's WhisperTranscribeStream buffer loop, src/grpc_server.cpp:98-309).

The session is checked against a Python restatement of that loop driven by a
second, identically configured engine that receives the same sequence of
transcribe_pcm16 calls (so even the fallback sampler's RNG streams match):
partial cadence, the 30-s forced finalization, end of speech, the WAV-header
skip (including the reference's "first chunk <= 44 bytes" quirk) and odd
trailing bytes. Then many concurrent sessions on a batching engine."""
import ctypes as C
import json
import os
import struct
import threading

import numpy as np
import pytest

import mwx
from test_stt_engine import LIB, _transcribe, lib as stt_lib

STEP = 8000          # Settings::stream_buffer_samples default
MAX = 16000 * 30     # src/grpc_server.cpp:132


def lib():
    L = stt_lib()
    L.mwx_stt_new_ex.restype = C.c_void_p
    L.mwx_stt_new_ex.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_char_p,
                                 C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    L.mwx_stt_stream_new.restype = C.c_void_p
    L.mwx_stt_stream_new.argtypes = [C.c_void_p]
    L.mwx_stt_stream_free.argtypes = [C.c_void_p]
    L.mwx_stt_stream_feed.restype = C.c_int
    L.mwx_stt_stream_feed.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_char_p, C.c_int]
    return L


def test_stream_exports():
    L = C.CDLL(LIB)
    for n in ("mwx_stt_new_ex", "mwx_stt_stream_new", "mwx_stt_stream_free",
              "mwx_stt_stream_feed"):
        assert hasattr(L, n)


def feed(L, s, chunk: bytes):
    cap = 1 << 20
    buf = C.create_string_buffer(cap)
    r = L.mwx_stt_stream_feed(s, chunk, len(chunk), buf, cap)
    assert r >= 0, r
    return json.loads(buf.value.decode())


def wav_header(n_bytes):
    return (b"RIFF" + struct.pack("<I", 36 + n_bytes) + b"WAVEfmt " +
            struct.pack("<IHHIIHH", 16, 1, 1, 16000, 32000, 2, 16) + b"data" +
            struct.pack("<I", n_bytes))


def expected_events(L, eng, chunks):
    """The reference loop (src/grpc_server.cpp:133-300) restated in Python over
    `eng`'s transcribe_pcm16 results."""
    buf = np.zeros(0, np.int16)
    last = 0
    first, wav, skip = True, False, 0
    per_chunk = []
    for ch in chunks:
        evs = []
        if len(ch) == 0:
            if len(buf):
                _, res, _ = _transcribe(L, eng, buf, lang=b"", beam=-1, temp=-1.0)
                for r in res:
                    t = bytes.fromhex(r["text"])
                    if t:
                        evs.append(("final", t, r, [(bytes.fromhex(w["text"]), np.float32(w["t0"]) / np.float32(100),
                                                     np.float32(w["t1"]) / np.float32(100), w["p"])
                                                    for w in r["tokens"]]))
                buf = np.zeros(0, np.int16)
                last = 0
            per_chunk.append(evs)
            continue
        data = ch
        if first:
            if len(ch) >= 12 and ch[:4] == b"RIFF" and ch[8:12] == b"WAVE":
                wav = True
                if len(ch) > 44:
                    skip = 44
            first = False
        if wav and skip > 0:
            if len(data) >= skip:
                data, skip = data[skip:], 0
            else:
                skip -= len(data)
                data = b""
        if len(data):
            n = len(data) // 2
            buf = np.concatenate([buf, np.frombuffer(data[:2 * n], np.int16)])
        if len(buf) - last >= STEP:
            _, res, _ = _transcribe(L, eng, buf, lang=b"", beam=-1, temp=-1.0)
            last = len(buf)
            texts = [r for r in res if bytes.fromhex(r["text"])]
            if texts:
                evs.append(("partial", b"".join(bytes.fromhex(r["text"]) + b" " for r in texts),
                            texts[-1], None))
            if len(buf) > MAX:
                for r in texts:
                    evs.append(("forced", bytes.fromhex(r["text"]), r, None))
                buf = np.zeros(0, np.int16)
                last = 0
        per_chunk.append(evs)
    return per_chunk


def check(got, want):
    assert len(got) == len(want)
    for g, (kind, text, r, words) in zip(got, want):
        assert bytes.fromhex(g["text"]) == text
        assert g["final"] == (kind != "partial")
        assert (g["gender"], g["emotion"], g["speaker"]) == (r["gender"], r["emotion"], r["speaker"])
        assert np.float32(g["arousal"]) == np.float32(r["arousal"])
        assert g["speaker_vec"] == r["speaker_vec"]
        detail = kind != "forced"  # the forced final carries no pitch/energy detail
        for f in ("pitch_mean", "pitch_std", "energy_mean", "energy_std", "spectral_centroid",
                  "zero_crossing_rate"):
            assert np.float32(g[f]) == (np.float32(r[f]) if detail else 0.0), f
        if kind == "final":
            assert [(bytes.fromhex(w["word"]), np.float32(w["start"]), np.float32(w["end"]), w["p"])
                    for w in g["words"]] == words
        else:
            assert g["words"] == []


@pytest.mark.gpu
def test_stream_session_matches_reference_loop(tmp_path):
    path = str(tmp_path / "ggml-micro.bin")
    mwx.write_synthetic_model(path, "micro-rich", mwx.GGML_F16, 0)
    L = lib()
    d = str(tmp_path).encode()
    pcm = mwx.synth_pcm16(77, n=46 * 16000)  # 12 s, end of speech, then past the 30-s cap
    raw = pcm.tobytes()
    # a WAV first chunk, odd-sized chunks, an end of speech mid-way, more audio
    cut = 12 * 16000 * 2
    chunks = [wav_header(len(raw)) + raw[:3001]]
    p = 3001
    while p < cut:
        chunks.append(raw[p:p + 3333])
        p += 3333
    chunks.append(b"")
    while p < len(raw):
        chunks.append(raw[p:p + 6400])
        p += 6400
    chunks.append(b"")
    chunks.append(b"")  # EOS on an empty buffer: nothing
    mk = lambda: L.mwx_stt_new_ex(d, b"ggml-micro.bin", 1, 20000, 1, b"en", 500, 0, 1, 2000, STEP)
    ref_eng, eng = mk(), mk()
    assert ref_eng and eng
    try:
        want = expected_events(L, ref_eng, chunks)
        s = L.mwx_stt_stream_new(eng)
        got = [feed(L, s, ch) for ch in chunks]
        L.mwx_stt_stream_free(s)
    finally:
        L.mwx_stt_free(ref_eng)
        L.mwx_stt_free(eng)
    for g, w in zip(got, want):
        check(g, w)
    kinds = [k for evs in want for (k, *_rest) in evs]
    assert "partial" in kinds and "final" in kinds and "forced" in kinds, kinds


@pytest.mark.gpu
def test_stream_short_wav_first_chunk_quirk(tmp_path):
    """A first chunk of <= 44 bytes that starts a WAV container skips nothing
    (src/grpc_server.cpp:197-199): its bytes are appended as samples."""
    path = str(tmp_path / "ggml-micro.bin")
    mwx.write_synthetic_model(path, "micro-rich", mwx.GGML_F16, 0)
    L = lib()
    d = str(tmp_path).encode()
    raw = mwx.synth_pcm16(3, n=9 * 16000).tobytes()
    chunks = [wav_header(len(raw))[:40], raw[:20000], raw[20000:], b""]
    mk = lambda: L.mwx_stt_new_ex(d, b"ggml-micro.bin", 1, 20000, 1, b"en", 500, 0, 1, 2000, STEP)
    ref_eng, eng = mk(), mk()
    try:
        want = expected_events(L, ref_eng, chunks)
        s = L.mwx_stt_stream_new(eng)
        got = [feed(L, s, ch) for ch in chunks]
        L.mwx_stt_stream_free(s)
    finally:
        L.mwx_stt_free(ref_eng)
        L.mwx_stt_free(eng)
    for g, w in zip(got, want):
        check(g, w)


@pytest.mark.gpu
def test_concurrent_streams_share_batches(tmp_path):
    """Eight live streams on one engine with max_batch 8: their partial
    re-transcriptions are gathered into shared mwx_full_batch runs, and each
    stream's events equal those of the same stream alone on its own engine."""
    path = str(tmp_path / "ggml-micro.bin")
    mwx.write_synthetic_model(path, "micro-rich", mwx.GGML_F16, 0)
    L = lib()
    d = str(tmp_path).encode()
    raws = [mwx.synth_pcm16(90 + k, n=(5 + k) * 16000).tobytes() for k in range(8)]
    step_bytes = 2 * STEP
    chunk_lists = [[r[i:i + step_bytes] for i in range(0, len(r), step_bytes)] + [b""]
                   for r in raws]
    # streams advance in lock step, as live audio does; shorter ones are
    # padded with end-of-speech chunks (a no-op on an empty buffer)
    n_max = max(len(c) for c in chunk_lists)
    chunk_lists = [c + [b""] * (n_max - len(c)) for c in chunk_lists]
    alone = []
    for chunks in chunk_lists:
        eng = L.mwx_stt_new_ex(d, b"ggml-micro.bin", 1, 20000, 1, b"en", 500, 0, 1, 2000, STEP)
        s = L.mwx_stt_stream_new(eng)
        alone.append([feed(L, s, ch) for ch in chunks])
        L.mwx_stt_stream_free(s)
        L.mwx_stt_free(eng)
    eng = L.mwx_stt_new_ex(d, b"ggml-micro.bin", 1, 60000, 1, b"en", 500, 0, 8, 300000, STEP)
    out = [None] * len(raws)
    barrier = threading.Barrier(len(raws), timeout=120)

    def run(i):
        s = L.mwx_stt_stream_new(eng)
        evs = []
        for ch in chunk_lists[i]:
            barrier.wait()
            evs.append(feed(L, s, ch))
        L.mwx_stt_stream_free(s)
        out[i] = evs

    try:
        ts = [threading.Thread(target=run, args=(i,)) for i in range(len(raws))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        batches = L.mwx_stt_batches(eng)
    finally:
        L.mwx_stt_free(eng)
    n_calls = sum(1 for c in chunk_lists for ch in c if ch)  # each non-empty chunk re-transcribes
    assert out == alone
    assert batches < n_calls, (batches, n_calls)


@pytest.mark.gpu
def test_stream_events_kept_when_buffer_too_small(tmp_path):
    """A too-small output buffer does not lose a chunk's events: the chunk is
    consumed, the call returns -(needed + 2), and mwx_stt_stream_drain hands
    the same events over (feeding again before draining is refused)."""
    path = str(tmp_path / "ggml-micro.bin")
    mwx.write_synthetic_model(path, "micro-rich", mwx.GGML_F16, 0)
    L = lib()
    L.mwx_stt_stream_drain.restype = C.c_int
    L.mwx_stt_stream_drain.argtypes = [C.c_void_p, C.c_char_p, C.c_int]
    pcm = mwx.synth_pcm16(3, n=2 * STEP).tobytes()
    d = str(tmp_path).encode()
    evs = []
    for small in (False, True):
        eng = L.mwx_stt_new_ex(d, b"ggml-micro.bin", 1, 5000, 1, b"en", 500, 0, 1, 0, STEP)
        s = L.mwx_stt_stream_new(eng)
        try:
            if not small:
                evs.append(feed(L, s, pcm))
                continue
            tiny = C.create_string_buffer(4)
            r = L.mwx_stt_stream_feed(s, pcm, len(pcm), tiny, 4)
            assert r < -3
            assert L.mwx_stt_stream_feed(s, pcm, len(pcm), tiny, 4) == -3  # pending: drain first
            cap = -r - 2
            buf = C.create_string_buffer(cap)
            assert L.mwx_stt_stream_drain(s, buf, cap) >= 0
            evs.append(json.loads(buf.value.decode()))
            assert L.mwx_stt_stream_drain(s, buf, cap) >= 0 and json.loads(buf.value.decode()) == []
        finally:
            L.mwx_stt_stream_free(s)
            L.mwx_stt_free(eng)
    assert evs[0] == evs[1] and len(evs[0]) > 0
