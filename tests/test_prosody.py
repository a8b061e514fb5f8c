"""Segment prosody and speaker clustering (reference
src/prosody_extractor.cpp, src/speaker_cluster.cpp, called per kept segment at
src/stt_engine.cpp:313-337).

Bar: bit-exact. The golden vectors (tests/golden/prosody_ref.npz) were made by
the reference's own code compiled unchanged (oracle/_ref, see
tests/golden/make_prosody_golden.py); the oracle restatement
(oracle/prosody_oracle.cpp) is pinned to them and, where oracle/_ref is built,
to the reference on further seeded inputs. The GPU kernel (k_prosody.hip,
through the C ABI mwx_prosody_batch) and the host SttEngine's clusterer are
checked against both."""
import ctypes as C
import os

import numpy as np
import pytest

import mwx
import orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "prosody_ref.npz")
REF = os.path.join(ROOT, "oracle", "_ref", "libref_prosody.so")
STT = os.path.join(ROOT, "sentiric-stt-whisper-service_amd", "libmwx_stt.so")


def gold():
    return np.load(GOLD)


def f32(pcm16):
    return (pcm16.astype(np.float32) / np.float32(32768.0)).astype(np.float32)


def rec_bits(r):
    """float32 bit patterns of the 8 scalars + speaker_vec, then gender, emotion."""
    f = [getattr(r, n) for n in orc.PROSODY_FLOATS] + list(r.speaker_vec)
    return np.array(f, np.float32).view(np.uint32), r.gender, r.emotion


def assert_same(got, want_bits, want_g, want_e, what=""):
    b, g, e = rec_bits(got)
    if not np.array_equal(b, want_bits):
        bad = np.nonzero(b != want_bits)[0]
        names = list(orc.PROSODY_FLOATS) + [f"speaker_vec[{i}]" for i in range(8)]
        raise AssertionError(f"{what}: " + ", ".join(
            f"{names[i]} {b[i:i+1].view(np.float32)[0]!r} != {want_bits[i:i+1].view(np.float32)[0]!r}"
            for i in bad))
    assert (g, e) == (want_g, want_e), what


def golden_cases(G):
    for i in range(len(G["lens"])):
        s, n = int(G["starts"][i]), int(G["lens"][i])
        yield i, G["pcm16"][s:s + n], int(G["sample_rate"][i]), tuple(float(x) for x in G["opts"][i])


def ref_lib():
    if not os.path.exists(REF):
        return None
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "make_prosody_golden", os.path.join(ROOT, "tests", "golden", "make_prosody_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m, m.load_ref()


def extra_cases():
    """Seeded inputs beyond the fixture: synthetic speech clips cut at random
    ranges (up to 30 s), pure tones on the f0 grid, noise, silence runs."""
    rng = np.random.default_rng(1234)
    out = []
    clip = mwx.pcm16_to_f32(mwx.synth_pcm16(11, n=30 * 16000))
    out.append(clip)
    for _ in range(12):
        n = int(rng.integers(160, 160000))
        s = int(rng.integers(0, len(clip) - n))
        out.append(clip[s:s + n])
    t = np.arange(16000) / 16000.0
    for f in (99.5, 100.0, 150.0, 300.0, 480.0, 520.0):
        out.append((0.3 * np.sin(2 * np.pi * f * t)).astype(np.float32))
    out.append(rng.normal(0, 0.05, 24000).astype(np.float32))
    sil = np.zeros(20000, np.float32)
    out.append(np.concatenate([clip[:30000], sil, clip[30000:60000]]))
    return out


# ---------------------------------------------------------------- CPU -----

def test_oracle_matches_reference_golden_vectors():
    G = gold()
    for i, pcm16, sr, opts in golden_cases(G):
        got = orc.prosody(f32(pcm16) if len(pcm16) else None, sr, *opts)
        assert_same(got, G["bits"][i], int(G["gender"][i]), int(G["emotion"][i]), f"case {i}")
    # the fixture spans the reference's branches
    assert set(G["gender"].tolist()) == {0, 1, 2}
    assert set(G["emotion"].tolist()) == {0, 1, 2, 3}


def test_oracle_matches_reference_build_on_more_inputs():
    r = ref_lib()
    if r is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    m, L = r
    for k, x in enumerate(extra_cases()):
        for opts in ((0.07, 170.0, 60.0, 500.0), (0.13, 190.0, 70.0, 450.0)):
            wb, wg, we = m.ref_prosody(L, x, 16000, opts)
            assert_same(orc.prosody(x, 16000, *opts), wb, wg, we, f"extra {k} {opts}")


def _host_cluster_ids(vecs, thr):
    L = C.CDLL(STT)
    L.mwx_stt_cluster_ids.restype = C.c_int
    L.mwx_stt_cluster_ids.argtypes = [C.POINTER(C.c_float), C.c_int, C.c_float, C.c_char_p,
                                      C.c_int]
    a = np.ascontiguousarray(vecs, np.float32)
    buf = C.create_string_buffer(1 << 16)
    n = L.mwx_stt_cluster_ids(a.ctypes.data_as(C.POINTER(C.c_float)), len(a), thr, buf, 1 << 16)
    assert n >= 0
    return buf.value.decode().splitlines()


def test_speaker_clustering_matches_reference_golden():
    G = gold()
    vecs = G["cluster_vecs"]
    for thr, want in zip(G["cluster_thr"], G["cluster_ids"]):
        c = orc.Clusterer(float(thr))
        assert [c.assign(v) for v in vecs] == list(want)
        assert _host_cluster_ids(vecs, float(thr)) == list(want)


def test_speaker_clustering_matches_reference_build():
    r = ref_lib()
    if r is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    m, L = r
    rng = np.random.default_rng(99)
    for trial in range(20):
        centers = rng.uniform(0, 1, (int(rng.integers(1, 6)), 8)).astype(np.float32)
        vecs = np.array([centers[rng.integers(len(centers))] + rng.normal(0, 0.05, 8)
                         for _ in range(60)], np.float32)
        vecs[rng.integers(60)] = 0
        thr = float(rng.choice([0.5, 0.88, 0.95, 0.99]))
        want = m.ref_cluster_ids(L, vecs, thr)
        assert _host_cluster_ids(vecs, thr) == want, trial


def test_prosody_abi_declared():
    L = mwx.lib()
    for n in ("mwx_prosody_batch", "mwx_prosody_batch_device", "mwx_prosody_default_params"):
        assert hasattr(L, n)
    p = L.mwx_prosody_default_params()
    assert (p.lpf_alpha, p.gender_threshold, p.min_pitch, p.max_pitch) == (
        np.float32(0.07), 170.0, 60.0, 500.0)


# ---------------------------------------------------------------- GPU -----

@pytest.fixture(scope="module")
def gctx(make_model):
    ctx = mwx.Context(make_model("micro", mwx.GGML_F16))
    yield ctx
    ctx.close()


@pytest.mark.gpu
def test_gpu_prosody_golden(gctx):
    """Every golden case, one launch per (sample rate, options) group."""
    G = gold()
    groups = {}
    for i, pcm16, sr, opts in golden_cases(G):
        groups.setdefault((sr, opts), []).append(i)
    pcm = f32(G["pcm16"])
    for (sr, opts), idx in groups.items():
        p = mwx.ProsodyParams(*opts)
        got = gctx.prosody_batch(pcm, G["starts"][idx], G["lens"][idx], sr, p)
        for i, r in zip(idx, got):
            assert_same(r, G["bits"][i], int(G["gender"][i]), int(G["emotion"][i]), f"case {i}")


@pytest.mark.gpu
def test_gpu_prosody_long_segments_match_oracle(gctx):
    """Segments up to 30 s (the speculative low-pass splits these across 256
    threads) and silence runs (the checked serial pass); host and device
    input."""
    xs = extra_cases()
    pcm = np.concatenate(xs)
    lens = np.array([len(x) for x in xs], np.int64)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    r = ref_lib()
    for opts in ((0.07, 170.0, 60.0, 500.0), (0.13, 190.0, 70.0, 450.0), (0.01, 170.0, 60.0, 500.0)):
        got = gctx.prosody_batch(pcm, starts, lens, 16000, mwx.ProsodyParams(*opts))
        for k, (x, g) in enumerate(zip(xs, got)):
            wb, wg, we = rec_bits(orc.prosody(x, 16000, *opts))
            assert_same(g, wb, wg, we, f"segment {k} {opts}")
            if r is not None:
                assert_same(g, *r[0].ref_prosody(r[1], x, 16000, opts), f"segment {k} vs ref")
        print(opts, "serial runs per segment:", [g.serial_runs for g in got])
    d = gctx.upload(pcm)
    try:
        got_d = gctx.prosody_batch(d, starts, lens)
        got_h = gctx.prosody_batch(pcm, starts, lens)
        assert [rec_bits(a)[0].tolist() for a in got_d] == [rec_bits(a)[0].tolist() for a in got_h]
    finally:
        d.free()


@pytest.mark.gpu
def test_gpu_prosody_many_segments_and_bounds(gctx):
    """A clip cut into many overlapping segments (one workgroup each), the
    160-sample gate, and argument checks."""
    x = mwx.pcm16_to_f32(mwx.synth_pcm16(5, n=20 * 16000))
    rng = np.random.default_rng(3)
    lens = rng.integers(0, 48000, 300).astype(np.int64)
    lens[:6] = [0, 1, 159, 160, 161, 320]
    starts = np.array([rng.integers(0, len(x) - n + 1) for n in lens], np.int64)
    got = gctx.prosody_batch(x, starts, lens)
    for k, (s, n, g) in enumerate(zip(starts, lens, got)):
        w = orc.prosody(x[s:s + n] if n >= 160 else None)
        assert_same(g, *rec_bits(w), f"segment {k} ({s}, {n})")
    with pytest.raises(RuntimeError):
        gctx.prosody_batch(x, [len(x) - 10], [20])
    with pytest.raises(RuntimeError):
        gctx.prosody_batch(x, [0], [1000], sample_rate=50)
    assert gctx.prosody_batch(x, [], []) == []
