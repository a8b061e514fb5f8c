"""Generates tests/golden/prosody_ref.npz: golden vectors for segment prosody
and speaker clustering, produced by the REFERENCE's own code
(src/prosody_extractor.cpp, src/speaker_cluster.cpp compiled unchanged from
/root/reference/src into oracle/_ref/libref_prosody.so by oracle/Makefile).

Inputs are synthetic voices stored as int16 PCM (the engine's pcm16 -> f32
conversion x / 32768 is exact), so the fixture does not depend on libm.
Outputs are stored as exact float32 bit patterns.

Run from the repo root after `make -C oracle`:
    python tests/golden/make_prosody_golden.py
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import orc  # noqa: E402

OUT = os.path.join(HERE, "prosody_ref.npz")


def voice(rng, n, sr, f0, amp, hnum=6, jitter=0.0, noise=0.0, rate=4.0):
    """A harmonic voice with an f0 glide, a syllable envelope and noise."""
    t = np.arange(n) / sr
    f = f0 * (1.0 + jitter * np.sin(2 * np.pi * 0.7 * t))
    ph = 2 * np.pi * np.cumsum(f) / sr
    sig = sum(np.sin(h * ph + rng.uniform(0, 6.28)) / h for h in range(1, hnum + 1))
    env = 0.55 + 0.45 * np.sin(2 * np.pi * rate * t + rng.uniform(0, 6.28))
    sig = amp * env * sig / max(1e-9, np.max(np.abs(sig)))
    return sig + noise * rng.standard_normal(n)


def to16(x):
    return np.clip(np.round(np.asarray(x) * 32767), -32768, 32767).astype(np.int16)


def cases():
    """(int16 pcm, sample_rate, (lpf_alpha, gender_threshold, min_pitch, max_pitch))."""
    rng = np.random.default_rng(20261016)
    D = (0.07, 170.0, 60.0, 500.0)
    out = []
    sr = 16000
    # lengths around the 160-sample gate and frame boundaries
    for n in (0, 1, 100, 159, 160, 161, 319, 320, 479):
        out.append((to16(voice(rng, n, sr, 140.0, 0.3)) if n else np.zeros(0, np.int16), sr, D))
    # low / high / whispered / loud / noisy voices, 0.25-2 s
    for f0, amp, noise, n in ((95, 0.25, 0.002, 8000), (120, 0.6, 0.01, 12000),
                              (210, 0.3, 0.003, 8000), (260, 0.08, 0.001, 6000),
                              (300, 0.9, 0.02, 16000), (180, 0.02, 0.004, 4000),
                              (150, 0.0, 0.01, 6000), (110, 0.15, 0.0, 4000),
                              (230, 0.5, 0.05, 10000), (90, 0.95, 0.0, 8000)):
        out.append((to16(voice(rng, n, sr, f0, amp, jitter=0.08, noise=noise)), sr, D))
    # digital silence, silence then onset, onset then silence, DC offset, clipping
    z = np.zeros(4000)
    v = voice(rng, 4000, sr, 170.0, 0.4, noise=0.003)
    out.append((to16(z), sr, D))
    out.append((to16(np.concatenate([z, v])), sr, D))
    out.append((to16(np.concatenate([v, z, v * 0.5])), sr, D))
    out.append((to16(v * 0.3 + 0.2), sr, D))
    out.append((to16(np.clip(v * 4.0, -1, 1)), sr, D))
    # option variants
    v2 = voice(rng, 8000, sr, 200.0, 0.35, jitter=0.1, noise=0.004)
    for opts in ((0.2, 170.0, 60.0, 500.0), (0.02, 170.0, 60.0, 500.0),
                 (0.07, 150.0, 80.0, 400.0), (0.5, 250.0, 100.0, 300.0)):
        out.append((to16(v2), sr, opts))
    # other sample rates (frame = sample_rate / 100)
    for r in (8000, 22050, 48000):
        out.append((to16(voice(rng, r // 2, r, 160.0, 0.4, noise=0.003)), r, D))
    return out


def load_ref():
    path = os.path.join(ROOT, "oracle", "_ref", "libref_prosody.so")
    L = C.CDLL(path)
    fp = C.POINTER(C.c_float)
    L.ref_extract_prosody.restype = C.c_int
    L.ref_extract_prosody.argtypes = [fp, C.c_long, C.c_int, C.c_float, C.c_float, C.c_float,
                                      C.c_float, C.c_void_p]
    L.ref_clusterer_new.restype = C.c_void_p
    L.ref_clusterer_new.argtypes = [C.c_float]
    L.ref_clusterer_free.argtypes = [C.c_void_p]
    L.ref_clusterer_assign.restype = C.c_int
    L.ref_clusterer_assign.argtypes = [C.c_void_p, fp, C.c_int, C.c_char_p, C.c_int]
    return L


class RefProsody(C.Structure):  # ref_prosody_shim.cpp RefProsody
    _fields_ = [(n, C.c_float) for n in orc.PROSODY_FLOATS] + [
        ("speaker_vec", C.c_float * 8), ("n_vec", C.c_int), ("gender", C.c_char * 8),
        ("emotion", C.c_char * 16)]


GENDER = {b"?": 0, b"M": 1, b"F": 2}
EMOTION = {b"neutral": 0, b"excited": 1, b"angry": 2, b"sad": 3}


def ref_prosody(L, pcm_f32, sr, opts):
    r = RefProsody()
    ptr = pcm_f32.ctypes.data_as(C.POINTER(C.c_float)) if len(pcm_f32) else None
    L.ref_extract_prosody(ptr, len(pcm_f32), sr, *opts, C.byref(r))
    assert r.n_vec == 8
    f = np.array([getattr(r, n) for n in orc.PROSODY_FLOATS] + list(r.speaker_vec), np.float32)
    return f.view(np.uint32), GENDER[r.gender], EMOTION[r.emotion]


def ref_cluster_ids(L, vecs, thr):
    h = L.ref_clusterer_new(thr)
    ids = []
    for v in vecs:
        a = np.ascontiguousarray(v, np.float32)
        buf = C.create_string_buffer(64)
        L.ref_clusterer_assign(h, a.ctypes.data_as(C.POINTER(C.c_float)), 8, buf, 64)
        ids.append(buf.value.decode())
    L.ref_clusterer_free(h)
    return ids


def main():
    L = load_ref()
    cs = cases()
    pcm = np.concatenate([c[0] for c in cs])
    lens = np.array([len(c[0]) for c in cs], np.int64)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    srs = np.array([c[1] for c in cs], np.int32)
    opts = np.array([c[2] for c in cs], np.float32)
    bits, gender, emotion = [], [], []
    for c in cs:
        x = (c[0].astype(np.float32) / np.float32(32768.0)).astype(np.float32)
        b, g, e = ref_prosody(L, x, c[1], tuple(float(o) for o in c[2]))
        bits.append(b)
        gender.append(g)
        emotion.append(e)
    bits = np.array(bits, np.uint32)
    # clustering: the prosody speaker vectors of the voiced cases in order,
    # then seeded perturbations of them (same-speaker repeats), a zero vector
    # and exact duplicates; two thresholds
    vecs = bits[:, 8:16].view(np.float32)
    rng = np.random.default_rng(7)
    seq = [vecs[i] for i in range(len(vecs)) if lens[i] >= 160]
    for _ in range(40):
        base = seq[rng.integers(len(seq))]
        seq.append((base + rng.normal(0, 0.03, 8)).astype(np.float32))
    seq.append(np.zeros(8, np.float32))
    seq.extend(seq[3:6])
    cvec = np.array(seq, np.float32)
    cl_thr = np.array([0.88, 0.97], np.float32)
    cl_ids = np.array([ref_cluster_ids(L, cvec, float(t)) for t in cl_thr])
    np.savez_compressed(OUT, pcm16=pcm, starts=starts, lens=lens, sample_rate=srs, opts=opts,
                        bits=bits, gender=np.array(gender, np.int32),
                        emotion=np.array(emotion, np.int32), cluster_vecs=cvec,
                        cluster_thr=cl_thr, cluster_ids=cl_ids)
    print(f"{OUT}: {len(cs)} prosody cases ({len(pcm)} samples), {len(cvec)} cluster vectors; "
          f"gender {np.bincount(gender, minlength=3)}, emotion {np.bincount(emotion, minlength=4)}, "
          f"speakers {[len(set(x)) for x in cl_ids]}")


if __name__ == "__main__":
    main()
