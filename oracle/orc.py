"""ctypes binding of the CPU oracle (liborc.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker. See oracle/mwx_oracle.cpp for what the
oracle restates (whisper.cpp v1.8.2 semantics; parity with whisper.cpp itself
is unpinned because the reference ships no fixtures and whisper.cpp is not
available offline).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ORC_LIB: the sanitizer build (tests/san/Makefile) for tests/test_sanitizers.py
LIB_PATH = os.environ.get("ORC_LIB") or os.path.join(HERE, "liborc.so")
ORC_EXACT = 1
ORC_MXFP8 = 2  # encoder / cross-K/V matmuls on MX-fp8 operands (engine MWX_COMPUTE_MXFP8)

_lib = None
EXT_ENC = C.CFUNCTYPE(None, C.c_void_p, C.c_int)
EXT_LOGITS = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_float))
TAP_LOGITS = EXT_LOGITS  # (user, tokens, n, logits_last): the oracle's own decoded rows


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    L = C.CDLL(LIB_PATH)
    P = C.c_void_p
    fp = C.POINTER(C.c_float)
    L.orc_load.restype = P
    L.orc_load.argtypes = [C.c_char_p, C.c_int]
    L.orc_free.argtypes = [P]
    L.orc_set_threads.argtypes = [C.c_int]
    L.orc_set_enc_layer_limit.argtypes = [C.c_int]
    L.orc_set_external.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.orc_hparams.argtypes = [P, C.POINTER(C.c_int)]
    L.orc_wtype.restype = C.c_int
    L.orc_wtype.argtypes = [P]
    L.orc_special.argtypes = [P, C.POINTER(C.c_int)]
    L.orc_tensor.restype = C.c_long
    L.orc_tensor.argtypes = [P, C.c_char_p, fp, C.c_long]
    L.orc_token_str.restype = C.c_char_p
    L.orc_token_str.argtypes = [P, C.c_int]
    L.orc_filters.restype = fp
    L.orc_filters.argtypes = [P]
    L.orc_mel.restype = C.c_int
    L.orc_mel.argtypes = [P, fp, C.c_int, fp, C.c_int, C.POINTER(C.c_int)]
    L.orc_encode.argtypes = [P, fp, C.c_int, C.c_int, fp]
    L.orc_cross.argtypes = [P, fp, fp, fp]
    L.orc_encode_stem.argtypes = [P, fp, C.c_int, C.c_int, fp]
    L.orc_encode_post.argtypes = [P, fp, fp]
    L.orc_encode_layer.argtypes = [P, C.c_int, fp, C.POINTER(fp), C.POINTER(fp), fp]
    L.orc_decode_seq.argtypes = [P, fp, fp, C.POINTER(C.c_int), C.c_int, fp]
    L.orc_full.restype = P
    L.orc_full.argtypes = [P, C.POINTER(C.c_int), fp, C.c_char_p, C.c_char_p, fp, C.c_int,
                           C.POINTER(C.c_int)]
    L.orc_full_free.argtypes = [P]
    L.orc_full_n_segments.restype = C.c_int
    L.orc_full_n_segments.argtypes = [P]
    L.orc_full_segment_text.restype = C.c_char_p
    L.orc_full_segment_text.argtypes = [P, C.c_int]
    L.orc_full_segment_times.argtypes = [P, C.c_int, C.POINTER(C.c_int64)]
    L.orc_full_n_tokens.restype = C.c_int
    L.orc_full_n_tokens.argtypes = [P, C.c_int]
    L.orc_full_token.argtypes = [P, C.c_int, C.c_int, C.POINTER(C.c_int), fp,
                                 C.POINTER(C.c_int64)]
    L.orc_full_lang_id.restype = C.c_int
    L.orc_full_lang_id.argtypes = [P]
    L.orc_full_n_windows.restype = C.c_int
    L.orc_full_n_windows.argtypes = [P]
    L.orc_full_window_tokens.restype = C.c_int
    L.orc_full_window_tokens.argtypes = [P, C.c_int, C.POINTER(C.c_int), C.c_int]
    L.orc_process_logits.restype = None
    L.orc_process_logits.argtypes = [P, fp, C.POINTER(C.c_int), C.c_int, C.c_int, C.c_int,
                                     C.POINTER(C.c_int), fp, fp, fp, fp, C.POINTER(C.c_int), fp]
    L.orc_trace_enable.argtypes = [C.c_int]
    L.orc_trace_count.restype = C.c_int
    L.orc_trace_get.argtypes = [C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_double)]
    L.orc_trace_ctx.argtypes = [C.POINTER(C.c_int)]
    L.orc_trace_follow.argtypes = [C.POINTER(C.c_int), C.c_int]
    L.orc_trace_follow_break.restype = C.c_long
    L.orc_set_logits_tap.argtypes = [C.c_void_p, C.c_void_p]
    L.orc_prosody.restype = None
    L.orc_prosody.argtypes = [fp, C.c_int64, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, P]
    L.orc_resample.restype = C.c_long
    L.orc_resample.argtypes = [fp, C.c_long, C.c_int, C.c_int, fp, C.c_long]
    L.orc_clusterer_new.restype = P
    L.orc_clusterer_new.argtypes = [C.c_float]
    L.orc_clusterer_free.argtypes = [P]
    L.orc_clusterer_assign.restype = C.c_int
    L.orc_clusterer_assign.argtypes = [P, fp, C.c_int, C.c_char_p, C.c_int]
    _lib = L
    return L


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


@dataclass
class OToken:
    id: int
    tid: int
    p: float
    plog: float
    pt: float
    ptsum: float
    t0: int
    t1: int


@dataclass
class OSegment:
    t0: int
    t1: int
    text: str
    tokens: List[OToken] = field(default_factory=list)
    raw: bytes = b""  # segment text bytes as produced (may be partial UTF-8)


@dataclass
class FullOptions:
    strategy: int = 0
    best_of: int = 5
    beam_size: int = 5
    translate: bool = False
    no_timestamps: bool = False
    token_timestamps: bool = False
    suppress_nst: bool = False
    suppress_blank: bool = True
    tdrz: bool = False
    bench_fixed_steps: int = 0
    no_context: bool = True
    temperature: float = 0.0
    temperature_inc: float = 0.2
    entropy_thold: float = 2.4
    logprob_thold: float = -1.0
    no_speech_thold: float = 0.6
    max_initial_ts: float = 1.0
    length_penalty: float = -1.0
    thold_pt: float = 0.01
    thold_ptsum: float = 0.01
    language: str = "en"
    initial_prompt: Optional[str] = None

    @classmethod
    def service_defaults(cls, beam_size: int = 1) -> "FullOptions":
        """Parameters SttEngine::transcribe sets (src/stt_engine.cpp:204-243)
        with the Settings defaults of src/config.h (greedy when beam_size=1).
        best_of is set for greedy only (stt_engine.cpp:235-238); beam search
        keeps whisper_full_default_params' -1, i.e. one decoder at t > 0."""
        return cls(strategy=0 if beam_size <= 1 else 1, best_of=5 if beam_size <= 1 else -1,
                   beam_size=beam_size,
                   token_timestamps=True, suppress_nst=True, no_speech_thold=0.85,
                   entropy_thold=2.40, logprob_thold=-0.7, temperature=0.0, language="auto")


TRACE_KINDS = {1: "draw", 2: "argmax", 3: "assign", 4: "ts_mass", 5: "best", 6: "fallback",
               7: "no_speech", 8: "exact_tie", 9: "status"}


@dataclass
class TraceEv:
    """One float-sensitive decision of full() (mwx_oracle.cpp TraceKind):
    where it was taken (window seek, temperature index, step, decoder), what
    was decided (a, b) and the oracle-side margin it was decided by."""
    kind: str
    seek: int
    it: int
    step: int
    dec: int
    a: int
    b: int
    margin: float
    v: float
    forced: int = 0  # follow mode: the guide's outcome was taken over the oracle's own
    own_a: int = 0  # the oracle's own outcome (forced events)
    own_b: int = 0
    fmargin: float = 0.0  # how far the oracle's arithmetic is from the taken outcome
    lo: float = 0.0  # draws: the taken id's cumulative-probability interval [lo, hi)
    hi: float = 0.0

    def key(self):
        return (self.kind, self.seek, self.it, self.step, self.dec, self.a, self.b)


KIND_IDS = {v: k for k, v in TRACE_KINDS.items()}


def _read_trace() -> List[TraceEv]:
    L = lib()
    evs = []
    ints = (C.c_int * 10)()
    dbl = (C.c_double * 5)()
    for i in range(L.orc_trace_count()):
        L.orc_trace_get(i, ints, dbl)
        v = list(ints)
        evs.append(TraceEv(TRACE_KINDS[v[0]], *v[1:7], dbl[0], dbl[1], v[7], v[8], v[9],
                           dbl[2], dbl[3], dbl[4]))
    return evs


def trace_ctx():
    """(seek, temperature index, step, decoder) full() is at — read inside a
    full_external logits callback: the logits it asks for feed that decoder's
    decision at step + 1 (step -1: the prompt, shared by all decoders)."""
    v = (C.c_int * 4)()
    lib().orc_trace_ctx(v)
    return tuple(v)


def first_divergence(ta: List[TraceEv], tb: List[TraceEv]) -> Optional[int]:
    """Index of the first event whose decision differs between two traces
    (None if one is a prefix of the other and both have the same length)."""
    for i, (x, y) in enumerate(zip(ta, tb)):
        if x.key() != y.key():
            return i
    return None if len(ta) == len(tb) else min(len(ta), len(tb))


class Oracle:
    def __init__(self, path: str, exact: bool = False, threads: Optional[int] = None,
                 mxfp8: bool = False):
        L = lib()
        if threads:
            L.orc_set_threads(threads)
        self.h = L.orc_load(path.encode(), (ORC_EXACT if exact else 0) | (ORC_MXFP8 if mxfp8 else 0))
        if not self.h:
            raise RuntimeError(f"oracle failed to load {path}")
        hp = (C.c_int * 11)()
        L.orc_hparams(self.h, hp)
        self.hp = list(hp)
        sp = (C.c_int * 9)()
        L.orc_special(self.h, sp)
        (self.eot, self.sot, self.translate, self.transcribe, self.solm, self.prev, self.nosp,
         self.not_, self.beg) = list(sp)

    def close(self):
        if self.h:
            lib().orc_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def n_vocab(self):
        return self.hp[0]

    @property
    def n_mels(self):
        return self.hp[9]

    @property
    def d(self):
        return self.hp[2]

    @property
    def n_text_layer(self):
        return self.hp[8]

    def tensor(self, name: str) -> np.ndarray:
        """Loaded values of one tensor (quantized types: dequantized, f16-rounded)."""
        L = lib()
        n = L.orc_tensor(self.h, name.encode(), None, 0)
        if n < 0:
            raise KeyError(name)
        out = np.empty(n, np.float32)
        L.orc_tensor(self.h, name.encode(), _fp(out), n)
        return out

    def filters(self) -> np.ndarray:
        p = lib().orc_filters(self.h)
        return np.ctypeslib.as_array(p, shape=(self.n_mels * 201,)).reshape(self.n_mels, 201).copy()

    def token_str(self, i: int) -> str:
        return lib().orc_token_str(self.h, i).decode("utf-8", "replace")

    def token_bytes(self, i: int) -> bytes:
        return lib().orc_token_str(self.h, i)

    def mel(self, pcm: np.ndarray):
        pcm = np.ascontiguousarray(pcm, dtype=np.float32)
        n_len = (len(pcm) + 480000) // 160
        out = np.empty((self.n_mels, n_len), dtype=np.float32)
        org = C.c_int()
        r = lib().orc_mel(self.h, _fp(pcm), len(pcm), _fp(out), out.size, C.byref(org))
        assert r == n_len
        return out, org.value

    def encode(self, mel: np.ndarray, seek: int = 0) -> np.ndarray:
        mel = np.ascontiguousarray(mel, dtype=np.float32)
        out = np.empty((self.hp[1], self.d), dtype=np.float32)
        lib().orc_encode(self.h, _fp(mel), mel.shape[1], seek, _fp(out))
        return out

    def encode_stem(self, mel: np.ndarray, seek: int = 0) -> np.ndarray:
        """The conv stem's residual stream [n_ctx][d] (input of encoder layer 0)."""
        mel = np.ascontiguousarray(mel, dtype=np.float32)
        out = np.empty((self.hp[1], self.d), dtype=np.float32)
        lib().orc_encode_stem(self.h, _fp(mel), mel.shape[1], seek, out.ctypes.data_as(C.POINTER(C.c_float)))
        return out

    def encode_post(self, x: np.ndarray) -> np.ndarray:
        """The encoder output (ln_post) of a residual stream after the last layer."""
        x = np.ascontiguousarray(x, dtype=np.float32)
        out = np.empty_like(x)
        lib().orc_encode_post(self.h, _fp(x), _fp(out))
        return out

    def encode_layer(self, il: int, x: np.ndarray, ext=None, want_operands: bool = False):
        """Encoder layer il on the residual stream x [n_ctx][d]: returns the
        next residual stream, and with want_operands the four GEMM A operands
        it used (attn LN out, attention out, mlp LN out, GELU out). ext: up to
        four arrays (None entries: computed) that replace those operands."""
        n, d = self.hp[1], self.d
        x = np.ascontiguousarray(x, dtype=np.float32)
        shapes = [(n, d), (n, d), (n, d), (n, 4 * d)]
        ext_arr = [None if ext is None or ext[g] is None else
                   np.ascontiguousarray(ext[g], dtype=np.float32).reshape(shapes[g]) for g in range(4)]
        outs = [np.empty(sh, np.float32) for sh in shapes] if want_operands else [None] * 4
        FP = C.POINTER(C.c_float)
        ext_p = (FP * 4)(*[FP() if a is None else _fp(a) for a in ext_arr])
        out_p = (FP * 4)(*[FP() if a is None else _fp(a) for a in outs])
        y = np.empty((n, d), np.float32)
        lib().orc_encode_layer(self.h, il, _fp(x), ext_p, out_p, _fp(y))
        return (y, outs) if want_operands else y

    def cross(self, enc: np.ndarray):
        enc = np.ascontiguousarray(enc, dtype=np.float32)
        k = np.empty((self.n_text_layer, self.hp[1], self.d), dtype=np.float32)
        v = np.empty_like(k)
        lib().orc_cross(self.h, _fp(enc), _fp(k), _fp(v))
        return k, v

    def decode_seq(self, k, v, tokens) -> np.ndarray:
        toks = np.ascontiguousarray(tokens, dtype=np.int32)
        out = np.empty((len(toks), self.n_vocab), dtype=np.float32)
        lib().orc_decode_seq(self.h, _fp(np.ascontiguousarray(k)), _fp(np.ascontiguousarray(v)),
                             toks.ctypes.data_as(C.POINTER(C.c_int)), len(toks), _fp(out))
        return out

    def process_logits(self, raw, history, has_ts: bool, seek_delta: int, *,
                       suppress_blank=True, suppress_nst=False, no_timestamps=False, tdrz=False,
                       bench_fixed_steps=0, ts_mass_rule=True, temperature=0.0,
                       max_initial_ts=1.0):
        """whisper_process_logits + greedy whisper_sample_token on one raw
        logits row for a decoder whose sampled tokens are `history`; returns
        (logits, logprobs, probs, (id, tid, p, plog, pt, ptsum))."""
        V = self.n_vocab
        raw = np.ascontiguousarray(raw, np.float32)
        assert raw.shape == (V,)
        hist = np.ascontiguousarray(history, np.int32)
        ip = (C.c_int * 6)(int(suppress_blank), int(suppress_nst), int(no_timestamps), int(tdrz),
                           int(bench_fixed_steps), 0 if ts_mass_rule else 1)
        fpv = (C.c_float * 2)(temperature, max_initial_ts)
        lg, lp, pr = (np.empty(V, np.float32) for _ in range(3))
        ti = (C.c_int * 2)()
        tf = (C.c_float * 4)()
        lib().orc_process_logits(self.h, _fp(raw), hist.ctypes.data_as(C.POINTER(C.c_int)),
                                 len(hist), int(has_ts), int(seek_delta), ip, fpv, _fp(lg),
                                 _fp(lp), _fp(pr), ti, tf)
        return lg, lp, pr, (ti[0], ti[1], tf[0], tf[1], tf[2], tf[3])

    def traced(self, fn, *args, **kw):
        """(fn(*args, **kw), [TraceEv]) with the decision trace recorded."""
        L = lib()
        L.orc_trace_enable(1)
        try:
            out = fn(*args, **kw)
            return out, _read_trace()
        finally:
            L.orc_trace_enable(0)

    def traced_follow(self, guide: List[TraceEv], pcm: np.ndarray, opt: FullOptions, tap=None):
        """full() on the oracle's own logits in follow mode: at every traced
        decision it takes the outcome `guide` recorded (events whose outcome
        differs come back forced, with the oracle's own outcome and its
        distance to the guide's). tap(tokens, logits_last) sees every row the
        oracle decodes. Returns ((rc, segs, lang, windows), [TraceEv], break)
        where break is the index at which the run stopped following (None:
        followed to the end)."""
        L = lib()
        flat = (C.c_int * (7 * len(guide)))(*[x for e in guide for x in
                                              (KIND_IDS[e.kind], e.seek, e.it, e.step, e.dec,
                                               e.a, e.b)])
        cb = None
        if tap is not None:
            V = self.n_vocab

            def _tap(user, toks, n, lg):
                tap([toks[i] for i in range(n)],
                    np.ctypeslib.as_array(lg, shape=(V,)).copy())

            cb = TAP_LOGITS(_tap)
            L.orc_set_logits_tap(C.cast(cb, C.c_void_p), None)
        L.orc_trace_follow(flat, len(guide))
        L.orc_trace_enable(1)
        try:
            out = self.full(pcm, opt)
            brk = L.orc_trace_follow_break()
            return out, _read_trace(), (None if brk < 0 else int(brk))
        finally:
            L.orc_trace_enable(0)
            L.orc_trace_follow(None, 0)
            L.orc_set_logits_tap(None, None)

    def full_external(self, pcm: np.ndarray, opt: FullOptions, encode_fn, logits_fn):
        """full() with every decode answered by callbacks: encode_fn(seek) and
        logits_fn(tokens) -> last-token logits [n_vocab] (e.g. from the device)."""
        V = self.n_vocab

        def _enc(user, seek):
            encode_fn(int(seek))

        def _lg(user, toks, n, out):
            lg = logits_fn([toks[i] for i in range(n)])
            C.memmove(out, np.ascontiguousarray(lg, np.float32).ctypes.data, V * 4)

        enc_cb = EXT_ENC(_enc)
        lg_cb = EXT_LOGITS(_lg)
        lib().orc_set_external(C.cast(enc_cb, C.c_void_p), C.cast(lg_cb, C.c_void_p), None)
        try:
            return self.full(pcm, opt)
        finally:
            lib().orc_set_external(None, None, None)

    def full(self, pcm: np.ndarray, opt: FullOptions):
        pcm = np.ascontiguousarray(pcm, dtype=np.float32)
        ip = (C.c_int * 11)(opt.strategy, opt.best_of, opt.beam_size, int(opt.translate),
                            int(opt.no_timestamps), int(opt.token_timestamps),
                            int(opt.suppress_nst), int(opt.suppress_blank), int(opt.tdrz),
                            opt.bench_fixed_steps, int(opt.no_context))
        fpv = (C.c_float * 9)(opt.temperature, opt.temperature_inc, opt.entropy_thold,
                              opt.logprob_thold, opt.no_speech_thold, opt.max_initial_ts,
                              opt.length_penalty, opt.thold_pt, opt.thold_ptsum)
        rc = C.c_int()
        L = lib()
        r = L.orc_full(self.h, ip, fpv, opt.language.encode(),
                       opt.initial_prompt.encode() if opt.initial_prompt else None, _fp(pcm),
                       len(pcm), C.byref(rc))
        segs = []
        for i in range(L.orc_full_n_segments(r)):
            t = (C.c_int64 * 2)()
            L.orc_full_segment_times(r, i, t)
            raw = L.orc_full_segment_text(r, i)
            seg = OSegment(t[0], t[1], raw.decode("utf-8", "replace"), raw=raw)
            for j in range(L.orc_full_n_tokens(r, i)):
                ids = (C.c_int * 2)()
                f = (C.c_float * 4)()
                tt = (C.c_int64 * 2)()
                L.orc_full_token(r, i, j, ids, f, tt)
                seg.tokens.append(OToken(ids[0], ids[1], f[0], f[1], f[2], f[3], tt[0], tt[1]))
            segs.append(seg)
        lang = L.orc_full_lang_id(r)
        windows = []
        for w in range(L.orc_full_n_windows(r)):
            buf = (C.c_int * 1024)()
            n = L.orc_full_window_tokens(r, w, buf, 1024)
            windows.append(list(buf)[:n])
        L.orc_full_free(r)
        return rc.value, segs, lang, windows


# ---------------------------------------------------------------------------
# Segment prosody / speaker clustering (prosody_oracle.cpp; src/
# prosody_extractor.cpp, src/speaker_cluster.cpp)
# ---------------------------------------------------------------------------
class ProsodyRec(C.Structure):
    """mwx_prosody / AffectiveTags (gender 0 '?', 1 'M', 2 'F'; emotion 0
    neutral, 1 excited, 2 angry, 3 sad)."""
    _fields_ = [(n, C.c_float) for n in ("pitch_mean", "pitch_std", "energy_mean", "energy_std",
                                         "spectral_centroid", "zero_crossing_rate", "arousal",
                                         "valence")] + [
        ("speaker_vec", C.c_float * 8), ("gender", C.c_int), ("emotion", C.c_int),
        ("serial_runs", C.c_int), ("reserved", C.c_int)]


PROSODY_FLOATS = ("pitch_mean", "pitch_std", "energy_mean", "energy_std", "spectral_centroid",
                  "zero_crossing_rate", "arousal", "valence")


def prosody_key(r) -> tuple:
    """Everything the reference returns, as exact bit patterns (serial_runs,
    a diagnostic, excluded)."""
    f = [getattr(r, n) for n in PROSODY_FLOATS] + list(r.speaker_vec)
    return tuple(np.array(f, np.float32).view(np.uint32).tolist()) + (r.gender, r.emotion)


def prosody(pcm: Optional[np.ndarray], sample_rate: int = 16000, lpf_alpha: float = 0.07,
            gender_threshold: float = 170.0, min_pitch: float = 60.0,
            max_pitch: float = 500.0) -> ProsodyRec:
    out = ProsodyRec()
    if pcm is None:
        lib().orc_prosody(None, 0, sample_rate, lpf_alpha, gender_threshold, min_pitch, max_pitch,
                          C.byref(out))
        return out
    a = np.ascontiguousarray(pcm, np.float32)
    lib().orc_prosody(_fp(a), len(a), sample_rate, lpf_alpha, gender_threshold, min_pitch,
                      max_pitch, C.byref(out))
    return out


class Clusterer:
    def __init__(self, threshold: float = 0.88):
        self.h = lib().orc_clusterer_new(threshold)

    def assign(self, vec) -> str:
        a = np.ascontiguousarray(vec, np.float32)
        buf = C.create_string_buffer(64)
        lib().orc_clusterer_assign(self.h, _fp(a), len(a), buf, 64)
        return buf.value.decode()

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_clusterer_free(self.h)
            self.h = None



# ---------------------------------------------------------------------------
# Resampling (resample_oracle.cpp; SttEngine::resample_audio, src/stt_engine.cpp:87-106)
# ---------------------------------------------------------------------------
def resample(pcm: np.ndarray, src_rate: int, dst_rate: int) -> Optional[np.ndarray]:
    """libsamplerate src_simple(SRC_SINC_FASTEST, 1, end_of_input = 0) restated;
    None where the reference returns an empty buffer (same rate, empty input)
    and keeps the original."""
    a = np.ascontiguousarray(pcm, np.float32)
    cap = int(len(a) * (dst_rate / src_rate)) + 100
    out = np.empty(max(cap, 1), np.float32)
    n = lib().orc_resample(_fp(a), len(a), src_rate, dst_rate, _fp(out), cap)
    if n < 0:
        raise ValueError(f"orc_resample failed ({n})")
    return out[:n].copy() if n > 0 else None
