"""ctypes binding of the mwx C ABI (include/mwx.h, include/mwx_test.h).

Mirrors the whisper.h subset the reference service binds in
src/stt_engine.cpp (context / state lifecycle, whisper_full_with_state, segment
and token getters) plus the batched entry point mwx_full_batch. Used by the
tests and by bench.py; the service itself binds the same ABI from C++
(see INTEGRATION.md).

The library is loaded from this directory (built in-tree by
__graft_entry__.build()); a missing library raises immediately — there is no
CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MWX_LIB: an alternative build of the library (same ABI; A/B measurements)
LIB_PATH = os.environ.get("MWX_LIB") or os.path.join(HERE, "libmwx.so")

GGML_F16 = 1
GGML_BF16 = 30
# ggml block-quantized types written by whisper.cpp's quantize tool
GGML_Q4_0 = 2
GGML_Q4_1 = 3
GGML_Q5_0 = 6
GGML_Q5_1 = 7
GGML_Q8_0 = 8
GGML_Q2_K = 10
GGML_Q3_K = 11
GGML_Q4_K = 12
GGML_Q5_K = 13
GGML_Q6_K = 14
GGML_QUANT_TYPES = {"q4_0": GGML_Q4_0, "q4_1": GGML_Q4_1, "q5_0": GGML_Q5_0,
                    "q5_1": GGML_Q5_1, "q8_0": GGML_Q8_0, "q2_k": GGML_Q2_K,
                    "q3_k": GGML_Q3_K, "q4_k": GGML_Q4_K, "q5_k": GGML_Q5_K,
                    "q6_k": GGML_Q6_K}
SAMPLING_GREEDY = 0
SAMPLING_BEAM_SEARCH = 1


class ContextParams(C.Structure):
    _fields_ = [("use_gpu", C.c_bool), ("flash_attn", C.c_bool), ("gpu_device", C.c_int),
                ("compute", C.c_int)]


COMPUTE_MODEL = 0
COMPUTE_MXFP8 = 1  # encoder / cross-K/V GEMMs on MX-fp8 MFMA


class TokenData(C.Structure):
    _fields_ = [
        ("id", C.c_int32), ("tid", C.c_int32), ("p", C.c_float), ("plog", C.c_float),
        ("pt", C.c_float), ("ptsum", C.c_float), ("t0", C.c_int64), ("t1", C.c_int64),
        ("t_dtw", C.c_int64), ("vlen", C.c_float),
    ]


class _Greedy(C.Structure):
    _fields_ = [("best_of", C.c_int)]


class _Beam(C.Structure):
    _fields_ = [("beam_size", C.c_int), ("patience", C.c_float)]


ABORT_CB = C.CFUNCTYPE(C.c_bool, C.c_void_p)


class FullParams(C.Structure):
    _fields_ = [
        ("strategy", C.c_int), ("n_threads", C.c_int), ("n_max_text_ctx", C.c_int),
        ("offset_ms", C.c_int), ("duration_ms", C.c_int),
        ("translate", C.c_bool), ("no_context", C.c_bool), ("no_timestamps", C.c_bool),
        ("single_segment", C.c_bool), ("print_special", C.c_bool), ("print_progress", C.c_bool),
        ("print_realtime", C.c_bool), ("print_timestamps", C.c_bool),
        ("token_timestamps", C.c_bool), ("thold_pt", C.c_float), ("thold_ptsum", C.c_float),
        ("max_len", C.c_int), ("split_on_word", C.c_bool), ("max_tokens", C.c_int),
        ("audio_ctx", C.c_int), ("tdrz_enable", C.c_bool),
        ("initial_prompt", C.c_char_p), ("prompt_tokens", C.POINTER(C.c_int32)),
        ("prompt_n_tokens", C.c_int),
        ("language", C.c_char_p), ("detect_language", C.c_bool),
        ("suppress_blank", C.c_bool), ("suppress_nst", C.c_bool),
        ("temperature", C.c_float), ("max_initial_ts", C.c_float), ("length_penalty", C.c_float),
        ("temperature_inc", C.c_float), ("entropy_thold", C.c_float),
        ("logprob_thold", C.c_float), ("no_speech_thold", C.c_float),
        ("greedy", _Greedy), ("beam_search", _Beam),
        ("abort_callback", ABORT_CB), ("abort_callback_user_data", C.c_void_p),
        ("bench_fixed_steps", C.c_int),
    ]


class ProsodyParams(C.Structure):
    """mwx_prosody_params = the reference's ProsodyOptions
    (src/prosody_extractor.h:21-27)."""
    _fields_ = [("lpf_alpha", C.c_float), ("gender_threshold", C.c_float),
                ("min_pitch", C.c_float), ("max_pitch", C.c_float)]


class Prosody(C.Structure):
    """mwx_prosody = AffectiveTags (src/prosody_extractor.h:6-18)."""
    _fields_ = [(n, C.c_float) for n in ("pitch_mean", "pitch_std", "energy_mean", "energy_std",
                                         "spectral_centroid", "zero_crossing_rate", "arousal",
                                         "valence")] + [
        ("speaker_vec", C.c_float * 8), ("gender", C.c_int), ("emotion", C.c_int),
        ("serial_runs", C.c_int), ("reserved", C.c_int)]

    @property
    def gender_proxy(self) -> str:
        return ("?", "M", "F")[self.gender]

    @property
    def emotion_proxy(self) -> str:
        return ("neutral", "excited", "angry", "sad")[self.emotion]


_lib = None


def lib() -> C.CDLL:
    """Loads libmwx.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"mwx: {LIB_PATH} not built (run __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    P = C.c_void_p
    L.mwx_context_default_params.restype = ContextParams
    L.mwx_init_from_file_with_params.restype = P
    L.mwx_init_from_file_with_params.argtypes = [C.c_char_p, ContextParams]
    L.mwx_init_state.restype = P
    L.mwx_init_state.argtypes = [P]
    L.mwx_free_state.argtypes = [P]
    L.mwx_free.argtypes = [P]
    L.mwx_full_default_params.restype = FullParams
    L.mwx_full_default_params.argtypes = [C.c_int]
    L.mwx_full_with_state.restype = C.c_int
    L.mwx_full_with_state.argtypes = [P, P, FullParams, C.POINTER(C.c_float), C.c_int]
    fpp = C.POINTER(C.c_float)
    L.mwx_device_buffer.restype = fpp
    L.mwx_device_buffer.argtypes = [P, C.c_size_t]
    L.mwx_device_upload.restype = C.c_int
    L.mwx_device_upload.argtypes = [P, fpp, fpp, C.c_size_t]
    L.mwx_device_buffer_free.restype = None
    L.mwx_device_buffer_free.argtypes = [P, fpp]
    L.mwx_full_batch_pcm16.restype = C.c_int
    L.mwx_full_batch_pcm16.argtypes = [P, C.POINTER(P), FullParams, C.POINTER(C.c_void_p),
                                       C.POINTER(C.c_int), C.c_int]
    L.mwx_full_batch.restype = C.c_int
    L.mwx_full_batch.argtypes = [P, C.POINTER(P), FullParams, C.POINTER(C.POINTER(C.c_float)),
                                 C.POINTER(C.c_int), C.c_int]
    L.mwx_full_n_segments_from_state.restype = C.c_int
    L.mwx_full_n_segments_from_state.argtypes = [P]
    L.mwx_full_get_segment_text_from_state.restype = C.c_char_p
    L.mwx_full_get_segment_text_from_state.argtypes = [P, C.c_int]
    for n in ("t0", "t1"):
        f = getattr(L, f"mwx_full_get_segment_{n}_from_state")
        f.restype = C.c_int64
        f.argtypes = [P, C.c_int]
    L.mwx_full_get_segment_speaker_turn_next_from_state.restype = C.c_bool
    L.mwx_full_get_segment_speaker_turn_next_from_state.argtypes = [P, C.c_int]
    L.mwx_full_get_segment_no_speech_prob_from_state.restype = C.c_float
    L.mwx_full_get_segment_no_speech_prob_from_state.argtypes = [P, C.c_int]
    L.mwx_full_n_tokens_from_state.restype = C.c_int
    L.mwx_full_n_tokens_from_state.argtypes = [P, C.c_int]
    L.mwx_full_get_token_data_from_state.restype = TokenData
    L.mwx_full_get_token_data_from_state.argtypes = [P, C.c_int, C.c_int]
    L.mwx_full_lang_id_from_state.restype = C.c_int
    L.mwx_full_lang_id_from_state.argtypes = [P]
    L.mwx_token_to_str.restype = C.c_char_p
    L.mwx_token_to_str.argtypes = [P, C.c_int32]
    for n in ("eot", "sot", "beg", "not", "nosp", "transcribe", "translate"):
        f = getattr(L, f"mwx_token_{n}")
        f.restype = C.c_int32
        f.argtypes = [P]
    for n in ("n_vocab", "n_text_ctx", "n_audio_ctx", "n_mels", "is_multilingual", "model_wtype"):
        f = getattr(L, f"mwx_{n}")
        f.restype = C.c_int
        f.argtypes = [P]
    L.mwx_model_quantize.restype = C.c_int
    L.mwx_model_quantize.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
    L.mwx_write_synthetic_model.restype = C.c_int
    L.mwx_write_synthetic_model.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_uint64]
    L.mwx_perf_enable.restype = None
    L.mwx_perf_enable.argtypes = [P, C.c_char_p]
    L.mwx_perf_read.restype = C.c_int
    L.mwx_perf_read.argtypes = [P, C.POINTER(C.c_double), C.POINTER(C.c_int)]
    L.mwx_perf_read_class.restype = C.c_int
    L.mwx_perf_read_class.argtypes = [P, C.c_char_p, C.POINTER(C.c_double), C.POINTER(C.c_int)]
    L.mwx_tokenize.restype = C.c_int
    L.mwx_tokenize.argtypes = [P, C.c_char_p, C.POINTER(C.c_int32), C.c_int]
    L.mwx_test_mel.restype = C.c_int
    L.mwx_test_mel.argtypes = [P, P, C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_float), C.c_long]
    L.mwx_test_encode.restype = C.c_int
    L.mwx_test_encode.argtypes = [P, P, C.POINTER(C.c_float), C.c_int, C.c_int,
                                  C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float)]
    L.mwx_test_decode.restype = C.c_int
    L.mwx_test_decode.argtypes = [P, P, C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_float)]
    L.mwx_test_decode_last.restype = C.c_int
    L.mwx_test_decode_last.argtypes = [P, P, C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_float)]
    L.mwx_test_decode_last_prefill.restype = C.c_int
    L.mwx_test_decode_last_prefill.argtypes = [P, P, C.POINTER(C.c_int), C.c_int,
                                               C.POINTER(C.c_float)]
    L.mwx_test_self_kv.restype = C.c_int
    L.mwx_test_self_kv.argtypes = [P, C.c_int, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float)]
    L.mwx_test_dequantize.restype = C.c_int
    L.mwx_test_dequantize.argtypes = [C.c_int, C.c_void_p, C.c_long, C.POINTER(C.c_float)]
    L.mwx_test_decode_counters.restype = C.c_int
    L.mwx_test_decode_counters.argtypes = [P, C.POINTER(C.c_long), C.POINTER(C.c_long), C.c_int]
    L.mwx_test_encode_dump.restype = C.c_int
    L.mwx_test_encode_dump.argtypes = [P, P, C.POINTER(C.c_float), C.c_int, C.c_int,
                                       C.POINTER(C.c_float), C.POINTER(C.c_void_p)]
    L.mwx_test_window_counters.restype = C.c_int
    L.mwx_test_window_counters.argtypes = [P, C.POINTER(C.c_long), C.POINTER(C.c_long),
                                           C.POINTER(C.c_long), C.c_int]
    L.mwx_test_runahead_fallbacks.restype = C.c_long
    L.mwx_test_runahead_fallbacks.argtypes = [P, C.c_int]
    L.mwx_test_set_xattn_mfs.restype = C.c_int
    L.mwx_test_set_xattn_mfs.argtypes = [C.c_int]
    L.mwx_test_set_dec_shared.restype = C.c_int
    L.mwx_test_set_dec_shared.argtypes = [C.c_int]
    L.mwx_test_set_gemm_8ph.restype = C.c_int
    L.mwx_test_set_ln_fold.restype = C.c_int
    L.mwx_test_set_ln_fold.argtypes = [C.c_int]
    L.mwx_test_mx_widen.restype = C.c_int
    L.mwx_test_mx_widen.argtypes = [P, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    L.mwx_test_set_gemm_8ph.argtypes = [C.c_int]
    L.mwx_test_set_ra_mismatch.restype = C.c_long
    L.mwx_test_set_ra_mismatch.argtypes = [C.c_long]
    u8p = C.POINTER(C.c_uint8)
    L.mwx_test_xattn_mx.restype = C.c_int
    L.mwx_test_xattn_mx.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, fpp, u8p, u8p,
                                    u8p, u8p, fpp]
    L.mwx_test_sample_draws.restype = C.c_int
    L.mwx_test_sample_draws.argtypes = [P, fpp, fpp, C.c_int, C.c_int, C.POINTER(C.c_double),
                                        C.POINTER(C.c_int), C.c_int, C.c_int, C.c_int,
                                        C.POINTER(C.c_int), C.POINTER(C.c_double)]
    L.mwx_resample_max_frames.restype = C.c_long
    L.mwx_resample_max_frames.argtypes = [C.c_int, C.c_int, C.c_int]
    L.mwx_resample.restype = C.c_int
    L.mwx_resample.argtypes = [P, P, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int]
    L.mwx_prosody_default_params.restype = ProsodyParams
    L.mwx_prosody_default_params.argtypes = []
    i64p = C.POINTER(C.c_int64)
    L.mwx_prosody_batch.restype = C.c_int
    L.mwx_prosody_batch.argtypes = [P, P, fpp, C.c_int64, i64p, i64p, C.c_int, C.c_int,
                                    C.POINTER(ProsodyParams), C.POINTER(Prosody)]
    L.mwx_prosody_batch_device.restype = C.c_int
    L.mwx_prosody_batch_device.argtypes = [P, P, C.c_void_p, C.c_void_p, C.c_int, C.c_int64,
                                           C.c_int, C.POINTER(ProsodyParams), C.c_void_p]
    _lib = L
    return L


def fptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class DevicePCM:
    """f32 PCM in a device buffer of the context's GPU (mwx_device_buffer)."""

    def __init__(self, ctx: "Context", pcm: np.ndarray):
        a = np.ascontiguousarray(pcm, dtype=np.float32)
        self.ctx, self.n = ctx, len(a)
        self.ptr = lib().mwx_device_buffer(ctx.ctx, max(1, self.n))
        if not self.ptr:
            raise MemoryError("mwx_device_buffer failed")
        if lib().mwx_device_upload(ctx.ctx, self.ptr, fptr(a), self.n) != 0:
            raise RuntimeError("mwx_device_upload failed")

    def free(self):
        if self.ptr:
            lib().mwx_device_buffer_free(self.ctx.ctx, self.ptr)
            self.ptr = None


def write_synthetic_model(path: str, arch: str, wtype: int = GGML_F16, seed: int = 0) -> None:
    rc = lib().mwx_write_synthetic_model(path.encode(), arch.encode(), wtype, seed)
    if rc != 0:
        raise RuntimeError(f"mwx_write_synthetic_model failed ({rc})")


def set_xattn_mfs(on: Optional[bool]) -> int:
    """mwx_test_set_xattn_mfs: the MX-fp8 grouped cross-attention on MFMA
    (True) or v_dot2 (False); None: the MWX_XATTN_MFS default."""
    return lib().mwx_test_set_xattn_mfs(-1 if on is None else int(bool(on)))


def set_dec_shared(on: Optional[bool]) -> int:
    """mwx_test_set_dec_shared: decode GEMMs at > 64 rows through the
    shared-A kernels (True) or the per-strip grids (False); None: the
    MWX_DEC_SHARED default."""
    return lib().mwx_test_set_dec_shared(-1 if on is None else int(bool(on)))


def set_gemm_8ph(on: Optional[bool]) -> int:
    """mwx_test_set_gemm_8ph: the encoder GEMM's 8-phase main loop (True) or
    the 2-stage ring (False); None: the MWX_GEMM_8PH default."""
    return lib().mwx_test_set_gemm_8ph(-1 if on is None else int(bool(on)))


def set_ln_fold(on: Optional[bool]) -> int:
    """mwx_test_set_ln_fold: the decode LayerNorms folded into the next
    split-K GEMM at one row (True) or launched separately (False); None: the
    MWX_LN_FOLD default (on)."""
    return lib().mwx_test_set_ln_fold(-1 if on is None else int(bool(on)))


def set_ra_mismatch(step: Optional[int]) -> int:
    """mwx_test_set_ra_mismatch: treat run-ahead step `step` of later attempts
    as a device/host disagreement (None: back to MWX_TEST_RA_MISMATCH, -1: off)."""
    return lib().mwx_test_set_ra_mismatch(-2 if step is None else int(step))


def dequantize(qtype: int, raw: bytes, n: int) -> np.ndarray:
    """mwx_test_dequantize: the engine's load-time dequantizer (host only)."""
    out = np.empty(n, np.float32)
    buf = np.frombuffer(raw, np.uint8)
    rc = lib().mwx_test_dequantize(qtype, buf.ctypes.data, n, out.ctypes.data_as(C.POINTER(C.c_float)))
    if rc != 0:
        raise ValueError(f"mwx_test_dequantize({qtype}, n={n}) returned {rc}")
    return out


def quantize_model(in_path: str, out_path: str, qtype: int) -> None:
    """mwx_model_quantize: whisper.cpp `quantize` tool rules."""
    rc = lib().mwx_model_quantize(in_path.encode(), out_path.encode(), qtype)
    if rc != 0:
        raise RuntimeError(f"mwx_model_quantize failed ({rc})")


def synth_pcm16(k: int, n: int = 480000, sr: int = 16000) -> np.ndarray:
    """Deterministic synthetic speech-like clip: 3 harmonic
    voices (F0 90-260 Hz, 8 harmonics with 1/h amplitude), 2-6 Hz amplitude
    modulation, white noise at -30 dBFS, peak 0.5, int16."""
    rng = np.random.default_rng(0x5EED0000 + k)
    t = np.arange(n, dtype=np.float64) / sr
    sig = np.zeros(n)
    for _ in range(3):
        f0 = rng.uniform(90.0, 260.0)
        rate = rng.uniform(2.0, 6.0)
        ph = rng.uniform(0, 2 * np.pi, size=9)
        voice = sum(np.sin(2 * np.pi * h * f0 * t + ph[h]) / h for h in range(1, 9))
        env = 0.5 * (1.0 + np.sin(2 * np.pi * rate * t + ph[0]))
        sig += env * voice
    sig /= np.max(np.abs(sig))
    sig += rng.normal(0.0, 10 ** (-30 / 20), size=n)
    sig *= 0.5 / np.max(np.abs(sig))
    return np.round(sig * 32767).astype(np.int16)


def pcm16_to_f32(pcm16: np.ndarray) -> np.ndarray:
    """SttEngine::transcribe_pcm16 conversion (src/stt_engine.cpp:123)."""
    return (pcm16.astype(np.float32) / np.float32(32768.0)).astype(np.float32)


@dataclass
class Token:
    id: int
    tid: int
    p: float
    plog: float
    pt: float
    ptsum: float
    t0: int
    t1: int
    text: str


@dataclass
class Segment:
    t0: int
    t1: int
    text: str
    no_speech_prob: float
    speaker_turn_next: bool
    tokens: List[Token] = field(default_factory=list)


class Context:
    """mwx_context + a pool of mwx_state objects."""

    def __init__(self, model_path: str, device: int = 0, compute: int = COMPUTE_MODEL):
        L = lib()
        cp = L.mwx_context_default_params()
        cp.gpu_device = device
        cp.compute = compute
        self.ctx = L.mwx_init_from_file_with_params(model_path.encode(), cp)
        if not self.ctx:
            raise RuntimeError(f"mwx_init_from_file_with_params failed for {model_path}")
        self.states: List[int] = []

    def close(self):
        L = lib()
        for s in self.states:
            L.mwx_free_state(s)
        self.states = []
        if self.ctx:
            L.mwx_free(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def state(self, i: int = 0) -> int:
        while len(self.states) <= i:
            s = lib().mwx_init_state(self.ctx)
            if not s:
                raise RuntimeError("mwx_init_state failed")
            self.states.append(s)
        return self.states[i]

    @staticmethod
    def default_params(strategy: int = SAMPLING_GREEDY) -> FullParams:
        return lib().mwx_full_default_params(strategy)

    def full(self, pcm: np.ndarray, params: FullParams, state_index: int = 0) -> int:
        pcm = np.ascontiguousarray(pcm, dtype=np.float32)
        return lib().mwx_full_with_state(self.ctx, self.state(state_index), params, fptr(pcm),
                                         len(pcm))

    def full_batch(self, pcms: Sequence[np.ndarray], params: FullParams) -> int:
        return self.full_batch_states(pcms, params, range(len(pcms)))

    def full_batch_pcm16(self, pcms: Sequence[np.ndarray], params: FullParams) -> int:
        """mwx_full_batch_pcm16: int16 PCM converted on the device."""
        n = len(pcms)
        arrs = [np.ascontiguousarray(p, dtype=np.int16) for p in pcms]
        states = (C.c_void_p * n)(*[self.state(i) for i in range(n)])
        ptrs = (C.c_void_p * n)(*[a.ctypes.data for a in arrs])
        lens = (C.c_int * n)(*[len(a) for a in arrs])
        self._keep = arrs
        return lib().mwx_full_batch_pcm16(self.ctx, states, params, ptrs, lens, n)

    def full_batch_states(self, pcms: Sequence[np.ndarray], params: FullParams,
                          state_indices: Sequence[int]) -> int:
        n = len(pcms)
        arrs = [np.ascontiguousarray(p, dtype=np.float32) for p in pcms]
        states = (C.c_void_p * n)(*[self.state(i) for i in state_indices])
        ptrs = (C.POINTER(C.c_float) * n)(*[fptr(a) for a in arrs])
        lens = (C.c_int * n)(*[len(a) for a in arrs])
        self._keep = arrs
        return lib().mwx_full_batch(self.ctx, states, params, ptrs, lens, n)

    def upload(self, pcm: np.ndarray) -> "DevicePCM":
        """Copies PCM into a buffer on this context's GPU (HBM-resident input)."""
        return DevicePCM(self, pcm)

    def full_batch_device(self, bufs: Sequence["DevicePCM"], params: FullParams,
                          state0: int = 0) -> int:
        """Batch over PCM already resident in this GPU's memory: no PCIe transfer.
        Clip i runs on state state0 + i (state0 owns the batch's workspace and
        stream, so batches on disjoint state ranges may run concurrently)."""
        n = len(bufs)
        states = (C.c_void_p * n)(*[self.state(state0 + i) for i in range(n)])
        ptrs = (C.POINTER(C.c_float) * n)(*[b.ptr for b in bufs])
        ln = (C.c_int * n)(*[b.n for b in bufs])
        return lib().mwx_full_batch(self.ctx, states, params, ptrs, ln, n)

    def segments(self, state_index: int = 0) -> List[Segment]:
        L = lib()
        s = self.state(state_index)
        out = []
        for i in range(L.mwx_full_n_segments_from_state(s)):
            seg = Segment(
                t0=L.mwx_full_get_segment_t0_from_state(s, i),
                t1=L.mwx_full_get_segment_t1_from_state(s, i),
                text=L.mwx_full_get_segment_text_from_state(s, i).decode("utf-8", "replace"),
                no_speech_prob=L.mwx_full_get_segment_no_speech_prob_from_state(s, i),
                speaker_turn_next=L.mwx_full_get_segment_speaker_turn_next_from_state(s, i),
            )
            for j in range(L.mwx_full_n_tokens_from_state(s, i)):
                td = L.mwx_full_get_token_data_from_state(s, i, j)
                seg.tokens.append(Token(td.id, td.tid, td.p, td.plog, td.pt, td.ptsum, td.t0,
                                        td.t1, L.mwx_token_to_str(self.ctx, td.id).decode(
                                            "utf-8", "replace")))
            out.append(seg)
        return out

    def token_records(self, state_index: int = 0) -> List[tuple]:
        """(id, t0, t1, p) of every token of every segment, in order: the
        per-token whisper.h accessors only (no text), for the gather."""
        L = lib()
        s = self.state(state_index)
        out = []
        for i in range(L.mwx_full_n_segments_from_state(s)):
            for j in range(L.mwx_full_n_tokens_from_state(s, i)):
                td = L.mwx_full_get_token_data_from_state(s, i, j)
                out.append((td.id, td.t0, td.t1, td.p))
        return out

    def lang_id(self, state_index: int = 0) -> int:
        return lib().mwx_full_lang_id_from_state(self.state(state_index))

    # ---- per-stage test entry points ----
    def hparam(self, name: str) -> int:
        return getattr(lib(), f"mwx_{name}")(self.ctx)

    def token(self, name: str) -> int:
        """special token id: eot, sot, beg, not, nosp, transcribe, translate"""
        return getattr(lib(), f"mwx_token_{name}")(self.ctx)

    def test_mel(self, pcm: np.ndarray, state_index: int = 0) -> np.ndarray:
        pcm = np.ascontiguousarray(pcm, dtype=np.float32)
        n_mels = self.hparam("n_mels")
        n_len = (len(pcm) + 480000) // 160
        out = np.empty((n_mels, n_len), dtype=np.float32)
        r = lib().mwx_test_mel(self.ctx, self.state(state_index), fptr(pcm), len(pcm), fptr(out),
                               out.size)
        if r != n_len:
            raise RuntimeError(f"mwx_test_mel returned {r}")
        return out

    def prosody_batch(self, pcm: np.ndarray, starts, lens, sample_rate: int = 16000,
                      params: Optional[ProsodyParams] = None, state_index: int = 0):
        """mwx_prosody_batch: prosody of segments [starts[i], starts[i] + lens[i])
        of pcm (a numpy f32 array or a DevicePCM)."""
        st = np.ascontiguousarray(starts, np.int64)
        ln = np.ascontiguousarray(lens, np.int64)
        out = (Prosody * max(1, len(st)))()
        if isinstance(pcm, DevicePCM):
            ptr, n = pcm.ptr, pcm.n
        else:
            a = np.ascontiguousarray(pcm, np.float32)
            ptr, n = fptr(a), len(a)
        p = params if params is not None else lib().mwx_prosody_default_params()
        rc = lib().mwx_prosody_batch(self.ctx, self.state(state_index), ptr, n,
                                     st.ctypes.data_as(C.POINTER(C.c_int64)),
                                     ln.ctypes.data_as(C.POINTER(C.c_int64)), len(st),
                                     sample_rate, C.byref(p), out)
        if rc != 0:
            raise RuntimeError(f"mwx_prosody_batch failed ({rc})")
        return list(out)[:len(st)]

    def resample(self, pcm, src_rate: int, dst_rate: int = 16000, state_index: int = 0):
        """mwx_resample (SttEngine::resample_audio on the GPU): the 16 kHz
        samples, or None where the reference returns an empty buffer (equal
        rates, empty input). `pcm` may be a numpy array or a DevicePCM."""
        L = lib()
        if isinstance(pcm, DevicePCM):
            ptr, n = pcm.ptr, pcm.n
        else:
            a = np.ascontiguousarray(pcm, np.float32)
            ptr, n = a.ctypes.data, len(a)
        cap = L.mwx_resample_max_frames(n, src_rate, dst_rate)
        out = np.empty(max(cap, 1), np.float32)
        r = L.mwx_resample(self.ctx, self.state(state_index), ptr, n, src_rate, dst_rate,
                           out.ctypes.data, cap)
        if r < 0:
            raise RuntimeError(f"mwx_resample failed ({r})")
        return out[:r].copy() if r > 0 else None

    def test_sample_draws(self, probs: np.ndarray, logprobs: np.ndarray, u: np.ndarray,
                          ndraw: np.ndarray, exact: bool = False, reps: int = 1):
        """mwx_test_sample_draws: ids [R][KD] and mean us per launch."""
        pr = np.ascontiguousarray(probs, np.float32)
        lp = np.ascontiguousarray(logprobs, np.float32)
        uu = np.ascontiguousarray(u, np.float64)
        nd = np.ascontiguousarray(ndraw, np.int32)
        R, V = pr.shape
        KD = uu.shape[1]
        ids = np.zeros((R, KD), np.int32)
        us = C.c_double()
        rc = lib().mwx_test_sample_draws(self.ctx, fptr(pr), fptr(lp), R, V,
                                         uu.ctypes.data_as(C.POINTER(C.c_double)),
                                         nd.ctypes.data_as(C.POINTER(C.c_int)), KD, int(exact),
                                         reps, ids.ctypes.data_as(C.POINTER(C.c_int)),
                                         C.byref(us))
        if rc != 0:
            raise RuntimeError(f"mwx_test_sample_draws failed ({rc})")
        return ids, us.value

    def test_gemm_mx(self, a: np.ndarray, w: np.ndarray) -> np.ndarray:
        """c = MX-fp8(bf16(a)) @ MX-fp8(bf16(w))^T on the block-scaled fp8 MFMA."""
        a = np.ascontiguousarray(a, dtype=np.float32)
        w = np.ascontiguousarray(w, dtype=np.float32)
        M, K = a.shape
        N = w.shape[0]
        c = np.empty((M, N), np.float32)
        fn = lib().mwx_test_gemm_mx
        fn.restype = C.c_int
        fn.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float),
                       C.POINTER(C.c_float), C.POINTER(C.c_float)]
        if fn(self.ctx, M, N, K, fptr(a), fptr(w), fptr(c)) != 0:
            raise RuntimeError("mwx_test_gemm_mx failed")
        return c

    def test_gemm_gelu(self, a: np.ndarray, w: np.ndarray, bias: np.ndarray, bf16: bool,
                       use_table: bool) -> np.ndarray:
        """gelu_ggml(a @ w^T + bias) by the encoder FFN1 GEMM (gemm_big, staged
        GELU epilogue), operands rounded to bf16 / f16; table lookup or tanhf."""
        a = np.ascontiguousarray(a, dtype=np.float32)
        w = np.ascontiguousarray(w, dtype=np.float32)
        bias = np.ascontiguousarray(bias, dtype=np.float32)
        M, K = a.shape
        N = w.shape[0]
        out = np.empty((M, N), np.float32)
        fn = lib().mwx_test_gemm_gelu
        fn.restype = C.c_int
        fn.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float),
                       C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int, C.c_int,
                       C.POINTER(C.c_float)]
        if fn(self.ctx, M, N, K, fptr(a), fptr(w), fptr(bias), int(bf16), int(use_table),
              fptr(out)) != 0:
            raise RuntimeError("mwx_test_gemm_gelu failed")
        return out

    def test_encode(self, pcm: np.ndarray, seek: int = 0, cross: bool = True,
                    state_index: int = 0):
        pcm = np.ascontiguousarray(pcm, dtype=np.float32)
        L_a = self.hparam("n_audio_ctx")
        d = self.d
        nl = self.n_text_layer
        enc = np.empty((L_a, d), dtype=np.float32)
        k = np.empty((nl, L_a, d), dtype=np.float32) if cross else None
        v = np.empty((nl, L_a, d), dtype=np.float32) if cross else None
        null = C.POINTER(C.c_float)()
        r = lib().mwx_test_encode(self.ctx, self.state(state_index), fptr(pcm), len(pcm), seek,
                                  fptr(enc),
                                  fptr(k) if cross else null, fptr(v) if cross else null)
        if r != 0:
            raise RuntimeError(f"mwx_test_encode returned {r}")
        return enc, k, v

    def test_encode_dump(self, pcm: np.ndarray, seek: int = 0, state_index: int = 0):
        """mwx_test_encode_dump: (x [L+1][n_ctx][d] f32 — the residual stream
        after the stem and after each layer, [a0, a1, a2, a3] — per layer the
        four GEMM A operands before MX quantization, as float32 from the
        model's 16-bit type)."""
        pcm = np.ascontiguousarray(pcm, dtype=np.float32)
        n_ctx, d, L = self.hparam("n_audio_ctx"), self.d, self._hp_from_file()[4]
        x = np.empty((L + 1, n_ctx, d), np.float32)
        a = [np.empty((L, n_ctx, d * (4 if g == 3 else 1)), np.uint16) for g in range(4)]
        ptrs = (C.c_void_p * 4)(*[arr.ctypes.data for arr in a])
        r = lib().mwx_test_encode_dump(self.ctx, self.state(state_index), fptr(pcm), len(pcm), seek,
                                       fptr(x), ptrs)
        if r != 0:
            raise RuntimeError(f"mwx_test_encode_dump returned {r}")
        bf16 = self.hparam("model_wtype") == GGML_BF16
        conv = ((lambda u: (u.astype(np.uint32) << 16).view(np.float32)) if bf16 else
                (lambda u: u.view(np.float16).astype(np.float32)))
        return x, [conv(arr) for arr in a]

    def test_decode(self, tokens: Sequence[int]) -> np.ndarray:
        toks = np.ascontiguousarray(tokens, dtype=np.int32)
        V = self.hparam("n_vocab")
        out = np.empty((len(toks), V), dtype=np.float32)
        r = lib().mwx_test_decode(self.ctx, self.state(), toks.ctypes.data_as(C.POINTER(C.c_int)),
                                  len(toks), fptr(out))
        if r != 0:
            raise RuntimeError(f"mwx_test_decode returned {r}")
        return out

    def decode_counters(self, state_index: int = 0, reset: bool = True):
        """(decode steps launched, prompt positions prefilled) on a state since
        the last reset (mwx_test_decode_counters)."""
        st, pf = C.c_long(), C.c_long()
        lib().mwx_test_decode_counters(self.state(state_index), C.byref(st), C.byref(pf),
                                       1 if reset else 0)
        return st.value, pf.value

    def window_counters(self, state_index: int = 0, reset: bool = True):
        """(clip windows decoded, decode attempts run, clip-steps) on a state
        since the last reset (mwx_test_window_counters); attempts - windows =
        fallbacks; clip-steps = decode steps summed over the clips live in them."""
        w, a, cs = C.c_long(), C.c_long(), C.c_long()
        lib().mwx_test_window_counters(self.state(state_index), C.byref(w), C.byref(a),
                                       C.byref(cs), 1 if reset else 0)
        return w.value, a.value, cs.value

    def runahead_fallbacks(self, state_index: int = 0, reset: bool = True) -> int:
        """Run-ahead attempts redone on the host loop (mwx_test_runahead_fallbacks)."""
        return lib().mwx_test_runahead_fallbacks(self.state(state_index), 1 if reset else 0)

    def test_mx_widen(self, codes: np.ndarray, e8: np.ndarray) -> np.ndarray:
        """mwx_test_mx_widen: e4m3 codes (uint8, groups of 8) widened to f16
        with one E8M0 exponent per group, as the cross-attention kernels do."""
        codes = np.ascontiguousarray(codes, np.uint8)
        e8 = np.ascontiguousarray(e8, np.uint8)
        assert codes.size == 8 * e8.size
        out = np.empty(codes.size, np.uint16)
        r = lib().mwx_test_mx_widen(self.ctx, codes.ctypes.data, e8.ctypes.data, e8.size,
                                    out.ctypes.data)
        if r != 0:
            raise RuntimeError(f"mwx_test_mx_widen returned {r}")
        return out.view(np.float16)

    def test_xattn_mx(self, q: np.ndarray, k8: np.ndarray, ks: np.ndarray, v8: np.ndarray,
                      vs: np.ndarray, nq: int) -> np.ndarray:
        """mwx_test_xattn_mx: q [R][H*64] f32; k8 / v8 uint8 [R/nq][H][n][64];
        ks / vs uint8 [R/nq][H][n][2]. Returns o [R][H*64] f32."""
        R, D = q.shape
        G, H, n, _ = k8.shape
        assert G * nq == R and H * 64 == D
        q = np.ascontiguousarray(q, dtype=np.float32)
        arrs = [np.ascontiguousarray(a, dtype=np.uint8) for a in (k8, ks, v8, vs)]
        o = np.empty((R, D), dtype=np.float32)
        u8 = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint8))
        rc = lib().mwx_test_xattn_mx(self.ctx, R, H, n, nq, q.ctypes.data_as(C.POINTER(C.c_float)),
                                     *[u8(a) for a in arrs], o.ctypes.data_as(C.POINTER(C.c_float)))
        if rc != 0:
            raise RuntimeError(f"mwx_test_xattn_mx failed ({rc})")
        return o

    def test_decode_last(self, tokens: Sequence[int], out: Optional[np.ndarray] = None,
                         state_index: int = 0) -> np.ndarray:
        toks = np.ascontiguousarray(tokens, dtype=np.int32)
        if out is None:
            out = np.empty(self.hparam("n_vocab"), dtype=np.float32)
        r = lib().mwx_test_decode_last(self.ctx, self.state(state_index),
                                       toks.ctypes.data_as(C.POINTER(C.c_int)), len(toks), fptr(out))
        if r != 0:
            raise RuntimeError(f"mwx_test_decode_last returned {r}")
        return out

    def test_self_kv(self, layer: int, n_pos: int, state_index: int = 0):
        """(K, V) of row 0's self-attention cache, layer `layer`, positions < n_pos."""
        H = self.d // 64
        k = np.empty((n_pos, H, 64), np.float32)
        v = np.empty_like(k)
        r = lib().mwx_test_self_kv(self.state(state_index), layer, n_pos, fptr(k), fptr(v))
        if r != 0:
            raise RuntimeError(f"mwx_test_self_kv returned {r}")
        return k, v

    def test_decode_last_prefill(self, tokens: Sequence[int], state_index: int = 0) -> np.ndarray:
        """test_decode_last with tokens[:-1] through the batched prompt prefill."""
        toks = np.ascontiguousarray(tokens, dtype=np.int32)
        out = np.empty(self.hparam("n_vocab"), dtype=np.float32)
        r = lib().mwx_test_decode_last_prefill(self.ctx, self.state(state_index),
                                               toks.ctypes.data_as(C.POINTER(C.c_int)), len(toks),
                                               fptr(out))
        if r != 0:
            raise RuntimeError(f"mwx_test_decode_last_prefill returned {r}")
        return out

    @property
    def d(self) -> int:
        return self._hp_from_file()[2]

    @property
    def n_text_layer(self) -> int:
        return self._hp_from_file()[8]

    def _hp_from_file(self):
        if not hasattr(self, "_hp"):
            raise RuntimeError("hparams unknown: use Context.open()")
        return self._hp

    @classmethod
    def open(cls, model_path: str, device: int = 0, compute: int = COMPUTE_MODEL) -> "Context":
        c = cls(model_path, device, compute)
        c._hp = read_hparams(model_path)
        return c


def read_hparams(path: str) -> List[int]:
    with open(path, "rb") as f:
        b = f.read(48)
    return list(np.frombuffer(b[4:48], dtype=np.int32))


def token_ids(segs: List[Segment]) -> List[int]:
    return [t.id for s in segs for t in s.tokens]
