"""ggml block-quantized model files (whisper.cpp `quantize` tool output:
q4_0, q4_1, q5_0, q5_1, q8_0 on every 2-D tensor but the positional embeddings;
conv kernels stay f16). Checks the writer's blocks and the oracle's loader
against an independent numpy restatement of ggml-common.h / ggml-quants.c
(dequantize_row_q*, quantize_row_q*_ref) — CPU only."""
import struct

import numpy as np
import pytest

import mwx
import orc

BLOCK = {mwx.GGML_Q4_0: 18, mwx.GGML_Q4_1: 20, mwx.GGML_Q5_0: 22, mwx.GGML_Q5_1: 24,
         mwx.GGML_Q8_0: 34}
FTYPE = {mwx.GGML_Q4_0: 2, mwx.GGML_Q4_1: 3, mwx.GGML_Q8_0: 7, mwx.GGML_Q5_0: 8,
         mwx.GGML_Q5_1: 9}


def read_tensors(path):
    """Walk a whisper ggml .bin: returns hparams and {name: (type, ne, raw bytes)}."""
    with open(path, "rb") as f:
        buf = f.read()
    o = 4
    hp = list(struct.unpack_from("<11i", buf, o))
    o += 44
    n_mel, n_fft = struct.unpack_from("<2i", buf, o)
    o += 8 + 4 * n_mel * n_fft
    (nv,) = struct.unpack_from("<i", buf, o)
    o += 4
    for _ in range(nv):
        (ln,) = struct.unpack_from("<I", buf, o)
        o += 4 + ln
    out = {}
    while o < len(buf):
        nd, nl, tt = struct.unpack_from("<3i", buf, o)
        o += 12
        ne = list(struct.unpack_from(f"<{nd}i", buf, o))
        o += 4 * nd
        name = buf[o:o + nl].decode()
        o += nl
        n = int(np.prod(ne))
        size = n * 4 if tt == 0 else n * 2 if tt in (1, 30) else n // 32 * BLOCK[tt]
        out[name] = (tt, ne, buf[o:o + size])
        o += size
    return hp, out


def np_dequant(tt, raw, n):
    """ggml dequantize_row_q4_0 / q4_1 / q5_0 / q5_1 / q8_0 (f32)."""
    b = np.frombuffer(raw, np.uint8).reshape(n // 32, BLOCK[tt])
    d = b[:, 0:2].copy().view(np.float16).astype(np.float32)
    if tt == mwx.GGML_Q8_0:
        q = b[:, 2:].view(np.int8).astype(np.float32)
        return (q * d).reshape(-1)
    has_min = tt in (mwx.GGML_Q4_1, mwx.GGML_Q5_1)
    m = b[:, 2:4].copy().view(np.float16).astype(np.float32) if has_min else 0.0
    qs_off = {mwx.GGML_Q4_0: 2, mwx.GGML_Q4_1: 4, mwx.GGML_Q5_0: 6, mwx.GGML_Q5_1: 8}[tt]
    qs = b[:, qs_off:qs_off + 16].astype(np.int32)
    q = np.concatenate([qs & 0x0F, qs >> 4], axis=1)
    if tt in (mwx.GGML_Q5_0, mwx.GGML_Q5_1):
        qh_off = 2 if tt == mwx.GGML_Q5_0 else 4
        qh = b[:, qh_off:qh_off + 4].copy().view(np.uint32).astype(np.int64)
        q = q | (((qh >> np.arange(32)) & 1) << 4).astype(np.int32)
    if has_min:
        y = q.astype(np.float32) * d + m
    else:
        y = (q - (8 if tt == mwx.GGML_Q4_0 else 16)).astype(np.float32) * d
    return y.reshape(-1)


def np_quantize_q8_0(x):
    """ggml quantize_row_q8_0_ref."""
    x = x.reshape(-1, 32)
    amax = np.abs(x).max(axis=1, keepdims=True)
    d = amax / np.float32(127.0)
    idv = np.where(d != 0, np.float32(1.0) / np.where(d != 0, d, 1), 0).astype(np.float32)
    q = np.round(x * idv)  # roundf: half away from zero; ties do not occur for these values
    return d.astype(np.float16), q.astype(np.int8)


QTYPES = [mwx.GGML_Q4_0, mwx.GGML_Q4_1, mwx.GGML_Q5_0, mwx.GGML_Q5_1, mwx.GGML_Q8_0]


@pytest.mark.parametrize("tt", QTYPES, ids=["q4_0", "q4_1", "q5_0", "q5_1", "q8_0"])
def test_quantized_file_layout_and_oracle_dequant(make_model, tt):
    path = make_model("micro", tt)
    hp, ts = read_tensors(path)
    assert hp[10] == 2000 + FTYPE[tt]  # GGML_QNT_VERSION * 1000 + ftype
    # quantize-tool rules: 2-D weights quantized; conv kernels f16; 1-D, conv
    # biases and positional embeddings f32
    assert ts["encoder.conv1.weight"][0] == mwx.GGML_F16
    assert ts["encoder.conv1.bias"][0] == 0
    assert ts["decoder.positional_embedding"][0] == 0
    assert ts["decoder.blocks.0.attn_ln.weight"][0] == 0
    for name in ("decoder.token_embedding.weight", "encoder.blocks.0.mlp.0.weight",
                 "decoder.blocks.1.cross_attn.key.weight"):
        assert ts[name][0] == tt, name
    o = orc.Oracle(path)
    ref16 = orc.Oracle(make_model("micro", mwx.GGML_F16))
    for name in ("encoder.blocks.1.attn.query.weight", "decoder.blocks.2.mlp.2.weight",
                 "decoder.token_embedding.weight"):
        t, ne, raw = ts[name]
        n = int(np.prod(ne))
        want = np_dequant(t, raw, n).astype(np.float16).astype(np.float32)
        got = o.tensor(name)
        np.testing.assert_array_equal(got, want)
        # the blocks encode the same seeded weights as the f16 file, to within
        # the quantization step of each block
        x = ref16.tensor(name).reshape(-1, 32)
        step = (x.max(axis=1) - x.min(axis=1)) / {2: 15, 3: 15, 6: 31, 7: 31, 8: 254}[t]
        err = np.abs(got.reshape(-1, 32) - x).max(axis=1)
        assert np.all(err <= step * 1.01 + 1e-3), name


def test_q8_0_blocks_match_ggml_reference_quantizer(make_model):
    """The writer's q8_0 blocks are quantize_row_q8_0_ref of the seeded f32
    weights. The f16 file holds the same weights rounded to f16, so quantizing
    those must reproduce the scales (to f16 rounding) and codes (to one step)."""
    _, ts = read_tensors(make_model("micro", mwx.GGML_Q8_0))
    x = orc.Oracle(make_model("micro", mwx.GGML_F16)).tensor("decoder.blocks.0.attn.out.weight")
    d_np, q_np = np_quantize_q8_0(x)
    raw = np.frombuffer(ts["decoder.blocks.0.attn.out.weight"][2], np.uint8).reshape(-1, 34)
    q = raw[:, 2:].view(np.int8)
    d = raw[:, 0:2].copy().view(np.float16)
    assert np.abs(q.astype(int) - q_np.astype(int)).max() <= 1
    np.testing.assert_allclose(d.astype(np.float32).reshape(-1), d_np.astype(np.float32).reshape(-1),
                               rtol=2e-3)


def np_mx_round(x):
    """MX-fp8 rule of the engine's fp8 compute mode (independent numpy
    restatement): per 32 k, X = 2^E with E the smallest integer such that
    max|x| <= 448 * 2^E; elements rounded to e4m3fn (nearest even, subnormal
    step 2^-9) in units of X."""
    x = x.astype(np.float32).reshape(-1, 32)
    amax = np.abs(x).max(axis=1)
    E = np.zeros(len(x), np.int64)
    nz = amax > 0
    E[nz] = np.ceil(np.log2(amax[nz].astype(np.float64) / 448.0)).astype(np.int64)
    X = np.ldexp(np.float32(1.0), E).astype(np.float32)[:, None]
    v = x / X
    a = np.abs(v)
    e = np.floor(np.log2(np.where(a > 0, a, 1.0))).astype(np.int64)
    step = np.where(e < -6, np.float32(2.0 ** -9), np.ldexp(np.float32(1.0), e - 3)).astype(np.float32)
    q = (np.rint(a / step) * step * np.sign(v)).astype(np.float32)
    return (q * X).reshape(-1)


MX_DEC_WEIGHTS = ("decoder.blocks.0.attn.query.weight", "decoder.blocks.1.attn.out.weight",
                  "decoder.blocks.2.cross_attn.query.weight", "decoder.blocks.0.cross_attn.out.weight",
                  "decoder.blocks.1.mlp.0.weight", "decoder.blocks.2.mlp.2.weight",
                  "decoder.token_embedding.weight")


def test_mxfp8_weights_follow_the_mx_rule(make_model):
    """Oracle MX-fp8 mode: encoder and cross-K/V weights — and, for a bf16
    model, every decoder projection and the tied token embedding — are the MX
    rounding of the file's 16-bit weights (numpy restatement); the rest (conv
    stem, positional embeddings, LayerNorms, biases) is untouched. An f16
    model keeps 16-bit decoder weights."""
    path = make_model("micro", mwx.GGML_BF16)
    plain, mx = orc.Oracle(path), orc.Oracle(path, mxfp8=True)
    for name in ("encoder.blocks.0.attn.query.weight", "encoder.blocks.1.mlp.2.weight",
                 "decoder.blocks.2.cross_attn.value.weight") + MX_DEC_WEIGHTS:
        np.testing.assert_array_equal(mx.tensor(name), np_mx_round(plain.tensor(name)))
    for name in ("encoder.conv1.weight", "decoder.positional_embedding",
                 "decoder.blocks.0.attn_ln.weight", "decoder.blocks.0.mlp.0.bias"):
        np.testing.assert_array_equal(mx.tensor(name), plain.tensor(name))
    path16 = make_model("micro", mwx.GGML_F16)
    plain16, mx16 = orc.Oracle(path16), orc.Oracle(path16, mxfp8=True)
    for name in MX_DEC_WEIGHTS:
        np.testing.assert_array_equal(mx16.tensor(name), plain16.tensor(name))


def np_quantize_q8_0_exact(x):
    """quantize_row_q8_0_ref bit for bit: d = amax / 127 (f32), id = 1/d,
    q = roundf(x * id) (half away from zero), d stored as f16."""
    x = x.astype(np.float32).reshape(-1, 32)
    amax = np.abs(x).max(axis=1, keepdims=True)
    d = (amax / np.float32(127.0)).astype(np.float32)
    idv = np.where(d != 0, np.float32(1.0) / np.where(d != 0, d, np.float32(1)), 0).astype(np.float32)
    v = (x * idv).astype(np.float32)
    q = np.sign(v) * np.floor(np.abs(v) + np.float32(0.5))
    return d.astype(np.float16), q.astype(np.int8)


@pytest.mark.parametrize("tt", QTYPES, ids=["q4_0", "q4_1", "q5_0", "q5_1", "q8_0"])
def test_model_quantize_tool(make_model, tmp_path, tt):
    """mwx_model_quantize (whisper.cpp `quantize` rules) on an f16 file: 2-D
    weights become `tt` blocks of the f16 values, positional embeddings / conv
    biases / 1-D tensors / 3-D conv kernels are copied byte for byte, ftype
    2000 + ftype; q8_0 blocks equal quantize_row_q8_0_ref exactly."""
    src = make_model("micro", mwx.GGML_F16)
    dst = str(tmp_path / "q.bin")
    mwx.quantize_model(src, dst, tt)
    hp_s, ts_s = read_tensors(src)
    hp_d, ts_d = read_tensors(dst)
    assert hp_d[:10] == hp_s[:10] and hp_d[10] == 2000 + FTYPE[tt]
    assert list(ts_d) == list(ts_s)
    for name, (t, ne, raw) in ts_s.items():
        td, ned, rawd = ts_d[name]
        assert ned == ne
        if len(ne) == 2 and name not in ("encoder.positional_embedding",
                                         "decoder.positional_embedding",
                                         "encoder.conv1.bias", "encoder.conv2.bias"):
            assert td == tt, name
            n = int(np.prod(ne))
            x = np.frombuffer(raw, np.float16).astype(np.float32)
            got = np_dequant(tt, rawd, n)
            xb = x.reshape(-1, 32)
            step = (xb.max(axis=1) - xb.min(axis=1)) / {2: 15, 3: 15, 6: 31, 7: 31, 8: 254}[tt]
            assert np.all(np.abs(got.reshape(-1, 32) - xb).max(axis=1) <= step * 1.01 + 1e-6), name
            if tt == mwx.GGML_Q8_0:
                d, q = np_quantize_q8_0_exact(x)
                b = np.frombuffer(rawd, np.uint8).reshape(-1, 34)
                np.testing.assert_array_equal(b[:, 2:].view(np.int8), q)
                np.testing.assert_array_equal(b[:, 0:2].copy().view(np.float16), d)
        else:
            assert (td, rawd) == (t, raw), name
    # the oracle (and so the engine's loader, same reader rules) accepts it
    o = orc.Oracle(dst)
    assert o.tensor("decoder.blocks.0.mlp.0.weight").shape[0] > 0
