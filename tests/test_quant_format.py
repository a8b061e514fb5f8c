"""ggml block-quantized model files (whisper.cpp `quantize` tool output:
q4_0, q4_1, q5_0, q5_1, q8_0 and the 256-element K types q2_K .. q6_K on every
2-D tensor but the positional embeddings; conv kernels stay f16). Checks the
writer's blocks and the oracle's loader against an independent numpy
restatement of ggml-common.h / ggml-quants.c (dequantize_row_q*,
quantize_row_q*_ref) — CPU only.

K-quant parity is unpinned against ggml itself (no ggml source, binary or
K-quantized file is in the reference or this image): the engine (quant.cpp,
ggml's loop order), the oracle (per-element restatement) and the numpy
restatement here (vectorised over super-blocks) are three independent
readings of ggml-quants.c dequantize_row_q2_K .. q6_K that must agree bit for
bit, on blocks whose every code / scale / min / high-bit plane is exercised."""
import struct

import numpy as np
import pytest

import mwx
import orc

BLOCK = {mwx.GGML_Q4_0: 18, mwx.GGML_Q4_1: 20, mwx.GGML_Q5_0: 22, mwx.GGML_Q5_1: 24,
         mwx.GGML_Q8_0: 34, mwx.GGML_Q2_K: 84, mwx.GGML_Q3_K: 110, mwx.GGML_Q4_K: 144,
         mwx.GGML_Q5_K: 176, mwx.GGML_Q6_K: 210}
FTYPE = {mwx.GGML_Q4_0: 2, mwx.GGML_Q4_1: 3, mwx.GGML_Q8_0: 7, mwx.GGML_Q5_0: 8,
         mwx.GGML_Q5_1: 9, mwx.GGML_Q2_K: 10, mwx.GGML_Q3_K: 11, mwx.GGML_Q4_K: 12,
         mwx.GGML_Q5_K: 13, mwx.GGML_Q6_K: 14}
KTYPES = [mwx.GGML_Q2_K, mwx.GGML_Q3_K, mwx.GGML_Q4_K, mwx.GGML_Q5_K, mwx.GGML_Q6_K]


def blk_elems(tt):
    return 256 if tt in KTYPES else 32


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
        size = n * 4 if tt == 0 else n * 2 if tt in (1, 30) else n // blk_elems(tt) * BLOCK[tt]
        out[name] = (tt, ne, buf[o:o + size])
        o += size
    return hp, out


def np_dequant_k(tt, raw, n):
    """ggml dequantize_row_q2_K .. q6_K (f32), vectorised over super-blocks:
    each block's 256 outputs as [half 2][group 4][lane 32] planes."""
    b = np.frombuffer(raw, np.uint8).reshape(n // 256, BLOCK[tt])
    f16 = lambda o: b[:, o:o + 2].copy().view(np.float16).astype(np.float32)  # noqa: E731
    f = np.float32
    if tt in (mwx.GGML_Q2_K, mwx.GGML_Q3_K):
        qs = b[:, 16:80] if tt == mwx.GGML_Q2_K else b[:, 32:96]
        qs = qs.reshape(-1, 2, 1, 32).astype(np.int32)                 # [blk][half][1][32]
        q = (qs >> (2 * np.arange(4))[None, None, :, None]) & 3        # [blk][half][grp][32]
        if tt == mwx.GGML_Q2_K:
            sc = b[:, 0:16].reshape(-1, 2, 4, 2, 1).astype(np.int32)   # sub-block = 16 lanes
            d, dmin = f16(80)[:, :, None, None, None], f16(82)[:, :, None, None, None]
            q5 = q.reshape(-1, 2, 4, 2, 16).astype(f)
            y = (d * (sc & 15).astype(f)) * q5 - dmin * (sc >> 4).astype(f)
            return y.reshape(-1)
        hm = b[:, 0:32].astype(np.int32)
        bit = np.arange(8).reshape(2, 4)                              # [half][grp] -> hmask bit
        high = (hm[:, None, None, :] >> bit[None, :, :, None]) & 1
        q = q - np.where(high == 1, 0, 4)
        raw12 = b[:, 96:108].astype(np.int32)
        s = np.arange(16)
        lo = np.where(s < 8, raw12[:, s % 8] & 15, raw12[:, s % 8] >> 4)
        hi = (raw12[:, 8 + s % 4] >> (2 * (s // 4))) & 3
        scales = (lo | (hi << 4)) - 32                                 # [blk][16]
        d = f16(108)[:, :, None, None, None]
        y = (d * scales.reshape(-1, 2, 4, 2, 1).astype(f)) * q.reshape(-1, 2, 4, 2, 16).astype(f)
        return y.reshape(-1)
    if tt in (mwx.GGML_Q4_K, mwx.GGML_Q5_K):
        t = b[:, 4:16].astype(np.int32)
        j = np.arange(8)
        jl = np.minimum(j, 3)
        sc = np.where(j < 4, t[:, jl] & 63, (t[:, (j + 4) % 12] & 15) | ((t[:, (j - 4) % 12] >> 6) << 4))
        mn = np.where(j < 4, t[:, jl + 4] & 63, (t[:, (j + 4) % 12] >> 4) | ((t[:, j % 12] >> 6) << 4))
        qo = 48 if tt == mwx.GGML_Q5_K else 16
        ql = b[:, qo:qo + 128].reshape(-1, 4, 1, 32).astype(np.int32)  # [blk][pair][1][32]
        q = (ql >> np.array([0, 4])[None, None, :, None]) & 15          # [blk][pair][nib][32]
        q = q.reshape(-1, 8, 32)
        if tt == mwx.GGML_Q5_K:
            qh = b[:, 16:48].astype(np.int32)
            q = q + (((qh[:, None, :] >> j[None, :, None]) & 1) << 4)
        d, dmin = f16(0), f16(2)
        y = (d * sc.astype(f))[:, :, None] * q.astype(f) - (dmin * mn.astype(f))[:, :, None]
        return y.reshape(-1)
    # q6_K
    ql = b[:, 0:128].reshape(-1, 2, 2, 32).astype(np.int32)            # [blk][half][run][32]
    lo = np.stack([ql[:, :, 0] & 15, ql[:, :, 1] & 15, ql[:, :, 0] >> 4, ql[:, :, 1] >> 4], axis=2)
    qh = b[:, 128:192].reshape(-1, 2, 1, 32).astype(np.int32)
    hi = (qh >> (2 * np.arange(4))[None, None, :, None]) & 3
    q = (lo | (hi << 4)) - 32                                           # [blk][half][grp][32]
    sc = b[:, 192:208].view(np.int8).reshape(-1, 2, 4, 2, 1).astype(f)
    d = f16(208)[:, :, None, None, None]
    y = (d * sc) * q.reshape(-1, 2, 4, 2, 16).astype(f)
    return y.reshape(-1)


def np_dequant(tt, raw, n):
    """ggml dequantize_row_q4_0 / q4_1 / q5_0 / q5_1 / q8_0 (f32); K types
    through np_dequant_k."""
    if tt in KTYPES:
        return np_dequant_k(tt, raw, n)
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


# ------------------------------------------------------------- K super-blocks
KIDS = ["q2_K", "q3_K", "q4_K", "q5_K", "q6_K"]


def random_k_blocks(tt, nblk, seed):
    """Arbitrary bytes in every field of a K super-block (all codes, scale
    and min values and high-bit planes occur), with finite f16 super-block
    scales d / dmin in [-2, 2]."""
    rng = np.random.default_rng(seed)
    b = rng.integers(0, 256, (nblk, BLOCK[tt]), dtype=np.uint8)
    offs = {mwx.GGML_Q2_K: (80, 82), mwx.GGML_Q3_K: (108,), mwx.GGML_Q4_K: (0, 2),
            mwx.GGML_Q5_K: (0, 2), mwx.GGML_Q6_K: (208,)}[tt]
    for o in offs:
        b[:, o:o + 2] = rng.uniform(-2, 2, nblk).astype(np.float16).view(np.uint8).reshape(nblk, 2)
    return b.tobytes()


@pytest.mark.parametrize("tt", KTYPES, ids=KIDS)
def test_k_dequant_engine_equals_numpy_on_arbitrary_blocks(tt):
    """The engine's load-time dequantizer (quant.cpp, ggml's loop order) and
    the numpy restatement agree bit for bit (f32) on 512 super-blocks of
    arbitrary bytes."""
    n = 512 * 256
    raw = random_k_blocks(tt, 512, tt)
    got = mwx.dequantize(tt, raw, n)
    want = np_dequant_k(tt, raw, n)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), \
        np.flatnonzero(got != want)[:8]
    with pytest.raises(ValueError):
        mwx.dequantize(tt, raw[:BLOCK[tt]], 128)  # not a whole super-block


@pytest.mark.parametrize("tt", KTYPES, ids=KIDS)
def test_k_quantized_file_three_dequantizers_agree(make_model, tt):
    """micro256 (rows of 256) written as `tt`: quantize-tool tensor types and
    ftype; for several weights the oracle's loader (per-element restatement,
    then f16), the engine's dequantizer and numpy agree bit for bit; the
    blocks encode the f16 file's seeded weights to within one code step of
    their sub-block; the bit planes that carry high bits / signs are used."""
    path = make_model("micro256", tt)
    hp, ts = read_tensors(path)
    assert hp[10] == 2000 + FTYPE[tt]
    assert ts["encoder.conv1.weight"][0] == mwx.GGML_F16
    assert ts["decoder.positional_embedding"][0] == 0
    for name in ("decoder.token_embedding.weight", "encoder.blocks.0.mlp.0.weight",
                 "decoder.blocks.1.cross_attn.key.weight"):
        assert ts[name][0] == tt, name
    o = orc.Oracle(path)
    ref16 = orc.Oracle(make_model("micro256", mwx.GGML_F16))
    sub = 32 if tt in (mwx.GGML_Q4_K, mwx.GGML_Q5_K) else 16
    qmax = {mwx.GGML_Q2_K: 3, mwx.GGML_Q3_K: 7, mwx.GGML_Q4_K: 15, mwx.GGML_Q5_K: 31,
            mwx.GGML_Q6_K: 63}[tt]
    for name in ("encoder.blocks.1.attn.query.weight", "decoder.blocks.2.mlp.2.weight",
                 "decoder.token_embedding.weight"):
        t, ne, raw = ts[name]
        n = int(np.prod(ne))
        want = np_dequant_k(t, raw, n)
        assert np.array_equal(mwx.dequantize(t, raw, n), want), name
        got = o.tensor(name)
        np.testing.assert_array_equal(got, want.astype(np.float16).astype(np.float32))
        x = ref16.tensor(name).reshape(-1, sub)
        # one code step of the sub-block's range, plus the 6- / 4-bit scale
        # and min quantization (relative to the super-block's largest)
        step = (x.max(axis=1) - np.minimum(x.min(axis=1), 0)) / qmax
        sblk = np.abs(x).reshape(-1, 256 // sub, sub).max(axis=(1, 2)).repeat(256 // sub)
        err = np.abs(got.reshape(-1, sub) - x).max(axis=1)
        assert np.all(err <= 1.01 * step + 0.02 * sblk + 1e-3), (name, (err - step).max())
    raw = np.frombuffer(ts["decoder.blocks.0.mlp.0.weight"][2], np.uint8).reshape(-1, BLOCK[tt])
    plane = {mwx.GGML_Q2_K: raw[:, 16:80], mwx.GGML_Q3_K: raw[:, 0:32],
             mwx.GGML_Q4_K: raw[:, 16:144], mwx.GGML_Q5_K: raw[:, 16:48],
             mwx.GGML_Q6_K: raw[:, 128:192]}[tt]
    bits = np.unpackbits(plane, axis=1).mean(axis=0)
    assert bits.min() > 0.01 and bits.max() < 0.99, (bits.min(), bits.max())


@pytest.mark.parametrize("tt", KTYPES, ids=KIDS)
def test_model_quantize_tool_k(make_model, tmp_path, tt):
    """mwx_model_quantize with K types: micro256 f16 -> `tt`, the quantize
    tool's copy rules; the blocks decode (numpy) to within the encoder's bound
    of the f16 values; a 384-wide (tiny) model fails as ggml's quantizer does."""
    src = make_model("micro256", mwx.GGML_F16)
    dst = str(tmp_path / "qk.bin")
    mwx.quantize_model(src, dst, tt)
    hp_s, ts_s = read_tensors(src)
    hp_d, ts_d = read_tensors(dst)
    assert hp_d[:10] == hp_s[:10] and hp_d[10] == 2000 + FTYPE[tt]
    assert list(ts_d) == list(ts_s)
    for name, (t, ne, raw) in ts_d.items():
        if t == tt:
            assert len(ne) == 2 and ts_s[name][0] == mwx.GGML_F16
        else:
            assert raw == ts_s[name][2], name
    t, ne, raw = ts_d["decoder.blocks.1.attn.value.weight"]
    x = np.frombuffer(ts_s["decoder.blocks.1.attn.value.weight"][2], np.float16).astype(np.float32)
    y = np_dequant_k(t, raw, x.size)
    assert np.abs(y - x).max() <= 0.6 * np.abs(x).max()
    assert np.corrcoef(x, y)[0, 1] > (0.8 if tt == mwx.GGML_Q2_K else 0.97)
    with pytest.raises(RuntimeError):
        mwx.quantize_model(make_model("tiny", mwx.GGML_F16), str(tmp_path / "bad.bin"), tt)


def test_mx_round_helper_matches_e4m3_codes():
    """tests/test_gpu_c5.py's vectorised MX rounding (used to count e4m3
    boundary flips) equals the code-level e4m3 encode / decode of
    test_gpu_parity.py on random blocks spanning many scales."""
    import numpy as np
    from test_gpu_c5 import _mx_round
    from test_gpu_parity import _e4m3_decode, _e4m3_encode
    rng = np.random.default_rng(5)
    a = (rng.standard_normal((64, 256)) * np.exp2(rng.uniform(-20, 12, (64, 1)))).astype(np.float32)
    a[3, :40] = 0.0
    h = a.reshape(-1, 32).astype(np.float64)
    E = np.ceil(np.log2(np.maximum(np.abs(h).max(axis=1, keepdims=True), 1e-30) / 448.0))
    ref = _e4m3_decode(_e4m3_encode(h / np.exp2(E))) * np.exp2(E)
    assert np.array_equal(_mx_round(a), ref.reshape(a.shape))
