"""Pins the oracle against golden vectors from an independent implementation
(HF transformers Whisper, fp32) on the same seeded weights and input —
tests/golden/make_golden.py generated them. The reference itself ships no
fixtures for this path."""
import os

import numpy as np
import pytest

import mwx
import orc

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "hf_golden.npz"))


@pytest.fixture(scope="module")
def pcm():
    return mwx.pcm16_to_f32(mwx.synth_pcm16(0))


@pytest.mark.parametrize("key,arch", [("mel80", "micro"), ("mel128", "micro-v3")])
def test_mel_matches_hf_feature_extractor(make_model, pcm, key, arch):
    o = orc.Oracle(make_model(arch))
    mel, n_len_org = o.mel(pcm)
    assert mel.shape[1] == 6000 and n_len_org == 2999
    rows = GOLD[f"{key}_rows"]
    # frames 0..2997: HF reflect-pads the clip end, whisper.cpp zero-pads
    np.testing.assert_allclose(mel[rows, :2998], GOLD[f"{key}_hf"], atol=1e-4, rtol=0)


# (arch, weight type, golden key prefix): the micro network and the two
# benchmarked geometries, large-v3 (d 1280, 20 heads, 128 mels, vocab 51866;
# 2 + 2 layers, bf16 = C3) and base at full depth (d 512, 6 + 6 layers, f16 = C2)
NETS = [("micro", mwx.GGML_F16, ""), ("large-v3-l2", mwx.GGML_BF16, "v3_"),
        ("base", mwx.GGML_F16, "base_")]


@pytest.mark.parametrize("arch,wtype,pre", NETS)
def test_encoder_matches_hf(make_model, pcm, arch, wtype, pre):
    """The oracle's exact-f32 mode: encoder output rows and statistics equal
    HF transformers' Whisper encoder (fp32) on the same weights and mel."""
    o = orc.Oracle(make_model(arch, wtype), exact=True)
    mel, _ = o.mel(pcm)
    enc = o.encode(mel)
    np.testing.assert_allclose(enc[GOLD[pre + "enc_rows"]], GOLD[pre + "enc_hf"], atol=2e-4, rtol=0)
    assert abs(enc.mean() - GOLD[pre + "enc_hf_mean"]) < 1e-5
    assert abs(enc.std() - GOLD[pre + "enc_hf_std"]) < 1e-5


@pytest.mark.parametrize("arch,wtype,pre", NETS)
def test_decoder_logits_match_hf(make_model, pcm, arch, wtype, pre):
    """Teacher-forced logits of the KV-cached decoder (exact-f32 mode) against
    HF's decoder over the same encoder output: top-10 ids and values, and a
    strided sample of the whole vocabulary."""
    o = orc.Oracle(make_model(arch, wtype), exact=True)
    mel, _ = o.mel(pcm)
    k, v = o.cross(o.encode(mel))
    lg = o.decode_seq(k, v, GOLD[pre + "tf_tokens"])
    top = np.argsort(-lg, axis=1)[:, :10]
    assert (top[:, :3] == GOLD[pre + "dec_top_ids"][:, :3]).all()
    np.testing.assert_allclose(np.take_along_axis(lg, GOLD[pre + "dec_top_ids"], 1),
                               GOLD[pre + "dec_top_vals"], atol=2e-3, rtol=0)
    np.testing.assert_allclose(lg[:, GOLD[pre + "dec_sample_ids"]], GOLD[pre + "dec_sample_vals"],
                               atol=2e-3, rtol=0)


@pytest.mark.parametrize("arch,wtype,pre", NETS[1:])
def test_ggml_mode_tracks_hf_at_benchmarked_geometry(make_model, pcm, arch, wtype, pre):
    """The oracle's default (whisper.cpp-semantics) mode — 16-bit rounding of
    the activations at ggml's points, f16 cross / self K/V — stays within its
    rounding noise of HF fp32 at the benched geometries: encoder within 2% of
    the activations' scale, logits within 0.1 of a std-8 distribution, and
    the top-1 token the same wherever HF's top-2 margin exceeds that noise."""
    o = orc.Oracle(make_model(arch, wtype))
    mel, _ = o.mel(pcm)
    enc = o.encode(mel)
    d = np.abs(enc[GOLD[pre + "enc_rows"]] - GOLD[pre + "enc_hf"])
    assert d.mean() < 0.02 * GOLD[pre + "enc_hf_std"], d.mean()
    k, v = o.cross(enc)
    lg = o.decode_seq(k, v, GOLD[pre + "tf_tokens"])
    hv = GOLD[pre + "dec_top_vals"]
    got = np.take_along_axis(lg, GOLD[pre + "dec_top_ids"], 1)
    assert np.abs(got - hv).max() < 0.1, np.abs(got - hv).max()
    clear = (hv[:, 0] - hv[:, 1]) > 0.2
    assert (lg.argmax(1)[clear] == GOLD[pre + "dec_top_ids"][clear, 0]).all()
