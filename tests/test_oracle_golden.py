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


def test_encoder_matches_hf(make_model, pcm):
    o = orc.Oracle(make_model("micro"), exact=True)
    mel, _ = o.mel(pcm)
    enc = o.encode(mel)
    np.testing.assert_allclose(enc[GOLD["enc_rows"]], GOLD["enc_hf"], atol=2e-4, rtol=0)
    assert abs(enc.mean() - GOLD["enc_hf_mean"]) < 1e-5
    assert abs(enc.std() - GOLD["enc_hf_std"]) < 1e-5


def test_decoder_logits_match_hf(make_model, pcm):
    o = orc.Oracle(make_model("micro"), exact=True)
    mel, _ = o.mel(pcm)
    k, v = o.cross(o.encode(mel))
    lg = o.decode_seq(k, v, GOLD["tf_tokens"])
    top = np.argsort(-lg, axis=1)[:, :10]
    assert (top[:, :3] == GOLD["dec_top_ids"][:, :3]).all()
    np.testing.assert_allclose(np.take_along_axis(lg, GOLD["dec_top_ids"], 1), GOLD["dec_top_vals"],
                               atol=2e-3, rtol=0)
    np.testing.assert_allclose(lg[:, GOLD["dec_sample_ids"]], GOLD["dec_sample_vals"], atol=2e-3, rtol=0)
