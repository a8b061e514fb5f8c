"""ggml .bin writer/reader round trip, special-token layout per vocabulary
size (whisper_vocab + loader shift) and the mel filterbank."""
import numpy as np
import pytest

import mwx
import orc

# (arch, eot, sot, translate, transcribe, solm, prev, nosp, not, beg)
SPECIALS = [
    ("micro", 50256, 50257, 50357, 50358, 50359, 50360, 50361, 50362, 50363),      # .en 51864
    ("micro-ml", 50257, 50258, 50358, 50359, 50360, 50361, 50362, 50363, 50364),   # v1/v2 51865
    ("micro-v3", 50257, 50258, 50359, 50360, 50361, 50362, 50363, 50364, 50365),   # v3 51866
]


@pytest.mark.parametrize("row", SPECIALS, ids=[r[0] for r in SPECIALS])
def test_special_tokens(make_model, row):
    o = orc.Oracle(make_model(row[0]))
    assert [o.eot, o.sot, o.translate, o.transcribe, o.solm, o.prev, o.nosp, o.not_, o.beg] == list(row[1:])
    assert o.token_str(o.eot) == "[_EOT_]"
    assert o.token_str(o.beg) == "[_BEG_]"
    assert o.token_str(o.beg + 1) == "[_TT_1]"
    assert o.token_str(o.n_vocab - 1) == "[_TT_1500]"
    assert o.token_str(220) == " "


def test_hparams_and_types(make_model):
    for arch, hp in (("micro", [51864, 1500, 128, 2, 2, 448, 128, 2, 3, 80, 1]),
                     ("micro-v3", [51866, 1500, 128, 2, 2, 448, 128, 2, 3, 128, 1])):
        o = orc.Oracle(make_model(arch))
        assert o.hp == hp
    o = orc.Oracle(make_model("micro", mwx.GGML_BF16))
    assert o.hp[10] == 24 and orc.lib().orc_wtype(o.h) == 30


def test_writer_is_deterministic(make_model, tmp_path):
    a = make_model("micro", 1, 7)
    b = str(tmp_path / "again.bin")
    mwx.write_synthetic_model(b, "micro", 1, 7)
    assert open(a, "rb").read() == open(b, "rb").read()


def test_unknown_arch_rejected(tmp_path):
    with pytest.raises(RuntimeError):
        mwx.write_synthetic_model(str(tmp_path / "x.bin"), "nope", 1, 0)


@pytest.mark.parametrize("n_mels,arch", [(80, "micro"), (128, "micro-v3")])
def test_mel_filterbank_matches_librosa_slaney(make_model, n_mels, arch):
    tf = pytest.importorskip("transformers.audio_utils")
    ref = tf.mel_filter_bank(num_frequency_bins=201, num_mel_filters=n_mels, min_frequency=0.0,
                             max_frequency=8000.0, sampling_rate=16000, norm="slaney",
                             mel_scale="slaney").T
    got = orc.Oracle(make_model(arch)).filters()
    assert got.shape == (n_mels, 201)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-7)
