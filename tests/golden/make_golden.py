"""Generates tests/golden/*.npz — golden vectors from an INDEPENDENT
implementation (HF transformers Whisper, fp32, CPU) used to pin the oracle.

The reference (sentiric-stt-whisper-service) ships no fixtures for its hot path
and its inference dependency (whisper.cpp v1.8.2) is not available offline, so
the oracle (oracle/mwx_oracle.cpp) is cross-checked against HF transformers'
Whisper on the same seeded weights instead:

  * mel: WhisperFeatureExtractor (80 and 128 bins) on synthetic clip 0. HF
    reflect-pads the clip end where whisper.cpp zero-pads, so only frames
    0..2997 are comparable.
  * encoder / decoder: WhisperForConditionalGeneration built from a local
    config with the weights of the seeded `micro` ggml file and of the two
    benchmarked geometries (large-v3 d 1280 / 20 heads / 128 mels / vocab
    51866 with 2 + 2 layers in bf16; base d 512 at full 6 + 6 depth in f16),
    activation forced
    to the tanh GELU ggml uses (conv GELU patched too), run on the oracle's own
    mel so only the network math is compared. The oracle is run in its "exact"
    (fp32, no 16-bit rounding) mode for this comparison.

Run from the repo root:  python tests/golden/make_golden.py
Requires libmwx.so (model writer) and oracle/liborc.so (both CPU-side code).
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "sentiric-stt-whisper-service_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import mwx  # noqa: E402
import orc  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
MEL_ROWS = [0, 7, 19, 40, 63, 79]
MEL_ROWS_128 = [0, 9, 33, 64, 100, 127]
TF_TOKENS = [50257, 300, 1234, 50363, 777, 40000, 220, 50400]


def read_ggml(path):
    """Minimal reader of the whisper ggml .bin layout -> {name: float32 array}."""
    with open(path, "rb") as f:
        b = f.read()
    off = 4
    hp = np.frombuffer(b, np.int32, 11, off)
    off += 44
    nm, nf = np.frombuffer(b, np.int32, 2, off)
    off += 8 + 4 * nm * nf
    nv = int(np.frombuffer(b, np.int32, 1, off)[0])
    off += 4
    for _ in range(nv):
        ln = int(np.frombuffer(b, np.uint32, 1, off)[0])
        off += 4 + ln
    t = {}
    while off < len(b):
        nd, nl, tt = np.frombuffer(b, np.int32, 3, off)
        off += 12
        ne = list(np.frombuffer(b, np.int32, nd, off))
        off += 4 * nd
        name = b[off:off + nl].decode()
        off += nl
        n = int(np.prod(ne))
        if tt == 0:
            a = np.frombuffer(b, np.float32, n, off).copy()
            off += 4 * n
        elif tt == 1:
            a = np.frombuffer(b, np.float16, n, off).astype(np.float32)
            off += 2 * n
        else:
            raw = np.frombuffer(b, np.uint16, n, off).astype(np.uint32) << 16
            a = raw.view(np.float32).copy()
            off += 2 * n
        t[name] = a.reshape(list(reversed(ne)))
    return hp, t


def hf_model(hp, t):
    from transformers import WhisperConfig, WhisperForConditionalGeneration
    d = int(hp[2])
    cfg = WhisperConfig(
        vocab_size=int(hp[0]), num_mel_bins=int(hp[9]), encoder_layers=int(hp[4]),
        encoder_attention_heads=int(hp[3]), decoder_layers=int(hp[8]),
        decoder_attention_heads=int(hp[7]), encoder_ffn_dim=4 * d, decoder_ffn_dim=4 * d,
        d_model=d, max_source_positions=int(hp[1]), max_target_positions=int(hp[5]),
        activation_function="gelu_new", scale_embedding=False, dropout=0.0,
        attention_dropout=0.0, activation_dropout=0.0)
    cfg._attn_implementation = "eager"
    m = WhisperForConditionalGeneration(cfg).eval()
    sd = {}
    sd["model.encoder.conv1.weight"] = t["encoder.conv1.weight"]
    sd["model.encoder.conv1.bias"] = t["encoder.conv1.bias"].reshape(-1)
    sd["model.encoder.conv2.weight"] = t["encoder.conv2.weight"]
    sd["model.encoder.conv2.bias"] = t["encoder.conv2.bias"].reshape(-1)
    sd["model.encoder.embed_positions.weight"] = t["encoder.positional_embedding"]
    sd["model.encoder.layer_norm.weight"] = t["encoder.ln_post.weight"]
    sd["model.encoder.layer_norm.bias"] = t["encoder.ln_post.bias"]
    sd["model.decoder.embed_tokens.weight"] = t["decoder.token_embedding.weight"]
    sd["model.decoder.embed_positions.weight"] = t["decoder.positional_embedding"]
    sd["model.decoder.layer_norm.weight"] = t["decoder.ln.weight"]
    sd["model.decoder.layer_norm.bias"] = t["decoder.ln.bias"]
    amap = {"query": "q_proj", "key": "k_proj", "value": "v_proj", "out": "out_proj"}

    def attn(src, dst):
        for a, b in amap.items():
            sd[f"{dst}.{b}.weight"] = t[f"{src}.{a}.weight"]
            if f"{src}.{a}.bias" in t:
                sd[f"{dst}.{b}.bias"] = t[f"{src}.{a}.bias"]

    for l in range(int(hp[4])):
        s, dd = f"encoder.blocks.{l}", f"model.encoder.layers.{l}"
        attn(f"{s}.attn", f"{dd}.self_attn")
        for a, b in (("attn_ln", "self_attn_layer_norm"), ("mlp_ln", "final_layer_norm"),
                     ("mlp.0", "fc1"), ("mlp.2", "fc2")):
            sd[f"{dd}.{b}.weight"] = t[f"{s}.{a}.weight"]
            sd[f"{dd}.{b}.bias"] = t[f"{s}.{a}.bias"]
    for l in range(int(hp[8])):
        s, dd = f"decoder.blocks.{l}", f"model.decoder.layers.{l}"
        attn(f"{s}.attn", f"{dd}.self_attn")
        attn(f"{s}.cross_attn", f"{dd}.encoder_attn")
        for a, b in (("attn_ln", "self_attn_layer_norm"), ("cross_attn_ln", "encoder_attn_layer_norm"),
                     ("mlp_ln", "final_layer_norm"), ("mlp.0", "fc1"), ("mlp.2", "fc2")):
            sd[f"{dd}.{b}.weight"] = t[f"{s}.{a}.weight"]
            sd[f"{dd}.{b}.bias"] = t[f"{s}.{a}.bias"]
    sd = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    missing = [k for k in missing if k != "proj_out.weight"]
    assert not missing and not unexpected, (missing, unexpected)
    m.proj_out.weight = m.model.decoder.embed_tokens.weight
    return m


def network_golden(arch, wtype, tf_tokens, pcm, prefix, out):
    """HF fp32 encoder rows / stats and teacher-forced logits for the seeded
    `arch` model (weight type `wtype`), on the oracle's own mel."""
    path = os.path.join("/tmp", f"golden_{arch}_{wtype}.bin")
    mwx.write_synthetic_model(path, arch, wtype, 0)
    hp, t = read_ggml(path)
    o = orc.Oracle(path, exact=True)
    mel, _ = o.mel(pcm)
    feats = torch.from_numpy(np.ascontiguousarray(mel[:, :3000]))[None]
    orig_gelu = torch.nn.functional.gelu
    torch.nn.functional.gelu = lambda x, approximate="none": orig_gelu(x, approximate="tanh")
    try:
        m = hf_model(hp, t)
        with torch.no_grad():
            enc = m.model.encoder(feats).last_hidden_state
            dec = m(encoder_outputs=(enc,), decoder_input_ids=torch.tensor([tf_tokens])).logits[0]
    finally:
        torch.nn.functional.gelu = orig_gelu
    enc = enc[0].numpy()
    dec = dec.numpy()
    out[prefix + "enc_rows"] = np.array([0, 1, 2, 500, 1000, 1499], np.int32)
    out[prefix + "enc_hf"] = enc[out[prefix + "enc_rows"]].astype(np.float32)
    out[prefix + "enc_hf_mean"] = np.float64(enc.mean())
    out[prefix + "enc_hf_std"] = np.float64(enc.std())
    out[prefix + "tf_tokens"] = np.array(tf_tokens, np.int32)
    top = np.argsort(-dec, axis=1)[:, :10]
    out[prefix + "dec_top_ids"] = top.astype(np.int32)
    out[prefix + "dec_top_vals"] = np.take_along_axis(dec, top, axis=1).astype(np.float32)
    out[prefix + "dec_lse"] = np.log(np.exp(dec - dec.max(1, keepdims=True)).sum(1)) + dec.max(1)
    out[prefix + "dec_sample_ids"] = np.arange(0, dec.shape[1], 997, dtype=np.int32)
    out[prefix + "dec_sample_vals"] = dec[:, out[prefix + "dec_sample_ids"]].astype(np.float32)
    # quick self-check
    enc_o = o.encode(mel)
    print(arch, "enc max|diff| vs oracle-exact:", np.abs(enc_o - enc).max(), "std", enc.std())
    k, v = o.cross(enc_o)
    lg = o.decode_seq(k, v, tf_tokens)
    print(arch, "logits max|diff|:", np.abs(lg - dec).max(), "std", dec.std())
    o.close()
    os.remove(path)


# the benchmarked geometries (BASELINE.json configs[1..4]): large-v3 (d 1280,
# 20 heads, 128 mels, vocab 51866; 2 + 2 layers so HF and the oracle stay
# cheap, bf16 = C3's weight type) and base at full depth (d 512, 6 + 6 layers,
# f16 = C2's weight type)
GEOMETRIES = [
    ("micro", mwx.GGML_F16, TF_TOKENS, ""),
    ("large-v3-l2", mwx.GGML_BF16, [50258, 50259, 50360, 300, 1234, 40000, 220, 50400, 50364],
     "v3_"),
    ("base", mwx.GGML_F16, [50258, 50259, 50359, 300, 1234, 40000, 220, 50400, 50363], "base_"),
]


def main():
    from transformers import WhisperFeatureExtractor
    pcm = mwx.pcm16_to_f32(mwx.synth_pcm16(0))
    out = {}
    # ---- mel (HF feature extractor) ----
    for nm, rows, key in ((80, MEL_ROWS, "mel80"), (128, MEL_ROWS_128, "mel128")):
        fe = WhisperFeatureExtractor(feature_size=nm)
        feats = fe(pcm, sampling_rate=16000, return_tensors="np").input_features[0]
        out[f"{key}_rows"] = np.array(rows, np.int32)
        out[f"{key}_hf"] = feats[rows, :2998].astype(np.float32)
        out[f"{key}_hf_mean"] = np.float64(feats[:, :2998].mean())
    # ---- networks (exact oracle mode vs HF fp32) ----
    for arch, wtype, toks, prefix in GEOMETRIES:
        network_golden(arch, wtype, toks, pcm, prefix, out)
    np.savez_compressed(os.path.join(OUT, "hf_golden.npz"), **out)
    print("wrote", os.path.join(OUT, "hf_golden.npz"))


if __name__ == "__main__":
    main()
