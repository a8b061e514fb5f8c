"""Diagnose a greedy token divergence between the device and the oracle: replay
the oracle's token loop on the device's logits, and at every step also compute
the oracle's own logits for the same prefix (its encoder / cross K/V at the
same seek); print the steps where the two argmaxes differ and the logit margin
of the two competing tokens on both sides."""
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sentiric-stt-whisper-service_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]
import numpy as np
import mwx
import orc
from test_gpu_parity import service_params

arch, clip, secs = sys.argv[1], int(sys.argv[2]), float(sys.argv[3])
path = f"/tmp/near_tie_{arch}.bin"
mwx.write_synthetic_model(path, arch, mwx.GGML_F16, 0)
pcm = mwx.pcm16_to_f32(mwx.synth_pcm16(clip, int(secs * 16000)))
o = orc.Oracle(path)
opt = orc.FullOptions.service_defaults()
opt.temperature_inc = 0.0
opt.language = "en"
ctx = mwx.Context.open(path)
p = service_params(ctx, temperature_inc=0.0, language=b"en")
assert ctx.full(pcm, p, state_index=0) == 0
ids = [t.id for s in ctx.segments(0) for t in s.tokens]
_, osegs, _, _ = o.full(pcm, opt)
oids = [t.id for s in osegs for t in s.tokens]
first = next((i for i, (a, b) in enumerate(zip(ids, oids)) if a != b), None)
print("device tokens", len(ids), "oracle tokens", len(oids), "first difference", first,
      None if first is None else (ids[first], oids[first]))
mel, _ = o.mel(pcm)
ctx.state(1)
state = {"seek": 0, "kv": None}
rows = []


def enc(seek):
    ctx.test_encode(pcm, seek=seek, cross=False, state_index=1)
    state["seek"] = seek


steps = []


def logits(tokens):
    dl = ctx.test_decode_last(tokens, state_index=1)
    steps.append((state["seek"], list(tokens), dl.copy()))
    return dl


def enc_only(seek):
    enc(seek)


_, rsegs, _, _ = o.full_external(pcm, opt, enc_only, logits)
rids = [t.id for s in rsegs for t in s.tokens]
print("replay == device tokens:", rids == ids)
# the oracle's own logits for the same prefixes (after the replay: the oracle's
# external hooks are cleared)
cache = {}
for seek, toks, dl in steps:
    if seek not in cache:
        cache[seek] = o.cross(o.encode(mel, seek))
    k, v = cache[seek]
    ol = o.decode_seq(k, v, toks)[-1]
    da, oa = int(np.argmax(dl)), int(np.argmax(ol))
    if da != oa:
        rows.append((seek, len(toks), da, oa, float(dl[da] - dl[oa]), float(ol[oa] - ol[da]),
                     float(np.abs(dl - ol).max())))
print("steps whose raw-logit argmax differs (seek, prefix len, device id, oracle id, device margin, "
      "oracle margin, max |dlogit|):")
for r in rows[:20]:
    print(r)
