"""Prefill vs stepwise self-K/V caches and logits (teacher-forced), repeated on
fresh and reused states: where (layer, position) the two first differ."""
import sys
import numpy as np
sys.path.insert(0, "sentiric-stt-whisper-service_amd")
import mwx

arch = sys.argv[1] if len(sys.argv) > 1 else "tiny.en"
path = f"/tmp/diag_{arch}.bin"
mwx.write_synthetic_model(path, arch, mwx.GGML_F16, 0)
ctx = mwx.Context.open(path)
pcm = mwx.pcm16_to_f32(mwx.synth_pcm16(1, 480000))
L = ctx.n_text_layer
rng = np.random.default_rng(7)
si = 0
for trial, (n, fresh) in enumerate([(9, True), (9, True), (3, True), (9, False), (70, True),
                                    (70, False), (9, True)]):
    if fresh or trial == 0:
        a_i, b_i = si, si + 1
        si += 2
        for st in (a_i, b_i):
            ctx.test_encode(pcm, cross=False, state_index=st)
    toks = [int(t) for t in rng.integers(0, 50000, n)]
    a = ctx.test_decode_last(toks, state_index=a_i)
    b = ctx.test_decode_last_prefill(toks, state_index=b_i)
    first = None
    for l in range(L):
        ka, va = ctx.test_self_kv(l, n - 1, a_i)
        kb, vb = ctx.test_self_kv(l, n - 1, b_i)
        bad = np.nonzero((np.abs(ka - kb).max(axis=(1, 2)) > 0) | (np.abs(va - vb).max(axis=(1, 2)) > 0))[0]
        if len(bad):
            first = (l, bad.tolist()[:10],
                     float(np.abs(ka - kb).max()), float(np.abs(va - vb).max()))
            break
    print(f"trial {trial} n={n} fresh={fresh}: logits maxdiff {np.abs(a - b).max():.6f}; first "
          f"differing (layer, positions, |dK|, |dV|): {first}", flush=True)
