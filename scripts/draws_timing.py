"""Times the draw kernels alone (mwx_test_sample_draws) on flat / peaked rows."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sentiric-stt-whisper-service_amd"))
import numpy as np
import mwx
path = "/tmp/draws_micro.bin"
mwx.write_synthetic_model(path, "micro", mwx.GGML_F16, 0)
ctx = mwx.Context.open(path)
rng = np.random.default_rng(1)
R, V, KD = 160, 51866, 5
for scale in (0.5, 4.0, 30.0):
    logits = rng.normal(0, 1, (R, V)) * scale
    pr = np.exp(logits - logits.max(axis=1, keepdims=True))
    pr = (pr / pr.sum(axis=1, keepdims=True)).astype(np.float32)
    lp = np.log(np.maximum(pr, 1e-30)).astype(np.float32)
    u = rng.random((R, KD))
    nd = np.full(R, KD, np.int32)
    for exact in (False, True):
        ids, us = ctx.test_sample_draws(pr, lp, u, nd, exact=exact, reps=10)
        print(f"scale {scale} exact={exact}: {us:.1f} us", flush=True)
ctx.close()
