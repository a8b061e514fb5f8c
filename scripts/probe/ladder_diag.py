"""Diagnostic (GPU): beam search with best_of = -1 walking the temperature
ladder — the device run vs the oracle's loop on the device's logits; prints
the first differing token and the closest draws. Measurement probe, not a test."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "sentiric-stt-whisper-service_amd")]
import mwx  # noqa: E402
import orc  # noqa: E402
from test_gpu_parity import beam_opt, beam_params, pcm_clip  # noqa: E402
from test_gpu_beam_oracle import replay_traced  # noqa: E402

path = "/tmp/ladder_micro_rich.bin"
mwx.write_synthetic_model(path, "micro-rich", 1, 0)
ctx = mwx.Context.open(path)
o = orc.Oracle(path)
for best_of in (-1, 5):
    for clip in (0, 2):
        pcm = pcm_clip(50 + clip, 14.0 + 4 * clip)
        p, opt = beam_params(ctx, 0.2), beam_opt(0.2)
        p.greedy.best_of = opt.best_of = best_of
        p.logprob_thold = opt.logprob_thold = 0.5
        res = {}
        for mode in ("ra", "host"):
            if mode == "host":
                os.environ["MWX_NO_RUNAHEAD"] = "1"
            idx = len(ctx.states)
            assert ctx.full(pcm, p, state_index=idx) == 0
            res[mode] = [t.id for s in ctx.segments(idx) for t in s.tokens]
            os.environ.pop("MWX_NO_RUNAHEAD", None)
        rsegs, tr, rows = replay_traced(ctx, o, pcm, opt)
        rid = [t.id for s in rsegs for t in s.tokens]
        first = next((i for i, (a, b) in enumerate(zip(res["ra"], rid)) if a != b), None)
        print(f"best_of {best_of} clip {clip}: ra==host {res['ra'] == res['host']}, "
              f"device==replay {res['ra'] == rid}, first diff {first}, "
              f"n {len(res['ra'])} / {len(rid)}")
        if first is not None:
            print("  device", res["ra"][:first + 3], "\n  replay", rid[:first + 3])
        draws = sorted((e for e in tr if e.kind == "draw"), key=lambda e: e.margin)[:6]
        for e in draws:
            print(f"  close draw: seek {e.seek} it {e.it} step {e.step} dec {e.dec} "
                  f"id {e.b} margin {e.margin:.3g}")
        last = [e for e in tr if e.kind in ("fallback", "best")]
        print("  fallback/best:", [(e.kind, e.seek, e.it, e.a) for e in last][:14])
        sys.stdout.flush()
ctx.close()
