"""Debug: beam search on the micro-rich model, device vs oracle token streams."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "sentiric-stt-whisper-service_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import mwx  # noqa: E402
import orc  # noqa: E402

d = tempfile.mkdtemp()
path = os.path.join(d, "rich.bin")
mwx.write_synthetic_model(path, "micro-rich", mwx.GGML_F16, 0)
o = orc.Oracle(path)
with mwx.Context.open(path) as ctx:
    for k in (0, 2):
        pcm = mwx.pcm16_to_f32(mwx.synth_pcm16(k, 480000))
        p = ctx.default_params(mwx.SAMPLING_BEAM_SEARCH)
        p.beam_search.beam_size = 5
        p.token_timestamps = True
        p.suppress_nst = True
        p.no_speech_thold = 0.85
        p.entropy_thold = 2.4
        p.logprob_thold = -0.7
        p.temperature = 0.0
        p.temperature_inc = 0.0
        p.greedy.best_of = 5
        p.language = b"en"
        idx = len(ctx.states)
        assert ctx.full(pcm, p, state_index=idx) == 0
        segs = ctx.segments(idx)
        opt = orc.FullOptions.service_defaults(beam_size=5)
        opt.temperature_inc = 0.0
        opt.language = "en"
        _, osegs, _, win = o.full(pcm, opt)
        dt = [(t.id, round(t.p, 4), round(t.plog, 4)) for s in segs for t in s.tokens]
        ot = [(t.id, round(t.p, 4), round(t.plog, 4)) for s in osegs for t in s.tokens]
        print("clip", k, "dev", len(dt), "oracle", len(ot))
        for i in range(max(len(dt), len(ot))):
            a = dt[i] if i < len(dt) else None
            b = ot[i] if i < len(ot) else None
            print(i, a, b, "" if (a and b and a[0] == b[0]) else "<<<")
        print("windows", win)
