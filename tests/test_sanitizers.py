"""Sanitizer runs of the CPU-side code (SURVEY.md §5 aux: race detection /
memory errors; the reference builds with warnings only, CMakeLists.txt:16).

* The host SttEngine (state pool + EngineBusy, dynamic batcher, streaming
  loop, text filters, speaker clusterer, C shim) built with ASan + UBSan and
  with TSan over tests/san/mwx_stub.cpp — a CPU stand-in for libmwx.so that
  exists only in this test build — and driven from many threads by
  tests/san/host_check.cpp.
* The CPU oracle (liborc) built with ASan + UBSan and run in a python child
  with libasan preloaded: full transcriptions (greedy with fallback, beam,
  token timestamps, two windows), the resampler at every rate, prosody.

Any sanitizer report aborts the child; -fno-sanitize-recover makes UBSan
findings fatal too. GPU code is not covered (GPU sanitizers are not
available on the MI355X pool)."""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tests", "san")
BUILD = os.path.join(SAN, "_build")


@pytest.fixture(scope="module")
def san_build():
    subprocess.check_call(["make", "-s", "-j", "3", "-C", SAN])
    return BUILD


def _run(cmd, env, timeout=600):
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, tail
    return r


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_engine_under_sanitizers(san_build, tmp_path, kind):
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    env["TSAN_OPTIONS"] = "halt_on_error=1:second_deadlock_stack=1"
    r = _run([os.path.join(san_build, f"host_{kind}"), str(tmp_path)], env)
    assert "host_check: 0 failure(s)" in r.stdout


def _gcc_runtime(name):
    return subprocess.check_output(["gcc", f"-print-file-name={name}"], text=True).strip()


def test_oracle_under_asan_ubsan(san_build, tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "sentiric-stt-whisper-service_amd"))
    import mwx

    model = str(tmp_path / "micro-rich.bin")
    mwx.write_synthetic_model(model, "micro-rich", mwx.GGML_F16, 0)
    script = textwrap.dedent(f"""
        import sys
        import numpy as np
        sys.path.insert(0, {os.path.join(ROOT, 'oracle')!r})
        import orc
        o = orc.Oracle({model!r})
        rng = np.random.default_rng(3)
        t = np.arange(33 * 16000) / 16000
        pcm = (0.3 * np.sin(2 * np.pi * 180 * t) * (1 + np.sin(2 * np.pi * 3 * t))
               + 0.01 * rng.standard_normal(t.size)).astype(np.float32)
        for beam, n in ((1, pcm.size), (5, 6 * 16000)):
            opt = orc.FullOptions.service_defaults(beam_size=beam)
            opt.language = "en"
            _, segs, _, windows = o.full(pcm[:n], opt)
            assert beam > 1 or len(windows) > 1, len(windows)
        for sr in (8000, 22050, 44100, 48000):
            y = orc.resample(pcm[: sr // 2], sr, 16000)
            assert y is not None and len(y) > 0
        r = orc.prosody(pcm[:32000], 16000)
        print("oracle san ok", len(segs))
    """)
    env = dict(os.environ)
    env["ORC_LIB"] = os.path.join(san_build, "liborc_san.so")
    env["LD_PRELOAD"] = _gcc_runtime("libasan.so")
    # python itself leaks by design; leak checking is covered by the host run
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    env["OMP_NUM_THREADS"] = "4"
    r = _run([sys.executable, "-c", script], env, timeout=900)
    assert "oracle san ok" in r.stdout
