"""Shared pytest setup: the `gpu` marker, import paths, and synthetic models
generated on the fly (seeded, in the ggml .bin layout) in a session temp dir."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sentiric-stt-whisper-service_amd")
for p in (PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def model_dir(tmp_path_factory):
    return str(tmp_path_factory.mktemp("models"))


_made = {}


@pytest.fixture(scope="session")
def make_model(model_dir):
    import mwx

    def make(arch: str, wtype: int = 1, seed: int = 0) -> str:
        key = (arch, wtype, seed)
        if key not in _made:
            path = os.path.join(model_dir, f"{arch}-{wtype}-{seed}.bin")
            mwx.write_synthetic_model(path, arch, wtype, seed)
            _made[key] = path
        return _made[key]

    return make
