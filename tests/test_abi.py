"""The C-ABI library builds, loads without a GPU and exports every entry
point declared in include/*.h (no compute calls here)."""
import ctypes
import os
import re

from conftest import PKG, ROOT


def _declared(header: str):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = re.sub(r"//[^\n]*", "", txt)
    return sorted(set(re.findall(r"\b(mwx_\w+)\s*\(", txt)))


def test_headers_declare_entry_points():
    names = _declared("mwx.h")
    for must in ("mwx_init_from_file_with_params", "mwx_full_with_state", "mwx_full_batch",
                 "mwx_full_get_token_data_from_state", "mwx_token_eot", "mwx_log_set"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(os.path.join(PKG, "libmwx.so"))
    missing = [n for h in ("mwx.h", "mwx_test.h") for n in _declared(h) if not hasattr(lib, n)]
    assert not missing, missing


def test_oracle_library_loads():
    import orc
    L = orc.lib()
    for n in ("orc_load", "orc_mel", "orc_encode", "orc_cross", "orc_decode_seq", "orc_full"):
        assert hasattr(L, n)


def test_option_a_drop_in_compiles_and_links(tmp_path):
    """INTEGRATION.md Option A: the reference SttEngine's whisper.h calls and
    parameter fields, with the mwx.h names, compile and link against
    libmwx.so (tests/abi/option_a_drop_in.cpp; linked, not run)."""
    import subprocess
    pkg = os.path.join(ROOT, "sentiric-stt-whisper-service_amd")
    r = subprocess.run(["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror",
                        "-I" + os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "abi", "option_a_drop_in.cpp"),
                        "-L" + pkg, "-lmwx", "-Wl,-rpath," + pkg, "-o", str(tmp_path / "a")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
