"""The C-ABI library loads and exports every symbol include/vdiff.h declares (CPU, no compute)."""
import ctypes
import os
import re

from conftest import ROOT

from vdiff import _lib


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "vdiff.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(vd_[a-z0-9_]+)\s*\(", src))


def test_library_exports_header_symbols():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    declared = _header_symbols()
    assert len(declared) >= 20
    for name in sorted(declared):
        assert hasattr(lib, name), name
    assert declared == set(_lib.EXPORTED_SYMBOLS), declared ^ set(_lib.EXPORTED_SYMBOLS)


def test_version_and_error_channel():
    lib = _lib.load()
    assert lib.vd_version() == _lib.ABI_VERSION
    # an invalid call fails loudly without touching the GPU
    rc = lib.vd_q_sample(None, None, None, None, None, None, 0, 0, 0, None)
    assert rc == 1
    assert b"null" in lib.vd_last_error()


def test_structs_match_header():
    assert ctypes.sizeof(_lib.ConvDesc) == 21 * 4
    assert ctypes.sizeof(_lib.AttnDesc) == 4 * 4 + 6 * 8 + 4 + 4
    # vd_xattn_desc: the query descriptor, int kv_len (+4 padding), three int64 strides
    assert ctypes.sizeof(_lib.XAttnDesc) == ctypes.sizeof(_lib.AttnDesc) + 8 + 3 * 8
