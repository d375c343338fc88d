"""CPU tests of the C-ABI library: it loads and exports every symbol the
public header declares; calls that need a device fail with a status code
(never abort) when there is none."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "wvgpu.h")


def header_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(wvg_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from weaviate_amd import _lib

    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_covers_header():
    from weaviate_amd import _lib

    assert set(header_symbols()) == set(_lib.SIGNATURES)


def test_abi_version_and_error_path():
    from weaviate_amd import _lib

    lib = _lib.load()
    assert lib.wvg_abi_version() == _lib.ABI_VERSION == 2
    # a null-argument call returns a negative status and sets the message
    rc = lib.wvg_device_count(None)
    assert rc == _lib.WVG_ERR_INVALID
    assert b"null" in lib.wvg_last_error()


def test_library_is_gfx950_code_object():
    from weaviate_amd import _lib

    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="only meaningful without a GPU")
def test_open_without_device_fails_cleanly():
    from weaviate_amd import _lib

    lib = _lib.load()
    h = ctypes.c_void_p()
    rc = lib.wvg_open(0, ctypes.byref(h))
    assert rc in (_lib.WVG_ERR_DEVICE, _lib.WVG_ERR_INVALID)
    assert not h.value


def test_exports_equal_header():
    """The product library exports exactly the header's entry points: no
    tuning setter (wvgx_*), no A/B knobs -- those live in the tools build."""
    import subprocess

    from weaviate_amd import _lib

    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], check=True, capture_output=True,
                         text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.split() and ln.split()[-1].startswith("wvg")}
    assert exported == set(header_symbols())


def test_options_struct_matches_library():
    import ctypes as ct

    from weaviate_amd import _lib

    lib = _lib.load()
    o = _lib.Options()
    lib.wvg_options_default(ct.byref(o))
    assert o.size == ct.sizeof(_lib.Options)
    assert (o.mfma_min_queries, o.cache_reuse, o.merge_wait_us, o.batch_screen, o.coalesce) == (32, 1, 0, 1, 1)
    bad = _lib.Options()
    lib.wvg_options_default(ct.byref(bad))
    bad.size = 3
    h = ct.c_void_p()
    assert lib.wvg_open_ex(0, ct.byref(bad), ct.byref(h)) == _lib.WVG_ERR_INVALID
    assert not h.value
