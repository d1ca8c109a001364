"""C-ABI library: builds for gfx950, loads without a GPU and exports every
symbol include/tpe_engine.h declares (no compute calls here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'tpe_engine.h')


def declared():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(tpe_[a-z_]+)\s*\(', src)))


def test_header_declarations_match_binding():
    from hyperopt_amd import _engine as E
    assert declared() == sorted(E.EXPORTS)


def test_library_exports_every_symbol():
    from hyperopt_amd import _engine as E
    if not os.path.exists(E.LIB_PATH):
        pytest.skip('libtpe_engine.so not built (run __graft_entry__.build())')
    lib = E.load_library()
    for name in declared():
        assert hasattr(lib, name), name
    assert lib.tpe_version().startswith(b'tpe-mi355x')
    n = ctypes.c_int32(-1)
    assert lib.tpe_device_count(ctypes.byref(n)) == 0


def test_engine_fails_loudly_without_gpu():
    """No CPU fallback: without a device the engine raises."""
    from hyperopt_amd import _engine as E
    if not os.path.exists(E.LIB_PATH):
        pytest.skip('library not built')
    n = ctypes.c_int32(0)
    E.load_library().tpe_device_count(ctypes.byref(n))
    if n.value > 0:
        pytest.skip('a GPU is visible')
    with pytest.raises(E.EngineUnavailable):
        E.Engine(0)


def test_struct_layouts_match_header():
    from hyperopt_amd import _engine as E
    assert ctypes.sizeof(E.TpeHp) == 72
    assert E.RESULT_DTYPE.itemsize == 32


def test_shard_align_matches_header():
    from hyperopt_amd import _engine as E
    m = re.search(r'#define\s+TPE_SHARD_ALIGN\s+(\d+)', open(HEADER).read())
    assert m and int(m.group(1)) == E.SHARD_ALIGN
