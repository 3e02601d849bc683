"""The C-ABI library loads, exports every symbol include/casim.h declares, and the
Python binding's record layouts match the compiled structs (no compute calls)."""
import ctypes as C
import os
import re

import pytest

from autoscaler_amd import abi, native

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "casim.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(ca_[a-z0-9_]+)\s*\(", src, re.M)))


def test_library_built_and_loads():
    assert os.path.exists(native.LIB_PATH), "run __graft_entry__.build()"
    lib = native.load()
    assert lib.ca_abi_version() == abi.CASIM_ABI_VERSION


def test_every_declared_symbol_is_exported():
    lib = native.load()
    decl = declared_functions()
    assert len(decl) >= 25
    missing = [f for f in decl if not hasattr(lib, f)]
    assert not missing, missing
    assert set(decl) == set(native.exported_symbols())


def test_struct_layouts_match():
    lib = native.load()
    out = (C.c_int32 * 32)()
    n = lib.ca_abi_struct_sizes(out, 32)
    assert list(out[:n]) == abi.EXPECTED_SIZES


def test_status_strings():
    lib = native.load()
    assert lib.ca_status_string(abi.CA_EUNSUPPORTED).decode().startswith("unsupported")


def test_no_device_here_fails_loudly():
    if native.device_count() > 0:
        pytest.skip("a HIP device is present")
    with pytest.raises(native.CasimError):
        native.Mirror(0)
