"""The C-ABI library loads on the host and exports every symbol declared in
include/vaeteb.h (no GPU needed: no compute calls here)."""
import ctypes
import os

from vaeteb import _lib


def test_header_parses_and_all_symbols_exported():
    protos = _lib.parse_header()
    assert len(protos) >= 20
    dll = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in protos if not hasattr(dll, n)]
    assert not missing, missing


def test_bound_library_reports_version_and_errors():
    lib = _lib.lib()
    assert lib.fns["vt_abi_version"]() >= 1
    assert isinstance(lib.last_error(), str)


def test_argument_errors_map_to_value_error():
    import pytest
    # shape validation happens before any device work, so this is safe without a GPU
    with pytest.raises(ValueError):
        _lib.call("vt_fe_spectrum", None, 0, 4096, 8192, 2048, 0, None, None, None)
    with pytest.raises(ValueError):
        _lib.call("vt_fft", None, None, 1, 12, 0, None, 1, None)   # not a power of two


def test_library_is_in_tree():
    assert os.path.commonpath([_lib.LIB_PATH, os.path.dirname(os.path.dirname(__file__))])
