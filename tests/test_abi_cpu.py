"""The C-ABI library builds/loads on a CPU host and exports every entry point
include/vsrk.h declares (no compute calls without a device)."""
import re
from pathlib import Path

from vsr_amd import _native

HEADER = Path(__file__).resolve().parent.parent / "include" / "vsrk.h"


def declared():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"\b(vsrk_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    names = declared()
    assert "vsrk_conv_fwd" in names and "vsrk_conv_wgrad" in names and len(names) >= 10


def test_library_exports_every_declared_symbol(native):
    for name in declared():
        assert hasattr(native, name), f"{name} declared in include/vsrk.h but not exported"


def test_binding_table_matches_header():
    assert sorted(_native.exported_symbols()) == declared()


def test_version_and_error_text(native):
    assert native.vsrk_version().decode().startswith("vsrk")
    assert isinstance(native.vsrk_last_error(), bytes)


def test_workspace_queries_are_host_only(native):
    import ctypes as C
    from vsr_amd._native import ConvDesc, Tensor5
    d = ConvDesc(3, 3, 3, 1, 1, 1, 0, 0, 1.0, 0, 1)
    x = Tensor5(None, 4, 16, 128, 128, 64, 0, 0, 0, 0, 1, 1)
    y = Tensor5(None, 4, 16, 128, 128, 32, 0, 0, 0, 0, 1, 1)
    assert native.vsrk_conv_wgrad_workspace_size(C.byref(d), C.byref(x), C.byref(y)) > 0
    assert native.vsrk_conv_packed_elems(32, 64, 3, 3, 3, 0) == 27 * 128 * 64
