"""The C-ABI library builds/loads on a CPU host and exports every entry point
include/*.h declares (vsrk.h: the generator path; vsrk_data.h: the batch
gather) -- no compute calls without a device."""
import re
from pathlib import Path

from vsr_amd import _native

INCLUDE = Path(__file__).resolve().parent.parent / "include"
HEADER = INCLUDE / "vsrk.h"


def declared():
    text = "".join(p.read_text() for p in sorted(INCLUDE.glob("*.h")))
    return sorted(set(re.findall(r"\b(vsrk_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    names = declared()
    assert "vsrk_conv_fwd" in names and "vsrk_conv_wgrad" in names and len(names) >= 10


def test_library_exports_every_declared_symbol(native):
    for name in declared():
        assert hasattr(native, name), f"{name} declared in include/ but not exported"


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


# ---- INTEGRATION.md's reference-side binding stub vs _native vs the header --
DOC = HEADER.parent.parent / "INTEGRATION.md"
_CTYPE = {"int32_t": "c_int", "int64_t": "c_long", "float": "c_float", "double": "c_double"}


def _doc_structs():
    import ctypes as C
    text = DOC.read_text()
    ns = {"C": C}
    for name in ("Tensor5", "ConvDesc"):
        m = re.search(rf"^class {name}\(C\.Structure\):.*?\]\n", text, re.S | re.M)
        assert m, f"INTEGRATION.md has no {name} struct"
        exec(m.group(0), ns)  # our own document's ctypes declaration
    return ns["Tensor5"], ns["ConvDesc"]


def _header_fields(struct):
    body = re.search(rf"typedef struct {struct} \{{(.*?)\}} {struct};", HEADER.read_text(), re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    out = []
    for decl in filter(None, (d.strip() for d in body.split(";"))):
        ptr = "*" in decl
        typ, names = decl.replace("*", " ").replace("const ", "").split(None, 1)
        for n in (x.strip() for x in names.split(",")):
            out.append((n, "c_void_p" if ptr else _CTYPE[typ]))
    return out


def _fields(cls):
    return [(n, t.__name__) for n, t in cls._fields_]


def test_integration_doc_structs_match_binding_and_header():
    import ctypes as C
    t5, cd = _doc_structs()
    for doc, nat, hdr in ((t5, _native.Tensor5, "vsrk_tensor5"), (cd, _native.ConvDesc, "vsrk_conv_desc")):
        assert _fields(doc) == _fields(nat), hdr
        assert _fields(nat) == _header_fields(hdr), hdr
        assert C.sizeof(doc) == C.sizeof(nat)


def test_integration_doc_names_every_net():
    text = DOC.read_text()
    for net in ("EDSRNet", "DUFNet", "DRFNet", "DRFSISRNet"):
        assert f"{net}" in text.split("## 2.")[0], net
