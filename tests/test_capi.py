"""CPU-side checks of the C-ABI library: it loads and exports every symbol include/oc_engine.h
declares (no compute calls: there is no GPU here), and layout arithmetic agrees."""
import ctypes
import os
import re

import pytest

import oc_testlib as tl
from gym_cooking_amd import capi, levels

HEADER = os.path.join(tl.ROOT, "include", "oc_engine.h")


def _declared():
    src = open(HEADER).read()
    decl = r"^(?:int|void|const char\s*\*)\s*\*?\s*(oc_[a-z_]+)\s*\("  # function declarations
    return sorted(set(re.findall(decl, src, re.M)))


def test_header_declarations_match_binding():
    assert _declared() == sorted(capi.EXPORTED_SYMBOLS)


def test_library_exports_every_symbol():
    if not os.path.isfile(capi.LIB_PATH):
        pytest.skip("liboc_engine.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(capi.LIB_PATH)
    for sym in _declared():
        assert hasattr(lib, sym), sym
    lib = capi.load_library()
    assert lib.oc_abi_version() == capi.OC_ABI_VERSION
    hdr = open(HEADER).read()
    assert "#define OC_ABI_VERSION %d" % capi.OC_ABI_VERSION in hdr


def test_create_layout_and_validation_without_gpu():
    """oc_create / oc_get_layout are host-only: exercise them (and the level validation)."""
    if not os.path.isfile(capi.LIB_PATH):
        pytest.skip("liboc_engine.so not built")
    lib = capi.load_library()
    lv = levels.load_level("partial-divider_salad")
    d = capi.level_desc(lv, 2)
    h = ctypes.c_void_p()
    assert lib.oc_create(ctypes.byref(d), 2, 100, 0, ctypes.byref(h)) == 0
    lay = capi.OcLayout()
    assert lib.oc_get_layout(h, 1 << 20, ctypes.byref(lay)) == 0
    P = capi.layout_planes(2, 4)
    assert lay.num_planes == P["num_planes"] == 17  # S(A=2) = 3A + 11 bytes per env
    assert lay.pitch == 1 << 20 and lay.state_bytes == 17 << 20
    assert (lay.plane_item_loc, lay.plane_t, lay.plane_flags) == (P["item_loc"], P["t"], P["flags"])
    n = ctypes.c_int64()
    # 256 rows of 5 counters, then oc_step_n's tickets: one line for the groups, one per group of
    # 32 blocks of its grid (<= 5 blocks per CU, 256 CUs when no device is visible)
    assert lib.oc_stats_size(h, 1 << 20, ctypes.byref(n)) == 0 and n.value == (256 * 5 + (1 + 40) * 16) * 8
    assert lib.oc_destroy(h) == 0
    # bad levels are rejected with a message
    bad = capi.level_desc(lv, 2)
    bad.tiles[bad.item_cell[0]] = 0  # an item on a Floor square
    assert lib.oc_create(ctypes.byref(bad), 2, 100, 0, ctypes.byref(h)) == capi_err("ELEVEL")
    assert b"not on a counter" in lib.oc_last_error()
    edge = capi.level_desc(lv, 2)
    edge.tiles[0] = 0  # a Floor on the border loads (an off-grid action raises in step: ERR)
    assert lib.oc_create(ctypes.byref(edge), 2, 100, 0, ctypes.byref(h)) == 0
    assert lib.oc_destroy(h) == 0
    assert lib.oc_create(ctypes.byref(d), 5, 100, 0, ctypes.byref(h)) == capi_err("EINVAL")


def capi_err(name):
    return {"EINVAL": -1, "EHIP": -2, "ELEVEL": -3}[name]


def test_integration_stub_matches_binding():
    """INTEGRATION.md section 3's ctypes stub (what a maintainer would paste into the reference)
    declares the same structs, field for field and type for type, as the binding, asserts the
    binding's ABI version, and its argtypes lines name exported entry points."""
    import ctypes
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "INTEGRATION.md")) as f:
        text = f.read()
    sec = text[text.index("## 3. Direct C-ABI binding"):text.index("## 4.")]
    code = sec[sec.index("```python") + len("```python"):sec.index("```", sec.index("```python") + 3)]
    classes = re.findall(r"(class \w+\(ctypes.Structure\):.*?)(?=\n\S|\Z)", code, re.S)
    ns = {"ctypes": ctypes}
    for c in classes:
        exec(c, ns)
    for doc, ours in (("oc_level_desc", capi.OcLevelDesc), ("oc_layout", capi.OcLayout)):
        a, b = ns[doc]._fields_, ours._fields_
        assert [n for n, _ in a] == [n for n, _ in b], doc
        assert [ctypes.sizeof(t) for _, t in a] == [ctypes.sizeof(t) for _, t in b], doc
        assert ctypes.sizeof(ns[doc]) == ctypes.sizeof(ours)
    assert re.search(r"oc_abi_version\(\) == (\d+)", code).group(1) == str(capi.OC_ABI_VERSION)
    lib = capi.load_library()
    for name in re.findall(r"lib\.(oc_\w+)\.argtypes", code):
        assert hasattr(lib, name), name
