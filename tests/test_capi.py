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
    decl = r"^(?:int|void|const char\s*\*)\s*\*?\s*(oc_[a-z_0-9]+)\s*\("  # function declarations
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


def test_host_only_handle_and_handle_errors():
    """oc_create(..., OC_DEVICE_HOST) makes a host-only handle: no HIP call at all (oc_create
    skips the device query and the device tables).  Its device entry points refuse it with
    OC_EINVAL before touching HIP, its host ones work, and each failure is also recorded on the
    handle (oc_get_last_error)."""
    if not os.path.isfile(capi.LIB_PATH):
        pytest.skip("liboc_engine.so not built")
    lib = capi.load_library()
    lv = levels.load_level("partial-divider_salad")
    d = capi.level_desc(lv, 2)
    h = ctypes.c_void_p()
    assert lib.oc_create(ctypes.byref(d), 2, 100, capi.OC_DEVICE_HOST, ctypes.byref(h)) == 0
    buf = ctypes.create_string_buffer(256)
    assert lib.oc_get_last_error(h, buf, len(buf)) == 0 and buf.value == b""
    lay = capi.OcLayout()
    assert lib.oc_get_layout(h, 4096, ctypes.byref(lay)) == 0
    s = (ctypes.c_uint8 * lay.state_bytes)()
    a = (ctypes.c_uint8 * (2 * lay.pitch))()
    assert lib.oc_step(h, s, s, a, None, None, None, 4096, None) == capi_err("EINVAL")
    assert b"host-only handle" in lib.oc_last_error()
    n = lib.oc_get_last_error(h, buf, len(buf))
    assert n > 0 and buf.value == lib.oc_last_error()
    small = ctypes.create_string_buffer(8)  # truncated, NUL-terminated; the full length returned
    assert lib.oc_get_last_error(h, small, len(small)) == n and len(small.value) == 7
    for call in (lambda: lib.oc_reset(h, s, 4096, None),
                 lambda: lib.oc_gen_actions(h, a, 4096, 0, 0, 0, None),
                 lambda: lib.oc_state_checksum(h, s, 4096, s, None)):
        assert call() == capi_err("EINVAL") and b"host-only handle" in lib.oc_last_error()
    nn = ctypes.c_int32()
    assert lib.oc_reachability(h, ctypes.byref(nn), None, 0, None, 0) == 0 and nn.value > 0
    assert lib.oc_set_likelihood_form(h, 7) == capi_err("EINVAL")
    assert lib.oc_get_last_error(h, buf, len(buf)) > 0 and b"likelihood form 7" in buf.value
    assert lib.oc_set_likelihood_form(h, capi.OC_LIK_FORM_GROUPED) == 0
    assert lib.oc_destroy(h) == 0
    assert lib.oc_create(ctypes.byref(d), 2, 100, -2, ctypes.byref(h)) == capi_err("EINVAL")


def test_cpu_stepper_on_host_only_handle():
    """engine.CpuStepper steps on a host-only handle (oc_cpu_step), threaded, and its handle
    refuses a device call."""
    if not os.path.isfile(capi.LIB_PATH):
        pytest.skip("liboc_engine.so not built")
    import numpy as np
    from gym_cooking_amd.engine import CpuStepper
    cs = CpuStepper("partial-divider_salad", 2, 70000, nthreads=4)
    s0 = cs.new_state()
    s1 = np.empty_like(s0)
    act = np.full(2 * cs.pitch, 3, np.uint8)
    tot = np.zeros(5, np.uint64)
    cs.step(s0, s1, act, totals=tot)
    assert not np.array_equal(s0, s1)
    lib = cs.lib
    assert lib.oc_reset(cs._h, s1.ctypes.data, cs.B, None) == capi_err("EINVAL")
