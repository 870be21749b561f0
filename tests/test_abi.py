"""libvhx.so loads and exports every function include/*.h declares (no compute call: no GPU needed)."""
import ctypes
import os
import re

from voxelhex_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions(headers=("vhx.h", "vhx_boxtree.h", "vhx_stream.h")):
    names = set()
    for h in headers:
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^\s*[A-Za-z_][\w \*]*?\b(vhx_\w+)\s*\(", text, flags=re.M):
            names.add(m.group(1))
    return names


def test_every_declared_symbol_is_exported_and_bound():
    lib = ctypes.CDLL(N.LIB_PATH)
    declared = declared_functions()
    assert len(declared) >= 25
    bound = {name for name, _, _ in N.SIGNATURES}
    assert declared == bound, (declared ^ bound)
    for name in declared:
        assert hasattr(lib, name), name


def test_integration_binds_every_declared_function():
    """INTEGRATION.md's Rust `extern "C"` block names every function of the device and streaming headers (the
    reference-side binding a maintainer would add; the C++ host tree of vhx_boxtree.h stands in for the Rust BoxTree
    and is not bound from Rust)."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    bound = set(re.findall(r"pub fn (vhx_\w+)\s*\(", text))
    missing = declared_functions(("vhx.h", "vhx_stream.h")) - bound
    assert not missing, sorted(missing)


def test_abi_version_and_struct_sizes():
    assert N.lib().vhx_abi_version() == 6
    assert ctypes.sizeof(N.TreeDesc) == 8 * 4 + 7 * 8
    assert ctypes.sizeof(N.Camera) == 4 * 4 + 4 * 12 + 8 + 64
    assert ctypes.sizeof(N.Hits) == 9 * 8


def test_gpu_entry_points_fail_cleanly_without_a_device():
    n = ctypes.c_int(-1)
    assert N.lib().vhx_device_count(ctypes.byref(n)) == 0
    if n.value == 0:
        h = ctypes.c_void_p()
        assert N.lib().vhx_create(0, ctypes.byref(h)) == N.VHX_E_NO_DEVICE
