"""The C-ABI library loads on a CPU-only machine and exports every function
include/dpf_amd.h declares (no compute calls)."""
import ctypes
import os
import re
import subprocess

from distributed_point_functions_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dpf_amd.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dpf_amd_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    assert len(names) >= 40
    for must in ("dpf_amd_evaluate_seeds", "dpf_amd_expand_and_correct",
                 "dpf_amd_evaluate_points", "dpf_amd_evaluate_points_batched", "dpf_amd_inner_product",
                 "dpf_amd_evaluate_until", "dpf_amd_pir_server_handle_request"):
        assert must in names


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (dpf_amd_\w+)", out))
    assert set(declared_functions()) <= exported


def test_integration_index_lists_every_declared_symbol():
    """INTEGRATION.md's generated index (tools/abi_index.py --write) names
    every function the header declares, so the binding guide cannot fall
    behind the boundary."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    begin, end = doc.index("<!-- abi-index:begin -->"), doc.index("<!-- abi-index:end -->")
    listed = set(re.findall(r"\| `(dpf_amd_\w+)` \|", doc[begin:end]))
    assert set(declared_functions()) == listed, set(declared_functions()) ^ listed


def test_version_and_error_plumbing():
    L = _lib.lib()
    assert L.dpf_amd_version().decode().startswith("dpf_amd")
    # Tier-1 argument validation runs on the host before any HIP call.
    rc = L.dpf_amd_evaluate_seeds(1, 3, 2, None, None, None, 0, None, None, None,
                                  0, 0, 0, 0, None, None, None)
    assert rc == 3
    assert b"num_correction_words" in L.dpf_amd_last_error()


def test_no_torch_types_in_the_abi():
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)  # code, not comments
    for bad in ("torch", "at::", "c10", "std::", "Tensor"):
        assert bad not in text


def test_kernel_choice_hooks_are_per_thread():
    """dpf_amd_set_expand_depth / dpf_amd_set_scan_m4 change only the calling
    thread's launches (no GPU needed: the setters touch no device state)."""
    import threading
    from distributed_point_functions_amd import _lib
    L = _lib.lib()
    assert L.dpf_amd_set_expand_depth(4) == 0
    assert L.dpf_amd_set_scan_m4(1) in (-1, 0, 1)
    seen = {}

    def other():
        seen["depth"] = L.dpf_amd_set_expand_depth(2)
        seen["depth_back"] = L.dpf_amd_set_expand_depth(0)
        seen["scan"] = L.dpf_amd_set_scan_m4(0)

    t = threading.Thread(target=other)
    t.start()
    t.join()
    assert seen["depth"] == 0 and seen["depth_back"] == 2
    assert seen["scan"] != 1 or os.environ.get("DPF_AMD_SCAN_M4") == "1"
    assert L.dpf_amd_set_expand_depth(0) == 4
    assert L.dpf_amd_set_scan_m4(-1) == 1


def test_expand_roots_hook_validates_and_is_per_thread():
    """dpf_amd_set_expand_roots: -1 / 0 / 1, -2 (unchanged) otherwise, per
    thread (no GPU needed)."""
    import threading
    from distributed_point_functions_amd import _lib
    L = _lib.lib()
    start = -1 if os.environ.get("DPF_AMD_EXPAND_ROOTS") != "0" else 0
    assert L.dpf_amd_set_expand_roots(2) == -2
    assert L.dpf_amd_set_expand_roots(-2) == -2
    assert L.dpf_amd_set_expand_roots(1) == start
    seen = {}

    def other():
        seen["first"] = L.dpf_amd_set_expand_roots(0)
        seen["back"] = L.dpf_amd_set_expand_roots(start)

    t = threading.Thread(target=other)
    t.start()
    t.join()
    assert seen == {"first": start, "back": 0}
    assert L.dpf_amd_set_expand_roots(start) == 1


def test_walk_and_dcf_kernel_hooks_validate_and_are_per_thread():
    """dpf_amd_set_walk_mode (0 / 1 / 2) and dpf_amd_set_dcf_kernel (0 / 1):
    invalid values are refused unchanged, and another thread keeps its own
    setting."""
    import threading
    from distributed_point_functions_amd import _lib
    L = _lib.lib()
    assert L.dpf_amd_set_walk_mode(3) == -2
    assert L.dpf_amd_set_dcf_kernel(2) == -2
    assert L.dpf_amd_set_walk_mode(1) == 0
    assert L.dpf_amd_set_dcf_kernel(1) == 0
    seen = {}

    def other():
        seen["walk"] = L.dpf_amd_set_walk_mode(2)
        seen["dcf"] = L.dpf_amd_set_dcf_kernel(0)

    t = threading.Thread(target=other)
    t.start()
    t.join()
    assert seen == {"walk": 0, "dcf": 0}
    assert L.dpf_amd_set_walk_mode(0) == 1
    assert L.dpf_amd_set_dcf_kernel(0) == 1


def test_prefix_expand_and_thread_cache_hooks():
    """dpf_amd_set_prefix_expand (0 / 1 / 2) is per thread and refuses other
    values; dpf_amd_set_thread_cache_cap refuses a negative cap (no GPU: the
    setters touch no device state)."""
    import threading
    from distributed_point_functions_amd import _lib
    L = _lib.lib()
    assert L.dpf_amd_set_prefix_expand(3) == -2
    assert L.dpf_amd_set_prefix_expand(-1) == -2
    assert L.dpf_amd_set_prefix_expand(2) == 0
    assert L.dpf_amd_set_prefix_expand(1) == 2
    seen = {}

    def other():
        seen["mode"] = L.dpf_amd_set_prefix_expand(0)

    t = threading.Thread(target=other)
    t.start()
    t.join()
    assert seen == {"mode": 0}
    assert L.dpf_amd_set_prefix_expand(0) == 1
    assert L.dpf_amd_set_thread_cache_cap(-1) == 3
    assert b"cap" in L.dpf_amd_last_error()
    assert L.dpf_amd_set_thread_cache_cap(64) == 0


def test_library_is_stamped_with_its_sources():
    """build() stamps the hash of csrc/ and include/ into the library
    (dpf_amd_version "... src:<sha256>") and relinks when the loaded one's
    stamp is not the tree's: the library the tests load is the one these
    sources build."""
    from distributed_point_functions_amd import _lib, build_native
    v = _lib.lib().dpf_amd_version().decode()
    assert v.rsplit("src:", 1)[-1] == build_native.source_hash()
    assert build_native.library_source_hash() == build_native.source_hash()
