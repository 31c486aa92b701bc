"""Builds the native library libdpf_amd.so (HIP kernels for gfx950 + the C++
host library + the C ABI) in-tree with hipcc.

    python -m distributed_point_functions_amd.build_native [--force]
"""
from __future__ import annotations

import concurrent.futures
import glob
import hashlib
import os
import re
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OUT_DIR = os.path.join(PKG, "_native")
OBJ_DIR = os.path.join(OUT_DIR, "obj")
LIB = os.path.join(OUT_DIR, "libdpf_amd.so")
# C++ API consumer test (tests/cpp/api_test.cc) linked against LIB.
CPP_TEST_SRC = os.path.join(ROOT, "tests", "cpp", "api_test.cc")
CPP_TEST = os.path.join(OUT_DIR, "cpp_api_test")
# C++ API wall-clock bench of the BASELINE configs c1-c3 (tools/cpp_api_bench.cc).
CPP_BENCH_SRC = os.path.join(ROOT, "tools", "cpp_api_bench.cc")
CPP_BENCH = os.path.join(OUT_DIR, "cpp_api_bench")
# The reference's published experiment workloads through the C++ API
# (tools/experiments_bench.cc; driven by bench.py --experiments).
EXP_BENCH_SRC = os.path.join(ROOT, "tools", "experiments_bench.cc")
EXP_BENCH = os.path.join(OUT_DIR, "experiments_bench")
ARCH = os.environ.get("DPF_AMD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
            "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]


def _hashed_files():
    """Every file the library is built from: csrc/ and include/ (sorted)."""
    fs = []
    for d, pats in ((CSRC, ("*.h", "*.cc", "*.hip")),
                    (os.path.join(ROOT, "include"), ("*.h", os.path.join("dpf_amd", "*.h")))):
        for pat in pats:
            fs += glob.glob(os.path.join(d, pat))
    return sorted(fs)


def source_hash() -> str:
    """SHA-256 over the library's sources (relative path and bytes of each)
    and its build flags: what dpf_amd_version() reports after "src:"."""
    h = hashlib.sha256()
    h.update(repr((ARCH, CXXFLAGS[:5])).encode())
    for f in _hashed_files():
        h.update(os.path.relpath(f, ROOT).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()


def library_source_hash(path: str = LIB):
    """The source hash stamped into a built library (read from its bytes,
    without loading it), or None."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    m = re.search(rb"T-table AES in LDS\) src:([0-9a-f]{64}|unknown)", data)
    return m.group(1).decode() if m else None


def _sources():
    # largest device translation units first so the parallel build ends early
    srcs = glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cc"))
    return sorted(srcs, key=lambda s: ("k_expand" not in s, not s.endswith(".hip"), s))


def _headers_mtime():
    hs = (glob.glob(os.path.join(CSRC, "*.h")) +
          glob.glob(os.path.join(ROOT, "include", "*.h")) +
          glob.glob(os.path.join(ROOT, "include", "dpf_amd", "*.h")))
    return max([os.path.getmtime(h) for h in hs] + [0])


_INCLUDE_RE = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _deps(src: str):
    """`src` and the project headers it includes (quoted includes, followed
    recursively through csrc/ and include/), sorted."""
    seen, todo = set(), [src]
    while todo:
        f = todo.pop()
        if f in seen:
            continue
        seen.add(f)
        with open(f, errors="replace") as fh:
            text = fh.read()
        for inc in _INCLUDE_RE.findall(text):
            for d in (os.path.dirname(f), CSRC, os.path.join(ROOT, "include")):
                cand = os.path.join(d, inc)
                if os.path.exists(cand):
                    todo.append(os.path.normpath(cand))
                    break
    return sorted(seen)


def _object_key(src: str, cmd) -> str:
    """What an object is built from: its compile command and the bytes of
    its source and every header it includes."""
    h = hashlib.sha256("\0".join(cmd).encode())
    for f in _deps(src):
        with open(f, "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read() + b"\0")
    return h.hexdigest()


def _compile(src: str, force: bool, obj_dir: str = OBJ_DIR, defines=()) -> str:
    """Compiles `src` unless its object was built from the same bytes and
    command (content hashes, not mtimes)."""
    obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
    stamp = obj + ".key"
    cmd = ["hipcc"] + CXXFLAGS + ["-D" + d for d in defines] + ["-c", src, "-o", obj + ".tmp"]
    if src.endswith(".hip"):
        cmd[1:1] = ["--offload-arch=" + ARCH, "-x", "hip"]
    else:
        # host-only C++ (no device pass), HIP runtime API from ROCm
        cmd[1:1] = ["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I" + os.path.join(ROCM, "include"),
                    "-maes", "-msse4.1"]
    key = _object_key(src, cmd)
    if not force and os.path.exists(obj) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read() == key:
                return obj
    subprocess.check_call(cmd)
    os.replace(obj + ".tmp", obj)
    with open(stamp, "w") as f:
        f.write(key)
    return obj


def build(force: bool = False, jobs: int = 8) -> str:
    """Compiles the units whose bytes or command changed (content hashes) and
    relinks whenever the library's stamped source hash is not the tree's — a
    stale or foreign .so is replaced whatever its mtime."""
    os.makedirs(OBJ_DIR, exist_ok=True)
    srcs = _sources()
    want = source_hash()
    # the hash goes into the one unit that defines dpf_amd_version
    defines = {os.path.join(CSRC, "kernels_capi.cc"): ('DPF_AMD_SOURCE_HASH="%s"' % want,)}
    with concurrent.futures.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, defines=defines.get(s, ())), srcs))
    if (force or not os.path.exists(LIB) or library_source_hash() != want or
            os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs)):
        tmp = LIB + ".tmp%d" % os.getpid()
        subprocess.check_call(["hipcc", "--offload-arch=" + ARCH, "-shared", "-fPIC",
                               "-o", tmp] + objs + ["-lpthread"])
        os.replace(tmp, LIB)
    for src, exe in ((CPP_TEST_SRC, CPP_TEST), (CPP_BENCH_SRC, CPP_BENCH),
                     (EXP_BENCH_SRC, EXP_BENCH)):
        if os.path.exists(src) and (
                force or not os.path.exists(exe) or
                os.path.getmtime(exe) < max(os.path.getmtime(LIB), os.path.getmtime(src),
                                            _headers_mtime())):
            # the reference's C++ API, compiled as a caller would: plain g++ on
            # include/ and the shared library, no HIP toolchain
            tmp = exe + ".tmp%d" % os.getpid()
            subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall",
                                   "-I" + os.path.join(ROOT, "include"), src,
                                   "-L" + OUT_DIR, "-ldpf_amd", "-Wl,-rpath,$ORIGIN", "-o", tmp])
            os.replace(tmp, exe)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
