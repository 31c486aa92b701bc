"""Builds the native library libdpf_amd.so (HIP kernels for gfx950 + the C++
host library + the C ABI) in-tree with hipcc.

    python -m distributed_point_functions_amd.build_native [--force]
"""
from __future__ import annotations

import concurrent.futures
import glob
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


def _deps_mtime(src: str) -> float:
    """Newest mtime of `src` and the project headers it includes (quoted
    includes, followed recursively through csrc/ and include/)."""
    seen, todo, newest = set(), [src], 0.0
    while todo:
        f = todo.pop()
        if f in seen:
            continue
        seen.add(f)
        newest = max(newest, os.path.getmtime(f))
        with open(f, errors="replace") as fh:
            text = fh.read()
        for inc in _INCLUDE_RE.findall(text):
            for d in (os.path.dirname(f), CSRC, os.path.join(ROOT, "include")):
                cand = os.path.join(d, inc)
                if os.path.exists(cand):
                    todo.append(os.path.normpath(cand))
                    break
    return newest


def _compile(src: str, force: bool, obj_dir: str = OBJ_DIR, defines=()) -> str:
    obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= _deps_mtime(src):
        return obj
    cmd = ["hipcc"] + CXXFLAGS + ["-D" + d for d in defines] + ["-c", src, "-o", obj + ".tmp"]
    if src.endswith(".hip"):
        cmd[1:1] = ["--offload-arch=" + ARCH, "-x", "hip"]
    else:
        # host-only C++ (no device pass), HIP runtime API from ROCm
        cmd[1:1] = ["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I" + os.path.join(ROCM, "include"),
                    "-maes", "-msse4.1"]
    subprocess.check_call(cmd)
    os.replace(obj + ".tmp", obj)
    return obj


def build(force: bool = False, jobs: int = 8) -> str:
    os.makedirs(OBJ_DIR, exist_ok=True)
    srcs = _sources()
    with concurrent.futures.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    if (force or not os.path.exists(LIB) or
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
