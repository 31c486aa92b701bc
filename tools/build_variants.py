"""Builds A/B variants of one kernel translation unit into
distributed_point_functions_amd/_native/var_<name>/libdpf_amd.so (select one
at run time with DPF_AMD_LIB=<path>).  The other objects are the main build's.

    python tools/build_variants.py k_expand_c5.hip name1:DEF=1,DEF2=3 name2:...
    python tools/build_variants.py all name:DEF=1     # every .hip TU
    python tools/build_variants.py k_pir.hip+kernels_capi.cc name:DEF=1
"""
import concurrent.futures
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_point_functions_amd import build_native as B  # noqa: E402


def main():
    tu = sys.argv[1]  # one unit, several joined by "+", or "all" (every .hip unit)
    tus = tu.split("+")
    B.build()
    objs = [os.path.join(B.OBJ_DIR, os.path.basename(s) + ".o") for s in B._sources()]
    others = [o for o in objs if os.path.basename(o)[:-2] not in tus]

    def one(spec):
        name, _, defs = spec.partition(":")
        d = os.path.join(B.OUT_DIR, "var_" + name)
        os.makedirs(d, exist_ok=True)
        dl = [x for x in defs.split(",") if x]
        if tu == "all":  # every device translation unit with the defines
            mine = [B._compile(src, True, d, dl) for src in B._sources() if src.endswith(".hip")]
            rest = [o for o in objs if not o.endswith(".hip.o")]
            parts = mine + rest
        else:
            parts = [B._compile(os.path.join(B.CSRC, t), True, d, dl) for t in tus] + others
        lib = os.path.join(d, "libdpf_amd.so")
        subprocess.check_call(["hipcc", "--offload-arch=" + B.ARCH, "-shared", "-fPIC", "-o", lib] +
                              parts + ["-lpthread"])
        return lib

    with concurrent.futures.ThreadPoolExecutor(8) as ex:
        for lib in ex.map(one, sys.argv[2:]):
            print(lib)


if __name__ == "__main__":
    main()
