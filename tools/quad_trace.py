"""Phase times of KEvaluatePointsQuad from in-kernel timestamps (diagnostic).

Build the traced variant first (CPU):
    python tools/build_variants.py k_walk.hip qt:DPF_QUAD_TRACE=1
then on the GPU box:
    DPF_AMD_LIB=.../var_qt/libdpf_amd.so python tools/quad_trace.py
One key's EvaluateAt of 16,384 random points (log_domain 128, uint128: the
per-call c2 shape).  Prints, over the blocks of the last launch, the median /
max of each phase (tables, walk, hash + emit) in microseconds, the shader
clock the block ran at and the walk's cycles per level.
"""
import ctypes
import json
import os
import random
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_point_functions_amd import _lib  # noqa: E402
from distributed_point_functions_amd import value_types as V  # noqa: E402
from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters  # noqa: E402


def main():
    torch.cuda.set_device(0)
    dpf = DistributedPointFunction.create(DpfParameters(128, V.Integer(128)))
    k0 = dpf.generate_keys(12345, 678, seeds=(1, 2))[0]
    rng = random.Random(7)
    pts = [rng.getrandbits(128) for _ in range(16384)]
    for _ in range(10):
        dpf.evaluate_at(k0, 0, pts)
    lib = _lib.lib()
    fn = lib.dpf_amd_debug_quad_trace
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    buf = np.zeros(4096 * 8, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    t = buf.reshape(4096, 8).astype(np.int64)
    t = t[t[:, 1] > 0]
    clk = t[:, 0::2]
    rt = t[:, 1::2]
    ph = np.diff(rt, axis=1) / 100.0  # 100 MHz -> us
    cyc = np.diff(clk, axis=1)
    res = {"blocks": int(t.shape[0]), "span_us": float((rt[:, 3].max() - rt[:, 0].min()) / 100.0),
           "start_spread_us": float((rt[:, 0].max() - rt[:, 0].min()) / 100.0),
           "shader_mhz": float(np.median(cyc.sum(1) / (rt[:, 3] - rt[:, 0]) * 100.0)),
           "walk_cycles_per_level": float(np.median(cyc[:, 1]) / 128.0)}
    for i, n in enumerate(["tables", "walk", "hash_emit"]):
        res[n + "_us"] = {"median": float(np.median(ph[:, i])), "max": float(ph[:, i].max())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
