"""Phase times of KExpandCoop from in-kernel timestamps (diagnostic).

Build the traced variants first (CPU):
    python tools/build_variants.py k_expand_direct8.hip ct8:DPF_COOP_TRACE=1
    python tools/build_variants.py k_expand_direct16.hip ct16:DPF_COOP_TRACE=1
then on the GPU box:
    DPF_AMD_LIB=.../var_ct8/libdpf_amd.so python tools/coop_trace.py c1
    DPF_AMD_LIB=.../var_ct16/libdpf_amd.so python tools/coop_trace.py sel
Prints, over the blocks of the last launch, the median / max of each phase
(tables, walk, BFS, leaves) in microseconds and the spread of block starts.
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_configs as B  # noqa: E402
from distributed_point_functions_amd import _lib, kernels  # noqa: E402
from distributed_point_functions_amd import value_types as V  # noqa: E402
from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters  # noqa: E402


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "c1"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if what == "c1":
        vt, ld = V.Integer(64), 20
    else:
        vt, ld = V.XorWrapper(128), 26
    dpf = DistributedPointFunction.create(DpfParameters(ld, vt))
    k0 = dpf.generate_keys(12345, 678 if vt.bits < 128 else 1 << 77, seeds=(1, 2))[0]
    kd = B.key_dev(dpf, k0, 0, dev)
    desc = dpf.value_type_descriptor(0)
    L = kd["L"]
    cepb = 1 << (ld - L)
    leaves = min(1 << L, 1 << 19)
    out = torch.empty(leaves * cepb * desc.out_stride, dtype=torch.uint8, device=dev)

    def step():
        kernels.expand_and_correct(kd["seed"], kd["cb"], L, kd["cw"], kd["ccl"], kd["ccr"],
                                   desc, kd["corr"], kd["party"], cepb, 0, leaves, out)

    with kernels.forced_expand_depth(-2):
        ms = B.ev_time(step, 20)
        step()
    torch.cuda.synchronize()
    lib = _lib.lib()
    fn = lib.dpf_amd_debug_coop_trace
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    buf = np.zeros(4096 * 8, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    blocks = leaves // 2048
    t = buf.reshape(4096, 8)[:blocks, :5].astype(np.int64)
    t0 = t[:, 0].min()
    ph = np.diff(t, axis=1) / 100.0  # 100 MHz -> us
    names = ["tables", "walk", "bfs", "leaves"]
    res = {"config": what, "tree_leaves": leaves, "blocks": blocks, "event_ms": round(ms * 1e3, 4),
           "span_us": (t[:, 4].max() - t0) / 100.0,
           "start_spread_us": (t[:, 0].max() - t0) / 100.0}
    for i, n in enumerate(names):
        res[n + "_us"] = {"median": float(np.median(ph[:, i])), "max": float(ph[:, i].max())}
    # the shader clock the blocks ran at (s_memtime against s_memrealtime)
    cf = lib.dpf_amd_debug_coop_clock
    cf.restype = ctypes.c_int
    cf.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    clk = np.zeros(4096 * 8, dtype=np.uint64)
    if cf(clk.ctypes.data, clk.nbytes) == 0:
        ck = clk.reshape(4096, 8)[:blocks, :5].astype(np.int64)
        res["shader_mhz"] = float(np.median((ck[:, 4] - ck[:, 0]) / (t[:, 4] - t[:, 0]) * 100.0))
    # quad BFS levels (slots 5-7: after the 128-, 256- and 512-child levels)
    q = buf.reshape(4096, 8)[:blocks].astype(np.int64)
    if (q[:, 5:8] > 0).all():
        marks = [q[:, 2], q[:, 5], q[:, 6], q[:, 7], q[:, 3]]
        for i, n in enumerate(["bfs128", "bfs256", "bfs512", "bfs1024"]):
            res[n + "_us"] = float(np.median((marks[i + 1] - marks[i]) / 100.0))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
