"""One rank's share of c5 at N = 1 / 2 / 4 / 8 on one GPU (scaling probe).

At N ranks bench.py's rank r expands tree blocks [r 2^32/N, (r+1) 2^32/N) of
the c5 key; this times rank 0's slice for each N on one device (event-timed,
back to back) and prints the per-rank time, the rounds of resident blocks it
is, and the strong-scaling efficiency t(2^32) / (N t(slice)) one rank's
kernel alone would allow.

    python tools/c5_slice_probe.py [--ns 1,2,4,8] [--reps 5]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from distributed_point_functions_amd import kernels, sharding  # noqa: E402
from distributed_point_functions_amd import value_types as V  # noqa: E402
from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    vt = V.Tuple(V.Integer(32), V.IntModN(64, bench.P64))
    dpf = DistributedPointFunction.create(DpfParameters(32, vt, 48))
    k0, _ = dpf.generate_keys(0x9E3779B9, (123456789, 987654321), seeds=(0xA5A5, 0x5A5A))
    ka = bench.key_arrays(dpf, k0, 0, dev)
    desc = dpf.value_type_descriptor(0)
    L = ka["L"]
    total = 1 << L
    res = {}
    out = torch.empty(total * desc.out_stride, dtype=torch.uint8, device=dev)
    for n in [int(x) for x in args.ns.split(",")]:
        lo, hi = sharding.block_range(total, n, 0)

        def step():
            kernels.expand_and_correct(ka["seed"], ka["cb"], L, ka["cw"], ka["ccl"], ka["ccr"],
                                       desc, ka["corr"], ka["party"], 1, lo, hi, out)
        step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            step()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        res[n] = ms
        blocks = (hi - lo) // 256 // 512
        print(json.dumps({"n": n, "leaves": hi - lo, "ms": round(ms, 3),
                          "rounds_of_blocks": round(blocks / 512, 2),
                          "efficiency_vs_n1": round(res[1] / (n * ms), 4) if 1 in res else None}),
              flush=True)


if __name__ == "__main__":
    main()
