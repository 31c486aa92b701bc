"""Per-wave timeline of one KExpand launch of c3's shape (diagnostic).

Build the traced variant first (CPU):
    python tools/build_variants.py k_expand_direct8.hip et:DPF_EXPAND_TRACE=1
then on the GPU box:
    DPF_AMD_LIB=.../var_et/libdpf_amd.so python tools/expand_trace.py [--roots 15,16]
Prints, for n prefix roots x 7 levels (uint64, KExpand<4>): the launch's
event time, the spread of wave starts, the table fill, walk and DFS phases
(median / max), the distribution of wave end times, the number of waves alive
over time, per-CU spans and the shader clock.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_point_functions_amd import _lib, kernels as K  # noqa: E402
from distributed_point_functions_amd import value_types as V  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--roots", default="15,16")
    ap.add_argument("--depth", type=int, default=0)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    desc = V.Integer(64).descriptor(1)
    levels = 7
    gen = torch.Generator(device=dev)
    gen.manual_seed(3)
    cw = torch.randint(-2**63, 2**63 - 1, (levels, 2), dtype=torch.int64, device=dev, generator=gen)
    ccl = torch.randint(0, 2, (levels,), dtype=torch.uint8, device=dev, generator=gen)
    ccr = torch.randint(0, 2, (levels,), dtype=torch.uint8, device=dev, generator=gen)
    lib = _lib.lib()
    fn = lib.dpf_amd_debug_expand_trace
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    for lr in [int(x) for x in args.roots.split(",")]:
        n = 1 << lr
        seeds = torch.randint(-2**63, 2**63 - 1, (n, 2), dtype=torch.int64, device=dev, generator=gen)
        seeds[:, 0] &= ~1
        cbs = torch.randint(0, 2, (n,), dtype=torch.uint8, device=dev, generator=gen)
        out = torch.empty((n << levels) * 2 * 8, dtype=torch.uint8, device=dev)

        def run():
            K.expand_and_correct(seeds, cbs, levels, cw, ccl, ccr, desc, [5, 7], 0, 2, 0,
                                 n << levels, out)

        with K.forced_expand_depth(args.depth):
            for _ in range(5):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            torch.cuda.synchronize()
        D = args.depth or 4
        waves = (n << levels >> D) // 64
        buf = np.zeros(16384 * 8, dtype=np.uint64)
        assert fn(buf.ctypes.data, buf.nbytes) == 0
        t = buf.reshape(16384, 8)[:min(waves, 16384)].astype(np.int64)
        t0 = t[:, 0].min()
        rel = (t[:, :4] - t0) / 100.0  # us
        ends = np.sort(rel[:, 3])
        res = {"roots": lr, "waves": int(waves), "event_us": round(e0.elapsed_time(e1) * 1e3, 1),
               "span_us": round(float(ends[-1]), 1),
               "start_spread_us": round(float(rel[:, 0].max()), 2),
               "fill_us": [round(float(np.median(rel[:, 1] - rel[:, 0])), 2),
                           round(float((rel[:, 1] - rel[:, 0]).max()), 2)],
               "walk_us": [round(float(np.median(rel[:, 2] - rel[:, 1])), 2),
                           round(float((rel[:, 2] - rel[:, 1]).max()), 2)],
               "dfs_us": [round(float(np.median(rel[:, 3] - rel[:, 2])), 1),
                          round(float((rel[:, 3] - rel[:, 2]).min()), 1),
                          round(float((rel[:, 3] - rel[:, 2]).max()), 1)],
               "end_pct_us": {p: round(float(np.percentile(ends, p)), 1)
                              for p in (1, 10, 25, 50, 75, 90, 99, 100)},
               "start_pct_us": {p: round(float(np.percentile(rel[:, 0], p)), 1)
                                for p in (1, 50, 90, 99, 100)}}
        clk = (t[:, 5] - t[:, 4]) / np.maximum(1, t[:, 3] - t[:, 0]) * 100.0
        res["shader_mhz_median"] = round(float(np.median(clk)), 0)
        # waves alive over time, 10 us bins
        span = ends[-1]
        bins = np.arange(0, span + 10, 10)
        alive = [int(((rel[:, 0] <= b) & (rel[:, 3] > b)).sum()) for b in bins]
        res["alive_every_10us"] = alive
        # per CU (HW_ID se/sh/cu + XCC): first start, last end
        hw = t[:, 6]
        cu = (hw >> 8) & 0xF
        sh = (hw >> 12) & 0x1
        se = (hw >> 13) & 0x7
        xcc = t[:, 7] & 0xF
        key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
        spans, lastend = [], []
        for k in np.unique(key):
            m = key == k
            spans.append(rel[m, 3].max() - rel[m, 0].min())
            lastend.append(rel[m, 3].max())
        spans, lastend = np.array(spans), np.array(lastend)
        res["cus"] = int(len(spans))
        res["cu_last_end_pct_us"] = {p: round(float(np.percentile(lastend, p)), 1)
                                     for p in (0, 10, 50, 90, 100)}
        print(json.dumps(res), flush=True)
        del out, seeds, cbs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
