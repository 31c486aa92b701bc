"""Expansion kernel variants across launch sizes (single key and batched
keys) on one MI355X: kernel time per forced variant (dpf_amd_set_expand_depth:
D = 1/2/4/5/6/8 KExpand, -1/-2/-3 KExpandCoop E = 0/1/-2, 0 automatic), HIP events on the
launch stream.  XorWrapper<uint128> (the PIR selection type) and uint64 (c1).

    python tools/expand_sweep.py [single|large|batched]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_configs as B  # noqa: E402
from distributed_point_functions_amd import kernels  # noqa: E402
from distributed_point_functions_amd import value_types as V  # noqa: E402
from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
mode = sys.argv[1] if len(sys.argv) > 1 else "single"


def keyset(ld, vt, q):
    dpf = DistributedPointFunction.create(DpfParameters(ld, vt))
    keys = [dpf.generate_keys((12345 + 7 * i) % (1 << ld), 678 if vt.bits < 128 else 1 << 77,
                              seeds=(1 + i, 2 + i))[0] for i in range(q)]
    kd = [B.key_dev(dpf, k, 0, dev) for k in keys]
    return dpf, kd


if mode in ("single", "large"):
    cases = [(V.Integer(64), 12), (V.Integer(64), 16), (V.XorWrapper(128), 16),
             (V.Integer(64), 17), (V.Integer(64), 18), (V.Integer(64), 20),
             (V.XorWrapper(128), 19), (V.Integer(64), 22), (V.Integer(64), 24),
             (V.XorWrapper(128), 24)]
    if mode == "large":  # 2^24-2^28 tree leaves: D = 4 / 5 / 6 / 8 around the D = 8 threshold
        cases = [(V.Integer(64), 25), (V.Integer(64), 26), (V.Integer(64), 27),
                 (V.Integer(64), 28), (V.Integer(64), 29)]
    for vt, ld in cases:
        dpf, (kd,) = keyset(ld, vt, 1)
        desc = dpf.value_type_descriptor(0)
        L = kd["L"]
        cepb = 1 << (ld - L)
        out = torch.empty((1 << L) * cepb * desc.out_stride, dtype=torch.uint8, device=dev)
        res = {}
        depths = (4, 5, 6, 8, 0) if mode == "large" else (2, 4, 5, 8, -3, -1, -2, 0)
        for D in depths:  # the automatic choice last (warm clocks)
            def step():
                kernels.expand_and_correct(kd["seed"], kd["cb"], L, kd["cw"], kd["ccl"], kd["ccr"],
                                           desc, kd["corr"], kd["party"], cepb, 0, 1 << L, out)
            with kernels.forced_expand_depth(D):
                res["D%d" % D] = round(B.ev_time(step, 20) * 1e3, 4)
        print(json.dumps({"mode": "single", "type": repr(vt), "log_domain": ld, "tree_leaves": 1 << L,
                          "ms": res}), flush=True)
else:
    for ld, q in [(19, 8), (26, 1), (19, 64), (22, 16), (16, 100)]:
        vt = V.XorWrapper(128)
        dpf, kd = keyset(ld, vt, q)
        desc = dpf.value_type_descriptor(0)
        L = kd[0]["L"]
        leaves = min(1 << L, (1 << 26) // 128 if ld >= 19 else 1 << L)  # PIR: ceil(N/128) blocks
        seeds = torch.cat([k["seed"] for k in kd])
        cbs = torch.cat([k["cb"] for k in kd])
        cws = torch.cat([k["cw"] for k in kd])
        ccl = torch.cat([k["ccl"] for k in kd])
        ccr = torch.cat([k["ccr"] for k in kd])
        corr = [k["corr"] for k in kd]
        parties = [k["party"] for k in kd]
        out = torch.empty(q * leaves * 16, dtype=torch.uint8, device=dev)
        res = {}
        for D in (2, 4, 5, 6, 8, -3, -1, -2, 0):  # the automatic choice last (warm clocks)
            def step():
                kernels.expand_and_correct_batched(seeds, cbs, L, cws, ccl, ccr, desc, corr,
                                                   parties, 1, 0, leaves, out)
            with kernels.forced_expand_depth(D):
                res["D%d" % D] = round(B.ev_time(step, 10) * 1e3, 4)
        aes = q * 3 * leaves
        print(json.dumps({"mode": "batched", "keys": q, "leaves_per_key": leaves, "ms": res,
                          "best_lds_frac": aes * 160 / (min(res.values()) / 1e3) / B.LDS_PEAK_LOOKUPS}),
              flush=True)
