"""Point-walk kernel choice across launch sizes (round 5): one key's points
(log_domain 128, uint128) through the Tier-1 batched entry point with the
walk forced to four lanes per point (mode 1, KEvaluatePointsQuad) or one
lane per point (mode 2, KEvaluatePoints), event-timed back to back and
alternated, outputs compared.  GPU box:  python tools/walk_sweep.py
"""
import json
import os
import random
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_configs as B  # noqa: E402
from distributed_point_functions_amd import kernels  # noqa: E402
from distributed_point_functions_amd import value_types as V  # noqa: E402
from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dpf = DistributedPointFunction.create(DpfParameters(128, V.Integer(128)))
    desc = dpf.value_type_descriptor(0)
    k0 = dpf.generate_keys(12345, 678, seeds=(1, 2))[0]
    kd = B.key_dev(dpf, k0, 0, dev)
    L = kd["L"]
    kcorr = kernels.u128_tensor(kd["corr"], dev)
    rng = random.Random(5)
    for lg in (14, 15, 16, 17, 18):
        n = 1 << lg
        pts = kernels.u128_tensor([rng.getrandbits(128) for _ in range(n)], dev)
        outs = {m: torch.empty(n * 16, dtype=torch.uint8, device=dev) for m in (1, 2)}
        res = {1: [], 2: []}
        for _ in range(3):
            for mode in (1, 2):
                def step():
                    kernels.evaluate_points_batched(1, n, kd["seed"], kd["cb"], pts, 0, L,
                                                    kd["cw"], kd["ccl"], kd["ccr"], desc,
                                                    party_all=kd["party"],
                                                    key_value_corrections=kcorr,
                                                    out=outs[mode])
                with kernels.forced_walk_mode(mode):
                    res[mode].append(round(B.ev_time(step, 10) * 1e6, 1))
        torch.cuda.synchronize()
        print(json.dumps({"points": n, "quad_us": res[1], "lane_us": res[2],
                          "equal": bool(torch.equal(outs[1], outs[2]))}), flush=True)


if __name__ == "__main__":
    main()
