"""c1 (2^19 tree leaves, uint64) through KExpandCoop with E = 0 (512 blocks,
two per CU) against E = 1 (256 blocks, one per CU, the production choice),
alternated, event-timed like tools/bench_configs.py; the two outputs must be
byte-identical.  GPU box:  python tools/c1_coop_ab.py [rounds]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_configs as B  # noqa: E402
from distributed_point_functions_amd import kernels  # noqa: E402
from distributed_point_functions_amd import value_types as V  # noqa: E402
from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dpf = DistributedPointFunction.create(DpfParameters(20, V.Integer(64)))
    k0 = dpf.generate_keys(777777, 123456789123, seeds=(0x51, 0x52))[0]
    desc = dpf.value_type_descriptor(0)
    ka = B.key_dev(dpf, k0, 0, dev)
    L = ka["L"]
    cepb = 1 << (20 - L)
    outs = {d: torch.empty((1 << 20) * 8, dtype=torch.uint8, device=dev) for d in (-1, -2)}

    def step(d):
        kernels.expand_and_correct(ka["seed"], ka["cb"], L, ka["cw"], ka["ccl"], ka["ccr"],
                                   desc, ka["corr"], ka["party"], cepb, 0, 1 << L, outs[d])
    res = {-1: [], -2: []}
    for _ in range(rounds):
        for d in (-2, -1):
            with kernels.forced_expand_depth(d):
                res[d].append(round(B.ev_time(lambda: step(d), 40) * 1e6, 2))
    torch.cuda.synchronize()
    same = bool(torch.equal(outs[-1], outs[-2]))
    print(json.dumps({"c1_us_E1_256_blocks": res[-2], "c1_us_E0_512_blocks": res[-1],
                      "identical": same}), flush=True)


if __name__ == "__main__":
    main()
