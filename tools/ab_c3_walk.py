"""c3 (heavy hitters, 16 levels x 2^16 prefixes) with the per-level prefix
walk on four lanes per seed (walk mode 0, automatic: the DPF-key EvaluateSeeds
of <= 2^16 seeds runs KEvaluatePointsQuad without the value hash) against one
lane per seed (walk mode 2, KEvaluateSeeds), alternated; device outputs and
host outputs, both checked by the share sums of tools/bench_configs.py.
GPU box:  python tools/ab_c3_walk.py [rounds]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_configs as B  # noqa: E402
from distributed_point_functions_amd import kernels  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for _ in range(rounds):
        for mode in (0, 2):
            with kernels.forced_walk_mode(mode):
                r = B.c3(dev, 8)
            print(json.dumps({"walk_mode": mode, "device_out_ms_total": round(r["device_out_ms_total"], 3),
                              "host_out_ms_total": round(r["host_out_ms_total"], 3),
                              "correct": r["correct"]}), flush=True)


if __name__ == "__main__":
    main()
