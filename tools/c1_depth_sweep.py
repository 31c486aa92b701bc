"""c1 (2^20 uint64 leaves = 2^19 tree leaves) expansion time per forced DFS
depth D (dpf_amd_set_expand_depth): how the automatic choice compares."""
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
for ld in [int(x) for x in (sys.argv[1:] or ["20", "24"])]:
    dpf = DistributedPointFunction.create(DpfParameters(ld, V.Integer(64)))
    k0, _ = dpf.generate_keys(12345, 678, seeds=(1, 2))
    kd = B.key_dev(dpf, k0, 0, dev)
    desc = dpf.value_type_descriptor(0)
    L = kd["L"]
    cepb = 1 << (ld - L)
    out = torch.empty((1 << L) * cepb * 8, dtype=torch.uint8, device=dev)
    res = {}
    for D in ((0, 1, 2, 4, 8) if ld <= 24 else (4, 8)):
        def step():
            kernels.expand_and_correct(kd["seed"], kd["cb"], L, kd["cw"], kd["ccl"], kd["ccr"],
                                       desc, kd["corr"], kd["party"], cepb, 0, 1 << L, out)
        with kernels.forced_expand_depth(D):
            res["D%d" % D] = round(B.ev_time(step, 20) * 1e3, 4)
    print({"log_domain": ld, "ms": res}, flush=True)
