"""HandleRequest timing probe in a Python (torch) process: c4 (2^26 x 256 B)
database built from resident rows, Q = 1 / 8 / 64 plain requests, per-request
wall time; run with DPF_AMD_TRACE_HOST=1 for the library's phase times and
under rocprofv3 --kernel-trace for the kernels.

    python tools/pir_hr_probe.py [--queries 1,8,64] [--reps 5] [--log-n 26]
        [--devices 0,0,0,0,0,0,0,0] [--force-peer]

--devices shards the rows over the listed devices (entries may repeat: N
shards' code on fewer GPUs); --force-peer takes the cross-device copy
branches between shards on one device.
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", default="1,8,64")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--log-n", type=int, default=26)
    ap.add_argument("--devices", default="")
    ap.add_argument("--force-peer", action="store_true")
    args = ap.parse_args()
    import torch
    from distributed_point_functions_amd import _lib
    from distributed_point_functions_amd import pir as P
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    n, rec = 1 << args.log_n, 256
    dev = torch.device("cuda", 0)
    rows = torch.randint(0, 256, (n * rec,), dtype=torch.uint8, device=dev)
    if args.force_peer:
        _lib.lib().dpf_amd_set_force_peer_copies(1)
    devs = [int(d) for d in args.devices.split(",")] if args.devices else None
    db = P.DenseDpfPirDatabase(devs)
    db.insert_fixed_device(rows, n, rec).build()
    server = P.DenseDpfPirServer.create_plain(n, db)
    dpf = DistributedPointFunction.create(DpfParameters((n - 1).bit_length(), V.XorWrapper(128)))
    rng = np.random.default_rng(5)
    for q in [int(x) for x in args.queries.split(",")]:
        idx = [int(i) for i in rng.integers(0, n, q)]
        pairs = P.client_keys(dpf, n, idx, seeds=[(3 + 2 * j, 4 + 2 * j) for j in range(q)])
        req = P.pir_request_plain([a for a, _ in pairs])
        server.handle_request(req)
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            server.handle_request(req)
            ts.append(1e3 * (time.perf_counter() - t0))
        print("Q=%d shards=%d best %.3f ms mean %.3f ms" % (q, len(devs or [0]), min(ts),
                                                          sum(ts) / len(ts)), flush=True)


if __name__ == "__main__":
    main()
