"""c3's expansion shape in isolation: n prefix roots (random seeds), 7 tree
levels below each, uint64 outputs (two per tree leaf), KExpand at the
automatic depth or a forced one; event-timed, with the LDS-lookup fraction
(490 lookups per tree leaf at D = 4: 3 walk + 30 tree + 16 value AES per 16
leaves, 160 each; likewise for a forced D).  Used to see whether the 2^16-root launch (2^19 threads,
1024 blocks = two rounds of 512 slots) loses to its tail.

    python tools/c3_expand_probe.py [--roots 15,16,17,18] [--depths 0,4]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_point_functions_amd import kernels as K  # noqa: E402
from distributed_point_functions_amd import value_types as V  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--roots", default="15,16,17,18")
    ap.add_argument("--depths", default="0,4")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    vt = V.Integer(64)
    desc = vt.descriptor(1)
    levels = 7
    gen = torch.Generator(device=dev)
    gen.manual_seed(3)
    cw = torch.randint(-2**63, 2**63 - 1, (levels, 2), dtype=torch.int64, device=dev, generator=gen)
    ccl = torch.randint(0, 2, (levels,), dtype=torch.uint8, device=dev, generator=gen)
    ccr = torch.randint(0, 2, (levels,), dtype=torch.uint8, device=dev, generator=gen)
    for lr in [int(x) for x in args.roots.split(",")]:
        n = 1 << lr
        seeds = torch.randint(-2**63, 2**63 - 1, (n, 2), dtype=torch.int64, device=dev, generator=gen)
        seeds[:, 0] &= ~1
        cbs = torch.randint(0, 2, (n,), dtype=torch.uint8, device=dev, generator=gen)
        out = torch.empty((n << levels) * 2 * 8, dtype=torch.uint8, device=dev)
        for d in [int(x) for x in args.depths.split(",")]:
            def run():
                K.expand_and_correct(seeds, cbs, levels, cw, ccl, ccr, desc, [5, 7], 0, 2, 0,
                                     n << levels, out)
            with K.forced_expand_depth(d):
                run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    run()
                e1.record()
                torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            leaves = n << levels
            D = d or 4  # the automatic depth of this shape
            # per 2^D tree leaves: (levels - D) walk + 2^(D+1) - 2 tree + 2^D value AES
            aes = ((levels - D) + (1 << (D + 1)) - 2 + (1 << D)) / (1 << D) if D > 0 else None
            lookups = leaves * 160 * aes if aes else None
            frac = lookups / (ms / 1e3) / (256 * 32 * 2.4e9) if lookups else None
            print("roots 2^%d depth %s: %.3f ms, %.2f ns per tree leaf%s" % (
                lr, d or "auto", ms, ms * 1e6 / leaves,
                ", LDS-lookup fraction %.3f" % frac if frac else ""), flush=True)
        del out, seeds, cbs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
