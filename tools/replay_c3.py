"""Replays a c3 case dumped by tools/cpp_api_bench (DPF_AMD_BENCH_DUMP=file)
through the Python mirror and the CPU oracle, level by level: reports the
share-sum check and the first positions where a party's outputs differ from
the oracle.  Debugging aid for the Tier-2 incremental path."""
import struct
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))))

from distributed_point_functions_amd import value_types as V  # noqa: E402
from distributed_point_functions_amd.dpf import (  # noqa: E402
    DistributedPointFunction, DpfKey, DpfParameters, decode_value)
from oracle import pyoracle as po  # noqa: E402

H = 16


def main(path, levels=H):
    data = open(path, "rb").read()
    off = 0
    keys = []
    for _ in range(2):
        n = struct.unpack_from("<Q", data, off)[0]
        off += 8
        keys.append(DpfKey(data[off:off + n]))
        off += n
    lo, hi = struct.unpack_from("<QQ", data, off)
    off += 16
    alpha = lo | (hi << 64)
    betas, prefixes = [], []
    for _ in range(H):
        b, n = struct.unpack_from("<QQ", data, off)
        off += 16
        betas.append(b)
        prefixes.append(np.frombuffer(data, np.uint64, 2 * n, off).reshape(-1, 2).copy()
                        if n else [])
        off += 16 * n
    spec = ("int", 64)
    dpf = DistributedPointFunction.create_incremental(
        [DpfParameters(8 * (i + 1), V.Integer(64)) for i in range(H)])
    od = po.Dpf([(8 * (i + 1), spec, 0) for i in range(H)])
    okeys = []
    for k in keys:
        vcs = [[decode_value(V.Integer(64), v)[0] for v in
                (k.correction_words[dpf.hierarchy_to_tree(h)].value_correction
                 if h < H - 1 else k.last_level_value_correction)] for h in range(H)]
        okeys.append(po.Key.from_parts(k.seed, k.party, [c.seed for c in k.correction_words],
                                       [int(c.control_left) for c in k.correction_words],
                                       [int(c.control_right) for c in k.correction_words],
                                       vcs))
    ctxs = [dpf.create_evaluation_context(k) for k in keys]
    octxs = [od.create_evaluation_context(k) for k in okeys]
    for i in range(levels):
        pre = prefixes[i]
        plist = [int(a) | (int(b) << 64) for a, b in pre] if len(pre) else []
        outs = []
        for p in range(2):
            got = dpf.evaluate_next(pre, ctxs[p], raw=True).view(np.uint64)
            want = od.evaluate_until_words(i, plist, octxs[p])[:, 0, 0]
            bad = np.nonzero(got != want)[0]
            print("level %d party %d: %d outputs, %d differ from the oracle%s" % (
                i, p, len(got), len(bad), (" first at %s" % bad[:5].tolist()) if len(bad) else ""))
            outs.append(got)
        s = outs[0] + outs[1]
        nz = np.nonzero(s)[0]
        print("level %d: %d non-zero share sums, value ok %s" % (
            i, len(nz), bool(len(nz) == 1 and int(s[nz[0]]) == betas[i])), flush=True)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else H)
