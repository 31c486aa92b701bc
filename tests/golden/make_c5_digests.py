"""Generates tests/golden/c5_subtree_digests.json: one SHA-256 per 2^20-leaf
subtree of BOTH parties' full 2^32-leaf expansion of the c5 test key, from
the pinned CPU oracle (oracle/dpf_oracle.c, the restatement of ExpandSeeds
cc:289-372 + HashExpandedSeeds cc:523-547 + the correction loop h:846-862).

    python tests/golden/make_c5_digests.py [--procs 8]

The key is the one tests/test_fullsize_gpu.py expands on the device
(`_keys(C5, 32, seed=5)` of tests/test_kernels_gpu.py, reproduced below from
its parameters, which the JSON records).  Each digest covers the 16 MiB of a
subtree in the host layout of Tuple<uint32_t, IntModN<uint64_t, 2^64-59>>
that the product writes (libstdc++ tuple order: IntModN u64 at byte 0, u32 at
byte 8, 4 zero padding bytes), so the device test hashes its output buffer
slices directly.  8192 digests pin every one of the 2 x 2^32 leaf values.
About a minute on the build container's 8 cores (24 M leaves/s/core).
"""
import argparse
import hashlib
import json
import multiprocessing as mp
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

P64 = 18446744073709551557  # 2**64 - 59
SPEC = ("tuple", [("int", 32), ("intmodn", 64, P64)])
LOG_DOMAIN = 32
LOG_SUBTREE = 20
SECURITY = 48
KEY_SEED = 5  # tests/test_kernels_gpu.py _keys(..., seed=5)
OUT = os.path.join(HERE, "c5_subtree_digests.json")


def key_params():
    """alpha, beta, keygen seeds of `_keys(C5, 32, seed=5)` (same RNG draws)."""
    rng = random.Random(KEY_SEED * 1000 + LOG_DOMAIN)
    beta = (rng.getrandbits(32), rng.randrange(P64))
    alpha = rng.randrange(1 << LOG_DOMAIN)
    seeds = (rng.getrandbits(128), rng.getrandbits(128))
    return alpha, beta, seeds


def host_layout_bytes(words):
    """Oracle words (n, 2 scalars, 2 u64) -> host-layout bytes of n elements."""
    import numpy as np
    n = words.shape[0]
    hl = np.zeros((n, 2), dtype=np.uint64)
    hl[:, 0] = words[:, 1, 0]  # IntModN<uint64_t> at offset 0
    hl[:, 1] = words[:, 0, 0]  # uint32_t at offset 8, zero padding above
    return hl.tobytes()


def _worker(job):
    party, first, last = job
    import numpy as np
    from oracle import pyoracle as po
    alpha, beta, seeds = key_params()
    d = po.Dpf([(LOG_DOMAIN, SPEC, SECURITY)])
    keys = d.generate_keys(alpha, [beta], seeds=seeds)
    key = keys[party]
    buf = np.zeros(2 * 2 * (1 << LOG_SUBTREE), dtype=np.uint64)
    out = []
    for s in range(first, last):
        d.expand_subtree_words(key, s << LOG_SUBTREE, LOG_SUBTREE, buf)
        words = buf.reshape(-1, 2, 2)
        out.append(hashlib.sha256(host_layout_bytes(words)).hexdigest())
    return party, first, out


def subtree_digest_jobs(nsub, procs):
    per = (nsub + 4 * procs - 1) // (4 * procs)
    return [(p, s, min(nsub, s + per)) for p in (0, 1) for s in range(0, nsub, per)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=os.cpu_count() or 8)
    args = ap.parse_args()
    from oracle import pyoracle as po
    po.build()
    nsub = 1 << (LOG_DOMAIN - LOG_SUBTREE)
    t0 = time.time()
    digests = {0: [None] * nsub, 1: [None] * nsub}
    with mp.get_context("spawn").Pool(args.procs) as pool:
        for party, first, out in pool.imap_unordered(_worker, subtree_digest_jobs(nsub, args.procs)):
            digests[party][first:first + len(out)] = out
    assert all(x is not None for p in (0, 1) for x in digests[p])
    alpha, beta, seeds = key_params()
    doc = {
        "what": "SHA-256 of each 2^20-leaf subtree (host layout, 16 B/leaf) of the full "
                "2^32-leaf EvaluateNext output of both parties of the c5 test key, "
                "from oracle/dpf_oracle.c",
        "generator": "tests/golden/make_c5_digests.py",
        "spec": "tuple<int32, intmodn<64, 2^64-59>>", "log_domain_size": LOG_DOMAIN,
        "security_parameter": SECURITY, "log_subtree_leaves": LOG_SUBTREE,
        "alpha": alpha, "beta": list(beta), "keygen_seeds": [str(s) for s in seeds],
        "host_layout": "u64 IntModN at byte 0, u32 at byte 8, bytes 12-15 zero",
        "sha256": {"0": digests[0], "1": digests[1]},
    }
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=0)
    print("wrote %s (%d digests) in %.1f s" % (OUT, 2 * nsub, time.time() - t0))


if __name__ == "__main__":
    main()
