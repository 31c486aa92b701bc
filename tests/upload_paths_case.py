"""One process's run of the host-to-device paths (helper of
tests/test_upload_paths_gpu.py, started as a child so each run reads its own
DPF_AMD_UPLOAD / DPF_AMD_ZERO_COPY / DPF_AMD_HOST_WRITE): EvaluateAt of a
uint128 key at log domain 128 (one launch with points read in place and the
key part host-written), of a uint32 key at log domain 20 (several elements
per block: element indices staged with the points), a full-domain
EvaluateUntil and two incremental levels with prefixes (the copy-ring
uploads).  Prints one JSON line of sha256 digests of the outputs."""
import hashlib
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_point_functions_amd import value_types as V  # noqa: E402
from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters  # noqa: E402


def digest(a) -> str:
    return hashlib.sha256(a.tobytes()).hexdigest()[:24]


def main():
    rng = random.Random(11)
    out = {}
    d128 = DistributedPointFunction.create(DpfParameters(128, V.Integer(128)))
    k0, k1 = d128.generate_keys(rng.getrandbits(128), rng.getrandbits(128), seeds=(5, 6))
    pts = [rng.getrandbits(128) for _ in range(3000)]
    out["at128"] = [digest(d128.evaluate_at(k, 0, pts, raw=True)) for k in (k0, k1)]
    d20 = DistributedPointFunction.create(DpfParameters(20, V.Integer(32)))
    j0, j1 = d20.generate_keys(rng.getrandbits(20), 123456, seeds=(7, 8))
    p20 = [rng.getrandbits(20) for _ in range(5000)]
    out["at20"] = [digest(d20.evaluate_at(k, 0, p20, raw=True)) for k in (j0, j1)]
    out["until20"] = digest(d20.evaluate_next([], d20.create_evaluation_context(j0), raw=True))
    inc = DistributedPointFunction.create_incremental(
        [DpfParameters(8, V.Integer(64)), DpfParameters(16, V.Integer(64))])
    a0, _ = inc.generate_keys_incremental(rng.getrandbits(16), [3, 4], seeds=(9, 10))
    ctx = inc.create_evaluation_context(a0)
    l0 = inc.evaluate_next([], ctx, raw=True)
    l1 = inc.evaluate_next(sorted(rng.sample(range(256), 40)), ctx, raw=True)
    out["incremental"] = [digest(l0), digest(l1)]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
