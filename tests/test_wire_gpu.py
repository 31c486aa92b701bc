"""Wire-format parity on the paths that need the device: a PirRequest
serialized by google.protobuf (tests/golden/wire/wire.json) answered by the
native DenseDpfPirServer (wire decode, DPF selection expansion, scan,
PirResponse encode), and EvaluationContexts carrying partial evaluations
after EvaluateNext, re-serialized by protobuf byte for byte and matching the
oracle's partial evaluations (distributed_point_function.cc:478-521).
"""
import ast
import json
import os

import numpy as np
import pytest

from oracle import pyoracle as po
from tests import wire_schema as W

pytestmark = pytest.mark.gpu

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "wire")


@pytest.fixture(scope="module")
def fx():
    with open(os.path.join(HERE, "wire.json")) as f:
        return json.load(f)


def test_pir_server_answers_protobuf_request(cuda, fx):
    """A PirRequest built and serialized by google.protobuf (PlainRequest with
    both parties' keys for one index) answered by the native server; the
    response is canonical protobuf and its two masked responses XOR to the
    record."""
    from distributed_point_functions_amd import pir as P
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    n, idx = 3000, 2077
    records = np.random.default_rng(11).integers(0, 256, (n, 40), dtype=np.uint8)
    db = P.DenseDpfPirDatabase()
    db.insert_fixed(records)
    server = P.DenseDpfPirServer.create_plain(n, db)
    dpf = DistributedPointFunction.create(DpfParameters((n - 1).bit_length(), V.XorWrapper(128)))
    (k0, k1), = P.client_keys(dpf, n, [idx], seeds=[(5, 6)])
    req = W.cls("PirRequest")()
    for k in (k0, k1):
        req.dpf_pir_request.plain_request.dpf_key.add().ParseFromString(bytes(k))
    data = req.SerializeToString(deterministic=True)
    assert data.hex() != fx["pir"]["plain_request"]
    assert data == P.pir_request_plain([k0, k1])
    resp = server.handle_request(data)
    assert W.canonical("PirResponse", resp) == resp
    m = W.cls("PirResponse").FromString(resp)
    r0, r1 = m.dpf_pir_response.masked_response
    assert bytes(a ^ b for a, b in zip(r0, r1)) == records[idx].tobytes()


@pytest.mark.parametrize("name", ["incremental_u32", "incremental_mixed"])
def test_context_with_partial_evaluations_is_canonical_and_matches_oracle(cuda, fx, name):
    from distributed_point_functions_amd import dpf as D
    from distributed_point_functions_amd import value_types as V
    case = next(c for c in fx["keys"] if c["name"] == name)

    def spec(s):
        return ("tuple", [spec(c) for c in s[1]]) if s[0] == "tuple" else tuple(s)
    levels = [(ld, spec(s), sec) for ld, s, sec in case["levels"]]
    dpf = D.DistributedPointFunction.create_incremental(
        [D.DpfParameters(ld, V.from_spec(s), sec) for ld, s, sec in levels])
    ctx = dpf.parse_evaluation_context(bytes.fromhex(case["ctx0"]))
    od = po.Dpf(levels)
    seeds = tuple(int(s) for s in case["seeds"])
    ok0, _ = od.generate_keys(int(case["alpha"]), ast.literal_eval(case["betas_str"]),
                              seeds=seeds)
    octx = od.create_evaluation_context(ok0)
    prefixes = []
    for h in range(len(levels) - 1):
        dpf.evaluate_next(prefixes, ctx, raw=True)
        od.evaluate_until(h, prefixes, octx)
        data = ctx.serialize()
        assert W.canonical("EvaluationContext", data) == data
        m = W.cls("EvaluationContext").FromString(data)
        assert m.previous_hierarchy_level == h
        if prefixes:
            got = sorted(((e.prefix.high << 64) | e.prefix.low, (e.seed.high << 64) | e.seed.low,
                          e.control_bit) for e in m.partial_evaluations)
            want = sorted((a, b, bool(c)) for a, b, c in octx.partial_evaluations())
            assert got == want
            assert m.partial_evaluations_level == octx.partial_evaluations_level
        ld = levels[h][0]
        alpha_prefix = int(case["alpha"]) >> (levels[-1][0] - ld)
        prefixes = sorted({alpha_prefix, 0, (1 << ld) - 1})
