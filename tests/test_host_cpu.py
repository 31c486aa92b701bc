"""Host logic of the product library on CPU (no kernel launches).

  - key generation (host AES) reproduces the oracle's golden keys bit-exactly
    and round-trips through the DpfKey wire format;
  - validation errors carry the reference's status codes and messages
    (dpf/distributed_point_function_test.cc:83-112, 160-190, 265-300,
    510-650);
  - value-type layout matches libstdc++ (tuple members reversed, naturally
    aligned) and the hierarchy/tree bookkeeping (proto_validator.cc:113-158);
  - without a GPU every evaluation entry point fails loudly (no CPU fallback).
"""
import json
import os

import pytest

from distributed_point_functions_amd import value_types as V
from distributed_point_functions_amd import wire
from distributed_point_functions_amd._lib import DpfAmdError
from distributed_point_functions_amd.dpf import (DistributedPointFunction, DpfKey, DpfParameters,
                                                 decode_value)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden.json")
P32 = 4294967291
P64 = 18446744073709551557


def _spec(s):
    if s[0] == "tuple":
        return ("tuple", [_spec(c) for c in s[1]])
    return tuple(s)


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def _key_fields(dpf, k: DpfKey, levels):
    return {"seed": k.seed, "party": k.party,
            "cw_seeds": [c.seed for c in k.correction_words],
            "ccl": [int(c.control_left) for c in k.correction_words],
            "ccr": [int(c.control_right) for c in k.correction_words],
            "value_corrections": _value_corrections(k, levels, dpf)}


def _value_corrections(k, levels, dpf):
    """Per hierarchy level, flattened value corrections (oracle order)."""
    out = []
    for h, (ld, spec, _) in enumerate(levels):
        vt = V.from_spec(spec)
        L = dpf.hierarchy_to_tree(h)
        if h == len(levels) - 1:
            vals = k.last_level_value_correction
        else:
            vals = k.correction_words[L].value_correction  # cc:131-148
        out.append([x for v in vals for x in decode_value(vt, v)])
    return out


def test_product_keygen_matches_golden_keys(golden):
    for case in golden["dpf"]:
        levels = [(ld, _spec(s), sec) for ld, s, sec in case["levels"]]
        params = [DpfParameters(ld, V.from_spec(s), sec) for ld, s, sec in levels]
        dpf = DistributedPointFunction.create_incremental(params)
        betas = [V.from_spec(l[1]).unflatten(iter(b)) for l, b in zip(levels, case["betas"])]
        k0, k1 = dpf.generate_keys_incremental(case["alpha"], betas, seeds=case["seeds"])
        for k, want in ((k0, case["key0"]), (k1, case["key1"])):
            got = _key_fields(dpf, k, levels)
            assert got["seed"] == want["seed"], case["name"]
            assert got["party"] == want["party"]
            assert got["cw_seeds"] == want["cw_seeds"], case["name"]
            assert got["ccl"] == want["ccl"] and got["ccr"] == want["ccr"], case["name"]
            assert got["value_corrections"] == want["value_corrections"], case["name"]
            # wire round trip
            assert DpfKey(bytes(k)) == k


def test_random_keygen_differs_and_shares_structure():
    dpf = DistributedPointFunction.create(DpfParameters(20, V.UINT64))
    a0, a1 = dpf.generate_keys(5, 7)
    b0, _ = dpf.generate_keys(5, 7)
    assert a0.seed != b0.seed  # CSPRNG seeds
    assert a0.party == 0 and a1.party == 1
    assert len(a0.correction_words) == dpf.hierarchy_to_tree(0)
    assert [c.seed for c in a0.correction_words] == [c.seed for c in a1.correction_words]


@pytest.mark.parametrize("ld,spec,tree", [
    (20, ("int", 64), 19), (20, ("int", 8), 16), (128, ("int", 128), 128),
    (26, ("xor", 128), 26), (32, ("tuple", [("int", 32), ("intmodn", 64, P64)]), 32),
    (0, ("int", 32), 0), (5, ("int", 32), 3)])
def test_tree_levels(ld, spec, tree):
    sec = 48 if "intmodn" in repr(spec) else 0.0
    dpf = DistributedPointFunction.create(DpfParameters(ld, V.from_spec(spec), sec))
    assert dpf.hierarchy_to_tree(0) == tree


def test_c5_value_layout_and_descriptor():
    vt = V.Tuple(V.Integer(32), V.IntModN(64, P64))
    assert vt.size == 16 and vt.scalar_offsets() == [8, 0]
    dpf = DistributedPointFunction.create(DpfParameters(32, vt, 48))
    d = dpf.value_type_descriptor(0)
    assert (d.num_scalars, d.blocks_needed, d.elements_per_block, d.out_stride) == (2, 2, 1, 16)
    assert (d.scalars[0].out_offset, d.scalars[1].out_offset) == (8, 0)
    assert d.scalars[1].modulus[0] == P64


def test_tuple_layout_reverse_order():
    vt = V.Tuple(V.Integer(8), V.Integer(16), V.Integer(32))
    assert vt.size == 8 and vt.scalar_offsets() == [6, 4, 0]
    vt = V.Tuple(V.Integer(64), V.Integer(8))
    assert vt.size == 16 and vt.scalar_offsets() == [8, 0]


# ----------------------------------------------------------- error messages
def _err(fn):
    with pytest.raises(DpfAmdError) as e:
        fn()
    return e.value


def test_create_fails_for_tuple_with_different_intmodn():
    e = _err(lambda: DistributedPointFunction.create(
        DpfParameters(10, V.Tuple(V.IntModN(32, 3), V.IntModN(64, 4)))))
    assert e.code == 12
    assert e.message == "All elements of type IntModN in a tuple must be the same"


def test_create_fails_for_invalid_value_type():
    class Empty(V.ValueType):
        def to_proto(self):
            return b""
    p = DpfParameters(10, Empty())
    e = _err(lambda: DistributedPointFunction.create(p))
    assert e.code == 3 and e.message.startswith("ValidateValueType: Unsupported ValueType")


def test_create_fails_for_bad_log_domain_order():
    e = _err(lambda: DistributedPointFunction.create_incremental(
        [DpfParameters(10, V.UINT64), DpfParameters(10, V.UINT64)]))
    assert e.code == 3
    assert e.message == "`log_domain_size` fields must be in ascending order in `parameters`"


def test_c5_default_security_parameter_rejected():
    # int_mod_n.cc:29-67: 40 + 32 bits of security need more than the 66 bits
    # a 64-bit modulus sample can provide.
    e = _err(lambda: DistributedPointFunction.create(
        DpfParameters(32, V.Tuple(V.Integer(32), V.IntModN(64, P64)))))
    assert e.code == 3


def test_generate_keys_errors():
    dpf = DistributedPointFunction.create(DpfParameters(10, V.UINT32))
    e = _err(lambda: dpf.generate_keys(1 << 10, 1))
    assert e.code == 3 and e.message == "`alpha` must be smaller than the output domain size"
    e = _err(lambda: dpf.generate_keys(0, 1 << 32))
    assert e.code == 3
    e = _err(lambda: dpf.generate_keys_incremental(0, [1, 2]))
    assert e.code == 3
    assert e.message == ("`beta` has to have the same size as `parameters` passed at "
                         "construction")


def test_evaluation_validation_errors_before_any_device_work():
    params = [DpfParameters(5, V.UINT128), DpfParameters(10, V.UINT128)]
    dpf = DistributedPointFunction.create_incremental(params)
    k0, _ = dpf.generate_keys_incremental(3, [1, 2], seeds=(11, 12))
    ctx = dpf.create_evaluation_context(k0)
    e = _err(lambda: dpf.evaluate_until(-1, [], ctx))
    assert e.message == "`hierarchy_level` must be non-negative and less than parameters_.size()"
    e = _err(lambda: dpf.evaluate_until(2, [], ctx))
    assert e.message == "`hierarchy_level` must be non-negative and less than parameters_.size()"
    e = _err(lambda: dpf.evaluate_until(0, [0], ctx))
    assert e.message == ("`prefixes` must be empty if and only if this is the first call with "
                         "`ctx`.")
    strange = V.Tuple(V.Integer(8), V.Integer(32), V.Integer(8), V.Integer(16), V.Integer(8))
    e = _err(lambda: dpf.evaluate_until(0, [], ctx, value_type=strange))
    assert e.message == "Value type T doesn't match parameters at `hierarchy_level`"


def test_output_size_too_large():
    params = [DpfParameters(10, V.UINT128), DpfParameters(100, V.UINT128)]
    dpf = DistributedPointFunction.create_incremental(params)
    k0, _ = dpf.generate_keys_incremental(123, [456, 789], seeds=(1, 2))
    ctx = dpf.create_evaluation_context(k0)
    e = _err(lambda: dpf.evaluate_until(1, [], ctx))
    assert e.message == ("Output size would be larger than 2**62. Please evaluate fewer "
                         "hierarchy levels at once.")


def test_context_serialize_parse_round_trip():
    params = [DpfParameters(5, V.UINT64), DpfParameters(12, V.UINT64)]
    dpf = DistributedPointFunction.create_incremental(params)
    k0, _ = dpf.generate_keys_incremental(17, [1, 2], seeds=(5, 6))
    ctx = dpf.create_evaluation_context(k0)
    data = ctx.serialize()
    ctx2 = dpf.parse_evaluation_context(data)
    assert ctx2.serialize() == data
    assert ctx2.previous_hierarchy_level == -1
    d = wire.decode(data)
    assert DpfKey(d[2][-1]) == k0  # EvaluationContext.key (proto:156-171)


def test_evaluation_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    dpf = DistributedPointFunction.create(DpfParameters(8, V.UINT64))
    k0, _ = dpf.generate_keys(3, 4, seeds=(1, 2))
    ctx = dpf.create_evaluation_context(k0)
    e = _err(lambda: dpf.evaluate_next([], ctx))
    assert e.code == 13  # INTERNAL: HIP error surfaced, no CPU fallback
    e = _err(lambda: dpf.evaluate_at(k0, 0, [1, 2]))
    assert e.code == 13


# --- RegisterValueType (dpf/distributed_point_function.cc:567-582, 620-633;
# distributed_point_function_test.cc:130-167) ------------------------------

TUPLE_U32_NOT_REGISTERED = (
    "No value correction function known for the following parameters:\n"
    "log_domain_size: 10\n"
    "value_type {\n"
    "  tuple {\n"
    "    elements {\n"
    "      integer {\n"
    "        bitsize: 32\n"
    "      }\n"
    "    }\n"
    "  }\n"
    "}\n"
    "security_parameter: 50\n"
    "Did you call RegisterValueType<T>() with your value type?")


def test_keygen_fails_if_value_type_not_registered():
    vt = V.Tuple(V.Integer(32))
    dpf = DistributedPointFunction.create(DpfParameters(10, vt))
    beta = vt.value_proto((42,))  # an explicit Value proto, as the reference test
    with pytest.raises(DpfAmdError) as e:
        dpf.generate_keys(23, beta)
    assert e.value.code == 9  # FAILED_PRECONDITION
    assert e.value.message.startswith("No value correction function known")
    assert e.value.message == TUPLE_U32_NOT_REGISTERED
    dpf.register_value_type(vt)
    k0, k1 = dpf.generate_keys(23, beta)
    assert k0.party == 0 and k1.party == 1


def test_templated_keygen_registers_the_type():
    """GenerateKeys with a typed value (ToValue<T>) registers T first."""
    for vt, beta in ((V.Tuple(V.Integer(32), V.IntModN(64, P64)), (7, 11)),
                     (V.XorWrapper(128), 1 << 77), (V.IntModN(32, P32), 5)):
        dpf = DistributedPointFunction.create(DpfParameters(12, vt, 48))
        dpf.generate_keys(99, beta)
        dpf.generate_keys(99, vt.value_proto(beta))  # now registered


@pytest.mark.parametrize("bits", [8, 16, 32, 64, 128])
def test_single_integers_are_registered_at_construction(bits):
    vt = V.Integer(bits)
    dpf = DistributedPointFunction.create(DpfParameters(9, vt))
    dpf.generate_keys(3, vt.value_proto(1))


def test_unregistered_level_of_an_incremental_dpf_is_reported():
    t = V.Tuple(V.Integer(16), V.Integer(16))
    dpf = DistributedPointFunction.create_incremental(
        [DpfParameters(4, V.Integer(64)), DpfParameters(8, t)])
    with pytest.raises(DpfAmdError) as e:
        dpf.generate_keys_incremental(5, [V.Integer(64).value_proto(1), t.value_proto((1, 2))])
    assert e.value.code == 9
    assert "log_domain_size: 8\n" in e.value.message


def test_dcf_value_proto_needs_registration():
    from distributed_point_functions_amd.dcf import DcfParameters, DistributedComparisonFunction
    vt = V.Tuple(V.Integer(32), V.Integer(32))
    d = DistributedComparisonFunction.create(DcfParameters(DpfParameters(8, vt)))
    with pytest.raises(DpfAmdError) as e:
        d.generate_keys(17, vt.value_proto((1, 2)))
    assert e.value.code == 9
    d.generate_keys(17, (1, 2))  # templated: registers
    d.generate_keys(17, vt.value_proto((1, 2)))


@pytest.mark.parametrize("spec", [("int", 8), ("int", 64), ("int", 128), ("xor", 128),
                                  ("intmodn", 64, 2 ** 64 - 59),
                                  ("tuple", [("int", 32), ("intmodn", 64, 2 ** 64 - 59)]),
                                  ("tuple", [("int", 16), ("tuple", [("int", 8), ("xor", 128)])])])
def test_decode_matches_elementwise_conversion(spec):
    """ValueType.decode / decode_flat (ndarray.tolist fast paths) equal the
    element-by-element conversion they replace, for plain, flat-tuple and
    nested-tuple types."""
    import numpy as np
    from distributed_point_functions_amd import value_types as V
    vt = V.from_spec(spec)
    raw = np.frombuffer(np.random.default_rng(3).bytes(257 * vt.numpy_dtype().itemsize),
                        dtype=vt.numpy_dtype())
    cols = []
    for i, s in enumerate(vt.scalars()):
        c = raw["f%d" % i]
        cols.append([int(lo) | (int(hi) << 64) for lo, hi in c] if s.bits == 128
                    else [int(x) for x in c])
    assert vt.decode(raw) == [vt.unflatten(iter(v)) for v in zip(*cols)]
    assert vt.decode_flat(raw) == [list(v) for v in zip(*cols)]


def test_u128_words_every_input_form():
    """128-bit packing: small ints, wide ints, mixed, negative (two's
    complement, as the reference's absl::uint128 conversion), numpy scalars,
    and (n, 2) uint64 arrays passed through."""
    import numpy as np
    from distributed_point_functions_amd.value_types import MASK64, u128_words

    def ref(values):
        return np.array([[int(v) & MASK64, (int(v) >> 64) & MASK64] for v in values],
                        dtype=np.uint64).reshape(-1)
    rng = np.random.default_rng(4)
    cases = [[int(x) for x in rng.integers(0, 2 ** 63, 100)],
             [int.from_bytes(rng.bytes(16), "little") for _ in range(100)],
             [5, 2 ** 100, 0, 2 ** 128 - 1], [2 ** 64, 1], [-1, 3], [np.uint64(9), 2 ** 70], [],
             [np.int64(-1)], [np.int64(-5), np.int64(7)], [np.int32(-2)], [2 ** 63, 1],
             [np.uint64(2 ** 64 - 1)], [True, 0]]
    for values in cases:
        assert np.array_equal(u128_words(values), ref(values)), values[:3]
    arr = np.array([[1, 2], [3, 4]], dtype=np.uint64)
    assert np.array_equal(u128_words(arr), arr.reshape(-1))


def test_bench_lds_roofline_of_the_many_query_scan():
    """bench.py's floor for the 64-query Four-Russians pass: 15 row stores
    at 128 B/clk + 64 row reads at 256 B/clk per KiB = 94 LDS cycles."""
    import bench
    r = bench.m4_lds_roofline(1 << 34, 64, 4.0)
    assert r["cycles_per_kib"] == 94
    assert abs(r["floor_ms"] - (1 << 24) * 94 / (256 * 2.4e9) * 1e3) < 1e-9
    assert abs(r["frac"] - r["floor_ms"] / 4.0) < 1e-12


def test_bench_launch_decision():
    """bench.py --gpus N: spawns its N ranks when nothing launched them, runs
    as one rank when WORLD_SIZE matches, refuses a mismatched world size or
    more RCCL ranks than GPUs; --in-process / --experiments stay one process."""
    import argparse
    import bench

    def a(gpus, **kw):
        return argparse.Namespace(gpus=gpus, in_process=kw.get("ip", False),
                                  experiments=kw.get("ex", False),
                                  library_multi_device=kw.get("lmd", False))
    assert bench.launch_decision(a(1), {}, 1) == ("run", None)
    assert bench.launch_decision(a(8), {}, 8) == ("spawn", 8)
    assert bench.launch_decision(a(8), {"WORLD_SIZE": "8"}, 8) == ("run", None)
    assert bench.launch_decision(a(1), {"WORLD_SIZE": "1"}, 8) == ("run", None)
    how, msg = bench.launch_decision(a(8), {"WORLD_SIZE": "1"}, 8)
    assert how == "error" and "WORLD_SIZE=1" in msg
    how, msg = bench.launch_decision(a(2), {}, 1)
    assert how == "error" and "DPF_AMD_BENCH_BACKEND=gloo" in msg
    assert bench.launch_decision(a(2), {"DPF_AMD_BENCH_BACKEND": "gloo"}, 1) == ("spawn", 2)
    assert bench.launch_decision(a(4, ip=True), {}, 1) == ("run", None)
    assert bench.launch_decision(a(4, ex=True), {}, 1) == ("run", None)
    assert bench.launch_decision(a(1, lmd=True), {}, 1) == ("run", None)


def test_bench_library_multi_device_child_command():
    """The child covers every rank's device in rank order and forces the
    peer-copy branches when ranks share a device (the one-GPU rehearsal)."""
    import argparse
    import bench
    args = argparse.Namespace(steps=3, warmup=1, log_domain=32, pir_log_records=26)
    cmd = bench.library_multi_device_cmd([(1, 1, "b"), (0, 0, "a")], args)
    assert "--library-multi-device" in cmd and "--force-peer" not in cmd
    assert cmd[cmd.index("--devices") + 1] == "0,1"
    cmd = bench.library_multi_device_cmd([(0, 0, "a"), (1, 0, "a")], args)
    assert cmd[cmd.index("--devices") + 1] == "0,0" and "--force-peer" in cmd


def test_bench_library_multi_device_failures_keep_the_line_complete():
    """Whatever the child does — fails without output, hangs past its limit,
    prints its result and then fails, or succeeds — the parent returns a dict
    the bench line can carry, with `correct` and the error when there is one;
    the rank-specific environment never reaches the child."""
    import json
    import sys
    import bench
    py = sys.executable
    r = bench.run_library_multi_device([py, "-c", "import sys; sys.stderr.write('boom'); sys.exit(3)"],
                                       60)
    assert r["correct"] is False and r["child_rc"] == 3 and "boom" in r["stderr_tail"]
    r = bench.run_library_multi_device([py, "-c", "import time; time.sleep(30)"], 1)
    assert r["correct"] is False and "limit" in r["error"]
    line = json.dumps({"library_multi_device": {"correct": True, "c5": {}}})
    r = bench.run_library_multi_device([py, "-c", "print('noise'); print(%r)" % line], 60)
    assert r["correct"] is True and r["child_rc"] == 0
    r = bench.run_library_multi_device(
        [py, "-c", "import sys; print(%r); sys.exit(1)" % line], 60)
    assert r["correct"] is False and "exit code 1" in r["error"]
    env_probe = "import os, json; print(json.dumps({'library_multi_device': " \
                "{'correct': 'RANK' not in os.environ and 'WORLD_SIZE' not in os.environ}}))"
    old = dict(os.environ)
    os.environ.update(RANK="0", WORLD_SIZE="2")
    try:
        r = bench.run_library_multi_device([py, "-c", env_probe], 60)
    finally:
        os.environ.clear()
        os.environ.update(old)
    assert r["correct"] is True
    r = bench.run_library_multi_device(["/nonexistent/python"], 60)
    assert r["correct"] is False and "could not start" in r["error"]
    json.dumps(r)


def test_bench_spawns_ranks_without_torchrun():
    """`bench.py --gpus 2` with no launcher starts torch.distributed.run as a
    child with 2 ranks (on CPU the ranks stop at their first device call, so
    only the launch and its exit status are checked)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DPF_AMD_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--steps", "1"], capture_output=True, text=True, env=env, timeout=300)
    assert "starting 2 rank processes" in p.stdout
    assert "--nproc-per-node=2" in p.stdout
    assert p.returncode != 0  # no GPU here: the ranks fail, and the parent says so


def test_evaluate_at_ctx_rejects_out_of_range_context_levels():
    """A parsed (untrusted) EvaluationContext whose stored levels do not index
    the hierarchy is INVALID_ARGUMENT before any host table lookup or device
    work (EvaluateAt h:356-378 with ctx; the levels are fields 3 and 5 of
    the proto, and a repeated scalar field's last value wins)."""
    dpf = DistributedPointFunction.create_incremental(
        [DpfParameters(5, V.UINT64), DpfParameters(10, V.UINT64)])
    k0, _ = dpf.generate_keys_incremental(3, [1, 2], seeds=(11, 12))
    data = dpf.create_evaluation_context(k0).serialize()
    for field, v, what in ((5, 99, "partial_evaluations_level"),
                           (5, -1, "partial_evaluations_level"),
                           (5, 2, "partial_evaluations_level"),
                           (3, 7, "previous_hierarchy_level"),
                           (3, -5, "previous_hierarchy_level")):
        ctx = dpf.parse_evaluation_context(data + wire.field_varint(field, v))
        e = _err(lambda: dpf.evaluate_at_ctx(1, [3], ctx))
        assert e.code == 3 and e.message == "ctx.%s out of range" % what, (field, v)
        e = _err(lambda: dpf.evaluate_at_ctx(1, [], ctx))  # before the empty-points return
        assert e.code == 3, (field, v)
    # a context of other parameters
    other = DistributedPointFunction.create_incremental(
        [DpfParameters(6, V.UINT64), DpfParameters(10, V.UINT64)])
    ctx = other.parse_evaluation_context(data)
    e = _err(lambda: other.evaluate_at_ctx(1, [3], ctx))
    assert e.code == 3
