"""Wire-format parity against an independent protobuf runtime
(google.protobuf with the reference's schema, tests/wire_schema.py) and the
fixtures it wrote (tests/golden/wire/make_wire.py):

  - DpfKey bytes from our GenerateKeys equal the protobuf serialization of
    the oracle's key for 17 value-type / hierarchy cases;
  - CreateEvaluationContext bytes equal the reference's fresh context
    (distributed_point_function.cc:712-727);
  - the reference's proto_validator_test.textproto context parses and
    re-serializes byte-identically, and the validator checks of
    dpf/internal/proto_validator_test.cc:189-284 give the reference's
    messages on mutations of it;
  - PIR / DCF / cuckoo messages built by our helpers equal protobuf's.
No GPU: key generation, contexts and validation are host code.
"""
import ast
import json
import os

import pytest

from tests import wire_schema as W

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "wire")


@pytest.fixture(scope="module")
def fx():
    with open(os.path.join(HERE, "wire.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def api():
    from distributed_point_functions_amd import _lib, dcf, dpf, pir, value_types
    return dpf, value_types, pir, dcf, _lib


def _spec(s):
    if s[0] == "tuple":
        return ("tuple", [_spec(c) for c in s[1]])
    return tuple(s)


def _dpf(api, levels):
    D, V = api[0], api[1]
    return D.DistributedPointFunction.create_incremental(
        [D.DpfParameters(ld, V.from_spec(_spec(s)), sec) for ld, s, sec in levels])


def _cases():
    with open(os.path.join(HERE, "wire.json")) as f:
        return [c["name"] for c in json.load(f)["keys"]]


@pytest.mark.parametrize("name", _cases())
def test_generate_keys_bytes_equal_protobuf_serialization_of_oracle_key(api, fx, name):
    case = next(c for c in fx["keys"] if c["name"] == name)
    dpf = _dpf(api, case["levels"])
    betas = ast.literal_eval(case["betas_str"])
    k0, k1 = dpf.generate_keys_incremental(int(case["alpha"]), betas,
                                           seeds=[int(s) for s in case["seeds"]])
    assert bytes(k0).hex() == case["key0"]
    assert bytes(k1).hex() == case["key1"]
    ctx = dpf.create_evaluation_context(k0)
    assert ctx.serialize().hex() == case["ctx0"]
    # our parser accepts protobuf's bytes and writes them back unchanged
    again = dpf.parse_evaluation_context(bytes.fromhex(case["ctx0"]))
    assert again.serialize().hex() == case["ctx0"]
    assert again.previous_hierarchy_level == -1


# ----------------------------------------------- proto_validator_test fixture
def _validator_ctx():
    with open(os.path.join(HERE, "proto_validator_ctx.binpb"), "rb") as f:
        data = f.read()
    return data, W.cls("EvaluationContext").FromString(data)


def _validator_dpf(api, ctx):
    D, V = api[0], api[1]
    params = [D.DpfParameters(p.log_domain_size, V.Integer(p.value_type.integer.bitsize),
                              p.security_parameter) for p in ctx.parameters]
    return D.DistributedPointFunction.create_incremental(params)


def test_proto_validator_context_round_trips(api):
    data, msg = _validator_ctx()
    assert msg.previous_hierarchy_level == -1 and len(msg.key.correction_words) == 6
    dpf = _validator_dpf(api, msg)
    ctx = dpf.parse_evaluation_context(data)
    assert ctx.serialize() == data
    assert ctx.previous_hierarchy_level == -1
    # the key alone validates (CreateEvaluationContext) and rebuilds the same context
    assert dpf.create_evaluation_context(api[0].DpfKey(msg.key.SerializeToString())
                                         ).serialize() == data


def _raises(api, fn, code, message, prefix=False):
    with pytest.raises(api[4].DpfAmdError) as e:
        fn()
    assert e.value.code == code
    got = str(e.value.message if hasattr(e.value, "message") else e.value)
    assert got.startswith(message) if prefix else message in got, got


@pytest.mark.parametrize("mutation,message,prefix", [
    ("clear_seed", "key.seed must be present", False),
    ("clear_last", "key.last_level_value_correction must be present", False),
    ("clear_value_corrections", "Malformed DpfKey: expected correction_words", True),
])
def test_validate_dpf_key_messages(api, mutation, message, prefix):
    """proto_validator_test.cc:189-215 through CreateEvaluationContext."""
    _, msg = _validator_ctx()
    dpf = _validator_dpf(api, msg)
    key = msg.key
    if mutation == "clear_seed":
        key.ClearField("seed")
    elif mutation == "clear_last":
        key.ClearField("last_level_value_correction")
    else:
        for cw in key.correction_words:
            cw.ClearField("value_correction")
    kb = api[0].DpfKey(key.SerializeToString())
    _raises(api, lambda: dpf.create_evaluation_context(kb), 3, message, prefix)


@pytest.mark.parametrize("mutation,message", [
    ("clear_key", "ctx.key must be present"),
    ("drop_parameter", "Number of parameters in `ctx` doesn't match"),
    ("log_domain_plus_one", "Parameter 0 in `ctx` doesn't match"),
    ("security_plus_one", "Parameter 0 in `ctx` doesn't match"),
    ("fully_evaluated", "This context has already been fully evaluated"),
    ("partial_level_too_large", "ctx.partial_evaluations_level must be less than or equal to "
                                "ctx.previous_hierarchy_level"),
])
def test_validate_evaluation_context_messages(api, mutation, message):
    """proto_validator_test.cc:217-285 through EvaluateNext (validation
    precedes any device work)."""
    _, msg = _validator_ctx()
    dpf = _validator_dpf(api, msg)
    if mutation == "clear_key":
        msg.ClearField("key")
    elif mutation == "drop_parameter":
        del msg.parameters[-1]
    elif mutation == "log_domain_plus_one":
        msg.parameters[0].log_domain_size += 1
    elif mutation == "security_plus_one":
        msg.parameters[0].security_parameter += 1
    elif mutation == "fully_evaluated":
        msg.previous_hierarchy_level = len(msg.parameters) - 1
    else:
        msg.previous_hierarchy_level = 0
        msg.partial_evaluations_level = 1
        msg.partial_evaluations.add()
    ctx = dpf.parse_evaluation_context(msg.SerializeToString())
    _raises(api, lambda: dpf.evaluate_until(1, [0], ctx), 3, message)


def test_validate_evaluation_context_default_security_parameter(api):
    """proto_validator_test.cc:244-253: security_parameter 0 on both sides."""
    D, V = api[0], api[1]
    _, msg = _validator_ctx()
    msg.parameters[0].security_parameter = 0
    params = [D.DpfParameters(p.log_domain_size, V.Integer(32), p.security_parameter)
              for p in msg.parameters]
    dpf = D.DistributedPointFunction.create_incremental(params)
    ctx = dpf.parse_evaluation_context(msg.SerializeToString())
    # passes validation: it then only fails for lack of a device, never with
    # a validation message
    try:
        dpf.evaluate_until(0, [], ctx, raw=True)
    except api[4].DpfAmdError as e:
        assert "doesn't match" not in str(e) and "must be" not in str(e), str(e)


# ------------------------------------------------------------ PIR / DCF / cuckoo
def test_pir_messages_equal_protobuf(api, fx):
    P = api[2]
    p = fx["pir"]
    keys = [bytes.fromhex(k) for k in p["keys"]]
    assert P.pir_request_plain(keys).hex() == p["plain_request"]
    assert P.helper_request(keys[1:], bytes.fromhex(p["helper_otp"])).hex() == p["helper_request"]
    assert P.pir_request_leader(keys[:1], bytes.fromhex(p["leader_encrypted"])).hex() == \
        p["leader_request"]
    assert P.pir_request_encrypted_helper(bytes.fromhex(p["encrypted_payload"])).hex() == \
        p["encrypted_helper_request"]
    assert [r.hex() for r in P.parse_response(bytes.fromhex(p["response"]))] == \
        p["response_records"]
    assert P.pir_config(p["dense_config_num_elements"]).hex() == p["dense_config"]


def test_dcf_key_wraps_dpf_key(api, fx):
    d = fx["dcf"]
    k = api[3].DcfKey(bytes.fromhex(d["dcf_key"]))
    assert bytes(k.key).hex() == d["dpf_key"]
    assert W.canonical("DcfKey", bytes(k)) == bytes(k)


def test_cuckoo_messages_equal_protobuf(api, fx):
    from distributed_point_functions_amd import cuckoo_pir as C
    c = fx["cuckoo"]
    seed = bytes.fromhex(c["seed"])
    assert C.cuckoo_hashing_params(seed, c["num_buckets"], c["num_hash_functions"]).hex() == \
        c["params"]
    assert C.cuckoo_pir_config(c["config_num_elements"]).hex() == c["config"]
    got = C.parse_cuckoo_hashing_params(bytes.fromhex(c["params"]))
    assert got == {"hash_family": 1, "seed": seed, "num_hash_functions": 3,
                   "num_buckets": c["num_buckets"]}
    # GenerateParams (native) output is canonical protobuf with a 16-byte seed
    params = C.generate_params(c["config_num_elements"])
    assert W.canonical("CuckooHashingParams", params) == params
    m = W.cls("CuckooHashingParams").FromString(params)
    assert m.num_hash_functions == 3 and m.num_buckets == int(1.5 * c["config_num_elements"])
    assert m.hash_family_config.hash_family == 1 and len(m.hash_family_config.seed) == 16
