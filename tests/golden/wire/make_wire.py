"""Generates tests/golden/wire/: protobuf wire-format fixtures, serialized by
the google.protobuf runtime (tests/wire_schema.py) rather than by our codecs.

  proto_validator_ctx.binpb  the EvaluationContext of the reference's
                             dpf/internal/proto_validator_test.textproto
                             (parsed with text_format, serialized here)
  wire.json                  per value-type case: the oracle's keys
                             (oracle/dpf_oracle.c, pinned by tests/golden)
                             as DpfKey bytes, the fresh EvaluationContext
                             the reference's CreateEvaluationContext builds
                             (distributed_point_function.cc:712-727), and
                             PIR / DCF / cuckoo messages built from them

Run from the repo root (needs /root/reference for the textproto):
    python tests/golden/wire/make_wire.py
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)

from google.protobuf import text_format  # noqa: E402

from oracle import pyoracle as po  # noqa: E402
from tests import wire_schema as W  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
TEXTPROTO = "/root/reference/dpf/internal/proto_validator_test.textproto"
M64 = (1 << 64) - 1
P64 = 2 ** 64 - 59

# name, levels [(log_domain_size, spec, security_parameter)], alpha, betas
CASES = [
    ("u8", [(10, ("int", 8), 0)], 513, [200]),
    ("u16", [(10, ("int", 16), 0)], 7, [65535]),
    ("u32", [(10, ("int", 32), 0)], 1023, [0xDEADBEEF]),
    ("u64", [(12, ("int", 64), 0)], 4000, [(1 << 64) - 3]),
    ("u128", [(12, ("int", 128), 0)], 1, [(1 << 127) + 12345]),
    ("u128_small_beta", [(9, ("int", 128), 0)], 0, [42]),
    ("xor128", [(11, ("xor", 128), 0)], 2047, [(0x0123456789ABCDEF << 64) | 0xFEDCBA9876543210]),
    ("xor64", [(11, ("xor", 64), 0)], 1000, [0xAAAA5555AAAA5555]),
    ("intmodn_u32", [(10, ("intmodn", 32, 4294967291), 0)], 3, [4294967290]),
    ("intmodn_u64", [(10, ("intmodn", 64, P64), 48.5)], 999, [P64 - 1]),
    ("tuple_u32_intmodn_u64", [(14, ("tuple", [("int", 32), ("intmodn", 64, P64)]), 54)],
     12345, [(7, 11)]),
    ("tuple_u32_u32", [(10, ("tuple", [("int", 32), ("int", 32)]), 0)], 5, [(1, 2)]),
    ("tuple_nested", [(10, ("tuple", [("int", 64), ("tuple", [("int", 8), ("xor", 64)])]), 0)],
     600, [(1 << 63, (255, 0x1234))]),
    ("incremental_u32", [(4, ("int", 32), 44), (6, ("int", 32), 46), (8, ("int", 32), 48)],
     0xA5, [1, 2, 3]),
    ("incremental_mixed", [(8, ("int", 64), 0), (16, ("int", 128), 0), (32, ("xor", 128), 0)],
     0xC0FFEE11, [10, 1 << 100, 77]),
    ("domain_0", [(0, ("int", 64), 0)], 0, [99]),
    ("domain_128", [(128, ("int", 64), 0)], (1 << 128) - 1, [5]),
]


def set_block(msg, v):
    msg.SetInParent()
    msg.high = v >> 64
    msg.low = v & M64


def key_message(od, levels, ok):
    """DpfKey of an oracle key, laid out as the reference's GenerateKeys
    writes it (value corrections in correction_words[hierarchy_to_tree[h]],
    the last level's in last_level_value_correction)."""
    m = W.cls("DpfKey")()
    set_block(m.seed, ok.seed)
    for s, cl, cr in zip(ok.cw_seeds(), ok.ccl(), ok.ccr()):
        cw = m.correction_words.add()
        set_block(cw.seed, s)
        cw.control_left = bool(cl)
        cw.control_right = bool(cr)
    vcs = ok.value_corrections()
    H = len(levels)
    for h, (_, spec, _) in enumerate(levels):
        ns = po.num_scalars(spec)
        target = (m.last_level_value_correction if h == H - 1
                  else m.correction_words[od.hierarchy_to_tree(h)].value_correction)
        for e in range(len(vcs[h]) // ns):
            W.value(target.add(), spec, list(vcs[h][e * ns:(e + 1) * ns]))
    m.party = ok.party
    return m


def parameters_message(msg, ld, spec, sec):
    msg.log_domain_size = ld
    W.value_type(msg.value_type, spec)
    msg.security_parameter = sec


def context_message(levels, key_msg):
    """CreateEvaluationContext: the validator's parameters (security
    parameter defaulted to 40 + log_domain_size, proto_validator.cc:117-125),
    the key, previous_hierarchy_level = -1."""
    c = W.cls("EvaluationContext")()
    for ld, spec, sec in levels:
        parameters_message(c.parameters.add(), ld, spec, sec if sec else 40 + ld)
    c.key.CopyFrom(key_msg)
    c.previous_hierarchy_level = -1
    return c


def ser(m):
    return m.SerializeToString(deterministic=True)


def main():
    ctx = W.cls("EvaluationContext")()
    with open(TEXTPROTO) as f:
        text_format.Parse(f.read(), ctx)
    with open(os.path.join(HERE, "proto_validator_ctx.binpb"), "wb") as f:
        f.write(ser(ctx))

    out = {"keys": [], "pir": {}, "dcf": {}, "cuckoo": {}}
    for i, (name, levels, alpha, betas) in enumerate(CASES):
        od = po.Dpf(levels)
        seeds = (0x1111 * (i + 1), (0x2222 * (i + 1)) << 64 | 0x33)
        ok0, ok1 = od.generate_keys(alpha, betas, seeds=seeds)
        k0, k1 = key_message(od, levels, ok0), key_message(od, levels, ok1)
        out["keys"].append({
            "name": name, "levels": [[ld, spec, sec] for ld, spec, sec in levels],
            "alpha": str(alpha), "betas": json.loads(json.dumps(betas, default=str)),
            "betas_str": repr(betas), "seeds": [str(s) for s in seeds],
            "key0": ser(k0).hex(), "key1": ser(k1).hex(),
            "ctx0": ser(context_message(levels, k0)).hex()})

    # PIR messages (pir/private_information_retrieval.proto) over the xor128 keys
    xk = next(k for k in out["keys"] if k["name"] == "xor128")
    keys0 = [bytes.fromhex(xk["key0"]), bytes.fromhex(xk["key1"])]
    D = W.cls("DpfKey")
    Req = W.cls("PirRequest")
    plain = Req()
    for kb in keys0:
        plain.dpf_pir_request.plain_request.dpf_key.add().CopyFrom(D.FromString(kb))
    helper = W.cls("DpfPirRequest.HelperRequest")()
    helper.plain_request.dpf_key.add().CopyFrom(D.FromString(keys0[1]))
    helper.one_time_pad_seed = bytes(range(16))
    leader = Req()
    leader.dpf_pir_request.leader_request.plain_request.dpf_key.add().CopyFrom(
        D.FromString(keys0[0]))
    leader.dpf_pir_request.leader_request.encrypted_helper_request.encrypted_request = \
        b"\x01ciphertext\x00\xff"
    enc = Req()
    enc.dpf_pir_request.encrypted_helper_request.encrypted_request = b"\x02opaque"
    resp = W.cls("PirResponse")()
    for r in (b"", b"\x00" * 16, bytes(range(40))):
        resp.dpf_pir_response.masked_response.append(r)
    cfg = W.cls("PirConfig")()
    cfg.dense_dpf_pir_config.num_elements = 1 << 20
    out["pir"] = {"keys": [k.hex() for k in keys0],
                  "plain_request": ser(plain).hex(), "helper_request": ser(helper).hex(),
                  "helper_otp": bytes(range(16)).hex(),
                  "leader_request": ser(leader).hex(),
                  "leader_encrypted": b"\x01ciphertext\x00\xff".hex(),
                  "encrypted_helper_request": ser(enc).hex(),
                  "encrypted_payload": b"\x02opaque".hex(),
                  "response": ser(resp).hex(),
                  "response_records": ["", "00" * 16, bytes(range(40)).hex()],
                  "dense_config_num_elements": 1 << 20, "dense_config": ser(cfg).hex()}
    # DCF key wraps a DpfKey (dcf/distributed_comparison_function.proto:30-32)
    dk = W.cls("DcfKey")()
    dk.key.CopyFrom(D.FromString(bytes.fromhex(out["keys"][3]["key0"])))
    out["dcf"] = {"dpf_key": out["keys"][3]["key0"], "dcf_key": ser(dk).hex()}
    # cuckoo hashing params (private_information_retrieval.proto:93-100)
    cp = W.cls("CuckooHashingParams")()
    cp.hash_family_config.hash_family = 1
    cp.hash_family_config.seed = bytes(range(16))
    cp.num_hash_functions = 3
    cp.num_buckets = 1572864
    cc = W.cls("PirConfig")()
    cc.cuckoo_hashing_sparse_dpf_pir_config.hash_family = 1
    cc.cuckoo_hashing_sparse_dpf_pir_config.num_elements = 1 << 20
    out["cuckoo"] = {"seed": bytes(range(16)).hex(), "num_hash_functions": 3,
                     "num_buckets": 1572864, "params": ser(cp).hex(),
                     "config_num_elements": 1 << 20, "config": ser(cc).hex()}
    with open(os.path.join(HERE, "wire.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", len(out["keys"]), "key cases")


if __name__ == "__main__":
    main()
