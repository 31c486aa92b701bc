"""Generates tests/golden/golden.json from the pinned CPU oracle.

    python tests/golden/make_golden.py

The oracle (oracle/dpf_oracle.c) is pinned to the reference's own known
answers before anything is written (AES-MMO KAT, dpf/aes_128_fixed_key_hash_
test.cc:120-141; IntModN sampling KAT, dpf/int_mod_n_test.cc:162-193); the
script refuses to write fixtures if a pin fails. The fixtures are data only
(keys, inputs, expected outputs or their SHA-256 digests); they let the GPU
parity tests and the product keygen be checked without rebuilding the oracle.

Inputs follow the reference tests where they define them:
  * EvaluateSeeds inputs: dpf/internal/evaluate_prg_hwy_test.cc:60-93
  * value types: dpf/distributed_point_function_test.cc:984-1013
  * security_parameter 48 for the IntModN tuple types: same file :950
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

P32 = 4294967291           # 2**32 - 5
P64 = 18446744073709551557  # 2**64 - 59
KEY_LEFT = (0x5be037ccf6a03de5 << 64) | 0x935f08d0a5b6a2fd   # cc:55-60
KEY_RIGHT = (0xef94b6aedebb026c << 64) | 0xe2ea1fe0f66f4d0b
KEY_VALUE = (0x05a5d1588c5423e3 << 64) | 0x46a31101b21d1c98

# (name, spec, security_parameter or None for the default 40 + log_domain)
TYPES = [
    ("u8", ("int", 8), None),
    ("u16", ("int", 16), None),
    ("u32", ("int", 32), None),
    ("u64", ("int", 64), None),
    ("u128", ("int", 128), None),
    ("xor128", ("xor", 128), None),
    ("xor64", ("xor", 64), None),
    ("tuple_u32_u64", ("tuple", [("int", 32), ("int", 64)]), None),
    ("tuple_u64_u64", ("tuple", [("int", 64), ("int", 64)]), None),
    ("tuple_u8_u16_u32", ("tuple", [("int", 8), ("int", 16), ("int", 32)]), None),
    ("intmodn32", ("intmodn", 32, P32), 48),
    ("intmodn64", ("intmodn", 64, P64), 48),
    ("tuple_u32_intmodn64", ("tuple", [("int", 32), ("intmodn", 64, P64)]), 48),
    ("tuple_intmodn64_x2", ("tuple", [("intmodn", 64, P64), ("intmodn", 64, P64)]), 48),
]


def digest(elements):
    """SHA-256 of a list of flattened elements (lists of ints)."""
    return hashlib.sha256(json.dumps(elements, separators=(",", ":")).encode()).hexdigest()


def key_dict(k):
    return {"seed": k.seed, "party": k.party, "cw_seeds": k.cw_seeds(),
            "ccl": k.ccl(), "ccr": k.ccr(), "value_corrections": k.value_corrections()}


def random_value(spec, rng):
    if spec[0] == "tuple":
        return [random_value(s, rng) for s in spec[1]]
    if spec[0] in ("int", "xor"):
        return rng.getrandbits(spec[1])
    return rng.randrange(spec[2])


def pin(po):
    kat0 = po.aes_mmo(0, [(0x0123012301230123 << 64) | 0x0123012301230123,
                          (0x4567456745674567 << 64) | 0x4567456745674567])
    assert kat0 == [(0x73c2dc14812be4ef << 64) | 0xeac64d09c8adf8ed,
                    (0xb8f33653a53a8436 << 64) | 0xaedf39b62de91d95], "AES KAT"
    data = b"this is a length 32 test string."
    got = po.intmodn_sample(data, 4, P32, 5)
    r = int.from_bytes(data[:16], "little")
    want = []
    for i in range(5):
        want.append(r % P32)
        if i < 4:
            r = ((r // P32) << 32) | int.from_bytes(data[16 + 4 * i:20 + 4 * i], "little")
    assert got == want, "IntModN KAT"


def dpf_case(po, name, spec, sec, ld, rng, full):
    sec_v = sec if sec is not None else 40 + ld
    d = po.Dpf([(ld, spec, sec_v)])
    alpha = rng.getrandbits(ld) if ld else 0
    beta = random_value(spec, rng)
    seeds = (rng.getrandbits(128), rng.getrandbits(128))
    k0, k1 = d.generate_keys(alpha, [beta], seeds=seeds)
    case = {"name": "%s_ld%d" % (name, ld), "levels": [[ld, spec, sec_v]], "alpha": alpha,
            "betas": [po.flatten_value(spec, beta)], "seeds": list(seeds),
            "key0": key_dict(k0), "key1": key_dict(k1), "eval": []}
    outs = []
    for k in (k0, k1):
        outs.append(d.evaluate_until(0, [], d.create_evaluation_context(k)))
    case["eval"].append({
        "level": 0, "prefixes": [], "count": len(outs[0]),
        "digest0": digest(outs[0]), "digest1": digest(outs[1]),
        "values0": outs[0] if full else outs[0][:4],
        "at_alpha0": outs[0][alpha], "at_alpha1": outs[1][alpha]})
    pts = sorted({alpha} | {rng.getrandbits(ld) if ld else 0 for _ in range(6)})
    case["evaluate_at"] = {"level": 0, "points": pts,
                           "out0": d.evaluate_at(k0, 0, pts), "out1": d.evaluate_at(k1, 0, pts)}
    return case


def incremental_case(po, rng):
    spec = ("int", 64)
    lds = [3, 7, 12, 20]
    levels = [(ld, spec, 40 + ld) for ld in lds]
    d = po.Dpf(levels)
    alpha = rng.getrandbits(lds[-1])
    betas = [rng.getrandbits(64) for _ in lds]
    seeds = (rng.getrandbits(128), rng.getrandbits(128))
    k0, k1 = d.generate_keys(alpha, betas, seeds=seeds)
    case = {"name": "incremental_u64", "levels": [list(l) for l in levels], "alpha": alpha,
            "betas": [[b] for b in betas], "seeds": list(seeds),
            "key0": key_dict(k0), "key1": key_dict(k1), "eval": []}
    ctxs = [d.create_evaluation_context(k) for k in (k0, k1)]
    prefixes = []
    for h, ld in enumerate(lds):
        outs = [d.evaluate_until(h, prefixes, c) for c in ctxs]
        case["eval"].append({"level": h, "prefixes": list(prefixes), "count": len(outs[0]),
                             "digest0": digest(outs[0]), "digest1": digest(outs[1]),
                             "values0": outs[0][:4]})
        if h + 1 < len(lds):
            # next prefixes: outputs of this level (extensions of this level's
            # prefixes), always including alpha's prefix (sorted, distinct)
            if prefixes:
                delta = ld - lds[h - 1]
                expanded = [(p << delta) | j for p in prefixes for j in range(1 << delta)]
            else:
                expanded = list(range(1 << ld))
            a = alpha >> (lds[-1] - ld)
            prefixes = sorted({a} | set(rng.sample(expanded, min(5, len(expanded)))))
    return case


def evaluate_seeds_cases(po):
    out = []
    for n in (1, 101):
        for levels in (1, 64, 128):
            for per_seed in (False, True):
                seeds = [(i << 64) | (i + 1) for i in range(n)]
                paths = [((23 * i + 42) << 64) | (42 * i + 23) for i in range(n)]
                cbs = [1 if i % 7 == 0 else 0 for i in range(n)]
                ncw = levels * n if per_seed else levels
                cws = [((i + 1) << 64) | i for i in range(ncw)]
                ccl = [1 if i % 23 == 0 else 0 for i in range(ncw)]
                ccr = [1 if i % 42 != 0 else 0 for i in range(ncw)]
                s, c = po.evaluate_seeds(seeds, cbs, paths, 0, cws, ccl, ccr, KEY_LEFT,
                                         KEY_RIGHT, levels)
                out.append({"num_seeds": n, "num_levels": levels, "per_seed_cw": per_seed,
                            "digest": digest([s, c]), "first_seed": s[0],
                            "first_bit": c[0]})
    return out


def pir_case(po, rng):
    sizes = [0, 1, 3, 7, 16, 17, 31, 32, 63, 64, 80, 81] * 20
    records = [bytes(rng.getrandbits(8) for _ in range(s)) for s in sizes]
    nb = (len(records) + 127) // 128
    sels = [[rng.getrandbits(128) for _ in range(nb)] for _ in range(2)]
    outs = po.inner_product(records, sels)
    return {"records_hex": [r.hex() for r in records], "selections": sels,
            "out_hex": [o.hex() for o in outs]}


def main():
    from oracle import pyoracle as po
    po.build()
    pin(po)
    rng = random.Random(20261015)
    g = {"generator": "tests/golden/make_golden.py", "aes_mmo": {}, "dpf": []}
    blocks = [rng.getrandbits(128) for _ in range(16)]
    g["aes_mmo"] = {"blocks": blocks, "left": po.aes_mmo(KEY_LEFT, blocks),
                    "right": po.aes_mmo(KEY_RIGHT, blocks),
                    "value": po.aes_mmo(KEY_VALUE, blocks)}
    g["evaluate_seeds"] = evaluate_seeds_cases(po)
    for name, spec, sec in TYPES:
        for ld in (0, 5, 10):
            g["dpf"].append(dpf_case(po, name, spec, sec, ld, rng, full=(ld <= 5)))
    g["dpf"].append(dpf_case(po, "u64", ("int", 64), None, 20, rng, full=False))
    g["dpf"].append(incremental_case(po, rng))
    g["pir"] = pir_case(po, rng)
    path = os.path.join(HERE, "golden.json")
    with open(path, "w") as f:
        json.dump(g, f, separators=(",", ":"))
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
