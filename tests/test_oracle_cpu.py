"""The CPU oracle against the reference's own known answers and the committed
golden fixtures (CPU only; no GPU, no product code).

Known answers (reference tests):
  - AES-MMO: dpf/aes_128_fixed_key_hash_test.cc:120-141 (AES-NI and portable)
  - IntModN sampling: dpf/int_mod_n_test.cc:162-193 (+ GetNumBytesRequired)
  - Tuple FromBytes: dpf/internal/value_type_helpers_test.cc:230-255
Properties (distributed_point_function_test.cc:652-1142): share-sum of the two
parties is beta at alpha and zero elsewhere.
"""
import json
import os

import pytest

from oracle import pyoracle as po
from tests.golden.make_golden import KEY_LEFT, KEY_RIGHT, KEY_VALUE, P32, digest, key_dict

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden.json")
SEED0 = (0x0123012301230123 << 64) | 0x0123012301230123
SEED1 = (0x4567456745674567 << 64) | 0x4567456745674567
KEY1 = (0x1111111111111111 << 64) | 0x1111111111111111
KAT0 = [(0x73c2dc14812be4ef << 64) | 0xeac64d09c8adf8ed,
        (0xb8f33653a53a8436 << 64) | 0xaedf39b62de91d95]
KAT1 = [(0x934704aff58fa233 << 64) | 0xd3c20d1b9cc18d8f,
        (0x530098817046d284 << 64) | 0x43e61d3273a04f7c]


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.mark.parametrize("portable", [False, True])
def test_aes_mmo_known_answers(portable):
    po.lib().or_force_portable_aes(1 if portable else 0)
    try:
        assert po.aes_mmo(0, [SEED0, SEED1]) == KAT0
        assert po.aes_mmo(KEY1, [SEED0, SEED1]) == KAT1
    finally:
        po.lib().or_force_portable_aes(0)


def test_aes_portable_equals_aesni_on_random_blocks():
    import random
    rng = random.Random(3)
    blocks = [rng.getrandbits(128) for _ in range(257)]
    key = rng.getrandbits(128)
    a = po.aes_mmo(key, blocks)
    po.lib().or_force_portable_aes(1)
    try:
        b = po.aes_mmo(key, blocks)
    finally:
        po.lib().or_force_portable_aes(0)
    assert a == b


def test_fips197_block():
    # FIPS-197 Appendix C.1 AES-128 vector (pins the raw cipher under MMO).
    key = bytes(range(16))
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    assert po.aes_encrypt_block(key, pt).hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"


def test_intmodn_sampling_known_answer():
    data = b"this is a length 32 test string."
    got = po.intmodn_sample(data, 4, P32, 5)
    r = int.from_bytes(b"this is a length", "little")
    want = [r % P32]
    for chunk in (b" 32 ", b"test", b" str", b"ing."):
        r = ((r // P32) << 32) | int.from_bytes(chunk, "little")
        want.append(r % P32)
    assert got == want


def test_intmodn_num_bytes_required_known_answer():
    import ctypes
    out = ctypes.c_int()
    rc = po.lib().or_intmodn_num_bytes_required(5, 32, ctypes.c_uint64(P32), ctypes.c_uint64(0),
                                                ctypes.c_double(40.0), ctypes.byref(out))
    assert rc == 0 and out.value == 32


def test_tuple_from_bytes_known_answers():
    data = b"A 128 bit string"
    (el,) = po.convert_bytes(("tuple", [("int", 64), ("int", 64)]), data)
    assert el == [int.from_bytes(b"A 128 bi", "little"), int.from_bytes(b"t string", "little")]
    data = b"A 128+32 bit string."
    (el,) = po.convert_bytes(("tuple", [("intmodn", 32, P32), ("intmodn", 32, P32)]), data)
    block = int.from_bytes(b"A 128+32 bit str", "little")
    e0 = block % P32
    block = ((block // P32) << 32) | int.from_bytes(b"ing.", "little")
    assert el == [e0, block % P32]


def test_oracle_reproduces_golden_aes(golden):
    g = golden["aes_mmo"]
    assert po.aes_mmo(KEY_LEFT, g["blocks"]) == g["left"]
    assert po.aes_mmo(KEY_RIGHT, g["blocks"]) == g["right"]
    assert po.aes_mmo(KEY_VALUE, g["blocks"]) == g["value"]


def test_oracle_reproduces_golden_evaluate_seeds(golden):
    for c in golden["evaluate_seeds"]:
        n, levels = c["num_seeds"], c["num_levels"]
        seeds = [(i << 64) | (i + 1) for i in range(n)]
        paths = [((23 * i + 42) << 64) | (42 * i + 23) for i in range(n)]
        cbs = [1 if i % 7 == 0 else 0 for i in range(n)]
        ncw = levels * n if c["per_seed_cw"] else levels
        cws = [((i + 1) << 64) | i for i in range(ncw)]
        ccl = [1 if i % 23 == 0 else 0 for i in range(ncw)]
        ccr = [1 if i % 42 != 0 else 0 for i in range(ncw)]
        s, cb = po.evaluate_seeds(seeds, cbs, paths, 0, cws, ccl, ccr, KEY_LEFT, KEY_RIGHT,
                                  levels)
        assert digest([s, cb]) == c["digest"]


def _cases(golden):
    return [c["name"] for c in golden["dpf"]]


def test_oracle_reproduces_golden_dpf(golden):
    for case in golden["dpf"]:
        levels = [(ld, _spec(spec), sec) for ld, spec, sec in case["levels"]]
        d = po.Dpf(levels)
        betas = [po.unflatten(l[1], b) for l, b in zip(levels, case["betas"])]
        k0, k1 = d.generate_keys(case["alpha"], betas, seeds=tuple(case["seeds"]))
        assert key_dict(k0) == case["key0"], case["name"]
        assert key_dict(k1) == case["key1"], case["name"]
        ctxs = [d.create_evaluation_context(k) for k in (k0, k1)]
        for ev in case["eval"]:
            o0 = d.evaluate_until(ev["level"], ev["prefixes"], ctxs[0])
            o1 = d.evaluate_until(ev["level"], ev["prefixes"], ctxs[1])
            assert digest(o0) == ev["digest0"], case["name"]
            assert digest(o1) == ev["digest1"], case["name"]
        if "evaluate_at" in case:
            e = case["evaluate_at"]
            assert d.evaluate_at(k0, e["level"], e["points"]) == e["out0"]
            assert d.evaluate_at(k1, e["level"], e["points"]) == e["out1"]


def _spec(s):
    """JSON lists back to the oracle's tuple specs."""
    if s[0] == "tuple":
        return ("tuple", [_spec(c) for c in s[1]])
    return tuple(s)


def test_golden_share_sum_property(golden):
    """out0 + out1 == beta at alpha and 0 elsewhere (full expansions)."""
    for case in golden["dpf"]:
        if len(case["levels"]) != 1:
            continue
        ld, spec, _ = case["levels"][0]
        spec = _spec(spec)
        ev = case["eval"][0]
        assert po.add_values(spec, ev["at_alpha0"], ev["at_alpha1"]) == case["betas"][0]
        if len(ev["values0"]) == ev["count"]:  # fully stored
            d = po.Dpf([tuple([ld, spec, case["levels"][0][2]])])
            k0, k1 = d.generate_keys(case["alpha"], [po.unflatten(spec, case["betas"][0])],
                                     seeds=tuple(case["seeds"]))
            o1 = d.evaluate_until(0, [], d.create_evaluation_context(k1))
            zero = [0] * po.num_scalars(spec)
            for i, (a, b) in enumerate(zip(ev["values0"], o1)):
                want = case["betas"][0] if i == case["alpha"] else zero
                assert po.add_values(spec, a, b) == want, (case["name"], i)


def test_golden_incremental_share_sum(golden):
    case = next(c for c in golden["dpf"] if c["name"] == "incremental_u64")
    levels = [(ld, _spec(spec), sec) for ld, spec, sec in case["levels"]]
    d = po.Dpf(levels)
    k0, k1 = d.generate_keys(case["alpha"], [b[0] for b in case["betas"]],
                             seeds=tuple(case["seeds"]))
    ctxs = [d.create_evaluation_context(k) for k in (k0, k1)]
    last = levels[-1][0]
    for ev in case["eval"]:
        h = ev["level"]
        ld = levels[h][0]
        o0 = d.evaluate_until(h, ev["prefixes"], ctxs[0])
        o1 = d.evaluate_until(h, ev["prefixes"], ctxs[1])
        prev = levels[h - 1][0] if h else 0
        idx = [(p << (ld - prev)) | j for p in (ev["prefixes"] or [0])
               for j in range(1 << (ld - prev))]
        a = case["alpha"] >> (last - ld)
        for i, x in enumerate(idx):
            s = (o0[i][0] + o1[i][0]) % (1 << 64)
            assert s == (case["betas"][h][0] if x == a else 0)


def test_oracle_reproduces_golden_inner_product(golden):
    g = golden["pir"]
    records = [bytes.fromhex(r) for r in g["records_hex"]]
    outs = po.inner_product(records, g["selections"])
    assert [o.hex() for o in outs] == g["out_hex"]
    # and against the unpacked definition (pir/testing/pir_selection_bits.cc:27-44)
    width = max(len(r) for r in records)
    for q, sel in enumerate(g["selections"]):
        acc = bytearray(width)
        for i, r in enumerate(records):
            if (sel[i // 128] >> (i % 128)) & 1:
                for j, b in enumerate(r):
                    acc[j] ^= b
        assert bytes(acc).hex() == g["out_hex"][q]


# ------------------------------------------------ AES-128-CTR seeded PRNG
# Aes128CtrSeededPrng (pir/prng/aes_128_ctr_seeded_prng.cc:60-101): key =
# seed, all-zero IV, AES_ctr128_encrypt of zeros (big-endian 128-bit counter).
CTR_FIXED_SEED_KAT = bytes.fromhex(
    "c6a13b37878f5b826f4f8162a1c8d879734613 9595c0b41e497bbde365f42d0a".replace(" ", ""))


def test_aes_ctr_prng_fixed_seed_known_answer():
    """aes_128_ctr_seeded_prng_test.cc:129-148."""
    assert po.aes_ctr_prng(bytes(range(16)), 32) == CTR_FIXED_SEED_KAT
    assert po.aes_ctr_prng(bytes(range(16)), 0) == b""


def _evp_aes_128_ctr(key: bytes, iv: bytes, chunks):
    """libcrypto EVP_aes_128_ctr over zero bytes, one EncryptUpdate per chunk."""
    import ctypes
    import ctypes.util
    name = ctypes.util.find_library("crypto")
    if not name:
        pytest.skip("libcrypto not present")
    L = ctypes.CDLL(name)
    L.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
    L.EVP_aes_128_ctr.restype = ctypes.c_void_p
    L.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p] * 5
    L.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_char_p,
                                    ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_int]
    L.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
    ctx = L.EVP_CIPHER_CTX_new()
    try:
        assert L.EVP_EncryptInit_ex(ctx, L.EVP_aes_128_ctr(), None, key, iv) == 1
        out = b""
        for n in chunks:
            buf = ctypes.create_string_buffer(max(n, 1))
            outl = ctypes.c_int(0)
            assert L.EVP_EncryptUpdate(ctx, buf, ctypes.byref(outl), bytes(n), n) == 1
            out += buf.raw[:outl.value]
        return out
    finally:
        L.EVP_CIPHER_CTX_free(ctx)


@pytest.mark.parametrize("seed_hex,length", [
    ("000102030405060708090a0b0c0d0e0f", 32),
    ("ffffffffffffffffffffffffffffffff", 1000),
    ("0123456789abcdeffedcba9876543210", 4099),
    ("8899aabbccddeeff0011223344556677", 1 << 16),
])
def test_aes_ctr_prng_matches_libcrypto(seed_hex, length):
    seed = bytes.fromhex(seed_hex)
    want = _evp_aes_128_ctr(seed, bytes(16), [length])
    assert po.aes_ctr_prng(seed, length) == want
    # GetRandomBytes in pieces continues the same stream (test.cc:81-91)
    assert _evp_aes_128_ctr(seed, bytes(16), [7, 0, 16, 1, length - 24]) == want


def test_c5_subtree_digest_fixture_matches_oracle():
    """The committed per-subtree digests of the headline key
    (tests/golden/c5_subtree_digests.json, 2 x 4096 SHA-256) are the
    oracle's: recompute the first, alpha's and the last subtree of both
    parties (the GPU test compares all 8192 with the device output)."""
    import hashlib
    import sys
    import numpy as np
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_c5_digests as mk
    with open(mk.OUT) as f:
        gold = json.load(f)
    alpha, beta, seeds = mk.key_params()
    assert gold["alpha"] == alpha and tuple(gold["beta"]) == beta
    assert [int(s) for s in gold["keygen_seeds"]] == list(seeds)
    d = po.Dpf([(mk.LOG_DOMAIN, mk.SPEC, mk.SECURITY)])
    keys = d.generate_keys(alpha, [beta], seeds=seeds)
    nsub = 1 << (mk.LOG_DOMAIN - mk.LOG_SUBTREE)
    for party in (0, 1):
        assert len(gold["sha256"][str(party)]) == nsub
        for s in (0, alpha >> mk.LOG_SUBTREE, nsub - 1):
            words = d.expand_subtree_words(keys[party], s << mk.LOG_SUBTREE,
                                           mk.LOG_SUBTREE).reshape(-1, 2, 2)
            got = hashlib.sha256(mk.host_layout_bytes(words)).hexdigest()
            assert got == gold["sha256"][str(party)][s], (party, s)
    # party 1 holds the negated shares, so no subtree digest of the two
    # parties coincides (the fixture is not degenerate)
    assert not set(gold["sha256"]["0"]) & set(gold["sha256"]["1"])
    assert len(set(gold["sha256"]["0"])) == nsub
