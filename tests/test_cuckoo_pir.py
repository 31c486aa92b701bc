"""Cuckoo-hashed sparse (keyword) PIR: hash family, cuckoo placement, database
and server, against the CPU restatement in oracle/cuckoo_oracle.py.

Follows the reference's tests:
  - SHA-256 hash family NIST vector and modular reduction:
    pir/hashing/sha256_hash_family_test.cc:36-59;
  - hash family config / CreateHashFunctions errors:
    pir/hashing/hash_family_config_test.cc, hash_family_test.cc;
  - cuckoo database builder errors, placement properties, inner products:
    pir/cuckoo_hashed_dpf_pir_database_test.cc:64-272;
  - server creation errors, plain / leader / helper end to end:
    pir/cuckoo_hashing_sparse_dpf_pir_server_test.cc,
    pir/cuckoo_hashing_sparse_dpf_pir_client_test.cc.
The CPU tests only run host code (hashing, placement, protos); the `gpu`
tests build the HBM tables and run HandleRequest.
"""
import hashlib
import random

import pytest

from oracle import cuckoo_oracle as co

NIST_SEED = bytes.fromhex("5a86b737eaea8ee976a0a24da63e7ed7")
NIST_INPUT = bytes.fromhex(
    "eefad18a101c1211e2b3650c5187c2a8a650547208251f6d4237e661c7bf4c77f3353903"
    "94c37fa1a9f9be836ac28509")
NIST_OUTPUT = bytes.fromhex("42e61e174fbb3897d6dd6cef3dd2802fe67b331953b06114a65c772859dfc1aa")


@pytest.fixture(scope="module")
def C():
    from distributed_point_functions_amd import cuckoo_pir
    return cuckoo_pir


def _err(fn):
    from distributed_point_functions_amd._lib import DpfAmdError
    with pytest.raises(DpfAmdError) as e:
        fn()
    return e.value.code, e.value.message


# ------------------------------------------------------------------ oracle pins
def test_oracle_sha256_hash_nist_vector():
    assert hashlib.sha256(NIST_SEED + NIST_INPUT).digest() == NIST_OUTPUT
    want = int.from_bytes(NIST_OUTPUT, "little")
    assert all(co.sha256_hash(NIST_SEED, NIST_INPUT, i) == want % i for i in range(1, 1000))


def test_oracle_mt19937_64_known_answer():
    r = co.MT19937_64()
    for _ in range(9999):
        r()
    assert r() == 9981545732273789042


def test_oracle_absl_uniform_range_and_balance():
    r = co.MT19937_64(7)
    counts = [0, 0, 0]
    for _ in range(3000):
        counts[co._absl_uniform(r, 3)] += 1
    assert all(900 < c < 1100 for c in counts)
    r = co.MT19937_64(7)
    assert {co._absl_uniform(r, 4) for _ in range(200)} == {0, 1, 2, 3}


# ------------------------------------------------------------------ hashing (C ABI)
def test_sha256_hash_matches_nist_vector(C):
    want = int.from_bytes(NIST_OUTPUT, "little")
    for i in range(1, 1000):
        assert C.sha256_hash(NIST_SEED, NIST_INPUT, i) == want % i


@pytest.mark.parametrize("n", [0, 1, 31, 55, 56, 63, 64, 65, 119, 120, 128, 1000])
def test_sha256_hash_padding_boundaries(C, n):
    rng = random.Random(n)
    seed = bytes(rng.randrange(256) for _ in range(rng.choice([0, 5, 16, 70])))
    data = bytes(rng.randrange(256) for _ in range(n))
    for ub in [1, 2, 3, 150, 1 << 20, (1 << 31) - 1]:
        assert C.sha256_hash(seed, data, ub) == co.sha256_hash(seed, data, ub)


def test_hash_positions_follow_family_seed(C):
    params = C.cuckoo_hashing_params(b"0123456789abcdef", 1000, 5)
    for q in [b"a", b"key17", b"x" * 100]:
        assert C.hash_positions(params, q) == [f(q, 1000) for f in
                                               co.hash_functions(b"0123456789abcdef", 5)]


def test_hash_family_errors(C):
    from distributed_point_functions_amd import _lib
    import ctypes
    out = (ctypes.c_int * 3)()
    cfg = C.hash_family_config(C.HASH_FAMILY_SHA256, b"")
    assert _err(lambda: _lib.check(_lib.lib().dpf_amd_hash_family_evaluate(
        cfg, len(cfg), 3, b"a", 1, 10, out))) == (3, "`seed` must not be empty")
    cfg = C.hash_family_config(C.HASH_FAMILY_UNSPECIFIED, b"s")
    assert _err(lambda: _lib.check(_lib.lib().dpf_amd_hash_family_evaluate(
        cfg, len(cfg), 3, b"a", 1, 10, out))) == (3, "Hash family unspecified")
    cfg = C.hash_family_config(7, b"s")
    assert _err(lambda: _lib.check(_lib.lib().dpf_amd_hash_family_evaluate(
        cfg, len(cfg), 3, b"a", 1, 10, out))) == (3, "Unknown hash family specified")
    cfg = C.hash_family_config(C.HASH_FAMILY_SHA256, b"s")
    assert _err(lambda: _lib.check(_lib.lib().dpf_amd_hash_family_evaluate(
        cfg, len(cfg), -1, b"a", 1, 10, out))) == (3, "num_hash_functions must not be negative")


# ------------------------------------------------------------------ params / protos
def test_generate_params(C):
    p = C.parse_cuckoo_hashing_params(C.generate_params(1234))
    assert p["hash_family"] == C.HASH_FAMILY_SHA256
    assert len(p["seed"]) == 16
    assert p["num_hash_functions"] == 3
    assert p["num_buckets"] == 1851  # int64(1.5 * 1234)
    assert C.parse_cuckoo_hashing_params(C.generate_params(1234))["seed"] != p["seed"]


def test_generate_params_rejects_dense_config(C):
    from distributed_point_functions_amd import _lib, pir
    import ctypes
    cfg = pir.pir_config(100)
    buf = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    assert _err(lambda: _lib.check(_lib.lib().dpf_amd_cuckoo_generate_params(
        cfg, len(cfg), ctypes.byref(buf), ctypes.byref(n)))) == (
        3, "`config` must be a valid CuckooHashingSparseDpfPirConfig")


# ------------------------------------------------------------------ placement
def _records(n, seed=0, max_len=40):
    rng = random.Random(seed)
    recs = {}
    while len(recs) < n:
        k = bytes(rng.randrange(1, 256) for _ in range(rng.randrange(1, 24)))
        recs[k] = bytes(rng.randrange(256) for _ in range(rng.randrange(0, max_len)))
    return recs


@pytest.mark.parametrize("n,buckets,k", [(1, 2, 2), (10, 15, 3), (300, 450, 3), (500, 600, 4),
                                         (64, 64, 2)])
def test_placement_matches_oracle_and_hash_property(C, n, buckets, k):
    seed = bytes(range(16))
    params = C.cuckoo_hashing_params(seed, buckets, k)
    db = C.CuckooHashedDpfPirDatabase(params)
    recs = _records(n, seed=n)
    for key, v in recs.items():
        db.insert(key, v)
    table = db.place()
    assert table == co.cuckoo_place(list(recs), seed, buckets, k)
    fns = co.hash_functions(seed, k)
    for b, key in enumerate(table):
        if key is not None:
            assert key in recs and b in [f(key, buckets) for f in fns]
    assert len({x for x in table if x is not None}) == sum(x is not None for x in table)


def test_first_insert_of_a_key_wins(C):
    params = C.cuckoo_hashing_params(b"s" * 16, 6)
    db = C.CuckooHashedDpfPirDatabase(params)
    db.insert(b"k", b"first").insert(b"k", b"second")
    assert sum(x is not None for x in db.place()) == 1


def test_builder_errors(C):
    db = C.CuckooHashedDpfPirDatabase(C.cuckoo_hashing_params(b"s" * 16, 0))
    assert _err(db.place) == (3, "`num_buckets` must be positive")
    db = C.CuckooHashedDpfPirDatabase(C.cuckoo_hashing_params(b"s" * 16, 10, 0))
    assert _err(db.place) == (3, "`num_hash_functions` must be positive")
    db = C.CuckooHashedDpfPirDatabase(C.cuckoo_hashing_params(b"", 10))
    assert _err(db.place) == (3, "`seed` must not be empty")
    db = C.CuckooHashedDpfPirDatabase(C.cuckoo_hashing_params(b"s" * 16, 10, 1))
    db.insert(b"a", b"b")
    assert _err(db.place) == (3, "hash_functions.size() must be at least 2")
    db = C.CuckooHashedDpfPirDatabase(C.cuckoo_hashing_params(b"s" * 16, 10))
    db.insert(b"", b"Value")
    assert _err(db.place) == (3, "Key cannot be empty")


# ================================================================== GPU
def _setup(C, n, seed=0, max_len=40):
    from distributed_point_functions_amd import dpf as D, value_types as V
    hseed = bytes((seed + i) & 0xFF for i in range(16))
    nb = int(1.5 * n)
    params = C.cuckoo_hashing_params(hseed, nb)
    recs = _records(n, seed=seed, max_len=max_len)
    ld = max(0, (nb - 1).bit_length())
    dpf = D.DistributedPointFunction.create(D.DpfParameters(ld, V.XorWrapper(128)))
    return params, recs, dpf


def _db(C, params, recs):
    db = C.CuckooHashedDpfPirDatabase(params)
    for k, v in recs.items():
        db.insert(k, v)
    return db


def _pad(b, n):
    return b + bytes(n - len(b))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 100, 2000])
def test_plain_servers_reconstruct_bucket_rows(C, cuda, n):
    """XOR of the two servers' responses = the key row and value row of every
    requested bucket, bit-exact against the oracle's tables."""
    params, recs, dpf = _setup(C, n, seed=n)
    hseed = C.parse_cuckoo_hashing_params(params)["seed"]
    nb = C.parse_cuckoo_hashing_params(params)["num_buckets"]
    keys_t, vals_t = co.cuckoo_tables(recs, hseed, nb, 3)
    kw = max(len(k) for k in keys_t)
    vw = max(len(v) for v in vals_t)
    s0 = C.CuckooHashingSparseDpfPirServer.create_plain(params, _db(C, params, recs))
    s1 = C.CuckooHashingSparseDpfPirServer.create_plain(params, _db(C, params, recs))
    client = C.CuckooHashingSparseDpfPirClient(params, dpf)
    rng = random.Random(n)
    queries = rng.sample(sorted(recs), min(5, n)) + [b"missing-key"]
    r0, r1 = client.create_requests(queries)
    resp0, resp1 = s0.handle_request(r0), s1.handle_request(r1)
    from distributed_point_functions_amd.pir import parse_response
    raw = [bytes(a ^ b for a, b in zip(x, y))
           for x, y in zip(parse_response(resp0), parse_response(resp1))]
    buckets = [h for q in queries for h in C.hash_positions(params, q)]
    assert len(raw) == 2 * len(buckets)
    for j, b in enumerate(buckets):
        assert raw[2 * j] == _pad(keys_t[b], kw)
        assert raw[2 * j + 1] == _pad(vals_t[b], vw)
    got = client.handle_responses(queries, resp0, resp1)
    served = {k for k in keys_t if k}
    for q, g in zip(queries, got):
        if q in served:
            assert g == _pad(recs[q], vw)
        else:
            assert g is None


@pytest.mark.gpu
def test_single_server_response_matches_oracle_inner_product(C, cuda):
    """One server's masked response = the oracle's XOR inner product of its
    DPF share with the tables."""
    from oracle import pyoracle as po
    from distributed_point_functions_amd.pir import client_keys, parse_response, \
        pir_request_plain
    params, recs, dpf = _setup(C, 300, seed=3)
    p = C.parse_cuckoo_hashing_params(params)
    keys_t, vals_t = co.cuckoo_tables(recs, p["seed"], p["num_buckets"], 3)
    server = C.CuckooHashingSparseDpfPirServer.create_plain(params, _db(C, params, recs))
    idx = [0, 17, p["num_buckets"] - 1]
    seeds = [(2 * j + 1, 2 * j + 2) for j in range(len(idx))]
    pairs = client_keys(dpf, p["num_buckets"], idx, seeds=seeds)
    resp = parse_response(server.handle_request(pir_request_plain([a for a, _ in pairs])))
    ld = max(0, (p["num_buckets"] - 1).bit_length())
    od = po.Dpf([(ld, ("xor", 128), 40 + ld)])
    nblk = (p["num_buckets"] + 127) // 128
    for j, i in enumerate(idx):
        ok0, _ = od.generate_keys(i // 128, [1 << (i % 128)], seeds=seeds[j])
        sel = [v[0] for v in od.evaluate_until(0, [], od.create_evaluation_context(ok0))[:nblk]]
        bits = [(sel[r // 128] >> (r % 128)) & 1 for r in range(p["num_buckets"])]
        assert resp[2 * j] == co.inner_product(keys_t, bits)
        assert resp[2 * j + 1] == co.inner_product(vals_t, bits)
        assert resp[2 * j] == po.inner_product(keys_t, [sel])[0]


@pytest.mark.gpu
def test_server_creation_errors(C, cuda):
    params, recs, _ = _setup(C, 50)
    p = C.parse_cuckoo_hashing_params(params)
    wrong = C.cuckoo_hashing_params(p["seed"], p["num_buckets"] + 1)
    assert _err(lambda: C.CuckooHashingSparseDpfPirServer.create_plain(
        wrong, _db(C, params, recs))) == (
        3, "Number of selection bits in the database does not match `params.num_buckets`")
    unspecified = C.cuckoo_hashing_params(p["seed"], p["num_buckets"], 3,
                                          C.HASH_FAMILY_UNSPECIFIED)
    assert _err(lambda: C.CuckooHashingSparseDpfPirServer.create_plain(
        unspecified, _db(C, params, recs))) == (
        3, "params.hash_family_config.hash_family must be set")
    server = C.CuckooHashingSparseDpfPirServer.create_plain(params, _db(C, params, recs))
    from distributed_point_functions_amd.pir import pir_request_plain
    assert _err(lambda: server.handle_request(pir_request_plain([]))) == (
        3, "`dpf_key` must not be empty")
    pub = server.public_params()
    from distributed_point_functions_amd import wire
    assert bytes(wire.decode(pub)[1][-1]) == params


@pytest.mark.gpu
def test_build_twice_fails(C, cuda):
    params, recs, _ = _setup(C, 20)
    db = _db(C, params, recs).build()
    assert db.size() == 20 and db.num_selection_bits() == 30
    assert _err(db.build) == (9, "Database already built")


@pytest.mark.gpu
def test_leader_helper_end_to_end(C, cuda):
    from oracle import pyoracle as po
    from distributed_point_functions_amd import pir as P
    params, recs, dpf = _setup(C, 500, seed=11)
    p = C.parse_cuckoo_hashing_params(params)
    keys_t, vals_t = co.cuckoo_tables(recs, p["seed"], p["num_buckets"], 3)
    queries = sorted(recs)[:3]
    buckets = [h for q in queries for h in C.hash_positions(params, q)]
    pairs = P.client_keys(dpf, p["num_buckets"], buckets)
    otp_seed = bytes(range(16, 32))
    encrypted = b"ct:" + P.helper_request([b for _, b in pairs], otp_seed)

    def decrypter(ct, info):
        assert info == C.CuckooHashingSparseDpfPirServer.ENCRYPTION_CONTEXT_INFO
        return ct[3:]
    helper = C.CuckooHashingSparseDpfPirServer.create_helper(params, _db(C, params, recs),
                                                             decrypter)

    def sender(req, while_waiting):
        while_waiting()
        return helper.handle_request(req)
    leader = C.CuckooHashingSparseDpfPirServer.create_leader(params, _db(C, params, recs), sender)
    resp = P.parse_response(leader.handle_request(
        P.pir_request_leader([a for a, _ in pairs], encrypted)))
    pad = po.aes_ctr_prng(otp_seed, sum(len(r) for r in resp))
    off, plain = 0, []
    for r in resp:
        plain.append(bytes(x ^ y for x, y in zip(r, pad[off:off + len(r)])))
        off += len(r)
    kw = max(len(k) for k in keys_t)
    vw = max(len(v) for v in vals_t)
    for j, b in enumerate(buckets):
        assert plain[2 * j] == _pad(keys_t[b], kw)
        assert plain[2 * j + 1] == _pad(vals_t[b], vw)
