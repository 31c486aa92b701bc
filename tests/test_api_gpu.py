"""GPU parity of the reference's public API (Tier 2 of the C ABI): bit-exact
against the committed golden fixtures and the CPU oracle.

Follows the reference's tests:
  - full-domain / EvaluateAt over value types: distributed_point_function_
    test.cc:984-1079;
  - incremental contexts (EvaluateNext on surviving prefixes, context state):
    652-930;
  - EvaluateAndApply vs per-level EvaluateAt: 1081-1142;
  - dense PIR database inner product vs the unpacked definition:
    pir/dense_dpf_pir_database_test.cc:274-326;
  - PIR server plain / batched / concurrent: pir/dense_dpf_pir_server_test.cc:
    288-366; Leader + Helper end to end with the one-time pad:
    pir/dense_dpf_pir_client_test.cc:98-139, 230-244.
"""
import json
import os
import random
import threading
import zlib

import numpy as np
import pytest

from tests.test_pir_grid_gpu import device_row_stride

from oracle import pyoracle as po
from tests.golden.make_golden import digest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden.json")


def _spec(s):
    if s[0] == "tuple":
        return ("tuple", [_spec(c) for c in s[1]])
    return tuple(s)


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def api(cuda):
    from distributed_point_functions_amd import dpf, pir, value_types
    return dpf, value_types, pir


def _make(api, levels):
    D, V, _ = api
    params = [D.DpfParameters(ld, V.from_spec(s), sec) for ld, s, sec in levels]
    return D.DistributedPointFunction.create_incremental(params)


def test_golden_full_domain_and_evaluate_at(api, golden):
    D, V, _ = api
    for case in golden["dpf"]:
        if len(case["levels"]) != 1:
            continue
        levels = [(ld, _spec(s), sec) for ld, s, sec in case["levels"]]
        vt = V.from_spec(levels[0][1])
        dpf = _make(api, levels)
        beta = vt.unflatten(iter(case["betas"][0]))
        k0, k1 = dpf.generate_keys(case["alpha"], beta, seeds=case["seeds"])
        ev = case["eval"][0]
        for k, want in ((k0, ev["digest0"]), (k1, ev["digest1"])):
            got = vt.decode_flat(dpf.evaluate_next([], dpf.create_evaluation_context(k), raw=True))
            assert len(got) == ev["count"]
            assert digest(got) == want, case["name"]
        e = case["evaluate_at"]
        for k, want in ((k0, e["out0"]), (k1, e["out1"])):
            got = vt.decode_flat(dpf.evaluate_at(k, 0, e["points"], raw=True))
            assert got == want, case["name"]


def test_golden_incremental_with_context_state(api, golden):
    D, V, _ = api
    case = next(c for c in golden["dpf"] if c["name"] == "incremental_u64")
    levels = [(ld, _spec(s), sec) for ld, s, sec in case["levels"]]
    dpf = _make(api, levels)
    k0, k1 = dpf.generate_keys_incremental(case["alpha"], [b[0] for b in case["betas"]],
                                           seeds=case["seeds"])
    od = po.Dpf(levels)
    ok0, ok1 = od.generate_keys(case["alpha"], [b[0] for b in case["betas"]],
                                seeds=tuple(case["seeds"]))
    for k, ok, dk in ((k0, ok0, "digest0"), (k1, ok1, "digest1")):
        ctx = dpf.create_evaluation_context(k)
        octx = od.create_evaluation_context(ok)
        for ev in case["eval"]:
            vt = V.from_spec(levels[ev["level"]][1])
            got = vt.decode_flat(dpf.evaluate_next(ev["prefixes"], ctx, raw=True))
            assert digest(got) == ev[dk]
            od.evaluate_until(ev["level"], ev["prefixes"], octx)
            assert ctx.previous_hierarchy_level == octx.previous_hierarchy_level
            if ev["level"] + 1 < len(levels):
                assert ctx.partial_evaluations_level == octx.partial_evaluations_level
                assert sorted(ctx.partial_evaluations()) == sorted(
                    (p, s, bool(c)) for p, s, c in octx.partial_evaluations())


@pytest.mark.parametrize("spec", [("int", 64), ("int", 128), ("xor", 128),
                                  ("tuple", [("int", 32), ("int", 32)])])
def test_incremental_heavy_hitters_shape(api, spec):
    """c3 in miniature: hierarchy every 8 bits, EvaluateNext on surviving
    prefixes; bit-exact vs the oracle at every level, context serialised and
    re-parsed between levels (resumable state)."""
    lds = [8, 16, 24, 32]
    levels = [(ld, spec, 40 + ld) for ld in lds]
    rng = random.Random(zlib.crc32(repr(spec).encode()))
    alpha = rng.getrandbits(32)
    vt = api[1].from_spec(spec)
    betas = [vt.unflatten(iter([rng.getrandbits(s[1]) for s in po.scalar_specs(spec)]))
             for _ in lds]
    seeds = (rng.getrandbits(128), rng.getrandbits(128))
    dpf = _make(api, levels)
    od = po.Dpf(levels)
    k0, _ = dpf.generate_keys_incremental(alpha, betas, seeds=seeds)
    ok0, _ = od.generate_keys(alpha, betas, seeds=seeds)
    ctx = dpf.create_evaluation_context(k0)
    octx = od.create_evaluation_context(ok0)
    prefixes = []
    for h, ld in enumerate(lds):
        got = vt.decode_flat(dpf.evaluate_next(prefixes, ctx, raw=True))
        want = od.evaluate_until(h, prefixes, octx)
        assert got == want, h
        ctx = dpf.parse_evaluation_context(ctx.serialize())
        if h + 1 < len(lds):
            prev = lds[h - 1] if h else 0
            outs = [(p << (ld - prev)) | j for p in (prefixes or [0])
                    for j in range(1 << (ld - prev))]
            keep = set(rng.sample(outs, 64)) | {alpha >> (32 - ld)}
            prefixes = sorted(keep)


@pytest.mark.parametrize("lds", [[0, 1, 2], [8, 16, 32, 64], [0, 128], [128],
                                 list(range(0, 129, 16))])
def test_evaluate_and_apply_matches_per_level_evaluate_at(api, lds):
    spec = ("int", 64)
    levels = [(ld, spec, 0) for ld in lds]  # default security_parameter
    top = (1 << lds[-1]) - 1
    alpha = top
    dpf = _make(api, levels)
    od = po.Dpf(levels)
    betas = [1000 + i for i in range(len(lds))]
    k0, k1 = dpf.generate_keys_incremental(alpha, betas, seeds=(3, 4))
    ok0, ok1 = od.generate_keys(alpha, betas, seeds=(3, 4))
    points = [p & top for p in (23, 42, 123, 0, (1 << 128) - 1)]
    keys, okeys = [k0, k1, k0, k1, k0], [ok0, ok1, ok0, ok1, ok0]
    seen = []
    dpf.evaluate_and_apply(keys, points, lambda vals: seen.append(list(vals)) or True)
    assert len(seen) == len(lds)
    for h, ld in enumerate(lds):
        shift = lds[-1] - ld
        for i, (ok, p) in enumerate(zip(okeys, points)):
            prefix = p >> shift if shift < 128 else 0
            assert seen[h][i] == od.evaluate_at(ok, h, [prefix])[0][0], (h, i)


@pytest.mark.parametrize("spec,lds", [(("int", 32), [4, 12, 20]), (("int", 128), [16, 128]),
                                      (("xor", 128), [7, 19])])
def test_evaluate_and_apply_repeated_keys(api, spec, lds):
    """Many points per key object, interleaved and in runs (the library
    uploads each distinct key once and indexes it per point), both parties,
    every level against the oracle (h:1072-1198)."""
    levels = [(ld, spec, 0) for ld in lds]
    dpf = _make(api, levels)
    od = po.Dpf(levels)
    rng = random.Random(11)
    top = (1 << lds[-1]) - 1
    keys, okeys, alphas = [], [], []
    for s in range(3):
        alpha = rng.randrange(top + 1)
        alphas += [alpha, alpha]
        betas = [rng.randrange(1, 1 << 31) for _ in lds]
        k = dpf.generate_keys_incremental(alpha, betas, seeds=(10 + s, 20 + s))
        ok = od.generate_keys(alpha, betas, seeds=(10 + s, 20 + s))
        keys += list(k)
        okeys += list(ok)
    order = [i % 6 for i in range(120)] + [j for j in range(6) for _ in range(40)]
    head = order[:60]
    rng.shuffle(head)
    order[:60] = head
    points = [rng.randrange(top + 1) for _ in order]
    for i in range(0, len(points), 7):  # some points on their key's alpha path
        points[i] = alphas[order[i]]
    seen = []
    dpf.evaluate_and_apply([keys[j] for j in order], points,
                           lambda vals: seen.append(list(vals)) or True)
    assert len(seen) == len(lds)
    for h, ld in enumerate(lds):
        shift = lds[-1] - ld
        want = [od.evaluate_at(okeys[j], h, [p >> shift])[0][0] for j, p in zip(order, points)]
        assert seen[h] == want, h


def test_evaluate_and_apply_stops_when_op_returns_false(api):
    levels = [(8, ("int", 32), 48), (16, ("int", 32), 56)]
    dpf = _make(api, levels)
    k0, _ = dpf.generate_keys_incremental(5, [1, 2], seeds=(1, 2))
    calls = []
    dpf.evaluate_and_apply([k0], [5], lambda v: calls.append(v) and False)
    assert len(calls) == 1


# --------------------------------------------------------------------- PIR
def _records(n, size, seed):
    rng = np.random.default_rng(seed)
    return [bytes(rng.integers(0, 256, size if size else rng.integers(0, 100),
                               dtype=np.uint8)) for _ in range(n)]


def test_pir_database_inner_product_golden(api, golden):
    _, _, P = api
    g = golden["pir"]
    db = P.DenseDpfPirDatabase()
    for r in g["records_hex"]:
        db.insert(bytes.fromhex(r))
    db.build()
    assert db.size == len(g["records_hex"])
    assert [o.hex() for o in db.inner_product_with(g["selections"])] == g["out_hex"]


@pytest.mark.parametrize("n,size", [(1, 16), (127, 80), (128, 81), (1000, 256), (4099, 17)])
def test_pir_database_inner_product_vs_oracle(api, n, size):
    _, _, P = api
    records = _records(n, size, n)
    rng = random.Random(n)
    sels = [[rng.getrandbits(128) for _ in range((n + 127) // 128)] for _ in range(3)]
    db = P.DenseDpfPirDatabase()
    db.insert_fixed(np.frombuffer(b"".join(records), np.uint8).reshape(n, size))
    db.build()
    assert db.inner_product_with(sels) == po.inner_product(records, sels)


@pytest.mark.parametrize("size", [1, 16, 17, 32, 40, 80, 200, 240, 272, 500, 528, 1008, 1040,
                                  2064])
def test_pir_database_every_record_width(api, size):
    """KPirScanG maps every 16-byte-aligned width onto the wave (G = 64 ..
    1 records per wave-instruction, idle lanes, 64-chunk slices with a narrow
    tail): rows are stored at the reference's 16-byte alignment (whole
    128-byte lines from ~1.8 KiB on, where that costs at most 1/16), and 1,
    16 and 20 queries (two passes) answer as the oracle on a ragged last tile."""
    _, _, P = api
    n = 3001
    records = _records(n, size, size)
    arr = np.frombuffer(b"".join(records), np.uint8).reshape(n, size)
    rng = random.Random(size)
    sels = [[rng.getrandbits(128) for _ in range((n + 127) // 128)] for _ in range(20)]
    want = po.inner_product(records, sels)
    db = P.DenseDpfPirDatabase()
    db.insert_fixed(arr)
    db.build()
    assert db.record_stride == device_row_stride(size)
    assert db.max_value_size == size
    assert db.inner_product_with(sels) == want
    assert db.inner_product_with(sels[:16]) == want[:16]
    assert db.inner_product_with(sels[:1]) == want[:1]


def _pir_setup(api, n, size, seed=0):
    D, V, P = api
    records = _records(n, size, seed)
    ld = max(0, (n - 1).bit_length())
    dpf = D.DistributedPointFunction.create(D.DpfParameters(ld, V.XorWrapper(128)))
    return records, dpf


def _plain_server(api, records):
    _, _, P = api
    db = P.DenseDpfPirDatabase()
    for r in records:
        db.insert(r)
    return P.DenseDpfPirServer.create_plain(len(records), db)


def test_pir_plain_server_matches_oracle_and_reconstructs(api):
    _, _, P = api
    n = 1000
    records, dpf = _pir_setup(api, n, 48)
    server = _plain_server(api, records)
    idx = [0, 5, 500, 999, 128, 127]
    pairs = P.client_keys(dpf, n, idx, seeds=[(2 * i + 1, 2 * i + 2) for i in range(len(idx))])
    r0 = P.parse_response(server.handle_request(P.pir_request_plain([a for a, _ in pairs])))
    r1 = P.parse_response(server.handle_request(P.pir_request_plain([b for _, b in pairs])))
    for i, a, b in zip(idx, r0, r1):
        assert bytes(x ^ y for x, y in zip(a, b)) == records[i]
    # response of one server == oracle inner product with the oracle's expansion
    ld = max(0, (n - 1).bit_length())
    od = po.Dpf([(ld, ("xor", 128), 40 + ld)])
    nb = (n + 127) // 128
    for j, i in enumerate(idx):
        ok0, _ = od.generate_keys(i // 128, [1 << (i % 128)], seeds=(2 * j + 1, 2 * j + 2))
        sel = [v[0] for v in od.evaluate_until(0, [], od.create_evaluation_context(ok0))[:nb]]
        assert r0[j] == po.inner_product(records, [sel])[0]


def test_pir_batched_equals_singles_and_concurrent(api):
    _, _, P = api
    n = 777
    records, dpf = _pir_setup(api, n, 33, seed=3)
    server = _plain_server(api, records)
    idx = list(range(0, n, 97))
    keys = [a for a, _ in P.client_keys(dpf, n, idx)]
    batched = P.parse_response(server.handle_request(P.pir_request_plain(keys)))
    singles = [P.parse_response(server.handle_request(P.pir_request_plain([k])))[0]
               for k in keys]
    assert batched == singles
    results, errors = [None] * 16, []

    def worker(t):
        try:
            results[t] = P.parse_response(server.handle_request(P.pir_request_plain(keys)))
        except Exception as e:  # pragma: no cover
            errors.append(e)
    threads = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errors and all(r == batched for r in results)


def test_pir_fold_slots_reused_across_request_sizes(api):
    """A database large enough for the masked scan's atomic fold slots: the
    slots are kept zeroed by the fold between requests (FoldSlots), so a
    sequence of requests of different sizes — different slot widths in the
    same buffer — must each reconstruct exactly."""
    _, _, P = api
    n = 1 << 17
    records, dpf = _pir_setup(api, n, 32, seed=11)
    server0 = _plain_server(api, records)
    rng = np.random.default_rng(11)
    for q in (1, 8, 3, 1, 5, 8, 2):
        idx = [int(i) for i in rng.integers(0, n, q)]
        pairs = P.client_keys(dpf, n, idx)
        r0 = P.parse_response(server0.handle_request(P.pir_request_plain([a for a, _ in pairs])))
        r1 = P.parse_response(server0.handle_request(P.pir_request_plain([b for _, b in pairs])))
        for i, a, b in zip(idx, r0, r1):
            assert bytes(x ^ y for x, y in zip(a, b)) == records[i], (q, i)


def test_pir_leader_helper_end_to_end_with_one_time_pad(api):
    _, _, P = api
    n = 3000
    records, dpf = _pir_setup(api, n, 64, seed=7)
    idx = [2, 1500, 2999]
    pairs = P.client_keys(dpf, n, idx)
    otp_seed = bytes(range(16))
    helper_req = P.helper_request([b for _, b in pairs], otp_seed)
    encrypted = b"ct:" + helper_req  # stand-in for Tink HybridEncrypt

    def decrypter(ct, info):
        assert info == P.DenseDpfPirServer.ENCRYPTION_CONTEXT_INFO
        return ct[3:]

    def mk_db():
        db = P.DenseDpfPirDatabase()
        for r in records:
            db.insert(r)
        return db
    helper = P.DenseDpfPirServer.create_helper(n, mk_db(), decrypter)

    def sender(req, while_waiting):
        while_waiting()
        return helper.handle_request(req)
    leader = P.DenseDpfPirServer.create_leader(n, mk_db(), sender)
    resp = P.parse_response(leader.handle_request(
        P.pir_request_leader([a for a, _ in pairs], encrypted)))
    pad = po.aes_ctr_prng(otp_seed, sum(len(r) for r in resp))
    off = 0
    for i, r in zip(idx, resp):
        assert bytes(x ^ y for x, y in zip(r, pad[off:off + len(r)])) == records[i]
        off += len(r)


def test_pir_leader_requires_while_waiting(api):
    from distributed_point_functions_amd._lib import DpfAmdError
    _, _, P = api
    n = 200
    records, dpf = _pir_setup(api, n, 16)
    db = P.DenseDpfPirDatabase()
    for r in records:
        db.insert(r)
    leader = P.DenseDpfPirServer.create_leader(n, db, lambda req, ww: b"")
    (a, _), = P.client_keys(dpf, n, [3])
    with pytest.raises(DpfAmdError) as e:
        leader.handle_request(P.pir_request_leader([a], b"x"))
    assert e.value.code == 9
    assert e.value.message == ("HandleRequest: `while_waiting` was not called from `sender` "
                               "passed at construction.")


def test_incremental_unsorted_duplicate_and_missing_prefixes(api):
    """The partial-evaluation lookup's paths: sorted prefixes take the
    one-pass merge join, shuffled / repeated ones the hash path (reference
    btree semantics: outputs in the caller's order, duplicates repeated), and
    a prefix whose parent was never evaluated fails with the reference's
    message — all checked against the oracle."""
    D, V, _ = api
    spec = ("int", 64)
    lds = [8, 16, 24]
    levels = [(ld, spec, 40 + ld) for ld in lds]
    rng = random.Random(77)
    alpha = rng.getrandbits(24)
    betas = [rng.getrandbits(64) for _ in lds]
    seeds = (rng.getrandbits(128), rng.getrandbits(128))
    dpf = _make(api, levels)
    od = po.Dpf(levels)
    k0, _ = dpf.generate_keys_incremental(alpha, betas, seeds=seeds)
    ok0, _ = od.generate_keys(alpha, betas, seeds=seeds)
    vt = V.from_spec(spec)
    for order in ("sorted", "shuffled"):
        ctx = dpf.create_evaluation_context(k0)
        octx = od.create_evaluation_context(ok0)
        assert vt.decode_flat(dpf.evaluate_next([], ctx, raw=True)) == od.evaluate_until(0, [], octx)
        p1 = sorted(set(rng.sample(range(256), 40)) | {alpha >> 16})
        if order == "shuffled":
            p1 = p1 + p1[:5]  # duplicates
            rng.shuffle(p1)
        got = vt.decode_flat(dpf.evaluate_next(p1, ctx, raw=True))
        assert got == od.evaluate_until(1, p1, octx), order
        base = sorted(set(p1))
        p2 = sorted({(p << 8) | rng.randrange(256) for p in base for _ in range(3)})
        if order == "shuffled":
            rng.shuffle(p2)
        got = vt.decode_flat(dpf.evaluate_next(p2, ctx, raw=True))
        assert got == od.evaluate_until(2, p2, octx), order
    # a level-1 prefix whose level-0 parent was not among the evaluated ones
    ctx = dpf.create_evaluation_context(k0)
    octx = od.create_evaluation_context(ok0)
    dpf.evaluate_next([], ctx, raw=True)
    od.evaluate_until(0, [], octx)
    dpf.evaluate_next([1, 2, 3], ctx, raw=True)
    od.evaluate_until(1, [1, 2, 3], octx)
    with pytest.raises(Exception) as ours:
        dpf.evaluate_next([(7 << 8) | 1], ctx, raw=True)
    with pytest.raises(Exception) as ref:
        od.evaluate_until(2, [(7 << 8) | 1], octx)
    assert "Prefix not present in ctx.partial_evaluations" in str(ours.value)
    assert str(ours.value).split(":")[-1].strip() == str(ref.value).split(":")[-1].strip()


@pytest.mark.parametrize("n", [100, 1 << 14])
def test_incremental_prefix_range_error_names_the_first_bad_prefix(api, n):
    """EvaluateUntil's prefix range check (h:735-745): the first prefix at or
    above 2^previous_log_domain_size is reported with the reference's message,
    for short lists (checked up front) and long ones (checked inside the
    de-duplication's parallel pass), and the context is left untouched so the
    same level still evaluates afterwards."""
    D, V, _ = api
    spec = ("int", 64)
    levels = [(ld, spec, 40 + ld) for ld in (8, 16)]
    rng = random.Random(79)
    alpha, betas = rng.getrandbits(16), [rng.getrandbits(64) for _ in range(2)]
    seeds = (rng.getrandbits(128), rng.getrandbits(128))
    dpf = _make(api, levels)
    od = po.Dpf(levels)
    k0, _ = dpf.generate_keys_incremental(alpha, betas, seeds=seeds)
    ok0, _ = od.generate_keys(alpha, betas, seeds=seeds)
    vt = V.from_spec(spec)
    ctx = dpf.create_evaluation_context(k0)
    octx = od.create_evaluation_context(ok0)
    dpf.evaluate_next([], ctx, raw=True)
    od.evaluate_until(0, [], octx)
    good = sorted(rng.randrange(256) for _ in range(n))
    bad = list(good)
    bad[n // 3] = 300
    bad[2 * n // 3] = 999
    with pytest.raises(Exception) as ours:
        dpf.evaluate_next(bad, ctx, raw=True)
    with pytest.raises(Exception) as ref:
        od.evaluate_until(1, bad, octx)
    assert "Index 300 out of range for hierarchy level 0" in str(ours.value)
    assert str(ours.value).split(":")[-1].strip() == str(ref.value).split(":")[-1].strip()
    got = vt.decode_flat(dpf.evaluate_next(good, ctx, raw=True))
    assert got == od.evaluate_until(1, good, octx)


def test_incremental_duplicate_partial_evaluation_past_the_queries(api):
    """A duplicate stored prefix with a mismatching seed is rejected wherever
    it sits in ctx.partial_evaluations (cc:390-405 builds its btree from the
    whole list), including after the last entry a sorted query reaches; a
    duplicate with the same seed and control bit is accepted."""
    from distributed_point_functions_amd import wire
    D, V, _ = api
    spec = ("int", 64)
    levels = [(ld, spec, 40 + ld) for ld in (8, 16, 24)]
    rng = random.Random(78)
    alpha = rng.getrandbits(24)
    betas = [rng.getrandbits(64) for _ in levels]
    seeds = (rng.getrandbits(128), rng.getrandbits(128))
    dpf = _make(api, levels)
    od = po.Dpf(levels)
    k0, _ = dpf.generate_keys_incremental(alpha, betas, seeds=seeds)
    ok0, _ = od.generate_keys(alpha, betas, seeds=seeds)
    vt = V.from_spec(spec)
    ctx = dpf.create_evaluation_context(k0)
    octx = od.create_evaluation_context(ok0)
    dpf.evaluate_next([], ctx, raw=True)
    od.evaluate_until(0, [], octx)
    p1 = list(range(40))
    assert vt.decode_flat(dpf.evaluate_next(p1, ctx, raw=True)) == od.evaluate_until(1, p1, octx)
    pes = ctx.partial_evaluations()
    assert len(pes) > 2 and [p for p, _, _ in pes] == sorted({p for p, _, _ in pes})
    last_prefix, last_seed, last_cb = pes[-1]
    p2 = [(0 << 8) | 3, (1 << 8) | 9]  # their stored parents come first in the list

    def with_extra(seed, cb):
        pe = (wire.field_bytes(1, wire.block(last_prefix)) +
              wire.field_bytes(2, wire.block(seed)) + wire.field_varint(3, int(cb)))
        return dpf.parse_evaluation_context(ctx.serialize() + wire.field_bytes(4, pe))

    with pytest.raises(Exception) as e:
        dpf.evaluate_next(p2, with_extra(last_seed ^ (1 << 77), last_cb), raw=True)
    assert "Duplicate prefix in `ctx.partial_evaluations()` with mismatching seed or " \
           "control bit" in str(e.value)
    with pytest.raises(Exception) as e:
        dpf.evaluate_next(p2, with_extra(last_seed, not last_cb), raw=True)
    assert "Duplicate prefix" in str(e.value)
    same = with_extra(last_seed, last_cb)
    assert vt.decode_flat(dpf.evaluate_next(p2, same, raw=True)) == od.evaluate_until(2, p2, octx)
