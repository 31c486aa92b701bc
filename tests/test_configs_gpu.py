"""BASELINE.json configs c2, c3 and c4 at their full sizes, bit-exact against
the CPU oracle (test_fullsize_gpu.py covers c1's and c5's expansion kernels).

c2  EvaluateAt of 2^20 random points over 64 keys, log_domain_size 128,
    uint128 (workload of dpf/distributed_point_function_benchmark.cc:97-152
    and experiments/synthetic_data_benchmarks.cc:45-308): through the batched
    multi-key kernel and through the Tier-2 EvaluateAt API; every point
    compared with the oracle's EvaluateAt.
c3  incremental heavy hitters, 16 hierarchy levels 8, 16, ..., 128 bits,
    uint64, 2^16 distinct surviving prefixes per level, each an 8-bit
    extension of a previous-level prefix (generator of
    distributed_point_function_benchmark.cc:154-191): every output and the
    EvaluationContext state (previous level, partial-evaluation level and
    entries) compared with the oracle at every level; share sum of both
    parties = beta_i on alpha's prefix, 0 elsewhere.
c4  dense PIR over 2^26 records x 256 B (pir/dense_dpf_pir_database_
    benchmark.cc:37-157): full-size XOR scans with Q in {1, 8, 64} (and 100,
    the benchmark's largest batch) whose selection vectors are non-zero only
    in four 2^16-record windows, compared with the oracle inner product over
    those windows; bench.py's 8-rank row split run rank by rank with the
    device XOR fold equals the 1-rank result; HandleRequest on the full
    database reconstructs random records from two servers' responses.
"""
import random

import numpy as np
import pytest

from oracle import pyoracle as po

pytestmark = pytest.mark.gpu

M64 = (1 << 64) - 1


@pytest.fixture(scope="module")
def K(cuda):
    from distributed_point_functions_amd import kernels
    return kernels


# ---------------------------------------------------------------------------
# c2: 64 keys x 16,384 points, log_domain_size 128, uint128
# ---------------------------------------------------------------------------

def test_c2_full_size_batched_and_api_match_oracle(K, cuda):
    import torch
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    rng = random.Random(2)
    nkeys, per = 64, 1 << 14
    spec = ("int", 128)
    dpf = DistributedPointFunction.create(DpfParameters(128, V.Integer(128)))
    od = po.Dpf([(128, spec, 0)])  # default security parameter
    L = dpf.hierarchy_to_tree(0)
    assert L == 128
    keys, okeys, alphas, betas = [], [], [], []
    for k in range(nkeys):
        alpha, beta = rng.getrandbits(128), rng.getrandbits(128)
        seeds = (1000 + 2 * k, 1001 + 2 * k)
        keys.append(dpf.generate_keys(alpha, beta, seeds=seeds))
        okeys.append(od.generate_keys(alpha, [beta], seeds=seeds))
        alphas.append(alpha)
        betas.append(beta)
    prng = np.random.default_rng(2)
    pts = prng.integers(0, 1 << 63, size=(nkeys * per, 2), dtype=np.uint64) * 2 + \
        prng.integers(0, 2, size=(nkeys * per, 2), dtype=np.uint64)
    for k in range(nkeys):  # alpha among each key's points
        pts[k * per + 7] = (alphas[k] & M64, alphas[k] >> 64)
    # parties alternate over the keys
    party_of = [k % 2 for k in range(nkeys)]
    want = np.concatenate([od.evaluate_at_words(okeys[k][party_of[k]], 0,
                                                pts[k * per:(k + 1) * per])
                           for k in range(nkeys)])
    # one multi-key launch (dpf_amd_evaluate_points_batched)
    ks = [okeys[k][party_of[k]] for k in range(nkeys)]
    desc = V.Integer(128).descriptor(od.blocks_needed(0))
    u8 = lambda a: torch.tensor(a, dtype=torch.uint8, device=cuda)  # noqa: E731
    out = K.evaluate_points_batched(
        nkeys, per, K.u128_tensor([k.seed for k in ks], cuda), u8([k.party for k in ks]),
        torch.from_numpy(pts.view(np.int64)).to(cuda), 0, L,
        K.u128_tensor([c for k in ks for c in k.cw_seeds()[:L]], cuda),
        u8([c for k in ks for c in k.ccl()[:L]]), u8([c for k in ks for c in k.ccr()[:L]]),
        desc, key_party=torch.tensor([k.party for k in ks], dtype=torch.int8, device=cuda),
        key_value_corrections=K.u128_tensor([c for k in ks for c in k.value_corrections()[0]],
                                            cuda))
    got = out.cpu().numpy().view(np.uint64).reshape(-1, 2)
    assert np.array_equal(got, want[:, 0, :])
    # the Tier-2 API, key by key (EvaluateAt<absl::uint128>(key, 0, points))
    for k in range(nkeys):
        api = dpf.evaluate_at(keys[k][party_of[k]], 0, pts[k * per:(k + 1) * per], raw=True)
        a = api.view(np.uint64).reshape(-1, 2)
        assert np.array_equal(a, want[k * per:(k + 1) * per, 0, :]), k
    # EvaluateAndApply<absl::uint128> over all 2^20 (key, point) pairs
    # (h:1072-1198), each key object repeated for its 16,384 points (c2a)
    seen = []
    kl = [keys[k][party_of[k]] for k in range(nkeys) for _ in range(per)]
    dpf.evaluate_and_apply(kl, pts, lambda v: seen.append(v) or True)
    assert len(seen) == 1
    assert seen[0] == [int(lo) | (int(hi) << 64) for lo, hi in want[:, 0, :]]
    # share sum at alpha (and 0 at a non-alpha point) with the other party
    for k in range(0, nkeys, 9):
        other = dpf.evaluate_at(keys[k][1 - party_of[k]], 0, pts[k * per:k * per + 9], raw=True)
        mine = got[k * per:k * per + 9]
        o = other.view(np.uint64).reshape(-1, 2)
        s = [((int(a[0]) | int(a[1]) << 64) + (int(b[0]) | int(b[1]) << 64)) % (1 << 128)
             for a, b in zip(mine, o)]
        assert s[7] == betas[k] and s[0] == 0, k


# ---------------------------------------------------------------------------
# c3: heavy hitters, 16 levels x 8 bits, 2^16 prefixes per level
# ---------------------------------------------------------------------------

def _c3_prefixes(rng, alpha, H):
    prefixes = [[]]
    for i in range(1, H):
        if i == 1:
            cur = list(range(256))
        else:
            cur = set()
            prev = prefixes[i - 1]
            while len(cur) < (1 << 16):
                cur.add((prev[rng.randrange(len(prev))] << 8) | rng.randrange(256))
            cur = sorted(cur)
        ap = alpha >> (128 - 8 * i)
        if ap not in cur:
            cur[rng.randrange(len(cur))] = ap
            cur = sorted(cur)
        prefixes.append(cur)
    return prefixes


def test_c3_full_size_outputs_and_context_match_oracle(cuda):
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    rng = random.Random(3)
    H = 16
    spec = ("int", 64)
    params = [DpfParameters(8 * (i + 1), V.Integer(64)) for i in range(H)]
    dpf = DistributedPointFunction.create_incremental(params)
    od = po.Dpf([(8 * (i + 1), spec, 0) for i in range(H)])
    alpha = rng.getrandbits(128)
    betas = [rng.getrandbits(64) for _ in range(H)]
    seeds = (0x31, 0x32)
    k0, k1 = dpf.generate_keys_incremental(alpha, betas, seeds=seeds)
    ok0, _ = od.generate_keys(alpha, betas, seeds=seeds)
    prefixes = _c3_prefixes(rng, alpha, H)
    rows = [np.array([[p & M64, p >> 64] for p in ps], dtype=np.uint64).reshape(-1, 2)
            if ps else [] for ps in prefixes]
    ctx0, ctx1 = dpf.create_evaluation_context(k0), dpf.create_evaluation_context(k1)
    octx = od.create_evaluation_context(ok0)
    for i in range(H):
        a = dpf.evaluate_next(rows[i], ctx0, raw=True).view(np.uint64)
        want = od.evaluate_until_words(i, prefixes[i], octx)[:, 0, 0]
        assert a.shape == want.shape and np.array_equal(a, want), i
        assert ctx0.previous_hierarchy_level == octx.previous_hierarchy_level == i
        if i + 1 < H:
            assert ctx0.partial_evaluations_level == octx.partial_evaluations_level, i
            got_pe = sorted(ctx0.partial_evaluations())
            want_pe = sorted((p, s, bool(c)) for p, s, c in octx.partial_evaluations())
            assert len(got_pe) == len(want_pe) and got_pe == want_pe, i
        b = dpf.evaluate_next(rows[i], ctx1, raw=True).view(np.uint64)
        s = a + b
        nz = np.nonzero(s)[0]
        assert len(nz) == 1 and int(s[nz[0]]) == betas[i], i
        # the non-zero sits at alpha's prefix, element (alpha's next 8 bits)
        per = len(a) // max(1, len(prefixes[i]))
        pos = (prefixes[i].index(alpha >> (128 - 8 * i)) * per if i else 0) + \
            ((alpha >> (128 - 8 * (i + 1))) & 0xFF)
        assert nz[0] == pos, i


# ---------------------------------------------------------------------------
# c4: 2^26 records x 256 B
# ---------------------------------------------------------------------------

N4, REC = 1 << 26, 256
WINDOW = 1 << 16


@pytest.fixture(scope="module")
def c4_db(cuda):
    import torch
    host = np.frombuffer(np.random.default_rng(4).bytes(N4 * REC), dtype=np.uint8)
    dev = torch.from_numpy(host).to(cuda)
    rng = random.Random(44)
    starts = sorted({0, N4 - WINDOW} | {rng.randrange(N4 // WINDOW) * WINDOW for _ in range(2)})
    while len(starts) < 4:
        starts = sorted(set(starts) | {rng.randrange(N4 // WINDOW) * WINDOW})
    d = dict(host=host.reshape(N4, REC), dev=dev, windows=starts)
    del dev, host
    yield d
    d.clear()
    torch.cuda.empty_cache()


def _window_selections(c4, q, seed):
    """Q selection vectors of N4/128 blocks, random bits inside the windows
    and zero elsewhere; also the window-only blocks the oracle sees."""
    rng = np.random.default_rng(seed)
    nb = N4 // 128
    sel = np.zeros((q, nb, 2), dtype=np.uint64)
    for s in c4["windows"]:
        b0, b1 = s // 128, (s + WINDOW) // 128
        sel[:, b0:b1] = rng.integers(0, 1 << 63, size=(q, b1 - b0, 2), dtype=np.uint64) * 2 + \
            rng.integers(0, 2, size=(q, b1 - b0, 2), dtype=np.uint64)
    return sel


def _oracle_windows(c4, sel):
    recs = [c4["host"][i].tobytes() for s in c4["windows"] for i in range(s, s + WINDOW)]
    blocks = [[int(w[0]) | (int(w[1]) << 64)
               for s in c4["windows"] for w in sel[k, s // 128:(s + WINDOW) // 128]]
              for k in range(sel.shape[0])]
    return po.inner_product(recs, blocks)


@pytest.mark.parametrize("q", [1, 8, 64, 100])
def test_c4_full_size_scan_matches_oracle_on_windows(K, cuda, c4_db, q):
    import torch
    sel = _window_selections(c4_db, q, q)
    d_sel = torch.from_numpy(sel.reshape(-1, 2).view(np.int64)).to(cuda)
    out = K.inner_product(c4_db["dev"], N4, REC, d_sel, q).cpu().numpy().reshape(q, REC)
    want = _oracle_windows(c4_db, sel)
    for k in range(q):
        assert out[k].tobytes() == want[k], k


def test_c4_eight_rank_row_split_fold_equals_one_rank(K, cuda, c4_db):
    import torch
    from distributed_point_functions_amd import sharding
    q = 8
    rng = np.random.default_rng(8)
    sel = rng.integers(0, 1 << 63, size=(q, N4 // 128, 2), dtype=np.uint64) * 2
    d_sel = torch.from_numpy(sel.view(np.int64)).to(cuda)  # (q, nb, 2)
    full = K.inner_product(c4_db["dev"], N4, REC, d_sel.reshape(-1, 2), q)
    world = 8
    parts = torch.empty(world * q * REC, dtype=torch.uint8, device=cuda)
    for rank in range(world):
        r_lo, r_hi, b_lo, b_hi = sharding.pir_row_shard(N4, world, rank)
        shard_sel = d_sel[:, b_lo:b_hi].contiguous().reshape(-1, 2)
        K.inner_product(c4_db["dev"][r_lo * REC:r_hi * REC], r_hi - r_lo, REC, shard_sel, q,
                        out=parts[rank * q * REC:(rank + 1) * q * REC])
    folded = K.xor_fold(parts, world, q * REC)
    assert torch.equal(folded, full)


def test_c4_full_size_handle_request_reconstructs(c4_db):
    from distributed_point_functions_amd import pir as P
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    servers = []
    for _ in range(2):
        db = P.DenseDpfPirDatabase()
        db.insert_fixed(c4_db["host"])
        db.build()
        assert db.size == N4
        servers.append(P.DenseDpfPirServer.create_plain(N4, db))
    dpf = DistributedPointFunction.create(DpfParameters(26, V.XorWrapper(128)))
    rng = random.Random(26)
    idx = [0, N4 - 1, 127, 128] + [rng.randrange(N4) for _ in range(4)]
    pairs = P.client_keys(dpf, N4, idx)
    r0 = P.parse_response(servers[0].handle_request(P.pir_request_plain([a for a, _ in pairs])))
    r1 = P.parse_response(servers[1].handle_request(P.pir_request_plain([b for _, b in pairs])))
    for i, a, b in zip(idx, r0, r1):
        assert bytes(x ^ y for x, y in zip(a, b)) == c4_db["host"][i].tobytes(), i


def test_c4_full_size_handle_request_on_sharded_database(c4_db):
    """c4 through the library's multi-GPU path (rows in 8 shards, here all on
    this GPU): the server's responses equal the single-shard server's bit for
    bit, and the two parties' shares reconstruct the records."""
    from distributed_point_functions_amd import pir as P
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    sharded = P.DenseDpfPirDatabase([0] * 8)
    sharded.insert_fixed(c4_db["host"])
    sharded.build()
    sh = sharded.shards()
    assert len(sh) == 8 and sh[-1][2] == N4 and all(r0 % 128 == 0 for _, r0, _ in sh)
    plain = P.DenseDpfPirDatabase()
    plain.insert_fixed(c4_db["host"])
    plain.build()
    s_sharded = P.DenseDpfPirServer.create_plain(N4, sharded)
    s_plain = P.DenseDpfPirServer.create_plain(N4, plain)
    dpf = DistributedPointFunction.create(DpfParameters(26, V.XorWrapper(128)))
    rng = random.Random(2626)
    idx = [0, N4 - 1, (N4 // 8) - 1, N4 // 8] + [rng.randrange(N4) for _ in range(4)]
    pairs = P.client_keys(dpf, N4, idx)
    req0 = P.pir_request_plain([a for a, _ in pairs])
    req1 = P.pir_request_plain([b for _, b in pairs])
    r0 = P.parse_response(s_sharded.handle_request(req0))
    assert r0 == P.parse_response(s_plain.handle_request(req0))
    r1 = P.parse_response(s_plain.handle_request(req1))
    for i, a, b in zip(idx, r0, r1):
        assert bytes(x ^ y for x, y in zip(a, b)) == c4_db["host"][i].tobytes(), i


def test_c4_full_size_forced_peer_copies_on_sharded_database(c4_db):
    """The cross-device branches of the multi-GPU database forced on one GPU
    (dpf_amd_set_force_peer_copies): hipMemcpyPeer of each shard's rows out
    of the resident c4 tensor at build, hipMemcpyPeerAsync of the Q x 256 B
    partials into the first shard's device before the fold
    (pir/dense_dpf_pir_server.cc:92-127 spread over 8 shards).  Window scans
    equal the oracle, HandleRequest equals the single-shard server, and the
    parties' shares reconstruct the records."""
    from distributed_point_functions_amd import _lib
    from distributed_point_functions_amd import pir as P
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    L = _lib.lib()
    L.dpf_amd_set_force_peer_copies(1)
    try:
        sharded = P.DenseDpfPirDatabase([0] * 8).insert_fixed_device(c4_db["dev"], N4, REC).build()
        assert len(sharded.shards()) == 8
        sel = _window_selections(c4_db, 2, 2026)
        lists = [[int(w[0]) | (int(w[1]) << 64) for w in sel[k]] for k in range(2)]
        assert sharded.inner_product_with(lists) == _oracle_windows(c4_db, sel)
        plain = P.DenseDpfPirDatabase()
        plain.insert_fixed(c4_db["host"])
        plain.build()
        s_sharded = P.DenseDpfPirServer.create_plain(N4, sharded)
        s_plain = P.DenseDpfPirServer.create_plain(N4, plain)
        dpf = DistributedPointFunction.create(DpfParameters(26, V.XorWrapper(128)))
        rng = random.Random(8026)
        idx = [0, N4 - 1, (N4 // 8) - 1, N4 // 8] + [rng.randrange(N4) for _ in range(4)]
        pairs = P.client_keys(dpf, N4, idx)
        req0 = P.pir_request_plain([a for a, _ in pairs])
        req1 = P.pir_request_plain([b for _, b in pairs])
        r0 = P.parse_response(s_sharded.handle_request(req0))
        assert r0 == P.parse_response(s_plain.handle_request(req0))
        r1 = P.parse_response(s_sharded.handle_request(req1))
        for i, a, b in zip(idx, r0, r1):
            assert bytes(x ^ y for x, y in zip(a, b)) == c4_db["host"][i].tobytes(), i
    finally:
        L.dpf_amd_set_force_peer_copies(0)
