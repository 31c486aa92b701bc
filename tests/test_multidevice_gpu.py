"""Multi-GPU inside the library, rehearsed on one GPU by repeating device ids.

A sharded DenseDpfPirDatabase (dpf_amd_pir_db_set_devices) splits its rows
into 128-record-aligned shards, one per device entry; HandleRequest expands
each shard's selection blocks (a leaf range of every key) on the shard's
device, scans there, and folds the Q x record partials on the first shard's
device — the reference's single InnerProductWith call
(pir/dense_dpf_pir_server.cc:92-127, pir/pir_database_interface.h:65-66)
spread over GPUs.  ExpandLeavesOnDevices splits one key's domain the same
way (c5).  With devices {0, 0, ...} every shard runs on this GPU through the
same code path (per-device streams, the partials' combine, the fold), and
the results must equal the single-shard library and the oracle bit for bit.
Shards on one device take the device-local copy branches by default; the
`forced_peer` tests turn on dpf_amd_set_force_peer_copies so the
cross-device branches (hipMemcpyPeer of rows at build — packed, then
re-strided for record sizes that are not a multiple of 16 —, and
hipMemcpyPeerAsync of the partials) execute here too.  Two distinct GPUs
are exercised only when the box has them (test_two_devices_*); the 8-GPU
node is the driver's.
"""
import random

import numpy as np
import pytest

from oracle import pyoracle as po

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def P(cuda):
    from distributed_point_functions_amd import pir
    return pir


def _db(P, records, devices=None):
    db = P.DenseDpfPirDatabase(devices)
    db.insert_fixed(records)
    db.build()
    return db


def _sel(rng, q, n):
    return [[rng.getrandbits(128) for _ in range((n + 127) // 128)] for _ in range(q)]


@pytest.mark.parametrize("n,size,shards", [(1000, 240, 4), (128 * 37 + 5, 256, 3),
                                           (300, 16, 5), (4096, 1040, 2), (1, 32, 3)])
def test_shard_layout(P, n, size, shards):
    recs = np.random.default_rng(n).integers(0, 256, (n, size), dtype=np.uint8)
    db = _db(P, recs, [0] * shards)
    sh = db.shards()
    blocks = (n + 127) // 128
    assert len(sh) == min(shards, blocks)
    assert sh[0][1] == 0 and sh[-1][2] == n
    for (d, r0, r1), nxt in zip(sh, sh[1:] + [(0, n, n)]):
        assert d == 0 and r0 % 128 == 0 and r1 == nxt[1] and r1 > r0


@pytest.mark.parametrize("n,size,q", [(1000, 240, 1), (1000, 240, 5), (128 * 37 + 5, 256, 20),
                                      (300, 16, 3), (4096, 1040, 2), (5000, 80, 64)])
def test_sharded_inner_product_matches_single_shard_and_oracle(P, n, size, q):
    rng = random.Random(n * 7 + q)
    recs = np.random.default_rng(n + q).integers(0, 256, (n, size), dtype=np.uint8)
    one = _db(P, recs)
    four = _db(P, recs, [0, 0, 0, 0])
    sels = _sel(rng, q, n)
    want = one.inner_product_with(sels)
    assert four.inner_product_with(sels) == want
    rows = [recs[i].tobytes() for i in range(n)]
    assert want == po.inner_product(rows, sels)


def test_sharded_handle_request_reconstructs_and_equals_single_shard(P):
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    n, size = 128 * 300 + 17, 256
    recs = np.random.default_rng(9).integers(0, 256, (n, size), dtype=np.uint8)
    sharded = [P.DenseDpfPirServer.create_plain(n, _db(P, recs, [0] * 4)) for _ in range(2)]
    plain = P.DenseDpfPirServer.create_plain(n, _db(P, recs))
    dpf = DistributedPointFunction.create(DpfParameters((n - 1).bit_length(), V.XorWrapper(128)))
    rng = random.Random(3)
    # indices at shard boundaries (each shard holds 75 blocks) and random ones
    idx = [0, n - 1, 128 * 75 - 1, 128 * 75, 128 * 150, 128 * 225 + 5] + \
        [rng.randrange(n) for _ in range(4)]
    pairs = P.client_keys(dpf, n, idx)
    req0 = P.pir_request_plain([a for a, _ in pairs])
    req1 = P.pir_request_plain([b for _, b in pairs])
    r0 = P.parse_response(sharded[0].handle_request(req0))
    r1 = P.parse_response(sharded[1].handle_request(req1))
    assert r0 == P.parse_response(plain.handle_request(req0))
    for i, a, b in zip(idx, r0, r1):
        assert bytes(x ^ y for x, y in zip(a, b)) == recs[i].tobytes(), i


def test_sharded_handle_request_many_keys(P):
    """One request of 20 keys (the batched per-leaf walk expands each shard's
    leaf range) and one of 3 keys over 8 shards."""
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    n, size = 20000, 64
    recs = np.random.default_rng(20).integers(0, 256, (n, size), dtype=np.uint8)
    dpf = DistributedPointFunction.create(DpfParameters((n - 1).bit_length(), V.XorWrapper(128)))
    rng = random.Random(20)
    for shards, nq in ((8, 3), (3, 20)):
        servers = [P.DenseDpfPirServer.create_plain(n, _db(P, recs, [0] * shards))
                   for _ in range(2)]
        idx = [rng.randrange(n) for _ in range(nq)]
        pairs = P.client_keys(dpf, n, idx)
        r0 = P.parse_response(servers[0].handle_request(P.pir_request_plain([a for a, _ in pairs])))
        r1 = P.parse_response(servers[1].handle_request(P.pir_request_plain([b for _, b in pairs])))
        for i, a, b in zip(idx, r0, r1):
            assert bytes(x ^ y for x, y in zip(a, b)) == recs[i].tobytes(), (shards, i)


def test_set_devices_validates(P):
    from distributed_point_functions_amd import _lib
    with pytest.raises(_lib.DpfAmdError):
        P.DenseDpfPirDatabase([0, 1 << 20])


def test_expand_leaves_on_devices_matches_one_launch_and_oracle(cuda):
    import torch
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    p64 = 2 ** 64 - 59
    spec = ("tuple", [("int", 32), ("intmodn", 64, p64)])
    ld = 20
    vt = V.from_spec(spec)
    dpf = DistributedPointFunction.create(DpfParameters(ld, vt, 48))
    k0, _ = dpf.generate_keys(777777, (5, 6), seeds=(11, 12))
    n = 1 << ld
    full = torch.empty(n * 16, dtype=torch.uint8, device=cuda)
    dpf.expand_leaves_on_devices(k0, [(0, 0, n, full)])
    cuts = [0, 1, 4097, 1 << 19, n - 3, n]
    parts = [torch.empty((hi - lo) * 16, dtype=torch.uint8, device=cuda)
             for lo, hi in zip(cuts, cuts[1:])]
    dpf.expand_leaves_on_devices(k0, [(0, lo, hi, t) for (lo, hi), t in
                                      zip(zip(cuts, cuts[1:]), parts)])
    assert torch.equal(torch.cat(parts), full)
    od = po.Dpf([(ld, spec, 48)])
    ok0, _ = od.generate_keys(777777, [(5, 6)], seeds=(11, 12))
    want = od.evaluate_until_words(0, [], od.create_evaluation_context(ok0))
    got = full.cpu().numpy().view(np.uint64).reshape(-1, 2)
    assert np.array_equal(got[:, 0], want[:, 1, 0]) and np.array_equal(got[:, 1], want[:, 0, 0])


@pytest.mark.parametrize("size,shards", [(256, None), (40, [0, 0, 0]), (1040, [0, 0])])
def test_insert_fixed_device_equals_host_built(P, cuda, size, shards):
    """A database built from rows already in HBM (written by a torch kernel
    just before the build, on another stream than the library's) scans like
    the host-built one, also re-strided (40 B rows -> 48 B) and sharded."""
    import torch
    n = 128 * 21 + 9
    g = torch.Generator(device=cuda)
    g.manual_seed(size)
    rows = torch.randint(0, 256, (n * size,), dtype=torch.uint8, device=cuda, generator=g)
    dev_db = P.DenseDpfPirDatabase(shards).insert_fixed_device(rows, n, size).build()
    host_db = _db(P, rows.cpu().numpy().reshape(n, size))
    rng = random.Random(size)
    sels = _sel(rng, 6, n)
    assert dev_db.inner_product_with(sels) == host_db.inner_product_with(sels)


@pytest.fixture
def forced_peer(P):
    from distributed_point_functions_amd import _lib
    L = _lib.lib()
    L.dpf_amd_set_force_peer_copies(1)
    yield
    L.dpf_amd_set_force_peer_copies(0)


@pytest.mark.parametrize("n,size,q,shards", [(1000, 240, 5, 4), (128 * 37 + 5, 256, 20, 3),
                                             (300, 16, 3, 5), (4096, 1040, 2, 2)])
def test_forced_peer_inner_product_matches_oracle(P, forced_peer, n, size, q, shards):
    rng = random.Random(n * 11 + q)
    recs = np.random.default_rng(n * 3 + q).integers(0, 256, (n, size), dtype=np.uint8)
    db = _db(P, recs, [0] * shards)
    sels = _sel(rng, q, n)
    rows = [recs[i].tobytes() for i in range(n)]
    assert db.inner_product_with(sels) == po.inner_product(rows, sels)


@pytest.mark.parametrize("size,shards", [(256, [0, 0, 0]), (40, [0, 0, 0]), (1040, [0, 0])])
def test_forced_peer_device_rows_build(P, cuda, forced_peer, size, shards):
    """Rows in HBM copied to each shard by hipMemcpyPeer (40 B rows: one peer
    copy of the packed rows, then the 48 B re-stride on the shard device)."""
    import torch
    n = 128 * 21 + 9
    g = torch.Generator(device=cuda)
    g.manual_seed(size + 1)
    rows = torch.randint(0, 256, (n * size,), dtype=torch.uint8, device=cuda, generator=g)
    dev_db = P.DenseDpfPirDatabase(shards).insert_fixed_device(rows, n, size).build()
    host = rows.cpu().numpy().reshape(n, size)
    rng = random.Random(size + 1)
    sels = _sel(rng, 6, n)
    assert dev_db.inner_product_with(sels) == po.inner_product(
        [host[i].tobytes() for i in range(n)], sels)


def test_invalid_device_ids_are_rejected(cuda):
    """ExpandLeavesOnDevices checks every device id before any launch."""
    import torch
    from distributed_point_functions_amd import _lib
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    dpf = DistributedPointFunction.create(DpfParameters(12, V.Integer(64)))
    k0, _ = dpf.generate_keys(5, 6)
    out = torch.empty(4096 * 8, dtype=torch.uint8, device=cuda)
    with pytest.raises(_lib.DpfAmdError) as e:
        dpf.expand_leaves_on_devices(k0, [(0, 0, 1024, out), (1 << 20, 1024, 2048, out)])
    assert e.value.code == 3 and "invalid device id" in e.value.message


@pytest.mark.skipif("not __import__('torch').cuda.is_available() or "
                    "__import__('torch').cuda.device_count() < 2",
                    reason="needs two GPUs")
def test_two_devices_sharded_inner_product_and_expansion(P):
    import torch
    n, size, q = 128 * 40 + 3, 240, 7
    recs = np.random.default_rng(2).integers(0, 256, (n, size), dtype=np.uint8)
    rng = random.Random(2)
    sels = _sel(rng, q, n)
    assert _db(P, recs, [0, 1]).inner_product_with(sels) == _db(P, recs).inner_product_with(sels)
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    dpf = DistributedPointFunction.create(DpfParameters(20, V.Integer(64)))
    k0, _ = dpf.generate_keys(12345, 6, seeds=(1, 2))
    nt = 1 << dpf.hierarchy_to_tree(0)  # tree leaves, two uint64 elements each
    half = nt // 2
    a = torch.empty(half * 16, dtype=torch.uint8, device="cuda:0")
    b = torch.empty(half * 16, dtype=torch.uint8, device="cuda:1")
    full = torch.empty(nt * 16, dtype=torch.uint8, device="cuda:0")
    dpf.expand_leaves_on_devices(k0, [(0, 0, half, a), (1, half, nt, b)])
    dpf.expand_leaves_on_devices(k0, [(0, 0, nt, full)])
    assert torch.equal(torch.cat([a, b.to("cuda:0")]), full)
