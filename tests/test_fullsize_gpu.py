"""Parity of the expansion kernels that the production launches select, and
of the benchmarked configuration at its full size.

`dpf_amd_expand_and_correct` picks the kernel from the launch size
(kernels_capi.cc): KExpand<8> (register DFS of depth 8 per thread) once a
launch covers >= 2^25 tree leaves, KExpand<4> from 2^22, the cooperative
KExpandCoop (2^10 leaves per block below 2^19 tree leaves, 2^11 from there)
below that when the tree has >= 11 levels, KExpand<D> with D = 4 / 2 / 1 on
smaller trees.  These tests
  * force D in {1, 2, 4, 8} and each KExpandCoop variant
    (dpf_amd_set_expand_depth) on small domains and compare every output of
    every value type with the oracle;
  * run the automatic choice at sizes where it picks KExpandCoop (2^11-2^21
    tree leaves), KExpand<4> (2^24) and KExpand<8> (2^25) and compare every
    output with the oracle;
  * run the c5 bench configuration itself (log_domain_size 32,
    Tuple<uint32, IntModN<uint64, 2^64-59>>, the KExpand<8, EmitU32ModN64>
    launch the bench times) for both parties: every one of the 2^32 leaves
    of both parties is compared with the oracle through per-2^20-leaf-subtree
    SHA-256 digests (tests/golden/c5_subtree_digests.json); the share sum
    over all leaves (beta at alpha, 0 elsewhere — the reference's own
    full-domain property, distributed_point_function_test.cc:652-696) checks
    the alpha path; leaf-range slices above 2^31 equal the matching part of
    the full launch, and bench.py's 8-rank subtree split
    (sharding.block_range), run rank by rank on this GPU, reproduces the
    1-rank output.
"""
import random

import numpy as np
import pytest

from oracle import pyoracle as po

from tests.golden.make_golden import KEY_LEFT, KEY_RIGHT
from tests.test_kernels_gpu import P64, TYPES, _keys, u8

pytestmark = pytest.mark.gpu

C5 = ("tuple", [("int", 32), ("intmodn", 64, P64)])


@pytest.fixture(scope="module")
def K(cuda):
    from distributed_point_functions_amd import kernels
    return kernels


def _key_arrays(K, cuda, d, key):
    L = d.hierarchy_to_tree(0)
    return dict(
        seed=K.u128_tensor([key.seed], cuda), cb=u8([key.party], cuda), L=L,
        cw=K.u128_tensor(key.cw_seeds()[:L] or [0], cuda), ccl=u8(key.ccl()[:L] or [0], cuda),
        ccr=u8(key.ccr()[:L] or [0], cuda), corr=key.value_corrections()[0], party=key.party)


def _expand(K, cuda, d, key, spec, leaf_begin=0, leaf_end=None, out=None):
    """Device expansion (uint8 tensor of host-layout T) through the C ABI."""
    from distributed_point_functions_amd import value_types as vtm
    vt = vtm.from_spec(spec)
    ka = _key_arrays(K, cuda, d, key)
    cepb = 1 << (d.levels[0][0] - ka["L"])
    return K.expand_and_correct(ka["seed"], ka["cb"], ka["L"], ka["cw"], ka["ccl"], ka["ccr"],
                                vt.descriptor(d.blocks_needed(0)), ka["corr"], ka["party"],
                                cepb, leaf_begin, leaf_end, out)


def _chunked_equal(a, b, chunk=1 << 32) -> bool:
    """torch.equal without a full-size temporary (64 GiB buffers)."""
    import torch
    if a.numel() != b.numel():
        return False
    return all(torch.equal(a[i:i + chunk], b[i:i + chunk]) for i in range(0, a.numel(), chunk))


def _assert_host_layout_equals_words(spec, got: np.ndarray, words: np.ndarray, what=""):
    """got: host-layout bytes of n elements; words: oracle (n, ns, 2) uint64."""
    from distributed_point_functions_amd import value_types as vtm
    vt = vtm.from_spec(spec)
    arr = got.view(vt.numpy_dtype())
    assert arr.shape[0] == words.shape[0], what
    for i, s in enumerate(vt.scalars()):
        col = arr["f%d" % i]
        if s.bits == 128:
            ok = np.array_equal(col[:, 0], words[:, i, 0]) and \
                np.array_equal(col[:, 1], words[:, i, 1])
        else:
            ok = np.array_equal(col.astype(np.uint64), words[:, i, 0]) and \
                not words[:, i, 1].any()
        if not ok:
            bad = np.nonzero(col.astype(np.uint64) != words[:, i, 0])[0] \
                if s.bits != 128 else np.nonzero(col[:, 0] != words[:, i, 0])[0]
            pytest.fail("%s: scalar %d differs from the oracle at %d elements (first %s)" %
                        (what, i, len(bad), bad[:5]))


# ---------------------------------------------------------------------------
# Every DFS depth, every value type, whole domain vs oracle
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("depth", [1, 2, 4, 5, 6, 8])
@pytest.mark.parametrize("spec", TYPES, ids=[repr(t) for t in TYPES])
def test_forced_depth_matches_oracle(K, cuda, spec, depth):
    """Every DFS depth KExpand is instantiated with, every emitter (D = 6
    included: the batched PIR selection's depth, instantiated for every
    type since round 6; D = 5: c3's levels and 2^23-2^24-leaf expansions)."""
    d, k0, k1, alpha, beta = _keys(spec, 14, seed=depth)
    assert d.hierarchy_to_tree(0) >= depth
    with K.forced_expand_depth(depth):
        for key in (k0, k1):
            want = d.evaluate_until_words(0, [], d.create_evaluation_context(key))
            got = _expand(K, cuda, d, key, spec).cpu().numpy()
            _assert_host_layout_equals_words(spec, got, want, "party %d" % key.party)


RANGE_TYPES = [C5, ("int", 64), ("xor", 128)]


@pytest.mark.parametrize("depth", [4, 5, 6, 8])
@pytest.mark.parametrize("spec", RANGE_TYPES, ids=[repr(t) for t in RANGE_TYPES])
def test_forced_depth_leaf_ranges(K, cuda, spec, depth):
    """Ragged leaf ranges that start and end inside a 2^D-leaf subtree, both
    parties (tree leaves; the 8-byte type returns two elements per leaf)."""
    d, k0, k1, _, _ = _keys(spec, 15, seed=3)
    n = 1 << d.hierarchy_to_tree(0)
    with K.forced_expand_depth(depth):
        for key in (k0, k1):
            want = d.evaluate_until_words(0, [], d.create_evaluation_context(key))
            e = len(want) // n  # elements per tree leaf
            for lo, hi in [(0, n), (1, n - 1), (63, 65), (255, 257), (3000, 3001),
                           (4097, 20000), (n - 300, n)]:
                if hi > n:
                    continue
                got = _expand(K, cuda, d, key, spec, lo, hi).cpu().numpy()
                _assert_host_layout_equals_words(spec, got, want[lo * e:hi * e],
                                                 "party %d [%d, %d)" % (key.party, lo, hi))


@pytest.mark.parametrize("spec", RANGE_TYPES, ids=[repr(t) for t in RANGE_TYPES])
def test_depth6_many_roots_matches_oracle(K, cuda, spec):
    """KExpand<6> from many roots with one walk level per thread — the shape
    of an incremental level (2^k prefix roots, 7 tree levels below each,
    dpf.cc EvaluateUntilOnDevice) — against the oracle's expansion of the
    same roots (ExpandSeeds cc:289-372, HashExpandedSeeds cc:523-547)."""
    import torch
    from distributed_point_functions_amd import value_types as vtm
    d, k0, k1, _, _ = _keys(spec, 20, seed=6)
    L = d.hierarchy_to_tree(0)
    top = L - 7  # roots at tree level L - 7, 7 levels expanded below each
    nroots = 1 << top
    vt = vtm.from_spec(spec)
    for key in (k0, k1):
        want = d.evaluate_until_words(0, [], d.create_evaluation_context(key))
        e = len(want) >> L
        # the roots themselves: every node of level `top` (oracle walk,
        # evaluate_prg_hwy.cc:552-634)
        seeds, cbs = po.evaluate_seeds([key.seed] * nroots, [key.party] * nroots,
                                       list(range(nroots)), 0, key.cw_seeds()[:top],
                                       key.ccl()[:top], key.ccr()[:top], KEY_LEFT, KEY_RIGHT,
                                       top)
        ka = _key_arrays(K, cuda, d, key)
        cw = K.u128_tensor(key.cw_seeds()[top:L], cuda)
        ccl = u8(key.ccl()[top:L], cuda)
        ccr = u8(key.ccr()[top:L], cuda)
        for lo, hi in [(0, nroots << 7), (5, (nroots << 7) - 77), (127, 129)]:
            with K.forced_expand_depth(6):
                got = K.expand_and_correct(K.u128_tensor(seeds, cuda), u8(cbs, cuda), 7, cw, ccl,
                                           ccr, vt.descriptor(d.blocks_needed(0)), ka["corr"],
                                           ka["party"], e, lo, hi)
            _assert_host_layout_equals_words(spec, got.cpu().numpy(), want[lo * e:hi * e],
                                             "party %d [%d, %d)" % (key.party, lo, hi))
    torch.cuda.empty_cache()


@pytest.mark.parametrize("coop", [-1, -2, -3])
@pytest.mark.parametrize("spec", TYPES, ids=[repr(t) for t in TYPES])
def test_cooperative_kernel_matches_oracle(K, cuda, spec, coop):
    """KExpandCoop (1024 / 2048 leaves per block: wave-0 walk to 64
    sub-roots, four LDS breadth-first levels, one leaf per thread; 256 leaves
    per block: two quad levels and the value hash on quads) forced on a
    2^16-element domain of every value type, both parties."""
    d, k0, k1, alpha, beta = _keys(spec, 16, seed=20 - coop)
    assert d.hierarchy_to_tree(0) >= 11
    with K.forced_expand_depth(coop):
        for key in (k0, k1):
            want = d.evaluate_until_words(0, [], d.create_evaluation_context(key))
            got = _expand(K, cuda, d, key, spec).cpu().numpy()
            _assert_host_layout_equals_words(spec, got, want, "party %d" % key.party)


@pytest.mark.parametrize("coop", [-1, -2, -3])
def test_cooperative_kernel_leaf_ranges(K, cuda, coop):
    """Ragged leaf ranges inside and across the 2^10 / 2^11 / 2^8-leaf blocks."""
    d, k0, _, _, _ = _keys(C5, 15, seed=4)
    want = d.evaluate_until_words(0, [], d.create_evaluation_context(k0))
    n = 1 << d.hierarchy_to_tree(0)
    with K.forced_expand_depth(coop):
        for lo, hi in [(0, n), (1, n - 1), (1023, 1025), (2047, 2049), (3000, 3001),
                       (4097, 20000), (n - 300, n)]:
            got = _expand(K, cuda, d, k0, C5, lo, hi).cpu().numpy()
            _assert_host_layout_equals_words(C5, got, want[lo:hi], "[%d, %d)" % (lo, hi))


@pytest.mark.parametrize("ld", [12, 20, 21, 22, 25])
def test_automatic_cooperative_launch_matches_oracle(K, cuda, ld):
    """The automatic choice around the cooperative kernel: uint64 at
    log_domain_size 12 (2^11 tree leaves, two blocks) -> 1024-leaf blocks;
    20 (c1: 2^19 tree leaves), 21 and 22 (2^20, 2^21) -> 2048-leaf blocks;
    25 (2^24) -> KExpand<4>; every output against the oracle."""
    import torch
    spec = ("int", 64)
    d, k0, k1, alpha, beta = _keys(spec, ld, seed=19)
    for key in (k0, k1):
        want = d.evaluate_until_words(0, [], d.create_evaluation_context(key))
        got = _expand(K, cuda, d, key, spec).cpu().numpy()
        _assert_host_layout_equals_words(spec, got, want, "ld %d party %d" % (ld, key.party))
    torch.cuda.empty_cache()


ROOTS = [(C5, 25), (("int", 64), 26), (("xor", 128), 25)]


@pytest.mark.parametrize("spec,ld", ROOTS, ids=["%r-ld%d" % a for a in ROOTS])
def test_roots_stage_matches_oracle(K, cuda, spec, ld):
    """The roots stage of large KExpand<8> launches (kernels_capi.cc: the
    nodes six levels above the 256-leaf subtrees computed once by
    KExpandCoop<0, EmitNodes>, each thread walking six levels from there)
    forced on 2^25-tree-leaf domains — the whole domain and ragged ranges that
    start and end inside a subtree, a 64-subtree root group and a 1024-node
    block of the roots stage — both parties against the oracle."""
    import torch
    d, k0, k1, alpha, beta = _keys(spec, ld, seed=23)
    L = d.hierarchy_to_tree(0)
    assert L - 8 >= 17
    n = 1 << L
    ranges = [(1, n - 1), (255, 257), ((64 << 8) - 1, (3 * 64 << 8) + 5),
              ((1024 * 64 << 8) - 3, (1024 * 64 << 8) + 300), (12345, 12345 + (1 << 20) + 77),
              (n - 300, n)]
    with K.forced_expand_roots(1), K.forced_expand_depth(8):
        for key in (k0, k1):
            want = d.evaluate_until_words(0, [], d.create_evaluation_context(key))
            got = _expand(K, cuda, d, key, spec).cpu().numpy()
            _assert_host_layout_equals_words(spec, got, want, "ld %d party %d" % (ld, key.party))
            del got
            e = len(want) // n  # elements per tree leaf
            for lo, hi in ranges:
                got = _expand(K, cuda, d, key, spec, lo, hi).cpu().numpy()
                _assert_host_layout_equals_words(spec, got, want[lo * e:hi * e],
                                                 "party %d [%d, %d)" % (key.party, lo, hi))
            del want
    torch.cuda.empty_cache()


def test_forced_expand_roots_knob_validates():
    from distributed_point_functions_amd import kernels as K
    with pytest.raises(ValueError):
        with K.forced_expand_roots(2):
            pass


def test_forced_depth_knob_validates():
    from distributed_point_functions_amd import kernels as K
    with pytest.raises(ValueError):
        with K.forced_expand_depth(3):
            pass


# ---------------------------------------------------------------------------
# The automatic choice at the sizes where it selects D = 4 and D = 8
# ---------------------------------------------------------------------------

AUTO = [  # (spec, log_domain) -> tree levels L; KExpandCoop at L = 20 / 24, KExpand<8> at L = 25
    (C5, 20), (C5, 25),
    (("int", 64), 21), (("int", 64), 25), (("int", 64), 26),
    (("xor", 128), 20), (("xor", 128), 25),
]


@pytest.mark.parametrize("spec,ld", AUTO, ids=["%r-ld%d" % a for a in AUTO])
def test_production_depth_full_domain_matches_oracle(K, cuda, spec, ld):
    import torch
    d, k0, k1, alpha, beta = _keys(spec, ld, seed=11)
    L = d.hierarchy_to_tree(0)
    assert L in (20, 24, 25)
    for key in (k0, k1):
        want = d.evaluate_until_words(0, [], d.create_evaluation_context(key))
        got = _expand(K, cuda, d, key, spec).cpu().numpy()
        _assert_host_layout_equals_words(spec, got, want, "ld %d party %d" % (ld, key.party))
        del got, want
    torch.cuda.empty_cache()


# ---------------------------------------------------------------------------
# c5 at full size: log_domain_size 32, both parties, 2 x 64 GiB in HBM
# ---------------------------------------------------------------------------

@pytest.fixture(scope="module")
def c5_full(K, cuda):
    import torch
    d, k0, k1, alpha, beta = _keys(C5, 32, seed=5)
    assert d.hierarchy_to_tree(0) == 32
    n = 1 << 32
    outs = []
    for key in (k0, k1):
        out = torch.empty(n * 16, dtype=torch.uint8, device=cuda)
        _expand(K, cuda, d, key, C5, out=out)
        outs.append(out)
    torch.cuda.synchronize()
    yield dict(d=d, keys=(k0, k1), alpha=alpha, beta=beta, outs=outs, n=n)
    outs.clear()
    torch.cuda.empty_cache()


def test_c5_full_domain_share_sum_on_device(c5_full):
    """out0 + out1 == beta at alpha and 0 at every other of the 2^32 leaves
    (u32 wraps mod 2^32, IntModN adds mod p = 2^64 - 59).

    This is an alpha-path check: off the path both parties hold the same seed
    and control bit (cc:196-209), so any deterministic function of the seed
    sums to 0 there after party 1's negation.  The bit-exact pin of every
    leaf is test_c5_full_domain_every_subtree_digest_matches_oracle."""
    import torch
    n, alpha = c5_full["n"], c5_full["alpha"]
    a = c5_full["outs"][0].view(torch.int64).view(-1, 2)
    b = c5_full["outs"][1].view(torch.int64).view(-1, 2)
    chunk = 1 << 27
    nonzero = []
    for c0 in range(0, n, chunk):
        x, y = a[c0:c0 + chunk], b[c0:c0 + chunk]
        # IntModN share in word 0 (< p < 2^64): a + b in {0, p}; p = -59 as int64
        s1 = x[:, 0] + y[:, 0]
        zero1 = (s1 == -59) | ((x[:, 0] == 0) & (y[:, 0] == 0))
        zero0 = ((x[:, 1] + y[:, 1]) & 0xFFFFFFFF) == 0
        idx = torch.nonzero(~(zero0 & zero1)).flatten()
        nonzero += [c0 + int(i) for i in idx[:8].cpu()]
        # the u32 slot's padding word stays zero, the IntModN share is < p
        assert not bool(((x[:, 1] >> 32) != 0).any()), c0
        assert not bool((((x[:, 0] < 0) & (x[:, 0] >= -59))).any()), c0
    assert nonzero == [alpha]
    xa = [int(v) & 0xFFFFFFFFFFFFFFFF for v in a[alpha].cpu()]
    xb = [int(v) & 0xFFFFFFFFFFFFFFFF for v in b[alpha].cpu()]
    beta0, beta1 = c5_full["beta"]
    assert (xa[1] + xb[1]) % (1 << 32) == beta0
    assert (xa[0] + xb[0]) % P64 == beta1


def _device_subtree_sha256(out, log_sub=20, subs_per_chunk=64, workers=16):
    """SHA-256 of every 2^log_sub-leaf (16 B/leaf) slice of a device buffer:
    1 GiB chunks copied into two pinned host buffers on a side stream (the
    copy of chunk c + 1 overlaps the hashing of chunk c), each chunk's
    16 MiB slices hashed by a thread pool (hashlib releases the GIL)."""
    import concurrent.futures as cf
    import hashlib
    import torch
    sub = 16 << log_sub
    chunk = sub * subs_per_chunk
    total = out.numel()
    assert total % chunk == 0
    nchunks = total // chunk
    bufs = [torch.empty(chunk, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    views = [memoryview(b.numpy()) for b in bufs]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    done = [torch.cuda.Event(), torch.cuda.Event()]

    def issue(c):
        with torch.cuda.stream(side):
            bufs[c % 2].copy_(out[c * chunk:(c + 1) * chunk], non_blocking=True)
            done[c % 2].record(side)

    digests = []
    with cf.ThreadPoolExecutor(workers) as ex:
        issue(0)
        for c in range(nchunks):
            done[c % 2].synchronize()
            if c + 1 < nchunks:
                issue(c + 1)  # the other buffer: its hashes finished last iteration
            v = views[c % 2]
            digests += list(ex.map(lambda i: hashlib.sha256(v[i * sub:(i + 1) * sub]).hexdigest(),
                                   range(subs_per_chunk)))
    return digests


def test_c5_full_domain_every_subtree_digest_matches_oracle(c5_full):
    """Bit-exact parity of all 2 x 2^32 leaf values of the headline launch:
    the SHA-256 of each 2^20-leaf subtree of both parties' device output
    (host layout) equals the oracle's (tests/golden/c5_subtree_digests.json,
    written by tests/golden/make_c5_digests.py from oracle/dpf_oracle.c for
    this same key: ExpandSeeds cc:289-372, HashExpandedSeeds cc:523-547, the
    correction loop h:846-862)."""
    import json
    import os
    import time
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                        "c5_subtree_digests.json")
    with open(path) as f:
        gold = json.load(f)
    d, k0, k1, alpha, beta = _keys(C5, 32, seed=5)
    assert (gold["alpha"], tuple(gold["beta"])) == (alpha, tuple(beta))
    assert gold["log_subtree_leaves"] == 20
    for party in (0, 1):
        t0 = time.time()
        got = _device_subtree_sha256(c5_full["outs"][party])
        want = gold["sha256"][str(party)]
        assert len(got) == len(want) == 4096
        bad = [i for i in range(4096) if got[i] != want[i]]
        print("party %d: 4096 subtree digests in %.1f s, %d differ" %
              (party, time.time() - t0, len(bad)))
        assert not bad, "party %d: %d of 4096 subtrees differ from the oracle (first %s)" % (
            party, len(bad), bad[:8])


def test_c5_full_domain_sampled_subtrees_match_oracle(c5_full):
    """First, last, alpha's and 5 seeded random 2^20-leaf subtrees of both
    parties' 2^32-leaf launches equal the oracle's expansion bit for bit."""
    d, alpha = c5_full["d"], c5_full["alpha"]
    log_blocks = 20
    nsub = c5_full["n"] >> log_blocks
    rng = random.Random(2032)
    subs = sorted({0, nsub - 1, alpha >> log_blocks} | {rng.randrange(nsub) for _ in range(5)})
    for party, key in enumerate(c5_full["keys"]):
        out = c5_full["outs"][party]
        for s in subs:
            first = s << log_blocks
            want = d.expand_subtree_words(key, first, log_blocks).reshape(-1, 2, 2)
            got = out[first * 16:(first + (1 << log_blocks)) * 16].cpu().numpy()
            _assert_host_layout_equals_words(C5, got, want, "party %d subtree %d" % (party, s))


def test_c5_leaf_ranges_above_2_31_equal_full_launch(K, cuda, c5_full):
    """Leaf-range launches (the sharded entry) beginning past 2^31 produce
    exactly the corresponding slice of the full launch; one is also checked
    against the oracle."""
    import torch
    d, key = c5_full["d"], c5_full["keys"][0]
    full = c5_full["outs"][0]
    rng = random.Random(31)
    ranges = [((1 << 31) + 12345, (1 << 31) + 12345 + (1 << 21) + 7),
              ((1 << 32) - (1 << 22) - 1, 1 << 32),
              ((1 << 31), (1 << 31) + 1)]
    for _ in range(2):
        lo = (1 << 31) + rng.randrange(1 << 30)
        ranges.append((lo, lo + rng.randrange(1, 1 << 22)))
    for lo, hi in ranges:
        got = _expand(K, cuda, d, key, C5, lo, hi)
        assert torch.equal(got, full[lo * 16:hi * 16]), (lo, hi)
    lo, hi = ranges[0]
    first = lo >> 20 << 20
    want = d.expand_subtree_words(key, first, 22).reshape(-1, 2, 2)[lo - first:hi - first]
    got = _expand(K, cuda, d, key, C5, lo, hi).cpu().numpy()
    _assert_host_layout_equals_words(C5, got, want, "range above 2^31")


def test_c5_eight_rank_split_reproduces_one_rank(K, cuda, c5_full):
    """bench.py's N = 8 split (sharding.block_range over 2^32 tree blocks),
    each rank's launch run in turn on this GPU into its slice of one buffer,
    equals the single-rank output byte for byte."""
    import torch
    from distributed_point_functions_amd import sharding
    d, key, n = c5_full["d"], c5_full["keys"][0], c5_full["n"]
    full = c5_full["outs"][0]
    # reuse party 1's buffer (its checks ran first in this module)
    buf = c5_full["outs"][1]
    for world in (8, 3):
        for rank in range(world):
            lo, hi = sharding.block_range(n, world, rank)
            _expand(K, cuda, d, key, C5, lo, hi, out=buf[lo * 16:hi * 16])
        assert _chunked_equal(buf, full), world


@pytest.mark.parametrize("variant", [0, 2, 4, 5, 6, 8, -1, -2, -3])
@pytest.mark.parametrize("spec,ld", [(("xor", 128), 14), (("int", 64), 15), (("int", 32), 16),
                                     (("int", 8), 18), (C5, 13)])
def test_batched_keys_match_oracle(K, cuda, spec, ld, variant):
    """dpf_amd_expand_and_correct_batched: several keys (both parties mixed,
    different alphas / betas) in one grid — KExpand with per-lane keys or
    KExpandCoop with per-block keys — on a ragged leaf range, every output
    against the oracle (C5 takes the per-key path)."""
    from distributed_point_functions_amd import value_types as vtm
    import torch
    ks = [_keys(spec, ld, seed=100 + i) for i in range(5)]
    keys = [(d, k0 if i % 2 else k1) for i, (d, k0, k1, _, _) in enumerate(ks)]
    d0 = keys[0][0]
    L = d0.hierarchy_to_tree(0)
    if variant > L or (variant < 0 and L < 10 - variant - 1):
        pytest.skip("variant needs more tree levels")
    n = 1 << L
    lo, hi = (3, n - 5) if n > 64 else (0, n)
    cepb = 1 << (ld - L)
    arrs = [_key_arrays(K, cuda, d, k) for d, k in keys]
    vt = vtm.from_spec(spec)
    with K.forced_expand_depth(variant):
        got = K.expand_and_correct_batched(
            torch.cat([a["seed"] for a in arrs]), torch.cat([a["cb"] for a in arrs]), L,
            torch.cat([a["cw"] for a in arrs]), torch.cat([a["ccl"] for a in arrs]),
            torch.cat([a["ccr"] for a in arrs]), vt.descriptor(d0.blocks_needed(0)),
            [a["corr"] for a in arrs], [a["party"] for a in arrs], cepb, lo, hi).cpu().numpy()
    per = (hi - lo) * cepb * vt.descriptor(d0.blocks_needed(0)).out_stride
    for i, (d, k) in enumerate(keys):
        want = d.evaluate_until_words(0, [], d.create_evaluation_context(k))
        _assert_host_layout_equals_words(spec, got[i * per:(i + 1) * per],
                                         want[lo * cepb:hi * cepb], "key %d" % i)
