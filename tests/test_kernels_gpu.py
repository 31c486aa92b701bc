"""GPU parity of the Tier-1 device seams against the CPU oracle.

Every test runs a HIP kernel through the C ABI (include/dpf_amd.h) and
compares bit-exactly with oracle/ (the C restatement of the reference).
Inputs follow the reference's own tests where they exist:
  - AES-MMO KAT: dpf/aes_128_fixed_key_hash_test.cc:120-141
  - EvaluateSeeds inputs: dpf/internal/evaluate_prg_hwy_test.cc:50-93, 183-205
  - share-sum / EvaluateAt: dpf/distributed_point_function_test.cc:1015-1079
"""
import random

import numpy as np
import pytest

from oracle import pyoracle as po

pytestmark = pytest.mark.gpu

M64 = (1 << 64) - 1
KEY0 = 0
KEY1 = (0x1111111111111111 << 64) | 0x1111111111111111
SEED0 = (0x0123012301230123 << 64) | 0x0123012301230123
SEED1 = (0x4567456745674567 << 64) | 0x4567456745674567
P64 = 18446744073709551557  # 2**64 - 59
P32 = 4294967291  # 2**32 - 5
P80 = (65535 << 64) | 18446744073709551551  # 2**80 - 65


@pytest.fixture(scope="module")
def K(cuda):
    from distributed_point_functions_amd import kernels
    return kernels


def u8(a, cuda):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint8)).to(cuda)


def test_aes_mmo_known_answers(K, cuda):
    blocks = K.u128_tensor([SEED0, SEED1], cuda)
    out0 = K.tensor_u128(K.aes128_mmo(KEY0, blocks))
    out1 = K.tensor_u128(K.aes128_mmo(KEY1, blocks))
    assert out0 == [(0x73c2dc14812be4ef << 64) | 0xeac64d09c8adf8ed,
                    (0xb8f33653a53a8436 << 64) | 0xaedf39b62de91d95]
    assert out1 == [(0x934704aff58fa233 << 64) | 0xd3c20d1b9cc18d8f,
                    (0x530098817046d284 << 64) | 0x43e61d3273a04f7c]


def test_aes_mmo_random_matches_oracle(K, cuda):
    rng = random.Random(7)
    blocks = [rng.getrandbits(128) for _ in range(20000)]
    key = rng.getrandbits(128)
    got = K.tensor_u128(K.aes128_mmo(key, K.u128_tensor(blocks, cuda)))
    assert got == po.aes_mmo(key, blocks)


@pytest.mark.parametrize("num_seeds", [1, 2, 101, 128, 1000])
@pytest.mark.parametrize("num_levels", [1, 2, 32, 63, 64, 127, 128])
@pytest.mark.parametrize("per_seed_cw", [False, True])
def test_evaluate_seeds_matches_oracle(K, cuda, num_seeds, num_levels, per_seed_cw):
    # Inputs of evaluate_prg_hwy_test.cc:60-93.
    seeds = [(i << 64) | (i + 1) for i in range(num_seeds)]
    paths = [((23 * i + 42) << 64) | (42 * i + 23) for i in range(num_seeds)]
    cbs = [1 if i % 7 == 0 else 0 for i in range(num_seeds)]
    ncw = num_levels * num_seeds if per_seed_cw else num_levels
    cws = [((i + 1) << 64) | i for i in range(ncw)]
    ccl = [1 if i % 23 == 0 else 0 for i in range(ncw)]
    ccr = [1 if i % 42 != 0 else 0 for i in range(ncw)]
    want_s, want_c = po.evaluate_seeds(seeds, cbs, paths, 0, cws, ccl, ccr, KEY0, KEY1,
                                       num_levels)
    so, co = K.evaluate_seeds(K.u128_tensor(seeds, cuda), u8(cbs, cuda),
                              K.u128_tensor(paths, cuda), 0, K.u128_tensor(cws, cuda),
                              u8(ccl, cuda), u8(ccr, cuda), KEY0, KEY1, num_levels)
    assert K.tensor_u128(so) == want_s
    assert [int(x) for x in co.cpu().numpy()] == want_c


@pytest.mark.parametrize("rightshift", [0, 1, 5, 63, 64, 100, 127, 128])
def test_evaluate_seeds_rightshift(K, cuda, rightshift):
    num_seeds, num_levels = 101, 128
    seeds = [(i << 64) | (i + 1) for i in range(num_seeds)]
    paths = [((23 * i + 42) << 64) | (42 * i + 23) for i in range(num_seeds)]
    cbs = [1 if i % 7 == 0 else 0 for i in range(num_seeds)]
    cws = [((i + 1) << 64) | i for i in range(num_levels)]
    ccl = [1 if i % 23 == 0 else 0 for i in range(num_levels)]
    ccr = [1 if i % 42 != 0 else 0 for i in range(num_levels)]
    want = po.evaluate_seeds(seeds, cbs, paths, rightshift, cws, ccl, ccr, KEY0, KEY1,
                             num_levels)
    so, co = K.evaluate_seeds(K.u128_tensor(seeds, cuda), u8(cbs, cuda),
                              K.u128_tensor(paths, cuda), rightshift,
                              K.u128_tensor(cws, cuda), u8(ccl, cuda), u8(ccr, cuda),
                              KEY0, KEY1, num_levels)
    assert (K.tensor_u128(so), [int(x) for x in co.cpu().numpy()]) == want


# The DPF's own PRG keys (distributed_point_function.cc:55-60): launches of up
# to 2^16 seeds with these keys run the four-lanes-per-seed walk
# (KEvaluatePointsQuad without the value hash).
# (per-seed correction words of 2^16 seeds x 63+ levels are left out: the
# oracle's time, not the kernel's)
SEEDS_CASES = [(n, lv, per) for n in (1, 101, 1000, 1 << 16) for lv in (1, 8, 63, 128)
               for per in (False, True) if not (per and n * lv > 1 << 20)]


@pytest.mark.parametrize("num_seeds,num_levels,per_seed_cw", SEEDS_CASES)
@pytest.mark.parametrize("walk", [0, 1, 2], ids=["auto", "quad", "lane"])
def test_evaluate_seeds_dpf_keys_every_walk(K, cuda, num_seeds, num_levels, per_seed_cw, walk):
    kl = (0x5be037ccf6a03de5 << 64) | 0x935f08d0a5b6a2fd
    kr = (0xef94b6aedebb026c << 64) | 0xe2ea1fe0f66f4d0b
    rng = np.random.default_rng(num_seeds * 131 + num_levels)
    seeds = [int(a) << 64 | int(b) for a, b in rng.integers(0, 1 << 63, (num_seeds, 2))]
    paths = [int(a) << 64 | int(b) for a, b in rng.integers(0, 1 << 63, (num_seeds, 2))]
    cbs = [int(x) for x in rng.integers(0, 2, num_seeds)]
    ncw = num_levels * num_seeds if per_seed_cw else num_levels
    cws = [int(a) << 64 | int(b) for a, b in rng.integers(0, 1 << 63, (ncw, 2))]
    ccl = [int(x) for x in rng.integers(0, 2, ncw)]
    ccr = [int(x) for x in rng.integers(0, 2, ncw)]
    for rs in (0, 3):
        want = po.evaluate_seeds(seeds, cbs, paths, rs, cws, ccl, ccr, kl, kr, num_levels)
        with K.forced_walk_mode(walk):
            s_in = K.u128_tensor(seeds, cuda)
            c_in = u8(cbs, cuda)
            so, co = K.evaluate_seeds(s_in, c_in, K.u128_tensor(paths, cuda), rs,
                                      K.u128_tensor(cws, cuda), u8(ccl, cuda), u8(ccr, cuda),
                                      kl, kr, num_levels)
            # in place, as the heavy-hitters level walks its prefixes
            K.evaluate_seeds(s_in, c_in, K.u128_tensor(paths, cuda), rs,
                             K.u128_tensor(cws, cuda), u8(ccl, cuda), u8(ccr, cuda), kl, kr,
                             num_levels, seeds_out=s_in, control_bits_out=c_in)
        got = (K.tensor_u128(so), [int(x) for x in co.cpu().numpy()])
        assert got == want
        assert (K.tensor_u128(s_in), [int(x) for x in c_in.cpu().numpy()]) == want


def test_evaluate_seeds_rejects_bad_correction_word_count(K, cuda):
    from distributed_point_functions_amd._lib import DpfAmdError
    s = K.u128_tensor([1] * 1000, cuda)
    c = u8([0] * 1000, cuda)
    with pytest.raises(DpfAmdError) as e:
        K.evaluate_seeds(s, c, s, 0, K.u128_tensor([0] * 12, cuda), u8([0] * 12, cuda),
                         u8([0] * 12, cuda), KEY0, KEY1, 10)
    assert e.value.code == 3
    assert "num_correction_words" in e.value.message


# ---------------------------------------------------------------------------
# Fused expansion vs oracle EvaluateUntil
# ---------------------------------------------------------------------------

TYPES = [
    ("int", 8), ("int", 16), ("int", 32), ("int", 64), ("int", 128),
    ("xor", 8), ("xor", 128),
    ("tuple", [("int", 32), ("int", 32)]),
    ("tuple", [("int", 32), ("int", 64)]),
    ("tuple", [("int", 8), ("int", 16), ("int", 32), ("int", 64)]),
    ("tuple", [("int", 32), ("tuple", [("int", 32), ("int", 32)]), ("int", 32)]),
    ("tuple", [("int", 32), ("int", 128)]),
    ("intmodn", 32, P32),
    ("tuple", [("int", 32), ("intmodn", 32, P32)]),
    ("tuple", [("int", 128), ("intmodn", 32, P32)]),
    ("tuple", [("intmodn", 32, P32)] * 5),
    ("tuple", [("intmodn", 64, P64)] * 2),
    ("tuple", [("int", 32), ("intmodn", 64, P64)]),
    ("tuple", [("intmodn", 128, P80)] * 2),
    ("tuple", [("xor", 32), ("int", 128)]),
    ("intmodn", 64, 1000000000000),
]


def _keys(spec, ld, sec=48, alpha=None, seed=1):
    rng = random.Random(seed * 1000 + ld)
    d = po.Dpf([(ld, spec, sec)])
    vt = po.scalar_specs(spec)
    beta_flat = []
    for s in vt:
        if s[0] == "intmodn":
            beta_flat.append(rng.randrange(s[2]))
        else:
            beta_flat.append(rng.getrandbits(s[1]))
    beta = po.unflatten(spec, beta_flat)
    if alpha is None:
        alpha = rng.randrange(1 << ld) if ld < 128 else rng.getrandbits(128)
    k0, k1 = d.generate_keys(alpha, [beta], seeds=(rng.getrandbits(128), rng.getrandbits(128)))
    return d, k0, k1, alpha, beta


def _expand_gpu(K, cuda, d, key, spec, leaf_begin=0, leaf_end=None):
    from distributed_point_functions_amd import value_types as vtm
    vt = vtm.from_spec(spec)
    L = d.hierarchy_to_tree(0)
    desc = vt.descriptor(d.blocks_needed(0))
    cepb = 1 << (d.levels[0][0] - L)
    out = K.expand_and_correct(
        K.u128_tensor([key.seed], cuda), u8([key.party], cuda), L,
        K.u128_tensor(key.cw_seeds()[:L] or [0], cuda), u8(key.ccl()[:L] or [0], cuda),
        u8(key.ccr()[:L] or [0], cuda), desc, key.value_corrections()[0], key.party, cepb,
        leaf_begin, leaf_end)
    arr = out.cpu().numpy().view(vt.numpy_dtype())
    return vt.decode_flat(arr)


@pytest.mark.parametrize("spec", TYPES, ids=[repr(t) for t in TYPES])
@pytest.mark.parametrize("ld", [0, 1, 5, 10])
def test_expand_matches_oracle(K, cuda, spec, ld):
    d, k0, k1, alpha, beta = _keys(spec, ld)
    for key in (k0, k1):
        want = d.evaluate_until(0, [], d.create_evaluation_context(key))
        got = _expand_gpu(K, cuda, d, key, spec)
        assert got == want


@pytest.mark.parametrize("spec", [("int", 64), ("tuple", [("int", 32), ("intmodn", 64, P64)]),
                                  ("xor", 128), ("int", 8)])
def test_expand_large_domain_and_share_sum(K, cuda, spec):
    from distributed_point_functions_amd import value_types as vtm
    ld = 17
    d, k0, k1, alpha, beta = _keys(spec, ld)
    vt = vtm.from_spec(spec)
    a = _expand_gpu(K, cuda, d, k0, spec)
    b = _expand_gpu(K, cuda, d, k1, spec)
    assert len(a) == 1 << ld
    fb = po.flatten_value(spec, beta)
    for i in range(len(a)):
        s = vt.flatten(vt.add(vt.unflatten(iter(a[i])), vt.unflatten(iter(b[i]))))
        assert s == (fb if i == alpha else [0] * len(fb)), i
    # and bit-exact against the oracle for party 0
    want = d.evaluate_until(0, [], d.create_evaluation_context(k0))
    assert a == want


def test_expand_leaf_ranges(K, cuda):
    spec = ("tuple", [("int", 32), ("intmodn", 64, P64)])
    d, k0, _, _, _ = _keys(spec, 14)
    want = d.evaluate_until(0, [], d.create_evaluation_context(k0))
    L = d.hierarchy_to_tree(0)
    n = 1 << L
    for lo, hi in [(0, n), (3, 1000), (256, 512), (n - 17, n), (5000, 5001), (0, 1)]:
        got = _expand_gpu(K, cuda, d, k0, spec, lo, hi)
        assert got == want[lo:hi], (lo, hi)


# ---------------------------------------------------------------------------
# Fused point evaluation vs oracle EvaluateAt
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("spec", TYPES[:12] + [TYPES[13], TYPES[17]],
                         ids=[repr(t) for t in TYPES[:12] + [TYPES[13], TYPES[17]]])
@pytest.mark.parametrize("ld", [0, 1, 2, 32, 128])
@pytest.mark.parametrize("walk", [1, 2], ids=["quad", "lane"])
def test_evaluate_points_matches_oracle(K, cuda, spec, ld, walk):
    """Both point-walk kernels (four lanes per point / one lane per point;
    value types of more than 256 bits always take the latter)."""
    from distributed_point_functions_amd import value_types as vtm
    d, k0, k1, alpha, beta = _keys(spec, ld)
    vt = vtm.from_spec(spec)
    rng = random.Random(ld)
    maxp = (1 << ld) - 1
    pts = [i & maxp for i in range(40)] + [rng.getrandbits(128) & maxp for _ in range(60)]
    pts.append(alpha)
    L = d.hierarchy_to_tree(0)
    epb = d.elements_per_block(0)
    bbits = ld - L
    for key in (k0, k1):
        want = d.evaluate_at(key, 0, pts)
        tree = [p >> bbits if epb > 1 else p for p in pts]
        bi = [p & ((1 << bbits) - 1) if epb > 1 else 0 for p in pts]
        n = len(pts)
        with K.forced_walk_mode(walk):
            out = K.evaluate_points(
                K.u128_tensor([key.seed] * n, cuda), u8([key.party] * n, cuda),
                K.u128_tensor(tree, cuda), 0, L, K.u128_tensor(key.cw_seeds()[:L], cuda),
                u8(key.ccl()[:L], cuda), u8(key.ccr()[:L], cuda),
                vt.descriptor(d.blocks_needed(0)), block_index=u8(bi, cuda),
                party_all=key.party, value_correction_all=key.value_corrections()[0])
        got = vt.decode_flat(out.cpu().numpy().view(vt.numpy_dtype()))
        assert got == want


@pytest.mark.parametrize("spec", [TYPES[0], TYPES[3], TYPES[4], TYPES[13], TYPES[17]],
                         ids=[repr(t) for t in (TYPES[0], TYPES[3], TYPES[4], TYPES[13],
                                                TYPES[17])])
@pytest.mark.parametrize("ld,nkeys,ppk", [(1, 3, 5), (32, 7, 37), (128, 4, 129),
                                          (20, 5, 70001)])
@pytest.mark.parametrize("walk", [0, 1, 2], ids=["auto", "quad", "lane"])
def test_evaluate_points_batched_matches_oracle(K, cuda, spec, ld, nkeys, ppk, walk):
    """One launch over several keys (alternating parties) == the oracle's
    per-key EvaluateAt.  The last case has > 2^18 points, so threads walk two
    points each (the i / i + T pairing)."""
    from distributed_point_functions_amd import value_types as vtm
    vt = vtm.from_spec(spec)
    rng = random.Random(ld * 31 + nkeys)
    keys = []
    for k in range(nkeys):
        d, k0, k1, alpha, beta = _keys(spec, ld, seed=k + 2)
        keys.append((d, (k0, k1)[k % 2], alpha))
    d = keys[0][0]
    L = d.hierarchy_to_tree(0)
    epb = d.elements_per_block(0)
    bbits = ld - L
    maxp = (1 << ld) - 1
    pts = []
    for k in range(nkeys):
        p = [rng.getrandbits(128) & maxp for _ in range(ppk)]
        p[0] = keys[k][2]
        pts.append(p)
    flat = [p for ps in pts for p in ps]
    tree = [p >> bbits if epb > 1 else p for p in flat]
    bi = [p & ((1 << bbits) - 1) if epb > 1 else 0 for p in flat]
    ks = [k for _, k, _ in keys]
    cws = [c for k in ks for c in (k.cw_seeds()[:L] or [0])]
    ccl = [c for k in ks for c in (k.ccl()[:L] or [0])]
    ccr = [c for k in ks for c in (k.ccr()[:L] or [0])]
    import torch
    with K.forced_walk_mode(walk):
        out = K.evaluate_points_batched(
            nkeys, ppk, K.u128_tensor([k.seed for k in ks], cuda),
            u8([k.party for k in ks], cuda), K.u128_tensor(tree, cuda), 0, L,
            K.u128_tensor(cws, cuda), u8(ccl, cuda), u8(ccr, cuda),
            vt.descriptor(d.blocks_needed(0)), block_index=u8(bi, cuda),
            key_party=torch.tensor([k.party for k in ks], dtype=torch.int8, device=cuda),
            key_value_corrections=K.u128_tensor(
                [c for k in ks for c in k.value_corrections()[0]], cuda))
    got = vt.decode_flat(out.cpu().numpy().view(vt.numpy_dtype()))
    step = max(1, ppk // 300)
    for k in range(nkeys):
        sample = list(range(0, ppk, step)) + [ppk - 1]
        # keys of one spec/ld share parameters, so any key's Dpf evaluates
        want = keys[k][0].evaluate_at(ks[k], 0, [pts[k][j] for j in sample])
        assert [got[k * ppk + j] for j in sample] == want, k


@pytest.mark.parametrize("ld,nkeys,ppk", [(7, 3, 128), (21, 15, 12288), (12, 2, 1000)])
def test_evaluate_points_batched_implicit_paths(K, cuda, ld, nkeys, ppk):
    """paths = NULL walks point j of every key to tree index j (the batched
    PIR selection expansion): equal to explicit paths, and to the oracle's
    full-domain expansion of each key's first ppk leaves."""
    import torch
    spec = ("xor", 128)
    from distributed_point_functions_amd import value_types as vtm
    vt = vtm.from_spec(spec)
    keys = []
    for k in range(nkeys):
        d, k0, k1, _, _ = _keys(spec, ld, seed=k + 40)
        keys.append((d, (k0, k1)[k % 2]))
    d = keys[0][0]
    L = d.hierarchy_to_tree(0)
    ks = [k for _, k in keys]
    args = (K.u128_tensor([k.seed for k in ks], cuda), u8([k.party for k in ks], cuda))
    rest = dict(key_party=torch.tensor([k.party for k in ks], dtype=torch.int8, device=cuda),
                key_value_corrections=K.u128_tensor(
                    [c for k in ks for c in k.value_corrections()[0]], cuda))
    cw = (K.u128_tensor([c for k in ks for c in (k.cw_seeds()[:L] or [0])], cuda),
          u8([c for k in ks for c in (k.ccl()[:L] or [0])], cuda),
          u8([c for k in ks for c in (k.ccr()[:L] or [0])], cuda))
    desc = vt.descriptor(d.blocks_needed(0))
    implicit = K.evaluate_points_batched(nkeys, ppk, *args, None, 0, L, *cw, desc, **rest)
    explicit = K.evaluate_points_batched(nkeys, ppk, *args,
                                         K.u128_tensor(list(range(ppk)) * nkeys, cuda), 0, L,
                                         *cw, desc, **rest)
    assert torch.equal(implicit, explicit)
    for walk in (1, 2):  # both point-walk kernels
        with K.forced_walk_mode(walk):
            other = K.evaluate_points_batched(nkeys, ppk, *args, None, 0, L, *cw, desc, **rest)
        assert torch.equal(implicit, other), walk
    got = implicit.cpu().numpy().view(np.uint64).reshape(nkeys, ppk, 2)
    for k in (0, nkeys - 1):
        full = keys[k][0].expand_subtree_words(ks[k], 0, L)
        assert np.array_equal(got[k], full.reshape(-1, 2)[:ppk]), k


@pytest.mark.parametrize("stride,opp", [(1, 32), (2, 8), (4, 4), (8, 256), (8, 3), (16, 5),
                                        (24, 7), (32, 64), (12, 4)])
def test_gather_rows(K, cuda, stride, opp):
    """Per-prefix slice gather (h:877-889) on 16-byte and byte paths, with
    aligned and unaligned row offsets."""
    import torch
    rng = np.random.default_rng(stride * 100 + opp)
    total_rows = 4096
    rows = rng.integers(0, 256, size=total_rows * stride, dtype=np.uint8)
    n = 300
    src = rng.integers(0, total_rows - opp, size=n).astype(np.int64)
    src[::3] = (src[::3] // opp) * opp  # EvaluateUntil's offsets are multiples of opp
    got = K.gather_rows(torch.from_numpy(src).to(cuda), opp, stride,
                        torch.from_numpy(rows).to(cuda)).cpu().numpy()
    r2 = rows.reshape(total_rows, stride)
    want = np.concatenate([r2[s:s + opp].reshape(-1) for s in src])
    assert np.array_equal(got, want)


# ---------------------------------------------------------------------------
# Dense PIR scan vs oracle InnerProduct
# ---------------------------------------------------------------------------

SCAN_CASES = [(1, 16, 1), (1000, 256, 1), (1000, 256, 3), (4096, 80, 8), (300, 17, 2),
              (777, 1104, 5), (129, 4096, 1), (5000, 64, 11),
              # many-query passes: Four-Russians P = 4 / 2 / 1 (16 / 32 / 64
              # queries per pass), ragged tiles, several 256-B slices, a
              # narrow last slice (1104 B = 4 x 256 + 80), 100 queries
              (1000, 256, 17), (3001, 256, 32), (4097, 512, 33), (130, 256, 64),
              (2500, 768, 100), (2049, 1104, 40), (640, 240, 16), (385, 64, 9),
              # 49-64 queries in one P = 1 pass (the fourth lane group in use)
              (3001, 256, 49), (2049, 1104, 57),
              # 9-15 queries: the Four-Russians scan from 9 on (P = 4)
              (3000, 256, 12), (2001, 1104, 15), (1500, 256, 10),
              # >= 64 scan blocks with a partial of <= 2 KiB: the masked scan
              # XORs block partials into 64 atomic fold slots (ragged last
              # tile, two 64-chunk slices at 1104 B, Q x 256 B = 2 KiB)
              (40000, 256, 1), (33001, 48, 3), (36001, 1104, 1), (50000, 256, 8),
              (40000, 16, 5)]


def _scan_case(K, cuda, n, size, q, mode, skip=0):
    import torch
    rng = np.random.default_rng(n * 7 + size)
    stride = (size + 15) // 16 * 16
    recs = rng.integers(0, 256, size=(n, size), dtype=np.uint8)
    db = np.zeros((n, stride), dtype=np.uint8)
    db[:, :size] = recs
    blocks = (n + 127) // 128 + 1
    # full-range words: every selection bit position (incl. 63 / 127) is exercised
    sel_words = rng.integers(0, 2**64, size=(q * blocks, 2), dtype=np.uint64).view(np.int64)
    sels = [[(int(sel_words[k * blocks + i, 0]) & M64) | ((int(sel_words[k * blocks + i, 1]) & M64) << 64)
             for i in range(blocks)] for k in range(q)]
    want = po.inner_product([bytes(r) for r in recs], sels)
    with K.forced_scan_m4(mode), K.scan_skip_unselected(skip):
        out = K.inner_product(torch.from_numpy(db).to(cuda), n, stride,
                              torch.from_numpy(sel_words).to(cuda), q)
    got = out.cpu().numpy().reshape(q, stride)[:, :size]
    for k in range(q):
        assert bytes(got[k]) == want[k], k


@pytest.mark.parametrize("n,size,q", SCAN_CASES)
def test_inner_product_matches_oracle(K, cuda, n, size, q):
    """Automatic kernel choice (the production path)."""
    _scan_case(K, cuda, n, size, q, -1)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("n,size,q", SCAN_CASES)
def test_inner_product_each_scan_kernel(K, cuda, n, size, q, mode):
    """Masked scan (KPirScanG) and Four-Russians scan (KPirScanM4) forced on
    every shape, including the ones the automatic choice never gives them."""
    _scan_case(K, cuda, n, size, q, mode)


@pytest.mark.parametrize("n,size,q", SCAN_CASES)
def test_inner_product_skipping_unselected_records(K, cuda, n, size, q):
    """The opt-in scan that reads only the records a pass selects (the
    reference's skip, inner_product_hwy.cc:213-221) answers as the oracle on
    every shape, masked scan forced (the Four-Russians passes are unchanged)."""
    _scan_case(K, cuda, n, size, q, 0, skip=1)


def test_inner_product_skip_sparse_and_empty_selections(K, cuda):
    """Skipping with selections of a few bits and of none: only the selected
    rows reach the sums, an all-zero selection gives zeros."""
    import torch
    n, size = 5003, 272
    rng = np.random.default_rng(3)
    db = rng.integers(0, 256, size=(n, size), dtype=np.uint8)
    blocks = (n + 127) // 128
    picks = [[], [0], [n - 1], [5, 77, 4095, 4096, 5002]]
    sels = []
    for p in picks:
        v = [0] * blocks
        for r in p:
            v[r // 128] |= 1 << (r % 128)
        sels.append(v)
    words = np.array([[v & M64, v >> 64] for s in sels for v in s], dtype=np.uint64).view(np.int64)
    with K.forced_scan_m4(0), K.scan_skip_unselected(1):
        out = K.inner_product(torch.from_numpy(db.reshape(-1)).to(cuda), n, size,
                              torch.from_numpy(words).to(cuda), len(sels))
    got = out.cpu().numpy().reshape(len(sels), size)
    for k, p in enumerate(picks):
        want = np.zeros(size, np.uint8)
        for r in p:
            want ^= db[r]
        assert np.array_equal(got[k], want), p


def test_handle_request_with_scan_skip_reconstructs(K, cuda):
    """HandleRequest on this thread with the skip on: both parties' answers
    still XOR to the records (a plain server, 3 queries)."""
    from distributed_point_functions_amd import pir as P
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    n, size = 20000, 256
    rng = np.random.default_rng(11)
    recs = rng.integers(0, 256, size=(n, size), dtype=np.uint8)
    servers = []
    for _ in range(2):
        db = P.DenseDpfPirDatabase()
        db.insert_fixed(recs)
        servers.append(P.DenseDpfPirServer.create_plain(n, db))
    dpf = DistributedPointFunction.create(DpfParameters((n - 1).bit_length(), V.XorWrapper(128)))
    idx = [0, 12345, n - 1]
    pairs = P.client_keys(dpf, n, idx, seeds=[(1 + j, 50 + j) for j in range(3)])
    with K.scan_skip_unselected(1):
        r0 = P.parse_response(servers[0].handle_request(P.pir_request_plain([a for a, _ in pairs])))
        r1 = P.parse_response(servers[1].handle_request(P.pir_request_plain([b for _, b in pairs])))
    for j, i in enumerate(idx):
        assert bytes(x ^ y for x, y in zip(r0[j], r1[j])) == recs[i].tobytes()


def test_scan_skip_knob_validates():
    from distributed_point_functions_amd import kernels as K
    with pytest.raises(ValueError):
        with K.scan_skip_unselected(2):
            pass


@pytest.mark.parametrize("n,size,qs", [(1 << 22, 256, (16, 40, 64, 100)),
                                       (1 << 18, 1104, (33,)),
                                       # masked scan with atomic fold slots
                                       # vs the Four-Russians partials
                                       (1 << 22, 256, (1, 8)), (1 << 20, 1104, (1,))])
def test_scan_kernels_agree_large(K, cuda, n, size, qs):
    """Random full selections over millions of records: the Four-Russians
    scan equals the masked scan (each pinned to the oracle above) and repeats
    bit-identically.  Small cases cannot show a table row written to the wrong
    place at random (an add-TID store issued without its M0 wait state gave
    exactly that at 2^26 records)."""
    import torch
    stride = (size + 15) // 16 * 16
    gen = torch.Generator(device=cuda)
    gen.manual_seed(n + size)
    db = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device=cuda, generator=gen)
    blocks = (n + 127) // 128
    for q in qs:
        sel = torch.randint(-2**63, 2**63 - 1, (q * blocks, 2), dtype=torch.int64, device=cuda,
                            generator=gen)
        outs = []
        for mode in (0, 1, 1):
            with K.forced_scan_m4(mode):
                outs.append(K.inner_product(db, n, stride, sel, q).clone())
        assert torch.equal(outs[1], outs[2]), "Four-Russians scan not repeatable (q=%d)" % q
        assert torch.equal(outs[0], outs[1]), "Four-Russians scan != masked scan (q=%d)" % q
