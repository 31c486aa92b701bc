"""GPU parity of the incremental API paths the reference's IncrementalDpfTest
drives (dpf/distributed_point_function_test.cc:308-930): EvaluateAt with a
context (h:356-378, EvaluateAtImpl h:1000-1011) and EvaluateUntil calls that
jump several hierarchy levels at once (level_step 2/3/5/7, h:695-891 walking
hierarchy_to_tree[h] - hierarchy_to_tree[prev] levels from stored partial
evaluations).

Every instantiation of test.cc:698-930 runs through the C ABI
(dpf_amd_evaluate_at_ctx / dpf_amd_evaluate_until) next to the CPU oracle:
every output element of both parties, and the EvaluationContext each call
leaves behind (previous_hierarchy_level, partial_evaluations_level and the
ordered partial evaluations), must equal the oracle's; the reference's share
sums are checked on top (tests/incremental_cases.py).
"""
import numpy as np
import pytest

from oracle import pyoracle as po
from tests import incremental_cases as IC

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def api(cuda):
    from distributed_point_functions_amd import dpf, value_types
    return dpf, value_types


def _make(api, levels):
    D, V = api
    params = [D.DpfParameters(ld, V.from_spec(s), sec) for ld, s, sec in levels]
    return D.DistributedPointFunction.create_incremental(params)


def _words(arr, bits):
    """Host-layout output of a single-integer type -> (n, 2) {lo, hi}."""
    f = arr["f0"]
    if bits == 128:
        return np.ascontiguousarray(f, dtype=np.uint64).reshape(-1, 2)
    return np.stack([f.astype(np.uint64), np.zeros(len(f), np.uint64)], axis=1)


def _same_ctx(ctx, octx):
    assert ctx.previous_hierarchy_level == octx.previous_hierarchy_level
    assert ctx.partial_evaluations_level == octx.partial_evaluations_level
    got = ctx.partial_evaluations()
    want = [(p, s, bool(c)) for p, s, c in octx.partial_evaluations()]
    assert got == want


def _evaluator(dpf, od, hier, ctxs, octxs):
    def evaluate(h, prefixes, single_point):
        bits = hier[h][1]
        outs = []
        for ctx, octx in zip(ctxs, octxs):
            if single_point:
                got = _words(dpf.evaluate_at_ctx(h, prefixes, ctx, raw=True), bits)
                want = od.evaluate_at_ctx_words(h, prefixes, octx)[:, 0, :]
            else:
                got = _words(dpf.evaluate_until(h, prefixes, ctx, raw=True), bits)
                want = od.evaluate_until_words(h, prefixes, octx)[:, 0, :]
            assert got.shape == want.shape, h
            bad = np.nonzero((got != want).any(axis=1))[0]
            assert len(bad) == 0, (h, single_point, bad[:5])
            _same_ctx(ctx, octx)
            outs.append(got)
        return outs
    return evaluate


@pytest.fixture(params=[0, 1, 2], ids=["prefix_expand", "unique_expand_gather", "host_bookkeeping"])
def expand_mode(request, api):
    """EvaluateUntil's strategies for calls with prefixes
    (dpf_amd_set_prefix_expand): each prefix's subtree expanded straight into
    the output with the de-duplication, the context lookup and the context's
    list on the device (0) or on the host (2), or the unique tree indices
    expanded and gathered (1)."""
    from distributed_point_functions_amd import _lib
    L = _lib.lib()
    prev = L.dpf_amd_set_prefix_expand(request.param)
    yield request.param
    L.dpf_amd_set_prefix_expand(prev)


# (single_point, EvaluateUntil strategy): EvaluateAt does not expand, so it
# runs once, under the default strategy
CALL_MODES = [(False, 0), (False, 1), (False, 2), (True, 0)]


@pytest.mark.parametrize("single_point,mode", CALL_MODES,
                         ids=["until-prefix_expand", "until-unique_expand_gather",
                              "until-host_bookkeeping", "at"])
@pytest.mark.parametrize("suite", IC.SUITES, ids=[s[0] for s in IC.SUITES])
def test_incremental_dpf_correctness_vs_oracle(api, suite, single_point, mode):
    from distributed_point_functions_amd import _lib
    L = _lib.lib()
    prev = L.dpf_amd_set_prefix_expand(mode)
    try:
        _incremental_suite(api, suite, single_point)
    finally:
        L.dpf_amd_set_prefix_expand(prev)


def _incremental_suite(api, suite, single_point):
    name, hier, alphas, betas_list, steps = suite
    levels = IC.levels_of(hier)
    dpf = _make(api, levels)
    od = po.Dpf(levels)
    for step in steps:
        for alpha in alphas:
            for betas in betas_list:
                seeds = (alpha + 7, step)
                keys = dpf.generate_keys_incremental(alpha, betas, seeds=seeds)
                okeys = od.generate_keys(alpha, betas, seeds=seeds)
                ctxs = [dpf.create_evaluation_context(k) for k in keys]
                octxs = [od.create_evaluation_context(k) for k in okeys]
                IC.run_case(hier, alpha, betas, step, single_point,
                            _evaluator(dpf, od, hier, ctxs, octxs))


def test_single_point_partial_evaluation_then_evaluate_until(api, expand_mode):
    """test.cc:190-235: EvaluateAt(0, {prefix}, ctx) at a 108-bit level, then
    EvaluateUntil(1, {prefix}, ctx) expands the 2^20 suffixes below it from
    the stored partial evaluation — every output and context vs the oracle."""
    levels = [(108, ("int", 32), 0), (128, ("int", 32), 0)]
    dpf = _make(api, levels)
    od = po.Dpf(levels)
    prefix, suffix, beta = 0xdeadbeef, 23, 42
    alpha = (prefix << 20) + suffix
    keys = dpf.generate_keys_incremental(alpha, [beta, beta], seeds=(5, 6))
    okeys = od.generate_keys(alpha, [beta, beta], seeds=(5, 6))
    outs = []
    for k, ok in zip(keys, okeys):
        ctx, octx = dpf.create_evaluation_context(k), od.create_evaluation_context(ok)
        a = _words(dpf.evaluate_at_ctx(0, [prefix], ctx, raw=True), 32)
        assert np.array_equal(a, od.evaluate_at_ctx_words(0, [prefix], octx)[:, 0, :])
        _same_ctx(ctx, octx)
        u = _words(dpf.evaluate_until(1, [prefix], ctx, raw=True), 32)
        assert np.array_equal(u, od.evaluate_until_words(1, [prefix], octx)[:, 0, :])
        assert ctx.previous_hierarchy_level == octx.previous_hierarchy_level == 1
        outs.append((a, u))
    assert int(IC.share_sum(outs[0][0], outs[1][0], 32)[0, 0]) == beta
    s = IC.share_sum(outs[0][1], outs[1][1], 32)
    want = np.zeros_like(s)
    want[suffix, 0] = beta
    assert np.array_equal(s, want)


def test_mixed_evaluate_until_and_evaluate_at_ctx(api, expand_mode):
    """EvaluateUntil on level 0 and 1 (partial evaluations stored at level
    0), then EvaluateAt with the context two levels further down (a walk of
    the stored evaluations over several tree levels), then a level-skipping
    EvaluateUntil from the points EvaluateAt stored; uint64 and uint128."""
    for bits in (64, 128):
        lds = [6, 12, 20, 33, 40]
        levels = [(ld, ("int", bits), 0) for ld in lds]
        dpf = _make(api, levels)
        od = po.Dpf(levels)
        rng = np.random.default_rng(bits)
        alpha = int(rng.integers(0, 1 << 40))
        betas = [11 + i for i in range(len(lds))]
        keys = dpf.generate_keys_incremental(alpha, betas, seeds=(8, 9))
        okeys = od.generate_keys(alpha, betas, seeds=(8, 9))
        p1 = sorted({int(x) for x in rng.integers(0, 1 << 6, 20)} | {alpha >> 34})
        low = [int(x) for x in rng.integers(0, 1 << 27, 300)]
        pts3 = [(p1[i % len(p1)] << 27) | x for i, x in enumerate(low)] + [alpha >> 7]
        outs = []
        for k, ok in zip(keys, okeys):
            ctx, octx = dpf.create_evaluation_context(k), od.create_evaluation_context(ok)
            for h, pre in ((0, []), (1, p1)):
                got = _words(dpf.evaluate_until(h, pre, ctx, raw=True), bits)
                assert np.array_equal(got, od.evaluate_until_words(h, pre, octx)[:, 0, :])
                _same_ctx(ctx, octx)
            got = _words(dpf.evaluate_at_ctx(3, pts3, ctx, raw=True), bits)
            assert np.array_equal(got, od.evaluate_at_ctx_words(3, pts3, octx)[:, 0, :])
            _same_ctx(ctx, octx)
            # 7 bits below every stored point, from the level-3 evaluations
            got = _words(dpf.evaluate_until(4, pts3, ctx, raw=True), bits)
            assert np.array_equal(got, od.evaluate_until_words(4, pts3, octx)[:, 0, :])
            assert ctx.previous_hierarchy_level == 4
            outs.append(got)
        s = IC.share_sum(outs[0], outs[1], bits)
        hit = len(pts3) - 1
        assert int(s[hit * 128 + (alpha & 127), 0]) == betas[4]
        s[hit * 128 + (alpha & 127)] = 0
        assert not s.any()


def test_evaluate_at_ctx_errors(api):
    """The reference's errors through the ctx overload: a point outside the
    domain, and a point whose prefix the context never evaluated."""
    from distributed_point_functions_amd._lib import DpfAmdError
    levels = [(4, ("int", 64), 0), (8, ("int", 64), 0)]
    dpf = _make(api, levels)
    k0, _ = dpf.generate_keys_incremental(3, [1, 2], seeds=(1, 2))
    ctx = dpf.create_evaluation_context(k0)
    dpf.evaluate_at_ctx(0, [1, 2], ctx)
    with pytest.raises(DpfAmdError) as e:
        dpf.evaluate_at_ctx(1, [0xff], ctx)
    assert e.value.code == 3
    assert "Prefix not present in ctx.partial_evaluations at hierarchy level 1" in str(e.value)
    with pytest.raises(DpfAmdError) as e:
        dpf.evaluate_at_ctx(1, [256], ctx)
    assert "`evaluation_points[0]` larger than the domain size at hierarchy level 1" in str(e.value)
    assert dpf.evaluate_at_ctx(1, [], ctx) == []


def test_device_bookkeeping_equals_host_path(api):
    """EvaluateUntil's device path (de-duplication, stored-evaluation lookup
    and the context's list in HBM, dpf_amd_set_prefix_expand(0)) against the
    host path (mode 2): identical outputs and identical serialized contexts
    at every level — sorted prefixes with duplicates, a context copied
    through its wire bytes midway (its list then on the host), unsorted
    prefixes (the device path declines, the host path's hash lookup runs) —
    and the reference's errors for a prefix outside the domain and one the
    context never evaluated."""
    from distributed_point_functions_amd import _lib
    from distributed_point_functions_amd._lib import DpfAmdError
    L = _lib.lib()
    lds = [8, 16, 24, 32, 40, 48]
    levels = [(ld, ("int", 64), 0) for ld in lds]
    dpf = _make(api, levels)
    rng = np.random.default_rng(55)
    alpha = int(rng.integers(0, 1 << 48))
    keys = dpf.generate_keys_incremental(alpha, [3 + i for i in range(len(lds))], seeds=(4, 5))
    pre = [[]]
    for h in range(1, len(lds)):
        prev = pre[-1] if h > 1 else list(range(256))
        cur = sorted(int(p) << 8 | int(x) for p, x in
                     zip(rng.choice(prev, 3000), rng.integers(0, 256, 3000)))
        cur.append(alpha >> (48 - lds[h - 1]))
        cur = sorted(cur)
        if h == 5:
            cur = cur + cur[:40]  # unsorted (and duplicated) at this level
        pre.append(cur if h > 1 else list(range(256)))
    for key in keys:
        runs = {}
        for mode in (0, 2):
            prev_mode = L.dpf_amd_set_prefix_expand(mode)
            try:
                ctx = dpf.create_evaluation_context(key)
                outs, wires = [], []
                for h in range(len(lds)):
                    if h == 4:  # continue from a copy through the wire format
                        ctx = dpf.parse_evaluation_context(ctx.serialize())
                    outs.append(dpf.evaluate_until(h, pre[h] if h else [], ctx, raw=True))
                    wires.append(ctx.serialize())
                runs[mode] = (outs, wires)
            finally:
                L.dpf_amd_set_prefix_expand(prev_mode)
        for h in range(len(lds)):
            assert np.array_equal(runs[0][0][h], runs[2][0][h]), h
            assert runs[0][1][h] == runs[2][1][h], h
    # the reference's errors from the device path's fallback
    for mode in (0, 2):
        prev_mode = L.dpf_amd_set_prefix_expand(mode)
        try:
            ctx = dpf.create_evaluation_context(keys[0])
            dpf.evaluate_until(0, [], ctx)
            dpf.evaluate_until(1, [1, 2, 3], ctx)
            with pytest.raises(DpfAmdError) as e:
                dpf.evaluate_until(2, [(1 << 16) + 5], ctx)
            assert e.value.code == 3
            assert "out of range for hierarchy level 1" in str(e.value)
            with pytest.raises(DpfAmdError) as e:
                dpf.evaluate_until(2, [(7 << 8) | 1], ctx)
            assert e.value.code == 3
            assert "Prefix not present in ctx.partial_evaluations at hierarchy level 1" in \
                str(e.value)
        finally:
            L.dpf_amd_set_prefix_expand(prev_mode)


def _hip():
    import ctypes
    return ctypes.CDLL("libamdhip64.so")


def test_context_outlives_the_callers_stream(api):
    """A context whose partial evaluations were written on a caller-owned
    stream (dpf_amd_evaluate_until_device's `stream`) is destroyed after that
    stream: the device-held list is returned on a stream the library owns,
    and later evaluations on a new caller stream (which may reuse the old
    handle's address) still match the oracle."""
    import ctypes
    import torch
    from distributed_point_functions_amd import _lib
    D, V = api
    hier = [(8, ("int", 64), 0), (16, ("int", 64), 0), (24, ("int", 64), 0)]
    dpf = _make(api, hier)
    od = po.Dpf(hier)
    alpha = 0xA1B2C3
    k0, _ = dpf.generate_keys_incremental(alpha, [1, 2, 3], seeds=(11, 12))
    ok0, _ = od.generate_keys(alpha, [1, 2, 3], seeds=(11, 12))
    L, hip = _lib.lib(), _hip()
    pre1 = list(range(0, 256, 3))
    pre2 = sorted({(p << 8) | q for p in pre1[:40] for q in (0, 17, 255)})
    tp = V.Integer(64).to_proto()
    for rep in range(3):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        ctx = dpf.create_evaluation_context(k0)
        octx = od.create_evaluation_context(ok0)
        for h, pre in ((0, []), (1, pre1)):
            n = ctypes.c_int64()
            out = torch.empty(((len(pre) or 1) << 8) * 8, dtype=torch.uint8, device="cuda")
            pw = po.u128_words(pre) if pre else np.zeros(2, np.uint64)
            _lib.check(L.dpf_amd_evaluate_until_device(
                dpf._h, h, pw.ctypes.data_as(ctypes.c_void_p), len(pre), tp, len(tp), ctx._h,
                ctypes.c_void_p(out.data_ptr()), out.numel(), ctypes.byref(n), s))
            want = od.evaluate_until_words(h, pre, octx)[:, 0, 0]
            got = out.cpu().numpy().view(np.uint64)[:n.value]
            assert np.array_equal(got, want), (rep, h)
        assert ctx.num_partial_evaluations > 0  # the device-held list of level 1
        assert hip.hipStreamDestroy(s) == 0
        del ctx  # after its stream: the list goes back on the library's stream
        # a fresh context, the thread's own stream: level 2 from level 1's list
        ctx = dpf.create_evaluation_context(k0)
        octx = od.create_evaluation_context(ok0)
        for h, pre in ((0, []), (1, pre1), (2, pre2)):
            got = _words(dpf.evaluate_until(h, pre, ctx, raw=True), 64)
            want = od.evaluate_until_words(h, pre, octx)[:, 0, :]
            assert np.array_equal(got, want), (rep, h)
    torch.cuda.synchronize()


def test_size_query_validates_prefixes(api):
    """dpf_amd_evaluate_until with out == NULL (the size query) rejects a
    prefix outside the previous level's domain with the reference's error
    (h:735-745), for short and for long prefix lists; with a negative
    capacity it only counts, and the evaluation reports the error."""
    import ctypes
    from distributed_point_functions_amd import _lib
    D, V = api
    hier = [(8, ("int", 64), 0), (16, ("int", 64), 0), (24, ("int", 64), 0)]
    dpf = _make(api, hier)
    k0, _ = dpf.generate_keys_incremental(77, [1, 2, 3], seeds=(1, 2))
    L = _lib.lib()
    tp = V.Integer(64).to_proto()
    for pre in ([3, 256], list(range(200)) * 100 + [300]):
        ctx = dpf.create_evaluation_context(k0)
        dpf.evaluate_until(0, [], ctx)
        pw = po.u128_words(pre)
        n = ctypes.c_int64(-1)
        rc = L.dpf_amd_evaluate_until(dpf._h, 1, pw.ctypes.data_as(ctypes.c_void_p), len(pre),
                                      tp, len(tp), ctx._h, None, 0, ctypes.byref(n))
        assert rc == 3
        msg = L.dpf_amd_last_error().decode()
        assert "Index %d out of range for hierarchy level 0" % max(pre) in msg, msg
        # capacity < 0: the two-call protocol's size-only query leaves the
        # range check to the evaluation call
        assert L.dpf_amd_evaluate_until(dpf._h, 1, pw.ctypes.data_as(ctypes.c_void_p), len(pre),
                                        tp, len(tp), ctx._h, None, -1, ctypes.byref(n)) == 0
        assert n.value == len(pre) * 256
        with pytest.raises(Exception, match="out of range for hierarchy level 0"):
            dpf.evaluate_until(1, pre, ctx)
        # in range: the size query answers
        ok = [p for p in pre if p < 256][:50]
        pw = po.u128_words(ok)
        assert L.dpf_amd_evaluate_until(dpf._h, 1, pw.ctypes.data_as(ctypes.c_void_p), len(ok),
                                        tp, len(tp), ctx._h, None, 0, ctypes.byref(n)) == 0
        assert n.value == len(ok) * 256


@pytest.mark.parametrize("depth", [4, 5, 6, 8])
def test_incremental_levels_under_forced_depth(api, depth):
    """The device incremental path (dpf.cc EvaluateUntilOnDevice: 7 tree
    levels below each prefix root for uint64 at 8-bit hierarchy steps, c3's
    shape) with the expansion's DFS depth forced — D = 6 walks one level per
    thread — every output and the context against the oracle."""
    from distributed_point_functions_amd import kernels as K
    hier = [(8, ("int", 64), 0), (16, ("int", 64), 0), (24, ("int", 64), 0), (32, ("int", 64), 0)]
    dpf = _make(api, hier)
    od = po.Dpf(hier)
    alpha = 0x5EEDF00D
    betas = [3, 5, 7, 9]
    k0, k1 = dpf.generate_keys_incremental(alpha, betas, seeds=(21, 22))
    ok0, ok1 = od.generate_keys(alpha, betas, seeds=(21, 22))
    rng = np.random.default_rng(depth)
    pre = [[], list(range(256))]
    for h in (2, 3):
        parents = sorted(rng.choice(pre[-1], size=min(len(pre[-1]), 1 << 10), replace=False))
        pre.append(sorted({(int(p) << 8) | int(q) for p in parents for q in rng.integers(0, 256, 4)}))
    with K.forced_expand_depth(depth):
        for key, okey in ((k0, ok0), (k1, ok1)):
            ctx, octx = dpf.create_evaluation_context(key), od.create_evaluation_context(okey)
            for h in range(4):
                got = _words(dpf.evaluate_until(h, pre[h], ctx, raw=True), 64)
                want = od.evaluate_until_words(h, pre[h], octx)[:, 0, :]
                assert np.array_equal(got, want), (depth, key.party, h)
                if h < 3:
                    _same_ctx(ctx, octx)
