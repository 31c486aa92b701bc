"""DistributedComparisonFunction (dcf/distributed_comparison_function.h/.cc).

CPU: Create errors with the reference's messages
(distributed_comparison_function_test.cc:58-72), and key generation equal
to the oracle's incremental DPF keys for level betas (beta where alpha's bit
is set, 0 elsewhere; dcf.cc:83-101) — the DCF keygen is host logic.

GPU: the fused BatchEvaluate kernel equals the oracle composition
sum_{h : bit (n-1-h) of x == 0} EvaluateAt(key, h, x >> (n - h)) bit-exactly,
and shares reconstruct beta on x < alpha, 0 elsewhere (GenEval,
distributed_comparison_function_test.cc:106-133), over the reference's test
types (:91-98) and its 64-bit-domain case (:193-243).
"""
import random

import pytest

from distributed_point_functions_amd import value_types as V
from distributed_point_functions_amd import wire
from distributed_point_functions_amd._lib import DpfAmdError
from distributed_point_functions_amd.dcf import (DcfKey, DcfParameters,
                                                 DistributedComparisonFunction)
from distributed_point_functions_amd.dpf import DpfParameters, decode_value
from oracle import pyoracle as po

P32 = 4294967291  # 2**32 - 5, the reference's MyIntModN

# (spec, log_domain) of DcfTestTypes (distributed_comparison_function_test.cc:91-98)
REF_TYPES = [
    (("int", 32), 1), (("int", 32), 2), (("int", 32), 5), (("int", 128), 5),
    (("tuple", [("int", 32), ("int", 32)]), 5),
    (("tuple", [("int", 32), ("int", 128)]), 5),
    (("tuple", [("intmodn", 32, P32), ("intmodn", 32, P32)]), 5),
]


def _dcf(spec, n):
    return DistributedComparisonFunction.create(
        DcfParameters(DpfParameters(n, V.from_spec(spec))))


def _beta42(spec):
    vt = V.from_spec(spec)
    return vt.unflatten(iter([42] * len(vt.scalars())))


def _oracle_keys(spec, n, alpha, beta, seeds):
    """The oracle's incremental DPF with the DCF's levels and betas."""
    od = po.Dpf([(i, spec, 0) for i in range(n)])
    vt = V.from_spec(spec)
    zero = vt.zero() if spec[0] != "xor" else beta  # SetToZero skips XorWrapper
    betas = [beta if (alpha >> (n - 1 - i)) & 1 else zero for i in range(n)]
    return od, od.generate_keys(alpha >> 1, betas, seeds=seeds)


def _oracle_dcf(od, key, n, x, spec):
    vt = V.from_spec(spec)
    acc = vt.zero()
    for h in range(n):
        if (x >> (n - 1 - h)) & 1:
            continue
        v = od.evaluate_at(key, h, [x >> (n - h)])[0]
        acc = vt.add(acc, vt.unflatten(iter(v)))
    return acc


# ---------------------------------------------------------------------------
# CPU
# ---------------------------------------------------------------------------

def test_create_fails_with_zero_log_domain_size():
    with pytest.raises(DpfAmdError) as e:
        _dcf(("int", 32), 0)
    assert e.value.code == 3 and "A DCF must have log_domain_size >= 1" in str(e.value)


def test_create_fails_without_value_type():
    import ctypes
    from distributed_point_functions_amd import _lib
    proto = wire.field_message(1, wire.field_varint(1, 5))  # no value_type
    h = ctypes.c_void_p()
    rc = _lib.lib().dpf_amd_dcf_create(proto, len(proto), ctypes.byref(h))
    assert rc == 3
    assert (_lib.lib().dpf_amd_last_error().decode() ==
            "parameters.value_type must be set for DistributedComparisonFunction::Create")


@pytest.mark.parametrize("spec,n", REF_TYPES + [(("int", 64), 64), (("xor", 64), 7)],
                         ids=lambda x: repr(x))
def test_keys_match_oracle(spec, n):
    """DCF keys = the oracle's incremental keys for the level betas; XorWrapper
    betas are not zeroed (SetToZero, dcf.cc:33-43, skips them)."""
    rng = random.Random(n)
    dcf = _dcf(spec, n)
    alpha = rng.randrange(1 << n)
    beta = _beta42(spec)
    seeds = (rng.getrandbits(128), rng.getrandbits(128))
    k0, k1 = dcf.generate_keys(alpha, beta, seeds=seeds)
    od = po.Dpf([(i, spec, 0) for i in range(n)])
    vt = V.from_spec(spec)
    zero = vt.zero() if spec[0] != "xor" else beta
    betas = [beta if (alpha >> (n - 1 - i)) & 1 else zero for i in range(n)]
    o0, o1 = od.generate_keys(alpha >> 1, betas, seeds=seeds)
    for k, o in ((k0, o0), (k1, o1)):
        assert DcfKey(bytes(k)) == k
        dk = k.key
        assert dk.seed == o.seed and dk.party == o.party
        assert [c.seed for c in dk.correction_words] == o.cw_seeds()
        assert [int(c.control_left) for c in dk.correction_words] == o.ccl()
        assert [int(c.control_right) for c in dk.correction_words] == o.ccr()
        last = [x for v in dk.last_level_value_correction for x in decode_value(vt, v)]
        assert last == o.value_corrections()[-1]


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("spec,n", REF_TYPES, ids=lambda x: repr(x))
def test_gen_eval_every_point(cuda, spec, n):
    """GenEval: every alpha, every x (domain <= 32), one BatchEvaluate per
    alpha over all x with both parties' keys."""
    dcf = _dcf(spec, n)
    vt = V.from_spec(spec)
    beta = _beta42(spec)
    zero = vt.zero()
    D = 1 << n
    for alpha in range(D):
        k0, k1 = dcf.generate_keys(alpha, beta, seeds=(alpha * 2 + 1, alpha * 2 + 2))
        r0 = dcf.batch_evaluate([k0] * D, list(range(D)))
        r1 = dcf.batch_evaluate([k1] * D, list(range(D)))
        for x in range(D):
            assert vt.add(r0[x], r1[x]) == (beta if x < alpha else zero), (alpha, x)


@pytest.mark.gpu
@pytest.mark.parametrize("spec,n", REF_TYPES[2:] + [(("int", 64), 64),
                                                     (("intmodn", 64, 18446744073709551557), 20),
                                                     (("tuple", [("int", 16), ("int", 8)]), 12),
                                                     (("int", 8), 7), (("int", 16), 11),
                                                     (("xor", 64), 9), (("xor", 128), 33)],
                         ids=lambda x: repr(x))
@pytest.mark.parametrize("kernel", [0, 1], ids=["auto", "generic"])
def test_batch_evaluate_matches_oracle(cuda, spec, n, kernel):
    """Mixed keys and parties in one batch == the oracle composition, with
    the automatic kernel (single integer / XorWrapper scalars run the
    register-only KDcfEvaluateDirect) and forced to the generic one."""
    from distributed_point_functions_amd import kernels as K
    rng = random.Random(n * 13 + len(repr(spec)))
    dcf = _dcf(spec, n)
    beta = _beta42(spec)
    keys, pts, want = [], [], []
    for j in range(6):
        alpha = rng.randrange(1 << n)
        seeds = (rng.getrandbits(128), rng.getrandbits(128))
        k0, k1 = dcf.generate_keys(alpha, beta, seeds=seeds)
        od, (o0, o1) = _oracle_keys(spec, n, alpha, beta, seeds)
        for party, (k, o) in enumerate(((k0, o0), (k1, o1))):
            for x in [alpha, max(alpha - 1, 0), rng.randrange(1 << n)]:
                keys.append(k)
                pts.append(x)
                want.append(_oracle_dcf(od, o, n, x, spec))
    with K.forced_dcf_kernel(kernel):
        got = dcf.batch_evaluate(keys, pts)
    assert got == want


@pytest.mark.gpu
def test_uint64_large_domain(cuda):
    """WorksCorrectlyOnUint64TWithLargeDomain (:193-243): alpha = 50."""
    dcf = _dcf(("int", 64), 64)
    k0, k1 = dcf.generate_keys(50, 42, seeds=(5, 6))
    rng = random.Random(64)
    xs = list(range(50)) + [rng.getrandbits(64) for _ in range(99)] + [50, 51]
    r0 = dcf.batch_evaluate([k0] * len(xs), xs)
    r1 = dcf.batch_evaluate([k1] * len(xs), xs)
    for x, a, b in zip(xs, r0, r1):
        assert (a + b) % (1 << 64) == (42 if x < 50 else 0), x


@pytest.mark.gpu
def test_batch_matches_single_and_errors(cuda):
    """BatchEvaluateMatchesSingleEvaluate (:171-191) and the size / malformed
    key errors (:135-169)."""
    dcf = _dcf(("int", 32), 5)
    k0, k1 = dcf.generate_keys(0, 42, seeds=(1, 2))
    assert dcf.batch_evaluate([k0, k1], [0, 1]) == [dcf.evaluate(k0, 0), dcf.evaluate(k1, 1)]
    with pytest.raises(DpfAmdError) as e:
        dcf.batch_evaluate([k0], [0, 1])
    assert e.value.code == 3 and "evaluation_points" in str(e.value)
    with pytest.raises(DpfAmdError) as e:
        dcf.evaluate(DcfKey(b""), 0)
    assert e.value.code == 3 and "key" in str(e.value)


@pytest.mark.gpu
@pytest.mark.parametrize("spec,n", [(("int", 64), 32), (("int", 8), 20), (("int", 128), 16),
                                    (("xor", 64), 24)], ids=lambda x: repr(x))
def test_batch_evaluate_many_pairs_kernels_agree(cuda, spec, n):
    """Thousands of (key, point) pairs over many waves, both parties: the
    automatic kernel (the register-only one for these single scalars) equals
    the generic kernel bit for bit, and the shares of integer types
    reconstruct beta on x < alpha, 0 elsewhere."""
    from distributed_point_functions_amd import kernels as K
    rng = random.Random(n * 7 + len(spec))
    dcf = _dcf(spec, n)
    vt = V.from_spec(spec)
    beta = _beta42(spec)
    keys0, keys1, xs, alphas = [], [], [], []
    for j in range(24):
        alpha = rng.randrange(1 << n)
        k0, k1 = dcf.generate_keys(alpha, beta, seeds=(2 * j + 11, 2 * j + 12))
        pts = [rng.randrange(1 << n) for _ in range(200)]
        pts += [max(alpha - 1, 0), alpha, min(alpha + 1, (1 << n) - 1)]
        keys0 += [k0] * len(pts)
        keys1 += [k1] * len(pts)
        xs += pts
        alphas += [alpha] * len(pts)
    with K.forced_dcf_kernel(0):
        a0, a1 = dcf.batch_evaluate(keys0, xs), dcf.batch_evaluate(keys1, xs)
    with K.forced_dcf_kernel(1):
        g0, g1 = dcf.batch_evaluate(keys0, xs), dcf.batch_evaluate(keys1, xs)
    assert a0 == g0 and a1 == g1
    if spec[0] == "int":
        zero = vt.zero()
        for x, al, r0, r1 in zip(xs, alphas, a0, a1):
            assert vt.add(r0, r1) == (beta if x < al else zero), (x, al)
