"""CPU pin of the oracle's incremental paths against the reference's own
property test, IncrementalDpfTest (dpf/distributed_point_function_test.cc:
308-930), before the GPU suite uses the oracle as its checker:

  - every instantiation of test.cc:698-930 (one to 129 hierarchy levels,
    level_step 1/2/3/5/7, single_point on and off) satisfies the share sums
    of EvaluateAndCheckLevel (test.cc:360-485);
  - EvaluateAt with a context equals EvaluateAt without one on the same
    points (the reference documents the two as equivalent, h:356-365), and
    the context ends at the evaluated level;
  - the EvaluateAt-then-EvaluateUntil scenario of
    TestSinglePointPartialEvaluation (test.cc:190-235).
"""
import numpy as np
import pytest

from oracle import pyoracle as po
from tests import incremental_cases as IC


def _oracle_evaluator(od, ctxs, keys):
    def evaluate(h, prefixes, single_point):
        outs = []
        for ctx, key in zip(ctxs, keys):
            if single_point:
                got = od.evaluate_at_ctx_words(h, prefixes, ctx)
                assert np.array_equal(got, od.evaluate_at_words(key, h, prefixes))
                assert ctx.previous_hierarchy_level == h
                assert ctx.partial_evaluations_level == h
                # the stored evaluations are the points' tree indices at h
                assert len(ctx.partial_evaluations()) == len(prefixes)
            else:
                got = od.evaluate_until_words(h, prefixes, ctx)
            outs.append(got[:, 0, :])
        return outs
    return evaluate


@pytest.mark.parametrize("single_point", [False, True])
@pytest.mark.parametrize("suite", IC.SUITES, ids=[s[0] for s in IC.SUITES])
def test_oracle_incremental_dpf_correctness(suite, single_point):
    name, hier, alphas, betas_list, steps = suite
    od = po.Dpf(IC.levels_of(hier))
    for step in steps:
        for alpha in alphas:
            for betas in betas_list:
                k0, k1 = od.generate_keys(alpha, betas, seeds=(alpha + 7, step))
                ctxs = [od.create_evaluation_context(k) for k in (k0, k1)]
                n = IC.run_case(hier, alpha, betas, step, single_point,
                                _oracle_evaluator(od, ctxs, (k0, k1)))
                assert n == len(range(step - 1, len(hier), step))


def test_oracle_single_point_partial_evaluation():
    """test.cc:190-235: EvaluateAt(0, {prefix}, ctx) on a 108-bit level, then
    EvaluateUntil(1, {prefix}, ctx) expands the 2^20 suffixes under it."""
    levels = [(108, ("int", 32), 0), (128, ("int", 32), 0)]
    od = po.Dpf(levels)
    prefix, suffix, beta = 0xdeadbeef, 23, 42
    alpha = (prefix << 20) + suffix
    k0, k1 = od.generate_keys(alpha, [beta, beta], seeds=(5, 6))
    c0, c1 = od.create_evaluation_context(k0), od.create_evaluation_context(k1)
    a = od.evaluate_at_ctx(0, [prefix], c0)
    b = od.evaluate_at_ctx(0, [prefix], c1)
    assert (a[0][0] + b[0][0]) % (1 << 32) == beta
    a = od.evaluate_until_words(1, [prefix], c0)[:, 0, :]
    b = od.evaluate_until_words(1, [prefix], c1)[:, 0, :]
    assert len(a) == len(b) == 1 << 20
    s = IC.share_sum(a, b, 32)
    want = np.zeros_like(s)
    want[suffix, 0] = beta
    assert np.array_equal(s, want)


def test_oracle_evaluate_at_ctx_missing_prefix():
    """A point whose prefix the context never evaluated: the reference's
    error (cc:419-423)."""
    levels = [(4, ("int", 64), 0), (8, ("int", 64), 0)]
    od = po.Dpf(levels)
    k0, _ = od.generate_keys(3, [1, 2], seeds=(1, 2))
    ctx = od.create_evaluation_context(k0)
    od.evaluate_at_ctx(0, [1, 2], ctx)
    with pytest.raises(po.OracleError) as e:
        od.evaluate_at_ctx(1, [0xff], ctx)
    assert e.value.code == 3
    assert e.value.message == "Prefix not present in ctx.partial_evaluations at hierarchy level 1"
