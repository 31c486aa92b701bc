"""The reference's IncrementalDpfTest, as data and one driver
(dpf/distributed_point_function_test.cc:308-930).

`SUITES` restates its five INSTANTIATE_TEST_SUITE_P parameter sets
(test.cc:698-930): hierarchies of (log_domain_size, element_bitsize), alphas,
beta vectors, level steps and the single-point switch.  `run_case` follows
TestCorrectness (test.cc:652-696) + EvaluateAndCheckLevel (test.cc:360-485):
1000 evaluation points (999 random, possibly duplicated, plus alpha), levels
level_step - 1, 2 * level_step - 1, ... evaluated either by EvaluateAt with a
context on the points' prefixes at that level (single_point) or by
EvaluateUntil on the prefixes at the previous evaluated level (full
expansion, which skips level_step - 1 hierarchy levels per call).

The driver is parameterised over an "evaluator" so the CPU suite runs it on
the oracle alone (share sums, plus EvaluateAt-with-context == EvaluateAt
without) and the GPU suite runs the product next to the oracle (every output
and the resulting EvaluationContext equal).
"""
from __future__ import annotations

import random
from typing import Callable, List, Sequence, Tuple

import numpy as np

MASK64 = (1 << 64) - 1

# (name, hierarchy, alphas, betas (one vector per instantiation), level_steps)
Hierarchy = List[Tuple[int, int]]

SUITES = []


def _suite(name, hierarchies, alphas, betas, steps):
    for i, hier in enumerate(hierarchies):
        SUITES.append(("%s_%d" % (name, i), hier, alphas, betas, steps))


# OneHierarchyLevelVaryElementSizes (test.cc:698-730)
_suite("one_level_sizes", [[(ld, b)] for ld in (4, 10) for b in (8, 16, 32, 64, 128)],
       [0, 1, 15], [[1], [100], [255]], [1])
# OneHierarchyLevelVaryDomainSizes (test.cc:732-797)
_suite("one_level_domains", [[(ld, b)] for b in (8, 64, 128) for ld in range(10)],
       [0], [[1], [100], [255]], [1])
# TwoHierarchyLevels (test.cc:799-838)
_suite("two_levels",
       [[(5, b), (10, b)] for b in (8, 16, 32, 64, 128)] +
       [[(0, b), (10, 128)] for b in (8, 16, 32, 64, 128)],
       [0, 1, 2, 100, 1023], [[1, 2], [80, 90], [255, 255]], [1, 2])
# ThreeHierarchyLevels (test.cc:840-913)
_suite("three_levels",
       [[(5, b), (10, b), (15, b)] for b in (8, 16, 32, 64, 128)] +
       [[(5, 8), (10, 16), (15, 32)],
        [(4, 8), (5, 8), (6, 8)], [(3, 16), (4, 16), (5, 16)], [(2, 32), (3, 32), (4, 32)],
        [(1, 64), (2, 64), (3, 64)], [(0, 128), (1, 128), (2, 128)]],
       [0, 1], [[1, 2, 3]], [1, 2])
# MaximumOutputDomainSize (test.cc:915-930): every bit a hierarchy level
_suite("max_domain", [[(i, 64) for i in range(129)]],
       [(42 << 64) | 23], [[1234567] * 129], [1, 2, 3, 5, 7])

NUM_POINTS = 1000


def evaluation_points(hier: Hierarchy, alpha: int, seed: int) -> List[int]:
    """test.cc:653-666: 999 uniform 128-bit points reduced to the last
    domain, then alpha."""
    rng = random.Random(seed)
    last = hier[-1][0]
    pts = [rng.getrandbits(128) for _ in range(NUM_POINTS - 1)]
    if last < 128:
        pts = [p % (1 << last) for p in pts]
    return pts + [alpha]


def prefix_for_level(hier: Hierarchy, h: int, index: int) -> int:
    """GetPrefixForLevel (test.cc:349-358)."""
    shift = hier[-1][0] - hier[h][0]
    return index >> shift if shift < 128 else 0


def levels_of(hier: Hierarchy):
    """The (log_domain, spec, security_parameter) triples of the oracle and
    the product (default security parameter, as the reference's test)."""
    return [(ld, ("int", b), 0) for ld, b in hier]


def share_sum(a: np.ndarray, b: np.ndarray, bits: int) -> np.ndarray:
    """(n, 2) {lo, hi} uint64 words of a + b mod 2^bits."""
    lo = a[:, 0] + b[:, 0]
    hi = a[:, 1] + b[:, 1] + (lo < a[:, 0]).astype(np.uint64)
    if bits < 64:
        lo &= np.uint64((1 << bits) - 1)
    if bits <= 64:
        hi[:] = 0
    return np.stack([lo, hi], axis=1)


def run_case(hier: Hierarchy, alpha: int, betas: Sequence[int], level_step: int,
             single_point: bool, evaluate: Callable, seed: int = 1) -> int:
    """Walks the levels of one TestCorrectness instantiation.  `evaluate(h,
    prefixes, single_point)` evaluates both parties and returns the two
    outputs as (n, 2) uint64 {lo, hi} word arrays (the level's one integer
    scalar per element); the share sums are checked here.  Returns the number
    of levels evaluated."""
    points = evaluation_points(hier, alpha, seed)
    num_levels = len(hier)
    previous = -1
    done = 0
    for h in range(level_step - 1, num_levels, level_step):
        bits = hier[h][1]
        ld = hier[h][0]
        if single_point:
            prefixes = [prefix_for_level(hier, h, p) for p in points]
        elif previous >= 0:
            prefixes = [prefix_for_level(hier, previous, p) for p in points]
        else:
            prefixes = []
        r0, r1 = evaluate(h, prefixes, single_point)
        assert r0.shape == r1.shape
        s = share_sum(r0, r1, bits)
        cur_alpha = prefix_for_level(hier, h, alpha)
        if single_point:
            assert len(r0) == len(prefixes)
            on_path = np.array([p == cur_alpha for p in prefixes])
        else:
            prev_ld = hier[previous][0] if previous >= 0 else 0
            opp = 1 << (ld - prev_ld)
            assert len(r0) == max(len(prefixes), 1) * opp
            prev_alpha = prefix_for_level(hier, previous, alpha) if previous >= 0 else 0
            under = np.array([previous < 0 or p == prev_alpha for p in (prefixes or [0])])
            on_path = np.repeat(under, opp) & (np.arange(len(r0)) % opp == cur_alpha % opp)
        want = np.zeros_like(s)
        want[on_path, 0] = np.uint64(betas[h] & MASK64)
        want[on_path, 1] = np.uint64(betas[h] >> 64)
        bad = np.nonzero((s != want).any(axis=1))[0]
        assert len(bad) == 0, (h, bad[:5])
        previous = h
        done += 1
    return done
