"""Concurrency of the const API under 1024 threads, as the reference's stress
tests: one Aes128FixedKeyHash shared by 1024 threads
(dpf/aes_128_fixed_key_hash_test.cc:155-174) and one DenseDpfPirServer
answering the same request from 1024 threads
(pir/dense_dpf_pir_server_test.cc:307-326).  Here the shared objects are a
DistributedPointFunction (EvaluateAt, full-domain EvaluateNext with one
context per thread) and a DenseDpfPirServer; every thread's result must equal
the single-threaded one.  ctypes releases the GIL during the library calls,
so the threads really run the host paths and kernels concurrently (each on
its own HIP stream).
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THREADS = 1024


def _run_threads(fn, threads_n=THREADS):
    results, errors = [None] * threads_n, []

    def worker(t):
        try:
            results[t] = fn(t)
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))
    threads = [threading.Thread(target=worker, args=(t,)) for t in range(threads_n)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    assert not errors, errors[:3]
    return results


def test_dpf_evaluate_concurrently_from_1024_threads(cuda):
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    vt = V.Tuple(V.Integer(32), V.IntModN(64, 2 ** 64 - 59))
    dpf = DistributedPointFunction.create(DpfParameters(12, vt, 48))
    k0, _ = dpf.generate_keys(1234, (5, 6), seeds=(11, 12))
    pts = [(17 * i + 3) % 4096 for i in range(64)] + [1234]
    want_at = dpf.evaluate_at(k0, 0, pts, raw=True).tobytes()
    want_full = dpf.evaluate_next([], dpf.create_evaluation_context(k0), raw=True).tobytes()

    def call(t):
        if t % 2:
            return dpf.evaluate_at(k0, 0, pts, raw=True).tobytes() == want_at
        ctx = dpf.create_evaluation_context(k0)
        return dpf.evaluate_next([], ctx, raw=True).tobytes() == want_full
    assert all(_run_threads(call))


def test_host_layout_padding_bytes_are_zero(cuda):
    """Rows of a host layout with holes ({u32, u64}: 4 unused bytes) carry
    zeros there, never stale device memory (host_device.h ClearPadding)."""
    import torch
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    # leave non-zero garbage in the stream-ordered pools first
    junk = torch.full((1 << 24,), 0xAB, dtype=torch.uint8, device=cuda)
    del junk
    vt = V.Tuple(V.Integer(32), V.IntModN(64, 2 ** 64 - 59))
    dpf = DistributedPointFunction.create(DpfParameters(12, vt, 48))
    k0, _ = dpf.generate_keys(77, (5, 6), seeds=(1, 2))
    outs = [dpf.evaluate_next([], dpf.create_evaluation_context(k0), raw=True),
            dpf.evaluate_at(k0, 0, list(range(0, 4096, 7)), raw=True)]
    for raw in outs:
        covered = np.zeros(raw.dtype.itemsize, bool)
        for name in raw.dtype.names:
            dt, off = raw.dtype.fields[name][:2]
            covered[off:off + dt.itemsize] = True
        assert not covered.all()
        rows = raw.view(np.uint8).reshape(len(raw), raw.dtype.itemsize)
        assert not rows[:, ~covered].any()


def test_pir_server_handle_request_from_1024_threads(cuda):
    from distributed_point_functions_amd import pir as P
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    n, size = 2000, 64
    rng = np.random.default_rng(1024)
    records = rng.integers(0, 256, (n, size), dtype=np.uint8)
    db = P.DenseDpfPirDatabase()
    db.insert_fixed(records)
    server = P.DenseDpfPirServer.create_plain(n, db)
    dpf = DistributedPointFunction.create(DpfParameters((n - 1).bit_length(), V.XorWrapper(128)))
    idx = [0, 77, 1999, 1024]
    pairs = P.client_keys(dpf, n, idx, seeds=[(2 * i + 5, 2 * i + 6) for i in range(len(idx))])
    req0 = P.pir_request_plain([a for a, _ in pairs])
    req1 = P.pir_request_plain([b for _, b in pairs])
    want0 = server.handle_request(req0)
    r1 = P.parse_response(server.handle_request(req1))
    for i, a, b in zip(idx, P.parse_response(want0), r1):
        assert bytes(x ^ y for x, y in zip(a, b)) == records[i].tobytes()
    assert all(_run_threads(lambda t: server.handle_request(req0) == want0))


def test_incremental_and_evaluate_and_apply_from_128_threads(cuda):
    """The incremental path's per-thread pinned scratch, the shared host
    worker pool (prefix de-duplication and merge join split over it at
    2^14+ prefixes) and the deferred context rewrite, plus EvaluateAndApply's
    key de-duplication, from 128 concurrent threads: every thread's levels
    and values equal the single-threaded ones."""
    import random
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    lds = [8, 16, 20]
    dpf = DistributedPointFunction.create_incremental(
        [DpfParameters(ld, V.Integer(64)) for ld in lds])
    alpha = 0xABCDE
    k0, k1 = dpf.generate_keys_incremental(alpha, [3, 4, 5], seeds=(21, 22))
    rng = random.Random(128)
    p1 = list(range(256))
    p2 = sorted(set(rng.sample(range(1 << 16), 20000)) | {alpha >> 4})

    def incremental():
        ctx = dpf.create_evaluation_context(k0)
        return [dpf.evaluate_next(p, ctx, raw=True).tobytes() for p in ([], p1, p2)]
    want_inc = incremental()
    keys = [k0, k1] * 3000
    pts = [rng.randrange(1 << 20) for _ in keys]
    pts[0] = alpha

    def apply():
        seen = []
        dpf.evaluate_and_apply(keys, pts, lambda v: seen.append(v) or True)
        return seen
    want_apply = apply()

    def call(t):
        return incremental() == want_inc if t % 2 else apply() == want_apply
    assert all(_run_threads(call, 128))


def test_thread_resources_recycled_across_thread_generations(cuda):
    """Per-thread streams, pinned staging and incremental scratch go back to
    a free list when a thread exits and the next thread takes them over
    (host_device.h ThreadRecycled): 6 generations of 48 short-lived threads
    run EvaluateAt, a 2^14-prefix EvaluateNext (pinned scratch, host pool)
    and an EvaluateAndApply with 2 MiB of points (pinned H2D staging), each
    generation starting while nothing of the previous one is alive; every
    result equals the single-threaded one."""
    import random
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    lds = [14, 18]
    dpf = DistributedPointFunction.create_incremental(
        [DpfParameters(ld, V.Integer(64)) for ld in lds])
    k0, k1 = dpf.generate_keys_incremental(777, [9, 10], seeds=(31, 32))
    rng = random.Random(6)
    p1 = list(range(1 << 14))
    pts = [rng.randrange(1 << 18) for _ in range(1 << 17)]
    keys = [k0] * (len(pts) // 2) + [k1] * (len(pts) // 2)

    def work(t):
        kind = t % 3
        if kind == 0:
            return dpf.evaluate_at(k0, 1, pts[:5000], raw=True).tobytes()
        if kind == 1:
            ctx = dpf.create_evaluation_context(k1)
            return [dpf.evaluate_next(p, ctx, raw=True).tobytes() for p in ([], p1)]
        seen = []
        dpf.evaluate_and_apply(keys, pts, lambda v: seen.append(v[::997]) or True)
        return seen
    want = [work(k) for k in range(3)]
    for _ in range(6):
        res = _run_threads(lambda t: work(t) == want[t % 3], 48)
        assert all(res)


def test_thread_resource_cache_cap(cuda):
    """With the idle-object cap at 4 (dpf_amd_set_thread_cache_cap), each
    generation of 32 exiting threads parks 28 surplus objects of every kind,
    which the next generation's first threads destroy (outside any
    thread-exit handler) while the others evaluate; every result still
    equals the single-threaded one."""
    from distributed_point_functions_amd import _lib
    from distributed_point_functions_amd import value_types as V
    from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
    L = _lib.lib()
    dpf = DistributedPointFunction.create_incremental(
        [DpfParameters(ld, V.Integer(64)) for ld in (10, 16)])
    k0, _ = dpf.generate_keys_incremental(4321, [1, 2], seeds=(41, 42))
    p1 = list(range(1 << 10))

    def work():
        ctx = dpf.create_evaluation_context(k0)
        return [dpf.evaluate_next(p, ctx, raw=True).tobytes() for p in ([], p1)]
    want = work()
    assert L.dpf_amd_set_thread_cache_cap(4) == 0
    try:
        for _ in range(4):
            assert all(_run_threads(lambda t: work() == want, 32))
    finally:
        assert L.dpf_amd_set_thread_cache_cap(64) == 0
    assert L.dpf_amd_set_thread_cache_cap(-1) == 3
