"""Measures the secondary BASELINE.json configs on one MI355X (the headline c5
and c4 Q=1 lines are bench.py's).  One JSON line per config on stdout.

    python tools/bench_configs.py [--only c1,c2,c3,c4q]

c1  full-domain EvaluateNext, log_domain 20, uint64 (1.5 AES/leaf)
c2  EvaluateAt of 2^20 random points over 64 keys, log_domain 128, uint128
    (129 AES/point); Tier-1 (device arrays, one launch per key and one
    multi-key launch) and Tier-2 (the EvaluateAt API, host vectors)
c3  incremental heavy hitters: 16 levels 8,16,..,128 bits, uint64, 2^16
    surviving prefixes per level (generator of distributed_point_function_
    benchmark.cc:154-191, distinct prefixes); Tier-2 EvaluateNext per level
c4q dense-PIR XOR scan at Q = 8 and 64 over 2^26 x 256 B (kernel only)
pirgrid the reference's PIR benchmark grid (dense_dpf_pir_database_benchmark.cc:
    125-157): 2^16 / 2^20 records x 32 / 256 / 2048 / 16384 B x batch 1 / 2 /
    10 / 100, scan and InnerProductWith
dcf DistributedComparisonFunction BatchEvaluate, log_domain 32, uint64
    (distributed_comparison_function_benchmark.cc:31-63 shape): 1024 keys
    via the Tier-2 API, and 2^20 (key, point) pairs through the fused kernel
cuckoo  cuckoo-hashed sparse PIR: 2^20 keyword records
    (16-byte keys, 240-byte values), 1.5 x 2^20 buckets, 3 SHA-256 hash
    functions; two plain servers, one keyword query (3 DPF keys per server)
    through HandleRequest (wire decode, device DPF selection, key- and
    value-table scans, response), reconstructed by the client

Kernel times are HIP events on the launch stream; API times are wall clock.
Every config also checks its outputs (share-sum / reconstruction).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import random
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_point_functions_amd import _lib, kernels  # noqa: E402
from distributed_point_functions_amd import value_types as V  # noqa: E402
from distributed_point_functions_amd.dpf import (  # noqa: E402
    DistributedPointFunction, DpfParameters, decode_value)

LDS_PEAK_LOOKUPS = 256 * 32 * 2.4e9
M64 = (1 << 64) - 1


def ev_time(fn, reps):
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


def wall_time(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def key_dev(dpf, key, level, dev):
    L = dpf.hierarchy_to_tree(level)
    cws = key.correction_words[:L]
    vt = dpf.parameters[level].value_type
    corr = [x for v in key.last_level_value_correction for x in decode_value(vt, v)]
    return dict(
        L=L,
        seed=kernels.u128_tensor([key.seed], dev),
        cb=torch.tensor([key.party], dtype=torch.uint8, device=dev),
        cw=kernels.u128_tensor([c.seed for c in cws] or [0], dev),
        ccl=torch.tensor([int(c.control_left) for c in cws] or [0], dtype=torch.uint8, device=dev),
        ccr=torch.tensor([int(c.control_right) for c in cws] or [0], dtype=torch.uint8, device=dev),
        corr=corr, party=key.party)


def lds_frac(aes_per_s):
    return aes_per_s * 160 / LDS_PEAK_LOOKUPS


def c1(dev, reps):
    dpf = DistributedPointFunction.create(DpfParameters(20, V.Integer(64)))
    k0, k1 = dpf.generate_keys(777777, 123456789123, seeds=(0x51, 0x52))
    desc = dpf.value_type_descriptor(0)
    ka = key_dev(dpf, k0, 0, dev)
    L = ka["L"]
    cepb = 1 << (20 - L)
    out = torch.empty((1 << 20) * 8, dtype=torch.uint8, device=dev)

    def step():
        kernels.expand_and_correct(ka["seed"], ka["cb"], L, ka["cw"], ka["ccl"], ka["ccr"],
                                   desc, ka["corr"], ka["party"], cepb, 0, 1 << L, out)
    t_k = ev_time(step, reps)
    ctx_reps = max(1, reps // 4)

    def api():
        dpf.evaluate_next([], dpf.create_evaluation_context(k0), raw=True)
    t_api = wall_time(api, ctx_reps)
    a = dpf.evaluate_next([], dpf.create_evaluation_context(k0), raw=True).view(np.uint64)
    b = dpf.evaluate_next([], dpf.create_evaluation_context(k1), raw=True).view(np.uint64)
    s = a + b
    ok = bool(s[777777] == 123456789123 and np.count_nonzero(s) == 1)
    aes = 2 * ((1 << L) - 1) + (1 << L)
    return {"config": "c1", "workload": "full-domain EvaluateNext log_domain=20 uint64",
            "leaves": 1 << 20, "kernel_ms": t_k * 1e3, "leaves_per_s": (1 << 20) / t_k,
            "api_ms": t_api * 1e3, "api_leaves_per_s": (1 << 20) / t_api,
            "aes_per_leaf": aes / (1 << 20), "lds_frac": lds_frac(aes / t_k), "correct": ok}


def c2(dev, reps):
    rng = random.Random(2)
    nkeys, per = 64, 1 << 14
    vt = V.Integer(128)
    dpf = DistributedPointFunction.create(DpfParameters(128, vt))
    desc = dpf.value_type_descriptor(0)
    keys, kd, pts = [], [], []
    for k in range(nkeys):
        alpha, beta = rng.getrandbits(128), rng.getrandbits(128)
        k0, k1 = dpf.generate_keys(alpha, beta, seeds=(1000 + 2 * k, 1001 + 2 * k))
        p = [rng.getrandbits(128) for _ in range(per)]
        p[0] = alpha
        keys.append((k0, k1, alpha, beta))
        kd.append(key_dev(dpf, k0, 0, dev))
        pts.append(kernels.u128_tensor(p, dev))
    L = kd[0]["L"]
    seeds = [kernels.u128_tensor([keys[k][0].seed] * per, dev) for k in range(nkeys)]
    cbs = [torch.full((per,), keys[k][0].party, dtype=torch.uint8, device=dev)
           for k in range(nkeys)]
    out = torch.empty(nkeys * per * 16, dtype=torch.uint8, device=dev)

    if C2_BATCHED_ONLY:  # profiling the batched kernel alone
        def tier1():
            pass
    else:
        def tier1():
            _tier1()

    def _tier1():
        for k in range(nkeys):
            kernels.evaluate_points(seeds[k], cbs[k], pts[k], 0, L, kd[k]["cw"], kd[k]["ccl"],
                                    kd[k]["ccr"], desc, party_all=kd[k]["party"],
                                    value_correction_all=kd[k]["corr"],
                                    out=out[k * per * 16:(k + 1) * per * 16])
    t1 = ev_time(tier1, reps)
    res = {"config": "c2", "workload": "EvaluateAt 2^20 points / 64 keys, log_domain=128, uint128",
           "points": nkeys * per, "aes_per_point": L + 1,
           "tier1_per_key_ms": t1 * 1e3, "tier1_per_key_points_per_s": nkeys * per / t1,
           "tier1_per_key_lds_frac": lds_frac(nkeys * per * (L + 1) / t1)}
    if hasattr(kernels, "evaluate_points_batched"):
        allp = torch.cat(pts)
        cw = torch.cat([d["cw"] for d in kd])
        ccl = torch.cat([d["ccl"] for d in kd])
        ccr = torch.cat([d["ccr"] for d in kd])
        kseed = torch.cat([d["seed"] for d in kd])
        kcb = torch.cat([d["cb"] for d in kd])
        kcorr = kernels.u128_tensor([x for d in kd for x in d["corr"]], dev)

        def multi():
            kernels.evaluate_points_batched(nkeys, per, kseed, kcb, allp, 0, L, cw, ccl, ccr,
                                            desc, party_all=0, key_value_corrections=kcorr,
                                            out=out)
        tm = ev_time(multi, reps)
        res.update({"tier1_multi_key_ms": tm * 1e3,
                    "tier1_multi_key_points_per_s": nkeys * per / tm,
                    "tier1_multi_key_lds_frac": lds_frac(nkeys * per * (L + 1) / tm)})
        got = out.view(torch.int64).view(-1, 2).cpu().numpy().view(np.uint64)
    if C2_BATCHED_ONLY:
        return res
    plist = [kernels.tensor_u128(p) for p in pts]

    def tier2():
        for k in range(nkeys):
            dpf.evaluate_at(keys[k][0], 0, plist[k], raw=True)
    t2 = wall_time(tier2, max(1, reps // 4))
    ok = True
    for k in range(0, nkeys, 16):
        a = dpf.evaluate_at(keys[k][0], 0, plist[k][:64], raw=True)
        b = dpf.evaluate_at(keys[k][1], 0, plist[k][:64], raw=True)
        s = [(vt.decode(a)[i] + vt.decode(b)[i]) % (1 << 128) for i in range(64)]
        ok &= s[0] == keys[k][3] and all(x == 0 for x in s[1:])
        if "tier1_multi_key_ms" in res:
            w = got[k * per:k * per + 64]
            ok &= [int(lo) | (int(hi) << 64) for lo, hi in w] == vt.decode(a)
    res.update({"tier2_api_ms": t2 * 1e3, "tier2_api_points_per_s": nkeys * per / t2,
                "correct": bool(ok)})
    return res


def c3(dev, reps):
    rng = random.Random(3)
    H = 16
    params = [DpfParameters(8 * (i + 1), V.Integer(64)) for i in range(H)]
    dpf = DistributedPointFunction.create_incremental(params)
    alpha = rng.getrandbits(128)
    betas = [rng.getrandbits(64) for _ in range(H)]
    k0, k1 = dpf.generate_keys_incremental(alpha, betas, seeds=(0x31, 0x32))
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
        # keep alpha's prefix so the check below sees the non-zero
        ap = alpha >> (128 - 8 * i)
        if ap not in cur:
            cur[rng.randrange(len(cur))] = ap
            cur = sorted(cur)
        prefixes.append(cur)
    # numpy {lo, hi} rows: the host-side list conversion is not library time
    prefixes = [np.array([[p & M64, p >> 64] for p in ps], dtype=np.uint64).reshape(-1, 2)
                if ps else [] for ps in prefixes]

    def run(key, keep=False, device_out=None):
        ctx = dpf.create_evaluation_context(key)
        outs, times = [], []
        for i in range(H):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if device_out is not None:
                o = dpf.evaluate_next(prefixes[i], ctx, out=device_out)
            else:
                o = dpf.evaluate_next(prefixes[i], ctx, raw=True)
            times.append(time.perf_counter() - t0)
            if keep:
                outs.append(o.view(np.uint64).copy())
        return outs, times
    dev_out = torch.empty((1 << 24) * 8, dtype=torch.uint8, device=dev)
    best = {}
    for mode, d_out in (("host", None), ("device", dev_out)):
        run(k0, device_out=d_out)
        for _ in range(max(1, reps // 4)):
            _, times = run(k0, device_out=d_out)
            if mode not in best or sum(times) < sum(best[mode]):
                best[mode] = times
    a, _ = run(k0, True)
    b, _ = run(k1, True)
    ok = True
    for i in range(H):
        s = a[i] + b[i]
        nz = np.nonzero(s)[0]
        ok &= len(nz) == 1 and int(s[nz[0]]) == betas[i]
    leaves = sum(len(x) for x in a)
    # LDS-lookup fraction of a whole level (device outputs): per prefix the
    # walk from the stored partial evaluation (8 levels) and to the prefix's
    # own node (1), then its 2^7-leaf subtree (2 (2^7 - 1) tree + 2^7 value
    # AES) — 391 AES x 160 lookups, over the level's wall time
    lvl = [len(prefixes[i]) * 391 * 160 / best["device"][i] / LDS_PEAK_LOOKUPS
           for i in range(2, H)]
    return {"config": "c3", "workload": "heavy hitters, 16 levels x 8 bits, uint64, 2^16 prefixes",
            "returned_leaves": leaves,
            "level_lds_frac_median": float(np.median(lvl)),
            "host_out_ms_total": 1e3 * sum(best["host"]),
            "host_out_ms_per_level": [round(1e3 * t, 3) for t in best["host"]],
            "host_out_leaves_per_s": leaves / sum(best["host"]),
            "device_out_ms_total": 1e3 * sum(best["device"]),
            "device_out_ms_per_level": [round(1e3 * t, 3) for t in best["device"]],
            "device_out_leaves_per_s": leaves / sum(best["device"]), "correct": bool(ok)}


C4Q_QUERIES = (1, 8, 16, 32, 64, 100)
C4Q_AB = True
C2_BATCHED_ONLY = False


def c4q(dev, reps):
    n, rec = 1 << 26, 256
    gen = torch.Generator(device=dev)
    gen.manual_seed(4)
    db = torch.randint(0, 256, (n * rec,), dtype=torch.uint8, device=dev, generator=gen)
    res = {"config": "c4q", "workload": "XOR scan 2^26 x 256 B"}
    for q in C4Q_QUERIES:
        sel = torch.randint(-2**63, 2**63 - 1, (q * (n // 128), 2), dtype=torch.int64,
                            device=dev, generator=gen)
        ws = torch.empty(max(16, _lib.lib().dpf_amd_inner_product_workspace_size(n, rec, q)),
                         dtype=torch.uint8, device=dev)
        out = torch.empty(q * rec, dtype=torch.uint8, device=dev)

        def scan():
            kernels.inner_product(db, n, rec, sel, q, ws, out)
        t = ev_time(scan, reps)
        res["q%d_ms" % q] = t * 1e3
        res["q%d_db_GBps" % q] = n * rec / t / 1e9
        res["q%d_hbm_frac" % q] = (n * rec + q * n // 8) / t / 8e12
        res["q%d_query_GBps" % q] = q * n * rec / t / 1e9
        if q >= 8 and C4Q_AB:
            # A/B of the two scan kernels (automatic choice timed above)
            ref = out.clone()
            for mode, name in ((0, "masked"), (1, "m4")):
                with kernels.forced_scan_m4(mode):
                    tm = ev_time(scan, reps)
                    res["q%d_%s_ms" % (q, name)] = tm * 1e3
                    res["q%d_%s_equal" % (q, name)] = bool(torch.equal(out, ref))
    del db
    return res


GRID_AVGS = (32, 256, 2048, 16384)
GRID_NS = (1 << 16, 1 << 20)
GRID_QS = (1, 2, 10, 100)
GRID_ALIGN = 0


def pirgrid(dev, reps):
    """The reference's dense-PIR benchmark grid
    (pir/dense_dpf_pir_database_benchmark.cc:125-157,
    BM_BatchedInnerProductOnVariableSizeValues): 2^16 / 2^20 records of 32 /
    256 / 2,048 / 16,384 B on average (sizes in [avg - 8, avg + 8), so rows of
    AlignBytes(avg + 7) bytes) at batches of 1, 2, 10, 100.  Per case: the
    scan alone on device-resident selections (HIP events; HBM fraction of
    rows + selections + results against 8 TB/s), and InnerProductWith through
    the API (host selections in, host results out; wall clock), whose
    results must equal the kernel's."""
    from distributed_point_functions_amd import pir as P
    gen = torch.Generator(device=dev)
    gen.manual_seed(125)
    rows = []
    for avg in GRID_AVGS:
        # the database's row stride for the largest value (pir.cc
        # DeviceRowStride: 16-byte aligned, whole 128-byte lines when that
        # costs at most 1/16 more), or a forced alignment (layout A/B)
        rec = (avg + 7 + 15) // 16 * 16
        if GRID_ALIGN > 16:
            rec = (rec + GRID_ALIGN - 1) // GRID_ALIGN * GRID_ALIGN
        elif GRID_ALIGN == 0 and ((rec + 127) // 128 * 128 - rec) * 16 <= rec:
            rec = (rec + 127) // 128 * 128
        for n in GRID_NS:
            db_t = torch.randint(0, 256, (n * rec,), dtype=torch.uint8, device=dev, generator=gen)
            db = P.DenseDpfPirDatabase()
            db.insert_fixed_device(db_t, n, rec).build()
            nb = n // 128
            for q in GRID_QS:
                sel = torch.randint(-2**63, 2**63 - 1, (q * nb, 2), dtype=torch.int64, device=dev,
                                    generator=gen)
                ws = torch.empty(max(16, _lib.lib().dpf_amd_inner_product_workspace_size(n, rec, q)),
                                 dtype=torch.uint8, device=dev)
                out = torch.empty(q * rec, dtype=torch.uint8, device=dev)

                def scan():
                    kernels.inner_product(db_t, n, rec, sel, q, ws, out)
                t = ev_time(scan, reps)
                host_sel = sel.cpu().numpy().view(np.uint64).reshape(q, nb, 2)
                api_res = []
                ta = wall_time(lambda: api_res.append(db.inner_product_with(host_sel)), reps)
                same = b"".join(api_res[-1]) == out.cpu().numpy().reshape(q, rec)[:, :rec].tobytes()
                algo = n * rec + q * nb * 16 + q * rec
                rows.append({"records": n, "avg_bytes": avg, "row_bytes": rec, "batch": q,
                             "scan_ms": t * 1e3, "scan_db_GBps": n * rec / t / 1e9,
                             "hbm_frac": algo / t / 8e12, "api_ms": ta * 1e3,
                             "api_db_GBps": n * rec / ta / 1e9, "api_equals_scan": same})
                del ws, sel, out
            del db, db_t
            torch.cuda.empty_cache()
    return {"config": "pirgrid",
            "workload": "dense_dpf_pir_database_benchmark.cc:125-157 grid (records x avg bytes x "
                        "batch), scan and InnerProductWith",
            "rows": rows}


def stride(dev, reps):
    """Dense scan at 2^26 rows with the reference's 16-byte-aligned row
    stride vs the same rows padded to a power-of-two / 1 KiB-multiple width,
    for 16 B and 1040 B records (why the builder stores rows
    unpadded)."""
    n = 1 << 26
    gen = torch.Generator(device=dev)
    gen.manual_seed(9)
    res = {"config": "stride", "workload": "XOR scan 2^26 rows, aligned vs padded stride"}
    for rec, aligned, padded in ((16, 16, 32), (1040, 1040, 2048)):
        db_a = torch.randint(0, 256, (n, aligned), dtype=torch.uint8, device=dev, generator=gen)
        db_p = torch.zeros((n, padded), dtype=torch.uint8, device=dev)
        db_p[:, :aligned] = db_a
        for q in (1, 16):
            sel = torch.randint(-2**63, 2**63 - 1, (q * (n // 128), 2), dtype=torch.int64,
                                device=dev, generator=gen)
            outs = []
            for name, db, st in (("aligned", db_a, aligned), ("padded", db_p, padded)):
                ws = torch.empty(max(16, _lib.lib().dpf_amd_inner_product_workspace_size(n, st, q)),
                                 dtype=torch.uint8, device=dev)
                out = torch.empty((q, st), dtype=torch.uint8, device=dev)
                t = ev_time(lambda: kernels.inner_product(db.view(-1), n, st, sel, q, ws,
                                                          out.view(-1)), reps)
                outs.append(out[:, :rec].clone())
                key = "r%d_%s_q%d" % (rec, name, q)
                res[key + "_ms"] = t * 1e3
                res[key + "_record_GBps"] = n * rec / t / 1e9
                del ws
            res["r%d_q%d_equal" % (rec, q)] = bool(torch.equal(outs[0], outs[1]))
        res["r%d_table_GB" % rec] = {"aligned": n * aligned / 1e9, "padded": n * padded / 1e9}
        del db_a, db_p
        torch.cuda.empty_cache()
    return res


def dcf(dev, reps):
    from distributed_point_functions_amd.dcf import DcfParameters, DistributedComparisonFunction
    rng = random.Random(5)
    n_log, nkeys = 32, 1024
    d = DistributedComparisonFunction.create(DcfParameters(DpfParameters(n_log, V.Integer(64))))
    alphas = [rng.getrandbits(n_log) for _ in range(nkeys)]
    betas = [rng.getrandbits(64) for _ in range(nkeys)]
    pairs = [d.generate_keys(a, b, seeds=(2 * i + 7, 2 * i + 8))
             for i, (a, b) in enumerate(zip(alphas, betas))]
    k0 = [p[0] for p in pairs]
    xs = [rng.getrandbits(n_log) for _ in range(nkeys)]
    t_api = wall_time(lambda: d.batch_evaluate(k0, xs, raw=True), max(1, reps // 2))
    r0 = d.batch_evaluate(k0, xs)
    r1 = d.batch_evaluate([p[1] for p in pairs], xs)
    ok = all((a + b) % (1 << 64) == (beta if x < al else 0)
             for a, b, x, al, beta in zip(r0, r1, xs, alphas, betas))
    # Tier 1: 2^20 evaluations, key i % 1024 at random points.
    H = n_log
    # the DCF's incremental DPF (log domains 0..n-1) gives the tree levels
    mirror = DistributedPointFunction.create_incremental(
        [DpfParameters(h, V.Integer(64)) for h in range(H)])
    tree_of = np.array([mirror.hierarchy_to_tree(h) for h in range(H)], dtype=np.int32)
    L = int(tree_of[-1])
    n = 1 << 20
    rep = n // nkeys
    seeds = np.zeros((nkeys, 2), np.uint64)
    cw = np.zeros((L, nkeys, 2), np.uint64)
    ccl = np.zeros((L, nkeys), np.uint8)
    ccr = np.zeros((L, nkeys), np.uint8)
    epb = 2  # ElementsPerBlock<uint64_t>: one value correction per element
    corr = np.zeros((H, nkeys, epb, 2), np.uint64)
    for i, k in enumerate(k0):
        dk = k.key
        seeds[i] = (dk.seed & M64, dk.seed >> 64)
        for a in range(L):
            c = dk.correction_words[a]
            cw[a, i] = (c.seed & M64, c.seed >> 64)
            ccl[a, i], ccr[a, i] = int(c.control_left), int(c.control_right)
        for h in range(H):
            vals = (dk.last_level_value_correction if h == H - 1
                    else dk.correction_words[int(tree_of[h])].value_correction)
            assert len(vals) == epb
            for e in range(epb):
                v = decode_value(V.Integer(64), vals[e])[0]
                corr[h, i, e] = (v & M64, v >> 64)
    tile = lambda a, axis: np.ascontiguousarray(np.repeat(a, rep, axis=axis))  # noqa: E731
    T = lambda a: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a).to(dev)  # noqa
    d_seeds = T(tile(seeds, 0))
    d_cb = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_party = torch.zeros(n, dtype=torch.int8, device=dev)
    pts = np.zeros((n, 2), np.uint64)
    pts[:, 0] = np.frombuffer(np.random.default_rng(6).bytes(8 * n), dtype=np.uint64) >> 32
    d_pts = T(pts)
    d_cw, d_ccl, d_ccr = T(tile(cw, 1)), T(tile(ccl, 1)), T(tile(ccr, 1))
    d_corr = T(tile(corr, 1))
    out = torch.empty(n * 8, dtype=torch.uint8, device=dev)
    desc = mirror.value_type_descriptor(H - 1)
    tree_c = tree_of.ctypes.data_as(ctypes.c_void_p)
    from distributed_point_functions_amd._lib import check, dptr, stream_ptr

    def run():
        check(_lib.lib().dpf_amd_dcf_evaluate(
            n, dptr(d_seeds), dptr(d_cb), dptr(d_party), dptr(d_pts), H, tree_c, dptr(d_cw),
            dptr(d_ccl), dptr(d_ccr), ctypes.byref(desc), dptr(d_corr), dptr(out),
            stream_ptr()))
    t_k = ev_time(run, reps)
    fused = out.clone()
    with kernels.forced_dcf_kernel(1):  # the generic kernel, for the record
        t_g = ev_time(run, reps)
    same = bool(torch.equal(out, fused))
    # algorithmic AES: tree levels + one value hash per 0 bit of the point
    zeros = sum(bin(int(x) ^ ((1 << H) - 1)).count("1") for x in pts[:4096, 0]) / 4096
    aes = n * (L + zeros)
    return {"config": "dcf", "workload": "DCF BatchEvaluate log_domain=32 uint64",
            "api_keys": nkeys, "api_ms": t_api * 1e3,
            "kernel_evaluations": n, "kernel_ms": t_k * 1e3,
            "kernel_evaluations_per_s": n / t_k, "generic_kernel_ms": t_g * 1e3,
            "kernels_equal": same, "aes_per_evaluation": aes / n,
            "lds_frac": aes * 160 / t_k / LDS_PEAK_LOOKUPS, "correct": bool(ok)}


def cuckoo(dev, reps):
    from distributed_point_functions_amd import cuckoo_pir as C
    from distributed_point_functions_amd import dpf as D
    n, vlen = 1 << 20, 240
    rng = np.random.default_rng(7)
    keys = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    vals = rng.integers(0, 256, (n, vlen), dtype=np.uint8)
    nb = int(1.5 * n)
    params = C.cuckoo_hashing_params(bytes(range(16)), nb)
    t0 = time.perf_counter()
    servers = []
    for _ in range(2):
        db = C.CuckooHashedDpfPirDatabase(params)
        for i in range(n):
            db.insert(keys[i].tobytes(), vals[i].tobytes())
        servers.append(C.CuckooHashingSparseDpfPirServer.create_plain(params, db))
    t_build = (time.perf_counter() - t0) / 2
    dpf = D.DistributedPointFunction.create(
        D.DpfParameters(max(0, (nb - 1).bit_length()), V.XorWrapper(128)))
    client = C.CuckooHashingSparseDpfPirClient(params, dpf)
    qi = [int(x) for x in rng.integers(0, n, 4)]
    queries = [keys[i].tobytes() for i in qi] + [b"not-a-stored-key"]
    r0, r1 = client.create_requests(queries)
    resp0 = servers[0].handle_request(r0)
    resp1 = servers[1].handle_request(r1)
    got = client.handle_responses(queries, resp0, resp1)
    # a key can be left in the unserved stash (reference semantics), so only
    # check that every served answer is the stored value
    ok = got[-1] is None and all(g is None or g == vals[i].tobytes()
                                 for g, i in zip(got, qi))
    served = sum(g is not None for g in got[:-1])
    t = wall_time(lambda: servers[0].handle_request(r0), reps)
    table_bytes = nb * (16 + vlen)
    return {"config": "cuckoo", "workload": "cuckoo-hashed sparse PIR, 2^20 x (16 B key, "
            "240 B value), 1.5x buckets, 3 hash functions",
            "queries_per_request": len(queries), "dpf_keys_per_request": 3 * len(queries),
            "handle_request_ms": t * 1e3,
            "table_GBps_per_key": 3 * len(queries) * table_bytes / t / 1e9,
            "db_build_s": t_build, "served": served, "correct": bool(ok)}


def cpp(dev, reps):
    """c1-c3 through the C++ API (tools/cpp_api_bench.cc, built by
    build_native against include/ and libdpf_amd.so) — what a reference
    caller would see; one JSON line per config."""
    import subprocess
    from distributed_point_functions_amd import build_native
    torch.cuda.synchronize()
    res = subprocess.run([build_native.CPP_BENCH, str(reps), "c1,c2,c2a,c3"], capture_output=True,
                         text=True, timeout=600)
    if res.returncode != 0:
        raise RuntimeError("cpp_api_bench failed: " + res.stderr[-2000:])
    lines = [json.loads(x) for x in res.stdout.splitlines() if x.startswith("{")]
    return {"config": "cpp", "workload": "C++ API c1, c2 (EvaluateAt, EvaluateAndApply), c3",
            "results": lines}


def cpp4(dev, reps):
    """c4 through the C++ API: DenseDpfPirServer::HandleRequest over 2^26 x
    256 B records at Q = 1, 8, 64 (tools/cpp_api_bench.cc)."""
    import subprocess
    from distributed_point_functions_amd import build_native
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    res = subprocess.run([build_native.CPP_BENCH, str(reps), "c4"], capture_output=True,
                         text=True, timeout=900)
    if res.returncode != 0:
        raise RuntimeError("cpp_api_bench c4 failed: " + res.stderr[-2000:])
    lines = [json.loads(x) for x in res.stdout.splitlines() if x.startswith("{")]
    return {"config": "cpp4", "workload": "C++ API c4 HandleRequest", "results": lines}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="c1,c2,c3,c4q,dcf,cuckoo,cpp")
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--c4q-queries", default=None, help="comma list, e.g. 64 (profiling)")
    ap.add_argument("--no-ab", action="store_true", help="c4q: skip the kernel A/B")
    ap.add_argument("--c2-batched-only", action="store_true", help="c2: the batched kernel only")
    ap.add_argument("--grid-align", type=int, default=0,
                    help="pirgrid: row stride rounded up to this many bytes (layout A/B; "
                         "0: the database's own rule)")
    ap.add_argument("--grid", default=None,
                    help="pirgrid subset as avg:n:q lists, e.g. 16384:1048576:1 (profiling)")
    args = ap.parse_args()
    global C4Q_QUERIES, C4Q_AB, C2_BATCHED_ONLY, GRID_AVGS, GRID_NS, GRID_QS, GRID_ALIGN
    GRID_ALIGN = args.grid_align
    if args.grid:
        a, n, q = args.grid.split(":")
        GRID_AVGS = tuple(int(x) for x in a.split(","))
        GRID_NS = tuple(int(x) for x in n.split(","))
        GRID_QS = tuple(int(x) for x in q.split(","))
    C2_BATCHED_ONLY = args.c2_batched_only
    if args.c4q_queries:
        C4Q_QUERIES = tuple(int(x) for x in args.c4q_queries.split(","))
    C4Q_AB = not args.no_ab
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for name in args.only.split(","):
        r = globals()[name](dev, args.reps)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
