"""Benchmark of the MI355X DPF / dense-PIR hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Headline (`value`): full-domain DPF evaluation leaves/s over the whole job —
config c5 of BASELINE.json: one key, log_domain_size = 32,
Tuple<uint32, IntModN<uint64, 2^64-59>>, security_parameter = 48
(EvaluateNext({}, ctx), dpf/distributed_point_function.h:695-891), 2^32
leaves per step, outputs kept in HBM in the host layout of the type.
With N ranks the key's domain is subtree-sharded (BASELINE.json c5): rank r
expands tree blocks [r 2^32/N, (r+1) 2^32/N) — its own prefix walk, disjoint
outputs, no collective on the data path; `value` = 2^32 leaves / the
max-over-ranks step time (strong scaling).

Secondary (`pir`): dense PIR config c4 — 2^26 records x 256 B, one query:
the Tier-1 selection expansion (only the ceil(N/128) leaves the scan reads)
+ the XOR scan over the whole database; rows sharded over ranks, the Q x 256
B partials are all-gathered with RCCL and XOR-folded.  GB/s = database
bytes / time per query.  `pir.handle_request` (one rank) times the
reference API itself, DenseDpfPirServer::HandleRequest through the C ABI
(wire decode, key validation, expansion, scan, response encode) at Q = 1, 8,
64 — the batch shapes of pir/dense_dpf_pir_database_benchmark.cc:37-157.

--in-process: one process drives all N GPUs through the library's own
multi-GPU entry points (ExpandLeavesOnDevices for c5; a DenseDpfPirDatabase
sharded over the N devices behind HandleRequest for c4) instead of one
process per GPU.

`cpu_baseline` times the oracle (the C restatement of the reference CPU
algorithm, AES-NI) single-threaded on a bounded slice of the same workload.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import time

import numpy as np
import torch
import torch.distributed as dist

from distributed_point_functions_amd import _lib, kernels, sharding
from distributed_point_functions_amd import value_types as V
from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters, decode_value

METRIC = ("DPF full-domain leaves/sec at 2^32 (whole node); "
          "dense-PIR scan GB/s at 1/2/4/8")
P64 = 2 ** 64 - 59
HBM_PEAK_GBS = 8000.0          # MI355X spec (MI355X_MICROARCH.md)
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # 78.64 T int32 lane-ops/s
OPS_PER_AES = 757.5            # bitsliced AES-128 gate count
LDS_LOOKUPS_PER_AES = 160      # T-table lookups per AES block
LDS_PEAK_LOOKUPS = 256 * 32 * 2.4e9  # ds_read_b32: 32 lane-lookups/clk/CU
AES_PER_LEAF_C5 = 4.0          # 2(2^32-1) tree + 2 * 2^32 value AES per 2^32 leaves
# T-table lookups per c5 leaf: 2 x 160 (tree children) + 160 + 121 (the value
# PRG pair seed, seed + 1 shares 27 lookups of rounds 1-2, and only word 0 of
# the second value block is used, so the compiler drops 12 of its 16
# last-round lookups — DESIGN.md §3.1).  Measured SQ_INSTS_LDS x 64 / leaf:
# 615 = 601 + the root-to-subtree walk (24 AES per 256-leaf subtree).
LDS_LOOKUPS_PER_LEAF_C5 = 601
# I_AES: VALU lane-instructions per AES block of the c5
# kernel, SQ_INSTS_VALU x 64 / (4 x 2^32) of profiles/r04g_pmc.json; the
# bench line recomputes it from a PMC profile of the loaded build when one
# is committed.
I_AES_C5 = 307.2


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, flush=True)


def bench_backend():
    return os.environ.get("DPF_AMD_BENCH_BACKEND", "nccl")


def launch_decision(args, env, device_count):
    """How `bench.py --gpus N` gets its N ranks, decided before any GPU call.

    Returns ("run", None) when this process is the whole job or one rank of
    an already launched one (WORLD_SIZE set), ("spawn", N) when it must start
    N rank processes itself (--gpus N > 1 and no WORLD_SIZE), or ("error",
    message) when the request cannot be honoured: a world size that is not
    --gpus, or more RCCL ranks than visible GPUs.  --in-process and
    --experiments / --library-multi-device drive their devices from this one
    process."""
    if args.in_process or args.experiments or args.library_multi_device:
        return "run", None
    world = env.get("WORLD_SIZE")
    if world is not None:
        if int(world) != args.gpus:
            return "error", ("launched with WORLD_SIZE=%s but --gpus %d: the line would not "
                             "describe the job" % (world, args.gpus))
        return "run", None
    if args.gpus <= 1:
        return "run", None
    if env.get("DPF_AMD_BENCH_BACKEND", "nccl") == "nccl" and args.gpus > device_count:
        return "error", ("--gpus %d with RCCL needs %d GPUs, %d visible (set "
                         "DPF_AMD_BENCH_BACKEND=gloo to rehearse N ranks on fewer GPUs)"
                         % (args.gpus, args.gpus, device_count))
    return "spawn", args.gpus


def spawn_ranks(n, argv):
    """Start the N-rank job as a child (torch.distributed.run on 127.0.0.1,
    one process per GPU) and return its exit code; rank 0 prints the line.
    This process has not touched the GPU, and it does not exec."""
    import socket
    import subprocess
    import sys
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=%d" % n, "--master-addr=127.0.0.1", "--master-port=%d" % port,
           os.path.abspath(__file__)] + list(argv)
    print("[bench] --gpus %d without WORLD_SIZE: starting %d rank processes (%s)"
          % (n, n, " ".join(cmd[1:5])), flush=True)
    return subprocess.call(cmd)


def setup():
    """One process per GPU over RCCL.  DPF_AMD_BENCH_BACKEND=gloo rehearses
    the N-rank data path on fewer GPUs (ranks share devices round-robin;
    collectives through host memory) — a correctness check of the sharding,
    not a measurement."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = bench_backend()
    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != world:
            raise SystemExit("process group has %d ranks, WORLD_SIZE=%d"
                             % (dist.get_world_size(), world))
    return world, rank, torch.device("cuda", local)


def rank_devices(world, device):
    """[(rank, device index, PCI bus id)] of every rank, gathered to all."""
    props = torch.cuda.get_device_properties(device)
    mine = (int(os.environ.get("RANK", "0")), device.index,
            "%04x:%02x:%02x" % (getattr(props, "pci_domain_id", 0),
                                getattr(props, "pci_bus_id", 0),
                                getattr(props, "pci_device_id", 0)))
    if world == 1:
        return [mine]
    out = [None] * world
    dist.all_gather_object(out, mine)
    return out


def barrier(world):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def key_arrays(dpf, key, level, device):
    """Device arrays of a DpfKey for the Tier-1 expansion seam."""
    L = dpf.hierarchy_to_tree(level)
    cws = key.correction_words[:L]
    vt = dpf.parameters[level].value_type
    vcs = key.last_level_value_correction
    corr = [x for v in vcs for x in decode_value(vt, v)]
    return dict(
        L=L,
        seed=kernels.u128_tensor([key.seed], device),
        cb=torch.tensor([key.party], dtype=torch.uint8, device=device),
        cw=kernels.u128_tensor([c.seed for c in cws], device),
        ccl=torch.tensor([int(c.control_left) for c in cws] or [0], dtype=torch.uint8, device=device),
        ccr=torch.tensor([int(c.control_right) for c in cws] or [0], dtype=torch.uint8, device=device),
        corr=corr, party=key.party)


def bench_dpf(args, world, rank, device):
    vt = V.Tuple(V.Integer(32), V.IntModN(64, P64))
    log_domain = args.log_domain
    dpf = DistributedPointFunction.create(DpfParameters(log_domain, vt, 48))
    alpha = 0x9E3779B9 % (1 << log_domain)
    # one key, the one the CPU baseline times
    k0, _ = dpf.generate_keys(alpha, (123456789, 987654321), seeds=(0xA5A5, 0x5A5A))
    ka = key_arrays(dpf, k0, 0, device)
    desc = dpf.value_type_descriptor(0)
    L = ka["L"]
    cepb = 1 << (log_domain - L)
    total = 1 << L
    lo, hi = sharding.block_range(total, world, rank)  # this rank's subtrees
    out = torch.empty((hi - lo) * cepb * desc.out_stride, dtype=torch.uint8, device=device)

    def step():
        kernels.expand_and_correct(ka["seed"], ka["cb"], L, ka["cw"], ka["ccl"], ka["ccr"],
                                   desc, ka["corr"], ka["party"], cepb, lo, hi, out)

    for _ in range(args.warmup):
        step()
    barrier(world)
    st = torch.cuda.current_stream()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(st)
    for _ in range(args.steps):
        step()
    ev1.record(st)
    barrier(world)
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps
    wall = max_over_ranks(wall, world)
    kernel_ms = max_over_ranks(kernel_ms, world)
    leaves = total * cepb  # the whole domain, over all ranks
    return dict(wall=wall, kernel_ms=kernel_ms, leaves=leaves, L=L, lo=lo, hi=hi)


def bench_pir(args, world, rank, device):
    n = 1 << args.pir_log_records
    rec = 256
    r_lo, r_hi, b_lo, b_hi = sharding.pir_row_shard(n, world, rank)
    per = r_hi - r_lo
    gen = torch.Generator(device=device)
    gen.manual_seed(1234 + rank)
    db = torch.randint(0, 256, (per * rec,), dtype=torch.uint8, device=device, generator=gen)
    log_domain = max(0, (n - 1).bit_length())
    dpf = DistributedPointFunction.create(DpfParameters(log_domain, V.XorWrapper(128)))
    idx = (n * 3) // 7 + 5
    k0, k1 = dpf.generate_keys(idx // 128, 1 << (idx % 128), seeds=(0x1111, 0x2222))
    desc = dpf.value_type_descriptor(0)
    keys = [key_arrays(dpf, k, 0, device) for k in (k0, k1)]
    sel = torch.empty(max(1, b_hi - b_lo) * 16, dtype=torch.uint8, device=device)
    ws = torch.empty(max(16, _lib.lib().dpf_amd_inner_product_workspace_size(per, rec, 1)),
                     dtype=torch.uint8, device=device)
    part = torch.empty(rec, dtype=torch.uint8, device=device)
    scan_ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def query(ka, timed_scan=False):
        kernels.expand_and_correct(ka["seed"], ka["cb"], ka["L"], ka["cw"], ka["ccl"], ka["ccr"],
                                   desc, ka["corr"], ka["party"], 1, b_lo, b_hi, sel)
        if timed_scan:
            scan_ev[0].record()
        kernels.inner_product(db, per, rec, sel.view(torch.int64).view(-1, 2), 1, ws, part)
        if timed_scan:
            scan_ev[1].record()
        return sharding.allgather_xor(part, world)

    # correctness: share0 ^ share1 == record idx (held by its owner rank)
    a = query(keys[0]).clone()
    b = query(keys[1]).clone()
    rec_idx = torch.zeros(rec, dtype=torch.uint8, device=device)
    if r_lo <= idx < r_hi:
        rec_idx.copy_(db[(idx - r_lo) * rec:(idx - r_lo + 1) * rec])
    if world > 1:
        if dist.get_backend() == "nccl":
            dist.all_reduce(rec_idx, op=dist.ReduceOp.SUM)
        else:
            h = rec_idx.cpu().to(torch.int32)
            dist.all_reduce(h, op=dist.ReduceOp.SUM)
            rec_idx.copy_(h.to(torch.uint8))
    ok = bool(torch.equal(a ^ b, rec_idx))
    for _ in range(args.warmup):
        query(keys[0])
    barrier(world)
    scan_ms = 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        query(keys[0], timed_scan=True)
        torch.cuda.synchronize()
        scan_ms += scan_ev[0].elapsed_time(scan_ev[1])
    barrier(world)
    wall = max_over_ranks(time.perf_counter() - t0, world) / args.steps
    scan_ms = max_over_ranks(scan_ms / args.steps, world)
    # The opt-in scan that reads only the selected records, as the
    # reference's InnerProduct does (inner_product_hwy.cc:213-221; the access
    # pattern then follows the selection share): reported beside the
    # default constant-time scan, never as the line's figures.
    skip = None
    if not args.skip_scan_skip:
        with kernels.scan_skip_unselected(1):
            a2 = query(keys[0]).clone()
            b2 = query(keys[1]).clone()
            sok = bool(torch.equal(a2 ^ b2, rec_idx))
            query(keys[0])
            nsel = int(np.unpackbits(sel.cpu().numpy()).sum())  # this rank's selected rows
            for _ in range(args.warmup):
                query(keys[0])
            barrier(world)
            sms = 0.0
            t0 = time.perf_counter()
            for _ in range(args.steps):
                query(keys[0], timed_scan=True)
                torch.cuda.synchronize()
                sms += scan_ev[0].elapsed_time(scan_ev[1])
            barrier(world)
            swall = max_over_ranks(time.perf_counter() - t0, world) / args.steps
            sms = max_over_ranks(sms / args.steps, world)
        skip = dict(ok=sok, wall_s=swall, scan_ms=sms, selected_rows=nsel,
                    read_bytes=nsel * rec + (b_hi - b_lo) * 16)
    # a 64-query batch over the same resident rows (the reference batches up
    # to 100 queries: pir/dense_dpf_pir_database_benchmark.cc): the
    # Four-Russians scan (KPirScanM4), random selection shares
    mq = 64
    msel = torch.randint(-2**63, 2**63 - 1, (mq * max(1, b_hi - b_lo), 2), dtype=torch.int64,
                         device=device, generator=gen)
    mws = torch.empty(max(16, _lib.lib().dpf_amd_inner_product_workspace_size(per, rec, mq)),
                      dtype=torch.uint8, device=device)
    mout = torch.empty(mq * rec, dtype=torch.uint8, device=device)
    kernels.inner_product(db, per, rec, msel, mq, mws, mout)
    barrier(world)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(args.steps):
        kernels.inner_product(db, per, rec, msel, mq, mws, mout)
    ev[1].record()
    barrier(world)
    mq_ms = max_over_ranks(ev[0].elapsed_time(ev[1]) / args.steps, world)
    del mws, msel, mout, ws, sel
    hr = shard = None
    if world == 1 and not args.skip_handle_request:
        torch.cuda.empty_cache()
        hr = bench_handle_request(args, n, rec, db, device)
        # one rank's share at N = 8 as a database of its own (2^23 records of
        # c4): the whole request on the shard, the per-GPU time of a node
        if n >= 8 * 128:
            torch.cuda.empty_cache()
            shard = (n // 8, bench_handle_request(args, n // 8, rec, db[:(n // 8) * rec], device,
                                                  queries=(1, 8)))
    return dict(ok=ok, wall_s=wall, scan_ms=scan_ms, db_bytes=n * rec, per_gpu_bytes=per * rec,
                records=n, mq=mq, mq_ms=mq_ms, hr=hr, shard=shard, skip=skip)


def bench_handle_request(args, n, rec, db_tensor, device, shard_devices=None,
                         queries=(1, 8, 64)):
    """DenseDpfPirServer::HandleRequest (pir/dense_dpf_pir_server.cc:92-127)
    through the C ABI, end to end per request: PirRequest wire decode, key
    validation, the selection expansion, the scan, PirResponse encode and the
    copy of the response to the host.  The database is built from the
    resident rows (device to device).  Returns {Q: ms per request}, and
    whether both parties' responses reconstruct every queried record."""
    from distributed_point_functions_amd import pir as P
    db = P.DenseDpfPirDatabase(shard_devices)
    db.insert_fixed_device(db_tensor, n, rec).build()
    server = P.DenseDpfPirServer.create_plain(n, db)
    log_domain = max(0, (n - 1).bit_length())
    dpf = DistributedPointFunction.create(DpfParameters(log_domain, V.XorWrapper(128)))
    rng = np.random.default_rng(77)
    out, ok = {}, True
    for q in queries:
        idx = [int(i) for i in rng.integers(0, n, q)]
        pairs = P.client_keys(dpf, n, idx, seeds=[(7 + 2 * j, 8 + 2 * j) for j in range(q)])
        req0 = P.pir_request_plain([a for a, _ in pairs])
        r0 = P.parse_response(server.handle_request(req0))  # warm-up
        # both parties' responses reconstruct every queried record
        r1 = P.parse_response(server.handle_request(P.pir_request_plain([b for _, b in pairs])))
        for j, i in enumerate(idx):
            want = db_tensor[i * rec:(i + 1) * rec].cpu().numpy().tobytes()
            ok = ok and bytes(x ^ y for x, y in zip(r0[j], r1[j])) == want
        reps = max(3, args.steps)
        t0 = time.perf_counter()
        for _ in range(reps):
            server.handle_request(req0)
        out[q] = 1e3 * (time.perf_counter() - t0) / reps
        if q == 1 and not getattr(args, "skip_scan_skip", True):
            # the same request with the opt-in skip of unselected records
            with kernels.scan_skip_unselected(1):
                s0 = P.parse_response(server.handle_request(req0))
                ok = ok and s0 == r0
                t0 = time.perf_counter()
                for _ in range(reps):
                    server.handle_request(req0)
                out["1_skip_unselected"] = 1e3 * (time.perf_counter() - t0) / reps
    del server, db
    return out, ok


def bench_in_process(args):
    """All N GPUs from one process through the library's multi-GPU API."""
    from distributed_point_functions_amd import pir as P
    devs = ([int(d) for d in args.devices.split(",")] if args.devices
            else list(range(args.gpus)))
    ngpu = len(devs)
    vt = V.Tuple(V.Integer(32), V.IntModN(64, P64))
    dpf = DistributedPointFunction.create(DpfParameters(args.log_domain, vt, 48))
    alpha = 0x9E3779B9 % (1 << args.log_domain)
    k0, _ = dpf.generate_keys(alpha, (123456789, 987654321), seeds=(0xA5A5, 0x5A5A))
    total = 1 << dpf.hierarchy_to_tree(0)
    slices = []
    for i, d in enumerate(devs):
        lo, hi = sharding.block_range(total, ngpu, i)
        slices.append((d, lo, hi, torch.empty((hi - lo) * 16, dtype=torch.uint8,
                                              device=torch.device("cuda", d))))
    for _ in range(args.warmup):
        dpf.expand_leaves_on_devices(k0, slices)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dpf.expand_leaves_on_devices(k0, slices)  # returns when every GPU is done
    wall = time.perf_counter() - t0
    del slices
    torch.cuda.empty_cache()
    pir = None
    if not args.skip_pir:
        n, rec = 1 << args.pir_log_records, 256
        gen = torch.Generator(device="cuda:0")
        gen.manual_seed(1234)
        src = torch.randint(0, 256, (n * rec,), dtype=torch.uint8, device="cuda:0", generator=gen)
        hr, ok = bench_handle_request(args, n, rec, src, torch.device("cuda", 0), devs)
        pir = dict(ms=hr, ok=ok, n=n, rec=rec)
    return dict(wall=wall, leaves=total, L=dpf.hierarchy_to_tree(0), pir=pir)


GOLDEN_C5 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden",
                         "c5_subtree_digests.json")
# torchrun's per-rank variables: the library_multi_device child is one
# process driving every device, not a rank
RANK_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
            "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT",
            "TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS", "TORCHELASTIC_RUN_ID",
            "TORCHELASTIC_USE_AGENT_STORE", "TORCHELASTIC_ERROR_FILE", "TORCH_NCCL_ASYNC_ERROR_HANDLING")


def bench_library_multi_device(args):
    """bench.py --library-multi-device (the child rank 0 starts at world > 1):
    the library's own multi-device entry points, one process over every
    device, checked on the spot.
      * c5: DistributedPointFunction::ExpandLeavesOnDevices of the full 2^32
        domain over the devices (disjoint subtree slices, one stream per
        device) for the key tests/golden/c5_subtree_digests.json was made
        from; sampled 2^20-leaf subtrees of every slice (its first, its last,
        a random one and alpha's) hashed and compared with the oracle's
        SHA-256 digests.
      * c4: a DenseDpfPirDatabase sharded over the devices (rows copied to
        each shard's device, partials peer-copied to the first device and
        XOR-folded, csrc/pir.cc) behind DenseDpfPirServer::HandleRequest
        (pir/dense_dpf_pir_server.cc:92-127) at Q = 1 and 8; both parties'
        responses reconstruct every queried record.
    Prints one JSON line {"library_multi_device": {...}}."""
    import hashlib
    import random
    from distributed_point_functions_amd import pir as P
    devs = [int(d) for d in args.devices.split(",")]
    with open(GOLDEN_C5) as f:
        gold = json.load(f)
    vt = V.Tuple(V.Integer(32), V.IntModN(64, P64))
    dpf = DistributedPointFunction.create(
        DpfParameters(gold["log_domain_size"], vt, gold["security_parameter"]))
    alpha = gold["alpha"]
    k0, _ = dpf.generate_keys(alpha, tuple(gold["beta"]),
                              seeds=tuple(int(x) for x in gold["keygen_seeds"]))
    total = 1 << dpf.hierarchy_to_tree(0)
    slices = []
    for i, d in enumerate(devs):
        lo, hi = sharding.block_range(total, len(devs), i)
        slices.append((d, lo, hi, torch.empty((hi - lo) * 16, dtype=torch.uint8,
                                              device=torch.device("cuda", d))))
    dpf.expand_leaves_on_devices(k0, slices)  # the checked output (and the warm-up)
    log_sub = gold["log_subtree_leaves"]
    want = gold["sha256"]["0"]
    rng = random.Random(2026)
    checked, bad = 0, []
    for d, lo, hi, out in slices:
        first, last = (lo + (1 << log_sub) - 1) >> log_sub, (hi >> log_sub) - 1  # whole subtrees
        if last < first:
            continue
        subs = {first, last, rng.randint(first, last)}
        if first <= alpha >> log_sub <= last:
            subs.add(alpha >> log_sub)
        for sub in sorted(subs):
            a = ((sub << log_sub) - lo) * 16
            got = hashlib.sha256(out[a:a + (16 << log_sub)].cpu().numpy()).hexdigest()
            checked += 1
            if got != want[sub]:
                bad.append(sub)
    for _ in range(max(0, args.warmup - 1)):
        dpf.expand_leaves_on_devices(k0, slices)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dpf.expand_leaves_on_devices(k0, slices)  # returns when every device is done
    c5_s = (time.perf_counter() - t0) / args.steps
    del slices
    torch.cuda.empty_cache()
    c5 = {"api": "DistributedPointFunction::ExpandLeavesOnDevices (dpf_amd_expand_leaves_on_devices)",
          "leaves": total, "ms_per_step": 1e3 * c5_s, "leaves_per_s": total / c5_s,
          "subtrees_checked": checked, "subtrees_differing": bad,
          "check": "SHA-256 of sampled 2^%d-leaf subtrees vs tests/golden/c5_subtree_digests.json "
                   "(oracle)" % log_sub,
          "correct": checked > 0 and not bad}
    n, rec = 1 << args.pir_log_records, 256
    gen = torch.Generator(device=torch.device("cuda", devs[0]))
    gen.manual_seed(1234)
    src = torch.randint(0, 256, (n * rec,), dtype=torch.uint8,
                        device=torch.device("cuda", devs[0]), generator=gen)
    hr, hr_ok = bench_handle_request(args, n, rec, src, torch.device("cuda", devs[0]), devs,
                                     queries=(1, 8))
    del src
    torch.cuda.empty_cache()
    c4 = {"api": "DenseDpfPirServer::HandleRequest (dpf_amd_pir_server_handle_request), "
                 "DenseDpfPirDatabase sharded over the devices",
          "records": n, "record_bytes": rec,
          "ms_per_request": {str(q): v for q, v in hr.items()},
          "db_GBps_at_q1": n * rec / (hr[1] / 1e3) / 1e9,
          "check": "both parties' responses XOR to every queried record", "correct": hr_ok}
    return {"devices": devs, "distinct_gpus": len(set(devs)), "force_peer": bool(args.force_peer),
            "c5": c5, "c4": c4, "correct": bool(c5["correct"] and c4["correct"])}


def library_multi_device_cmd(ranks, args):
    """The child's command line: every rank's device, in rank order; peer
    copies forced when ranks share a device (a rehearsal of N devices on
    fewer GPUs), so the cross-device branches still run."""
    import sys
    devs = [d for _, d, _ in sorted(ranks)]
    cmd = [sys.executable, "-u", os.path.abspath(__file__), "--library-multi-device",
           "--devices", ",".join(str(d) for d in devs), "--steps", str(args.steps),
           "--warmup", str(args.warmup), "--log-domain", str(args.log_domain),
           "--pir-log-records", str(args.pir_log_records)]
    if len(set(devs)) < len(devs):
        cmd.append("--force-peer")
    return cmd


def run_library_multi_device(cmd, timeout_s):
    """Runs the library_multi_device child (a fresh process: never an exec
    of this one) and returns its result for the bench line, or — when it
    fails, hangs past `timeout_s` or prints no result — a dict with
    correct: false and the error, so the line is always complete."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in RANK_ENV}
    t0 = time.perf_counter()
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s, env=env)
    except subprocess.TimeoutExpired as e:
        tail = e.stderr.decode(errors="replace") if isinstance(e.stderr, bytes) else (e.stderr or "")
        return {"correct": False, "error": "child killed after its %d s limit" % timeout_s,
                "stderr_tail": tail[-1500:], "child_s": time.perf_counter() - t0}
    except OSError as e:
        return {"correct": False, "error": "child could not start: %s" % e}
    el = time.perf_counter() - t0
    for line in reversed(p.stdout.splitlines()):
        if not line.startswith("{"):
            continue
        try:
            d = json.loads(line)
        except ValueError:
            continue
        if isinstance(d, dict) and isinstance(d.get("library_multi_device"), dict):
            r = d["library_multi_device"]
            r["child_rc"], r["child_s"] = p.returncode, el
            if p.returncode != 0:
                r["correct"] = False
                r.setdefault("error", "child exit code %d" % p.returncode)
            return r
    return {"correct": False, "child_rc": p.returncode, "child_s": el,
            "error": "child exit code %d without a result line" % p.returncode,
            "stderr_tail": (p.stderr or "")[-1500:]}


def m4_lds_roofline(db_bytes, q, ms, clock_ghz=2.4):
    """LDS floor of one KPirScanM4 pass over `db_bytes` for q <= 64 queries:
    (15 x 256 B / 128 B/clk + q x 256 B / 256 B/clk) per 4 records of 256 B,
    at the 2.4 GHz peak clock and at the clock the profile of this build
    measured under the kernel."""
    kib = db_bytes / 1024
    cycles_per_kib = 15 * 2 + q

    def floor(ghz):
        return kib * cycles_per_kib / (256 * ghz * 1e9) * 1e3
    out = {"bound": "lds", "cycles_per_kib": cycles_per_kib, "clock_ghz": clock_ghz,
           "floor_ms": floor(clock_ghz), "frac": floor(clock_ghz) / ms}
    clk = clock_view(traffic_from_profiles(SCAN_M4_KERNEL_RE)[2])
    if clk:
        out["measured"] = dict(clk, frac_at_measured_clock=floor(clk["clock_ghz"]) / ms)
    return out


def library_sha256():
    import hashlib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def library_identity():
    """The loaded library: its sha256 (what profiles/ are keyed to), the
    source hash stamped into it at build time (dpf_amd_version) and whether
    that is the hash of the csrc/ and include/ in this tree."""
    from distributed_point_functions_amd import build_native
    stamped = _lib.lib().dpf_amd_version().decode().rsplit("src:", 1)[-1]
    try:
        tree = build_native.source_hash()
    except OSError:
        tree = None
    return {"sha256": library_sha256(), "source_hash": stamped, "tree_source_hash": tree,
            "matches_sources": stamped == tree}


def traffic_from_profiles(kernel_re):
    """(HBM bytes per launch, profile file, PMC entry, error) of the kernel
    whose demangled name matches the regex `kernel_re`, from a committed PMC
    summary of THIS build (profiles/<round>_pmc.json, written by
    tools/summarize_profile.py from separate rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes of this bench, keyed by the profiled library's
    sha256).  When nothing matches, the first three are None and `error`
    says why (no summary of this library, or the kernel is not in it), so
    the bench line never carries a silent null."""
    import glob
    import re
    pat = re.compile(kernel_re)
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                          "profiles", "r*_pmc.json")), key=os.path.getmtime)
    sha = library_sha256()
    keyed = []
    for f in reversed(files):
        with open(f) as fh:
            d = json.load(fh)
        if d.get("_meta", {}).get("library_sha256") != sha:
            continue
        keyed.append(os.path.basename(f))
        for name, e in d.items():
            if pat.search(name) and isinstance(e, dict) and "hbm_bytes" in e:
                # a kernel profiled at several launch sizes (the c4 scan beside
                # the c4/8 shard request): the bench's leg is its largest launch
                big = e.get("largest_launches")
                if isinstance(big, dict) and "hbm_bytes" in big:
                    return big["hbm_bytes"], os.path.basename(f), big, None
                return e["hbm_bytes"], os.path.basename(f), e, None
    if not keyed:
        err = ("no profiles/r*_pmc.json is keyed to the loaded library (sha256 %s): "
               "profile this build with tools/profile_gpu.sh" % sha[:16])
    else:
        err = "kernel /%s/ not found in %s" % (kernel_re, ", ".join(keyed))
    return None, None, None, err


# Demangled kernel names as rocprofv3 reports them; template arguments after
# the ones that identify the launch are matched loosely.
EXPAND_C5_KERNEL_RE = r"KExpand<8, dpf_amd::EmitU32ModN64(, [^>]*)?>"
SCAN_Q1_KERNEL_RE = r"KPirScanG<1, 4(, [^>]*)?>"
SCAN_M4_KERNEL_RE = r"KPirScanM4<1>"


def clock_view(entry):
    """Shader clock and LDS-array busy fraction of a kernel from its PMC
    entry (GRBM_GUI_ACTIVE counts per XCD: / 8 XCDs / kernel time;
    SQ_LDS_IDX_ACTIVE counts LDS-array cycles over all 256 CUs)."""
    if not entry:
        return None
    c = entry.get("counters_per_launch", {})
    ns = entry.get("avg_duration_ns")
    if not ns or "GRBM_GUI_ACTIVE" not in c:
        return None
    cycles = c["GRBM_GUI_ACTIVE"] / 8.0
    out = {"clock_ghz": cycles / ns}
    if "SQ_LDS_IDX_ACTIVE" in c:
        out["lds_array_busy"] = c["SQ_LDS_IDX_ACTIVE"] / 256.0 / cycles
    if "SQ_INSTS_VALU" in c:
        out["valu_issue_busy"] = c["SQ_INSTS_VALU"] * 2.0 / 1024.0 / cycles
    return out


def valu_view(aes_s, entry):
    """VALU lane-instructions per second of the c5 kernel against the issue
    peak, with I_AES from the PMC entry of this build (its launch covers the
    whole 2^32 domain: 4 x 2^32 AES) or the frozen round-4 figure."""
    i_aes, src = I_AES_C5, "frozen: profiles/r04g_pmc.json"
    c = (entry or {}).get("counters_per_launch", {})
    if "SQ_INSTS_VALU" in c:
        i_aes, src = c["SQ_INSTS_VALU"] * 64 / (AES_PER_LEAF_C5 * 2 ** 32), "PMC of this build"
    achieved = aes_s * i_aes
    return {"i_aes": i_aes, "i_aes_source": src, "achieved": achieved / 1e12,
            "peak": VALU_PEAK_TOPS, "unit": "T lane-instructions/s",
            "frac": achieved / (VALU_PEAK_TOPS * 1e12)}


def _cpu_worker(job):
    """One CPU-baseline process: oracle expansion of 2^20-leaf subtrees
    first, first + stride, ... of the c5 key for `seconds`."""
    log_domain, first, stride, seconds = job
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle import pyoracle as po
    spec = ("tuple", [("int", 32), ("intmodn", 64, P64)])
    d = po.Dpf([(log_domain, spec, 48)])
    k0, _ = d.generate_keys(0x9E3779B9 % (1 << log_domain), [(123456789, 987654321)],
                            seeds=(0xA5A5, 0x5A5A))
    log_blocks = min(20, d.hierarchy_to_tree(0))
    nsub = 1 << (d.hierarchy_to_tree(0) - log_blocks)
    buf = np.zeros(2 * 2 * (1 << log_blocks), dtype=np.uint64)
    leaves, t0, i = 0, time.perf_counter(), first
    while True:
        d.expand_subtree_words(k0, (i % nsub) << log_blocks, log_blocks, buf)
        leaves += 1 << log_blocks
        i += stride
        el = time.perf_counter() - t0
        if el >= seconds or leaves >= (4096 << log_blocks):
            break
    return leaves, el, log_blocks, po.lib().or_have_aesni()


def cpu_baseline(args):
    """Oracle (reference CPU algorithm restated in C, AES-NI) on a bounded
    slice of the c5 workload: 2^20-leaf subtrees of the same 2^32-domain key.
    1 thread for >= args.cpu_seconds (the reference is single-threaded), and
    the same work split over the box's host cores (one process per core, up
    to 16 — the GPU box's CPU share) for half that time."""
    leaves, el, log_blocks, aesni = _cpu_worker((args.log_domain, 0, 1, args.cpu_seconds))
    out = dict(value=leaves / el, unit="leaves/s", cores=1, kind="port",
               sample="%d x 2^%d-leaf subtrees of the c5 key (%.1f s), oracle/dpf_oracle.c "
                      "ExpandSeeds+HashExpandedSeeds+correction, AES-NI %s" %
                      (leaves >> log_blocks, log_blocks, el, "on" if aesni else "off"))
    procs = max(1, min(16, os.cpu_count() or 1))
    if procs > 1:
        import multiprocessing as mp
        secs = max(2.0, args.cpu_seconds / 2)
        with mp.get_context("spawn").Pool(procs) as pool:
            res = pool.map(_cpu_worker, [(args.log_domain, p, procs, secs) for p in range(procs)])
        out["multicore"] = dict(value=sum(r[0] / r[1] for r in res), unit="leaves/s",
                                cores=procs,
                                sample="%d concurrent processes x ~%.0f s on disjoint subtrees "
                                       "(sum of per-process rates)" % (procs, secs))
    return out


# --- the reference's published experiments (experiments/README.md:20-108) ---

EXPERIMENT_PUBLISHED_S = {  # one key, 1 thread of a 2.3 GHz Xeon (README tables)
    (32, "hierarchical"): {"0.1": 1.36, "0.5": 2.22, "uniform": 3.31},
    (32, "direct"): {"0.1": 0.67, "0.5": 0.68, "uniform": 0.70},
    (128, "hierarchical"): {"0.1": 32.68, "0.5": 35.07, "uniform": 35.95},
    (128, "direct"): {"0.1": 3.08, "0.5": 3.13, "uniform": 3.13},
}


def experiment_nonzeros(log_domain, dist, n=1 << 20, seed=2021):
    """2^20 distinct non-zero buckets in [0, 2^log_domain), sorted, as an (n,
    2) uint64 {lo, hi} array.  The reference's CSV inputs are git-LFS
    pointers (absent), so the README's three distributions (README:8-15) are
    drawn here: "power law with 90 % of non-zeros in a fraction f of the
    domain" as x = floor(2^B u^a) with u uniform and a = ln f / ln 0.9 (so
    P(x < f 2^B) = 0.9), and uniform (a = 1); duplicates are redrawn."""
    import math
    rng = np.random.default_rng(seed + 7 * log_domain + {"0.1": 1, "0.5": 2, "uniform": 3}[dist])
    a = 1.0 if dist == "uniform" else math.log(float(dist)) / math.log(0.9)
    have = np.zeros((0, 2), dtype=np.uint64)  # (hi, lo) rows
    while len(have) < n:
        m = int((n - len(have)) * 1.5) + 1024
        v = rng.random(m) ** a
        if log_domain <= 53:
            hi = np.zeros(m, np.uint64)
            lo = np.floor(v * float(1 << log_domain)).astype(np.uint64)
        else:  # 53 bits from v, the rest uniform below them
            top = (v * float(1 << 53)).astype(np.uint64)
            r_lo = rng.integers(0, 1 << 63, m, dtype=np.uint64) * 2 + rng.integers(0, 2, m, dtype=np.uint64)
            sh = log_domain - 53  # bits below the 53 drawn ones
            if sh >= 64:
                r_hi = rng.integers(0, 1 << (sh - 64), m, dtype=np.uint64) if sh > 64 else np.zeros(m, np.uint64)
                hi = (top << np.uint64(sh - 64)) | r_hi
                lo = r_lo
            else:
                lo = (r_lo & np.uint64((1 << sh) - 1)) | (top << np.uint64(sh))
                hi = top >> np.uint64(64 - sh) if sh else np.zeros(m, np.uint64)
        have = np.unique(np.concatenate([have, np.stack([hi, lo], axis=1)]), axis=0)
    keep = np.sort(rng.choice(len(have), n, replace=False))
    hl = have[keep]
    return np.ascontiguousarray(np.stack([hl[:, 1], hl[:, 0]], axis=1))


def _shift_unique(lohi, s):
    """Sorted unique (n, 2) {lo, hi} words of x >> s (ComputePrefixes,
    experiments/synthetic_data_benchmarks.cc:100-121)."""
    lo, hi = lohi[:, 0], lohi[:, 1]
    if s >= 128:
        return np.zeros((1, 2), np.uint64)
    if s >= 64:
        lo, hi = hi >> np.uint64(s - 64), np.zeros_like(hi)
    elif s > 0:
        lo, hi = (lo >> np.uint64(s)) | (hi << np.uint64(64 - s)), hi >> np.uint64(s)
    keep = np.ones(len(lo), bool)
    keep[1:] = (lo[1:] != lo[:-1]) | (hi[1:] != hi[:-1])  # input sorted: runs of equals
    return np.ascontiguousarray(np.stack([lo[keep], hi[keep]], axis=1))


def _oracle_experiment(log_domain, lohi):
    """The oracle (1 core) on the same workload, one iteration of each mode:
    hierarchical over the README levels (prefixes prepared outside the timed
    region, as the reference's benchmark does), then EvaluateAt at the
    non-zeros."""
    from oracle import pyoracle as po
    levels = list(range(21, log_domain, 2)) + [log_domain]
    pre = [None] + [_shift_unique(lohi, log_domain - levels[i - 1]) for i in range(1, len(levels))]
    od = po.Dpf([(ld, ("int", 32), 0) for ld in levels])
    alpha = int(lohi[len(lohi) // 3, 0]) | (int(lohi[len(lohi) // 3, 1]) << 64)
    k0, _ = od.generate_keys(alpha, [1] * len(levels), seeds=(5, 6))
    ctx = od.create_evaluation_context(k0)
    t0 = time.perf_counter()
    for i in range(len(levels)):
        od.evaluate_until_words(i, [] if i == 0 else pre[i], ctx)
    hier = time.perf_counter() - t0
    d1 = po.Dpf([(log_domain, ("int", 32), 0)])
    k1, _ = d1.generate_keys(alpha, [1], seeds=(7, 8))
    t0 = time.perf_counter()
    d1.evaluate_at_words(k1, 0, lohi)
    direct = time.perf_counter() - t0
    return hier, direct


def main_experiments(args):
    """bench.py --experiments: the reference's published workloads through the
    C++ API (tools/experiments_bench.cc, GPU) with the oracle on one host
    core beside them; one JSON line per case and a summary line."""
    import subprocess
    import tempfile
    exe = os.path.join(os.path.dirname(_lib.LIB_PATH), "experiments_bench")
    rows = []
    for log_domain in (32, 128):
        for dist in ("0.1", "0.5", "uniform"):
            nz = experiment_nonzeros(log_domain, dist)
            with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
                nz.tofile(f)
                path = f.name
            try:
                out = subprocess.run([exe, path, str(log_domain), str(args.steps), dist],
                                     capture_output=True, text=True, timeout=900)
            finally:
                os.unlink(path)
            if out.returncode != 0:
                raise RuntimeError("experiments_bench failed: " + out.stderr[-2000:])
            gpu = {json.loads(l)["workload"]: json.loads(l) for l in out.stdout.splitlines()
                   if l.startswith("{")}
            cpu = None
            if not args.skip_cpu_baseline and (log_domain == 32 or dist == "uniform"):
                h, d = _oracle_experiment(log_domain, nz)
                cpu = {"hierarchical": h, "direct": d}
            for mode in ("hierarchical", "direct"):
                g = gpu[mode]
                row = dict(g)
                row["published_reference_s"] = EXPERIMENT_PUBLISHED_S[(log_domain, mode)][dist]
                row["speedup_vs_published"] = row["published_reference_s"] / g["best_s"]
                if cpu:
                    row["cpu_baseline"] = {"value_s": cpu[mode], "cores": 1, "kind": "port",
                                           "sample": "oracle/dpf_oracle.c, same non-zeros, "
                                                     "one iteration"}
                rows.append(row)
                print(json.dumps(row), flush=True)
    print(json.dumps({"experiments": "experiments/README.md:20-108 workloads, synthetic non-zeros",
                      "cases": len(rows),
                      "all_correct": all(r.get("correct") for r in rows)}), flush=True)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--log-domain", type=int, default=32)
    ap.add_argument("--pir-log-records", type=int, default=26)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--skip-cpu-baseline", action="store_true")
    ap.add_argument("--skip-pir", action="store_true")
    ap.add_argument("--skip-handle-request", action="store_true")
    ap.add_argument("--skip-scan-skip", action="store_true",
                    help="do not time the opt-in scan that reads only selected records")
    ap.add_argument("--devices", default="",
                    help="--in-process: comma-separated device list, one slice / shard per entry "
                         "(entries may repeat: a rehearsal of N devices' code on fewer GPUs)")
    ap.add_argument("--force-peer", action="store_true",
                    help="--in-process: take the cross-device copy branches even between "
                         "slices on one device (dpf_amd_set_force_peer_copies)")
    ap.add_argument("--experiments", action="store_true",
                    help="time the reference's published experiment workloads (one key, 2^20 "
                         "non-zeros, domains 2^32 / 2^128) through the C++ API instead")
    ap.add_argument("--in-process", action="store_true",
                    help="drive all --gpus GPUs from this one process through the library's "
                         "multi-GPU API (ExpandLeavesOnDevices, a sharded DenseDpfPirDatabase)")
    ap.add_argument("--library-multi-device", action="store_true",
                    help="(the child rank 0 starts at world > 1) time and check the library's own "
                         "multi-device path over --devices: ExpandLeavesOnDevices (c5) and a "
                         "sharded DenseDpfPirDatabase behind HandleRequest (c4)")
    ap.add_argument("--skip-library-multi-device", action="store_true",
                    help="at world > 1, do not run the library_multi_device child")
    ap.add_argument("--library-multi-device-timeout", type=int, default=300)
    args = ap.parse_args(argv)
    # torch.cuda.device_count() does not initialise the GPU on this image
    how, what = launch_decision(args, os.environ, torch.cuda.device_count())
    if how == "error":
        print("[bench] error: " + what, flush=True)
        return 2
    if how == "spawn":
        import sys
        return spawn_ranks(what, sys.argv[1:] if argv is None else argv)
    if args.experiments:
        return main_experiments(args)
    if args.library_multi_device:
        if args.force_peer:
            _lib.lib().dpf_amd_set_force_peer_copies(1)
        print(json.dumps({"library_multi_device": bench_library_multi_device(args)}), flush=True)
        return 0
    if args.in_process:
        if args.force_peer:
            _lib.lib().dpf_amd_set_force_peer_copies(1)
        return main_in_process(args)
    world, rank, device = setup()
    ranks = rank_devices(world, device)
    r = bench_dpf(args, world, rank, device)
    pir = None if args.skip_pir else bench_pir(args, world, rank, device)
    cpu = None
    # rank 0 times the host CPU after the GPU legs, the other ranks wait
    if rank == 0 and not args.skip_cpu_baseline:
        cpu = cpu_baseline(args)
    if world > 1:
        dist.barrier()
    out = None
    if rank == 0:
        leaves = r["leaves"]
        ms = 1000 * r["wall"] / args.steps
        value = leaves / (r["wall"] / args.steps)
        aes_per_launch = AES_PER_LEAF_C5 * leaves / world  # one launch per rank per step
        aes_s = aes_per_launch / (r["kernel_ms"] / 1e3)
        achieved = aes_s * OPS_PER_AES / 1e12
        lookups_s = LDS_LOOKUPS_PER_LEAF_C5 * (leaves / world) / (r["kernel_ms"] / 1e3)
        expand_traffic = traffic_from_profiles(EXPAND_C5_KERNEL_RE)
        clk = clock_view(expand_traffic[2])
        scan_traffic = traffic_from_profiles(SCAN_Q1_KERNEL_RE)
        out = {
            "metric": METRIC, "value": value, "unit": "leaves/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "tuple<u32,intmodn<u64>>", "data": "synthetic (fixed-seed DPF key)",
            "config": {"workload": "c5: full-domain EvaluateNext, log_domain_size=%d, "
                                   "Tuple<uint32,IntModN<uint64,2^64-59>>, "
                                   "security_parameter=48" % args.log_domain,
                       "leaves_per_step": leaves, "tree_levels": r["L"],
                       "parallelism": "one key's 2^%d domain subtree-sharded over %d GPU(s)" %
                                      (args.log_domain, world)},
            "world_size": world, "backend": bench_backend() if world > 1 else None,
            "library": library_identity(),
            # (rank, device index, PCI bus id) of every rank
            "rank_devices": ranks,
            # The T-table AES is bound by LDS lookup issue (ds_read_b32: 32
            # lane-lookups/clk/CU, conflict-free by construction): achieved =
            # leaves per launch x 601 lookups / kernel time (the subtree walk's
            # extra lookups, ~0.3%, are not counted).
            "roofline": {"bound": "lds",
                         "achieved": lookups_s / 1e12,
                         "peak": LDS_PEAK_LOOKUPS / 1e12, "unit": "T lookups/s",
                         "frac": lookups_s / LDS_PEAK_LOOKUPS,
                         # the profile is of the N = 1 launch (all 2^32 leaves);
                         # a rank's launch expands 1/N of them
                         "traffic": (expand_traffic[0] / world
                                     if expand_traffic[0] is not None else None),
                         "traffic_unit": "HBM bytes per launch (rocprofv3 PMC of this build%s)" %
                                         (", N = 1 profile / %d ranks" % world if world > 1 else ""),
                         "traffic_error": expand_traffic[3],
                         "traffic_profile": expand_traffic[1],
                         "algorithmic_bytes": leaves // world * 16,
                         "kernel": "KExpand<8,EmitU32ModN64>", "kernel_ms": r["kernel_ms"],
                         "aes_per_launch": aes_per_launch, "aes_per_leaf": AES_PER_LEAF_C5,
                         "aes_per_s_per_gpu": aes_s,
                         "lookups_per_leaf": LDS_LOOKUPS_PER_LEAF_C5,
                         # the part's clock under this kernel (profile of this
                         # build) and the fraction against the LDS peak at it
                         "measured": (dict(clk, frac_at_measured_clock=(
                             lookups_s / (LDS_PEAK_LOOKUPS * clk["clock_ghz"] / 2.4)))
                             if clk else None)},
            # SURVEY.md §8d's integer-VALU fraction: AES/s x I_AES / the
            # VALU issue peak (256 CU x 4 SIMD x 32 lanes x 2.4 GHz; the
            # 64-lane figure of BASELINE.md:56 undercounts CDNA4's SIMDs by 2)
            "valu": valu_view(aes_s, expand_traffic[2]),
            # Not a roofline: the implementation-independent reference point
            # of SURVEY.md §8d — AES/s priced at the 757.5 two-input gate ops
            # a bitsliced AES-128 needs per block, against the VALU issue
            # rate.  This T-table kernel does not perform those ops (it does
            # ~300 VALU + 160 LDS lookups per AES), so the ratio can exceed 1.
            "bitsliced_equivalent": {"gate_ops_per_aes": OPS_PER_AES,
                                     "equivalent_tops": achieved,
                                     "valu_peak_tops": VALU_PEAK_TOPS,
                                     "ratio_to_valu_peak": achieved / VALU_PEAK_TOPS},
            "cpu_baseline": cpu,
        }
        if pir is not None:
            gbs = pir["db_bytes"] / pir["wall_s"] / 1e9
            scan_gbs = pir["per_gpu_bytes"] / (pir["scan_ms"] / 1e3) / 1e9
            out["pir"] = {
                "metric": "dense-PIR scan GB/s", "value": gbs, "unit": "GB/s",
                "workload": "c4: %d records x 256 B, Q=1, Tier-1 selection expansion + "
                            "XOR scan%s (the reference API path is handle_request below)" %
                            (pir["records"], " + RCCL all-gather + fold" if world > 1 else ""),
                "ms_per_query": 1e3 * pir["wall_s"], "correct": pir["ok"],
                "scaling": "strong",
                "roofline": {"bound": "hbm", "achieved": scan_gbs, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": scan_gbs / HBM_PEAK_GBS,
                             "traffic": (scan_traffic[0] / world
                                         if scan_traffic[0] is not None else None),
                             "traffic_profile": scan_traffic[1],
                             "traffic_error": scan_traffic[3],
                             "algorithmic_bytes": pir["per_gpu_bytes"],
                             "kernel": "KPirScanG<1,4>+KXorFold", "kernel_ms": pir["scan_ms"]},
                "batch_%d" % pir["mq"]: {
                    "queries": pir["mq"], "ms_per_batch": pir["mq_ms"],
                    "query_GBps": pir["mq"] * pir["db_bytes"] / (pir["mq_ms"] / 1e3) / 1e9,
                    "db_GBps": pir["db_bytes"] / (pir["mq_ms"] / 1e3) / 1e9,
                    # The Four-Russians scan is bound by its LDS work, not
                    # HBM: per KiB of records 15 row stores
                    # (ds_write_addtid_b32, 128 B/clk) + Q/4 row reads of
                    # 256 B (ds_read_b128, 256 B/clk) = 94 LDS cycles at Q = 64.
                    "lds_roofline": m4_lds_roofline(pir["per_gpu_bytes"], pir["mq"],
                                                    pir["mq_ms"]),
                    "kernel": "KPirScanM4<1>+KXorFold (scan only, no selection DPF)"},
            }
            if pir.get("skip"):
                sk = pir["skip"]
                read_gbs = sk["read_bytes"] / (sk["scan_ms"] / 1e3) / 1e9
                out["pir"]["skip_unselected"] = {
                    "opt_in": "dpf_amd_set_scan_skip_unselected(1): the scan reads only the "
                              "selected records, as the reference's InnerProduct skips the others "
                              "(inner_product_hwy.cc:213-221); its access pattern follows the "
                              "selection share, so the default scan above reads every record",
                    "ms_per_query": 1e3 * sk["wall_s"], "scan_ms": sk["scan_ms"],
                    "db_GBps": pir["db_bytes"] / sk["wall_s"] / 1e9,
                    "scan_db_GBps": pir["per_gpu_bytes"] / (sk["scan_ms"] / 1e3) / 1e9,
                    "selected_rows_rank0": sk["selected_rows"],
                    "roofline": {"bound": "hbm", "achieved": read_gbs, "peak": HBM_PEAK_GBS,
                                 "unit": "GB/s", "frac": read_gbs / HBM_PEAK_GBS,
                                 "algorithmic_bytes": sk["read_bytes"],
                                 "algorithmic_is": "selected rows x 256 B + selection blocks "
                                                   "(rank 0)"},
                    "correct": sk["ok"]}
            if pir.get("hr"):
                hr, hr_ok = pir["hr"]
                out["pir"]["handle_request"] = {
                    "api": "DenseDpfPirServer::HandleRequest via dpf_amd_pir_server_handle_request "
                           "(wire decode + validation + selection expansion + scan + encode + D2H)",
                    "ms_per_request": {str(q): v for q, v in hr.items()},
                    "db_GBps_at_q1": pir["db_bytes"] / (hr[1] / 1e3) / 1e9 if 1 in hr else None,
                    "correct": hr_ok}
            if pir.get("shard"):
                sn, (shr, sok) = pir["shard"]
                out["pir"]["handle_request_one_eighth"] = {
                    "what": "the same API on a database of %d records (c4 / 8: one rank's row "
                            "shard at N = 8), one GPU" % sn,
                    "ms_per_request": {str(q): v for q, v in shr.items()},
                    "shard_GBps_at_q1": sn * 256 / (shr[1] / 1e3) / 1e9,
                    "correct": sok}
    if world > 1:
        # Every rank has freed its buffers (the legs' tensors are gone; the
        # caching allocator returns them here); then rank 0 starts the
        # library_multi_device child over all ranks' devices while the other
        # ranks exit, and folds its result (or its error) into the line.
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        dist.barrier()
        dist.destroy_process_group()
        if rank == 0:
            out["library_multi_device"] = (
                {"skipped": "--skip-library-multi-device"} if args.skip_library_multi_device
                else run_library_multi_device(library_multi_device_cmd(ranks, args),
                                              args.library_multi_device_timeout))
    if rank == 0:
        print(json.dumps(out), flush=True)


def main_in_process(args):
    r = bench_in_process(args)
    devs = [int(d) for d in args.devices.split(",")] if args.devices else list(range(args.gpus))
    args.gpus = len(set(devs))  # distinct GPUs; slices on a repeated device share it
    ms = 1000 * r["wall"] / args.steps
    per_gpu_leaves = r["leaves"] / args.gpus
    lookups_s = LDS_LOOKUPS_PER_LEAF_C5 * per_gpu_leaves / (ms / 1e3)
    expand_traffic = traffic_from_profiles(EXPAND_C5_KERNEL_RE)
    out = {
        "metric": METRIC, "value": r["leaves"] / (r["wall"] / args.steps), "unit": "leaves/s",
        "n_gpus": args.gpus, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "tuple<u32,intmodn<u64>>", "data": "synthetic (fixed-seed DPF key)",
        "config": {"workload": "c5: full-domain expansion, log_domain_size=%d, "
                               "Tuple<uint32,IntModN<uint64,2^64-59>>, security_parameter=48"
                               % args.log_domain,
                   "leaves_per_step": r["leaves"], "tree_levels": r["L"],
                   "parallelism": "in-process: DistributedPointFunction::ExpandLeavesOnDevices "
                                  "over %d GPU(s), disjoint subtree slices" % args.gpus,
                   "devices": devs},
        # per GPU: its slice's lookups over the step's wall time (the launch
        # and the wait for every device included, so a lower bound)
        "roofline": {"bound": "lds", "achieved": lookups_s / 1e12,
                     "peak": LDS_PEAK_LOOKUPS / 1e12, "unit": "T lookups/s",
                     "frac": lookups_s / LDS_PEAK_LOOKUPS,
                     # the profile is of the N = 1 launch (all leaves); each
                     # GPU's slices expand 1/N of them
                     "traffic": (expand_traffic[0] / args.gpus
                                 if expand_traffic[0] is not None else None),
                     "traffic_unit": "HBM bytes per GPU per step (rocprofv3 PMC of this build%s)"
                                     % (", N = 1 profile / %d GPUs" % args.gpus
                                        if args.gpus > 1 else ""),
                     "traffic_profile": expand_traffic[1],
                     "traffic_error": expand_traffic[3],
                     "algorithmic_bytes": int(per_gpu_leaves) * 16,
                     "kernel": "KExpand<8,EmitU32ModN64>", "kernel_ms": ms,
                     "kernel_ms_is": "step wall time of ExpandLeavesOnDevices",
                     "lookups_per_leaf": LDS_LOOKUPS_PER_LEAF_C5},
        "cpu_baseline": None if args.skip_cpu_baseline else cpu_baseline(args),
        "library": library_identity(),
    }
    if r["pir"]:
        p = r["pir"]
        q1 = p["ms"][1]
        per_gpu_bytes = p["n"] * p["rec"] / args.gpus
        gbs = per_gpu_bytes / (q1 / 1e3) / 1e9
        out["pir"] = {"api": "DenseDpfPirServer::HandleRequest, database sharded over devices %s"
                             % devs,
                      "metric": "dense-PIR scan GB/s", "unit": "GB/s",
                      "value": p["n"] * p["rec"] / (q1 / 1e3) / 1e9,
                      "ms_per_request": {str(q): v for q, v in p["ms"].items()},
                      "db_GBps_at_q1": p["n"] * p["rec"] / (q1 / 1e3) / 1e9,
                      "correct": p["ok"], "scaling": "strong",
                      # per GPU: its shard's bytes over the whole Q = 1
                      # request (decode, expansion, scan, peer-copied
                      # partials, fold, encode) — a lower bound on the scan's
                      "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS,
                                   "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                                   "algorithmic_bytes": per_gpu_bytes,
                                   "kernel": "KPirScanG<1,4>+KXorFold",
                                   "kernel_ms": q1,
                                   "kernel_ms_is": "HandleRequest wall time at Q = 1"}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    raise SystemExit(main())
