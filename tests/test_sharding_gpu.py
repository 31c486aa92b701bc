"""World-size-2 run of bench.py's multi-GPU data path on the device: two
ranks (both on cuda:0, gloo for the exchange) each expand their slice of one
key's domain through the product's leaf-range entry (dpf_amd_expand_and_
correct with [leaf_begin, leaf_end) from sharding.block_range) and scan
their 128-aligned PIR row shard (dpf_amd_inner_product over sharding.pir_
row_shard, selection bits expanded on the device for that block range).
The gathered slices equal the oracle's full-domain expansion and the folded
partials equal the oracle's inner product over the whole database.  c2 and c3
partition the same way through the product's EvaluateAt / EvaluateNext:
contiguous point slices, and prefixes owned by the rank that owns their
first-level ancestor (sharding.prefix_owner_bounds), each rank with its own
EvaluationContext; every level's gathered outputs equal the oracle's.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

P64 = 2 ** 64 - 59


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _host_fold(gathered, world, nbytes, out):
    g = gathered.view(world, nbytes)
    acc = g[0].clone()
    for i in range(1, world):
        acc ^= g[i]
    out.copy_(acc)


def _worker(rank, world, port, q):
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import bench
        from oracle import pyoracle as po
        from distributed_point_functions_amd import _lib, kernels, sharding
        from distributed_point_functions_amd import value_types as V
        from distributed_point_functions_amd.dpf import DistributedPointFunction, DpfParameters
        res = {}

        # (1) c5 type, one key's 2^20 domain subtree-sharded over the ranks
        ld = 20
        spec = ("tuple", [("int", 32), ("intmodn", 64, P64)])
        dpf = DistributedPointFunction.create(DpfParameters(ld, V.from_spec(spec), 48))
        alpha, beta, seeds = 0x9E3779B9 % (1 << ld), (123456789, 987654321), (0xA5A5, 0x5A5A)
        k0, _ = dpf.generate_keys(alpha, beta, seeds=seeds)
        ka = bench.key_arrays(dpf, k0, 0, dev)
        desc = dpf.value_type_descriptor(0)
        L = ka["L"]
        cepb = 1 << (ld - L)
        lo, hi = sharding.block_range(1 << L, world, rank)
        out = torch.empty((hi - lo) * cepb * desc.out_stride, dtype=torch.uint8, device=dev)
        kernels.expand_and_correct(ka["seed"], ka["cb"], L, ka["cw"], ka["ccl"], ka["ccr"],
                                   desc, ka["corr"], ka["party"], cepb, lo, hi, out)
        torch.cuda.synchronize()
        mine = out.cpu()
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(sizes, torch.tensor([mine.numel()]))
        parts = [torch.empty(int(s.item()), dtype=torch.uint8) for s in sizes]
        dist.all_gather(parts, mine)
        got = torch.cat(parts).numpy().view(np.uint64).reshape(-1, 2)  # {u64, u32|pad}
        od = po.Dpf([(ld, spec, 48)])
        ok0, _ = od.generate_keys(alpha, [beta], seeds=seeds)
        want = od.evaluate_until_words(0, [], od.create_evaluation_context(ok0))  # (n, 2, 2)
        res["dpf"] = bool(np.array_equal(got[:, 0], want[:, 1, 0]) and
                          np.array_equal(got[:, 1] & 0xFFFFFFFF, want[:, 0, 0]))

        # (2) dense PIR: selection expanded for this rank's blocks, row shard scan
        n, rec = 5000, 256
        rng = np.random.default_rng(17)
        records = rng.integers(0, 256, (n, rec), dtype=np.uint8)
        r_lo, r_hi, b_lo, b_hi = sharding.pir_row_shard(n, world, rank)
        per = r_hi - r_lo
        db = torch.from_numpy(records[r_lo:r_hi].reshape(-1).copy()).to(dev)
        pdpf = DistributedPointFunction.create(
            DpfParameters(max(0, (n - 1).bit_length()), V.XorWrapper(128)))
        idx = 4321
        shares = []
        for key in pdpf.generate_keys(idx // 128, 1 << (idx % 128), seeds=(0x1111, 0x2222)):
            kd = bench.key_arrays(pdpf, key, 0, dev)
            sel = torch.empty(max(1, b_hi - b_lo) * 16, dtype=torch.uint8, device=dev)
            kernels.expand_and_correct(kd["seed"], kd["cb"], kd["L"], kd["cw"], kd["ccl"],
                                       kd["ccr"], pdpf.value_type_descriptor(0), kd["corr"],
                                       kd["party"], 1, b_lo, b_hi, sel)
            part = torch.zeros(rec, dtype=torch.uint8, device=dev)
            if per > 0:
                kernels.inner_product(db, per, rec, sel.view(torch.int64).view(-1, 2), 1,
                                      None, part)
            torch.cuda.synchronize()
            shares.append(sharding.allgather_xor(part.cpu(), world, fold=_host_fold).numpy())
        res["pir"] = bytes(shares[0] ^ shares[1]) == records[idx].tobytes()

        # (3) c2: EvaluateAt points in contiguous per-rank slices (product
        # EvaluateAt on the device), concatenated == the oracle on all points
        spec64 = ("int", 64)
        vt64 = V.from_spec(spec64)
        d2 = DistributedPointFunction.create(DpfParameters(40, vt64, 48))
        od2 = po.Dpf([(40, spec64, 48)])
        a2, b2, s2 = 0x12345678AB, 99, (7, 8)
        key2, _ = d2.generate_keys(a2, b2, seeds=s2)
        okey2, _ = od2.generate_keys(a2, [b2], seeds=s2)
        prng = np.random.default_rng(23)
        pts = [int(x) for x in prng.integers(0, 1 << 40, 3001, dtype=np.int64)] + [a2]
        plo, phi = sharding.point_range(len(pts), world, rank)
        got = [None] * world
        dist.all_gather_object(got, vt64.decode_flat(d2.evaluate_at(key2, 0, pts[plo:phi],
                                                                    raw=True)))
        res["c2"] = [v for g in got for v in g] == od2.evaluate_at(okey2, 0, pts)

        # (4) c3: each rank's own context holds the partial evaluations of the
        # prefixes whose first-level ancestor it owns (product EvaluateNext)
        lv = [(ld, spec64, 40 + ld) for ld in (8, 16, 24)]
        d3 = DistributedPointFunction.create_incremental(
            [DpfParameters(ld, vt64, sec) for ld, _, sec in lv])
        od3 = po.Dpf(lv)
        k3, _ = d3.generate_keys_incremental(0xABCDE, [11, 22, 33], seeds=(5, 6))
        ok3k, _ = od3.generate_keys(0xABCDE, [11, 22, 33], seeds=(5, 6))
        ctx = d3.create_evaluation_context(k3)
        octx = od3.create_evaluation_context(ok3k)
        d3.evaluate_next([], ctx, raw=True)
        od3.evaluate_until(0, [], octx)
        prefixes = sorted(int(x) for x in prng.choice(256, 80, replace=False))
        bounds = sharding.prefix_owner_bounds(prefixes, world)
        ok3 = True
        for h, shift in ((1, 0), (2, 8)):
            mine = sharding.owned_prefixes(prefixes, bounds, rank, shift)
            got = [None] * world
            dist.all_gather_object(
                got, vt64.decode_flat(d3.evaluate_next(mine, ctx, raw=True)) if mine else [])
            ok3 &= [v for g in got for v in g] == od3.evaluate_until(h, prefixes, octx)
            prefixes = sorted({(p << 8) | y for p in prefixes for y in (3, 200)})
        res["c3"] = bool(ok3)
        _lib.lib()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, {"error": repr(e) + traceback.format_exc()}))


def test_world_size_2_product_data_path(cuda):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, res = q.get(timeout=100)
            results[rank] = res
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank in range(world):
        assert "error" not in results[rank], results[rank]
        assert results[rank] == {"dpf": True, "pir": True, "c2": True, "c3": True}, results[rank]
