"""World-size-2 tests of the multi-GPU partitioning on CPU (gloo).

Each rank computes its shard with the CPU oracle standing in for the device
kernels (the kernels' own parity is covered by the -m gpu tests); the
distributed logic under test is the product's: distributed_point_functions_
amd/sharding.py (subtree slices, 128-aligned PIR row shards, all-gather + XOR
fold of partials, additive-share all-reduce).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_point_functions_amd import sharding


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
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle import pyoracle as po
        res = {}

        # (1) PIR: rows sharded on 128-record boundaries, partials XOR-combined.
        rng = np.random.default_rng(5)
        n, rec = 1000, 48
        records = [bytes(rng.integers(0, 256, rec, dtype=np.uint8)) for _ in range(n)]
        nb = (n + 127) // 128
        sel = [int.from_bytes(rng.bytes(16), "little") for _ in range(nb)]
        r_lo, r_hi, b_lo, b_hi = sharding.pir_row_shard(n, world, rank)
        mine = po.inner_product(records[r_lo:r_hi], [sel[b_lo:b_hi]])[0] if r_hi > r_lo \
            else bytes(rec)
        part = torch.frombuffer(bytearray(mine), dtype=torch.uint8)
        combined = sharding.allgather_xor(part, world, fold=_host_fold)
        res["pir"] = bytes(combined.numpy()) == po.inner_product(records, [sel])[0]

        # (2) One key's full domain, subtree-sharded: concatenation == full.
        spec = ("int", 64)
        d = po.Dpf([(12, spec, 52)])
        k0, _ = d.generate_keys(77, [123], seeds=(9, 10))
        L = d.hierarchy_to_tree(0)
        lo, hi = sharding.block_range(1 << L, world, rank)
        cnt = hi - lo
        assert cnt & (cnt - 1) == 0
        words = d.expand_subtree_words(k0, lo, cnt.bit_length() - 1)
        t = torch.from_numpy(words.view(np.int64).copy())
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        full = d.evaluate_until_words(0, [], d.create_evaluation_context(k0))
        res["dpf"] = np.array_equal(torch.cat(out).numpy().view(np.uint64),
                                    full.reshape(-1))

        # (4) c2: EvaluateAt points in contiguous per-rank slices, concatenated.
        pts = [int.from_bytes(rng.bytes(2), "little") % (1 << 12) for _ in range(101)]
        plo, phi = sharding.point_range(len(pts), world, rank)
        got = [None] * world
        dist.all_gather_object(got, d.evaluate_at(k0, 0, pts[plo:phi]))
        res["c2"] = [v for g in got for v in g] == d.evaluate_at(k0, 0, pts)

        # (5) c3: each rank keeps its own context for the prefixes whose
        # first-level ancestor it owns; every level's outputs concatenate.
        lv = [(ld, spec, 40 + ld) for ld in (8, 16, 24)]
        dd = po.Dpf(lv)
        kk, _ = dd.generate_keys(0xABCDE, [11, 22, 33], seeds=(5, 6))
        mine_ctx, full_ctx = dd.create_evaluation_context(kk), dd.create_evaluation_context(kk)
        dd.evaluate_until(0, [], mine_ctx)
        dd.evaluate_until(0, [], full_ctx)
        p1 = sorted(int(x) for x in rng.choice(256, 60, replace=False)) + [255]
        bounds = sharding.prefix_owner_bounds(p1, world)
        ok3 = True
        prefixes = p1
        for h, shift in ((1, 0), (2, 8)):
            mine = sharding.owned_prefixes(prefixes, bounds, rank, shift)
            got = [None] * world
            dist.all_gather_object(got, dd.evaluate_until(h, mine, mine_ctx) if mine else [])
            ok3 &= [v for g in got for v in g] == dd.evaluate_until(h, prefixes, full_ctx)
            prefixes = sorted({(p << 8) | int(y) for p in prefixes for y in (3, 200)})
        res["c3"] = ok3

        # (3) Additive Z_2^64 shares summed over ranks wrap exactly.
        vals = [(2 ** 64 - 3), 5] if rank == 0 else [7, 2 ** 63 + 1]
        sh = torch.tensor(np.array(vals, dtype=np.uint64).view(np.int64))
        sharding.allreduce_additive(sh)
        got = [int(x) for x in sh.numpy().view(np.uint64)]
        res["additive"] = got == [(2 ** 64 - 3 + 7) % 2 ** 64, (5 + 2 ** 63 + 1) % 2 ** 64]
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, {"error": repr(e)}))


def test_block_range_and_row_shards_cover_exactly():
    for total in (1, 7, 128, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            spans = [sharding.block_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            rows = [sharding.pir_row_shard(total, world, r) for r in range(world)]
            assert rows[0][0] == 0 and rows[-1][1] == total
            assert all(r[0] % 128 == 0 or r[0] == total for r in rows)
            assert all(a[1] == b[0] for a, b in zip(rows, rows[1:]))


def test_prefix_owners_partition_every_level():
    """c3 ownership: every prefix of every level has exactly one owner, the
    owners' slices are contiguous and in rank order (outputs concatenate),
    and equal first-level prefixes share an owner."""
    import random
    rng = random.Random(3)
    for world in (1, 2, 3, 8):
        p1 = sorted(rng.randrange(1 << 10) for _ in range(97))
        bounds = sharding.prefix_owner_bounds(p1, world)
        levels = [(p1, 0)]
        p2 = sorted({(p << 6) | rng.randrange(64) for p in p1 for _ in range(3)})
        levels.append((p2, 6))
        levels.append((sorted({(p << 6) | 5 for p in p2}), 12))
        for prefixes, shift in levels:
            parts = [sharding.owned_prefixes(prefixes, bounds, r, shift) for r in range(world)]
            assert [x for part in parts for x in part] == prefixes
        owner = {}
        for r in range(world):
            for p in sharding.owned_prefixes(p1, bounds, r):
                assert owner.setdefault(p, r) == r
    with pytest.raises(ValueError):
        sharding.prefix_owner_bounds([3, 1], 2)


def test_world_size_2_gloo():
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
            rank, res = q.get(timeout=240)
            results[rank] = res
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank in range(world):
        assert "error" not in results[rank], results[rank]
        assert results[rank] == {"pir": True, "dpf": True, "c2": True, "c3": True,
                                 "additive": True}, results[rank]
