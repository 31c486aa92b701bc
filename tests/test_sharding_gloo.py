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
        assert results[rank] == {"pir": True, "dpf": True, "additive": True}, results[rank]
