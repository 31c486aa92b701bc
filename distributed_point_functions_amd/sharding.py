"""Multi-GPU partitioning of the hot path.

One process per GPU. The DPF domain (c1, c5), EvaluateAt batches (c2), the
incremental prefix lists (c3) and the PIR database (c4) all partition
without any data-path exchange; the only collective is the all-gather of the
tiny PIR partials (RCCL has no XOR reduction) and, for additive shares in
Z_2^k (k <= 64), an all-reduce SUM that is exact under wraparound.
"""
from __future__ import annotations

from typing import Callable, List, Sequence, Tuple

RECORDS_PER_SELECTION_BLOCK = 128  # bit r of block r/128 selects record r


def block_range(num_blocks: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced slice [lo, hi) of the 2^L tree blocks of one key's
    full domain owned by `rank` (subtree sharding: the slice is a union of
    whole subtrees, each rank walks its own prefix; outputs are disjoint and
    in domain order)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(num_blocks, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def pir_row_shard(num_records: int, world: int, rank: int) -> Tuple[int, int, int, int]:
    """Rows [r_lo, r_hi) and selection blocks [b_lo, b_hi) of `rank`'s shard
    of a dense PIR database. Shards are aligned to 128-record selection
    blocks so every rank expands whole DPF leaves of its own."""
    blocks = (num_records + RECORDS_PER_SELECTION_BLOCK - 1) // RECORDS_PER_SELECTION_BLOCK
    b_lo, b_hi = block_range(blocks, world, rank)
    r_lo = min(num_records, b_lo * RECORDS_PER_SELECTION_BLOCK)
    r_hi = min(num_records, b_hi * RECORDS_PER_SELECTION_BLOCK)
    return r_lo, r_hi, b_lo, b_hi


def point_range(num_points: int, world: int, rank: int) -> Tuple[int, int]:
    """c2 (EvaluateAt batches): `rank`'s contiguous slice [lo, hi) of the
    points (or of the keys of a batched call); results concatenate in order,
    no collective."""
    return block_range(num_points, world, rank)


def prefix_owner_bounds(prefixes: Sequence[int], world: int) -> List[int]:
    """c3 (incremental evaluation): owner boundaries, in prefix values, for
    the first prefixed hierarchy level.  `prefixes` is that level's sorted
    candidate list; rank r owns the values [bounds[r], bounds[r + 1]) — a
    contiguous, balanced slice of the list (equal values stay together).
    Every later level's prefix p belongs to the rank that owns its ancestor
    p >> (log_domain(level) - log_domain(first level)), which holds that
    ancestor's partial evaluations in its own EvaluationContext (cc:374-476),
    so no rank ever needs another's context."""
    n = len(prefixes)
    if world <= 0:
        raise ValueError("bad world")
    if any(prefixes[i] > prefixes[i + 1] for i in range(n - 1)):
        raise ValueError("prefixes must be sorted")
    bounds = [0]
    for r in range(1, world):
        lo, _ = block_range(n, world, r)
        bounds.append(max(bounds[-1], prefixes[lo] if lo < n else (prefixes[-1] + 1 if n else 0)))
    bounds.append(None)  # open upper end
    return bounds


def owned_prefixes(prefixes: Sequence[int], bounds: Sequence[int], rank: int,
                   shift: int = 0) -> List[int]:
    """The prefixes of a level owned by `rank` under `bounds`
    (prefix_owner_bounds), `shift` = log_domain(level) - log_domain(first
    prefixed level).  For a sorted list the ranks' slices are contiguous and
    in rank order, so the ranks' outputs concatenate to the single-process
    output."""
    lo, hi = bounds[rank], bounds[rank + 1]
    return [p for p in prefixes if (p >> shift) >= lo and (hi is None or (p >> shift) < hi)]


def allgather_xor(part, world: int, fold: Callable = None):
    """XOR-combine one equally-sized byte tensor per rank: all-gather (the
    only data-path collective of the sharded scan) + a local fold.
    `fold(gathered, world, nbytes, out)` defaults to the device kernel
    (kernels.xor_fold); CPU/gloo tests pass a host fold."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return part
    gathered = torch.empty(world * part.numel(), dtype=part.dtype, device=part.device)
    if part.is_cuda and dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(gathered, part.contiguous().view(-1))
    else:  # gloo (CPU tests; the 1-GPU multi-rank rehearsal): host buffers
        host = torch.empty(world * part.numel(), dtype=part.dtype)
        dist.all_gather(list(host.view(world, -1).unbind(0)), part.contiguous().view(-1).cpu())
        gathered.copy_(host)
    out = torch.empty_like(part)
    if fold is None:
        from . import kernels
        fold = kernels.xor_fold
    fold(gathered, world, part.numel(), out)
    return out


def allreduce_additive(shares):
    """Sum of additive shares over ranks, in place, exact mod 2^64 for
    uint8/16/32/64 shares carried in int64 (two's-complement wraparound)."""
    import torch
    import torch.distributed as dist
    if shares.dtype != torch.int64:
        raise TypeError("carry Z_2^k shares as int64")
    dist.all_reduce(shares, op=dist.ReduceOp.SUM)
    return shares
