"""CPU restatement of the reference's cuckoo-hashed sparse PIR bookkeeping
(TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker, never by the
product package).

Follows:
  SHA256HashFunction::operator()   pir/hashing/sha256_hash_family.cc:59-86
  WrapWithSeed / CreateHashFunctions
                                   pir/hashing/hash_family.h:45-53, hash_family.cc:27-39
  CuckooHashTable::Insert          pir/hashing/cuckoo_hash_table.cc:62-90
    rng_: std::mt19937_64, default seed (cuckoo_hash_table.h:107)
    random_hash_function_: absl::uniform_int_distribution<int>(0, k-1)
      (cuckoo_hash_table.h:106; Abseil @1d07cfed, WORKSPACE.bazel:65-72 —
      absent here, its published algorithm is restated in `_absl_uniform`)
  CuckooHashedDpfPirDatabase::Builder::Build
                                   pir/cuckoo_hashed_dpf_pir_database.cc:96-160
    (records in absl::btree_map order = sorted keys; max_relocations =
     number of records; unlimited stash whose keys are not served)
  InnerProduct                     pir/internal/inner_product_hwy.cc:270-296

Pinning: SHA-256 by the reference's NIST CAVP vector
(sha256_hash_family_test.cc:36-59); std::mt19937_64 by the C++ standard's
known answer ([rand.predef]: the 10000th output of a default-constructed
engine is 9981545732273789042). The absl distribution restatement has no
reference-produced vector (the reference's cuckoo tests check properties
only) — "parity unpinned" for the exact bucket assignment; the properties
(every served key sits in one of its hash buckets) are pinned by
cuckoo_hash_table_test.cc / cuckoo_hashed_dpf_pir_database_test.cc.
"""
from __future__ import annotations

import hashlib
from typing import Dict, List, Optional, Sequence

MASK64 = (1 << 64) - 1


def sha256_hash(seed: bytes, data: bytes, upper_bound: int) -> int:
    """SHA256(seed || data) as a 256-bit little-endian integer mod upper_bound."""
    return int.from_bytes(hashlib.sha256(seed + data).digest(), "little") % upper_bound


def hash_functions(family_seed: bytes, num_hash_functions: int):
    """Function i hashes with seed family_seed || str(i)."""
    return [lambda data, ub, s=family_seed + str(i).encode(): sha256_hash(s, data, ub)
            for i in range(num_hash_functions)]


class MT19937_64:
    """std::mt19937_64 (C++11 [rand.eng.mers] with the [rand.predef] params)."""

    def __init__(self, seed: int = 5489):
        self.mt = [0] * 312
        self.mt[0] = seed & MASK64
        for i in range(1, 312):
            self.mt[i] = (6364136223846793005 * (self.mt[i - 1] ^ (self.mt[i - 1] >> 62)) + i) \
                & MASK64
        self.idx = 312

    def _twist(self):
        mt = self.mt
        for i in range(312):
            x = (mt[i] & 0xFFFFFFFF80000000) | (mt[(i + 1) % 312] & 0x7FFFFFFF)
            xa = x >> 1
            if x & 1:
                xa ^= 0xB5026F5AA96619E9
            mt[i] = mt[(i + 156) % 312] ^ xa
        self.idx = 0

    def __call__(self) -> int:
        if self.idx >= 312:
            self._twist()
        y = self.mt[self.idx]
        self.idx += 1
        y ^= (y >> 29) & 0x5555555555555555
        y ^= (y << 17) & 0x71D67FFFEDA60000
        y ^= (y << 37) & 0xFFF7EEE000000000
        y ^= y >> 43
        return y & MASK64


def _absl_uniform(rng: MT19937_64, k: int) -> int:
    """absl::uniform_int_distribution<int>(0, k-1)(rng): 32-bit unsigned
    range; FastUniformBits<uint32_t> keeps the low 32 bits of one 64-bit
    draw; power-of-two lengths mask, others take the high half of a 32x32
    fixed-point product, rejecting low halves below -Lim % Lim."""
    r = (k - 1) & 0xFFFFFFFF
    lim = (r + 1) & 0xFFFFFFFF
    bits = rng() & 0xFFFFFFFF
    if r & lim == 0:
        return bits & r
    prod = bits * lim
    if prod & 0xFFFFFFFF < lim:
        threshold = ((1 << 32) - lim) % lim
        while prod & 0xFFFFFFFF < threshold:
            bits = rng() & 0xFFFFFFFF
            prod = bits * lim
    return prod >> 32


def cuckoo_place(keys: Sequence[bytes], family_seed: bytes, num_buckets: int,
                 num_hash_functions: int) -> List[Optional[bytes]]:
    """Build()'s placement: sorted keys, max_relocations = len(keys)."""
    fns = hash_functions(family_seed, num_hash_functions)
    rng = MT19937_64()
    table: List[Optional[bytes]] = [None] * num_buckets
    max_relocations = len(keys)
    for key in sorted(set(keys)):
        cur = key
        for _ in range(max_relocations):
            h = fns[_absl_uniform(rng, num_hash_functions)](cur, num_buckets)
            if table[h] is not None:
                cur, table[h] = table[h], cur
            else:
                table[h] = cur
                cur = None
                break
        # a key still in hand goes to the (unserved) stash
    return table


def cuckoo_tables(records: Dict[bytes, bytes], family_seed: bytes, num_buckets: int,
                  num_hash_functions: int):
    """(key table, value table) rows in bucket order; empty buckets are b""."""
    table = cuckoo_place(list(records), family_seed, num_buckets, num_hash_functions)
    keys = [k if k is not None else b"" for k in table]
    values = [records[k] if k is not None else b"" for k in table]
    return keys, values


def inner_product(rows: Sequence[bytes], selection_bits: Sequence[int]) -> bytes:
    """XOR of the rows whose selection bit is set, zero padded to the longest row."""
    width = max((len(r) for r in rows), default=0)
    acc = bytearray(width)
    for r, bit in zip(rows, selection_bits):
        if bit:
            for i, c in enumerate(r):
                acc[i] ^= c
    return bytes(acc)
