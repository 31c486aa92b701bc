"""EXPERIMENT generator: the last AES round of the
tree expansion's left/right AES pair computed on the VALU instead of the LDS.

Writes distributed_point_functions_amd/csrc/bs_last_round.h (built into the
library only with -DDPF_BS_LAST=1, an A/B variant: tools/build_variants.py).

The two states of Expand2 (the children of one parent, left and right PRG
key) are 8 dwords = 32 bytes.  A 3-layer SWAPMOVE network (12 swaps of bit
groups between register pairs, 4 VALU each) transposes them into 8 bit
planes — plane k holds bit k of all 32 bytes — the Boyar-Peralta S-box
circuit (tools/experiments/gen_bsaes.py) technology-mapped onto 3-input
LUTs (each one v_bitop3_b32) runs once on the planes for all 32 bytes, the
network transposes back, and ShiftRows + the last round key are two v_perm
and one XOR3 per output column.  That replaces the last round's 32 T-table
lookups (and their 32 address v_perm + 16 byte-extraction v_perm) by ~190
VALU operations.  Whether that trade pays depends on the LDS array's load
(90 % busy in the c5 kernel) against the VALU's (45 %) — measured, not
assumed.

The emitted S-box and the transpose network are simulated here on all 256
byte values and on random 32-byte inputs before the header is written.

    python tools/experiments/gen_bs_last_round.py
"""
from __future__ import annotations

import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
import gen_bsaes as G  # noqa: E402

OUT = os.path.join(ROOT, "distributed_point_functions_amd", "csrc", "bs_last_round.h")
M32 = 0xFFFFFFFF

# SWAPMOVE layers: (shift n, mask m, register pairs (a, b)); b's bits under m
# trade places with a's bits under m << n.
LAYERS = [
    (1, 0x55555555, [(0, 1), (2, 3), (4, 5), (6, 7)]),
    (2, 0x33333333, [(0, 2), (1, 3), (4, 6), (5, 7)]),
    (4, 0x0F0F0F0F, [(0, 4), (1, 5), (2, 6), (3, 7)]),
]


def swapmove(R, a, b, n, m):
    ta, tb = (R[a] >> n) & M32, (R[b] << n) & M32
    mb = (m << n) & M32
    R[b], R[a] = (m & ta) | (~m & R[b] & M32), (mb & tb) | (~mb & R[a] & M32)


def transpose(R, inverse=False):
    R = list(R)
    for n, m, pairs in (reversed(LAYERS) if inverse else LAYERS):
        for a, b in pairs:
            swapmove(R, a, b, n, m)
    return R


def check_transpose():
    rng = random.Random(1)
    for _ in range(200):
        R = [rng.getrandbits(32) for _ in range(8)]
        P = transpose(R)
        # plane k, bit 8p + j == bit k of byte p of register j
        for k in range(8):
            for p in range(4):
                for j in range(8):
                    assert (P[k] >> (8 * p + j)) & 1 == (R[j] >> (8 * p + k)) & 1
        assert transpose(P, inverse=True) == R


def sbox_luts():
    c = G.Circ()
    u = [c.inp("u%d" % i) for i in range(8)]  # u0 = MSB
    s = G.add_sbox(c, u, "")
    luts = G.map_luts(c, s)
    return c, u, s, luts


def emit_ops(c, u, s, luts):
    """(dst, leaves, tt) ops over plane registers p[k] (k = bit, LSB first)."""
    ops = []
    for n, leaves in luts:
        ops.append((n, leaves, G.lut_tt(c, n, leaves, {})))
    return ops


def simulate(ops, u, s, planes):
    val = {u[i]: planes[7 - i] for i in range(8)}
    for n, leaves, tt in ops:
        xs = [val[l] for l in leaves] + [0] * (3 - len(leaves))
        a, b, cc = xs
        r = 0
        for bit in range(8):
            if (tt >> bit) & 1:
                ta = a if (bit >> 2) & 1 else ~a
                tb = b if (bit >> 1) & 1 else ~b
                tcc = cc if bit & 1 else ~cc
                r |= ta & tb & tcc
        val[n] = r & M32
    return [val[s[7 - k]] for k in range(8)]


def check_sbox(ops, u, s):
    # 256 byte values in 8 rounds of 32 lanes
    for base in range(0, 256, 32):
        planes = [0] * 8
        for q in range(32):
            x = base + q
            for k in range(8):
                planes[k] |= ((x >> k) & 1) << q
        out = simulate(ops, u, s, planes)
        for q in range(32):
            y = sum(((out[k] >> q) & 1) << k for k in range(8))
            assert y == G.SBOX[base + q], (base + q, y)


def emit_header(ops, u, s):
    name = {u[i]: "p[%d]" % (7 - i) for i in range(8)}
    lines = []
    for idx, (n, leaves, tt) in enumerate(ops):
        v = "v%d" % idx
        args = [name[l] for l in leaves]
        if len(args) == 1:
            args = args * 3
        elif len(args) == 2:
            args = args + [args[1]]
        # the truth table was computed over the leaves in order; a duplicated
        # last leaf only ever sees equal bits, which the table covers
        lines.append("  const uint32_t %s = __builtin_amdgcn_bitop3_b32(%s, %s, %s, 0x%02x);" %
                     (v, args[0], args[1], args[2], tt))
        name[n] = v
    outs = ["  p[%d] = %s;" % (k, name[s[7 - k]]) for k in range(8)]
    sw = []
    for n, m, pairs in LAYERS:
        for a, b in pairs:
            sw.append("  BsSwapMove(R[%d], R[%d], %d, 0x%08xu);" % (a, b, n, m))
    sw_inv = []
    for n, m, pairs in reversed(LAYERS):
        for a, b in pairs:
            sw_inv.append("  BsSwapMove(R[%d], R[%d], %d, 0x%08xu);" % (a, b, n, m))
    return HEADER.format(nluts=len(ops), sbox="\n".join(lines + outs),
                         fwd="\n".join(sw), inv="\n".join(sw_inv))


HEADER = r'''// bs_last_round.h — GENERATED by tools/experiments/gen_bs_last_round.py
// (do not edit).  The last AES round of two states on the VALU: a SWAPMOVE
// bit transpose of the 8 state dwords into 8 planes, the Boyar-Peralta S-box
// as {nluts} v_bitop3_b32 LUTs over all 32 bytes at once, the inverse
// transpose.  Used only when the library is built with -DDPF_BS_LAST=1 (an
// A/B experiment, DESIGN.md §3.1).
#pragma once

#include <cstdint>

namespace dpf_amd {{

// b's bits under m trade places with a's bits under m << n (4 VALU ops).
__device__ __forceinline__ void BsSwapMove(uint32_t& a, uint32_t& b, int n, uint32_t m) {{
  const uint32_t ta = a >> n, tb = b << n, mb = m << n;
  const uint32_t nb = __builtin_amdgcn_bitop3_b32(m, ta, b, 0xca);   // m ? ta : b
  const uint32_t na = __builtin_amdgcn_bitop3_b32(mb, tb, a, 0xca);  // mb ? tb : a
  a = na;
  b = nb;
}}

// p[k]: bit k of 32 bytes -> their S-box images.
__device__ __forceinline__ void BsSbox(uint32_t (&p)[8]) {{
{sbox}
}}

// R[j] (byte p of register j) -> R[k] bit 8p + j = bit k of that byte.
__device__ __forceinline__ void BsTranspose(uint32_t (&R)[8]) {{
{fwd}
}}
__device__ __forceinline__ void BsTransposeBack(uint32_t (&R)[8]) {{
{inv}
}}

// SubBytes of 8 dwords (two AES states, column words), in place.
__device__ __forceinline__ void BsSubBytes8(uint32_t (&R)[8]) {{
  BsTranspose(R);
  BsSbox(R);
  BsTransposeBack(R);
}}

}}  // namespace dpf_amd
'''


def main():
    check_transpose()
    c, u, s, luts = sbox_luts()
    ops = emit_ops(c, u, s, luts)
    check_sbox(ops, u, s)
    # end to end on random dwords: transpose, S-box, back == bytewise S-box
    rng = random.Random(2)
    for _ in range(100):
        R = [rng.getrandbits(32) for _ in range(8)]
        P = simulate(ops, u, s, transpose(R))
        B = transpose(P, inverse=True)
        want = [sum(G.SBOX[(r >> (8 * q)) & 255] << (8 * q) for q in range(4)) for r in R]
        assert B == want
    with open(OUT, "w") as f:
        f.write(emit_header(ops, u, s))
    print("wrote %s: %d S-box LUTs + 2 x 48 transpose ops" % (OUT, len(ops)))


if __name__ == "__main__":
    main()
