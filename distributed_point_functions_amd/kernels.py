"""Python entry points of the Tier-1 device seams (include/dpf_amd.h), taking
torch tensors that already live in HBM.  128-bit arrays are int64 tensors of
shape (n, 2) holding {lo, hi} words; control bits are uint8 tensors.

These are thin launchers: every call goes straight to a HIP kernel on the
current torch stream.  Nothing here falls back to the CPU.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, dptr, stream_ptr


def u128_tensor(values, device="cuda") -> torch.Tensor:
    """Python ints -> (n, 2) int64 device tensor of {lo, hi} words."""
    w = np.zeros((len(values), 2), dtype=np.uint64)
    for i, v in enumerate(values):
        v = int(v)
        w[i, 0] = v & 0xFFFFFFFFFFFFFFFF
        w[i, 1] = (v >> 64) & 0xFFFFFFFFFFFFFFFF
    return torch.from_numpy(w.view(np.int64)).to(device)


def tensor_u128(t: torch.Tensor):
    w = t.detach().cpu().numpy().view(np.uint64).reshape(-1, 2)
    return [int(lo) | (int(hi) << 64) for lo, hi in w]


def _words(t):
    if t.dtype != torch.int64 or t.dim() != 2 or t.shape[1] != 2 or not t.is_contiguous():
        raise ValueError("128-bit arrays must be contiguous (n, 2) int64 tensors")
    return t


def aes128_mmo(key: int, blocks: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """Aes128FixedKeyHash(key).Evaluate (dpf/aes_128_fixed_key_hash.cc:57-98)."""
    _words(blocks)
    if out is None:
        out = torch.empty_like(blocks)
    check(_lib.lib().dpf_amd_aes128_mmo(key & 0xFFFFFFFFFFFFFFFF, key >> 64, dptr(blocks),
                                        dptr(out), blocks.shape[0], stream_ptr()))
    return out


def evaluate_seeds(seeds, control_bits, paths, paths_rightshift, correction_seeds,
                   ccl, ccr, key_left: int, key_right: int, num_levels: int,
                   seeds_out=None, control_bits_out=None):
    """dpf_internal::EvaluateSeeds (dpf/internal/evaluate_prg_hwy.h:70-77)."""
    n = seeds.shape[0]
    if seeds_out is None:
        seeds_out = torch.empty_like(seeds)
    if control_bits_out is None:
        control_bits_out = torch.empty_like(control_bits)
    M = 0xFFFFFFFFFFFFFFFF
    check(_lib.lib().dpf_amd_evaluate_seeds(
        n, num_levels, correction_seeds.shape[0], dptr(seeds), dptr(control_bits),
        dptr(paths), paths_rightshift, dptr(correction_seeds), dptr(ccl), dptr(ccr),
        key_left & M, key_left >> 64, key_right & M, key_right >> 64,
        dptr(seeds_out), dptr(control_bits_out), stream_ptr()))
    return seeds_out, control_bits_out


def _corr_words(values):
    w = np.zeros(2 * max(len(values), 1), dtype=np.uint64)
    for i, v in enumerate(values):
        w[2 * i] = int(v) & 0xFFFFFFFFFFFFFFFF
        w[2 * i + 1] = int(v) >> 64
    return w


def expand_and_correct(root_seeds, root_control_bits, num_levels, cw_seeds, ccl, ccr,
                       desc: "_lib.ValueTypeDesc", value_correction, party: int,
                       corrected_elements_per_block: int, leaf_begin: int = 0,
                       leaf_end: int = None, out: torch.Tensor = None):
    """Fused ExpandSeeds + HashExpandedSeeds + value correction (see
    dpf_amd_expand_and_correct).  Returns a uint8 tensor of host-layout T."""
    n = root_seeds.shape[0]
    if leaf_end is None:
        leaf_end = n << num_levels
    count = (leaf_end - leaf_begin) * corrected_elements_per_block
    if out is None:
        out = torch.empty(count * desc.out_stride, dtype=torch.uint8,
                          device=root_seeds.device)
    elif out.numel() * out.element_size() < count * desc.out_stride:
        raise ValueError("output buffer too small")
    corr = _corr_words(value_correction)
    check(_lib.lib().dpf_amd_expand_and_correct(
        n, dptr(root_seeds), dptr(root_control_bits), num_levels, dptr(cw_seeds),
        dptr(ccl), dptr(ccr), ctypes.byref(desc),
        corr.ctypes.data_as(ctypes.c_void_p), party, corrected_elements_per_block,
        leaf_begin, leaf_end, dptr(out), stream_ptr()))
    return out


def expand_and_correct_batched(root_seeds, root_control_bits, num_levels, cw_seeds, ccl, ccr,
                               desc: "_lib.ValueTypeDesc", value_corrections, parties,
                               corrected_elements_per_block: int, leaf_begin: int = 0,
                               leaf_end: int = None, out: torch.Tensor = None):
    """Leaves [leaf_begin, leaf_end) of every key in one launch (see
    dpf_amd_expand_and_correct_batched): root_seeds (q, 2) int64, control
    bits (q,), cw_seeds (q * num_levels, 2), ccl / ccr (q * num_levels,);
    value_corrections: q lists of 128-bit words, parties: q ints.  Returns a
    uint8 tensor: key k's host-layout values after key k - 1's."""
    q = root_seeds.shape[0]
    if leaf_end is None:
        leaf_end = 1 << num_levels
    count = q * (leaf_end - leaf_begin) * corrected_elements_per_block
    if out is None:
        out = torch.empty(count * desc.out_stride, dtype=torch.uint8, device=root_seeds.device)
    elif out.numel() * out.element_size() < count * desc.out_stride:
        raise ValueError("output buffer too small")
    corr = _corr_words([w for vc in value_corrections for w in vc])
    pa = np.ascontiguousarray(parties, dtype=np.int8)
    check(_lib.lib().dpf_amd_expand_and_correct_batched(
        q, dptr(root_seeds), dptr(root_control_bits), num_levels, dptr(cw_seeds), dptr(ccl),
        dptr(ccr), ctypes.byref(desc), corr.ctypes.data_as(ctypes.c_void_p),
        pa.ctypes.data_as(ctypes.c_void_p), corrected_elements_per_block, leaf_begin, leaf_end,
        dptr(out), stream_ptr()))
    return out


class forced_expand_depth:
    """Context manager forcing the fused expansion kernel's register-DFS
    depth (dpf_amd_set_expand_depth; tests run the deep kernels that large
    launches select on small domains)."""

    def __init__(self, depth: int):
        self.depth = depth

    def __enter__(self):
        prev = _lib.lib().dpf_amd_set_expand_depth(self.depth)
        if prev == -99:
            raise ValueError("expand depth must be 0, 1, 2, 4, 5, 6, 8, -1, -2 or -3")
        self.prev = prev
        return self

    def __exit__(self, *exc):
        _lib.lib().dpf_amd_set_expand_depth(self.prev)


class forced_expand_roots:
    """Context manager for the roots stage of large expansions
    (dpf_amd_set_expand_roots: -1 automatic, 0 never, 1 whenever eligible)."""

    def __init__(self, mode: int):
        self.mode = mode

    def __enter__(self):
        prev = _lib.lib().dpf_amd_set_expand_roots(self.mode)
        if prev < -1:
            raise ValueError("expand roots mode must be -1, 0 or 1")
        self.prev = prev
        return self

    def __exit__(self, *exc):
        _lib.lib().dpf_amd_set_expand_roots(self.prev)


class forced_scan_m4:
    """Context manager selecting dpf_amd_inner_product's scan kernel
    (dpf_amd_set_scan_m4: -1 automatic, 0 masked scan, 1 Four-Russians)."""

    def __init__(self, mode: int):
        self.mode = mode

    def __enter__(self):
        prev = _lib.lib().dpf_amd_set_scan_m4(self.mode)
        if prev < -1:
            raise ValueError("scan mode must be -1, 0 or 1")
        self.prev = prev
        return self

    def __exit__(self, *exc):
        _lib.lib().dpf_amd_set_scan_m4(self.prev)


class scan_skip_unselected:
    """Context manager for the opt-in scan that reads only selected records
    (dpf_amd_set_scan_skip_unselected: 1 skip, as the reference's scan; 0
    read every record, the default)."""

    def __init__(self, on: int = 1):
        self.on = int(on)

    def __enter__(self):
        prev = _lib.lib().dpf_amd_set_scan_skip_unselected(self.on)
        if prev < 0:
            raise ValueError("scan skip must be 0 or 1")
        self.prev = prev
        return self

    def __exit__(self, *exc):
        _lib.lib().dpf_amd_set_scan_skip_unselected(self.prev)


class forced_walk_mode:
    """Context manager selecting the point-walk kernel of this thread
    (dpf_amd_set_walk_mode: 0 automatic, 1 four lanes per point, 2 one lane
    per point)."""

    def __init__(self, mode: int):
        self.mode = mode

    def __enter__(self):
        prev = _lib.lib().dpf_amd_set_walk_mode(self.mode)
        if prev < 0:
            raise ValueError("walk mode must be 0, 1 or 2")
        self.prev = prev
        return self

    def __exit__(self, *exc):
        _lib.lib().dpf_amd_set_walk_mode(self.prev)


class forced_dcf_kernel:
    """Context manager selecting this thread's DCF kernel
    (dpf_amd_set_dcf_kernel: 0 automatic, 1 generic)."""

    def __init__(self, mode: int):
        self.mode = mode

    def __enter__(self):
        prev = _lib.lib().dpf_amd_set_dcf_kernel(self.mode)
        if prev < 0:
            raise ValueError("dcf kernel mode must be 0 or 1")
        self.prev = prev
        return self

    def __exit__(self, *exc):
        _lib.lib().dpf_amd_set_dcf_kernel(self.prev)


def evaluate_points(seeds, control_bits, paths, paths_rightshift, num_levels,
                    cw_seeds, ccl, ccr, desc, block_index=None, party=None,
                    party_all: int = 0, value_corrections=None,
                    value_correction_all=(), out=None, seeds_out=None,
                    control_bits_out=None):
    """Fused path walk + value hash + correction (dpf_amd_evaluate_points)."""
    n = seeds.shape[0]
    if out is None:
        out = torch.empty(n * desc.out_stride, dtype=torch.uint8, device=seeds.device)
    corr = _corr_words(value_correction_all)
    check(_lib.lib().dpf_amd_evaluate_points(
        n, dptr(seeds), dptr(control_bits), dptr(paths), paths_rightshift, num_levels,
        cw_seeds.shape[0], dptr(cw_seeds), dptr(ccl), dptr(ccr), ctypes.byref(desc),
        dptr(block_index), dptr(party), party_all, dptr(value_corrections),
        corr.ctypes.data_as(ctypes.c_void_p), dptr(out), dptr(seeds_out),
        dptr(control_bits_out), stream_ptr()))
    return out


def evaluate_points_batched(num_keys: int, points_per_key: int, key_seeds, key_control_bits,
                            paths, paths_rightshift: int, num_levels: int, cw_seeds, ccl, ccr,
                            desc, block_index=None, key_party=None, party_all: int = 0,
                            key_value_corrections=None, value_correction_all=(), out=None):
    """Batched EvaluateAt over num_keys keys (dpf_amd_evaluate_points_batched):
    point k * points_per_key + j belongs to key k; correction words are
    [key][level] arrays; paths None = point j of each key is tree index j."""
    n = num_keys * points_per_key
    if out is None:
        out = torch.empty(n * desc.out_stride, dtype=torch.uint8, device=key_seeds.device)
    corr = _corr_words(value_correction_all)
    check(_lib.lib().dpf_amd_evaluate_points_batched(
        num_keys, points_per_key, dptr(key_seeds), dptr(key_control_bits), dptr(paths),
        paths_rightshift, num_levels, dptr(cw_seeds), dptr(ccl), dptr(ccr), ctypes.byref(desc),
        dptr(block_index), dptr(key_party), party_all, dptr(key_value_corrections),
        corr.ctypes.data_as(ctypes.c_void_p), dptr(out), stream_ptr()))
    return out


def inner_product(db: torch.Tensor, num_records: int, record_stride: int,
                  selections: torch.Tensor, num_queries: int,
                  workspace: torch.Tensor = None, out: torch.Tensor = None):
    """XOR inner product of HBM-resident records with selection bit-vectors
    (pir_internal::InnerProduct semantics).  selections: (Q * blocks, 2) int64."""
    blocks = selections.shape[0] // max(num_queries, 1)
    L = _lib.lib()
    ws = L.dpf_amd_inner_product_workspace_size(num_records, record_stride, num_queries)
    if workspace is None or workspace.numel() < ws:
        workspace = torch.empty(max(ws, 16), dtype=torch.uint8, device=db.device)
    if out is None:
        out = torch.empty(num_queries * record_stride, dtype=torch.uint8, device=db.device)
    check(L.dpf_amd_inner_product(dptr(db), num_records, record_stride, dptr(selections),
                                  blocks, num_queries, dptr(workspace), dptr(out),
                                  stream_ptr()))
    return out


def gather_rows(src_offset: torch.Tensor, outputs_per_prefix: int, stride: int,
                rows: torch.Tensor, out: torch.Tensor = None):
    """out[i * opp + k] = rows[src_offset[i] + k] for rows of `stride` bytes
    (dpf_amd_gather_rows, the per-prefix slices of EvaluateUntil h:877-889)."""
    n = src_offset.numel()
    if out is None:
        out = torch.empty(n * outputs_per_prefix * stride, dtype=torch.uint8, device=rows.device)
    check(_lib.lib().dpf_amd_gather_rows(n, dptr(src_offset), outputs_per_prefix, stride,
                                         dptr(rows), dptr(out), stream_ptr()))
    return out


def xor_fold(parts: torch.Tensor, num_parts: int, nbytes: int, out=None):
    if out is None:
        out = torch.empty(nbytes, dtype=torch.uint8, device=parts.device)
    check(_lib.lib().dpf_amd_xor_fold(dptr(parts), num_parts, nbytes, dptr(out),
                                      stream_ptr()))
    return out
