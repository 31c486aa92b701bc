"""ctypes front-end of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product package never does.  See dpf_oracle.h for the
reference file:line each entry point restates.

Value types are given as nested "specs" (the product's ValueType objects
expose the same form through `.spec()`):
    ("int", bits) | ("xor", bits) | ("intmodn", base_bits, modulus)
    | ("tuple", [spec, ...])
Values are nested Python ints / tuples following the same structure and are
flattened in pre-order.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import List, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD_DIR = os.path.join(HERE, "_build")
LIB_PATH = os.path.join(BUILD_DIR, "libdpf_oracle.so")
SRC = os.path.join(HERE, "dpf_oracle.c")

MASK64 = (1 << 64) - 1


def build(force: bool = False) -> str:
    """Compile the oracle with gcc (recipe mirrored in oracle/Makefile)."""
    if (not force and os.path.exists(LIB_PATH)
            and os.path.getmtime(LIB_PATH) >= os.path.getmtime(SRC)):
        return LIB_PATH
    os.makedirs(BUILD_DIR, exist_ok=True)
    tmp = LIB_PATH + ".tmp%d" % os.getpid()
    subprocess.check_call([
        "gcc", "-O3", "-fPIC", "-shared", "-o", tmp, SRC, "-lm"])
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


class VtNode(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("bits", ctypes.c_int32),
                ("n_children", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("mod_lo", ctypes.c_uint64), ("mod_hi", ctypes.c_uint64)]


class OrKey(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64 * 2), ("party", ctypes.c_int32),
                ("num_cw", ctypes.c_int32),
                ("cw_seed", ctypes.POINTER(ctypes.c_uint64)),
                ("cw_ccl", ctypes.POINTER(ctypes.c_uint8)),
                ("cw_ccr", ctypes.POINTER(ctypes.c_uint8)),
                ("num_levels", ctypes.c_int32),
                ("vc_count", ctypes.POINTER(ctypes.c_int32)),
                ("vc", ctypes.POINTER(ctypes.c_uint64))]


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.or_last_error.restype = ctypes.c_char_p
        L.or_dpf_create.argtypes = [ctypes.c_int, P, P, P, P, ctypes.POINTER(P)]
        L.or_dpf_free.argtypes = [P]
        for f in ("or_dpf_tree_levels_needed",):
            getattr(L, f).argtypes = [P]
        for f in ("or_dpf_hierarchy_to_tree", "or_dpf_blocks_needed",
                  "or_dpf_num_scalars", "or_dpf_elements_per_block"):
            getattr(L, f).argtypes = [P, ctypes.c_int]
        L.or_dpf_security_parameter.argtypes = [P, ctypes.c_int]
        L.or_dpf_security_parameter.restype = ctypes.c_double
        L.or_generate_keys.argtypes = [P, ctypes.c_uint64, ctypes.c_uint64, P, P,
                                       ctypes.POINTER(ctypes.POINTER(OrKey)),
                                       ctypes.POINTER(ctypes.POINTER(OrKey))]
        L.or_key_free.argtypes = [ctypes.POINTER(OrKey)]
        L.or_key_alloc.argtypes = [ctypes.c_int, ctypes.c_int, P]
        L.or_key_alloc.restype = ctypes.POINTER(OrKey)
        L.or_ctx_create.argtypes = [P, ctypes.POINTER(OrKey), ctypes.POINTER(P)]
        L.or_ctx_free.argtypes = [P]
        L.or_ctx_previous_hierarchy_level.argtypes = [P]
        L.or_ctx_partial_evaluations_level.argtypes = [P]
        L.or_ctx_num_partial_evaluations.argtypes = [P]
        L.or_ctx_num_partial_evaluations.restype = ctypes.c_int64
        L.or_ctx_partial_evaluations.argtypes = [P, P, P, P]
        L.or_evaluate_until.argtypes = [P, ctypes.c_int, P, ctypes.c_int64, P, P,
                                        ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
        L.or_evaluate_at.argtypes = [P, ctypes.POINTER(OrKey), ctypes.c_int, P,
                                     ctypes.c_int64, P]
        L.or_evaluate_at_ctx.argtypes = [P, ctypes.c_int, P, ctypes.c_int64, P, P]
        L.or_evaluate_seeds.argtypes = [
            ctypes.c_int64, ctypes.c_int, ctypes.c_int64, P, P, P, ctypes.c_int,
            P, P, P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
            ctypes.c_uint64, P, P]
        L.or_expand_subtree.argtypes = [P, ctypes.POINTER(OrKey), ctypes.c_uint64,
                                        ctypes.c_uint64, ctypes.c_int, P]
        L.or_aes_mmo.argtypes = [ctypes.c_uint64, ctypes.c_uint64, P, P,
                                 ctypes.c_int64]
        L.or_aes128_encrypt_block.argtypes = [P, P, P]
        L.or_force_portable_aes.argtypes = [ctypes.c_int]
        L.or_bits_needed.argtypes = [P, ctypes.c_double, ctypes.POINTER(ctypes.c_int)]
        L.or_convert_bytes.argtypes = [P, P, ctypes.c_int64, P]
        L.or_intmodn_sample.argtypes = [P, ctypes.c_int, ctypes.c_uint64,
                                        ctypes.c_uint64, ctypes.c_int, P]
        L.or_intmodn_num_bytes_required.argtypes = [
            ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
            ctypes.c_double, ctypes.POINTER(ctypes.c_int)]
        for f in ("or_vt_num_scalars", "or_vt_elements_per_block",
                  "or_vt_directly_convertible"):
            getattr(L, f).argtypes = [P]
        L.or_inner_product.argtypes = [ctypes.c_int64, P, P, P, ctypes.c_int,
                                       ctypes.c_int64, P, ctypes.c_int64, P]
        L.or_aes_ctr_prng.argtypes = [P, ctypes.c_int64, P]
        _lib = L
    return _lib


class OracleError(Exception):
    def __init__(self, code: int, message: str):
        super().__init__("status %d: %s" % (code, message))
        self.code = code
        self.message = message


def _check(code: int):
    if code != 0:
        raise OracleError(code, lib().or_last_error().decode())


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


# ---------------------------------------------------------------- helpers
def u128_words(values: Sequence[int]) -> np.ndarray:
    if isinstance(values, np.ndarray):  # (n, 2) {lo, hi} words already
        return np.ascontiguousarray(values, dtype=np.uint64).reshape(-1)
    out = np.empty(2 * len(values), dtype=np.uint64)
    for i, v in enumerate(values):
        v = int(v)
        out[2 * i] = v & MASK64
        out[2 * i + 1] = (v >> 64) & MASK64
    return out


def words_u128(words: np.ndarray) -> List[int]:
    w = np.asarray(words, dtype=np.uint64).reshape(-1, 2)
    return [int(lo) | (int(hi) << 64) for lo, hi in w]


def spec_nodes(spec) -> List[Tuple]:
    kind = spec[0]
    if kind == "int":
        return [(1, spec[1], 0, 0)]
    if kind == "xor":
        return [(4, spec[1], 0, 0)]
    if kind == "intmodn":
        return [(3, spec[1], 0, int(spec[2]))]
    if kind == "tuple":
        out = [(2, 0, len(spec[1]), 0)]
        for c in spec[1]:
            out += spec_nodes(c)
        return out
    raise ValueError(spec)


def node_array(spec):
    nodes = spec_nodes(spec)
    arr = (VtNode * len(nodes))()
    for i, (k, b, nc, m) in enumerate(nodes):
        arr[i].kind, arr[i].bits, arr[i].n_children = k, b, nc
        arr[i].mod_lo, arr[i].mod_hi = m & MASK64, m >> 64
    return arr


def flatten_value(spec, value) -> List[int]:
    if spec[0] == "tuple":
        out = []
        for s, v in zip(spec[1], value):
            out += flatten_value(s, v)
        return out
    return [int(value)]


def num_scalars(spec) -> int:
    if spec[0] == "tuple":
        return sum(num_scalars(s) for s in spec[1])
    return 1


def unflatten(spec, scalars: List[int]):
    it = iter(scalars)

    def rec(s):
        if s[0] == "tuple":
            return tuple(rec(c) for c in s[1])
        return next(it)
    return rec(spec)


def scalar_specs(spec) -> List[Tuple]:
    if spec[0] == "tuple":
        out = []
        for s in spec[1]:
            out += scalar_specs(s)
        return out
    return [spec]


def add_values(spec, a, b):
    """Type-correct addition of two (flattened) values (tuple.h, int_mod_n.h,
    xor_wrapper.h)."""
    out = []
    for s, x, y in zip(scalar_specs(spec), a, b):
        if s[0] == "int":
            out.append((x + y) % (1 << s[1]))
        elif s[0] == "xor":
            out.append(x ^ y)
        else:
            out.append((x + y) % s[2])
    return out


# ---------------------------------------------------------------- API
def aes_mmo(key: int, blocks: Sequence[int]) -> List[int]:
    inp = u128_words(blocks)
    out = np.zeros_like(inp)
    _check(lib().or_aes_mmo(key & MASK64, key >> 64, _ptr(inp), _ptr(out), len(blocks)))
    return words_u128(out)


def aes_encrypt_block(key: bytes, block: bytes) -> bytes:
    k = (ctypes.c_uint8 * 16).from_buffer_copy(key)
    b = (ctypes.c_uint8 * 16).from_buffer_copy(block)
    o = (ctypes.c_uint8 * 16)()
    lib().or_aes128_encrypt_block(k, b, o)
    return bytes(o)


def bits_needed(spec, security_parameter: float) -> int:
    out = ctypes.c_int()
    _check(lib().or_bits_needed(node_array(spec), security_parameter, ctypes.byref(out)))
    return out.value


def convert_bytes(spec, data: bytes) -> List[List[int]]:
    """ConvertBytesToArrayOf<T>: returns epb flattened elements."""
    arr = node_array(spec)
    epb = lib().or_vt_elements_per_block(arr)
    ns = num_scalars(spec)
    buf = np.frombuffer(bytes(data), dtype=np.uint8).copy()
    out = np.zeros(2 * epb * ns, dtype=np.uint64)
    _check(lib().or_convert_bytes(arr, _ptr(buf), len(data), _ptr(out)))
    vals = words_u128(out)
    return [vals[i * ns:(i + 1) * ns] for i in range(epb)]


def intmodn_sample(data: bytes, base_bytes: int, modulus: int, n: int) -> List[int]:
    buf = np.frombuffer(bytes(data), dtype=np.uint8).copy()
    out = np.zeros(2 * n, dtype=np.uint64)
    lib().or_intmodn_sample(_ptr(buf), base_bytes, modulus & MASK64, modulus >> 64,
                            n, _ptr(out))
    return words_u128(out)


def evaluate_seeds(seeds, control_bits, paths, paths_rightshift, cw_seeds,
                   ccl, ccr, key_left, key_right, num_levels):
    n = len(seeds)
    s = u128_words(seeds)
    p = u128_words(paths)
    cb = np.asarray(control_bits, dtype=np.uint8).copy()
    cws = u128_words(cw_seeds)
    cl = np.asarray(ccl, dtype=np.uint8).copy()
    cr = np.asarray(ccr, dtype=np.uint8).copy()
    so = np.zeros(max(2 * n, 2), dtype=np.uint64)
    co = np.zeros(max(n, 1), dtype=np.uint8)
    _check(lib().or_evaluate_seeds(
        n, num_levels, len(cw_seeds), _ptr(s), _ptr(cb), _ptr(p), paths_rightshift,
        _ptr(cws), _ptr(cl), _ptr(cr), key_left & MASK64, key_left >> 64,
        key_right & MASK64, key_right >> 64, _ptr(so), _ptr(co)))
    return words_u128(so[:2 * n]), [int(x) for x in co[:n]]


def aes_ctr_prng(seed: bytes, length: int) -> bytes:
    s = (ctypes.c_uint8 * 16).from_buffer_copy(seed)
    out = (ctypes.c_uint8 * max(length, 1))()
    lib().or_aes_ctr_prng(s, length, out)
    return bytes(out)[:length]


def inner_product(records: Sequence[bytes], selections: Sequence[Sequence[int]]):
    """selections[q] = list of 128-bit blocks."""
    n = len(records)
    offsets = np.zeros(max(n, 1), dtype=np.int64)
    sizes = np.zeros(max(n, 1), dtype=np.int64)
    data = bytearray()
    for i, r in enumerate(records):
        offsets[i] = len(data)
        sizes[i] = len(r)
        data += r
    max_size = max([len(r) for r in records] + [0])
    dbuf = np.frombuffer(bytes(data) + b"\0", dtype=np.uint8).copy()
    q = len(selections)
    nb = len(selections[0]) if q else 0
    sel = u128_words([b for s in selections for b in s]) if q else np.zeros(2, np.uint64)
    out = np.zeros(max(q * max_size, 1), dtype=np.uint8)
    _check(lib().or_inner_product(n, _ptr(dbuf), _ptr(offsets), _ptr(sizes), q, nb,
                                  _ptr(sel), max_size, _ptr(out)))
    return [bytes(out[i * max_size:(i + 1) * max_size]) for i in range(q)]


class Key:
    """Flat DpfKey produced by the oracle's keygen (or built from arrays)."""

    def __init__(self, ptr):
        self._p = ptr

    def __del__(self):
        try:
            if self._p:
                lib().or_key_free(self._p)
        except Exception:
            pass

    @property
    def c(self):
        return self._p.contents

    @property
    def seed(self) -> int:
        return int(self.c.seed[0]) | (int(self.c.seed[1]) << 64)

    @property
    def party(self) -> int:
        return int(self.c.party)

    @property
    def num_cw(self) -> int:
        return int(self.c.num_cw)

    def cw_seeds(self) -> List[int]:
        n = self.num_cw
        return [int(self.c.cw_seed[2 * i]) | (int(self.c.cw_seed[2 * i + 1]) << 64)
                for i in range(n)]

    def ccl(self) -> List[int]:
        return [int(self.c.cw_ccl[i]) for i in range(self.num_cw)]

    def ccr(self) -> List[int]:
        return [int(self.c.cw_ccr[i]) for i in range(self.num_cw)]

    def value_corrections(self) -> List[List[int]]:
        out, off = [], 0
        for h in range(self.c.num_levels):
            n = self.c.vc_count[h]
            out.append([int(self.c.vc[2 * (off + j)]) | (int(self.c.vc[2 * (off + j) + 1]) << 64)
                        for j in range(n)])
            off += n
        return out

    @classmethod
    def from_parts(cls, seed, party, cw_seeds, ccl, ccr, vcs):
        counts = (ctypes.c_int32 * len(vcs))(*[len(v) for v in vcs])
        p = lib().or_key_alloc(len(cw_seeds), len(vcs), counts)
        k = p.contents
        k.seed[0], k.seed[1] = seed & MASK64, seed >> 64
        k.party = party
        for i, s in enumerate(cw_seeds):
            k.cw_seed[2 * i] = s & MASK64
            k.cw_seed[2 * i + 1] = s >> 64
            k.cw_ccl[i] = ccl[i]
            k.cw_ccr[i] = ccr[i]
        off = 0
        for v in vcs:
            for x in v:
                k.vc[2 * off] = x & MASK64
                k.vc[2 * off + 1] = x >> 64
                off += 1
        return cls(p)


class Dpf:
    """Oracle DistributedPointFunction (cc:589-640)."""

    def __init__(self, levels):
        """levels: list of (log_domain_size, spec, security_parameter)."""
        self.levels = list(levels)
        n = len(levels)
        lds = (ctypes.c_int32 * n)(*[l[0] for l in levels])
        secs = (ctypes.c_double * n)(*[float(l[2]) for l in levels])
        all_nodes = []
        counts = []
        for l in levels:
            nodes = spec_nodes(l[1])
            all_nodes += nodes
            counts.append(len(nodes))
        arr = (VtNode * len(all_nodes))()
        for i, (k, b, nc, m) in enumerate(all_nodes):
            arr[i].kind, arr[i].bits, arr[i].n_children = k, b, nc
            arr[i].mod_lo, arr[i].mod_hi = m & MASK64, m >> 64
        cnt = (ctypes.c_int32 * n)(*counts)
        h = ctypes.c_void_p()
        _check(lib().or_dpf_create(n, lds, secs, arr, cnt, ctypes.byref(h)))
        self._h = h

    def __del__(self):
        try:
            if self._h:
                lib().or_dpf_free(self._h)
        except Exception:
            pass

    @property
    def tree_levels_needed(self) -> int:
        return lib().or_dpf_tree_levels_needed(self._h)

    def hierarchy_to_tree(self, h: int) -> int:
        return lib().or_dpf_hierarchy_to_tree(self._h, h)

    def blocks_needed(self, h: int) -> int:
        return lib().or_dpf_blocks_needed(self._h, h)

    def elements_per_block(self, h: int) -> int:
        return lib().or_dpf_elements_per_block(self._h, h)

    def security_parameter(self, h: int) -> float:
        return lib().or_dpf_security_parameter(self._h, h)

    def generate_keys(self, alpha: int, betas, seeds=(1, 2)):
        flat = []
        for (ld, spec, _), b in zip(self.levels, betas):
            flat += flatten_value(spec, b)
        bw = u128_words(flat)
        sw = u128_words(list(seeds))
        k0 = ctypes.POINTER(OrKey)()
        k1 = ctypes.POINTER(OrKey)()
        _check(lib().or_generate_keys(self._h, alpha & MASK64, alpha >> 64, _ptr(bw),
                                      _ptr(sw), ctypes.byref(k0), ctypes.byref(k1)))
        return Key(k0), Key(k1)

    def create_evaluation_context(self, key: Key) -> "Ctx":
        c = ctypes.c_void_p()
        _check(lib().or_ctx_create(self._h, key._p, ctypes.byref(c)))
        return Ctx(c, key)

    def evaluate_until(self, level: int, prefixes: Sequence[int], ctx: "Ctx"):
        """Returns a list of flattened elements (lists of ints)."""
        pw = u128_words(prefixes) if len(prefixes) else np.zeros(2, np.uint64)
        cnt = ctypes.c_int64()
        _check(lib().or_evaluate_until(self._h, level, _ptr(pw), len(prefixes), ctx._h,
                                       None, 0, ctypes.byref(cnt)))
        ns = num_scalars(self.levels[level][1])
        out = np.zeros(max(2 * ns * cnt.value, 2), dtype=np.uint64)
        _check(lib().or_evaluate_until(self._h, level, _ptr(pw), len(prefixes), ctx._h,
                                       _ptr(out), cnt.value, ctypes.byref(cnt)))
        return self._elements(out, ns, cnt.value)

    def evaluate_until_words(self, level, prefixes, ctx) -> np.ndarray:
        """As evaluate_until but returns the raw (n, ns, 2) uint64 words."""
        pw = u128_words(prefixes) if len(prefixes) else np.zeros(2, np.uint64)
        cnt = ctypes.c_int64()
        _check(lib().or_evaluate_until(self._h, level, _ptr(pw), len(prefixes), ctx._h,
                                       None, 0, ctypes.byref(cnt)))
        ns = num_scalars(self.levels[level][1])
        out = np.zeros(max(2 * ns * cnt.value, 2), dtype=np.uint64)
        _check(lib().or_evaluate_until(self._h, level, _ptr(pw), len(prefixes), ctx._h,
                                       _ptr(out), cnt.value, ctypes.byref(cnt)))
        return out[:2 * ns * cnt.value].reshape(cnt.value, ns, 2)

    def evaluate_at(self, key: Key, level: int, points: Sequence[int]):
        ns = num_scalars(self.levels[level][1])
        pw = u128_words(points) if len(points) else np.zeros(2, np.uint64)
        out = np.zeros(max(2 * ns * len(points), 2), dtype=np.uint64)
        _check(lib().or_evaluate_at(self._h, key._p, level, _ptr(pw), len(points), _ptr(out)))
        return self._elements(out, ns, len(points))

    def evaluate_at_ctx(self, level: int, points: Sequence[int], ctx: "Ctx"):
        """EvaluateAt<T>(level, points, ctx) (h:356-378)."""
        ns = num_scalars(self.levels[level][1])
        return self._elements(self.evaluate_at_ctx_words(level, points, ctx).reshape(-1),
                              ns, len(points))

    def evaluate_at_ctx_words(self, level: int, points: Sequence[int], ctx: "Ctx"):
        """As evaluate_at_ctx but returns the raw (n, ns, 2) uint64 words."""
        ns = num_scalars(self.levels[level][1])
        pw = u128_words(points) if len(points) else np.zeros(2, np.uint64)
        n = len(points)
        out = np.zeros(max(2 * ns * n, 2), dtype=np.uint64)
        _check(lib().or_evaluate_at_ctx(self._h, level, _ptr(pw), n, ctx._h, _ptr(out)))
        return out[:2 * ns * n].reshape(n, ns, 2)

    def evaluate_at_words(self, key: Key, level: int, points) -> np.ndarray:
        """As evaluate_at but returns the raw (n, ns, 2) uint64 words;
        `points` may be an (n, 2) uint64 {lo, hi} array."""
        ns = num_scalars(self.levels[level][1])
        if isinstance(points, np.ndarray):
            pw = np.ascontiguousarray(points, dtype=np.uint64).reshape(-1)
        else:
            pw = u128_words(points) if len(points) else np.zeros(2, np.uint64)
        n = len(pw) // 2
        out = np.zeros(max(2 * ns * n, 2), dtype=np.uint64)
        _check(lib().or_evaluate_at(self._h, key._p, level, _ptr(pw), n, _ptr(out)))
        return out[:2 * ns * n].reshape(n, ns, 2)

    def expand_subtree_words(self, key: Key, first_block: int, log_blocks: int,
                             out: np.ndarray = None) -> np.ndarray:
        h = len(self.levels) - 1
        ns = num_scalars(self.levels[h][1])
        cepb = 1 << (self.levels[h][0] - self.hierarchy_to_tree(h))
        n = (1 << log_blocks) * cepb
        if out is None:
            out = np.zeros(2 * ns * n, dtype=np.uint64)
        _check(lib().or_expand_subtree(self._h, key._p, first_block & MASK64,
                                       first_block >> 64, log_blocks, _ptr(out)))
        return out

    @staticmethod
    def _elements(words, ns, n):
        vals = words_u128(words[:2 * ns * n])
        return [vals[i * ns:(i + 1) * ns] for i in range(n)]


class Ctx:
    def __init__(self, h, key):
        self._h = h
        self._key = key  # keep alive

    def __del__(self):
        try:
            if self._h:
                lib().or_ctx_free(self._h)
        except Exception:
            pass

    @property
    def previous_hierarchy_level(self) -> int:
        return lib().or_ctx_previous_hierarchy_level(self._h)

    @property
    def partial_evaluations_level(self) -> int:
        return lib().or_ctx_partial_evaluations_level(self._h)

    def partial_evaluations(self):
        n = lib().or_ctx_num_partial_evaluations(self._h)
        p = np.zeros(max(2 * n, 2), np.uint64)
        s = np.zeros(max(2 * n, 2), np.uint64)
        c = np.zeros(max(n, 1), np.uint8)
        lib().or_ctx_partial_evaluations(self._h, _ptr(p), _ptr(s), _ptr(c))
        return list(zip(words_u128(p[:2 * n]), words_u128(s[:2 * n]),
                        [int(x) for x in c[:n]]))
