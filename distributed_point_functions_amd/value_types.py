"""Value types of DPF outputs — the Python mirror of the reference's C++ value
types (uint8..absl::uint128, XorWrapper<T>, Tuple<T...>, IntModN<Base, m>;
dpf/xor_wrapper.h, dpf/tuple.h, dpf/int_mod_n.h) and of the `ValueType` proto
(dpf/distributed_point_function.proto:25-60).

Outputs are produced by the device in the *host C++ layout* of T (what
std::vector<T> would hold on x86-64 with libstdc++: std::tuple stores its
members in reverse order, each naturally aligned).  `numpy_dtype()` exposes
that layout so outputs can be viewed without copies; `decode()` turns them
into Python ints / tuples in declaration order.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

from . import _lib
from . import wire

MASK64 = (1 << 64) - 1
KIND_INTEGER, KIND_TUPLE, KIND_INT_MOD_N, KIND_XOR_WRAPPER = 1, 2, 3, 4


class ValueType:
    """Base class; see Integer, XorWrapper, IntModN, Tuple."""

    kind = 0

    # -- structure -------------------------------------------------------
    def spec(self):
        raise NotImplementedError

    def scalars(self) -> List["ValueType"]:
        return [self]

    @property
    def size(self) -> int:  # sizeof(T)
        raise NotImplementedError

    @property
    def align(self) -> int:  # alignof(T)
        raise NotImplementedError

    def scalar_offsets(self) -> List[int]:
        """Byte offset of each flattened scalar inside one host-layout T."""
        return [0]

    def directly_convertible(self) -> bool:
        return all(s.kind != KIND_INT_MOD_N for s in self.scalars())

    def total_bit_size(self) -> int:
        return sum(s.bits for s in self.scalars())

    def elements_per_block(self) -> int:
        """ElementsPerBlock<T>() (dpf/internal/value_type_helpers.h:525-537)."""
        if self.directly_convertible() and self.total_bit_size() <= 128:
            return 128 // self.total_bit_size()
        return 1

    # -- proto -----------------------------------------------------------
    def to_proto(self) -> bytes:
        """Serialized ValueType proto."""
        raise NotImplementedError

    # -- values ----------------------------------------------------------
    def flatten(self, value) -> List[int]:
        return [int(value)]

    def unflatten(self, it):
        return next(it)

    def zero(self):
        return self.unflatten(iter([0] * len(self.scalars())))

    def add(self, a, b):
        """Type-correct a + b (tuple.h, xor_wrapper.h, int_mod_n.h)."""
        out = []
        for s, x, y in zip(self.scalars(), self.flatten(a), self.flatten(b)):
            if s.kind == KIND_INTEGER:
                out.append((x + y) % (1 << s.bits))
            elif s.kind == KIND_XOR_WRAPPER:
                out.append(x ^ y)
            else:
                out.append((x + y) % s.modulus)
        return self.unflatten(iter(out))

    def value_proto(self, value) -> bytes:
        """Serialized Value proto of `value`."""
        raise NotImplementedError

    # -- host layout -----------------------------------------------------
    def numpy_dtype(self) -> np.dtype:
        names, formats, offsets = [], [], []
        for i, (s, off) in enumerate(zip(self.scalars(), self.scalar_offsets())):
            names.append("f%d" % i)
            nb = s.bits // 8
            formats.append(("<u8", (2,)) if nb == 16 else "<u%d" % nb)
            offsets.append(off)
        return np.dtype({"names": names, "formats": formats, "offsets": offsets,
                         "itemsize": self.size})

    def _columns(self, arr: np.ndarray) -> List[list]:
        """One list of Python ints per scalar (ndarray.tolist converts in C;
        128-bit scalars are (lo, hi) uint64 pairs)."""
        cols = []
        for i, s in enumerate(self.scalars()):
            c = arr["f%d" % i]
            if s.bits == 128:
                lo, hi = c[..., 0].tolist(), c[..., 1].tolist()
                cols.append([a | (b << 64) for a, b in zip(lo, hi)])
            else:
                cols.append(c.tolist())
        return cols

    def decode(self, arr: np.ndarray) -> list:
        """Host-layout array -> list of Python values."""
        cols = self._columns(arr)
        if not cols:
            return []
        if len(cols) == 1 and not isinstance(self, Tuple):
            return cols[0]  # a plain scalar type: the values themselves
        if isinstance(self, Tuple) and not any(isinstance(e, Tuple) for e in self.elements):
            return list(zip(*cols))  # a flat tuple: one Python tuple per element
        return [self.unflatten(iter(vals)) for vals in zip(*cols)]

    def decode_flat(self, arr: np.ndarray) -> List[List[int]]:
        """Host-layout array -> list of flattened scalar lists."""
        return [list(v) for v in zip(*self._columns(arr))]

    def descriptor(self, blocks_needed: int) -> "_lib.ValueTypeDesc":
        """dpf_amd_value_type for Tier-1 calls (blocks_needed from BitsNeeded)."""
        d = _lib.ValueTypeDesc()
        sc = self.scalars()
        if len(sc) > _lib.MAX_SCALARS:
            raise ValueError("too many tuple elements")
        d.num_scalars = len(sc)
        d.directly_convertible = 1 if self.directly_convertible() else 0
        d.elements_per_block = self.elements_per_block()
        d.element_size = (self.total_bit_size() + 7) // 8
        d.blocks_needed = blocks_needed
        d.out_stride = self.size
        in_off = 0
        for i, (s, off) in enumerate(zip(sc, self.scalar_offsets())):
            d.scalars[i].kind = s.kind
            d.scalars[i].bytes = s.bits // 8
            d.scalars[i].in_offset = in_off
            d.scalars[i].out_offset = off
            m = getattr(s, "modulus", 0)
            d.scalars[i].modulus[0] = m & MASK64
            d.scalars[i].modulus[1] = m >> 64
            in_off += s.bits // 8
        return d

    def __eq__(self, other):
        return isinstance(other, ValueType) and self.spec() == other.spec()

    def __hash__(self):
        return hash(repr(self.spec()))

    def __repr__(self):
        return "%s%r" % (type(self).__name__, self.spec()[1:])


def _check_bits(bits):
    if bits not in (8, 16, 32, 64, 128):
        raise ValueError("bitsize must be one of 8, 16, 32, 64, 128")


class Integer(ValueType):
    """uint8_t .. absl::uint128 (ValueType.Integer)."""

    kind = KIND_INTEGER

    def __init__(self, bits: int):
        _check_bits(bits)
        self.bits = bits

    def spec(self):
        return ("int", self.bits)

    @property
    def size(self):
        return self.bits // 8

    @property
    def align(self):
        return self.bits // 8

    def to_proto(self) -> bytes:
        return wire.field_message(1, wire.field_varint(1, self.bits))

    def value_proto(self, value) -> bytes:
        return wire.field_message(1, wire.value_integer(int(value)))


class XorWrapper(Integer):
    """XorWrapper<T> (dpf/xor_wrapper.h): + and - are XOR, negation is identity."""

    kind = KIND_XOR_WRAPPER

    def spec(self):
        return ("xor", self.bits)

    def to_proto(self) -> bytes:
        return wire.field_message(4, wire.field_varint(1, self.bits))

    def value_proto(self, value) -> bytes:
        return wire.field_message(4, wire.value_integer(int(value)))


class IntModN(ValueType):
    """IntModN<BaseInteger, kModulus> (dpf/int_mod_n.h)."""

    kind = KIND_INT_MOD_N

    def __init__(self, base_bits: int, modulus: int):
        _check_bits(base_bits)
        self.bits = base_bits
        self.modulus = int(modulus)

    def spec(self):
        return ("intmodn", self.bits, self.modulus)

    @property
    def size(self):
        return self.bits // 8

    @property
    def align(self):
        return self.bits // 8

    def to_proto(self) -> bytes:
        body = (wire.field_message(1, wire.field_varint(1, self.bits)) +
                wire.field_message(2, wire.value_integer(self.modulus)))
        return wire.field_message(3, body)

    def value_proto(self, value) -> bytes:
        return wire.field_message(3, wire.value_integer(int(value)))


class Tuple(ValueType):
    """Tuple<T...> (dpf/tuple.h)."""

    kind = KIND_TUPLE

    def __init__(self, *elements: ValueType):
        if len(elements) == 1 and isinstance(elements[0], (list, tuple)):
            elements = tuple(elements[0])
        self.elements = list(elements)

    def spec(self):
        return ("tuple", [e.spec() for e in self.elements])

    def scalars(self):
        out = []
        for e in self.elements:
            out += e.scalars()
        return out

    def _element_offsets(self):
        # libstdc++ std::tuple: members in reverse order, naturally aligned.
        offs = [0] * len(self.elements)
        end = 0
        for i in reversed(range(len(self.elements))):
            e = self.elements[i]
            off = (end + e.align - 1) // e.align * e.align
            offs[i] = off
            end = off + e.size
        return offs, end

    @property
    def align(self):
        return max([e.align for e in self.elements] + [1])

    @property
    def size(self):
        _, end = self._element_offsets()
        a = self.align
        return max(1, (end + a - 1) // a * a)

    def scalar_offsets(self):
        offs, _ = self._element_offsets()
        out = []
        for e, o in zip(self.elements, offs):
            out += [o + x for x in e.scalar_offsets()]
        return out

    def to_proto(self) -> bytes:
        body = b"".join(wire.field_message(1, e.to_proto()) for e in self.elements)
        return wire.field_message(2, body)

    def flatten(self, value) -> List[int]:
        if len(value) != len(self.elements):
            raise ValueError("tuple value has the wrong number of elements")
        out = []
        for e, v in zip(self.elements, value):
            out += e.flatten(v)
        return out

    def unflatten(self, it):
        return tuple(e.unflatten(it) for e in self.elements)

    def value_proto(self, value) -> bytes:
        body = b"".join(wire.field_message(1, e.value_proto(v))
                        for e, v in zip(self.elements, value))
        return wire.field_message(2, body)


def from_spec(spec) -> ValueType:
    k = spec[0]
    if k == "int":
        return Integer(spec[1])
    if k == "xor":
        return XorWrapper(spec[1])
    if k == "intmodn":
        return IntModN(spec[1], spec[2])
    if k == "tuple":
        return Tuple(*[from_spec(s) for s in spec[1]])
    raise ValueError(spec)


# Convenience aliases matching the reference's C++ type names.
UINT8, UINT16, UINT32, UINT64, UINT128 = (Integer(8), Integer(16), Integer(32),
                                          Integer(64), Integer(128))


def u128_words(values) -> np.ndarray:
    """128-bit values -> flat {lo, hi} uint64 words.  Accepts a sequence of
    Python ints or an (n, 2) uint64 array of {lo, hi} rows (passed through)."""
    if isinstance(values, np.ndarray):
        if values.dtype != np.uint64 or values.ndim != 2 or values.shape[1] != 2:
            raise ValueError("128-bit arrays must be (n, 2) uint64 {lo, hi} rows")
        return np.ascontiguousarray(values).reshape(-1)
    def small():  # all values in [0, 2^64): converted in C
        arr = np.asarray(values)
        if arr.dtype.kind not in "iu" or arr.ndim != 1 or arr.shape[0] != len(values):
            raise ValueError
        if arr.dtype.kind == "i" and arr.min() < 0:
            # a cast would wrap a negative (numpy) int to 64 bits; the exact
            # path below extends it to 128 bits as absl::uint128 does
            raise ValueError
        lo = arr.astype(np.uint64)
        out = np.zeros((len(values), 2), dtype=np.uint64)
        out[:, 0] = lo
        return out.reshape(-1)

    def wide():  # Python ints in [0, 2^128): their little-endian bytes are the words
        return np.frombuffer(b"".join(v.to_bytes(16, "little") for v in values),
                             dtype=np.uint64).copy()
    # try first the form the first value suggests; either is exact or raises
    first = values[0] if len(values) else 0
    order = (wide, small) if isinstance(first, int) and first >> 64 else (small, wide)
    for f in order:
        try:
            return f()
        except (OverflowError, AttributeError, TypeError, ValueError):
            pass
    lo = np.fromiter((int(v) & MASK64 for v in values), dtype=np.uint64, count=len(values))
    hi = np.fromiter(((int(v) >> 64) & MASK64 for v in values), dtype=np.uint64,
                     count=len(values))
    return np.stack([lo, hi], axis=1).reshape(-1)
