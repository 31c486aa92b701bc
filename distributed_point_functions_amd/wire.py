"""Protocol-buffers wire format (encoding + a generic decoder) for the
reference's messages (dpf/distributed_point_function.proto,
pir/private_information_retrieval.proto).  No protobuf runtime or generated
code is needed: the native library parses the same bytes in C++
(csrc/wire.cc), so serialized DpfKey / EvaluationContext / PirRequest /
PirResponse messages are interchangeable with the reference's.
"""
from __future__ import annotations

import struct
from typing import Dict, List, Tuple

MASK64 = (1 << 64) - 1


def varint(v: int) -> bytes:
    v &= MASK64  # negative int32/int64 encode as 10-byte two's complement
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def tag(field: int, wire_type: int) -> bytes:
    return varint((field << 3) | wire_type)


def field_varint(field: int, v: int) -> bytes:
    return tag(field, 0) + varint(v)


def field_bytes(field: int, data: bytes) -> bytes:
    return tag(field, 2) + varint(len(data)) + data


field_message = field_bytes


def field_double(field: int, v: float) -> bytes:
    return tag(field, 1) + struct.pack("<d", v)


def block(v: int) -> bytes:
    """Block{high=1, low=2}; proto3 omits zero scalars."""
    hi, lo = (v >> 64) & MASK64, v & MASK64
    out = b""
    if hi:
        out += field_varint(1, hi)
    if lo:
        out += field_varint(2, lo)
    return out


def value_integer(v: int) -> bytes:
    """Value.Integer as written by Uint128ToValueInteger
    (dpf/internal/value_type_helpers.cc:145-155)."""
    if v >> 64 == 0:
        return field_varint(1, v)
    return field_message(2, block(v))


def decode(data: bytes) -> Dict[int, List]:
    """Generic decoder: field number -> list of raw values (int for varint /
    fixed, bytes for length-delimited)."""
    out: Dict[int, List] = {}
    i, n = 0, len(data)
    while i < n:
        key, i = _read_varint(data, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(data, i)
        elif wt == 1:
            v = struct.unpack_from("<Q", data, i)[0]
            i += 8
        elif wt == 2:
            ln, i = _read_varint(data, i)
            v = bytes(data[i:i + ln])
            i += ln
        elif wt == 5:
            v = struct.unpack_from("<I", data, i)[0]
            i += 4
        else:
            raise ValueError("unsupported wire type %d" % wt)
        out.setdefault(f, []).append(v)
    return out


def _read_varint(data: bytes, i: int) -> Tuple[int, int]:
    shift, v = 0, 0
    while True:
        b = data[i]
        i += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, i
        shift += 7


def as_int32(v: int) -> int:
    v &= MASK64
    return v - (1 << 64) if v >> 63 else v


def decode_block(data: bytes) -> int:
    d = decode(data)
    return (d.get(1, [0])[-1] << 64) | d.get(2, [0])[-1]


def decode_value_integer(data: bytes) -> int:
    d = decode(data)
    if 2 in d:
        return decode_block(d[2][-1])
    return d.get(1, [0])[-1]
