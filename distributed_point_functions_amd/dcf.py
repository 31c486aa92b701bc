"""Python mirror of the reference's DistributedComparisonFunction
(dcf/distributed_comparison_function.h:30-187) over the Tier-2 C ABI.

A DCF with parameters (n, T) is an incremental DPF with n hierarchy levels of
log domain 0..n-1; keys evaluate to shares of beta on x < alpha and of 0
otherwise.  BatchEvaluate runs as one fused gfx950 kernel.  Keys travel as
serialized DcfKey protos; errors raise DpfAmdError with the reference's
status code and message.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _lib, wire
from ._lib import check, take_buffer
from .dpf import DpfKey, DpfParameters, _seq
from .value_types import ValueType, u128_words

MASK64 = (1 << 64) - 1


@dataclass
class DcfParameters:
    """DcfParameters proto (dcf/distributed_comparison_function.proto:25-28)."""

    parameters: DpfParameters

    def to_proto(self) -> bytes:
        return wire.field_message(1, self.parameters.to_proto())


class DcfKey:
    """A serialized DcfKey proto (proto:30-32); `.key` is the DpfKey."""

    def __init__(self, data: bytes):
        self.data = bytes(data)
        d = wire.decode(self.data)
        self.key = DpfKey(d[1][-1]) if 1 in d else DpfKey(b"")

    def __bytes__(self):
        return self.data

    def __eq__(self, other):
        return isinstance(other, DcfKey) and self.data == other.data


class DistributedComparisonFunction:
    """DistributedComparisonFunction (dcf/distributed_comparison_function.h:30)."""

    def __init__(self, handle, parameters: DcfParameters):
        self._h = handle
        self.parameters = parameters

    def __del__(self):
        try:
            if self._h:
                _lib.lib().dpf_amd_dcf_destroy(self._h)
        except Exception:
            pass

    @classmethod
    def create(cls, parameters: DcfParameters) -> "DistributedComparisonFunction":
        data = parameters.to_proto()
        h = ctypes.c_void_p()
        check(_lib.lib().dpf_amd_dcf_create(data, len(data), ctypes.byref(h)))
        return cls(h, parameters)

    @property
    def value_type(self) -> ValueType:
        return self.parameters.parameters.value_type

    def generate_keys(self, alpha: int, beta, seeds: Optional[Sequence[int]] = None):
        """Keys for shares of `beta` on x < alpha (dcf.cc:81-111).  `seeds`
        (two 128-bit ints) replaces the CSPRNG for reproducible fixtures."""
        if not isinstance(beta, bytes):  # templated GenerateKeys<T>: ToValue<T> registers T
            tp = self.value_type.to_proto()
            check(_lib.lib().dpf_amd_dcf_register_value_type(self._h, tp, len(tp)))
        b = beta if isinstance(beta, bytes) else self.value_type.value_proto(beta)
        sw = u128_words(list(seeds)) if seeds is not None else None
        k0 = ctypes.POINTER(ctypes.c_uint8)()
        k1 = ctypes.POINTER(ctypes.c_uint8)()
        n0, n1 = ctypes.c_size_t(), ctypes.c_size_t()
        check(_lib.lib().dpf_amd_dcf_generate_keys(
            self._h, alpha & MASK64, (alpha >> 64) & MASK64, b, len(b),
            sw.ctypes.data_as(ctypes.c_void_p) if sw is not None else None,
            ctypes.byref(k0), ctypes.byref(n0), ctypes.byref(k1), ctypes.byref(n1)))
        return DcfKey(take_buffer(k0, n0)), DcfKey(take_buffer(k1, n1))

    def batch_evaluate(self, keys: Sequence[DcfKey], evaluation_points, raw: bool = False,
                       value_type: ValueType = None):
        """BatchEvaluate<T> (h:141-187): keys[i] at evaluation_points[i]."""
        vt = value_type or self.value_type
        tp = vt.to_proto()
        datas = [bytes(k) for k in keys]
        arr = (ctypes.c_char_p * max(len(datas), 1))(*datas)
        lens = (ctypes.c_size_t * max(len(datas), 1))(*[len(d) for d in datas])
        npts = len(evaluation_points)
        pw = u128_words(_seq(evaluation_points)) if npts else np.zeros(2, np.uint64)
        out = np.zeros(max(len(keys), 1), dtype=vt.numpy_dtype())
        check(_lib.lib().dpf_amd_dcf_batch_evaluate(
            self._h, arr, lens, len(keys), pw.ctypes.data_as(ctypes.c_void_p), npts, tp,
            len(tp), out.ctypes.data_as(ctypes.c_void_p)))
        out = out[:len(keys)]
        return out if raw else vt.decode(out)

    def evaluate(self, key: DcfKey, x: int, value_type: ValueType = None):
        """Evaluate<T>(key, x) (h:99-110)."""
        return self.batch_evaluate([key], [x], value_type=value_type)[0]
