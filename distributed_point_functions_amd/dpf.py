"""Python mirror of the reference's DistributedPointFunction
(dpf/distributed_point_function.h:87-639) over the Tier-2 C ABI.

Method names follow the reference (snake_case), arguments keep their
meaning, and failures raise DpfAmdError carrying the absl::StatusCode number
and the reference's message.  Keys and contexts travel as protobuf wire
bytes (DpfKey / EvaluationContext), so they interoperate with the
reference's serialized protos.  All evaluation runs on the GPU.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

import numpy as np

from . import _lib, wire
from ._lib import check, take_buffer
from .value_types import ValueType, u128_words

MASK64 = (1 << 64) - 1


@dataclass
class DpfParameters:
    """DpfParameters proto (dpf/distributed_point_function.proto:92-105)."""

    log_domain_size: int
    value_type: ValueType
    security_parameter: float = 0.0

    def to_proto(self) -> bytes:
        out = b""
        if self.log_domain_size:
            out += wire.field_varint(1, self.log_domain_size)
        out += wire.field_message(3, self.value_type.to_proto())
        out += wire.field_double(4, self.security_parameter) if self.security_parameter else b""
        return out


@dataclass
class CorrectionWord:
    seed: int = 0
    control_left: bool = False
    control_right: bool = False
    value_correction: List[bytes] = field(default_factory=list)  # Value protos


class DpfKey:
    """A serialized DpfKey proto with decoded accessors
    (dpf/distributed_point_function.proto:137-148)."""

    def __init__(self, data: bytes):
        self.data = bytes(data)
        d = wire.decode(self.data)
        self.seed = wire.decode_block(d[1][-1]) if 1 in d else 0
        self.has_seed = 1 in d
        self.party = wire.as_int32(d.get(3, [0])[-1])
        self.correction_words = []
        for cw in d.get(2, []):
            c = wire.decode(cw)
            self.correction_words.append(CorrectionWord(
                seed=wire.decode_block(c[1][-1]) if 1 in c else 0,
                control_left=bool(c.get(2, [0])[-1]),
                control_right=bool(c.get(3, [0])[-1]),
                value_correction=list(c.get(5, []))))
        self.last_level_value_correction = list(d.get(5, []))

    def __bytes__(self):
        return self.data

    def __eq__(self, other):
        return isinstance(other, DpfKey) and self.data == other.data

    @staticmethod
    def build(seed: int, party: int, cws: Sequence[CorrectionWord],
              last_level_value_correction: Sequence[bytes]) -> "DpfKey":
        out = wire.field_message(1, wire.block(seed))
        for c in cws:
            body = wire.field_message(1, wire.block(c.seed))
            body += wire.field_varint(2, 1) if c.control_left else b""
            body += wire.field_varint(3, 1) if c.control_right else b""
            body += b"".join(wire.field_message(5, v) for v in c.value_correction)
            out += wire.field_message(2, body)
        if party:
            out += wire.field_varint(3, party)
        out += b"".join(wire.field_message(5, v) for v in last_level_value_correction)
        return DpfKey(out)


def _seq(values):
    """128-bit inputs: an (n, 2) uint64 {lo, hi} array as is, else a list."""
    return values if isinstance(values, np.ndarray) else list(values)


def decode_value(vt: ValueType, data: bytes):
    """Value proto -> flattened scalars of `vt`."""
    d = wire.decode(data)
    if vt.kind == 2:
        els = wire.decode(d[2][-1]).get(1, []) if 2 in d else []
        out = []
        for e, ed in zip(vt.elements, els):
            out += decode_value(e, ed)
        return out
    case = {1: 1, 3: 3, 4: 4}[vt.kind]
    return [wire.decode_value_integer(d[case][-1])] if case in d else [0]


class EvaluationContext:
    """EvaluationContext proto held by the native library (handle)."""

    def __init__(self, handle, dpf: "DistributedPointFunction"):
        self._h = handle
        self._dpf = dpf

    def __del__(self):
        try:
            if self._h:
                _lib.lib().dpf_amd_ctx_destroy(self._h)
        except Exception:
            pass

    @property
    def previous_hierarchy_level(self) -> int:
        return _lib.lib().dpf_amd_ctx_previous_hierarchy_level(self._h)

    @property
    def partial_evaluations_level(self) -> int:
        return _lib.lib().dpf_amd_ctx_partial_evaluations_level(self._h)

    @property
    def num_partial_evaluations(self) -> int:
        return _lib.lib().dpf_amd_ctx_num_partial_evaluations(self._h)

    def serialize(self) -> bytes:
        buf = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        check(_lib.lib().dpf_amd_ctx_serialize(self._h, ctypes.byref(buf), ctypes.byref(n)))
        return take_buffer(buf, n)

    def partial_evaluations(self):
        """[(prefix, seed, control_bit)] decoded from the proto."""
        d = wire.decode(self.serialize())
        out = []
        for pe in d.get(4, []):
            p = wire.decode(pe)
            out.append((wire.decode_block(p[1][-1]) if 1 in p else 0,
                        wire.decode_block(p[2][-1]) if 2 in p else 0,
                        bool(p.get(3, [0])[-1])))
        return out


class DistributedPointFunction:
    """DistributedPointFunction (dpf/distributed_point_function.h:87)."""

    def __init__(self, handle, parameters: List[DpfParameters]):
        self._h = handle
        self.parameters = parameters

    def __del__(self):
        try:
            if self._h:
                _lib.lib().dpf_amd_dpf_destroy(self._h)
        except Exception:
            pass

    # -- construction ------------------------------------------------------
    @classmethod
    def create(cls, parameters: DpfParameters) -> "DistributedPointFunction":
        return cls.create_incremental([parameters])

    @classmethod
    def create_incremental(cls, parameters: Sequence[DpfParameters]
                           ) -> "DistributedPointFunction":
        protos = [p.to_proto() for p in parameters]
        arr = (ctypes.c_char_p * max(len(protos), 1))(*protos)
        lens = (ctypes.c_size_t * max(len(protos), 1))(*[len(p) for p in protos])
        h = ctypes.c_void_p()
        check(_lib.lib().dpf_amd_dpf_create_incremental(arr, lens, len(protos),
                                                        ctypes.byref(h)))
        return cls(h, list(parameters))

    @property
    def tree_levels_needed(self) -> int:
        return _lib.lib().dpf_amd_dpf_tree_levels_needed(self._h)

    def hierarchy_to_tree(self, level: int) -> int:
        return _lib.lib().dpf_amd_dpf_hierarchy_to_tree(self._h, level)

    def value_type_descriptor(self, level: int) -> "_lib.ValueTypeDesc":
        d = _lib.ValueTypeDesc()
        check(_lib.lib().dpf_amd_dpf_value_type(self._h, level, ctypes.byref(d)))
        return d

    # -- keys ----------------------------------------------------------------
    def register_value_type(self, value_type: ValueType) -> None:
        """RegisterValueType<T>() (h:129-131)."""
        tp = value_type.to_proto()
        check(_lib.lib().dpf_amd_dpf_register_value_type(self._h, tp, len(tp)))

    def generate_keys(self, alpha: int, beta, seeds: Optional[Sequence[int]] = None):
        return self.generate_keys_incremental(alpha, [beta], seeds)

    def generate_keys_incremental(self, alpha: int, betas: Sequence,
                                  seeds: Optional[Sequence[int]] = None):
        """betas[i]: a Python value of parameters[i].value_type (or raw Value
        proto bytes).  A Python value is converted like the reference's
        templated overloads, which register its type (ToValue<T>, h:112-118);
        raw Value bytes need the type registered (register_value_type) unless
        it is a single unsigned integer.  `seeds` (two 128-bit ints) replaces
        the CSPRNG for reproducible fixtures only."""
        for p, b in zip(self.parameters, betas):
            if not isinstance(b, bytes):
                self.register_value_type(p.value_type)
        if len(betas) != len(self.parameters):
            protos = [b if isinstance(b, bytes) else b"" for b in betas]
        else:
            protos = [b if isinstance(b, bytes) else p.value_type.value_proto(b)
                      for p, b in zip(self.parameters, betas)]
        n = len(self.parameters)
        protos = (protos + [b""] * n)[:max(n, len(protos))]
        arr = (ctypes.c_char_p * max(len(protos), 1))(*protos)
        lens = (ctypes.c_size_t * max(len(protos), 1))(*[len(p) for p in protos])
        sw = None
        if seeds is not None:
            sw = u128_words(list(seeds))
        k0 = ctypes.POINTER(ctypes.c_uint8)()
        k1 = ctypes.POINTER(ctypes.c_uint8)()
        n0, n1 = ctypes.c_size_t(), ctypes.c_size_t()
        if len(betas) != n:
            raise _lib.DpfAmdError(3, "`beta` has to have the same size as `parameters` "
                                      "passed at construction")
        check(_lib.lib().dpf_amd_dpf_generate_keys(
            self._h, alpha & MASK64, (alpha >> 64) & MASK64, arr, lens,
            sw.ctypes.data_as(ctypes.c_void_p) if sw is not None else None,
            ctypes.byref(k0), ctypes.byref(n0), ctypes.byref(k1), ctypes.byref(n1)))
        return DpfKey(take_buffer(k0, n0)), DpfKey(take_buffer(k1, n1))

    def create_evaluation_context(self, key: DpfKey) -> EvaluationContext:
        data = bytes(key)
        h = ctypes.c_void_p()
        check(_lib.lib().dpf_amd_ctx_create(self._h, data, len(data), ctypes.byref(h)))
        return EvaluationContext(h, self)

    def parse_evaluation_context(self, data: bytes) -> EvaluationContext:
        h = ctypes.c_void_p()
        check(_lib.lib().dpf_amd_ctx_parse(self._h, data, len(data), ctypes.byref(h)))
        return EvaluationContext(h, self)

    # -- evaluation ----------------------------------------------------------
    def _type(self, level, value_type):
        if value_type is None:
            value_type = self.parameters[max(0, min(level, len(self.parameters) - 1))].value_type
        return value_type

    def evaluate_until(self, hierarchy_level: int, prefixes: Sequence[int],
                       ctx: EvaluationContext, value_type: ValueType = None,
                       raw: bool = False, out=None):
        """EvaluateUntil<T> (h:319-322).  Returns decoded values, or the
        host-layout numpy array with raw=True.  With `out` a torch GPU uint8
        tensor, the host-layout outputs stay in HBM (written into `out`,
        dpf_amd_evaluate_until_device) and `out` is returned."""
        vt = self._type(hierarchy_level, value_type)
        tp = vt.to_proto()
        pw = u128_words(_seq(prefixes)) if len(prefixes) else np.zeros(2, np.uint64)
        n = ctypes.c_int64()
        L = _lib.lib()
        pp = pw.ctypes.data_as(ctypes.c_void_p)
        # size only; the evaluation call below validates the prefixes
        check(L.dpf_amd_evaluate_until(self._h, hierarchy_level, pp, len(prefixes), tp, len(tp),
                                       ctx._h, None, -1, ctypes.byref(n)))
        if out is not None:
            check(L.dpf_amd_evaluate_until_device(
                self._h, hierarchy_level, pp, len(prefixes), tp, len(tp), ctx._h,
                ctypes.c_void_p(out.data_ptr()), out.numel() * out.element_size(),
                ctypes.byref(n), _lib.stream_ptr()))
            return out
        host = np.zeros(max(n.value, 1), dtype=vt.numpy_dtype())
        check(L.dpf_amd_evaluate_until(self._h, hierarchy_level, pp, len(prefixes), tp, len(tp),
                                       ctx._h, host.ctypes.data_as(ctypes.c_void_p),
                                       host.nbytes, ctypes.byref(n)))
        host = host[:n.value]
        return host if raw else vt.decode(host)

    def evaluate_next(self, prefixes: Sequence[int], ctx: EvaluationContext,
                      value_type: ValueType = None, raw: bool = False, out=None):
        """EvaluateNext<T> (h:324-333)."""
        if not len(prefixes):
            return self.evaluate_until(0, prefixes, ctx, value_type, raw, out)
        return self.evaluate_until(ctx.previous_hierarchy_level + 1, prefixes, ctx,
                                   value_type, raw, out)

    def expand_leaves_on_devices(self, key: DpfKey, slices) -> None:
        """One key's last-level leaves over devices
        (DistributedPointFunction::ExpandLeavesOnDevices): `slices` =
        [(device, leaf_begin, leaf_end, out)] with `out` a device tensor (or
        pointer) on that device holding (leaf_end - leaf_begin) elements in
        the host layout; returns when every device is done."""
        n = len(slices)
        data = bytes(key)
        devs = (ctypes.c_int * max(n, 1))(*[s[0] for s in slices])
        lo = (ctypes.c_int64 * max(n, 1))(*[s[1] for s in slices])
        hi = (ctypes.c_int64 * max(n, 1))(*[s[2] for s in slices])
        outs = (ctypes.c_void_p * max(n, 1))(
            *[s[3].data_ptr() if hasattr(s[3], "data_ptr") else s[3] for s in slices])
        check(_lib.lib().dpf_amd_expand_leaves_on_devices(self._h, data, len(data), n, devs,
                                                          lo, hi, outs))

    def evaluate_at(self, key: DpfKey, hierarchy_level: int, points: Sequence[int],
                    value_type: ValueType = None, raw: bool = False):
        """EvaluateAt<T>(key, level, points) (h:349-354)."""
        vt = self._type(hierarchy_level, value_type)
        tp = vt.to_proto()
        data = bytes(key)
        pw = u128_words(_seq(points)) if len(points) else np.zeros(2, np.uint64)
        out = np.zeros(max(len(points), 1), dtype=vt.numpy_dtype())
        check(_lib.lib().dpf_amd_evaluate_at(self._h, data, len(data), hierarchy_level,
                                             pw.ctypes.data_as(ctypes.c_void_p), len(points),
                                             tp, len(tp), out.ctypes.data_as(ctypes.c_void_p)))
        out = out[:len(points)]
        return out if raw else vt.decode(out)

    def evaluate_at_ctx(self, hierarchy_level: int, points: Sequence[int],
                        ctx: EvaluationContext, value_type: ValueType = None,
                        raw: bool = False):
        """EvaluateAt<T>(hierarchy_level, points, ctx) (h:356-378): starts
        from ctx's partial evaluations (from the root if it holds none) and
        rewrites them at `hierarchy_level` (EvaluateAtImpl h:1000-1011)."""
        vt = self._type(hierarchy_level, value_type)
        tp = vt.to_proto()
        pw = u128_words(_seq(points)) if len(points) else np.zeros(2, np.uint64)
        out = np.zeros(max(len(points), 1), dtype=vt.numpy_dtype())
        check(_lib.lib().dpf_amd_evaluate_at_ctx(self._h, hierarchy_level,
                                                 pw.ctypes.data_as(ctypes.c_void_p), len(points),
                                                 tp, len(tp), ctx._h,
                                                 out.ctypes.data_as(ctypes.c_void_p)))
        out = out[:len(points)]
        return out if raw else vt.decode(out)

    def evaluate_and_apply(self, keys: Sequence[DpfKey], points: Sequence[int],
                           op: Callable[[list], bool], rightshift: int = 0,
                           value_type: ValueType = None):
        """EvaluateAndApply<T, Fn> (h:403-407): op(values) after each level."""
        vt = self._type(0, value_type)
        tp = vt.to_proto()
        # one serialization per key object: the library parses (and uploads)
        # a key buffer passed for several points once
        ser = {}
        datas = [ser[id(k)] if id(k) in ser else ser.setdefault(id(k), bytes(k)) for k in keys]
        arr = (ctypes.c_char_p * max(len(datas), 1))(*datas)
        lens = (ctypes.c_size_t * max(len(datas), 1))(*[len(d) for d in datas])
        if len(points) != len(keys):
            raise _lib.DpfAmdError(3, "`keys.size()` != `evaluation_points.size()`")
        pw = u128_words(_seq(points)) if len(points) else np.zeros(2, np.uint64)
        H = len(self.parameters)
        out = np.zeros(max(H * len(keys), 1), dtype=vt.numpy_dtype())
        n = len(keys)
        errors = []

        def on_level(user, h, values, num):
            # called by the library after level h is evaluated; 0 stops the
            # remaining levels (h:1190-1196)
            try:
                return 1 if op(vt.decode(out[h * n:(h + 1) * n])) else 0
            except Exception as e:  # pragma: no cover - surfaced below
                errors.append(e)
                return 0
        cb = _lib.APPLY_FN(on_level)
        check(_lib.lib().dpf_amd_evaluate_and_apply(
            self._h, arr, lens, len(keys), pw.ctypes.data_as(ctypes.c_void_p), rightshift,
            tp, len(tp), out.ctypes.data_as(ctypes.c_void_p), cb, None))
        if errors:
            raise errors[0]
