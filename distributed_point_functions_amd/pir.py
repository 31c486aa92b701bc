"""Dense DPF-PIR server — Python mirror of the reference's pir/ API
(DenseDpfPirDatabase, DenseDpfPirServer::{CreatePlain, CreateLeader,
CreateHelper}, DpfPirServer::HandleRequest) over the C ABI.

The database lives in HBM; HandleRequest runs the selection-DPF expansion
and the XOR scan on the GPU. Requests / responses are PirRequest / PirResponse
protos in wire format (pir/private_information_retrieval.proto:62-151).
"""
from __future__ import annotations

import ctypes
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib, wire
from ._lib import check, take_buffer
from .value_types import u128_words

BITS_PER_BLOCK = 128


# ------------------------------------------------------------------ protos
def pir_config(num_elements: int) -> bytes:
    """PirConfig{dense_dpf_pir_config{num_elements}} (proto:28-33, 81-84)."""
    return wire.field_message(1, wire.field_varint(1, num_elements))


def plain_request(keys: Sequence[bytes]) -> bytes:
    """DpfPirRequest.PlainRequest (proto:105-108)."""
    return b"".join(wire.field_message(1, bytes(k)) for k in keys)


def pir_request_plain(keys: Sequence[bytes]) -> bytes:
    return wire.field_message(1, wire.field_message(1, plain_request(keys)))


def helper_request(keys: Sequence[bytes], one_time_pad_seed: bytes) -> bytes:
    """DpfPirRequest.HelperRequest (proto:123-126)."""
    return wire.field_message(1, plain_request(keys)) + wire.field_bytes(2, one_time_pad_seed)


def pir_request_leader(keys: Sequence[bytes], encrypted_helper_request: bytes) -> bytes:
    leader = (wire.field_message(1, plain_request(keys)) +
              wire.field_message(2, wire.field_bytes(1, encrypted_helper_request)))
    return wire.field_message(1, wire.field_message(2, leader))


def pir_request_encrypted_helper(encrypted_helper_request: bytes) -> bytes:
    return wire.field_message(1, wire.field_message(3, wire.field_bytes(1,
                                                                        encrypted_helper_request)))


def parse_response(data: bytes) -> List[bytes]:
    """PirResponse -> masked_response list (proto:70-74, 149-151)."""
    d = wire.decode(data)
    if 1 not in d:
        return []
    return [bytes(x) for x in wire.decode(d[1][-1]).get(1, [])]


# ---------------------------------------------------------------- database
class DenseDpfPirDatabase:
    """DenseDpfPirDatabase::Builder + the built, HBM-resident database
    (pir/dense_dpf_pir_database.h:41-95)."""

    def __init__(self, devices: Optional[Sequence[int]] = None):
        """`devices`: shard the records over these devices (128-record-aligned
        row ranges, one per entry; entries may repeat), see
        dpf_amd_pir_db_set_devices. None: one shard on the current device."""
        h = ctypes.c_void_p()
        check(_lib.lib().dpf_amd_pir_db_create(ctypes.byref(h)))
        self._h = h
        self._owned = True
        if devices:
            arr = (ctypes.c_int * len(devices))(*devices)
            check(_lib.lib().dpf_amd_pir_db_set_devices(self._h, arr, len(devices)))

    def __del__(self):
        try:
            if self._owned and self._h:
                _lib.lib().dpf_amd_pir_db_destroy(self._h)
        except Exception:
            pass

    def insert(self, record: bytes) -> "DenseDpfPirDatabase":
        check(_lib.lib().dpf_amd_pir_db_insert(self._h, bytes(record), len(record)))
        return self

    def insert_fixed(self, records: np.ndarray) -> "DenseDpfPirDatabase":
        """Bulk insert of an (n, record_size) uint8 array."""
        a = np.ascontiguousarray(records, dtype=np.uint8)
        check(_lib.lib().dpf_amd_pir_db_insert_fixed(self._h, a.ctypes.data_as(ctypes.c_void_p),
                                                     a.shape[0], a.shape[1]))
        return self

    def insert_packed(self, data, sizes) -> "DenseDpfPirDatabase":
        """Bulk insert of records of any sizes: `data` holds them back to
        back (bytes or a uint8 array), record i is sizes[i] bytes."""
        a = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) \
            else np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        sz = np.ascontiguousarray(sizes, dtype=np.int64)
        if int(sz.sum()) != a.size:
            raise ValueError("sizes do not add up to the data length")
        check(_lib.lib().dpf_amd_pir_db_insert_packed(
            self._h, a.ctypes.data_as(ctypes.c_void_p), sz.ctypes.data_as(ctypes.c_void_p),
            len(sz)))
        return self

    def insert_fixed_device(self, records, num_records: int, record_size: int) -> "DenseDpfPirDatabase":
        """Bulk insert of records already in device memory (a CUDA uint8
        tensor of num_records * record_size bytes); copied device to device
        at build time."""
        check(_lib.lib().dpf_amd_pir_db_insert_fixed_device(
            self._h, records.data_ptr(), records.device.index or 0, num_records, record_size))
        self._device_src = records  # keep alive until build
        return self

    def build(self) -> "DenseDpfPirDatabase":
        check(_lib.lib().dpf_amd_pir_db_build(self._h))
        return self

    @property
    def size(self) -> int:
        return _lib.lib().dpf_amd_pir_db_size(self._h)

    @property
    def max_value_size(self) -> int:
        return _lib.lib().dpf_amd_pir_db_max_value_size(self._h)

    def shards(self) -> List[Tuple[int, int, int]]:
        """[(device, row_begin, row_end)] of the built database."""
        out = []
        for i in range(_lib.lib().dpf_amd_pir_db_num_shards(self._h)):
            d, r0, r1 = ctypes.c_int(), ctypes.c_int64(), ctypes.c_int64()
            check(_lib.lib().dpf_amd_pir_db_shard(self._h, i, ctypes.byref(d), ctypes.byref(r0),
                                                  ctypes.byref(r1), None))
            out.append((d.value, r0.value, r1.value))
        return out

    @property
    def record_stride(self) -> int:
        """Device row stride in bytes of the built database (0 before build)."""
        stride = ctypes.c_int64(0)
        _lib.lib().dpf_amd_pir_db_device_records(self._h, ctypes.byref(stride))
        return stride.value

    def inner_product_with(self, selections: Sequence[Sequence[int]]) -> List[bytes]:
        """InnerProductWith (pir/pir_database_interface.h:65-66)."""
        if isinstance(selections, np.ndarray):
            # (q, blocks, 2) uint64 {lo, hi} words: no per-block Python ints
            if selections.ndim != 3 or selections.shape[2] != 2:
                raise ValueError("selections array must be (queries, blocks, 2) uint64")
            q, nb = selections.shape[0], selections.shape[1]
            if q == 0:
                return []
            if nb * BITS_PER_BLOCK < self.size:
                raise _lib.DpfAmdError(3, "`selections[0]` contains insufficient number of "
                                          "bits: %d, expected: %d"
                                       % (nb * BITS_PER_BLOCK, self.size))
            sel = np.ascontiguousarray(selections, dtype=np.uint64)
            return self._inner_product_words(sel, nb, q)
        q = len(selections)
        if q == 0:
            return []
        nb = len(selections[0])
        # pir_internal::InnerProduct's checks (inner_product_hwy.cc:306-323),
        # before the flat buffer of q * nb blocks crosses the C ABI
        for i, s_i in enumerate(selections):
            if len(s_i) * BITS_PER_BLOCK < self.size:
                raise _lib.DpfAmdError(3, "`selections[%d]` contains insufficient number of "
                                          "bits: %d, expected: %d"
                                       % (i, len(s_i) * BITS_PER_BLOCK, self.size))
            if len(s_i) != nb:
                raise _lib.DpfAmdError(3, "`selections[%d].size()` does not match "
                                          "`selections[0].size()`: actual%d, expected %d"
                                       % (i, len(s_i), nb))
        sel = u128_words([b for s in selections for b in s])
        return self._inner_product_words(sel, nb, q)

    def _inner_product_words(self, sel: np.ndarray, nb: int, q: int) -> List[bytes]:
        out = np.zeros(max(1, q * self.max_value_size), dtype=np.uint8)
        check(_lib.lib().dpf_amd_pir_db_inner_product(
            self._h, sel.ctypes.data_as(ctypes.c_void_p), nb, q,
            out.ctypes.data_as(ctypes.c_void_p)))
        m = self.max_value_size
        return [bytes(out[i * m:(i + 1) * m]) for i in range(q)]

    def _release(self):
        """The server takes ownership of the database handle."""
        self._owned = False
        return self._h


# ------------------------------------------------------------------ server
_FORWARD = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t,
                            ctypes.c_void_p, ctypes.c_void_p)
_DECRYPT = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t,
                            ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t, ctypes.c_void_p,
                            ctypes.c_void_p)


class PirCall:
    """The call handle a forward/decrypt callback talks back through."""

    def __init__(self, ptr):
        self._p = ptr

    def while_waiting(self):
        check(_lib.lib().dpf_amd_pir_call_while_waiting(self._p))

    def set_response(self, data: bytes):
        check(_lib.lib().dpf_amd_pir_call_set_response(self._p, bytes(data), len(data)))


class DenseDpfPirServer:
    """DenseDpfPirServer (pir/dense_dpf_pir_server.h:35-104)."""

    ENCRYPTION_CONTEXT_INFO = b"DenseDpfPirServer"

    def __init__(self, handle, keepalive=None):
        self._h = handle
        self._keepalive = keepalive

    def __del__(self):
        try:
            if self._h:
                _lib.lib().dpf_amd_pir_server_destroy(self._h)
        except Exception:
            pass

    @classmethod
    def create_plain(cls, num_elements: int, database: DenseDpfPirDatabase):
        cfg = pir_config(num_elements)
        h = ctypes.c_void_p()
        check(_lib.lib().dpf_amd_pir_server_create_plain(cfg, len(cfg), database._release(),
                                                         ctypes.byref(h)))
        return cls(h)

    @classmethod
    def create_leader(cls, num_elements: int, database: DenseDpfPirDatabase,
                      sender: Callable[[bytes, Callable[[], None]], bytes]):
        """sender(helper_request_bytes, while_waiting) -> helper PirResponse
        bytes (ForwardHelperRequestFn, pir/dpf_pir_server.h:92-94)."""
        def forward(req, n, call, user):
            c = PirCall(call)
            try:
                resp = sender(ctypes.string_at(req, n), c.while_waiting)
                c.set_response(resp)
                return 0
            except _lib.DpfAmdError as e:
                return e.code
            except Exception:
                return 13
        cb = _FORWARD(forward)
        cfg = pir_config(num_elements)
        h = ctypes.c_void_p()
        check(_lib.lib().dpf_amd_pir_server_create_leader(
            cfg, len(cfg), database._release(), cb, None, ctypes.byref(h)))
        return cls(h, keepalive=cb)

    @classmethod
    def create_helper(cls, num_elements: int, database: DenseDpfPirDatabase,
                      decrypter: Callable[[bytes, bytes], bytes]):
        """decrypter(ciphertext, context_info) -> serialized HelperRequest
        (DecryptHelperRequestFn, pir/dpf_pir_server.h:103-105)."""
        def decrypt(ct, n, info, ninfo, call, user):
            c = PirCall(call)
            try:
                c.set_response(decrypter(ctypes.string_at(ct, n), ctypes.string_at(info, ninfo)))
                return 0
            except _lib.DpfAmdError as e:
                return e.code
            except Exception:
                return 13
        cb = _DECRYPT(decrypt)
        cfg = pir_config(num_elements)
        h = ctypes.c_void_p()
        check(_lib.lib().dpf_amd_pir_server_create_helper(
            cfg, len(cfg), database._release(), cb, None, ctypes.byref(h)))
        return cls(h, keepalive=cb)

    def handle_request(self, request: bytes) -> bytes:
        """DpfPirServer::HandleRequest (pir/dpf_pir_server.h:123-124)."""
        buf = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        check(_lib.lib().dpf_amd_pir_server_handle_request(self._h, bytes(request), len(request),
                                                           ctypes.byref(buf), ctypes.byref(n)))
        return take_buffer(buf, n)


def client_keys(dpf, num_elements: int, indices: Sequence[int],
                seeds: Optional[Sequence[Sequence[int]]] = None):
    """Key pairs a DenseDpfPirClient would send for `indices`
    (pir/dense_dpf_pir_client.cc:77-103): alpha = i / 128,
    beta = XorWrapper<uint128>(1 << (i % 128)); `dpf` has log_domain_size =
    ceil(log2(num_elements)) and value type XorWrapper<uint128>."""
    out = []
    for j, i in enumerate(indices):
        if not 0 <= i < num_elements:
            raise _lib.DpfAmdError(3, "All `query_indices` out of bounds")
        out.append(dpf.generate_keys(i // BITS_PER_BLOCK, 1 << (i % BITS_PER_BLOCK),
                                     seeds=None if seeds is None else seeds[j]))
    return out
