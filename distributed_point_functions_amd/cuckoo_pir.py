"""Cuckoo-hashed sparse (keyword) DPF-PIR — Python mirror of the reference's
pir/cuckoo_hashed_dpf_pir_database.h, pir/cuckoo_hashing_sparse_dpf_pir_server.h
and pir/cuckoo_hashing_sparse_dpf_pir_client.h over the C ABI.

Keys are cuckoo-placed on the host (SHA-256 hash family, 3 hash functions,
1.5 buckets per element); the key table and the value table live in HBM and
one request costs one device DPF expansion per key plus two XOR scans.
"""
from __future__ import annotations

import ctypes
from typing import Callable, List, Optional, Sequence, Tuple

from . import _lib, wire
from ._lib import check, take_buffer
from .pir import (_DECRYPT, _FORWARD, PirCall, client_keys, parse_response,
                  pir_request_plain)

HASH_FAMILY_UNSPECIFIED = 0
HASH_FAMILY_SHA256 = 1
NUM_HASH_FUNCTIONS = 3          # cuckoo_hashing_sparse_dpf_pir_server.cc:36
BUCKETS_PER_ELEMENT = 1.5       # cuckoo_hashing_sparse_dpf_pir_server.cc:37


# ------------------------------------------------------------------ protos
def hash_family_config(hash_family: int, seed: bytes) -> bytes:
    """HashFamilyConfig (pir/hashing/hash_family_config.proto:22-35)."""
    return ((wire.field_varint(1, hash_family) if hash_family else b"") +
            (wire.field_bytes(2, seed) if seed else b""))


def cuckoo_pir_config(num_elements: int, hash_family: int = HASH_FAMILY_SHA256) -> bytes:
    """PirConfig{cuckoo_hashing_sparse_dpf_pir_config{hash_family, num_elements}}."""
    inner = ((wire.field_varint(1, hash_family) if hash_family else b"") +
             (wire.field_varint(2, num_elements) if num_elements else b""))
    return wire.field_message(2, inner)


def cuckoo_hashing_params(seed: bytes, num_buckets: int,
                          num_hash_functions: int = NUM_HASH_FUNCTIONS,
                          hash_family: int = HASH_FAMILY_SHA256) -> bytes:
    """CuckooHashingParams (private_information_retrieval.proto)."""
    return (wire.field_message(1, hash_family_config(hash_family, seed)) +
            (wire.field_varint(2, num_hash_functions) if num_hash_functions else b"") +
            (wire.field_varint(3, num_buckets) if num_buckets else b""))


def parse_cuckoo_hashing_params(data: bytes) -> dict:
    d = wire.decode(data)
    hfc = wire.decode(d[1][-1]) if 1 in d else {}
    return {"hash_family": hfc.get(1, [0])[-1], "seed": bytes(hfc.get(2, [b""])[-1]),
            "num_hash_functions": d.get(2, [0])[-1], "num_buckets": d.get(3, [0])[-1]}


def generate_params(num_elements: int, hash_family: int = HASH_FAMILY_SHA256) -> bytes:
    """CuckooHashingSparseDpfPirServer::GenerateParams (.cc:46-65)."""
    cfg = cuckoo_pir_config(num_elements, hash_family)
    buf = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    check(_lib.lib().dpf_amd_cuckoo_generate_params(cfg, len(cfg), ctypes.byref(buf),
                                                    ctypes.byref(n)))
    return take_buffer(buf, n)


# ----------------------------------------------------------------- hashing
def sha256_hash(seed: bytes, data: bytes, upper_bound: int) -> int:
    """SHA256HashFunction(seed)(data, upper_bound) (sha256_hash_family.cc:59-86)."""
    out = ctypes.c_int()
    check(_lib.lib().dpf_amd_sha256_hash(bytes(seed), len(seed), bytes(data), len(data),
                                         upper_bound, ctypes.byref(out)))
    return out.value


def hash_positions(params: bytes, data: bytes) -> List[int]:
    """The num_hash_functions buckets of `data` under `params`' hash family
    (CreateHashFunctions(CreateHashFamilyFromConfig(...)))."""
    p = parse_cuckoo_hashing_params(params)
    cfg = hash_family_config(p["hash_family"], p["seed"])
    k = p["num_hash_functions"]
    out = (ctypes.c_int * max(k, 1))()
    check(_lib.lib().dpf_amd_hash_family_evaluate(cfg, len(cfg), k, bytes(data), len(data),
                                                  p["num_buckets"], out))
    return list(out[:k])


# ---------------------------------------------------------------- database
class CuckooHashedDpfPirDatabase:
    """CuckooHashedDpfPirDatabase::Builder + built database (key and value
    tables in HBM)."""

    def __init__(self, params: bytes):
        self.params = bytes(params)
        self._h = ctypes.c_void_p()
        check(_lib.lib().dpf_amd_cuckoo_db_create(self.params, len(self.params),
                                                  ctypes.byref(self._h)))
        self._owned = True
        self._built = False

    def __del__(self):
        try:
            if self._owned and self._h:
                _lib.lib().dpf_amd_cuckoo_db_destroy(self._h)
        except Exception:
            pass

    def insert(self, key: bytes, value: bytes) -> "CuckooHashedDpfPirDatabase":
        check(_lib.lib().dpf_amd_cuckoo_db_insert(self._h, bytes(key), len(key), bytes(value),
                                                  len(value)))
        return self

    def place(self) -> List[Optional[bytes]]:
        """Host-only cuckoo placement: the key in each bucket (None = empty)."""
        nb = parse_cuckoo_hashing_params(self.params)["num_buckets"]
        lens = (ctypes.c_int64 * max(nb, 1))()
        check(_lib.lib().dpf_amd_cuckoo_db_place(self._h, lens, nb))
        total = sum(l for l in lens[:nb] if l > 0)
        keys = ctypes.create_string_buffer(max(total, 1))
        check(_lib.lib().dpf_amd_cuckoo_db_place_keys(self._h, keys, total))
        raw = keys.raw[:total]
        out, off = [], 0
        for l in lens[:nb]:
            if l < 0:
                out.append(None)
            else:
                out.append(raw[off:off + l])
                off += l
        return out

    def build(self) -> "CuckooHashedDpfPirDatabase":
        check(_lib.lib().dpf_amd_cuckoo_db_build(self._h))
        self._built = True
        return self

    def size(self) -> int:
        return _lib.lib().dpf_amd_cuckoo_db_size(self._h)

    def num_selection_bits(self) -> int:
        return _lib.lib().dpf_amd_cuckoo_db_num_selection_bits(self._h)

    def _release(self):
        self._owned = False
        return self._h


# ------------------------------------------------------------------ server
class CuckooHashingSparseDpfPirServer:
    """CuckooHashingSparseDpfPirServer (pir/cuckoo_hashing_sparse_dpf_pir_server.h:37-125)."""

    ENCRYPTION_CONTEXT_INFO = b"CuckooHashingSparseDpfPirServer"

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
    def create_plain(cls, params: bytes, database: CuckooHashedDpfPirDatabase):
        h = ctypes.c_void_p()
        check(_lib.lib().dpf_amd_cuckoo_server_create_plain(params, len(params),
                                                            database._release(),
                                                            ctypes.byref(h)))
        return cls(h)

    @classmethod
    def create_leader(cls, params: bytes, database: CuckooHashedDpfPirDatabase,
                      sender: Callable[[bytes, Callable[[], None]], bytes]):
        def forward(req, n, call, user):
            c = PirCall(call)
            try:
                c.set_response(sender(ctypes.string_at(req, n), c.while_waiting))
                return 0
            except _lib.DpfAmdError as e:
                return e.code
            except Exception:
                return 13
        cb = _FORWARD(forward)
        h = ctypes.c_void_p()
        check(_lib.lib().dpf_amd_cuckoo_server_create_leader(
            params, len(params), database._release(), cb, None, ctypes.byref(h)))
        return cls(h, keepalive=cb)

    @classmethod
    def create_helper(cls, params: bytes, database: CuckooHashedDpfPirDatabase,
                      decrypter: Callable[[bytes, bytes], bytes]):
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
        h = ctypes.c_void_p()
        check(_lib.lib().dpf_amd_cuckoo_server_create_helper(
            params, len(params), database._release(), cb, None, ctypes.byref(h)))
        return cls(h, keepalive=cb)

    def public_params(self) -> bytes:
        """PirServerPublicParams{cuckoo_hashing_sparse_dpf_pir_server_params}."""
        buf = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        check(_lib.lib().dpf_amd_pir_server_public_params(self._h, ctypes.byref(buf),
                                                          ctypes.byref(n)))
        return take_buffer(buf, n)

    def handle_request(self, request: bytes) -> bytes:
        buf = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        check(_lib.lib().dpf_amd_pir_server_handle_request(self._h, bytes(request), len(request),
                                                           ctypes.byref(buf), ctypes.byref(n)))
        return take_buffer(buf, n)


# ------------------------------------------------------------------ client
def _is_prefix_padded_with_zeros(data: bytes, prefix: bytes) -> bool:
    """cuckoo_hashing_sparse_dpf_pir_client.cc:41-51."""
    for i, c in enumerate(data):
        if i < len(prefix):
            if c != prefix[i]:
                return False
        elif c != 0:
            return False
    return True


class CuckooHashingSparseDpfPirClient:
    """Two-server plain-mode client (cuckoo_hashing_sparse_dpf_pir_client.cc:
    60-161 with the dense client's key generation, dense_dpf_pir_client.cc:
    77-103): each query string becomes num_hash_functions DPF key pairs, one
    per candidate bucket; a bucket whose recovered key equals the query
    (zero padded) yields the value."""

    def __init__(self, params: bytes, dpf):
        self.params = bytes(params)
        p = parse_cuckoo_hashing_params(self.params)
        if p["num_buckets"] <= 0:
            raise _lib.DpfAmdError(3, "`num_buckets` must be positive")
        if p["num_hash_functions"] <= 0:
            raise _lib.DpfAmdError(3, "`num_hash_functions` must be positive")
        self.num_buckets = p["num_buckets"]
        self.num_hash_functions = p["num_hash_functions"]
        self.dpf = dpf  # log_domain = ceil(log2(num_buckets)), XorWrapper<uint128>

    def create_requests(self, queries: Sequence[bytes]) -> Tuple[bytes, bytes]:
        """Plain PirRequests for server 0 and server 1."""
        indices = [h for q in queries for h in hash_positions(self.params, q)]
        pairs = client_keys(self.dpf, self.num_buckets, indices)
        return (pir_request_plain([k0 for k0, _ in pairs]),
                pir_request_plain([k1 for _, k1 in pairs]))

    def handle_responses(self, queries: Sequence[bytes], response0: bytes,
                         response1: bytes) -> List[Optional[bytes]]:
        r0, r1 = parse_response(response0), parse_response(response1)
        k = self.num_hash_functions
        if len(r0) != len(queries) * k * 2 or len(r1) != len(r0):
            raise _lib.DpfAmdError(3, "Number of responses must be equal to the number of "
                                      "queries times the number of hash functions times 2")
        raw = [bytes(a ^ b for a, b in zip(x, y)) for x, y in zip(r0, r1)]
        out: List[Optional[bytes]] = []
        for i, q in enumerate(queries):
            found = None
            for j in range(k):
                idx = 2 * (k * i + j)
                if found is None and _is_prefix_padded_with_zeros(raw[idx], q):
                    found = raw[idx + 1]
            out.append(found)
        return out
