"""google.protobuf message classes for the reference's wire schema, built
from descriptors in code (field names, numbers and types of
dpf/distributed_point_function.proto:25-171,
dcf/distributed_comparison_function.proto:25-32,
pir/hashing/hash_family_config.proto:22-32 and
pir/private_information_retrieval.proto:28-151) - no .proto file or protoc
needed.  Test infrastructure: tests/golden/wire/make_wire.py and
tests/test_wire_cpu.py / tests/test_wire_gpu.py use these classes as the
independent protobuf runtime our hand-written codecs (csrc/wire.cc,
distributed_point_functions_amd/wire.py) must agree with byte for byte.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PKG = "distributed_point_functions"
F = descriptor_pb2.FieldDescriptorProto

# (name, number, type, label, type_name or None, oneof index or None)
_OPT, _REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED
_I32, _I64, _U64, _BOOL, _DBL, _BYTES, _MSG, _ENUM = (
    F.TYPE_INT32, F.TYPE_INT64, F.TYPE_UINT64, F.TYPE_BOOL, F.TYPE_DOUBLE, F.TYPE_BYTES,
    F.TYPE_MESSAGE, F.TYPE_ENUM)


def _msg(name, fields, oneofs=(), nested=(), enums=()):
    m = descriptor_pb2.DescriptorProto(name=name)
    for o in oneofs:
        m.oneof_decl.add(name=o)
    for fname, num, typ, label, tname, oneof in fields:
        f = m.field.add(name=fname, number=num, type=typ, label=label)
        if tname:
            f.type_name = tname
        if oneof is not None:
            f.oneof_index = oneof
    m.nested_type.extend(nested)
    for ename, values in enums:
        e = m.enum_type.add(name=ename)
        for vname, vnum in values:
            e.value.add(name=vname, number=vnum)
    return m


def _t(name):
    return "." + PKG + "." + name


def _file():
    fd = descriptor_pb2.FileDescriptorProto(name="dpf_amd_wire_schema.proto", package=PKG,
                                            syntax="proto3")
    vt_int = _msg("Integer", [("bitsize", 1, _I32, _OPT, None, None)])
    vt_tuple = _msg("Tuple", [("elements", 1, _MSG, _REP, _t("ValueType"), None)])
    vt_mod = _msg("IntModN", [("base_integer", 1, _MSG, _OPT, _t("ValueType.Integer"), None),
                              ("modulus", 2, _MSG, _OPT, _t("Value.Integer"), None)])
    fd.message_type.append(_msg("ValueType", [
        ("integer", 1, _MSG, _OPT, _t("ValueType.Integer"), 0),
        ("tuple", 2, _MSG, _OPT, _t("ValueType.Tuple"), 0),
        ("int_mod_n", 3, _MSG, _OPT, _t("ValueType.IntModN"), 0),
        ("xor_wrapper", 4, _MSG, _OPT, _t("ValueType.Integer"), 0)],
        oneofs=["type"], nested=[vt_int, vt_tuple, vt_mod]))
    v_int = _msg("Integer", [("value_uint64", 1, _U64, _OPT, None, 0),
                             ("value_uint128", 2, _MSG, _OPT, _t("Block"), 0)], oneofs=["value"])
    v_tuple = _msg("Tuple", [("elements", 1, _MSG, _REP, _t("Value"), None)])
    fd.message_type.append(_msg("Value", [
        ("integer", 1, _MSG, _OPT, _t("Value.Integer"), 0),
        ("tuple", 2, _MSG, _OPT, _t("Value.Tuple"), 0),
        ("int_mod_n", 3, _MSG, _OPT, _t("Value.Integer"), 0),
        ("xor_wrapper", 4, _MSG, _OPT, _t("Value.Integer"), 0)],
        oneofs=["value"], nested=[v_int, v_tuple]))
    fd.message_type.append(_msg("DpfParameters", [
        ("log_domain_size", 1, _I32, _OPT, None, None),
        ("value_type", 3, _MSG, _OPT, _t("ValueType"), None),
        ("security_parameter", 4, _DBL, _OPT, None, None)]))
    fd.message_type.append(_msg("Block", [("high", 1, _U64, _OPT, None, None),
                                          ("low", 2, _U64, _OPT, None, None)]))
    fd.message_type.append(_msg("CorrectionWord", [
        ("seed", 1, _MSG, _OPT, _t("Block"), None),
        ("control_left", 2, _BOOL, _OPT, None, None),
        ("control_right", 3, _BOOL, _OPT, None, None),
        ("value_correction", 5, _MSG, _REP, _t("Value"), None)]))
    fd.message_type.append(_msg("DpfKey", [
        ("seed", 1, _MSG, _OPT, _t("Block"), None),
        ("correction_words", 2, _MSG, _REP, _t("CorrectionWord"), None),
        ("party", 3, _I32, _OPT, None, None),
        ("last_level_value_correction", 5, _MSG, _REP, _t("Value"), None)]))
    fd.message_type.append(_msg("PartialEvaluation", [
        ("prefix", 1, _MSG, _OPT, _t("Block"), None),
        ("seed", 2, _MSG, _OPT, _t("Block"), None),
        ("control_bit", 3, _BOOL, _OPT, None, None)]))
    fd.message_type.append(_msg("EvaluationContext", [
        ("parameters", 1, _MSG, _REP, _t("DpfParameters"), None),
        ("key", 2, _MSG, _OPT, _t("DpfKey"), None),
        ("previous_hierarchy_level", 3, _I32, _OPT, None, None),
        ("partial_evaluations", 4, _MSG, _REP, _t("PartialEvaluation"), None),
        ("partial_evaluations_level", 5, _I32, _OPT, None, None)]))
    # dcf/distributed_comparison_function.proto
    fd.message_type.append(_msg("DcfParameters", [
        ("parameters", 1, _MSG, _OPT, _t("DpfParameters"), None)]))
    fd.message_type.append(_msg("DcfKey", [("key", 1, _MSG, _OPT, _t("DpfKey"), None)]))
    # pir/hashing/hash_family_config.proto
    fd.message_type.append(_msg("HashFamilyConfig", [
        ("hash_family", 1, _ENUM, _OPT, _t("HashFamilyConfig.HashFamily"), None),
        ("seed", 2, _BYTES, _OPT, None, None)],
        enums=[("HashFamily", [("HASH_FAMILY_UNSPECIFIED", 0), ("HASH_FAMILY_SHA256", 1)])]))
    # pir/private_information_retrieval.proto
    fd.message_type.append(_msg("DenseDpfPirConfig", [("num_elements", 1, _I64, _OPT, None, None)]))
    fd.message_type.append(_msg("CuckooHashingSparseDpfPirConfig", [
        ("hash_family", 1, _ENUM, _OPT, _t("HashFamilyConfig.HashFamily"), None),
        ("num_elements", 2, _I64, _OPT, None, None)]))
    fd.message_type.append(_msg("CuckooHashingParams", [
        ("hash_family_config", 1, _MSG, _OPT, _t("HashFamilyConfig"), None),
        ("num_hash_functions", 2, _I32, _OPT, None, None),
        ("num_buckets", 3, _I64, _OPT, None, None)]))
    fd.message_type.append(_msg("PirConfig", [
        ("dense_dpf_pir_config", 1, _MSG, _OPT, _t("DenseDpfPirConfig"), 0),
        ("cuckoo_hashing_sparse_dpf_pir_config", 2, _MSG, _OPT,
         _t("CuckooHashingSparseDpfPirConfig"), 0)], oneofs=["wrapped_pir_config"]))
    plain = _msg("PlainRequest", [("dpf_key", 1, _MSG, _REP, _t("DpfKey"), None)])
    leader = _msg("LeaderRequest", [
        ("plain_request", 1, _MSG, _OPT, _t("DpfPirRequest.PlainRequest"), None),
        ("encrypted_helper_request", 2, _MSG, _OPT, _t("DpfPirRequest.EncryptedHelperRequest"),
         None)])
    enc = _msg("EncryptedHelperRequest", [("encrypted_request", 1, _BYTES, _OPT, None, None)])
    helper = _msg("HelperRequest", [
        ("plain_request", 1, _MSG, _OPT, _t("DpfPirRequest.PlainRequest"), None),
        ("one_time_pad_seed", 2, _BYTES, _OPT, None, None)])
    fd.message_type.append(_msg("DpfPirRequest", [
        ("plain_request", 1, _MSG, _OPT, _t("DpfPirRequest.PlainRequest"), 0),
        ("leader_request", 2, _MSG, _OPT, _t("DpfPirRequest.LeaderRequest"), 0),
        ("encrypted_helper_request", 3, _MSG, _OPT, _t("DpfPirRequest.EncryptedHelperRequest"),
         0)], oneofs=["wrapped_request"], nested=[plain, leader, enc, helper]))
    fd.message_type.append(_msg("PirRequest", [
        ("dpf_pir_request", 1, _MSG, _OPT, _t("DpfPirRequest"), 0)],
        oneofs=["wrapped_pir_request"]))
    fd.message_type.append(_msg("DpfPirResponse", [
        ("masked_response", 1, _BYTES, _REP, None, None)]))
    fd.message_type.append(_msg("PirResponse", [
        ("dpf_pir_response", 1, _MSG, _OPT, _t("DpfPirResponse"), 0)],
        oneofs=["wrapped_pir_response"]))
    fd.message_type.append(_msg("DenseDpfPirRequestClientState", [
        ("one_time_pad_seed", 1, _BYTES, _OPT, None, None)]))
    return fd


_POOL = descriptor_pool.DescriptorPool()
_POOL.Add(_file())


def cls(name: str):
    """Message class for a (possibly nested, dotted) message name."""
    return message_factory.GetMessageClass(_POOL.FindMessageTypeByName(PKG + "." + name))


def canonical(name: str, data: bytes) -> bytes:
    """Parse with the protobuf runtime and serialize back (deterministic)."""
    m = cls(name)()
    m.ParseFromString(data)
    return m.SerializeToString(deterministic=True)


# ------------------------------------------------------- messages from values
def value_integer(msg, v: int):
    """Uint128ToValueInteger (dpf/internal/value_type_helpers.cc:145-155)."""
    if v >> 64 == 0:
        msg.value_uint64 = v
    else:
        msg.value_uint128.high = v >> 64
        msg.value_uint128.low = v & ((1 << 64) - 1)


def value_type(msg, spec):
    """Fill a ValueType message from an oracle spec tuple."""
    kind = spec[0]
    if kind == "int":
        msg.integer.bitsize = spec[1]
    elif kind == "xor":
        msg.xor_wrapper.bitsize = spec[1]
    elif kind == "intmodn":
        msg.int_mod_n.base_integer.bitsize = spec[1]
        value_integer(msg.int_mod_n.modulus, spec[2])
    else:
        msg.tuple.SetInParent()
        for e in spec[1]:
            value_type(msg.tuple.elements.add(), e)


def value(msg, spec, scalars):
    """Fill a Value message of `spec` from flattened scalars (consumed)."""
    kind = spec[0]
    if kind == "int":
        value_integer(msg.integer, scalars.pop(0))
    elif kind == "xor":
        value_integer(msg.xor_wrapper, scalars.pop(0))
    elif kind == "intmodn":
        value_integer(msg.int_mod_n, scalars.pop(0))
    else:
        msg.tuple.SetInParent()
        for e in spec[1]:
            value(msg.tuple.elements.add(), e, scalars)
