// dpf.cc — DistributedPointFunction on MI355X.
//
// Host side (as in the reference): parameter / key / context validation
// (dpf/internal/proto_validator.cc), BitsNeeded and value algebra
// (dpf/internal/value_type_helpers.{h,cc}, dpf/int_mod_n.{h,cc}), key
// generation (dpf/distributed_point_function.cc:81-222, 642-710).
// Device side: every evaluation goes through the Tier-1 C ABI
// (dpf_amd_expand_and_correct / dpf_amd_evaluate_seeds /
// dpf_amd_evaluate_points / dpf_amd_gather_rows); there is no CPU path.
#include "dpf_amd/distributed_point_function.h"

#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <array>
#include <cmath>
#include <cstdio>
#include <mutex>
#include <set>
#include <sstream>
#include <unordered_map>

#include "host_aes.h"
#include "host_device.h"
#include "internal.h"

namespace distributed_point_functions {

using dpf_amd::HostAes;
using dpf_amd::u128;

namespace dpf_internal {

// ---------------------------------------------------------------------------
// Value::Integer <-> uint128 (value_type_helpers.cc:145-166)
// ---------------------------------------------------------------------------
Value::Integer Uint128ToValueInteger(uint128 v) {
  Value::Integer r;
  if (Uint128High64(v) == 0) {
    r.set_value_uint64(Uint128Low64(v));
  } else {
    r.mutable_value_uint128()->set_high(Uint128High64(v));
    r.mutable_value_uint128()->set_low(Uint128Low64(v));
  }
  return r;
}

StatusOr<uint128> ValueIntegerToUint128(const Value::Integer& in) {
  if (in.value_case() == Value::Integer::kValueUint128)
    return MakeUint128(in.value_uint128().high(), in.value_uint128().low());
  if (in.value_case() == Value::Integer::kValueUint64) return uint128{in.value_uint64()};
  return InvalidArgumentError("Unknown value case for the given integer Value");
}

namespace {

std::string U128ToString(uint128 v) {
  if (v == 0) return "0";
  std::string s;
  while (v) {
    s.push_back(static_cast<char>('0' + static_cast<int>(v % 10)));
    v /= 10;
  }
  std::reverse(s.begin(), s.end());
  return s;
}

// ---------------------------------------------------------------------------
// ValueType validation / equality / BitsNeeded
// ---------------------------------------------------------------------------
Status ValidateIntegerType(const ValueType::Integer& t) {
  int b = t.bitsize();
  if (b < 1) return InvalidArgumentError("`bitsize` must be positive");
  if (b > 128) return InvalidArgumentError("`bitsize` must be less than or equal to 128");
  if ((b & (b - 1)) != 0) return InvalidArgumentError("`bitsize` must be a power of 2");
  return OkStatus();
}

Status ValidateIntegerValue(const Value::Integer& v, const ValueType::Integer& t) {
  if (t.bitsize() < 128) {
    StatusOr<uint128> x = ValueIntegerToUint128(v);
    if (!x.ok()) return x.status();
    if (*x >= (uint128{1} << t.bitsize()))
      return InvalidArgumentError("Value (= " + U128ToString(*x) +
                                  ") too large for ValueType with bitsize = " +
                                  std::to_string(t.bitsize()));
  }
  return OkStatus();
}

Status ValidateValueType(const ValueType& vt) {  // proto_validator.cc:269-287
  switch (vt.type_case()) {
    case ValueType::kInteger:
      return ValidateIntegerType(vt.integer());
    case ValueType::kTuple:
      for (const ValueType& e : vt.tuple().elements()) DPF_RETURN_IF_ERROR(ValidateValueType(e));
      return OkStatus();
    case ValueType::kIntModN:
      DPF_RETURN_IF_ERROR(ValidateIntegerType(vt.int_mod_n().base_integer()));
      return ValidateIntegerValue(vt.int_mod_n().modulus(), vt.int_mod_n().base_integer());
    case ValueType::kXorWrapper:
      return ValidateIntegerType(vt.xor_wrapper());
    default:
      return InvalidArgumentError("ValidateValueType: Unsupported ValueType:\n" +
                                  vt.DebugString());
  }
}

}  // namespace

StatusOr<bool> ValueTypesAreEqual(const ValueType& lhs, const ValueType& rhs) {
  if (lhs.type_case() == ValueType::TYPE_NOT_SET || rhs.type_case() == ValueType::TYPE_NOT_SET)
    return InvalidArgumentError("Both arguments must be valid ValueTypes");
  if (lhs.type_case() == ValueType::kInteger && rhs.type_case() == ValueType::kInteger)
    return lhs.integer().bitsize() == rhs.integer().bitsize();
  if (lhs.type_case() == ValueType::kTuple && rhs.type_case() == ValueType::kTuple &&
      lhs.tuple().elements_size() == rhs.tuple().elements_size()) {
    bool result = true;
    for (int i = 0; i < lhs.tuple().elements_size(); ++i) {
      StatusOr<bool> e = ValueTypesAreEqual(lhs.tuple().elements(i), rhs.tuple().elements(i));
      if (!e.ok()) return e.status();
      result &= *e;
    }
    return result;
  }
  if (lhs.type_case() == ValueType::kIntModN && rhs.type_case() == ValueType::kIntModN) {
    StatusOr<uint128> a = ValueIntegerToUint128(lhs.int_mod_n().modulus());
    if (!a.ok()) return a.status();
    StatusOr<uint128> b = ValueIntegerToUint128(rhs.int_mod_n().modulus());
    if (!b.ok()) return b.status();
    return lhs.int_mod_n().base_integer().bitsize() == rhs.int_mod_n().base_integer().bitsize() &&
           *a == *b;
  }
  if (lhs.type_case() == ValueType::kXorWrapper && rhs.type_case() == ValueType::kXorWrapper)
    return lhs.xor_wrapper().bitsize() == rhs.xor_wrapper().bitsize();
  return false;
}

namespace {

// absl::uint128 -> double (absl/numeric/int128.h).
double ToDouble(uint128 v) {
  return static_cast<double>(Uint128Low64(v)) + std::ldexp(static_cast<double>(Uint128High64(v)), 64);
}

// IntModNBase::CheckParameters + GetNumBytesRequired (int_mod_n.cc:29-84).
StatusOr<int> IntModNBytesRequired(int num_samples, int base_bits, uint128 modulus,
                                   double security_parameter) {
  if (num_samples <= 0) return InvalidArgumentError("num_samples must be positive");
  if (base_bits <= 0) return InvalidArgumentError("base_integer_bitsize must be positive");
  if (base_bits > 128) return InvalidArgumentError("base_integer_bitsize must be at most 128");
  if (base_bits < 128 && (uint128{1} << base_bits) < modulus)
    return InvalidArgumentError("kModulus " + U128ToString(modulus) +
                                " out of range for base_integer_bitsize = " +
                                std::to_string(base_bits));
  const double sigma = 128 + 3 -
                       (std::log2(ToDouble(modulus)) + std::log2(static_cast<double>(num_samples)) +
                        std::log2(static_cast<double>(num_samples + 1)));
  if (security_parameter > sigma) {
    char buf[64];
    snprintf(buf, sizeof(buf), "%f", sigma);
    return InvalidArgumentError("For num_samples = " + std::to_string(num_samples) +
                                " and kModulus = " + U128ToString(modulus) +
                                " this approach can only provide " + buf +
                                " bits of statistical security. You can try calling this "
                                "function several times with smaller values of num_samples.");
  }
  return 16 + ((base_bits + 7) / 8) * (num_samples - 1);
}

}  // namespace

// BitsNeeded (value_type_helpers.cc:71-141), including the reference's
// iteration over elements(i) for i < num_other (lines 105-114).
StatusOr<int> BitsNeeded(const ValueType& vt, double security_parameter) {
  switch (vt.type_case()) {
    case ValueType::kInteger:
      return vt.integer().bitsize();
    case ValueType::kTuple: {
      int num_ints_mod_n = 0, num_other = 0;
      const ValueType* int_mod_n = nullptr;
      for (const ValueType& el : vt.tuple().elements()) {
        if (el.type_case() == ValueType::kIntModN) {
          if (!int_mod_n) {
            int_mod_n = &el;
          } else {
            StatusOr<bool> eq = ValueTypesAreEqual(el, *int_mod_n);
            if (!eq.ok()) return eq.status();
            if (!*eq)
              return UnimplementedError("All elements of type IntModN in a tuple must be the same");
          }
          ++num_ints_mod_n;
        } else {
          ++num_other;
        }
      }
      int bitsize_other = 0, bitsize_mod_n = 0;
      for (int i = 0; i < num_other; ++i) {
        double per = security_parameter + std::log2(static_cast<double>(num_other));
        StatusOr<int> b = BitsNeeded(vt.tuple().elements(i), per);
        if (!b.ok()) return b.status();
        bitsize_other += *b;
      }
      if (num_ints_mod_n > 0) {
        StatusOr<uint128> m = ValueIntegerToUint128(int_mod_n->int_mod_n().modulus());
        if (!m.ok()) return m.status();
        StatusOr<int> bytes = IntModNBytesRequired(
            num_ints_mod_n, int_mod_n->int_mod_n().base_integer().bitsize(), *m,
            security_parameter);
        if (!bytes.ok()) return bytes.status();
        bitsize_mod_n = *bytes * 8;
      }
      return bitsize_mod_n + bitsize_other;
    }
    case ValueType::kIntModN: {
      StatusOr<uint128> m = ValueIntegerToUint128(vt.int_mod_n().modulus());
      if (!m.ok()) return m.status();
      StatusOr<int> bytes = IntModNBytesRequired(1, vt.int_mod_n().base_integer().bitsize(), *m,
                                                 security_parameter);
      if (!bytes.ok()) return bytes.status();
      return 8 * *bytes;
    }
    case ValueType::kXorWrapper:
      return vt.xor_wrapper().bitsize();
    default:
      return InvalidArgumentError("BitsNeeded: Unsupported ValueType:\n" + vt.DebugString());
  }
}

namespace {

// ---------------------------------------------------------------------------
// Flattened value types
// ---------------------------------------------------------------------------
struct ScalarMeta {
  int kind;  // DPF_AMD_KIND_*
  int bits;
  uint128 modulus;
};

struct Node {  // layout computation
  int size = 0, align = 1;
};

void Flatten(const ValueType& vt, std::vector<ScalarMeta>* out) {
  switch (vt.type_case()) {
    case ValueType::kInteger:
      out->push_back({DPF_AMD_KIND_INTEGER, vt.integer().bitsize(), 0});
      break;
    case ValueType::kXorWrapper:
      out->push_back({DPF_AMD_KIND_XOR_WRAPPER, vt.xor_wrapper().bitsize(), 0});
      break;
    case ValueType::kIntModN: {
      StatusOr<uint128> m = ValueIntegerToUint128(vt.int_mod_n().modulus());
      out->push_back({DPF_AMD_KIND_INT_MOD_N, vt.int_mod_n().base_integer().bitsize(),
                      m.ok() ? *m : 0});
      break;
    }
    case ValueType::kTuple:
      for (const ValueType& e : vt.tuple().elements()) Flatten(e, out);
      break;
    default:
      break;
  }
}

// Host (libstdc++ / Itanium) layout: std::tuple members in reverse order,
// each at the next suitably aligned offset.  Appends scalar offsets
// (declaration order) relative to `base`.
Node Layout(const ValueType& vt, int base, std::vector<int>* offsets) {
  if (vt.type_case() == ValueType::kTuple) {
    const int n = vt.tuple().elements_size();
    std::vector<Node> nodes(n);
    std::vector<std::vector<int>> sub(n);
    for (int i = 0; i < n; ++i) nodes[i] = Layout(vt.tuple().elements(i), 0, &sub[i]);
    std::vector<int> elem_off(n);
    int end = 0, align = 1;
    for (int i = n - 1; i >= 0; --i) {
      int off = (end + nodes[i].align - 1) / nodes[i].align * nodes[i].align;
      elem_off[i] = off;
      end = off + nodes[i].size;
      align = std::max(align, nodes[i].align);
    }
    for (int i = 0; i < n; ++i)
      for (int o : sub[i]) offsets->push_back(base + elem_off[i] + o);
    Node r;
    r.align = align;
    r.size = std::max(1, (end + align - 1) / align * align);
    return r;
  }
  int bits = vt.type_case() == ValueType::kIntModN ? vt.int_mod_n().base_integer().bitsize()
             : vt.type_case() == ValueType::kXorWrapper ? vt.xor_wrapper().bitsize()
                                                         : vt.integer().bitsize();
  Node r;
  r.size = r.align = std::max(1, bits / 8);
  offsets->push_back(base);
  return r;
}

uint128 MaskBits(int bits) { return bits >= 128 ? ~uint128{0} : ((uint128{1} << bits) - 1); }

uint128 ScAdd(const ScalarMeta& s, uint128 a, uint128 b) {
  if (s.kind == DPF_AMD_KIND_INTEGER) return (a + b) & MaskBits(s.bits);
  if (s.kind == DPF_AMD_KIND_XOR_WRAPPER) return a ^ b;
  uint128 x = s.modulus - b;
  return a >= x ? a - x : s.modulus - x + a;
}
uint128 ScSub(const ScalarMeta& s, uint128 a, uint128 b) {
  if (s.kind == DPF_AMD_KIND_INTEGER) return (a - b) & MaskBits(s.bits);
  if (s.kind == DPF_AMD_KIND_XOR_WRAPPER) return a ^ b;
  return a >= b ? a - b : s.modulus - b + a;
}
uint128 ScNeg(const ScalarMeta& s, uint128 a) {
  if (s.kind == DPF_AMD_KIND_INTEGER) return (uint128{0} - a) & MaskBits(s.bits);
  if (s.kind == DPF_AMD_KIND_XOR_WRAPPER) return a;
  return a == 0 ? 0 : s.modulus - a;
}

uint128 LeBytes(const uint8_t* p, int n) {
  uint128 v = 0;
  for (int i = n - 1; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

}  // namespace

// Per hierarchy level metadata.
struct LevelMeta {
  std::vector<ScalarMeta> scalars;
  bool direct = true;
  int total_bits = 0;
  int epb = 1;
  int esz = 0;
  int bn = 1;
  int tree_level = 0;
  int log_domain = 0;
  dpf_amd_value_type desc{};  // conversion metadata + rule-based host layout

  // ConvertBytesToArrayOf<T> (vth:586-606) on the host (key generation).
  void Convert(const uint8_t* bytes, int len, std::vector<uint128>* out) const {
    const int ns = static_cast<int>(scalars.size());
    out->assign(static_cast<size_t>(epb) * ns, 0);
    if (direct) {
      for (int e = 0; e < epb; ++e) {
        int off = e * esz;
        for (int s = 0; s < ns; ++s) {
          int b = scalars[s].bits / 8;
          (*out)[e * ns + s] = off + b <= len ? LeBytes(bytes + off, b) : 0;
          off += b;
        }
      }
      return;
    }
    uint128 block = LeBytes(bytes, 16);
    int pos = 16;
    for (int s = 0; s < ns; ++s) {
      const ScalarMeta& m = scalars[s];
      const bool update = s + 1 < ns;
      const int b = m.bits / 8;
      if (m.kind == DPF_AMD_KIND_INT_MOD_N) {
        uint128 q = block / m.modulus, r = block % m.modulus;
        (*out)[s] = r;
        if (update) {
          block = b < 16 ? (q << (8 * b)) : 0;
          block |= pos + b <= len ? LeBytes(bytes + pos, b) : 0;
          pos += b;
        }
      } else {
        (*out)[s] = block & MaskBits(m.bits);
        if (update) {
          block = b < 16 ? (block & ~MaskBits(m.bits)) : 0;
          block |= pos + b <= len ? LeBytes(bytes + pos, b) : 0;
          pos += b;
        }
      }
    }
  }
};

class DpfState {
 public:
  std::vector<DpfParameters> parameters;
  int tree_levels_needed = 0;
  std::vector<int> hierarchy_to_tree;
  std::vector<int> tree_to_hierarchy;  // -1 if none
  std::vector<LevelMeta> levels;
  HostAes prg_left{MakeUint128(dpf_amd::kPrgKeyLeftHi, dpf_amd::kPrgKeyLeftLo)};
  HostAes prg_right{MakeUint128(dpf_amd::kPrgKeyRightHi, dpf_amd::kPrgKeyRightLo)};
  HostAes prg_value{MakeUint128(dpf_amd::kPrgKeyValueHi, dpf_amd::kPrgKeyValueLo)};
  // Value types with a value correction function (cc:567-582): keyed by the
  // deterministic serialization of the ValueType, as the reference's
  // value_correction_functions_ map.
  mutable std::mutex registry_mu;
  std::set<std::string> registered;
};

namespace {

Status ValidateValueOfType(const Value& value, const ValueType& type) {
  // proto_validator.cc:289-333
  switch (type.type_case()) {
    case ValueType::kInteger:
      if (value.value_case() != Value::kInteger)
        return InvalidArgumentError("Expected integer value");
      return ValidateIntegerValue(value.integer(), type.integer());
    case ValueType::kTuple: {
      if (value.value_case() != Value::kTuple) return InvalidArgumentError("Expected tuple value");
      if (value.tuple().elements_size() != type.tuple().elements_size())
        return InvalidArgumentError("Expected tuple value of size " +
                                    std::to_string(type.tuple().elements_size()) +
                                    " but got size " +
                                    std::to_string(value.tuple().elements_size()));
      for (int i = 0; i < type.tuple().elements_size(); ++i)
        DPF_RETURN_IF_ERROR(ValidateValueOfType(value.tuple().elements(i), type.tuple().elements(i)));
      return OkStatus();
    }
    case ValueType::kIntModN: {
      DPF_RETURN_IF_ERROR(ValidateIntegerValue(value.int_mod_n(), type.int_mod_n().base_integer()));
      StatusOr<uint128> v = ValueIntegerToUint128(value.int_mod_n());
      if (!v.ok()) return v.status();
      StatusOr<uint128> m = ValueIntegerToUint128(type.int_mod_n().modulus());
      if (!m.ok()) return m.status();
      if (*v >= *m)
        return InvalidArgumentError("Value (= " + U128ToString(*v) +
                                    ") is too large for modulus (= " + U128ToString(*m) + ")");
      return OkStatus();
    }
    case ValueType::kXorWrapper:
      if (value.value_case() != Value::kXorWrapper)
        return InvalidArgumentError("Expected XorWrapper value");
      return ValidateIntegerValue(value.xor_wrapper(), type.xor_wrapper());
    default:
      return InvalidArgumentError("ValidateValue: Unsupported ValueType:\n" + type.DebugString());
  }
}

// Flattens a (validated) Value of `type`.
Status FlattenValue(const Value& v, const ValueType& type, std::vector<uint128>* out) {
  if (type.type_case() == ValueType::kTuple) {
    if (v.value_case() != Value::kTuple)
      return InvalidArgumentError("The given Value is not a tuple");
    if (v.tuple().elements_size() != type.tuple().elements_size())
      return InvalidArgumentError("The tuple in the given Value has the wrong number of elements");
    for (int i = 0; i < type.tuple().elements_size(); ++i)
      DPF_RETURN_IF_ERROR(FlattenValue(v.tuple().elements(i), type.tuple().elements(i), out));
    return OkStatus();
  }
  const Value::Integer* in = nullptr;
  int bits = 0;
  switch (type.type_case()) {
    case ValueType::kInteger:
      if (v.value_case() != Value::kInteger)
        return InvalidArgumentError("The given Value is not an integer");
      in = &v.integer();
      bits = type.integer().bitsize();
      break;
    case ValueType::kIntModN: {
      if (v.value_case() != Value::kIntModN)
        return InvalidArgumentError("The given Value is not an IntModN");
      in = &v.int_mod_n();
      bits = type.int_mod_n().base_integer().bitsize();
      break;
    }
    case ValueType::kXorWrapper:
      in = &v.xor_wrapper();
      bits = type.xor_wrapper().bitsize();
      break;
    default:
      return InvalidArgumentError("unsupported value type");
  }
  StatusOr<uint128> x = ValueIntegerToUint128(*in);
  if (!x.ok()) return x.status();
  if (bits < 128 && *x > MaskBits(bits))
    return InvalidArgumentError("Value (= " + std::to_string(static_cast<uint64_t>(*x)) +
                                ") too large for the given type T (size " +
                                std::to_string(bits / 8) + ")");
  if (type.type_case() == ValueType::kIntModN) {
    StatusOr<uint128> m = ValueIntegerToUint128(type.int_mod_n().modulus());
    if (m.ok() && *x >= *m)
      return InvalidArgumentError("The given value (= " + U128ToString(*x) +
                                  ") is larger than kModulus (= " + U128ToString(*m) + ")");
  }
  out->push_back(*x);
  return OkStatus();
}

// Builds a Value of `type` from flattened scalars (ToValue<T>).
Value UnflattenValue(const ValueType& type, const uint128*& it) {
  Value v;
  switch (type.type_case()) {
    case ValueType::kTuple:
      for (const ValueType& e : type.tuple().elements())
        *v.mutable_tuple()->add_elements() = UnflattenValue(e, it);
      break;
    case ValueType::kIntModN:
      *v.mutable_int_mod_n() = Uint128ToValueInteger(*it++);
      break;
    case ValueType::kXorWrapper:
      *v.mutable_xor_wrapper() = Uint128ToValueInteger(*it++);
      break;
    default:
      *v.mutable_integer() = Uint128ToValueInteger(*it++);
      break;
  }
  return v;
}

bool AlmostEqual(double a, double b) { return std::abs(a - b) <= 0.0001; }

double DefaultSecurity(const DpfParameters& p) { return 40 + p.log_domain_size(); }

StatusOr<bool> ParametersAreEqual(const DpfParameters& lhs, const DpfParameters& rhs) {
  if (lhs.log_domain_size() != rhs.log_domain_size()) return false;
  if (!(AlmostEqual(lhs.security_parameter(), rhs.security_parameter()) ||
        (lhs.security_parameter() == 0 &&
         AlmostEqual(rhs.security_parameter(), DefaultSecurity(rhs))) ||
        (rhs.security_parameter() == 0 &&
         AlmostEqual(lhs.security_parameter(), DefaultSecurity(lhs)))))
    return false;
  return ValueTypesAreEqual(lhs.value_type(), rhs.value_type());
}

Status ValidateParameters(Span<const DpfParameters> parameters) {
  if (parameters.empty()) return InvalidArgumentError("`parameters` must not be empty");
  int previous = 0;
  for (size_t i = 0; i < parameters.size(); ++i) {
    int ld = parameters[i].log_domain_size();
    if (ld < 0) return InvalidArgumentError("`log_domain_size` must be non-negative");
    if (ld > 128) return InvalidArgumentError("`log_domain_size` must be <= 128");
    if (i > 0 && ld <= previous)
      return InvalidArgumentError(
          "`log_domain_size` fields must be in ascending order in `parameters`");
    previous = ld;
    if (!parameters[i].has_value_type()) return InvalidArgumentError("`value_type` is required");
    DPF_RETURN_IF_ERROR(ValidateValueType(parameters[i].value_type()));
    double sp = parameters[i].security_parameter();
    if (std::isnan(sp)) return InvalidArgumentError("`security_parameter` must not be NaN");
    if (sp < 0 || sp > 128) return InvalidArgumentError("`security_parameter` must be in [0, 128]");
  }
  return OkStatus();
}

}  // namespace

// Builds the per-level metadata (+ ProtoValidator::Create, proto_validator.cc:113-158).
StatusOr<std::unique_ptr<DpfState>> MakeDpfState(Span<const DpfParameters> parameters_in) {
  DPF_RETURN_IF_ERROR(ValidateParameters(parameters_in));
  auto st = std::make_unique<DpfState>();
  st->parameters.assign(parameters_in.begin(), parameters_in.end());
  for (DpfParameters& p : st->parameters)
    if (p.security_parameter() == 0) p.set_security_parameter(DefaultSecurity(p));
  // For backwards compatibility the reference registers all single unsigned
  // integers at construction (cc:620-633).
  for (int bits : {8, 16, 32, 64, 128}) {
    ValueType vt;
    vt.mutable_integer()->set_bitsize(bits);
    st->registered.insert(SerializeValueType(vt));
  }
  const int n = static_cast<int>(st->parameters.size());
  st->hierarchy_to_tree.resize(n);
  st->tree_to_hierarchy.assign(130, -1);
  st->levels.resize(n);
  int tree_levels_needed = 0;
  for (int i = 0; i < n; ++i) {
    const DpfParameters& p = st->parameters[i];
    StatusOr<int> bits = BitsNeeded(p.value_type(), p.security_parameter());
    if (!bits.ok()) return bits.status();
    int log_bits_needed = static_cast<int>(std::ceil(std::log2(*bits)));
    int tree_level = std::max(tree_levels_needed,
                              p.log_domain_size() - 7 + std::min(log_bits_needed, 7));
    st->tree_to_hierarchy[tree_level] = i;
    st->hierarchy_to_tree[i] = tree_level;
    tree_levels_needed = std::max(tree_levels_needed, tree_level + 1);

    LevelMeta& m = st->levels[i];
    Flatten(p.value_type(), &m.scalars);
    m.total_bits = 0;
    m.direct = true;
    for (const ScalarMeta& s : m.scalars) {
      m.total_bits += s.bits;
      if (s.kind == DPF_AMD_KIND_INT_MOD_N) m.direct = false;
    }
    m.epb = (m.direct && m.total_bits <= 128 && m.total_bits > 0) ? 128 / m.total_bits : 1;
    m.esz = (m.total_bits + 7) / 8;
    m.bn = (*bits + 127) / 128;
    m.tree_level = tree_level;
    m.log_domain = p.log_domain_size();
    dpf_amd_value_type& d = m.desc;
    memset(&d, 0, sizeof(d));
    d.num_scalars = static_cast<int32_t>(m.scalars.size());
    d.directly_convertible = m.direct ? 1 : 0;
    d.elements_per_block = m.epb;
    d.element_size = m.esz;
    d.blocks_needed = m.bn;
    std::vector<int> offs;
    Node node = Layout(p.value_type(), 0, &offs);
    d.out_stride = node.size;
    int in_off = 0;
    for (size_t s = 0; s < m.scalars.size() && s < DPF_AMD_MAX_SCALARS; ++s) {
      d.scalars[s].kind = m.scalars[s].kind;
      d.scalars[s].bytes = m.scalars[s].bits / 8;
      d.scalars[s].in_offset = in_off;
      d.scalars[s].out_offset = offs[s];
      d.scalars[s].modulus[0] = Uint128Low64(m.scalars[s].modulus);
      d.scalars[s].modulus[1] = Uint128High64(m.scalars[s].modulus);
      in_off += m.scalars[s].bits / 8;
    }
  }
  st->tree_levels_needed = tree_levels_needed;
  return st;
}

}  // namespace dpf_internal

using dpf_internal::DpfState;
using dpf_internal::LevelMeta;

// Protobuf text format (Message::DebugString): nested messages as
// "name {" ... "}", two-space indent, proto3 scalars omitted when zero
// (oneof members always printed), doubles as the shortest round-trip text.
namespace {

std::string Indent(int n) { return std::string(2 * n, ' '); }

std::string SimpleDtoa(double d) {
  char buf[64];
  snprintf(buf, sizeof(buf), "%.15g", d);
  if (strtod(buf, nullptr) != d) snprintf(buf, sizeof(buf), "%.17g", d);
  return buf;
}

void PrintValueInteger(const Value::Integer& v, int ind, std::ostringstream& os) {
  if (v.value_case() == Value::Integer::kValueUint64) {
    os << Indent(ind) << "value_uint64: " << v.value_uint64() << "\n";
  } else if (v.value_case() == Value::Integer::kValueUint128) {
    os << Indent(ind) << "value_uint128 {\n";
    if (v.value_uint128().high()) os << Indent(ind + 1) << "high: " << v.value_uint128().high() << "\n";
    if (v.value_uint128().low()) os << Indent(ind + 1) << "low: " << v.value_uint128().low() << "\n";
    os << Indent(ind) << "}\n";
  }
}

void PrintBitsize(const char* name, int32_t bitsize, int ind, std::ostringstream& os) {
  os << Indent(ind) << name << " {\n";
  if (bitsize) os << Indent(ind + 1) << "bitsize: " << bitsize << "\n";
  os << Indent(ind) << "}\n";
}

void PrintValueType(const ValueType& vt, int ind, std::ostringstream& os) {
  switch (vt.type_case()) {
    case ValueType::kInteger:
      PrintBitsize("integer", vt.integer().bitsize(), ind, os);
      break;
    case ValueType::kXorWrapper:
      PrintBitsize("xor_wrapper", vt.xor_wrapper().bitsize(), ind, os);
      break;
    case ValueType::kIntModN:
      os << Indent(ind) << "int_mod_n {\n";
      if (vt.int_mod_n().has_base_integer())
        PrintBitsize("base_integer", vt.int_mod_n().base_integer().bitsize(), ind + 1, os);
      if (vt.int_mod_n().has_modulus()) {
        os << Indent(ind + 1) << "modulus {\n";
        PrintValueInteger(vt.int_mod_n().modulus(), ind + 2, os);
        os << Indent(ind + 1) << "}\n";
      }
      os << Indent(ind) << "}\n";
      break;
    case ValueType::kTuple:
      os << Indent(ind) << "tuple {\n";
      for (const ValueType& e : vt.tuple().elements()) {
        os << Indent(ind + 1) << "elements {\n";
        PrintValueType(e, ind + 2, os);
        os << Indent(ind + 1) << "}\n";
      }
      os << Indent(ind) << "}\n";
      break;
    default:
      break;
  }
}

}  // namespace

std::string ValueType::DebugString() const {
  std::ostringstream os;
  PrintValueType(*this, 0, os);
  return os.str();
}

std::string DpfParameters::DebugString() const {
  std::ostringstream os;
  if (log_domain_size_) os << "log_domain_size: " << log_domain_size_ << "\n";
  if (has_value_type_) {
    os << "value_type {\n";
    PrintValueType(value_type_, 1, os);
    os << "}\n";
  }
  if (security_parameter_ != 0) os << "security_parameter: " << SimpleDtoa(security_parameter_) << "\n";
  return os.str();
}

Status DistributedPointFunction::RegisterValueTypeProto(const ValueType& value_type) {
  std::lock_guard<std::mutex> lock(state_->registry_mu);
  state_->registered.insert(SerializeValueType(value_type));
  return OkStatus();
}

bool DistributedPointFunction::IsValueTypeRegistered(const ValueType& value_type) const {
  std::lock_guard<std::mutex> lock(state_->registry_mu);
  return state_->registered.count(SerializeValueType(value_type)) != 0;
}

// ---------------------------------------------------------------------------
// Device helpers: csrc/host_device.h
// ---------------------------------------------------------------------------
using dpf_internal_host::AbiStatus;
using dpf_internal_host::ClearPadding;
using dpf_internal_host::CopyToHost;
using dpf_internal_host::CopyToHostSync;
using dpf_internal_host::DeviceBuffer;
using dpf_internal_host::HipStatus;
using dpf_internal_host::HostTrace;
using dpf_internal_host::HostPool;
using dpf_internal_host::ThreadStream;
using dpf_internal_host::StreamSyncGuard;
using dpf_internal_host::ThreadUploadRing;
using dpf_internal_host::UploadRing;

namespace {

struct CwArrays {
  std::vector<uint128> seeds;
  std::vector<uint8_t> ccl, ccr;
};

CwArrays KeyCws(const DpfKey& key, int start, int stop) {
  CwArrays c;
  for (int i = start; i < stop; ++i) {
    const CorrectionWord& cw = key.correction_words(i);
    c.seeds.push_back(MakeUint128(cw.seed().high(), cw.seed().low()));
    c.ccl.push_back(cw.control_left() ? 1 : 0);
    c.ccr.push_back(cw.control_right() ? 1 : 0);
  }
  return c;
}

struct U128Hash {
  size_t operator()(const uint128& v) const {
    uint64_t h = static_cast<uint64_t>(v) * 0x9E3779B97F4A7C15ull ^
                 (static_cast<uint64_t>(v >> 64) + 0x632BE59BD9B4E019ull);
    h ^= h >> 29;
    return static_cast<size_t>(h * 0xBF58476D1CE4E5B9ull);
  }
};

}  // namespace

// ---------------------------------------------------------------------------
// DistributedPointFunction
// ---------------------------------------------------------------------------

DistributedPointFunction::DistributedPointFunction(std::unique_ptr<DpfState> s)
    : state_(std::move(s)) {}
DistributedPointFunction::~DistributedPointFunction() = default;

StatusOr<std::unique_ptr<DistributedPointFunction>> DistributedPointFunction::Create(
    const DpfParameters& parameters) {
  return CreateIncremental(Span<const DpfParameters>(&parameters, 1));
}

StatusOr<std::unique_ptr<DistributedPointFunction>> DistributedPointFunction::CreateIncremental(
    Span<const DpfParameters> parameters) {
  StatusOr<std::unique_ptr<DpfState>> st = dpf_internal::MakeDpfState(parameters);
  if (!st.ok()) return st.status();
  return std::unique_ptr<DistributedPointFunction>(
      new DistributedPointFunction(std::move(*st)));
}

Span<const DpfParameters> DistributedPointFunction::parameters() const {
  return Span<const DpfParameters>(state_->parameters.data(), state_->parameters.size());
}
int DistributedPointFunction::num_hierarchy_levels() const {
  return static_cast<int>(state_->parameters.size());
}
int DistributedPointFunction::tree_levels_needed() const { return state_->tree_levels_needed; }
int DistributedPointFunction::hierarchy_to_tree(int h) const {
  return state_->hierarchy_to_tree[h];
}
int DistributedPointFunction::blocks_needed(int h) const { return state_->levels[h].bn; }
dpf_amd_value_type DistributedPointFunction::value_type_descriptor(int h) const {
  return state_->levels[h].desc;
}

Status DistributedPointFunction::CheckType(const ValueType& type, int level, bool at) const {
  const int n = num_hierarchy_levels();
  int lo = level, hi = level + 1;
  if (level < 0) {
    lo = 0;
    hi = n;
  } else if (level >= n) {
    return OkStatus();  // range errors are reported by the Raw entry points
  }
  for (int h = lo; h < hi; ++h) {
    StatusOr<bool> eq = dpf_internal::ValueTypesAreEqual(type, state_->parameters[h].value_type());
    if (!eq.ok()) return eq.status();
    if (!*eq) {
      if (at && level >= 0)
        return InvalidArgumentError("Value type T doesn't match parameters at `hierarchy_level`");
      return InvalidArgumentError("Value type T doesn't match parameters at `hierarchy_level`");
    }
  }
  return OkStatus();
}

// --- key generation (cc:81-222, 642-710) -----------------------------------

namespace {

// ComputeValueCorrection (cc:81-117) + ComputeValueCorrectionFor<T> (vth:614-648).
std::vector<uint128> ComputeValueCorrection(const DpfState& st, int h, const uint128 seeds[2],
                                            uint128 alpha_prefix,
                                            const std::vector<uint128>& beta, bool invert) {
  const LevelMeta& m = st.levels[h];
  const int bn = m.bn;
  std::vector<uint128> exp(2 * bn);
  for (int j = 0; j < bn; ++j) {
    exp[j] = seeds[0] + static_cast<uint128>(j);
    exp[bn + j] = seeds[1] + static_cast<uint128>(j);
  }
  st.prg_value.MmoHash(exp.data(), exp.data(), exp.size());
  const int bits = m.log_domain - m.tree_level;
  const int block_index = static_cast<int>(alpha_prefix & ((uint128{1} << bits) - 1));
  std::vector<uint128> a, b;
  m.Convert(reinterpret_cast<const uint8_t*>(exp.data()), 16 * bn, &a);
  m.Convert(reinterpret_cast<const uint8_t*>(exp.data() + bn), 16 * bn, &b);
  const int ns = static_cast<int>(m.scalars.size());
  for (int s = 0; s < ns; ++s)
    b[block_index * ns + s] = dpf_internal::ScAdd(m.scalars[s], b[block_index * ns + s], beta[s]);
  for (int e = 0; e < m.epb; ++e)
    for (int s = 0; s < ns; ++s) {
      uint128 v = dpf_internal::ScSub(m.scalars[s], b[e * ns + s], a[e * ns + s]);
      if (invert) v = dpf_internal::ScNeg(m.scalars[s], v);
      b[e * ns + s] = v;
    }
  return b;
}

void AddCorrectionValues(const DpfState& st, int h, const std::vector<uint128>& vc,
                         std::vector<Value>* out) {
  const LevelMeta& m = st.levels[h];
  const int ns = static_cast<int>(m.scalars.size());
  for (int e = 0; e < m.epb; ++e) {
    const uint128* it = vc.data() + e * ns;
    out->push_back(dpf_internal::UnflattenValue(st.parameters[h].value_type(), it));
  }
}

inline bool ExtractAndClearLowestBit(uint128& x) {
  bool bit = (x & 1) != 0;
  x &= ~uint128{1};
  return bit;
}

}  // namespace

StatusOr<std::pair<DpfKey, DpfKey>> DistributedPointFunction::GenerateKeysIncremental(
    uint128 alpha, const std::vector<uint128>& beta) {
  std::vector<Value> values;
  for (uint128 b : beta) {
    Value v;
    *v.mutable_integer() = dpf_internal::Uint128ToValueInteger(b);
    values.push_back(v);
  }
  return GenerateKeysIncremental(alpha, Span<const Value>(values.data(), values.size()));
}

StatusOr<std::pair<DpfKey, DpfKey>> DistributedPointFunction::GenerateKeysIncremental(
    uint128 alpha, Span<const Value> beta) {
  uint128 seeds[2];
  if (!dpf_amd::SecureRandom(seeds, sizeof(seeds)))
    return InternalError("Failed to obtain random bytes");
  return GenerateKeysIncrementalWithSeeds(alpha, beta, seeds[0], seeds[1]);
}

StatusOr<std::pair<DpfKey, DpfKey>> DistributedPointFunction::GenerateKeysIncrementalWithSeeds(
    uint128 alpha, Span<const Value> beta, uint128 seed0, uint128 seed1) {
  const DpfState& st = *state_;
  const int L = num_hierarchy_levels();
  if (static_cast<int>(beta.size()) != L)
    return InvalidArgumentError(
        "`beta` has to have the same size as `parameters` passed at construction");
  std::vector<std::vector<uint128>> flat(L);
  for (int i = 0; i < L; ++i) {
    DPF_RETURN_IF_ERROR(dpf_internal::ValidateValueOfType(beta[i], st.parameters[i].value_type()));
    DPF_RETURN_IF_ERROR(dpf_internal::FlattenValue(beta[i], st.parameters[i].value_type(), &flat[i]));
  }
  const int last_ld = st.parameters.back().log_domain_size();
  if (last_ld < 128 && alpha >= (uint128{1} << last_ld))
    return InvalidArgumentError("`alpha` must be smaller than the output domain size");
  // GetValueCorrectionFunction (cc:567-582), reached by every hierarchy
  // level's value correction in GenerateNext / the last level.
  for (int i = 0; i < L; ++i)
    if (!IsValueTypeRegistered(st.parameters[i].value_type()))
      return FailedPreconditionError(
          "No value correction function known for the following parameters:\n" +
          st.parameters[i].DebugString() +
          "Did you call RegisterValueType<T>() with your value type?");

  std::array<DpfKey, 2> keys;
  keys[0].set_party(0);
  keys[1].set_party(1);
  uint128 seeds[2] = {seed0, seed1};
  for (int p = 0; p < 2; ++p) {
    keys[p].mutable_seed()->set_high(Uint128High64(seeds[p]));
    keys[p].mutable_seed()->set_low(Uint128Low64(seeds[p]));
  }
  bool control_bits[2] = {false, true};
  for (int i = 1; i < st.tree_levels_needed; ++i) {  // GenerateNext (cc:121-222)
    CorrectionWord cw;
    const int h_prev = st.tree_to_hierarchy[i - 1];
    if (h_prev >= 0) {
      uint128 alpha_prefix = 0;
      const int shift = last_ld - st.parameters[h_prev].log_domain_size();
      if (shift < 128) alpha_prefix = alpha >> shift;
      std::vector<uint128> vc =
          ComputeValueCorrection(st, h_prev, seeds, alpha_prefix, flat[h_prev], control_bits[1]);
      AddCorrectionValues(st, h_prev, vc, cw.mutable_value_correction());
    }
    uint128 e[2][2];
    st.prg_left.MmoHash(seeds, e[0], 2);
    st.prg_right.MmoHash(seeds, e[1], 2);
    bool ecb[2][2];
    for (int b = 0; b < 2; ++b)
      for (int p = 0; p < 2; ++p) ecb[b][p] = ExtractAndClearLowestBit(e[b][p]);
    bool current_bit = false;
    if (last_ld - i < 128) current_bit = ((alpha >> (last_ld - i)) & 1) != 0;
    const int keep = current_bit ? 1 : 0, lose = 1 - keep;
    const uint128 seed_correction = e[lose][0] ^ e[lose][1];
    bool cc[2];
    cc[0] = ecb[0][0] ^ ecb[0][1] ^ current_bit ^ 1;
    cc[1] = ecb[1][0] ^ ecb[1][1] ^ current_bit;
    for (int p = 0; p < 2; ++p) {
      seeds[p] = e[keep][p];
      if (control_bits[p]) seeds[p] ^= seed_correction;
    }
    for (int p = 0; p < 2; ++p) control_bits[p] = ecb[keep][p] ^ (control_bits[p] && cc[keep]);
    cw.mutable_seed()->set_high(Uint128High64(seed_correction));
    cw.mutable_seed()->set_low(Uint128Low64(seed_correction));
    cw.set_control_left(cc[0]);
    cw.set_control_right(cc[1]);
    *keys[0].add_correction_words() = cw;
    *keys[1].add_correction_words() = cw;
  }
  std::vector<uint128> vc =
      ComputeValueCorrection(st, L - 1, seeds, alpha, flat[L - 1], control_bits[1]);
  std::vector<Value> last;
  AddCorrectionValues(st, L - 1, vc, &last);
  for (int p = 0; p < 2; ++p) *keys[p].mutable_last_level_value_correction() = last;
  return std::make_pair(std::move(keys[0]), std::move(keys[1]));
}

// --- validation of keys and contexts (proto_validator.cc:205-267) ----------

namespace {

Status ValidateDpfKey(const DpfState& st, const DpfKey& key) {
  if (!key.has_seed()) return InvalidArgumentError("key.seed must be present");
  if (key.last_level_value_correction().empty())
    return InvalidArgumentError("key.last_level_value_correction must be present");
  if (key.correction_words_size() != st.tree_levels_needed - 1)
    return InvalidArgumentError("Malformed DpfKey: expected " +
                                std::to_string(st.tree_levels_needed - 1) +
                                " correction words, but got " +
                                std::to_string(key.correction_words_size()));
  for (size_t i = 0; i < st.hierarchy_to_tree.size(); ++i) {
    const int t = st.hierarchy_to_tree[i];
    if (t == st.tree_levels_needed - 1) continue;
    if (key.correction_words(t).value_correction().empty())
      return InvalidArgumentError("Malformed DpfKey: expected correction_words[" +
                                  std::to_string(t) +
                                  "] to contain the value correction of hierarchy level " +
                                  std::to_string(i));
  }
  return OkStatus();
}

// `for_evaluate_at`: EvaluateAt may target any level of a context, so the
// "fully evaluated" check is skipped; the stored levels must still index the
// hierarchy (a parsed context is untrusted bytes).
Status ValidateEvaluationContext(const DpfState& st, const EvaluationContext& ctx,
                                 bool for_evaluate_at = false) {
  if (ctx.parameters_size() != static_cast<int>(st.parameters.size()))
    return InvalidArgumentError("Number of parameters in `ctx` doesn't match");
  for (int i = 0; i < ctx.parameters_size(); ++i) {
    StatusOr<bool> eq = dpf_internal::ParametersAreEqual(st.parameters[i], ctx.parameters(i));
    if (!eq.ok()) return eq.status();
    if (!*eq) return InvalidArgumentError("Parameter " + std::to_string(i) + " in `ctx` doesn't match");
  }
  if (!ctx.has_key()) return InvalidArgumentError("ctx.key must be present");
  DPF_RETURN_IF_ERROR(ValidateDpfKey(st, ctx.key()));
  const int num_levels = ctx.parameters_size();
  if (!for_evaluate_at && ctx.previous_hierarchy_level() >= num_levels - 1)
    return InvalidArgumentError("This context has already been fully evaluated");
  if (ctx.previous_hierarchy_level() < -1 || ctx.previous_hierarchy_level() >= num_levels)
    return InvalidArgumentError("ctx.previous_hierarchy_level out of range");
  if (ctx.partial_evaluations_level() < 0 || ctx.partial_evaluations_level() >= num_levels)
    return InvalidArgumentError("ctx.partial_evaluations_level out of range");
  if (ctx.partial_evaluations_size() > 0 &&
      ctx.partial_evaluations_level() > ctx.previous_hierarchy_level())
    return InvalidArgumentError(
        "ctx.partial_evaluations_level must be less than or equal to "
        "ctx.previous_hierarchy_level");
  return OkStatus();
}

// ValuesToArray<T> (vth:561-580) flattened.
Status CorrectionsFor(const DpfState& st, const DpfKey& key, int h, std::vector<uint128>* out) {
  const std::vector<Value>* vals;
  if (h < static_cast<int>(st.parameters.size()) - 1)
    vals = &key.correction_words(st.hierarchy_to_tree[h]).value_correction();
  else
    vals = &key.last_level_value_correction();
  const LevelMeta& m = st.levels[h];
  if (static_cast<int>(vals->size()) != m.epb)
    return InvalidArgumentError("values.size() (= " + std::to_string(vals->size()) +
                                ") does not match ElementsPerBlock<T>() (= " +
                                std::to_string(m.epb) + ")");
  out->clear();
  for (const Value& v : *vals)
    DPF_RETURN_IF_ERROR(dpf_internal::FlattenValue(v, st.parameters[h].value_type(), out));
  return OkStatus();
}

// Merges the conversion metadata of level h with the caller's host layout.
Status MergeLayout(const LevelMeta& m, const dpf_amd_value_type& layout, dpf_amd_value_type* out) {
  *out = m.desc;
  if (layout.num_scalars != m.desc.num_scalars)
    return InvalidArgumentError("Value type T doesn't match parameters at `hierarchy_level`");
  if (m.desc.num_scalars > DPF_AMD_MAX_SCALARS)
    return UnimplementedError("too many tuple elements");
  for (int s = 0; s < m.desc.num_scalars; ++s) {
    if (m.scalars[s].bits < 8)
      return UnimplementedError("element bit sizes below 8 are not supported");
    out->scalars[s].out_offset = layout.scalars[s].out_offset;
  }
  out->out_stride = layout.out_stride;
  return OkStatus();
}

}  // namespace

Status DistributedPointFunction::ValidateKey(const DpfKey& key) const {
  return ValidateDpfKey(*state_, key);
}

Status DistributedPointFunction::ValueCorrectionWords(const DpfKey& key, int level,
                                                      std::vector<uint128>* out) const {
  if (level < 0 || level >= num_hierarchy_levels())
    return InvalidArgumentError("`hierarchy_level` out of range");
  return CorrectionsFor(*state_, key, level, out);
}

StatusOr<EvaluationContext> DistributedPointFunction::CreateEvaluationContext(DpfKey key) const {
  DPF_RETURN_IF_ERROR(ValidateDpfKey(*state_, key));
  EvaluationContext r;
  for (const DpfParameters& p : state_->parameters) *r.add_parameters() = p;
  *r.mutable_key() = std::move(key);
  r.set_previous_hierarchy_level(-1);
  return r;
}

// --- evaluation --------------------------------------------------------------

// The partial evaluations of an EvaluationContext kept in HBM between
// EvaluateUntil calls: the previous level's unique tree
// indices (strictly increasing), their walked seeds and control bits, in one
// pool block on `device`.  EvaluateUntil's device path looks its prefixes up
// here; a caller reading the context's field gets host messages built once.
class ContextDeviceState {
 public:
  // Freed on a stream the library owns, never the caller's: a context
  // outlives the stream its EvaluateUntil ran on, and every kernel that wrote
  // or read the list finished before the state was attached to (or dropped
  // from) a context — EvaluateUntilOnDevice synchronizes its stream first.
  ~ContextDeviceState() {
    if (buf_ == nullptr) return;
    dpf_internal_host::DeviceGuard g(device_);
    dpf_internal_host::DevicePool::Get().Free(buf_, dpf_internal_host::ThreadStreamOn(device_));
  }
  // `s`: the stream the list is first written on (allocation only).
  static Status Create(int64_t capacity, hipStream_t s, std::shared_ptr<ContextDeviceState>* out) {
    auto st = std::shared_ptr<ContextDeviceState>(new ContextDeviceState());
    DPF_RETURN_IF_ERROR(HipStatus(hipGetDevice(&st->device_), "hipGetDevice"));
    const int64_t n = std::max<int64_t>(1, capacity);
    const int64_t bytes = 32 * n + ((n + 15) & ~int64_t{15}) + 16;
    DPF_RETURN_IF_ERROR(dpf_internal_host::DevicePool::Get().Alloc(bytes, s, &st->buf_));
    char* b = static_cast<char*>(st->buf_);
    st->prefixes_ = b;
    st->seeds_ = b + 16 * n;
    st->cbs_ = reinterpret_cast<uint8_t*>(b + 32 * n);
    st->count_dev_ = reinterpret_cast<int64_t*>(b + 32 * n + ((n + 15) & ~int64_t{15}));
    *out = std::move(st);
    return OkStatus();
  }
  int device() const { return device_; }
  char* prefixes() const { return prefixes_; }
  char* seeds() const { return seeds_; }
  uint8_t* cbs() const { return cbs_; }
  int64_t* count_dev() const { return count_dev_; }
  int64_t count() const { return count_; }
  void set_count(int64_t c) { count_ = c; }

  // The list as host messages, read back on first use (the kernels that
  // wrote it finished before the state was attached to a context).
  const std::vector<PartialEvaluation>& Host() const {
    std::call_once(once_, [this] {
      const size_t n = static_cast<size_t>(count_);
      std::vector<uint128> p(n), sd(n);
      std::vector<uint8_t> cb(n);
      dpf_internal_host::DeviceGuard g(device_);
      host_.resize(n);  // the size partial_evaluations_size() reported, whatever happens
      if (n == 0) return;
      if (hipMemcpy(p.data(), prefixes_, 16 * n, hipMemcpyDeviceToHost) != hipSuccess ||
          hipMemcpy(sd.data(), seeds_, 16 * n, hipMemcpyDeviceToHost) != hipSuccess ||
          hipMemcpy(cb.data(), cbs_, n, hipMemcpyDeviceToHost) != hipSuccess) {
        // an accessor cannot return a status: the entries stay zero and the
        // error goes to stderr
        std::fprintf(stderr, "[dpf_amd] reading back a context's partial evaluations failed: %s\n",
                     hipGetErrorString(hipGetLastError()));
        return;
      }
      for (size_t i = 0; i < n; ++i) {
        PartialEvaluation& x = host_[i];
        x.mutable_prefix()->set_high(Uint128High64(p[i]));
        x.mutable_prefix()->set_low(Uint128Low64(p[i]));
        x.mutable_seed()->set_high(Uint128High64(sd[i]));
        x.mutable_seed()->set_low(Uint128Low64(sd[i]));
        x.set_control_bit(cb[i] != 0);
      }
    });
    return host_;
  }

 private:
  ContextDeviceState() = default;
  int device_ = 0;
  void* buf_ = nullptr;
  char* prefixes_ = nullptr;
  char* seeds_ = nullptr;
  uint8_t* cbs_ = nullptr;
  int64_t* count_dev_ = nullptr;
  int64_t count_ = 0;
  mutable std::once_flag once_;
  mutable std::vector<PartialEvaluation> host_;
};

const std::vector<PartialEvaluation>& PartialEvaluationsOf(const ContextDeviceState& state) {
  return state.Host();
}
int PartialEvaluationsCountOf(const ContextDeviceState& state) {
  return static_cast<int>(state.count());
}

namespace {

// Per-thread host scratch of the incremental path, kept across calls: at
// 2^16 prefixes per level (c3) fresh vectors of a few MiB each cost more in
// page faults than the loops that fill them.  The seeds / control bits live in
// pinned memory, so the walked seeds come back by an asynchronous DMA.
struct IncrementalScratch {
  std::vector<int64_t> src;
  uint128* tree = nullptr;   // pinned: unique tree indices (the walk's paths)
  uint128* seeds = nullptr;  // pinned
  uint8_t* cbs = nullptr;    // pinned
  int* flag = nullptr;       // pinned: the gather's error flag (an async copy)
  int32_t* pidx = nullptr;   // pinned: per-prefix unique-root index (prefix expansion)
  uint8_t* plow = nullptr;   // pinned: per-prefix bits below its tree index
  size_t cap = 0;
  hipEvent_t done = nullptr;
  int device = -1;
  ~IncrementalScratch() {
    if (done) {
      (void)hipEventSynchronize(done);
      (void)hipEventDestroy(done);
    }
    if (tree) (void)hipHostFree(tree);
    if (seeds) (void)hipHostFree(seeds);
    if (cbs) (void)hipHostFree(cbs);
    if (flag) (void)hipHostFree(flag);
    if (pidx) (void)hipHostFree(pidx);
    if (plow) (void)hipHostFree(plow);
  }
  Status Reserve(size_t n) {
    if (!flag) DPF_RETURN_IF_ERROR(HipStatus(hipHostMalloc((void**)&flag, 64, 0), "hipHostMalloc"));
    int dev = 0;
    DPF_RETURN_IF_ERROR(HipStatus(hipGetDevice(&dev), "hipGetDevice"));
    if (done && device != dev) {  // events are recorded on streams of their device
      (void)hipEventSynchronize(done);
      (void)hipEventDestroy(done);
      done = nullptr;
    }
    if (!done) {
      DPF_RETURN_IF_ERROR(
          HipStatus(hipEventCreateWithFlags(&done, hipEventDisableTiming), "hipEventCreate"));
      device = dev;
    }
    if (n <= cap) return OkStatus();
    if (tree) (void)hipHostFree(tree);
    if (seeds) (void)hipHostFree(seeds);
    if (cbs) (void)hipHostFree(cbs);
    if (pidx) (void)hipHostFree(pidx);
    if (plow) (void)hipHostFree(plow);
    tree = nullptr;
    seeds = nullptr;
    cbs = nullptr;
    pidx = nullptr;
    plow = nullptr;
    cap = 0;
    size_t c = 1024;
    while (c < n) c <<= 1;
    DPF_RETURN_IF_ERROR(HipStatus(hipHostMalloc((void**)&tree, 16 * c, 0), "hipHostMalloc"));
    DPF_RETURN_IF_ERROR(HipStatus(hipHostMalloc((void**)&seeds, 16 * c, 0), "hipHostMalloc"));
    DPF_RETURN_IF_ERROR(HipStatus(hipHostMalloc((void**)&cbs, c, 0), "hipHostMalloc"));
    DPF_RETURN_IF_ERROR(HipStatus(hipHostMalloc((void**)&pidx, 4 * c, 0), "hipHostMalloc"));
    DPF_RETURN_IF_ERROR(HipStatus(hipHostMalloc((void**)&plow, c, 0), "hipHostMalloc"));
    cap = c;
    return OkStatus();
  }
};

IncrementalScratch& ThreadScratch() {
  return dpf_internal_host::ThreadRecycled<IncrementalScratch>::Get();
}

// The context rewrite of ComputePartialEvaluations, deferred: the walked
// seeds come back by DMA behind the walk, and the caller rewrites `ctx`
// (FinishContextUpdate) after it has queued the expansion, so the host work
// overlaps the GPU's.
// ctx.partial_evaluations = (prefix i, seed i, control bit i), the stored
// list of cc:505-519.  The list is resized in place (the previous level's
// entries are overwritten, not destroyed and value-initialised again) and
// filled over the host pool: 2^16 entries per c3 level.
void RewritePartialEvaluations(EvaluationContext& ctx, const uint128* prefixes,
                               const uint128* seeds, const uint8_t* cbs, int64_t n) {
  // a device-held list is replaced, not read back first
  if (ctx.device_state()) ctx.set_device_state(nullptr);
  std::vector<PartialEvaluation>* pe = ctx.mutable_partial_evaluations();
  pe->resize(n);
  HostPool::Get().ParallelRanges(n, 8192, [&](int, int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) {
      PartialEvaluation& x = (*pe)[i];
      x.mutable_prefix()->set_high(Uint128High64(prefixes[i]));
      x.mutable_prefix()->set_low(Uint128Low64(prefixes[i]));
      x.mutable_seed()->set_high(Uint128High64(seeds[i]));
      x.mutable_seed()->set_low(Uint128Low64(seeds[i]));
      x.set_control_bit(cbs[i] != 0);
    }
  });
}

#ifndef DPF_HOST_FUSED_LOOKUP
#define DPF_HOST_FUSED_LOOKUP 1  // stored-order check and merge join in one pool job
#endif

struct PendingContextUpdate {
  bool active = false;
  Span<const uint128> prefixes;
  int hierarchy_level = 0;
};

Status FinishContextUpdate(PendingContextUpdate& p, EvaluationContext& ctx) {
  if (!p.active) return OkStatus();
  p.active = false;
  HostTrace trace("FinishContextUpdate");
  IncrementalScratch& sc = ThreadScratch();
  DPF_RETURN_IF_ERROR(HipStatus(hipEventSynchronize(sc.done), "d2h"));
  trace.Mark("wait");
  RewritePartialEvaluations(ctx, p.prefixes.data(), sc.seeds, sc.cbs,
                            static_cast<int64_t>(p.prefixes.size()));
  ctx.set_partial_evaluations_level(p.hierarchy_level);
  trace.Mark("rewrite");
  return OkStatus();
}

// ComputePartialEvaluations (cc:374-476): selects the stored partial
// evaluations for `prefixes` (host map, as the reference's btree), walks them
// on the device to `hierarchy_level`'s tree level, and rewrites ctx.
// Returns device seeds / control bits for the prefixes, inside `buf`: every
// input of the walk goes up in one pinned slot and one DMA (c3: 2^16
// prefixes per level, where host work rivals the kernels).
Status ComputePartialEvaluations(const DpfState& st, Span<const uint128> prefixes,
                                 int hierarchy_level, bool update_ctx, EvaluationContext& ctx,
                                 hipStream_t s, DeviceBuffer* buf, void** seeds_dev,
                                 uint8_t** cb_dev, PendingContextUpdate* pending = nullptr) {
  HostTrace trace("PartialEvaluations");
  const int64_t n = static_cast<int64_t>(prefixes.size());
  int start_level = st.hierarchy_to_tree[ctx.partial_evaluations_level()];
  const int stop_level = st.hierarchy_to_tree[hierarchy_level];
  IncrementalScratch& sc = ThreadScratch();
  // prefixes already in the pinned scratch (EvaluateUntil's tree indices):
  // the caller reserved it, and they go up by DMA without a host copy
  const bool prefixes_pinned = prefixes.data() == sc.tree;
  if (!prefixes_pinned) {
    // a deferred DMA of an earlier call into the scratch must have landed
    if (sc.done) DPF_RETURN_IF_ERROR(HipStatus(hipEventSynchronize(sc.done), "d2h"));
    DPF_RETURN_IF_ERROR(sc.Reserve(n > 0 ? n : 1));
  }
  uint128* seeds = sc.seeds;
  uint8_t* cbs = sc.cbs;
  // A list the device path left in HBM (this device) is looked up there by
  // binary search (LookupPartialEvaluations), not read back to the host.
  const ContextDeviceState* dstate = ctx.device_state().get();
  int cur_dev = 0;
  DPF_RETURN_IF_ERROR(HipStatus(hipGetDevice(&cur_dev), "hipGetDevice"));
  const bool dev_lookup = dstate != nullptr && dstate->device() == cur_dev &&
                          dstate->count() > 0 && start_level <= stop_level && n > 0;
  if (dev_lookup) {
    // the seeds and control bits come from the lookup kernel below
  } else if (ctx.partial_evaluations_size() > 0 && start_level <= stop_level) {
    const int shift = stop_level - start_level;
    const auto& pes = ctx.partial_evaluations();
    const int64_t m = static_cast<int64_t>(pes.size());
    auto pe_prefix = [&](int64_t j) {
      return MakeUint128(pes[j].prefix().high(), pes[j].prefix().low());
    };
    auto query = [&](int64_t i) { return shift < 128 ? (prefixes[i] >> shift) : uint128{0}; };
    // Sorted fast path (the common case: prefixes come from a sorted
    // candidate list, and the stored evaluations are the previous call's
    // sorted tree indices): a merge join instead of the reference's btree,
    // split over the host pool (each query range binary-searches its start),
    // checking both orders on the way.  The reference rejects a mismatching
    // duplicate anywhere in the stored list (cc:390-405), so the merge
    // result stands only if the whole list is strictly increasing (then it
    // holds no duplicate at all).  Anything it cannot decide (an unsorted
    // side, a prefix it does not find) goes to the hash path, which also
    // produces the reference's errors.
    bool merged = m > 0;
    HostPool& pool = HostPool::Get();
    constexpr int kParts = static_cast<int>(HostPool::kWorkers) + 1;
    bool ok[kParts];
    // queries [b, e) against the stored list; false when the merge cannot
    // decide (an order violation or a prefix not found)
    auto merge_range = [&](int64_t b, int64_t e) {
      if (b >= e) return true;
      bool good = b == 0 || query(b - 1) <= query(b);
      const uint128 q0 = query(b);
      int64_t lo = 0, hi = m;  // first stored prefix >= q0
      while (lo < hi) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (pe_prefix(mid) < q0)
          lo = mid + 1;
        else
          hi = mid;
      }
      int64_t j = lo;
      uint128 prev = q0;
      for (int64_t i = b; i < e && good; ++i) {
        const uint128 q = query(i);
        if (q < prev) return false;
        prev = q;
        while (j < m && pe_prefix(j) < q) ++j;
        if (j == m || pe_prefix(j) != q) return false;
        seeds[i] = MakeUint128(pes[j].seed().high(), pes[j].seed().low());
        cbs[i] = pes[j].control_bit() ? 1 : 0;
      }
      return good;
    };
    auto stored_order = [&](int64_t b, int64_t e) {
      bool good = true;
      for (int64_t k = std::max<int64_t>(b, 1); k < e; ++k) good &= pe_prefix(k - 1) < pe_prefix(k);
      return good;
    };
#if DPF_HOST_FUSED_LOOKUP
    if (merged) {
      // One pool job: part r checks the strict order of its slice of the
      // stored list and merges its slice of the queries.
      const int64_t parts = std::max<int64_t>(
          1, std::min<int64_t>(kParts, std::max(n / 4096, m / 8192)));
      const int64_t mper = (m + parts - 1) / parts, nper = (n + parts - 1) / parts;
      pool.Run(static_cast<size_t>(parts), [&](size_t r) {
        const int64_t mb = std::min<int64_t>(static_cast<int64_t>(r) * mper, m);
        const int64_t nb = std::min<int64_t>(static_cast<int64_t>(r) * nper, n);
        ok[r] = stored_order(mb, std::min<int64_t>(mb + mper, m)) &&
                merge_range(nb, std::min<int64_t>(nb + nper, n));
      });
      for (int64_t r = 0; r < parts; ++r) merged &= ok[r];
    }
#else
    if (merged) {
      const int parts = pool.ParallelRanges(
          m, 8192, [&](int r, int64_t b, int64_t e) { ok[r] = stored_order(b, e); });
      for (int r = 0; r < parts; ++r) merged &= ok[r];
    }
    if (merged && n > 0) {
      const int parts = pool.ParallelRanges(
          n, 4096, [&](int r, int64_t b, int64_t e) { ok[r] = merge_range(b, e); });
      for (int r = 0; r < parts; ++r) merged &= ok[r];
    }
#endif
    if (!merged) {
      std::unordered_map<uint128, std::pair<uint128, bool>, U128Hash> prev;
      prev.reserve(m * 2);
      for (const PartialEvaluation& e : pes) {
        const uint128 prefix = MakeUint128(e.prefix().high(), e.prefix().low());
        const std::pair<uint128, bool> value{MakeUint128(e.seed().high(), e.seed().low()),
                                             e.control_bit()};
        auto it = prev.emplace(prefix, value).first;
        if (it->second != value)
          return InvalidArgumentError(
              "Duplicate prefix in `ctx.partial_evaluations()` with mismatching seed or "
              "control bit");
      }
      for (int64_t i = 0; i < n; ++i) {
        auto it = prev.find(query(i));
        if (it == prev.end())
          return InvalidArgumentError(
              "Prefix not present in ctx.partial_evaluations at hierarchy level " +
              std::to_string(hierarchy_level));
        seeds[i] = it->second.first;
        cbs[i] = it->second.second ? 1 : 0;
      }
    }
  } else {
    const uint128 seed = MakeUint128(ctx.key().seed().high(), ctx.key().seed().low());
    std::fill(seeds, seeds + n, seed);
    std::fill(cbs, cbs + n, static_cast<uint8_t>(ctx.key().party() != 0));
    start_level = 0;
  }
  trace.Mark("lookup");
  const int levels = stop_level - start_level;
  CwArrays cw = KeyCws(ctx.key(), start_level, stop_level);
  const bool walk = levels > 0 && n > 0;
  using Part = UploadRing::HostPart;
  // correction words (and the lookup's count) through the upload ring; the
  // pinned seeds / control bits (and pinned prefixes) by direct DMA
  const int64_t count_n = n;
  const Part cw_parts[4] = {{cw.seeds.data(), walk ? size_t(16) * levels : 0},
                            {cw.ccl.data(), walk ? size_t(levels) : 0},
                            {cw.ccr.data(), walk ? size_t(levels) : 0},
                            {&count_n, dev_lookup ? sizeof(int64_t) : 0}};
  size_t cw_off[4];
  const size_t cw_bytes = UploadRing::PackedLayout(cw_parts, 4, cw_off);
  const Part parts[3] = {{seeds, dev_lookup ? 0 : size_t(16) * n},
                         {cbs, dev_lookup ? 0 : size_t(n)},
                         {prefixes.data(), walk || dev_lookup ? size_t(16) * n : 0}};
  const size_t seeds_bytes[2] = {size_t(16) * n, size_t(n)};
  size_t off[7];
  Part laid[3] = {{seeds, seeds_bytes[0]}, {cbs, seeds_bytes[1]}, parts[2]};
  const size_t bytes = cw_bytes + UploadRing::PackedLayout(laid, 3, off) + 16;
  for (int i = 0; i < 3; ++i) {
    off[i] += cw_bytes;
    off[3 + i] = cw_off[i];
  }
  off[6] = bytes - 16;  // the lookup's flags
  DPF_RETURN_IF_ERROR(buf->Alloc(bytes, s));
  char* d = buf->as<char>();
  DPF_RETURN_IF_ERROR(ThreadUploadRing().CopyPacked(d, cw_parts, 4, cw_bytes, cw_off, s));
  for (int i = 0; i < 3; ++i) {
    if (parts[i].bytes == 0) continue;
    if (i < 2 || prefixes_pinned)
      DPF_RETURN_IF_ERROR(HipStatus(
          hipMemcpyAsync(d + off[i], parts[i].p, parts[i].bytes, hipMemcpyHostToDevice, s),
          "upload"));
    else
      DPF_RETURN_IF_ERROR(ThreadUploadRing().Copy(d + off[i], parts[i].p, parts[i].bytes, s));
  }
  *seeds_dev = d + off[0];
  *cb_dev = reinterpret_cast<uint8_t*>(d + off[1]);
  if (dev_lookup) {
    int* flags = reinterpret_cast<int*>(d + off[6]);
    DPF_RETURN_IF_ERROR(HipStatus(hipMemsetAsync(flags, 0, sizeof(int), s), "hipMemsetAsync"));
    const uint64_t root[2] = {ctx.key().seed().low(), ctx.key().seed().high()};
    DPF_RETURN_IF_ERROR(AbiStatus(dpf_amd::LookupPartialEvaluations(
        d + off[2], reinterpret_cast<const int64_t*>(d + cw_off[3]), n,
        stop_level - start_level, dstate->prefixes(), dstate->count(), dstate->seeds(),
        dstate->cbs(), root, ctx.key().party() != 0, false, d + off[0],
        reinterpret_cast<uint8_t*>(d + off[1]), flags, s)));
    // the reference reports a missing prefix before it changes the context
    int host_flags = 0;
    DPF_RETURN_IF_ERROR(HipStatus(
        hipMemcpyAsync(&host_flags, flags, sizeof(int), hipMemcpyDeviceToHost, s), "d2h"));
    DPF_RETURN_IF_ERROR(HipStatus(hipStreamSynchronize(s), "sync"));
    if (host_flags != 0)
      return InvalidArgumentError(
          "Prefix not present in ctx.partial_evaluations at hierarchy level " +
          std::to_string(hierarchy_level));
  }
  if (walk) {
    DPF_RETURN_IF_ERROR(AbiStatus(dpf_amd_evaluate_seeds(
        n, levels, levels, d + off[0], *cb_dev, d + off[2], 0, d + off[3],
        reinterpret_cast<const uint8_t*>(d + off[4]), reinterpret_cast<const uint8_t*>(d + off[5]),
        dpf_amd::kPrgKeyLeftLo, dpf_amd::kPrgKeyLeftHi, dpf_amd::kPrgKeyRightLo,
        dpf_amd::kPrgKeyRightHi, d + off[0], *cb_dev, s)));
  }
  trace.Mark("upload+walk_launch");
  if (!(update_ctx && n > 0)) ctx.clear_partial_evaluations();
  if (update_ctx && n > 0) {
    // seeds / cbs are pinned: the copies are true DMAs behind the walk
    DPF_RETURN_IF_ERROR(CopyToHost(seeds, *seeds_dev, 16 * n, s));
    DPF_RETURN_IF_ERROR(CopyToHost(cbs, *cb_dev, n, s));
    DPF_RETURN_IF_ERROR(HipStatus(hipEventRecord(sc.done, s), "hipEventRecord"));
    if (pending != nullptr) {
      pending->active = true;
      pending->prefixes = prefixes;
      pending->hierarchy_level = hierarchy_level;
      trace.Mark("d2h_queued");
      return OkStatus();
    }
    DPF_RETURN_IF_ERROR(HipStatus(hipEventSynchronize(sc.done), "sync"));
    RewritePartialEvaluations(ctx, prefixes.data(), seeds, cbs, n);
  }
  trace.Mark("d2h+ctx_rewrite");
  ctx.set_partial_evaluations_level(hierarchy_level);
  return OkStatus();
}

// EvaluateUntil with prefixes, on the device end to end:
// the prefixes go up once; their de-duplication, the range and order checks,
// the lookup of the stored partial evaluations (ComputePartialEvaluations,
// cc:374-476) and the walk run as kernels; the walked unique tree indices stay
// in HBM as the context's new list (a ContextDeviceState).  Sets *fallback
// (and leaves ctx as it was) when the host path must run instead: a context
// whose list is on the host or another device, unsorted prefixes, a prefix
// out of range or not in the list — the host path then gives the reference's
// result or error.
Status EvaluateUntilOnDevice(const DpfState& st, int hierarchy_level,
                             Span<const uint128> prefixes, EvaluationContext& ctx,
                             const dpf_amd_value_type& vt, const std::vector<uint128>& corr,
                             void* out, bool out_on_device, hipStream_t s, bool* fallback) {
  *fallback = true;
  HostTrace trace("EvaluateUntilOnDevice");
  const int L = static_cast<int>(st.parameters.size());
  const int prev_h = ctx.previous_hierarchy_level();
  const int prev_ld = st.parameters[prev_h].log_domain_size();
  const int prev_tree = st.hierarchy_to_tree[prev_h];
  const int stop_level = st.hierarchy_to_tree[hierarchy_level];
  const int log_domain_size = st.parameters[hierarchy_level].log_domain_size();
  const int bbits = prev_ld - prev_tree;  // prefix bits below its tree index (< 8)
  const int64_t n = static_cast<int64_t>(prefixes.size());
  if (n == 0 || n >= (int64_t{1} << 31) || bbits > 7 || stop_level < prev_ld) return OkStatus();
  int cur_dev = 0;
  DPF_RETURN_IF_ERROR(HipStatus(hipGetDevice(&cur_dev), "hipGetDevice"));
  // where the walk starts: the stored list (device-held, this device) or the root
  std::shared_ptr<const ContextDeviceState> old = ctx.device_state();
  bool from_root = true;
  int start_level = 0;
  if (old) {
    if (old->device() != cur_dev) return OkStatus();
    const int pe_level = ctx.partial_evaluations_level();
    const int sl = st.hierarchy_to_tree[pe_level];
    if (old->count() > 0 && sl <= prev_tree) {
      from_root = false;
      start_level = sl;
    }
  } else if (ctx.partial_evaluations_size() > 0) {
    return OkStatus();  // a host-held list (a parsed or host-path context)
  }
  const int walk_levels = prev_tree - start_level;
  const int down = stop_level - prev_ld;
  const int cepb = 1 << (log_domain_size - stop_level);
  const int64_t outputs_per_prefix = int64_t{1} << (log_domain_size - prev_ld);
  const int64_t total = n * outputs_per_prefix;
  const size_t stride = static_cast<size_t>(vt.out_stride);
  const bool update_ctx = hierarchy_level < L - 1;

  // work buffer: prefixes | prefix index | low bits | dedup block counts |
  // flags | correction words (walk, prefix roots, expansion) | prefix roots
  CwArrays kc = KeyCws(ctx.key(), start_level, prev_tree);
  CwArrays wc = KeyCws(ctx.key(), prev_tree, prev_ld);
  CwArrays ec = KeyCws(ctx.key(), prev_ld, stop_level);
  using Part = UploadRing::HostPart;
  const Part parts[9] = {{kc.seeds.data(), size_t(16) * walk_levels},
                         {kc.ccl.data(), size_t(walk_levels)},
                         {kc.ccr.data(), size_t(walk_levels)},
                         {wc.seeds.data(), size_t(16) * bbits},
                         {wc.ccl.data(), size_t(bbits)},
                         {wc.ccr.data(), size_t(bbits)},
                         {ec.seeds.data(), size_t(16) * down},
                         {ec.ccl.data(), size_t(down)},
                         {ec.ccr.data(), size_t(down)}};
  size_t coff[9];
  const size_t cw_bytes = UploadRing::PackedLayout(parts, 9, coff);
  auto al = [](size_t b) { return (b + 255) & ~size_t{255}; };
  const size_t o_p = 0;
  const size_t o_idx = o_p + al(16 * size_t(n));
  const size_t o_low = o_idx + al(4 * size_t(n));
  const size_t o_blk = o_low + al(size_t(n));
  const size_t o_flags = o_blk + al(8 * size_t(dpf_amd::DedupBlocks(n)));
  const size_t o_cw = o_flags + 256;
  const size_t o_ps = o_cw + al(cw_bytes);
  const size_t o_pcb = o_ps + al(16 * size_t(n));
  const size_t o_out = o_pcb + al(size_t(n));
  DeviceBuffer work;
  DPF_RETURN_IF_ERROR(work.Alloc(o_out + (out_on_device ? 0 : total * stride), s));
  char* w = work.as<char>();
  std::shared_ptr<ContextDeviceState> next;
  DPF_RETURN_IF_ERROR(ContextDeviceState::Create(n, s, &next));
  IncrementalScratch& sc = ThreadScratch();
  if (sc.done) DPF_RETURN_IF_ERROR(HipStatus(hipEventSynchronize(sc.done), "d2h"));
  DPF_RETURN_IF_ERROR(sc.Reserve(1));
  int64_t* readback = reinterpret_cast<int64_t*>(sc.flag);  // pinned: flags, count
  readback[0] = readback[1] = 0;
  // an early error return must not leave an async copy into `readback` in flight
  StreamSyncGuard drain(s);
  trace.Mark("setup");
  int* flags = reinterpret_cast<int*>(w + o_flags);
  DPF_RETURN_IF_ERROR(HipStatus(hipMemsetAsync(flags, 0, sizeof(int), s), "hipMemsetAsync"));
  // The prefixes are written by the host straight into fine-grained device
  // memory (large-BAR devices, UploadRing::Place) and read there by the
  // de-duplication, in place of a pinned-slot memcpy, a copy kernel and its
  // dependent-dispatch gap (~60 us of a c3 level): c3's 16 levels 6.43-6.93
  // -> 6.14-6.26 ms (profiles/ab_place_prefixes_r06/).  DPF_AMD_PLACE_PREFIXES=0
  // keeps the copy (A/B); devices without the host-write path copy anyway.
  static const bool place_prefixes = [] {
    const char* e = std::getenv("DPF_AMD_PLACE_PREFIXES");
    return !(e != nullptr && std::strcmp(e, "0") == 0);
  }();
  bool pplaced = false;
  int pslot = -1;
  char* pdev = nullptr;
  if (place_prefixes) {
    const UploadRing::HostPart pp{prefixes.data(), 16 * size_t(n)};
    const size_t off0 = 0;
    DPF_RETURN_IF_ERROR(
        ThreadUploadRing().Place(&pp, 1, 16 * size_t(n), &off0, &pplaced, &pslot, &pdev,
                                 UploadRing::kMaxPlaceLargeBytes));
  }
  const char* pref = pplaced ? pdev : w + o_p;
  if (!pplaced)
    DPF_RETURN_IF_ERROR(ThreadUploadRing().Copy(w + o_p, prefixes.data(), 16 * size_t(n), s));
  DPF_RETURN_IF_ERROR(ThreadUploadRing().CopyPacked(w + o_cw, parts, 9, cw_bytes, coff, s));
  trace.Mark("upload");
  const uint64_t limit[2] = {prev_ld < 64 ? (uint64_t{1} << prev_ld) : 0,
                             prev_ld >= 64 && prev_ld < 128 ? (uint64_t{1} << (prev_ld - 64)) : 0};
  int32_t* pidx = reinterpret_cast<int32_t*>(w + o_idx);
  uint8_t* plow = reinterpret_cast<uint8_t*>(w + o_low);
  DPF_RETURN_IF_ERROR(AbiStatus(dpf_amd::DedupPrefixes(
      pref, n, bbits, prev_ld < 128 ? limit : nullptr, pidx, plow, next->prefixes(),
      next->count_dev(), reinterpret_cast<int64_t*>(w + o_blk), flags, s)));
  const uint64_t root[2] = {ctx.key().seed().low(), ctx.key().seed().high()};
  DPF_RETURN_IF_ERROR(AbiStatus(dpf_amd::LookupPartialEvaluations(
      next->prefixes(), next->count_dev(), n, prev_tree - start_level,
      from_root ? nullptr : old->prefixes(), from_root ? 0 : old->count(),
      from_root ? nullptr : old->seeds(), from_root ? nullptr : old->cbs(), root,
      ctx.key().party() != 0, from_root, next->seeds(), next->cbs(), flags, s)));
  // the walk of every unique tree index to the previous level's tree level
  // (entries past the count are walked too: unused, and n bounds them)
  if (walk_levels > 0)
    DPF_RETURN_IF_ERROR(AbiStatus(dpf_amd_evaluate_seeds(
        n, walk_levels, walk_levels, next->seeds(), next->cbs(), next->prefixes(), 0,
        w + o_cw + coff[0], reinterpret_cast<const uint8_t*>(w + o_cw + coff[1]),
        reinterpret_cast<const uint8_t*>(w + o_cw + coff[2]), dpf_amd::kPrgKeyLeftLo,
        dpf_amd::kPrgKeyLeftHi, dpf_amd::kPrgKeyRightLo, dpf_amd::kPrgKeyRightHi, next->seeds(),
        next->cbs(), s)));
  // each prefix's own node, then its subtree (as the host path's fused branch)
  DPF_RETURN_IF_ERROR(AbiStatus(dpf_amd::PrefixRoots(
      n, pidx, plow, bbits, n, next->seeds(), next->cbs(), w + o_cw + coff[3],
      reinterpret_cast<const uint8_t*>(w + o_cw + coff[4]),
      reinterpret_cast<const uint8_t*>(w + o_cw + coff[5]), w + o_ps,
      reinterpret_cast<uint8_t*>(w + o_pcb), s)));
  void* final_dev = out_on_device ? out : static_cast<void*>(w + o_out);
  DPF_RETURN_IF_ERROR(ClearPadding(vt, final_dev, total * stride, s));
  DPF_RETURN_IF_ERROR(AbiStatus(dpf_amd_expand_and_correct(
      n, w + o_ps, reinterpret_cast<const uint8_t*>(w + o_pcb), down, w + o_cw + coff[6],
      reinterpret_cast<const uint8_t*>(w + o_cw + coff[7]),
      reinterpret_cast<const uint8_t*>(w + o_cw + coff[8]), &vt,
      reinterpret_cast<const uint64_t*>(corr.data()), ctx.key().party(), cepb, 0, n << down,
      final_dev, s)));
  if (pplaced) DPF_RETURN_IF_ERROR(ThreadUploadRing().ReleasePlaced(pslot, s));
  DPF_RETURN_IF_ERROR(CopyToHost(readback, flags, sizeof(int), s));
  DPF_RETURN_IF_ERROR(CopyToHost(readback + 1, next->count_dev(), sizeof(int64_t), s));
  trace.Mark("launch");
  // The flags first: on a fallback (unsorted, out of range, missing prefix)
  // the caller's host buffer is left untouched and the host path decides.
  DPF_RETURN_IF_ERROR(HipStatus(hipStreamSynchronize(s), "sync"));
  drain.Dismiss();
  trace.Mark("sync");
  if (readback[0] != 0) return OkStatus();  // the host path decides
  if (!out_on_device) DPF_RETURN_IF_ERROR(CopyToHostSync(out, final_dev, total * stride, s));
  trace.Mark("d2h");
  *fallback = false;
  if (update_ctx) {
    next->set_count(readback[1]);
    ctx.set_device_state(std::move(next));
  } else {
    ctx.clear_partial_evaluations();
  }
  ctx.set_partial_evaluations_level(prev_h);
  ctx.set_previous_hierarchy_level(hierarchy_level);
  return OkStatus();
}

}  // namespace

Status DistributedPointFunction::EvaluateUntilRaw(int hierarchy_level,
                                                  Span<const uint128> prefixes,
                                                  EvaluationContext& ctx,
                                                  const dpf_amd_value_type& layout, void* out,
                                                  int64_t out_capacity, int64_t* num_outputs,
                                                  bool out_on_device, void* stream) const {
  const DpfState& st = *state_;
  HostTrace trace("EvaluateUntil");
  DPF_RETURN_IF_ERROR(ValidateEvaluationContext(st, ctx));
  trace.Mark("validate_ctx");
  const int L = num_hierarchy_levels();
  if (hierarchy_level < 0 || hierarchy_level >= L)
    return InvalidArgumentError(
        "`hierarchy_level` must be non-negative and less than parameters_.size()");
  if (hierarchy_level <= ctx.previous_hierarchy_level())
    return InvalidArgumentError(
        "`hierarchy_level` must be greater than `ctx.previous_hierarchy_level`");
  if ((ctx.previous_hierarchy_level() < 0) != prefixes.empty())
    return InvalidArgumentError(
        "`prefixes` must be empty if and only if this is the first call with `ctx`.");
  int previous_log_domain_size = 0;
  const int prev_h = ctx.previous_hierarchy_level();
  // The prefixes' range check (h:735-745): the first prefix out of range is
  // the error, and it precedes every later one.  Large prefix lists are
  // checked inside the de-duplication's first parallel pass instead of a
  // serial loop of their own; every error return before that pass runs the
  // serial check first, so the reported error is the reference's.
  if (!prefixes.empty()) previous_log_domain_size = st.parameters[prev_h].log_domain_size();
  const uint128 prefix_limit = previous_log_domain_size < 128
                                   ? (uint128{1} << previous_log_domain_size)
                                   : uint128{0};  // 0: every prefix is in range
  auto range_check = [&]() -> Status {
    if (prefix_limit == 0) return OkStatus();
    for (uint128 p : prefixes)
      if (p >= prefix_limit)
        return InvalidArgumentError("Index " + dpf_internal::U128ToString(p) +
                                    " out of range for hierarchy level " + std::to_string(prev_h));
    return OkStatus();
  };
  // (a size query, out == nullptr, runs the serial check before it answers
  // unless out_capacity < 0: the two-call protocol's first call, whose
  // evaluation call validates the same prefixes right after — the C++
  // header template and the Python mirror)
  const bool size_unchecked = out == nullptr && out_capacity < 0;
  const bool range_deferred =
      out == nullptr || static_cast<int64_t>(prefixes.size()) >= (int64_t{1} << 14);
  if (!range_deferred) DPF_RETURN_IF_ERROR(range_check());
  auto early = [&](Status e) -> Status {
    if (range_deferred) DPF_RETURN_IF_ERROR(range_check());
    return e;
  };
  trace.Mark("range_check");
  const int log_domain_size = st.parameters[hierarchy_level].log_domain_size();
  if (log_domain_size - previous_log_domain_size > 62)
    return early(InvalidArgumentError(
        "Output size would be larger than 2**62. Please evaluate fewer hierarchy levels at "
        "once."));
  const int64_t num_prefixes = static_cast<int64_t>(prefixes.size());
  const int64_t outputs_per_prefix = int64_t{1} << (log_domain_size - previous_log_domain_size);
  const int64_t total = prefixes.empty() ? outputs_per_prefix : num_prefixes * outputs_per_prefix;
  *num_outputs = total;
  if (out == nullptr) return size_unchecked ? OkStatus() : early(OkStatus());
  if (out_capacity < total) return early(InvalidArgumentError("output buffer too small"));

  const LevelMeta& m = st.levels[hierarchy_level];
  dpf_amd_value_type vt;
  {
    Status e = MergeLayout(m, layout, &vt);
    if (!e.ok()) return early(e);
  }
  std::vector<uint128> corr;
  {
    Status e = CorrectionsFor(st, ctx.key(), hierarchy_level, &corr);
    if (!e.ok()) return early(e);
  }
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ThreadStream();
  trace.Mark("corrections");
  if (!prefixes.empty() && !dpf_amd::HostIncremental() && !dpf_amd::PrefixExpandOff()) {
    bool fallback = true;
    Status e = EvaluateUntilOnDevice(st, hierarchy_level, prefixes, ctx, vt, corr, out,
                                     out_on_device, s, &fallback);
    if (!e.ok()) return early(e);
    if (!fallback) return OkStatus();
    trace.Mark("device_path_declined");
  }

  // Unique tree indices in first-appearance order (h:772-796), and each
  // prefix's gather offset into the expansion (h:877-889).  Sorted prefixes
  // (the usual heavy-hitters candidate list) de-duplicate in two parallel
  // passes (count per range, then write); otherwise a hash map stands in for
  // the reference's btree.
  IncrementalScratch& sc = ThreadScratch();
  // a DMA an earlier call left in flight into the scratch must have landed
  if (sc.done) {
    Status e = HipStatus(hipEventSynchronize(sc.done), "d2h");
    if (!e.ok()) return early(e);
  }
  {
    Status e = sc.Reserve(num_prefixes > 0 ? num_prefixes : 1);
    if (!e.ok()) return early(e);
  }
  uint128* tree_indices = sc.tree;
  std::vector<int64_t>& src = sc.src;
  int64_t num_unique = 0;
  const int stop_level = st.hierarchy_to_tree[hierarchy_level];
  const int start_level = prefixes.empty() ? 0 : st.hierarchy_to_tree[prev_h];
  const int levels = stop_level - start_level;
  const int cepb = 1 << (log_domain_size - stop_level);
  // outputs of one tree index = 2^bbits prefixes x outputs_per_prefix, so
  // every offset below is in range by construction
  const int64_t seg = (int64_t{1} << levels) * cepb;
  // Per-prefix expansion (default; dpf_amd_set_prefix_expand): a prefix p of
  // the previous level is itself a tree node, at depth previous_log_domain_size;
  // when this level's tree level is not above it, expanding p's subtree gives
  // exactly p's outputs_per_prefix outputs, in prefix order.  The roots are
  // the partial evaluations of p's tree index walked down p's last bbits
  // bits, so no sibling subtree is expanded, no staging buffer is written and
  // no gather runs (c3: 2^16 prefixes, half the AES and none of the 256 MiB
  // staging round trip).  `src` then holds each prefix's unique-root index.
  const bool fused = !dpf_amd::PrefixExpandOff() && !prefixes.empty() &&
                     stop_level >= previous_log_domain_size && num_prefixes < (int64_t{1} << 31);
  if (!prefixes.empty()) {
    const int bbits = st.parameters[prev_h].log_domain_size() - st.hierarchy_to_tree[prev_h];
    const uint64_t bmask = (uint64_t{1} << bbits) - 1;  // bbits <= 7 (epb <= 128)
    if (!fused && static_cast<int64_t>(src.size()) < num_prefixes) src.resize(num_prefixes);
    constexpr int kParts = static_cast<int>(HostPool::kWorkers) + 1;
    int64_t count[kParts] = {}, first[kParts] = {};
    bool ordered[kParts], in_range[kParts];
    HostPool& pool = HostPool::Get();
    const uint128 lim = prefix_limit;
    const int parts = pool.ParallelRanges(num_prefixes, 8192, [&](int r, int64_t b, int64_t e) {
      bool ok = true, inr = true;
      int64_t u = 0;
      for (int64_t i = b; i < e; ++i) {
        inr &= lim == 0 || prefixes[i] < lim;
        if (i == 0) {
          ++u;
          continue;
        }
        ok &= prefixes[i - 1] <= prefixes[i];
        u += (prefixes[i] >> bbits) != (prefixes[i - 1] >> bbits);
      }
      ordered[r] = ok;
      in_range[r] = inr;
      count[r] = u;
    });
    bool sorted = true, all_in_range = true;
    for (int r = 0; r < parts; ++r) {
      sorted &= ordered[r];
      all_in_range &= in_range[r];
      first[r] = num_unique;
      num_unique += count[r];
    }
    if (!all_in_range) return range_check();  // the reference's message for the first one
    trace.Mark("dedup_count");
    if (sorted) {
      pool.ParallelRanges(num_prefixes, 8192, [&](int r, int64_t b, int64_t e) {
        int64_t u = first[r];
        for (int64_t i = b; i < e; ++i) {
          const uint128 t = prefixes[i] >> bbits;
          if (i == 0 || t != (prefixes[i - 1] >> bbits)) tree_indices[u++] = t;
          if (fused) {
            sc.pidx[i] = static_cast<int32_t>(u - 1);
            sc.plow[i] = static_cast<uint8_t>(static_cast<uint64_t>(prefixes[i]) & bmask);
          } else {
            src[i] = (u - 1) * seg +
                     static_cast<int64_t>(static_cast<uint64_t>(prefixes[i]) & bmask) *
                         outputs_per_prefix;
          }
        }
      });
    } else {
      num_unique = 0;
      std::unordered_map<uint128, int64_t, U128Hash> inverse;
      inverse.reserve(num_prefixes * 2);
      for (int64_t i = 0; i < num_prefixes; ++i) {
        const uint128 ti = prefixes[i] >> bbits;
        auto it = inverse.emplace(ti, num_unique);
        if (it.second) tree_indices[num_unique++] = ti;
        if (fused) {
          sc.pidx[i] = static_cast<int32_t>(it.first->second);
          sc.plow[i] = static_cast<uint8_t>(static_cast<uint64_t>(prefixes[i]) & bmask);
        } else {
          src[i] = it.first->second * seg +
                   static_cast<int64_t>(static_cast<uint64_t>(prefixes[i]) & bmask) *
                       outputs_per_prefix;
        }
      }
    }
  }

  trace.Mark("checks+dedup");
  // ExpandAndUpdateContext (cc:478-521): roots on the device.
  DeviceBuffer roots;
  void* root_seeds = nullptr;
  uint8_t* root_cb = nullptr;
  PendingContextUpdate pending;
  if (prefixes.empty()) {
    const uint128 seed = MakeUint128(ctx.key().seed().high(), ctx.key().seed().low());
    const uint8_t cb = static_cast<uint8_t>(ctx.key().party() != 0);
    const UploadRing::HostPart parts[2] = {{&seed, 16}, {&cb, 1}};
    size_t off[2];
    const size_t bytes = UploadRing::PackedLayout(parts, 2, off);
    DPF_RETURN_IF_ERROR(roots.Alloc(bytes, s));
    DPF_RETURN_IF_ERROR(ThreadUploadRing().CopyPacked(roots.get(), parts, 2, bytes, off, s));
    root_seeds = roots.as<char>() + off[0];
    root_cb = reinterpret_cast<uint8_t*>(roots.as<char>() + off[1]);
  } else {
    const bool update_ctx = hierarchy_level < L - 1;
    DPF_RETURN_IF_ERROR(ComputePartialEvaluations(
        st, Span<const uint128>(tree_indices, num_unique), prev_h, update_ctx,
        ctx, s, &roots, &root_seeds, &root_cb, &pending));
  }
  trace.Mark("partial_evaluations");
  if (fused) {
    const int prev_tree = st.hierarchy_to_tree[prev_h];
    const int walk = previous_log_domain_size - prev_tree;  // p's bits below its tree index
    const int down = stop_level - previous_log_domain_size;
    const size_t stride = static_cast<size_t>(vt.out_stride);
    CwArrays wc = KeyCws(ctx.key(), prev_tree, previous_log_domain_size);
    CwArrays ec = KeyCws(ctx.key(), previous_log_domain_size, stop_level);
    using Part = UploadRing::HostPart;
    // both correction-word ranges through the upload ring; the per-prefix
    // root index and low bits DMA'd straight from the pinned scratch
    const Part parts[6] = {{wc.seeds.data(), size_t(16) * walk},
                           {wc.ccl.data(), size_t(walk)},
                           {wc.ccr.data(), size_t(walk)},
                           {ec.seeds.data(), size_t(16) * down},
                           {ec.ccl.data(), size_t(down)},
                           {ec.ccr.data(), size_t(down)}};
    size_t off[6];
    const size_t cw_bytes = UploadRing::PackedLayout(parts, 6, off);
    const size_t idx_off = cw_bytes;
    const size_t low_off = idx_off + ((size_t(4) * num_prefixes + 15) & ~size_t{15});
    const size_t seeds_off = low_off + ((size_t(num_prefixes) + 15) & ~size_t{15});
    const size_t cb_off = seeds_off + size_t(16) * num_prefixes;
    DeviceBuffer work, result;
    DPF_RETURN_IF_ERROR(work.Alloc(cb_off + num_prefixes, s));
    char* d = work.as<char>();
    DPF_RETURN_IF_ERROR(ThreadUploadRing().CopyPacked(d, parts, 6, cw_bytes, off, s));
    DPF_RETURN_IF_ERROR(HipStatus(hipMemcpyAsync(d + idx_off, sc.pidx, size_t(4) * num_prefixes,
                                                 hipMemcpyHostToDevice, s),
                                  "upload"));
    DPF_RETURN_IF_ERROR(HipStatus(
        hipMemcpyAsync(d + low_off, sc.plow, size_t(num_prefixes), hipMemcpyHostToDevice, s),
        "upload"));
    void* pseeds = d + seeds_off;
    uint8_t* pcb = reinterpret_cast<uint8_t*>(d + cb_off);
    DPF_RETURN_IF_ERROR(AbiStatus(dpf_amd::PrefixRoots(
        num_prefixes, reinterpret_cast<const int32_t*>(d + idx_off),
        reinterpret_cast<const uint8_t*>(d + low_off), walk, num_unique, root_seeds, root_cb,
        d + off[0], reinterpret_cast<const uint8_t*>(d + off[1]),
        reinterpret_cast<const uint8_t*>(d + off[2]), pseeds, pcb, s)));
    void* final_dev = out;
    if (!out_on_device) {
      DPF_RETURN_IF_ERROR(result.Alloc(total * stride, s));
      final_dev = result.get();
    }
    DPF_RETURN_IF_ERROR(ClearPadding(vt, final_dev, total * stride, s));
    DPF_RETURN_IF_ERROR(AbiStatus(dpf_amd_expand_and_correct(
        num_prefixes, pseeds, pcb, down, d + off[3], reinterpret_cast<const uint8_t*>(d + off[4]),
        reinterpret_cast<const uint8_t*>(d + off[5]), &vt,
        reinterpret_cast<const uint64_t*>(corr.data()), ctx.key().party(), cepb, 0,
        num_prefixes << down, final_dev, s)));
    trace.Mark("prefix_expand_launch");
    // the context rewrite runs while the expansion does
    DPF_RETURN_IF_ERROR(FinishContextUpdate(pending, ctx));
    trace.Mark("ctx_rewrite");
    if (!out_on_device)
      DPF_RETURN_IF_ERROR(CopyToHostSync(out, final_dev, total * stride, s));
    else
      DPF_RETURN_IF_ERROR(HipStatus(hipStreamSynchronize(s), "sync"));
    trace.Mark("copy+sync");
    ctx.set_previous_hierarchy_level(hierarchy_level);
    return OkStatus();
  }
  CwArrays cw = KeyCws(ctx.key(), start_level, stop_level);
  DeviceBuffer cws, ccl, ccr;
  DPF_RETURN_IF_ERROR(cws.Upload(cw.seeds.data(), 16 * levels, s));
  DPF_RETURN_IF_ERROR(ccl.Upload(cw.ccl.data(), levels, s));
  DPF_RETURN_IF_ERROR(ccr.Upload(cw.ccr.data(), levels, s));
  const int64_t num_roots = prefixes.empty() ? 1 : num_unique;
  const int64_t expanded = (num_roots << levels) * cepb;
  const size_t stride = static_cast<size_t>(vt.out_stride);

  DeviceBuffer staging, result, gather_err, src_dev;
  DPF_RETURN_IF_ERROR(sc.Reserve(1));
  int* gather_flag = sc.flag;  // pinned: its copy does not wait for the kernels
  *gather_flag = 0;
  // an error return must not leave the async D2H of gather_flag in flight
  StreamSyncGuard drain(s);
  void* gather_src_dev = nullptr;
  const int64_t* gather_src_host = nullptr;
  void* expand_out = nullptr;
  if (prefixes.empty() && out_on_device) {
    expand_out = out;
  } else {
    DPF_RETURN_IF_ERROR(staging.Alloc(expanded * stride, s));
    expand_out = staging.get();
  }
  DPF_RETURN_IF_ERROR(ClearPadding(vt, expand_out, expanded * stride, s));
  DPF_RETURN_IF_ERROR(AbiStatus(dpf_amd_expand_and_correct(
      num_roots, root_seeds, root_cb, levels, cws.get(), ccl.as<uint8_t>(),
      ccr.as<uint8_t>(), &vt, reinterpret_cast<const uint64_t*>(corr.data()),
      ctx.key().party(), cepb, 0, num_roots << levels, expand_out, s)));

  trace.Mark("expand_launch");
  void* final_dev = expand_out;
  if (!prefixes.empty()) {
    // Per-prefix slices (h:877-889), offsets computed with the dedup above.
    DPF_RETURN_IF_ERROR(src_dev.Upload(src.data(), 8 * num_prefixes, s));
    gather_src_dev = src_dev.get();
    gather_src_host = src.data();
    if (out_on_device) {
      final_dev = out;
    } else {
      DPF_RETURN_IF_ERROR(result.Alloc(total * stride, s));
      final_dev = result.get();
    }
    DPF_RETURN_IF_ERROR(gather_err.Alloc(sizeof(int), s));
    DPF_RETURN_IF_ERROR(HipStatus(hipMemsetAsync(gather_err.get(), 0, sizeof(int), s), "memset"));
    DPF_RETURN_IF_ERROR(AbiStatus(dpf_amd_gather_rows_checked(
        num_prefixes, src_dev.as<int64_t>(), outputs_per_prefix, stride, expand_out, expanded,
        final_dev, gather_err.as<int>(), s)));
    DPF_RETURN_IF_ERROR(CopyToHost(gather_flag, gather_err.get(), sizeof(int), s));
  }
  // the context rewrite runs while the expansion and the gather do
  DPF_RETURN_IF_ERROR(FinishContextUpdate(pending, ctx));
  trace.Mark("ctx_rewrite");
  if (!out_on_device)
    DPF_RETURN_IF_ERROR(CopyToHostSync(out, final_dev, total * stride, s));
  else
    DPF_RETURN_IF_ERROR(HipStatus(hipStreamSynchronize(s), "sync"));
  if (*gather_flag) {  // the offsets were checked on the host: the device copy differs
    std::string detail;
    if (!prefixes.empty()) {
      std::vector<int64_t> back(num_prefixes);
      if (hipMemcpy(back.data(), gather_src_dev, 8 * num_prefixes, hipMemcpyDeviceToHost) ==
          hipSuccess) {
        int64_t bad = 0;
        for (int64_t i = 0; i < num_prefixes; ++i) {
          if (back[i] == gather_src_host[i]) continue;
          if (bad++ < 6)
            detail += " [" + std::to_string(i) + "] " + std::to_string(gather_src_host[i]) +
                      "->" + std::to_string(back[i]);
        }
        detail = " (" + std::to_string(bad) + " of " + std::to_string(num_prefixes) +
                 " differ:" + detail + ")";
      }
    }
    return InternalError("gather offsets corrupted between host and device" + detail);
  }
  drain.Dismiss();  // the stream was drained above
  trace.Mark("gather+copy+sync");
  ctx.set_previous_hierarchy_level(hierarchy_level);
  return OkStatus();
}

Status DistributedPointFunction::EvaluateAtRaw(const DpfKey& key, int hierarchy_level,
                                               Span<const uint128> evaluation_points,
                                               EvaluationContext* ctx,
                                               const dpf_amd_value_type& layout,
                                               void* out) const {
  const DpfState& st = *state_;
  HostTrace trace("EvaluateAt");
  if (ctx != nullptr && &key != &ctx->key())
    return InvalidArgumentError("`key` and `ctx->key()` must refer to the same object");
  if (hierarchy_level < 0) return InvalidArgumentError("`hierarchy_level` must be non-negative");
  if (hierarchy_level >= num_hierarchy_levels())
    return InvalidArgumentError(
        "`hierarchy_level` must be less than the number of parameters passed at construction");
  const int64_t n = static_cast<int64_t>(evaluation_points.size());
  const int log_domain_size = st.parameters[hierarchy_level].log_domain_size();
  uint128 max_point = Uint128Max();
  if (log_domain_size < 128) max_point = (uint128{1} << log_domain_size) - 1;
  for (int64_t i = 0; i < n; ++i)
    if (evaluation_points[i] > max_point)
      return InvalidArgumentError("`evaluation_points[" + std::to_string(i) +
                                  "]` larger than the domain size at hierarchy level " +
                                  std::to_string(hierarchy_level));
  DPF_RETURN_IF_ERROR(ValidateDpfKey(st, key));
  if (ctx != nullptr) DPF_RETURN_IF_ERROR(ValidateEvaluationContext(st, *ctx, true));
  if (n == 0) return OkStatus();
  const LevelMeta& m = st.levels[hierarchy_level];
  dpf_amd_value_type vt;
  DPF_RETURN_IF_ERROR(MergeLayout(m, layout, &vt));
  std::vector<uint128> corr;
  DPF_RETURN_IF_ERROR(CorrectionsFor(st, key, hierarchy_level, &corr));
  hipStream_t s = ThreadStream();
  trace.Mark("validate");

  // Tree indices and element indices of the points (h:1013-1019): for one
  // element per block the points are the tree indices themselves; otherwise
  // they go to per-thread scratch (fresh 16-byte-per-point vectors cost more
  // in page faults than the loop that fills them).
  const int bbits = log_domain_size - m.tree_level;
  struct PointScratch {
    std::vector<uint128> tree;
    std::vector<uint8_t> bidx;
  };
  PointScratch& ps = dpf_internal_host::ThreadRecycled<PointScratch>::Get();
  const uint128* tree = evaluation_points.data();
  const uint8_t* bidx = nullptr;
  if (m.epb > 1) {
    if (static_cast<int64_t>(ps.tree.size()) < n) ps.tree.resize(n);
    if (static_cast<int64_t>(ps.bidx.size()) < n) ps.bidx.resize(n);
    const uint128 bmask = (uint128{1} << bbits) - 1;
    for (int64_t i = 0; i < n; ++i) {
      ps.tree[i] = evaluation_points[i] >> bbits;
      ps.bidx[i] = static_cast<uint8_t>(evaluation_points[i] & bmask);
    }
    tree = ps.tree.data();
    bidx = ps.bidx.data();
  }
  if (ctx == nullptr) {
    // The common call (one EvaluateAt per key): every input in one pinned
    // slot and one DMA, inputs and outputs in one pooled allocation, the
    // key's seed passed once (the batched kernel with one key) — per-call
    // overhead, not the kernel, is what a caller of this API sees.
    const uint128 seed = MakeUint128(key.seed().high(), key.seed().low());
    const uint8_t cb = static_cast<uint8_t>(key.party() != 0);
    const int levels = m.tree_level;
    CwArrays cw = KeyCws(key, 0, levels);
    using Part = UploadRing::HostPart;
    // The points (and element indices) stay in a pinned slot the kernel reads
    // in place (zero-copy: each point's 16 bytes cross PCIe once, while the
    // block fills its tables); the key's seed and correction words, read at
    // every level, go to device memory.
    const Part pts[2] = {{tree, size_t(16) * n}, {bidx, m.epb > 1 ? size_t(n) : 0}};
    size_t poff[2];
    const size_t pts_bytes = UploadRing::PackedLayout(pts, 2, poff);
    bool staged = false;
    int slot = -1;
    const char* pdev = nullptr;
    DPF_RETURN_IF_ERROR(ThreadUploadRing().Stage(pts, 2, pts_bytes, poff, &staged, &slot, &pdev));
    const Part parts[6] = {{&seed, 16},
                           {cw.seeds.data(), size_t(16) * levels},
                           {cw.ccl.data(), size_t(levels)},
                           {cw.ccr.data(), size_t(levels)},
                           {&cb, 1},
                           {staged ? nullptr : tree, staged ? 0 : size_t(16) * n}};
    size_t off[6];
    const size_t in_bytes = UploadRing::PackedLayout(parts, 6, off);
    const size_t bi_off = in_bytes;
    const size_t out_off = bi_off + (m.epb > 1 && !staged ? ((size_t(n) + 15) & ~size_t{15}) : 0);
    DeviceBuffer buf;
    trace.Mark("prepare");
    const size_t out_bytes = size_t(n) * vt.out_stride;
    const bool host_out = out_bytes <= dpf_internal_host::HostOutMax();
    void* hout = nullptr;
    void* kout = nullptr;
    if (host_out)
      DPF_RETURN_IF_ERROR(
          dpf_internal_host::ThreadRecycled<dpf_internal_host::PinnedOut>::Get().Get(
              out_bytes, &hout, &kout));
    // with the points staged, the key's part is written by the host into
    // fine-grained device memory (no copy kernel in front of the walk)
    bool placed = false;
    int pslot = -1;
    char* pd = nullptr;
    if (staged)
      DPF_RETURN_IF_ERROR(ThreadUploadRing().Place(parts, 6, in_bytes, off, &placed, &pslot, &pd));
    const size_t dev_bytes = (placed ? 0 : out_off) + (host_out ? 0 : out_bytes);
    if (dev_bytes) DPF_RETURN_IF_ERROR(buf.Alloc(dev_bytes, s));
    char* d = placed ? pd : buf.as<char>();
    if (!host_out) kout = buf.as<char>() + (placed ? 0 : out_off);
    if (!placed) DPF_RETURN_IF_ERROR(ThreadUploadRing().CopyPacked(d, parts, 6, in_bytes, off, s));
    if (m.epb > 1 && !staged) DPF_RETURN_IF_ERROR(ThreadUploadRing().Copy(d + bi_off, bidx, n, s));
    if (host_out) {
      if (dpf_internal_host::HasPadding(vt)) std::memset(hout, 0, out_bytes);
    } else {
      DPF_RETURN_IF_ERROR(ClearPadding(vt, kout, out_bytes, s));
    }
    trace.Mark("alloc+upload");
    const void* paths = staged ? pdev + poff[0] : d + off[5];
    const uint8_t* bdev = m.epb > 1 ? reinterpret_cast<const uint8_t*>(
                                          staged ? pdev + poff[1] : d + bi_off)
                                    : nullptr;
    const Status launched = AbiStatus(dpf_amd_evaluate_points_batched(
        1, n, d + off[0], reinterpret_cast<const uint8_t*>(d + off[4]), paths, 0, levels,
        d + off[1], reinterpret_cast<const uint8_t*>(d + off[2]),
        reinterpret_cast<const uint8_t*>(d + off[3]), &vt, bdev, nullptr, key.party(), nullptr,
        reinterpret_cast<const uint64_t*>(corr.data()), kout, s));
    if (staged) DPF_RETURN_IF_ERROR(ThreadUploadRing().Release(slot, s));
    if (placed) DPF_RETURN_IF_ERROR(ThreadUploadRing().ReleasePlaced(pslot, s));
    DPF_RETURN_IF_ERROR(launched);
    trace.Mark("launch");
    if (host_out) {
      DPF_RETURN_IF_ERROR(HipStatus(hipStreamSynchronize(s), "sync"));
      trace.Mark("sync");
      std::memcpy(out, hout, out_bytes);
      trace.Mark("copy_out");
    } else {
      DPF_RETURN_IF_ERROR(CopyToHostSync(out, kout, out_bytes, s));
      trace.Mark("d2h+sync");
    }
    return OkStatus();
  }
  // With a context: the stored partial evaluations are walked to this
  // level's tree level first (EvaluateAt h:349-378 with ctx).
  DeviceBuffer pe, paths, bi, cws, ccl, ccr, dout;
  void* seeds = nullptr;
  uint8_t* cbs = nullptr;
  DPF_RETURN_IF_ERROR(ComputePartialEvaluations(st, Span<const uint128>(tree, n),
                                                hierarchy_level, true, *ctx, s, &pe, &seeds,
                                                &cbs));
  const int start_level = m.tree_level;
  const int levels = m.tree_level - start_level;
  CwArrays cw = KeyCws(key, start_level, m.tree_level);
  DPF_RETURN_IF_ERROR(paths.Upload(tree, 16 * n, s));
  if (bidx) DPF_RETURN_IF_ERROR(bi.Upload(bidx, n, s));
  DPF_RETURN_IF_ERROR(cws.Upload(cw.seeds.data(), 16 * levels, s));
  DPF_RETURN_IF_ERROR(ccl.Upload(cw.ccl.data(), levels, s));
  DPF_RETURN_IF_ERROR(ccr.Upload(cw.ccr.data(), levels, s));
  DPF_RETURN_IF_ERROR(dout.Alloc(n * vt.out_stride, s));
  DPF_RETURN_IF_ERROR(ClearPadding(vt, dout.get(), n * vt.out_stride, s));
  DPF_RETURN_IF_ERROR(AbiStatus(dpf_amd_evaluate_points(
      n, seeds, cbs, paths.get(), 0, levels, levels, cws.get(),
      ccl.as<uint8_t>(), ccr.as<uint8_t>(), &vt, bidx ? bi.as<uint8_t>() : nullptr, nullptr,
      key.party(), nullptr, reinterpret_cast<const uint64_t*>(corr.data()), dout.get(), nullptr,
      nullptr, s)));
  DPF_RETURN_IF_ERROR(CopyToHostSync(out, dout.get(), n * vt.out_stride, s));
  if (ctx) ctx->set_previous_hierarchy_level(hierarchy_level);
  return OkStatus();
}

Status DistributedPointFunction::EvaluateAndApplyRaw(Span<const DpfKey* const> keys,
                                                     Span<const uint128> evaluation_points,
                                                     int rightshift,
                                                     const dpf_amd_value_type& layout,
                                                     void* out, int* levels_done,
                                                     bool (*on_level)(void*, int),
                                                     void* user) const {
  const DpfState& st = *state_;
  HostTrace trace("EvaluateAndApply");
  if (evaluation_points.size() != keys.size())
    return InvalidArgumentError("`keys.size()` != `evaluation_points.size()`");
  const int64_t n = static_cast<int64_t>(keys.size());
  const int H = num_hierarchy_levels();
  *levels_done = 0;
  if (n == 0) return OkStatus();
  // The reference walks one seed per (key, point) pair with per-seed
  // correction words (h:1101-1134, evaluate_prg_hwy.cc:264-301).  Callers
  // pass the same key object for many points (a DCF batch, 64 keys x 2^14
  // points at c2), so keys are deduplicated by address: every distinct key
  // is validated and uploaded once, and each point carries its key's index.
  std::vector<int32_t> kidx(n);
  std::vector<const DpfKey*> uniq;
  {
    std::unordered_map<const DpfKey*, int32_t> seen;
    const DpfKey* prev = nullptr;
    int32_t prev_i = -1;
    for (int64_t i = 0; i < n; ++i) {
      const DpfKey* k = keys[i];
      if (k != prev) {
        auto ins = seen.emplace(k, static_cast<int32_t>(uniq.size()));
        if (ins.second) uniq.push_back(k);
        prev = k;
        prev_i = ins.first->second;
      }
      kidx[i] = prev_i;
    }
  }
  for (const DpfKey* k : uniq) DPF_RETURN_IF_ERROR(ValidateDpfKey(st, *k));
  const int64_t U = static_cast<int64_t>(uniq.size());
  trace.Mark("dedup+validate");
  hipStream_t s = ThreadStream();
  std::vector<uint128> sv(U);
  std::vector<uint8_t> cv(U);
  std::vector<int8_t> party(U);
  for (int64_t k = 0; k < U; ++k) {
    sv[k] = MakeUint128(uniq[k]->seed().high(), uniq[k]->seed().low());
    cv[k] = static_cast<uint8_t>(uniq[k]->party() != 0);
    party[k] = static_cast<int8_t>(uniq[k]->party());
  }
  // Per-point inputs: the paths and key indices (the walk state lives in
  // `state` between hierarchy levels, one seed + control bit per point).
  DeviceBuffer key_seeds, key_cbs, paths, kix, pty, state, state_cb, dout;
  DPF_RETURN_IF_ERROR(key_seeds.Upload(sv.data(), 16 * U, s));
  DPF_RETURN_IF_ERROR(key_cbs.Upload(cv.data(), U, s));
  DPF_RETURN_IF_ERROR(pty.Upload(party.data(), U, s));
  DPF_RETURN_IF_ERROR(paths.Upload(evaluation_points.data(), 16 * n, s));
  DPF_RETURN_IF_ERROR(kix.Upload(kidx.data(), 4 * n, s));
  if (H > 1) {
    DPF_RETURN_IF_ERROR(state.Alloc(16 * n, s));
    DPF_RETURN_IF_ERROR(state_cb.Alloc(n, s));
  }
  // Output buffer of the widest level (levels are evaluated one at a time).
  size_t max_stride = 0;
  for (int h = 0; h < H; ++h) {
    dpf_amd_value_type vt;
    DPF_RETURN_IF_ERROR(MergeLayout(st.levels[h], layout, &vt));
    max_stride = std::max<size_t>(max_stride, vt.out_stride);
  }
  DPF_RETURN_IF_ERROR(dout.Alloc(n * max_stride, s));
  trace.Mark("upload");
  const int last_ld = st.parameters.back().log_domain_size();
  int start_level = 0, stop_level = st.hierarchy_to_tree[0];
  char* host_out = static_cast<char*>(out);
  std::vector<uint128> tmp;
  std::vector<uint8_t> bidx;
  for (int h = 0; h < H; ++h) {
    if (h > 0) {
      start_level = stop_level;
      stop_level = st.hierarchy_to_tree[h];
    }
    const LevelMeta& m = st.levels[h];
    dpf_amd_value_type vt;
    DPF_RETURN_IF_ERROR(MergeLayout(m, layout, &vt));
    const int domain_rs = rightshift + last_ld - m.log_domain;
    const int tree_rs = rightshift + last_ld - m.tree_level;
    const int levels = stop_level - start_level;
    // correction words [key][level] and value corrections [key]
    std::vector<uint128> cws(static_cast<size_t>(levels) * U);
    std::vector<uint8_t> ccl(cws.size()), ccr(cws.size());
    const int per = m.epb * static_cast<int>(m.scalars.size());
    std::vector<uint128> corr(static_cast<size_t>(per) * U);
    for (int64_t k = 0; k < U; ++k) {
      for (int l = 0; l < levels; ++l) {
        const CorrectionWord& cw = uniq[k]->correction_words(start_level + l);
        cws[k * levels + l] = MakeUint128(cw.seed().high(), cw.seed().low());
        ccl[k * levels + l] = cw.control_left();
        ccr[k * levels + l] = cw.control_right();
      }
      DPF_RETURN_IF_ERROR(CorrectionsFor(st, *uniq[k], h, &tmp));
      std::copy(tmp.begin(), tmp.end(), corr.begin() + k * per);
    }
    const bool want_bidx = m.epb > 1 && domain_rs < 128;
    if (want_bidx) {
      const int bbits = m.log_domain - m.tree_level;
      const uint128 bmask = (uint128{1} << bbits) - 1;
      bidx.assign(n, 0);
      for (int64_t j = 0; j < n; ++j)
        bidx[j] = static_cast<uint8_t>((evaluation_points[j] >> domain_rs) & bmask);
    }
    using Part = UploadRing::HostPart;
    const Part parts[4] = {{cws.data(), 16 * cws.size()},
                           {ccl.data(), ccl.size()},
                           {ccr.data(), ccr.size()},
                           {corr.data(), 16 * corr.size()}};
    size_t off[4];
    const size_t in_bytes = UploadRing::PackedLayout(parts, 4, off);
    DeviceBuffer lvl, dbi;
    // host-written into fine-grained device memory where allowed, else one copy
    bool placed = false;
    int pslot = -1;
    char* d = nullptr;
    DPF_RETURN_IF_ERROR(ThreadUploadRing().Place(parts, 4, in_bytes, off, &placed, &pslot, &d));
    if (!placed) {
      DPF_RETURN_IF_ERROR(lvl.Alloc(in_bytes, s));
      d = lvl.as<char>();
      DPF_RETURN_IF_ERROR(ThreadUploadRing().CopyPacked(d, parts, 4, in_bytes, off, s));
    }
    if (want_bidx) DPF_RETURN_IF_ERROR(dbi.Upload(bidx.data(), n, s));
    DPF_RETURN_IF_ERROR(ClearPadding(vt, dout.get(), n * vt.out_stride, s));
    const bool first = h == 0;
    DPF_RETURN_IF_ERROR(AbiStatus(dpf_amd::EvaluatePointsIndexed(
        n, kix.as<int32_t>(), U, first ? key_seeds.get() : state.get(),
        first ? key_cbs.as<uint8_t>() : state_cb.as<uint8_t>(), first, paths.get(),
        std::min(tree_rs, 255), levels, d + off[0], reinterpret_cast<const uint8_t*>(d + off[1]),
        reinterpret_cast<const uint8_t*>(d + off[2]), &vt,
        want_bidx ? dbi.as<uint8_t>() : nullptr, pty.as<int8_t>(), d + off[3], dout.get(),
        h + 1 < H ? state.get() : nullptr, h + 1 < H ? state_cb.as<uint8_t>() : nullptr, s)));
    if (placed) DPF_RETURN_IF_ERROR(ThreadUploadRing().ReleasePlaced(pslot, s));
    DPF_RETURN_IF_ERROR(
        CopyToHostSync(host_out + h * n * vt.out_stride, dout.get(), n * vt.out_stride, s));
    trace.Mark("level");
    *levels_done = h + 1;
    // h:1190-1196: stop as soon as `op` returns false (the remaining levels
    // are never evaluated)
    if (on_level && !on_level(user, h)) break;
  }
  return OkStatus();
}

Status DistributedPointFunction::ExpandLeavesOnDevice(const DpfKey& key, int64_t leaf_begin,
                                                      int64_t leaf_end,
                                                      const dpf_amd_value_type& layout,
                                                      void* out, void* stream) const {
  const DpfState& st = *state_;
  DPF_RETURN_IF_ERROR(ValidateDpfKey(st, key));
  const int h = num_hierarchy_levels() - 1;
  const LevelMeta& m = st.levels[h];
  if (m.tree_level > 62) return InvalidArgumentError("domain too large to expand fully");
  dpf_amd_value_type vt;
  DPF_RETURN_IF_ERROR(MergeLayout(m, layout, &vt));
  std::vector<uint128> corr;
  DPF_RETURN_IF_ERROR(CorrectionsFor(st, key, h, &corr));
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ThreadStream();
  const uint128 seed = MakeUint128(key.seed().high(), key.seed().low());
  const uint8_t cb = static_cast<uint8_t>(key.party() != 0);
  const int L = m.tree_level;
  CwArrays cw = KeyCws(key, 0, L);
  // the key's inputs in one pinned slot and one copy (a PIR request's
  // selection expansion sits on the critical path in front of the scan)
  using Part = UploadRing::HostPart;
  const Part parts[5] = {{&seed, 16},
                         {&cb, 1},
                         {cw.seeds.data(), size_t(16) * L},
                         {cw.ccl.data(), size_t(L)},
                         {cw.ccr.data(), size_t(L)}};
  size_t off[5];
  const size_t bytes = UploadRing::PackedLayout(parts, 5, off);
  // written by the host into fine-grained device memory where the device
  // allows it (no copy kernel in front of the expansion), else one copy
  bool placed = false;
  int pslot = -1;
  char* d = nullptr;
  DPF_RETURN_IF_ERROR(ThreadUploadRing().Place(parts, 5, bytes, off, &placed, &pslot, &d));
  DeviceBuffer in;
  if (!placed) {
    DPF_RETURN_IF_ERROR(in.Alloc(bytes, s));
    d = in.as<char>();
    DPF_RETURN_IF_ERROR(ThreadUploadRing().CopyPacked(d, parts, 5, bytes, off, s));
  }
  const int cepb = 1 << (m.log_domain - L);
  const Status launched = AbiStatus(dpf_amd_expand_and_correct(
      1, d + off[0], reinterpret_cast<const uint8_t*>(d + off[1]), L, d + off[2],
      reinterpret_cast<const uint8_t*>(d + off[3]), reinterpret_cast<const uint8_t*>(d + off[4]),
      &vt, reinterpret_cast<const uint64_t*>(corr.data()), key.party(), cepb, leaf_begin,
      leaf_end, out, s));
  if (placed) DPF_RETURN_IF_ERROR(ThreadUploadRing().ReleasePlaced(pslot, s));
  return launched;
}


Status DistributedPointFunction::ExpandLeavesOnDevices(const DpfKey& key, Span<const int> devices,
                                                       Span<const int64_t> leaf_begin,
                                                       Span<const int64_t> leaf_end,
                                                       Span<void* const> outs,
                                                       const dpf_amd_value_type& layout) const {
  const size_t n = devices.size();
  if (leaf_begin.size() != n || leaf_end.size() != n || outs.size() != n)
    return InvalidArgumentError("`devices`, `leaf_begin`, `leaf_end` and `outs` must have the "
                                "same size");
  DPF_RETURN_IF_ERROR(ValidateDpfKey(*state_, key));
  for (int d : devices) DPF_RETURN_IF_ERROR(dpf_internal_host::CheckDevice(d));
  // Issue every device's launch first (each on this thread's stream for that
  // device), then wait for all of them.
  Status st = OkStatus();
  std::vector<hipStream_t> streams(n, nullptr);
  for (size_t i = 0; i < n && st.ok(); ++i) {
    dpf_internal_host::DeviceGuard g(devices[i]);
    streams[i] = dpf_internal_host::ThreadStreamOn(devices[i]);
    if (streams[i] == nullptr) {
      st = InternalError("no stream on device " + std::to_string(devices[i]));
      break;
    }
    st = ExpandLeavesOnDevice(key, leaf_begin[i], leaf_end[i], layout, outs[i], streams[i]);
  }
  for (size_t i = 0; i < n; ++i) {
    if (streams[i] == nullptr) continue;
    dpf_internal_host::DeviceGuard g(devices[i]);
    Status w = HipStatus(hipStreamSynchronize(streams[i]), "sync");
    if (st.ok()) st = w;
  }
  return st;
}

Status DistributedPointFunction::ExpandLeavesOnDeviceBatched(Span<const DpfKey* const> keys,
                                                             int64_t num_leaves,
                                                             const dpf_amd_value_type& layout,
                                                             void* out, void* stream) const {
  return ExpandLeavesOnDeviceBatched(keys, 0, num_leaves, layout, out, stream);
}

Status DistributedPointFunction::ExpandLeavesOnDeviceBatched(Span<const DpfKey* const> keys,
                                                             int64_t leaf_begin, int64_t leaf_end,
                                                             const dpf_amd_value_type& layout,
                                                             void* out, void* stream) const {
  const DpfState& st = *state_;
  const int64_t q = static_cast<int64_t>(keys.size());
  const int64_t num_leaves = leaf_end - leaf_begin;
  if (q == 0 || num_leaves <= 0) return OkStatus();
  for (const DpfKey* k : keys) DPF_RETURN_IF_ERROR(ValidateDpfKey(st, *k));
  const int h = num_hierarchy_levels() - 1;
  const LevelMeta& m = st.levels[h];
  if (m.tree_level > 62) return InvalidArgumentError("domain too large to expand fully");
  if (leaf_begin < 0 || leaf_end > (int64_t{1} << m.tree_level))
    return InvalidArgumentError("leaf range out of bounds");
  dpf_amd_value_type vt;
  DPF_RETURN_IF_ERROR(MergeLayout(m, layout, &vt));
  const int L = m.tree_level;
  const int cepb = 1 << (m.log_domain - L);
  // A per-leaf walk costs L + 1 AES against ~2 for the tree expansion, but
  // the whole batch is one upload and one launch: the better trade while the
  // batch is a few million AES (cuckoo-table selections, small databases).
  const bool walk = q > 1 && cepb == 1 &&
                    static_cast<double>(q) * num_leaves * (L + 1) <= static_cast<double>(1 << 25);
  char* o = static_cast<char*>(out);
  const bool single_direct = vt.directly_convertible && vt.num_scalars == 1 &&
                             vt.scalars[0].in_offset == 0 && vt.scalars[0].out_offset == 0 &&
                             vt.out_stride == vt.scalars[0].bytes && vt.blocks_needed == 1 &&
                             vt.elements_per_block * vt.scalars[0].bytes == 16;
  if (!walk && q > 1 && single_direct && L >= 11 && num_leaves < (int64_t{1} << 25)) {
    // One launch for every key (KExpandCoop, batched): the tree of each key
    // is computed once per 2^10-2^11-leaf block, all keys' blocks in one grid
    // (a 64-key c4 request: one launch instead of 64 small ones).
    const int64_t off_cw = 16 * q, off_corr = off_cw + 16 * q * L, off_cb = off_corr + 16 * q;
    const int64_t off_party = off_cb + q, off_ccl = off_party + q, off_ccr = off_ccl + q * L;
    std::vector<char> host(off_ccr + q * L + 16, 0);
    std::vector<uint128> corr;
    for (int64_t k = 0; k < q; ++k) {
      const DpfKey& key = *keys[k];
      const uint128 seed = MakeUint128(key.seed().high(), key.seed().low());
      memcpy(host.data() + 16 * k, &seed, 16);
      const CwArrays cw = KeyCws(key, 0, L);
      memcpy(host.data() + off_cw + 16 * k * L, cw.seeds.data(), 16 * L);
      memcpy(host.data() + off_ccl + k * L, cw.ccl.data(), L);
      memcpy(host.data() + off_ccr + k * L, cw.ccr.data(), L);
      DPF_RETURN_IF_ERROR(CorrectionsFor(st, key, h, &corr));
      uint64_t packed[2];
      DPF_RETURN_IF_ERROR(AbiStatus(dpf_amd::PackedCorrection(
          vt, reinterpret_cast<const uint64_t*>(corr.data()), cepb, packed)));
      memcpy(host.data() + off_corr + 16 * k, packed, 16);
      host[off_cb + k] = static_cast<char>(key.party() != 0);
      host[off_party + k] = static_cast<char>(key.party());
    }
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ThreadStream();
    // host-written into fine-grained device memory where allowed (as in
    // ExpandLeavesOnDevice), else one upload
    const UploadRing::HostPart part{host.data(), host.size()};
    bool placed = false;
    int pslot = -1;
    char* d = nullptr;
    DPF_RETURN_IF_ERROR(ThreadUploadRing().Place(&part, 1, host.size(), nullptr, &placed, &pslot, &d));
    DeviceBuffer dev;
    if (!placed) {
      DPF_RETURN_IF_ERROR(dev.Upload(host.data(), host.size(), s));
      d = dev.as<char>();
    }
    const Status launched = AbiStatus(dpf_amd::ExpandBatched(
        q, d, reinterpret_cast<const uint8_t*>(d + off_cb), L, d + off_cw,
        reinterpret_cast<const uint8_t*>(d + off_ccl), reinterpret_cast<const uint8_t*>(d + off_ccr),
        &vt, d + off_corr, reinterpret_cast<const int8_t*>(d + off_party), cepb, leaf_begin,
        leaf_end, out, s));
    if (placed) DPF_RETURN_IF_ERROR(ThreadUploadRing().ReleasePlaced(pslot, s));
    return launched;
  }
  if (!walk) {
    for (int64_t i = 0; i < q; ++i)
      DPF_RETURN_IF_ERROR(ExpandLeavesOnDevice(*keys[i], leaf_begin, leaf_end, layout,
                                               o + i * num_leaves * cepb * vt.out_stride, stream));
    return OkStatus();
  }
  std::vector<uint128> corr;
  DPF_RETURN_IF_ERROR(CorrectionsFor(st, *keys[0], h, &corr));
  const int64_t per = static_cast<int64_t>(corr.size());
  // One host image of every key's inputs: seeds [q] | correction seeds
  // [q][L] | value corrections [q][per] (16-byte words), then control bits
  // [q], parties [q], ccl [q][L], ccr [q][L].
  const int64_t off_cw = 16 * q, off_corr = off_cw + 16 * q * L;
  const int64_t off_cb = off_corr + 16 * q * per, off_party = off_cb + q;
  const int64_t off_ccl = off_party + q, off_ccr = off_ccl + q * L;
  std::vector<char> host(off_ccr + q * L + 16, 0);
  for (int64_t k = 0; k < q; ++k) {
    const DpfKey& key = *keys[k];
    const uint128 seed = MakeUint128(key.seed().high(), key.seed().low());
    memcpy(host.data() + 16 * k, &seed, 16);
    const CwArrays cw = KeyCws(key, 0, L);
    if (L > 0) {
      memcpy(host.data() + off_cw + 16 * k * L, cw.seeds.data(), 16 * L);
      memcpy(host.data() + off_ccl + k * L, cw.ccl.data(), L);
      memcpy(host.data() + off_ccr + k * L, cw.ccr.data(), L);
    }
    if (k > 0) DPF_RETURN_IF_ERROR(CorrectionsFor(st, key, h, &corr));
    if (static_cast<int64_t>(corr.size()) != per) return InternalError("correction size mismatch");
    memcpy(host.data() + off_corr + 16 * k * per, corr.data(), 16 * per);
    host[off_cb + k] = static_cast<char>(key.party() != 0);
    host[off_party + k] = static_cast<char>(key.party());
  }
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ThreadStream();
  DeviceBuffer dev;
  DPF_RETURN_IF_ERROR(dev.Upload(host.data(), host.size(), s));
  char* d = dev.as<char>();
  return AbiStatus(dpf_amd::EvaluatePointsBatchedRange(
      q, leaf_begin, num_leaves, d, reinterpret_cast<const uint8_t*>(d + off_cb), L, d + off_cw,
      reinterpret_cast<const uint8_t*>(d + off_ccl), reinterpret_cast<const uint8_t*>(d + off_ccr),
      &vt, reinterpret_cast<const int8_t*>(d + off_party), d + off_corr, out, s));
}

}  // namespace distributed_point_functions
