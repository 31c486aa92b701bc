// value_types.h — DPF output value types with the semantics of the
// reference's dpf/xor_wrapper.h, dpf/tuple.h and dpf/int_mod_n.h, and the
// type traits (ToValueType / ToValue / FromValue / host layout) that the
// header templates of DistributedPointFunction need
// (dpf/internal/value_type_helpers.h:59-516).
#ifndef DPF_AMD_VALUE_TYPES_H_
#define DPF_AMD_VALUE_TYPES_H_

#include <stddef.h>
#include <stdint.h>

#include <initializer_list>
#include <string>
#include <tuple>
#include <type_traits>
#include <utility>
#include <vector>

#include "dpf_amd.h"
#include "dpf_amd/protos.h"
#include "dpf_amd/status.h"

namespace distributed_point_functions {

// Minimal absl::Span replacement (read-only view).
template <typename T>
class Span {
 public:
  Span() = default;
  Span(T* data, size_t size) : data_(data), size_(size) {}
  template <typename A>
  Span(const std::vector<std::remove_const_t<T>, A>& v)  // NOLINT
      : data_(v.data()), size_(v.size()) {}
  template <typename A>
  Span(std::vector<std::remove_const_t<T>, A>& v)  // NOLINT
      : data_(v.data()), size_(v.size()) {}
  Span(std::initializer_list<std::remove_const_t<T>> l)  // NOLINT
      : data_(l.begin()), size_(l.size()) {}
  T* data() const { return data_; }
  size_t size() const { return size_; }
  bool empty() const { return size_ == 0; }
  T& operator[](size_t i) const { return data_[i]; }
  T* begin() const { return data_; }
  T* end() const { return data_ + size_; }
  Span subspan(size_t pos, size_t len) const { return Span(data_ + pos, len); }

 private:
  T* data_ = nullptr;
  size_t size_ = 0;
};

template <typename T>
Span<const T> MakeConstSpan(const T* p, size_t n) {
  return Span<const T>(p, n);
}
template <typename T>
Span<const T> MakeConstSpan(const std::vector<T>& v) {
  return Span<const T>(v.data(), v.size());
}

// XorWrapper<T> (xor_wrapper.h:25-83): + and - are XOR, -a == a.
template <typename T>
class XorWrapper {
 public:
  using WrappedType = T;
  constexpr XorWrapper() : wrapped_{} {}
  explicit constexpr XorWrapper(T wrapped) : wrapped_(wrapped) {}
  constexpr XorWrapper& operator+=(const XorWrapper& r) {
    wrapped_ ^= r.wrapped_;
    return *this;
  }
  constexpr XorWrapper& operator-=(const XorWrapper& r) {
    wrapped_ ^= r.wrapped_;
    return *this;
  }
  constexpr T& value() { return wrapped_; }
  constexpr const T& value() const { return wrapped_; }

 private:
  T wrapped_;
};
template <typename T>
constexpr XorWrapper<T> operator+(XorWrapper<T> a, const XorWrapper<T>& b) {
  return a += b;
}
template <typename T>
constexpr XorWrapper<T> operator-(XorWrapper<T> a, const XorWrapper<T>& b) {
  return a -= b;
}
template <typename T>
constexpr XorWrapper<T> operator-(const XorWrapper<T>& a) {
  return a;
}
template <typename T>
constexpr bool operator==(const XorWrapper<T>& a, const XorWrapper<T>& b) {
  return a.value() == b.value();
}
template <typename T>
constexpr bool operator!=(const XorWrapper<T>& a, const XorWrapper<T>& b) {
  return !(a == b);
}

// Tuple<T...> (tuple.h:29-118): element-wise +, -, unary -.
template <typename... T>
class Tuple {
 public:
  using Base = std::tuple<T...>;
  Tuple() {}
  Tuple(T... elements) : value_(elements...) {}  // NOLINT
  explicit Tuple(Base t) : value_(std::move(t)) {}
  Base& value() { return value_; }
  const Base& value() const { return value_; }

 private:
  Base value_;
};

namespace dpf_internal {
template <typename... T, size_t... I>
constexpr Tuple<T...> TupleAdd(const Tuple<T...>& a, const Tuple<T...>& b,
                               std::index_sequence<I...>) {
  return Tuple<T...>{(std::get<I>(a.value()) + std::get<I>(b.value()))...};
}
template <typename... T, size_t... I>
constexpr Tuple<T...> TupleNeg(const Tuple<T...>& a, std::index_sequence<I...>) {
  return Tuple<T...>{T(-std::get<I>(a.value()))...};
}
}  // namespace dpf_internal

template <typename... T>
constexpr Tuple<T...> operator+(const Tuple<T...>& a, const Tuple<T...>& b) {
  return dpf_internal::TupleAdd(a, b, std::make_index_sequence<sizeof...(T)>{});
}
template <typename... T>
constexpr Tuple<T...>& operator+=(Tuple<T...>& a, const Tuple<T...>& b) {
  return a = a + b;
}
template <typename... T>
constexpr Tuple<T...> operator-(const Tuple<T...>& a) {
  return dpf_internal::TupleNeg(a, std::make_index_sequence<sizeof...(T)>{});
}
template <typename... T>
constexpr Tuple<T...> operator-(const Tuple<T...>& a, const Tuple<T...>& b) {
  return a + (-b);
}
template <typename... T>
constexpr Tuple<T...>& operator-=(Tuple<T...>& a, const Tuple<T...>& b) {
  return a = a - b;
}
template <typename... T>
constexpr bool operator==(const Tuple<T...>& a, const Tuple<T...>& b) {
  return a.value() == b.value();
}
template <typename... T>
constexpr bool operator!=(const Tuple<T...>& a, const Tuple<T...>& b) {
  return a.value() != b.value();
}

namespace dpf_internal {

// IntModNImpl (int_mod_n.h:87-250).
template <typename BaseInteger, typename ModulusType, ModulusType kModulus>
class IntModNImpl {
 public:
  using Base = BaseInteger;
  constexpr IntModNImpl() : value_(0) {}
  explicit constexpr IntModNImpl(BaseInteger v) : value_(v % kModulus) {}
  constexpr IntModNImpl& operator=(const BaseInteger& a) {
    value_ = a % kModulus;
    return *this;
  }
  constexpr IntModNImpl& operator+=(const IntModNImpl& a) {
    Sub(static_cast<BaseInteger>(kModulus - a.value_));
    return *this;
  }
  constexpr IntModNImpl& operator-=(const IntModNImpl& a) {
    Sub(a.value_);
    return *this;
  }
  constexpr BaseInteger value() const { return value_; }
  static constexpr BaseInteger modulus() { return kModulus; }

 private:
  constexpr void Sub(const BaseInteger& a) {
    if (value_ >= a)
      value_ -= a;
    else
      value_ = static_cast<BaseInteger>(kModulus - a + value_);
  }
  BaseInteger value_;
};

template <typename B, typename M, M k>
constexpr IntModNImpl<B, M, k> operator+(IntModNImpl<B, M, k> a, const IntModNImpl<B, M, k>& b) {
  return a += b;
}
template <typename B, typename M, M k>
constexpr IntModNImpl<B, M, k> operator-(IntModNImpl<B, M, k> a, const IntModNImpl<B, M, k>& b) {
  return a -= b;
}
template <typename B, typename M, M k>
constexpr IntModNImpl<B, M, k> operator-(IntModNImpl<B, M, k> a) {
  IntModNImpl<B, M, k> r(B{0});
  r -= a;
  return r;
}
template <typename B, typename M, M k>
constexpr bool operator==(const IntModNImpl<B, M, k>& a, const IntModNImpl<B, M, k>& b) {
  return a.value() == b.value();
}
template <typename B, typename M, M k>
constexpr bool operator!=(const IntModNImpl<B, M, k>& a, const IntModNImpl<B, M, k>& b) {
  return a.value() != b.value();
}

}  // namespace dpf_internal

template <typename BaseInteger, unsigned __int128 kModulus>
using IntModN = dpf_internal::IntModNImpl<BaseInteger, unsigned __int128, kModulus>;

namespace dpf_internal {

Value::Integer Uint128ToValueInteger(uint128 v);
StatusOr<uint128> ValueIntegerToUint128(const Value::Integer& in);

// One flattened scalar of a host-layout T.
struct HostScalar {
  int kind;   // DPF_AMD_KIND_*
  int bytes;
  int out_offset;
  uint128 modulus;
};

template <typename T, typename = void>
struct ValueTypeHelper {
  static constexpr bool IsSupportedType() { return false; }
};

template <typename T>
struct is_unsigned_integer
    : std::integral_constant<bool, std::is_same<T, uint8_t>::value ||
                                       std::is_same<T, uint16_t>::value ||
                                       std::is_same<T, uint32_t>::value ||
                                       std::is_same<T, uint64_t>::value ||
                                       std::is_same<T, unsigned __int128>::value> {};

template <typename T>
struct ValueTypeHelper<T, std::enable_if_t<is_unsigned_integer<T>::value>> {
  static constexpr bool IsSupportedType() { return true; }
  static ValueType ToValueType() {
    ValueType r;
    r.mutable_integer()->set_bitsize(8 * sizeof(T));
    return r;
  }
  static Value ToValue(const T& in) {
    Value r;
    *r.mutable_integer() = Uint128ToValueInteger(in);
    return r;
  }
  static StatusOr<T> FromValue(const Value& v) {
    if (v.value_case() != Value::kInteger)
      return InvalidArgumentError("The given Value is not an integer");
    StatusOr<uint128> x = ValueIntegerToUint128(v.integer());
    if (!x.ok()) return x.status();
    if (sizeof(T) < 16 && static_cast<uint64_t>(*x) > static_cast<uint64_t>(T(~T(0))))
      return InvalidArgumentError("Value (= " + std::to_string((uint64_t)*x) +
                                  ") too large for the given type T (size " +
                                  std::to_string(sizeof(T)) + ")");
    return static_cast<T>(*x);
  }
  static void Scalars(const T& obj, const char* base, std::vector<HostScalar>& out) {
    out.push_back({DPF_AMD_KIND_INTEGER, (int)sizeof(T),
                   (int)(reinterpret_cast<const char*>(&obj) - base), 0});
  }
};

template <typename T>
struct ValueTypeHelper<XorWrapper<T>, void> {
  static constexpr bool IsSupportedType() { return ValueTypeHelper<T>::IsSupportedType(); }
  static ValueType ToValueType() {
    ValueType r;
    r.mutable_xor_wrapper()->set_bitsize(8 * sizeof(T));
    return r;
  }
  static Value ToValue(const XorWrapper<T>& in) {
    Value r;
    *r.mutable_xor_wrapper() = Uint128ToValueInteger(in.value());
    return r;
  }
  static StatusOr<XorWrapper<T>> FromValue(const Value& v) {
    StatusOr<uint128> x = ValueIntegerToUint128(v.xor_wrapper());
    if (!x.ok()) return x.status();
    if (sizeof(T) < 16 && static_cast<uint64_t>(*x) > static_cast<uint64_t>(T(~T(0))))
      return InvalidArgumentError("Value (= " + std::to_string((uint64_t)*x) +
                                  ") too large for the given type T (size " +
                                  std::to_string(sizeof(T)) + ")");
    return XorWrapper<T>(static_cast<T>(*x));
  }
  static void Scalars(const XorWrapper<T>& obj, const char* base, std::vector<HostScalar>& out) {
    out.push_back({DPF_AMD_KIND_XOR_WRAPPER, (int)sizeof(T),
                   (int)(reinterpret_cast<const char*>(&obj.value()) - base), 0});
  }
};

template <typename B, typename M, M kModulus>
struct ValueTypeHelper<IntModNImpl<B, M, kModulus>, void> {
  using Type = IntModNImpl<B, M, kModulus>;
  static constexpr bool IsSupportedType() { return is_unsigned_integer<B>::value; }
  static ValueType ToValueType() {
    ValueType r;
    r.mutable_int_mod_n()->mutable_base_integer()->set_bitsize(8 * sizeof(B));
    *r.mutable_int_mod_n()->mutable_modulus() = Uint128ToValueInteger(kModulus);
    return r;
  }
  static Value ToValue(const Type& in) {
    Value r;
    *r.mutable_int_mod_n() = Uint128ToValueInteger(in.value());
    return r;
  }
  static StatusOr<Type> FromValue(const Value& v) {
    if (v.value_case() != Value::kIntModN)
      return InvalidArgumentError("The given Value is not an IntModN");
    StatusOr<uint128> x = ValueIntegerToUint128(v.int_mod_n());
    if (!x.ok()) return x.status();
    if (*x >= static_cast<uint128>(kModulus))
      return InvalidArgumentError("The given value is larger than kModulus");
    return Type(static_cast<B>(*x));
  }
  static void Scalars(const Type& obj, const char* base, std::vector<HostScalar>& out) {
    out.push_back({DPF_AMD_KIND_INT_MOD_N, (int)sizeof(B),
                   (int)(reinterpret_cast<const char*>(&obj) - base),
                   static_cast<uint128>(kModulus)});
  }
};

template <typename... E>
struct ValueTypeHelper<Tuple<E...>, void> {
  using Type = Tuple<E...>;
  static constexpr bool IsSupportedType() {
    return (ValueTypeHelper<E>::IsSupportedType() && ...);
  }
  static ValueType ToValueType() {
    ValueType r;
    auto* t = r.mutable_tuple();
    (void)t;
    ((*t->add_elements() = ValueTypeHelper<E>::ToValueType()), ...);
    return r;
  }
  static Value ToValue(const Type& in) {
    Value r;
    auto* t = r.mutable_tuple();
    std::apply(
        [t](const E&... e) { ((*t->add_elements() = ValueTypeHelper<E>::ToValue(e)), ...); },
        in.value());
    return r;
  }
  static StatusOr<Type> FromValue(const Value& v) {
    if (v.value_case() != Value::kTuple)
      return InvalidArgumentError("The given Value is not a tuple");
    if (v.tuple().elements_size() != (int)sizeof...(E))
      return InvalidArgumentError("The tuple in the given Value has the wrong number of elements");
    Status status;
    int i = 0;
    Type r{[&]() -> E {
      StatusOr<E> x = ValueTypeHelper<E>::FromValue(v.tuple().elements(i++));
      if (!x.ok()) {
        if (status.ok()) status = x.status();
        return E{};
      }
      return *x;
    }()...};
    if (!status.ok()) return status;
    return r;
  }
  static void Scalars(const Type& obj, const char* base, std::vector<HostScalar>& out) {
    std::apply([&](const E&... e) { (ValueTypeHelper<E>::Scalars(e, base, out), ...); },
               obj.value());
  }
};

template <typename T>
struct is_supported_type : std::integral_constant<bool, ValueTypeHelper<T>::IsSupportedType()> {
};

// Host layout of T measured on a real object (so it is exactly what this
// compiler lays out): flattened scalars with their byte offsets.
template <typename T>
std::vector<HostScalar> HostScalarsOf() {
  T obj{};
  std::vector<HostScalar> out;
  ValueTypeHelper<T>::Scalars(obj, reinterpret_cast<const char*>(&obj), out);
  return out;
}

}  // namespace dpf_internal

template <typename T>
ValueType ToValueType() {
  return dpf_internal::ValueTypeHelper<T>::ToValueType();
}
template <typename T>
Value ToValue(const T& v) {
  return dpf_internal::ValueTypeHelper<T>::ToValue(v);
}
template <typename T>
StatusOr<T> FromValue(const Value& v) {
  return dpf_internal::ValueTypeHelper<T>::FromValue(v);
}

}  // namespace distributed_point_functions

#endif  // DPF_AMD_VALUE_TYPES_H_
