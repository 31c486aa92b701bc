// protos.h — the reference's proto messages as plain C++ classes with the
// accessor names of generated protobuf code (has_/mutable_/set_/add_/_size),
// plus protobuf wire-format (de)serialisation (csrc/wire.cc), so serialized
// messages are byte-compatible with the reference.
//   dpf/distributed_point_function.proto:25-171
//   pir/private_information_retrieval.proto:28-151
#ifndef DPF_AMD_PROTOS_H_
#define DPF_AMD_PROTOS_H_

#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

#include "dpf_amd/status.h"

namespace distributed_point_functions {

using uint128 = unsigned __int128;

inline constexpr uint128 MakeUint128(uint64_t high, uint64_t low) {
  return (static_cast<uint128>(high) << 64) | low;
}
inline constexpr uint64_t Uint128High64(uint128 v) { return static_cast<uint64_t>(v >> 64); }
inline constexpr uint64_t Uint128Low64(uint128 v) { return static_cast<uint64_t>(v); }
inline constexpr uint128 Uint128Max() { return ~static_cast<uint128>(0); }

#define DPF_AMD_SCALAR_FIELD(type, name)            \
  type name() const { return name##_; }             \
  void set_##name(type v) { name##_ = v; }          \
  void clear_##name() { name##_ = type(); }

#define DPF_AMD_MESSAGE_FIELD(type, name)                                 \
  bool has_##name() const { return has_##name##_; }                       \
  const type& name() const { return name##_; }                            \
  type* mutable_##name() {                                                \
    has_##name##_ = true;                                                 \
    return &name##_;                                                      \
  }                                                                       \
  void clear_##name() {                                                   \
    has_##name##_ = false;                                                \
    name##_ = type();                                                     \
  }

#define DPF_AMD_REPEATED_FIELD(type, name)                                     \
  int name##_size() const { return static_cast<int>(name##_.size()); }         \
  const type& name(int i) const { return name##_[i]; }                         \
  type* mutable_##name(int i) { return &name##_[i]; }                          \
  const std::vector<type>& name() const { return name##_; }                    \
  std::vector<type>* mutable_##name() { return &name##_; }                     \
  type* add_##name() {                                                         \
    name##_.emplace_back();                                                    \
    return &name##_.back();                                                    \
  }                                                                            \
  void clear_##name() { name##_.clear(); }

class Block {
 public:
  DPF_AMD_SCALAR_FIELD(uint64_t, high)
  DPF_AMD_SCALAR_FIELD(uint64_t, low)
  bool operator==(const Block& o) const { return high_ == o.high_ && low_ == o.low_; }

 private:
  uint64_t high_ = 0, low_ = 0;
};

class Value {
 public:
  class Integer {
   public:
    enum ValueCase { VALUE_NOT_SET = 0, kValueUint64 = 1, kValueUint128 = 2 };
    ValueCase value_case() const { return case_; }
    uint64_t value_uint64() const { return case_ == kValueUint64 ? u64_ : 0; }
    void set_value_uint64(uint64_t v) {
      case_ = kValueUint64;
      u64_ = v;
    }
    bool has_value_uint128() const { return case_ == kValueUint128; }
    const Block& value_uint128() const { return u128_; }
    Block* mutable_value_uint128() {
      case_ = kValueUint128;
      return &u128_;
    }

   private:
    ValueCase case_ = VALUE_NOT_SET;
    uint64_t u64_ = 0;
    Block u128_;
  };

  class Tuple {
   public:
    DPF_AMD_REPEATED_FIELD(Value, elements)

   private:
    std::vector<Value> elements_;
  };

  enum ValueCase { VALUE_NOT_SET = 0, kInteger = 1, kTuple = 2, kIntModN = 3, kXorWrapper = 4 };
  ValueCase value_case() const { return case_; }
  const Integer& integer() const { return integer_; }
  Integer* mutable_integer() { return Set(kInteger, &integer_); }
  const Tuple& tuple() const { return tuple_; }
  Tuple* mutable_tuple() { return Set(kTuple, &tuple_); }
  const Integer& int_mod_n() const { return integer_; }
  Integer* mutable_int_mod_n() { return Set(kIntModN, &integer_); }
  const Integer& xor_wrapper() const { return integer_; }
  Integer* mutable_xor_wrapper() { return Set(kXorWrapper, &integer_); }

 private:
  template <typename T>
  T* Set(ValueCase c, T* p) {
    if (case_ != c) {
      integer_ = Integer();
      tuple_ = Tuple();
    }
    case_ = c;
    return p;
  }
  ValueCase case_ = VALUE_NOT_SET;
  Integer integer_;  // integer / int_mod_n / xor_wrapper
  Tuple tuple_;
};

class ValueType {
 public:
  class Integer {
   public:
    DPF_AMD_SCALAR_FIELD(int32_t, bitsize)

   private:
    int32_t bitsize_ = 0;
  };

  class Tuple {
   public:
    DPF_AMD_REPEATED_FIELD(ValueType, elements)

   private:
    std::vector<ValueType> elements_;
  };

  class IntModN {
   public:
    DPF_AMD_MESSAGE_FIELD(Integer, base_integer)
    DPF_AMD_MESSAGE_FIELD(Value::Integer, modulus)

   private:
    bool has_base_integer_ = false, has_modulus_ = false;
    Integer base_integer_;
    Value::Integer modulus_;
  };

  enum TypeCase { TYPE_NOT_SET = 0, kInteger = 1, kTuple = 2, kIntModN = 3, kXorWrapper = 4 };
  TypeCase type_case() const { return case_; }
  const Integer& integer() const { return integer_; }
  Integer* mutable_integer() { return Set(kInteger, &integer_); }
  const Tuple& tuple() const { return tuple_; }
  Tuple* mutable_tuple() { return Set(kTuple, &tuple_); }
  const IntModN& int_mod_n() const { return int_mod_n_; }
  IntModN* mutable_int_mod_n() { return Set(kIntModN, &int_mod_n_); }
  const Integer& xor_wrapper() const { return integer_; }
  Integer* mutable_xor_wrapper() { return Set(kXorWrapper, &integer_); }
  std::string DebugString() const;

 private:
  template <typename T>
  T* Set(TypeCase c, T* p) {
    if (case_ != c) {
      integer_ = Integer();
      tuple_ = Tuple();
      int_mod_n_ = IntModN();
    }
    case_ = c;
    return p;
  }
  TypeCase case_ = TYPE_NOT_SET;
  Integer integer_;  // integer / xor_wrapper
  Tuple tuple_;
  IntModN int_mod_n_;
};

class DpfParameters {
 public:
  DPF_AMD_SCALAR_FIELD(int32_t, log_domain_size)
  DPF_AMD_MESSAGE_FIELD(ValueType, value_type)
  DPF_AMD_SCALAR_FIELD(double, security_parameter)
  std::string DebugString() const;

 private:
  int32_t log_domain_size_ = 0;
  bool has_value_type_ = false;
  ValueType value_type_;
  double security_parameter_ = 0;
};

class CorrectionWord {
 public:
  DPF_AMD_MESSAGE_FIELD(Block, seed)
  DPF_AMD_SCALAR_FIELD(bool, control_left)
  DPF_AMD_SCALAR_FIELD(bool, control_right)
  DPF_AMD_REPEATED_FIELD(Value, value_correction)

 private:
  bool has_seed_ = false;
  Block seed_;
  bool control_left_ = false, control_right_ = false;
  std::vector<Value> value_correction_;
};

class DpfKey {
 public:
  DPF_AMD_MESSAGE_FIELD(Block, seed)
  DPF_AMD_REPEATED_FIELD(CorrectionWord, correction_words)
  DPF_AMD_SCALAR_FIELD(int32_t, party)
  DPF_AMD_REPEATED_FIELD(Value, last_level_value_correction)

  std::string SerializeAsString() const;
  bool ParseFromString(const std::string& data);
  bool ParseFromArray(const void* data, size_t size);

 private:
  bool has_seed_ = false;
  Block seed_;
  std::vector<CorrectionWord> correction_words_;
  int32_t party_ = 0;
  std::vector<Value> last_level_value_correction_;
};

class PartialEvaluation {
 public:
  DPF_AMD_MESSAGE_FIELD(Block, prefix)
  DPF_AMD_MESSAGE_FIELD(Block, seed)
  DPF_AMD_SCALAR_FIELD(bool, control_bit)

 private:
  bool has_prefix_ = false, has_seed_ = false;
  Block prefix_, seed_;
  bool control_bit_ = false;
};

// The partial evaluations EvaluateUntil left on a GPU (library-internal,
// defined in the library): the list is read back into host messages only
// when a caller reads the field, once per list.
class ContextDeviceState;
const std::vector<PartialEvaluation>& PartialEvaluationsOf(const ContextDeviceState& state);
int PartialEvaluationsCountOf(const ContextDeviceState& state);

class EvaluationContext {
 public:
  DPF_AMD_REPEATED_FIELD(DpfParameters, parameters)
  DPF_AMD_MESSAGE_FIELD(DpfKey, key)
  DPF_AMD_SCALAR_FIELD(int32_t, previous_hierarchy_level)
  // repeated PartialEvaluation partial_evaluations (proto field 4): reads
  // see the device-held list when there is one; writes take it to the host
  int partial_evaluations_size() const {
    return device_ ? PartialEvaluationsCountOf(*device_)
                   : static_cast<int>(partial_evaluations_.size());
  }
  const PartialEvaluation& partial_evaluations(int i) const { return partial_evaluations()[i]; }
  const std::vector<PartialEvaluation>& partial_evaluations() const {
    return device_ ? PartialEvaluationsOf(*device_) : partial_evaluations_;
  }
  PartialEvaluation* mutable_partial_evaluations(int i) {
    ToHost();
    return &partial_evaluations_[i];
  }
  std::vector<PartialEvaluation>* mutable_partial_evaluations() {
    ToHost();
    return &partial_evaluations_;
  }
  PartialEvaluation* add_partial_evaluations() {
    ToHost();
    partial_evaluations_.emplace_back();
    return &partial_evaluations_.back();
  }
  void clear_partial_evaluations() {
    device_.reset();
    partial_evaluations_.clear();
  }
  DPF_AMD_SCALAR_FIELD(int32_t, partial_evaluations_level)

  std::string SerializeAsString() const;
  bool ParseFromString(const std::string& data);
  bool ParseFromArray(const void* data, size_t size);

  // Library-internal: the device-held partial evaluations (null when the
  // list is on the host).  Setting one replaces the host list.
  const std::shared_ptr<const ContextDeviceState>& device_state() const { return device_; }
  void set_device_state(std::shared_ptr<const ContextDeviceState> state) {
    partial_evaluations_.clear();
    device_ = std::move(state);
  }

 private:
  void ToHost() {
    if (!device_) return;
    partial_evaluations_ = PartialEvaluationsOf(*device_);
    device_.reset();
  }
  std::vector<DpfParameters> parameters_;
  bool has_key_ = false;
  DpfKey key_;
  int32_t previous_hierarchy_level_ = 0;
  std::vector<PartialEvaluation> partial_evaluations_;
  std::shared_ptr<const ContextDeviceState> device_;
  int32_t partial_evaluations_level_ = 0;
};

// --- DCF messages (dcf/distributed_comparison_function.proto:25-32) --------

class DcfParameters {
 public:
  DPF_AMD_MESSAGE_FIELD(DpfParameters, parameters)
  std::string SerializeAsString() const;
  bool ParseFromArray(const void* data, size_t size);

 private:
  bool has_parameters_ = false;
  DpfParameters parameters_;
};

class DcfKey {
 public:
  DPF_AMD_MESSAGE_FIELD(DpfKey, key)
  std::string SerializeAsString() const;
  bool ParseFromString(const std::string& data) { return ParseFromArray(data.data(), data.size()); }
  bool ParseFromArray(const void* data, size_t size);

 private:
  bool has_key_ = false;
  DpfKey key_;
};

// --- PIR messages (pir/private_information_retrieval.proto) ---------------

class DenseDpfPirConfig {
 public:
  DPF_AMD_SCALAR_FIELD(int64_t, num_elements)

 private:
  int64_t num_elements_ = 0;
};

// pir/hashing/hash_family_config.proto:22-35
class HashFamilyConfig {
 public:
  enum HashFamily { HASH_FAMILY_UNSPECIFIED = 0, HASH_FAMILY_SHA256 = 1 };
  DPF_AMD_SCALAR_FIELD(int, hash_family)
  const std::string& seed() const { return seed_; }
  std::string* mutable_seed() { return &seed_; }
  void set_seed(std::string s) { seed_ = std::move(s); }
  std::string SerializeAsString() const;
  bool ParseFromArray(const void* data, size_t size);

 private:
  int hash_family_ = HASH_FAMILY_UNSPECIFIED;
  std::string seed_;
};

// private_information_retrieval.proto: CuckooHashingSparseDpfPirConfig
class CuckooHashingSparseDpfPirConfig {
 public:
  DPF_AMD_SCALAR_FIELD(int, hash_family)
  DPF_AMD_SCALAR_FIELD(int64_t, num_elements)

 private:
  int hash_family_ = HashFamilyConfig::HASH_FAMILY_UNSPECIFIED;
  int64_t num_elements_ = 0;
};

// private_information_retrieval.proto: CuckooHashingParams
class CuckooHashingParams {
 public:
  DPF_AMD_MESSAGE_FIELD(HashFamilyConfig, hash_family_config)
  DPF_AMD_SCALAR_FIELD(int32_t, num_hash_functions)
  DPF_AMD_SCALAR_FIELD(int64_t, num_buckets)
  std::string SerializeAsString() const;
  bool ParseFromArray(const void* data, size_t size);

 private:
  bool has_hash_family_config_ = false;
  HashFamilyConfig hash_family_config_;
  int32_t num_hash_functions_ = 0;
  int64_t num_buckets_ = 0;
};

class PirConfig {
 public:
  enum WrappedPirConfigCase {
    WRAPPED_PIR_CONFIG_NOT_SET = 0,
    kDenseDpfPirConfig = 1,
    kCuckooHashingSparseDpfPirConfig = 2
  };
  WrappedPirConfigCase wrapped_pir_config_case() const { return case_; }
  const DenseDpfPirConfig& dense_dpf_pir_config() const { return dense_; }
  DenseDpfPirConfig* mutable_dense_dpf_pir_config() {
    case_ = kDenseDpfPirConfig;
    return &dense_;
  }
  const CuckooHashingSparseDpfPirConfig& cuckoo_hashing_sparse_dpf_pir_config() const {
    return cuckoo_;
  }
  CuckooHashingSparseDpfPirConfig* mutable_cuckoo_hashing_sparse_dpf_pir_config() {
    case_ = kCuckooHashingSparseDpfPirConfig;
    return &cuckoo_;
  }
  std::string SerializeAsString() const;
  bool ParseFromArray(const void* data, size_t size);

 private:
  WrappedPirConfigCase case_ = WRAPPED_PIR_CONFIG_NOT_SET;
  DenseDpfPirConfig dense_;
  CuckooHashingSparseDpfPirConfig cuckoo_;
};

class DpfPirRequest {
 public:
  class PlainRequest {
   public:
    DPF_AMD_REPEATED_FIELD(DpfKey, dpf_key)

   private:
    std::vector<DpfKey> dpf_key_;
  };
  class EncryptedHelperRequest {
   public:
    const std::string& encrypted_request() const { return encrypted_request_; }
    std::string* mutable_encrypted_request() { return &encrypted_request_; }
    void set_encrypted_request(std::string s) { encrypted_request_ = std::move(s); }

   private:
    std::string encrypted_request_;
  };
  class LeaderRequest {
   public:
    DPF_AMD_MESSAGE_FIELD(PlainRequest, plain_request)
    DPF_AMD_MESSAGE_FIELD(EncryptedHelperRequest, encrypted_helper_request)

   private:
    bool has_plain_request_ = false, has_encrypted_helper_request_ = false;
    PlainRequest plain_request_;
    EncryptedHelperRequest encrypted_helper_request_;
  };
  class HelperRequest {
   public:
    DPF_AMD_MESSAGE_FIELD(PlainRequest, plain_request)
    const std::string& one_time_pad_seed() const { return one_time_pad_seed_; }
    std::string* mutable_one_time_pad_seed() { return &one_time_pad_seed_; }
    std::string SerializeAsString() const;
    bool ParseFromString(const std::string& data);

   private:
    bool has_plain_request_ = false;
    PlainRequest plain_request_;
    std::string one_time_pad_seed_;
  };

  enum WrappedRequestCase {
    WRAPPED_REQUEST_NOT_SET = 0,
    kPlainRequest = 1,
    kLeaderRequest = 2,
    kEncryptedHelperRequest = 3
  };
  WrappedRequestCase wrapped_request_case() const { return case_; }
  const PlainRequest& plain_request() const { return plain_; }
  PlainRequest* mutable_plain_request() {
    case_ = kPlainRequest;
    return &plain_;
  }
  const LeaderRequest& leader_request() const { return leader_; }
  LeaderRequest* mutable_leader_request() {
    case_ = kLeaderRequest;
    return &leader_;
  }
  const EncryptedHelperRequest& encrypted_helper_request() const { return helper_; }
  EncryptedHelperRequest* mutable_encrypted_helper_request() {
    case_ = kEncryptedHelperRequest;
    return &helper_;
  }

 private:
  WrappedRequestCase case_ = WRAPPED_REQUEST_NOT_SET;
  PlainRequest plain_;
  LeaderRequest leader_;
  EncryptedHelperRequest helper_;
};

class PirRequest {
 public:
  enum WrappedPirRequestCase { WRAPPED_PIR_REQUEST_NOT_SET = 0, kDpfPirRequest = 1 };
  WrappedPirRequestCase wrapped_pir_request_case() const { return case_; }
  const DpfPirRequest& dpf_pir_request() const { return req_; }
  DpfPirRequest* mutable_dpf_pir_request() {
    case_ = kDpfPirRequest;
    return &req_;
  }
  std::string SerializeAsString() const;
  bool ParseFromArray(const void* data, size_t size);

 private:
  WrappedPirRequestCase case_ = WRAPPED_PIR_REQUEST_NOT_SET;
  DpfPirRequest req_;
};

class DpfPirResponse {
 public:
  DPF_AMD_REPEATED_FIELD(std::string, masked_response)

 private:
  std::vector<std::string> masked_response_;
};

class PirResponse {
 public:
  enum WrappedPirResponseCase { WRAPPED_PIR_RESPONSE_NOT_SET = 0, kDpfPirResponse = 1 };
  WrappedPirResponseCase wrapped_pir_response_case() const { return case_; }
  const DpfPirResponse& dpf_pir_response() const { return resp_; }
  DpfPirResponse* mutable_dpf_pir_response() {
    case_ = kDpfPirResponse;
    return &resp_;
  }
  std::string SerializeAsString() const;
  bool ParseFromArray(const void* data, size_t size);

 private:
  WrappedPirResponseCase case_ = WRAPPED_PIR_RESPONSE_NOT_SET;
  DpfPirResponse resp_;
};

class PirServerPublicParams {
 public:
  enum WrappedPirServerPublicParamsCase {
    WRAPPED_PIR_SERVER_PUBLIC_PARAMS_NOT_SET = 0,
    kCuckooHashingSparseDpfPirServerParams = 1
  };
  static const PirServerPublicParams& default_instance();
  WrappedPirServerPublicParamsCase wrapped_pir_server_public_params_case() const { return case_; }
  const CuckooHashingParams& cuckoo_hashing_sparse_dpf_pir_server_params() const {
    return cuckoo_;
  }
  CuckooHashingParams* mutable_cuckoo_hashing_sparse_dpf_pir_server_params() {
    case_ = kCuckooHashingSparseDpfPirServerParams;
    return &cuckoo_;
  }
  std::string SerializeAsString() const;
  bool ParseFromArray(const void* data, size_t size);

 private:
  WrappedPirServerPublicParamsCase case_ = WRAPPED_PIR_SERVER_PUBLIC_PARAMS_NOT_SET;
  CuckooHashingParams cuckoo_;
};

// Wire helpers for the remaining messages.
std::string SerializeValueType(const ValueType& vt);
bool ParseValueType(const void* data, size_t size, ValueType* out);
std::string SerializeValue(const Value& v);
bool ParseValue(const void* data, size_t size, Value* out);
std::string SerializeDpfParameters(const DpfParameters& p);
bool ParseDpfParameters(const void* data, size_t size, DpfParameters* out);

}  // namespace distributed_point_functions

#endif  // DPF_AMD_PROTOS_H_
