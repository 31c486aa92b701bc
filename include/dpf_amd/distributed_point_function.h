// distributed_point_function.h — the reference's DistributedPointFunction
// (dpf/distributed_point_function.h:87-639) re-implemented on MI355X: key
// generation and validation run on the host exactly as in the reference;
// every evaluation (full-domain / incremental expansion, point evaluation,
// EvaluateAndApply) runs in the gfx950 kernels behind include/dpf_amd.h.
//
// Drop-in notes: names, argument meaning, error codes and messages follow
// the reference.  absl::uint128 -> `uint128` (unsigned __int128, same
// layout), absl::Span -> `Span`, absl::Status(Or) -> `Status(Or)`.
// Value types follow the reference's registration contract (cc:567-582,
// 620-633): single unsigned integers are registered at construction,
// RegisterValueType<T>() / ToValue<T>() (and the templated GenerateKeys
// overloads, which call ToValue<T>) register T, and GenerateKeys* with a
// Value proto of an unregistered type returns FAILED_PRECONDITION.
#ifndef DPF_AMD_DISTRIBUTED_POINT_FUNCTION_H_
#define DPF_AMD_DISTRIBUTED_POINT_FUNCTION_H_

#include <stdint.h>

#include <memory>
#include <utility>
#include <vector>

#include "dpf_amd.h"
#include "dpf_amd/protos.h"
#include "dpf_amd/status.h"
#include "dpf_amd/value_types.h"

namespace distributed_point_functions {

namespace dpf_internal {
class DpfState;  // validator + per-level metadata (csrc/dpf.cc)

// Layout descriptor of T for the C ABI, from the real object layout.
template <typename T>
dpf_amd_value_type HostLayoutOf() {
  dpf_amd_value_type vt{};
  std::vector<HostScalar> sc = HostScalarsOf<T>();
  vt.num_scalars = static_cast<int32_t>(sc.size());
  vt.out_stride = static_cast<int32_t>(sizeof(T));
  int in_off = 0;
  for (size_t i = 0; i < sc.size() && i < DPF_AMD_MAX_SCALARS; ++i) {
    vt.scalars[i].kind = sc[i].kind;
    vt.scalars[i].bytes = sc[i].bytes;
    vt.scalars[i].in_offset = in_off;
    vt.scalars[i].out_offset = sc[i].out_offset;
    vt.scalars[i].modulus[0] = static_cast<uint64_t>(sc[i].modulus);
    vt.scalars[i].modulus[1] = static_cast<uint64_t>(sc[i].modulus >> 64);
    in_off += sc[i].bytes;
  }
  return vt;
}
}  // namespace dpf_internal

class DistributedPointFunction {
 public:
  static StatusOr<std::unique_ptr<DistributedPointFunction>> Create(
      const DpfParameters& parameters);
  static StatusOr<std::unique_ptr<DistributedPointFunction>> CreateIncremental(
      Span<const DpfParameters> parameters);

  ~DistributedPointFunction();
  DistributedPointFunction(const DistributedPointFunction&) = delete;
  DistributedPointFunction& operator=(const DistributedPointFunction&) = delete;

  // ToValue<T> (h:112-118): registers T, then converts.
  template <typename T>
  StatusOr<Value> ToValue(const T& in) {
    Status status = RegisterValueType<T>();
    if (!status.ok()) return status;
    return distributed_point_functions::ToValue(in);
  }
  // RegisterValueType<T> (h:129-131).
  template <typename T>
  Status RegisterValueType() {
    return RegisterValueTypeProto(ToValueType<T>());
  }
  // Non-template registration by ValueType proto (the C ABI's entry).
  Status RegisterValueTypeProto(const ValueType& value_type);
  bool IsValueTypeRegistered(const ValueType& value_type) const;

  // GenerateKeys overloads (h:171-196).
  StatusOr<std::pair<DpfKey, DpfKey>> GenerateKeys(uint128 alpha, uint128 beta) {
    std::vector<uint128> b{beta};
    return GenerateKeysIncremental(alpha, b);
  }
  StatusOr<std::pair<DpfKey, DpfKey>> GenerateKeys(uint128 alpha, Value beta) {
    std::vector<Value> b{std::move(beta)};
    return GenerateKeysIncremental(alpha, Span<const Value>(b.data(), b.size()));
  }
  template <typename T,
            typename = std::enable_if_t<!std::is_convertible<T, uint128>::value &&
                                        !std::is_convertible<T, Value>::value &&
                                        dpf_internal::is_supported_type<T>::value>>
  StatusOr<std::pair<DpfKey, DpfKey>> GenerateKeys(uint128 alpha, const T& beta) {
    StatusOr<Value> v = ToValue(beta);
    if (!v.ok()) return v.status();
    std::vector<Value> b{*v};
    return GenerateKeysIncremental(alpha, Span<const Value>(b.data(), b.size()));
  }

  // GenerateKeysIncremental overloads (h:237-271).
  StatusOr<std::pair<DpfKey, DpfKey>> GenerateKeysIncremental(
      uint128 alpha, const std::vector<uint128>& beta);
  template <typename T>
  StatusOr<std::pair<DpfKey, DpfKey>> GenerateKeysIncremental(uint128 alpha,
                                                              Span<const T> beta) {
    std::vector<Value> values;
    for (const T& b : beta) {
      StatusOr<Value> v = ToValue(b);
      if (!v.ok()) return v.status();
      values.push_back(*v);
    }
    return GenerateKeysIncremental(alpha, Span<const Value>(values.data(), values.size()));
  }
  StatusOr<std::pair<DpfKey, DpfKey>> GenerateKeysIncremental(uint128 alpha,
                                                              Span<const Value> beta);
  // As above with explicit root seeds instead of the CSPRNG (fixtures).
  StatusOr<std::pair<DpfKey, DpfKey>> GenerateKeysIncrementalWithSeeds(
      uint128 alpha, Span<const Value> beta, uint128 seed0, uint128 seed1);

  // CreateEvaluationContext (h:278).
  StatusOr<EvaluationContext> CreateEvaluationContext(DpfKey key) const;

  // EvaluateUntil / EvaluateNext (h:319-333).
  template <typename T>
  StatusOr<std::vector<T>> EvaluateUntil(int hierarchy_level, Span<const uint128> prefixes,
                                         EvaluationContext& ctx) const {
    DPF_RETURN_IF_ERROR(CheckType(ToValueType<T>(), hierarchy_level, false));
    int64_t n = 0;
    // size only (capacity -1: the prefixes are validated by the call below)
    DPF_RETURN_IF_ERROR(EvaluateUntilRaw(hierarchy_level, prefixes, ctx, LayoutOf<T>(),
                                         nullptr, -1, &n, false, nullptr));
    std::vector<T> out(n);
    DPF_RETURN_IF_ERROR(EvaluateUntilRaw(hierarchy_level, prefixes, ctx, LayoutOf<T>(),
                                         out.data(), n, &n, false, nullptr));
    return out;
  }
  template <typename T>
  StatusOr<std::vector<T>> EvaluateNext(Span<const uint128> prefixes,
                                        EvaluationContext& ctx) const {
    if (prefixes.empty()) return EvaluateUntil<T>(0, prefixes, ctx);
    return EvaluateUntil<T>(ctx.previous_hierarchy_level() + 1, prefixes, ctx);
  }

  // EvaluateAt (h:349-378).
  template <typename T>
  StatusOr<std::vector<T>> EvaluateAt(const DpfKey& key, int hierarchy_level,
                                      Span<const uint128> evaluation_points) const {
    DPF_RETURN_IF_ERROR(CheckType(ToValueType<T>(), hierarchy_level, true));
    std::vector<T> out(evaluation_points.size());
    DPF_RETURN_IF_ERROR(EvaluateAtRaw(key, hierarchy_level, evaluation_points, nullptr,
                                      LayoutOf<T>(), out.data()));
    return out;
  }
  template <typename T>
  StatusOr<std::vector<T>> EvaluateAt(int hierarchy_level,
                                      Span<const uint128> evaluation_points,
                                      EvaluationContext& ctx) const {
    DPF_RETURN_IF_ERROR(CheckType(ToValueType<T>(), hierarchy_level, true));
    std::vector<T> out(evaluation_points.size());
    DPF_RETURN_IF_ERROR(EvaluateAtRaw(ctx.key(), hierarchy_level, evaluation_points, &ctx,
                                      LayoutOf<T>(), out.data()));
    return out;
  }

  // EvaluateAndApply (h:403-407): op(Span<const T>) after every level; stops
  // when op returns false.
  template <typename T, typename Fn>
  Status EvaluateAndApply(Span<const DpfKey> keys, Span<const uint128> evaluation_points,
                          Fn op, int evaluation_points_rightshift = 0) const {
    std::vector<const DpfKey*> ptrs;
    for (const DpfKey& k : keys) ptrs.push_back(&k);
    return EvaluateAndApply<T>(Span<const DpfKey* const>(ptrs.data(), ptrs.size()),
                               evaluation_points, std::move(op),
                               evaluation_points_rightshift);
  }
  template <typename T, typename Fn>
  Status EvaluateAndApply(Span<const DpfKey* const> keys, Span<const uint128> evaluation_points,
                          Fn op, int evaluation_points_rightshift = 0) const {
    DPF_RETURN_IF_ERROR(CheckType(ToValueType<T>(), -1, true));
    const int levels = num_hierarchy_levels();
    std::vector<T> values(keys.size() * static_cast<size_t>(levels));
    int done = 0;
    // op runs after each level is evaluated; a false return stops the
    // evaluation of the remaining levels (h:1190-1196)
    struct Ctx {
      Fn* op;
      const T* values;
      size_t n;
    } ctx{&op, values.data(), keys.size()};
    auto on_level = [](void* user, int h) -> bool {
      Ctx* c = static_cast<Ctx*>(user);
      return (*c->op)(Span<const T>(c->values + h * c->n, c->n));
    };
    return EvaluateAndApplyRaw(keys, evaluation_points, evaluation_points_rightshift,
                               LayoutOf<T>(), values.data(), &done, on_level, &ctx);
  }

  Span<const DpfParameters> parameters() const;
  int num_hierarchy_levels() const;
  int tree_levels_needed() const;
  int hierarchy_to_tree(int level) const;
  int blocks_needed(int level) const;
  // Descriptor (conversion metadata + host layout) of level `level`'s type.
  dpf_amd_value_type value_type_descriptor(int level) const;

  // ---- Raw entry points (shared by the templates and the C ABI) ---------
  // Layout `vt` gives sizeof(T) and the scalar offsets; conversion metadata
  // is taken from the parameters.  With out_on_device, `out` is a device
  // pointer and no host copy happens (stream-ordered on `stream`).
  Status EvaluateUntilRaw(int hierarchy_level, Span<const uint128> prefixes,
                          EvaluationContext& ctx, const dpf_amd_value_type& vt, void* out,
                          int64_t out_capacity, int64_t* num_outputs, bool out_on_device,
                          void* stream) const;
  Status EvaluateAtRaw(const DpfKey& key, int hierarchy_level,
                       Span<const uint128> evaluation_points, EvaluationContext* ctx,
                       const dpf_amd_value_type& vt, void* out) const;
  // After each level's values are in `out`, `on_level(user, level)` (if
  // set) decides whether to continue.
  Status EvaluateAndApplyRaw(Span<const DpfKey* const> keys,
                             Span<const uint128> evaluation_points, int rightshift,
                             const dpf_amd_value_type& vt, void* out, int* levels_done,
                             bool (*on_level)(void*, int) = nullptr,
                             void* user = nullptr) const;
  // ProtoValidator::ValidateDpfKey (proto_validator.cc:205-236).
  Status ValidateKey(const DpfKey& key) const;
  // The value correction of `key` at hierarchy `level` as flattened 128-bit
  // scalar words, epb * num_scalars of them (ValuesToArray, vth:561-580).
  Status ValueCorrectionWords(const DpfKey& key, int level, std::vector<uint128>* out) const;
  // Checks that `type` equals the parameters' type at `level` (all levels if
  // level < 0) (h:709-716).
  Status CheckType(const ValueType& type, int level, bool at) const;
  // Device-resident full-domain slice: expands leaves [leaf_begin, leaf_end)
  // of the last hierarchy level of `key` (tree blocks of the single root),
  // writing host-layout values to device memory `out` (bench / sharding).
  Status ExpandLeavesOnDevice(const DpfKey& key, int64_t leaf_begin, int64_t leaf_end,
                              const dpf_amd_value_type& vt, void* out, void* stream) const;
  // Leaves [0, num_leaves) of every key, key i's at out + i * num_leaves *
  // cepb * out_stride (the selection vectors of a batched PIR request).  Small
  // batches take one upload and one launch (per-leaf walks); large ones one
  // tree expansion per key.
  Status ExpandLeavesOnDeviceBatched(Span<const DpfKey* const> keys, int64_t num_leaves,
                                     const dpf_amd_value_type& vt, void* out,
                                     void* stream) const;
  // Leaves [leaf_begin, leaf_end) of every key, key i's at out + i *
  // (leaf_end - leaf_begin) * cepb * out_stride (one database shard's
  // selection blocks).
  Status ExpandLeavesOnDeviceBatched(Span<const DpfKey* const> keys, int64_t leaf_begin,
                                     int64_t leaf_end, const dpf_amd_value_type& vt, void* out,
                                     void* stream) const;
  // One key's leaves spread over devices: slice i expands leaves
  // [leaf_begin[i], leaf_end[i]) on device devices[i] into that device's
  // memory outs[i], each on the calling thread's stream for the device; all
  // slices are issued before any is waited for, and the call returns when
  // every device is done (c5 subtree-sharded over the GPUs of one process).
  Status ExpandLeavesOnDevices(const DpfKey& key, Span<const int> devices,
                               Span<const int64_t> leaf_begin, Span<const int64_t> leaf_end,
                               Span<void* const> outs, const dpf_amd_value_type& vt) const;

 private:
  explicit DistributedPointFunction(std::unique_ptr<dpf_internal::DpfState> state);
  template <typename T>
  static dpf_amd_value_type LayoutOf() {
    return dpf_internal::HostLayoutOf<T>();
  }
  std::unique_ptr<dpf_internal::DpfState> state_;
};

}  // namespace distributed_point_functions

#endif  // DPF_AMD_DISTRIBUTED_POINT_FUNCTION_H_
