// distributed_comparison_function.h — the reference's
// DistributedComparisonFunction (dcf/distributed_comparison_function.h:30-187)
// on MI355X: a DCF is an incremental DPF whose level i has log domain i
// (Create) and whose level-i beta is zero where alpha's bit i is 0
// (GenerateKeys); both run on the host exactly as in the reference.
// BatchEvaluate runs as ONE fused gfx950 kernel (dpf_amd_dcf_evaluate) that
// walks every key's path once and sums the levels the comparison needs,
// instead of EvaluateAndApply's per-level passes + host accumulation.
#ifndef DPF_AMD_DISTRIBUTED_COMPARISON_FUNCTION_H_
#define DPF_AMD_DISTRIBUTED_COMPARISON_FUNCTION_H_

#include <memory>
#include <utility>
#include <vector>

#include "dpf_amd/distributed_point_function.h"

namespace distributed_point_functions {

class DistributedComparisonFunction {
 public:
  static StatusOr<std::unique_ptr<DistributedComparisonFunction>> Create(
      const DcfParameters& parameters);

  // Keys that evaluate to shares of `beta` on x < alpha and of 0 otherwise.
  StatusOr<std::pair<DcfKey, DcfKey>> GenerateKeys(uint128 alpha, const Value& beta);
  template <typename T,
            typename = std::enable_if_t<!std::is_convertible<T, Value>::value &&
                                        dpf_internal::is_supported_type<T>::value>>
  StatusOr<std::pair<DcfKey, DcfKey>> GenerateKeys(uint128 alpha, const T& beta) {
    StatusOr<Value> value = dpf_->ToValue(beta);  // registers T (dcf.h:60-67)
    if (!value.ok()) return value.status();
    return GenerateKeys(alpha, *value);
  }
  // As GenerateKeys with explicit root seeds instead of the CSPRNG (fixtures).
  StatusOr<std::pair<DcfKey, DcfKey>> GenerateKeysWithSeeds(uint128 alpha, const Value& beta,
                                                            uint128 seed0, uint128 seed1);

  template <typename T>
  StatusOr<T> Evaluate(const DcfKey& key, uint128 x) {
    T result{};
    DPF_RETURN_IF_ERROR(BatchEvaluate<T>(Span<const DcfKey>(&key, 1), Span<const uint128>(&x, 1),
                                         Span<T>(&result, 1)));
    return result;
  }

  template <typename T>
  StatusOr<std::vector<T>> BatchEvaluate(Span<const DcfKey> keys,
                                         Span<const uint128> evaluation_points) {
    std::vector<T> result(keys.size());
    DPF_RETURN_IF_ERROR(
        BatchEvaluate<T>(keys, evaluation_points, Span<T>(result.data(), result.size())));
    return result;
  }

  template <typename T>
  Status BatchEvaluate(Span<const DcfKey> keys, Span<const uint128> evaluation_points,
                       Span<T> output) {
    if (keys.size() != evaluation_points.size())
      return InvalidArgumentError("`keys` and `evaluation_points` must have the same size");
    if (output.size() != keys.size())
      return InvalidArgumentError(
          "`keys`, `evaluation_points`, and `output` must have the same size");
    DPF_RETURN_IF_ERROR(dpf_->CheckType(ToValueType<T>(), -1, true));
    std::vector<const DcfKey*> ptrs;
    for (const DcfKey& k : keys) ptrs.push_back(&k);
    return BatchEvaluateRaw(Span<const DcfKey* const>(ptrs.data(), ptrs.size()),
                            evaluation_points, dpf_internal::HostLayoutOf<T>(), output.data());
  }

  // Raw entry (templates, C ABI): writes keys.size() host-layout values.
  Status BatchEvaluateRaw(Span<const DcfKey* const> keys, Span<const uint128> evaluation_points,
                          const dpf_amd_value_type& layout, void* out) const;

  const DcfParameters& parameters() const { return parameters_; }
  const DistributedPointFunction& dpf() const { return *dpf_; }

  DistributedComparisonFunction(const DistributedComparisonFunction&) = delete;
  DistributedComparisonFunction& operator=(const DistributedComparisonFunction&) = delete;

 private:
  DistributedComparisonFunction(DcfParameters parameters,
                                std::unique_ptr<DistributedPointFunction> dpf);
  StatusOr<std::vector<Value>> LevelBetas(uint128 alpha, const Value& beta) const;

  const DcfParameters parameters_;
  const std::unique_ptr<DistributedPointFunction> dpf_;
};

}  // namespace distributed_point_functions

#endif  // DPF_AMD_DISTRIBUTED_COMPARISON_FUNCTION_H_
