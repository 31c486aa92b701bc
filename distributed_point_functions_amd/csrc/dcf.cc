// dcf.cc — DistributedComparisonFunction (dcf/distributed_comparison_function
// .cc:46-111, .h:141-187) over the MI355X DPF.  Create and GenerateKeys are
// the reference's host logic; BatchEvaluate uploads the keys' seeds and
// per-level correction words once and runs the fused gfx950 kernel
// (dpf_amd_dcf_evaluate) — no per-level passes, no host accumulation.
#include "dpf_amd/distributed_comparison_function.h"

#include <algorithm>
#include <string>
#include <utility>
#include <vector>

#include "host_device.h"

namespace distributed_point_functions {

using dpf_internal_host::AbiStatus;
using dpf_internal_host::ClearPadding;
using dpf_internal_host::CopyToHostSync;
using dpf_internal_host::DeviceBuffer;
using dpf_internal_host::HipStatus;
using dpf_internal_host::ThreadStream;

namespace {

// dcf.cc:33-43: zero integers, IntModN and tuples; XorWrapper values are
// left untouched, as in the reference.
void SetToZero(Value& value) {
  if (value.value_case() == Value::kInteger) {
    value.mutable_integer()->set_value_uint64(0);
  } else if (value.value_case() == Value::kIntModN) {
    value.mutable_int_mod_n()->set_value_uint64(0);
  } else if (value.value_case() == Value::kTuple) {
    for (int i = 0; i < value.tuple().elements_size(); ++i)
      SetToZero(*value.mutable_tuple()->mutable_elements(i));
  }
}

}  // namespace

DistributedComparisonFunction::DistributedComparisonFunction(
    DcfParameters parameters, std::unique_ptr<DistributedPointFunction> dpf)
    : parameters_(std::move(parameters)), dpf_(std::move(dpf)) {}

// dcf.cc:50-79.
StatusOr<std::unique_ptr<DistributedComparisonFunction>> DistributedComparisonFunction::Create(
    const DcfParameters& parameters) {
  if (parameters.parameters().log_domain_size() < 1)
    return InvalidArgumentError("A DCF must have log_domain_size >= 1");
  if (!parameters.parameters().has_value_type())
    return InvalidArgumentError(
        "parameters.value_type must be set for DistributedComparisonFunction::Create");
  std::vector<DpfParameters> dpf_parameters(parameters.parameters().log_domain_size());
  for (int i = 0; i < static_cast<int>(dpf_parameters.size()); ++i) {
    dpf_parameters[i].set_log_domain_size(i);
    *dpf_parameters[i].mutable_value_type() = parameters.parameters().value_type();
  }
  StatusOr<std::unique_ptr<DistributedPointFunction>> dpf =
      DistributedPointFunction::CreateIncremental(
          Span<const DpfParameters>(dpf_parameters.data(), dpf_parameters.size()));
  if (!dpf.ok()) return dpf.status();
  return std::unique_ptr<DistributedComparisonFunction>(
      new DistributedComparisonFunction(parameters, std::move(*dpf)));
}

// dcf.cc:83-95: beta at level i where bit (n - 1 - i) of alpha is set, 0
// elsewhere.
StatusOr<std::vector<Value>> DistributedComparisonFunction::LevelBetas(uint128 alpha,
                                                                       const Value& beta) const {
  const int n = parameters_.parameters().log_domain_size();
  std::vector<Value> values(n, beta);
  for (int i = 0; i < n; ++i) {
    const bool bit = (alpha & (uint128{1} << (n - i - 1))) != 0;
    if (!bit) SetToZero(values[i]);
  }
  return values;
}

StatusOr<std::pair<DcfKey, DcfKey>> DistributedComparisonFunction::GenerateKeys(
    uint128 alpha, const Value& beta) {
  StatusOr<std::vector<Value>> values = LevelBetas(alpha, beta);
  if (!values.ok()) return values.status();
  // The last bit of alpha is encoded in the last level's beta (dcf.cc:98-101).
  StatusOr<std::pair<DpfKey, DpfKey>> keys = dpf_->GenerateKeysIncremental(
      alpha >> 1, Span<const Value>(values->data(), values->size()));
  if (!keys.ok()) return keys.status();
  std::pair<DcfKey, DcfKey> r;
  *r.first.mutable_key() = std::move(keys->first);
  *r.second.mutable_key() = std::move(keys->second);
  return r;
}

StatusOr<std::pair<DcfKey, DcfKey>> DistributedComparisonFunction::GenerateKeysWithSeeds(
    uint128 alpha, const Value& beta, uint128 seed0, uint128 seed1) {
  StatusOr<std::vector<Value>> values = LevelBetas(alpha, beta);
  if (!values.ok()) return values.status();
  StatusOr<std::pair<DpfKey, DpfKey>> keys = dpf_->GenerateKeysIncrementalWithSeeds(
      alpha >> 1, Span<const Value>(values->data(), values->size()), seed0, seed1);
  if (!keys.ok()) return keys.status();
  std::pair<DcfKey, DcfKey> r;
  *r.first.mutable_key() = std::move(keys->first);
  *r.second.mutable_key() = std::move(keys->second);
  return r;
}

// h:141-187: EvaluateAndApply over the DPF keys with rightshift 1, summing
// level h's output where bit (n - h - 1) of the point is 0 — fused into one
// kernel launch.
Status DistributedComparisonFunction::BatchEvaluateRaw(Span<const DcfKey* const> keys,
                                                       Span<const uint128> evaluation_points,
                                                       const dpf_amd_value_type& layout,
                                                       void* out) const {
  if (keys.size() != evaluation_points.size())
    return InvalidArgumentError("`keys` and `evaluation_points` must have the same size");
  const DistributedPointFunction& dpf = *dpf_;
  const int64_t n = static_cast<int64_t>(keys.size());
  for (int64_t i = 0; i < n; ++i) DPF_RETURN_IF_ERROR(dpf.ValidateKey(keys[i]->key()));
  if (n == 0) return OkStatus();
  const int H = dpf.num_hierarchy_levels();
  const int L = dpf.hierarchy_to_tree(H - 1);
  std::vector<int32_t> tree_of(H);
  for (int h = 0; h < H; ++h) tree_of[h] = dpf.hierarchy_to_tree(h);

  // Conversion metadata of the (single) value type + the caller's layout.
  // blocks_needed can grow with the level's security parameter (40 + log
  // domain, IntModN sampling): hash the largest count at every level — a
  // level never reads past its own blocks.
  dpf_amd_value_type vt = dpf.value_type_descriptor(H - 1);
  for (int h = 0; h < H; ++h) vt.blocks_needed = std::max(vt.blocks_needed, dpf.blocks_needed(h));
  vt.out_stride = layout.out_stride;
  for (int s = 0; s < vt.num_scalars && s < layout.num_scalars; ++s)
    vt.scalars[s].out_offset = layout.scalars[s].out_offset;
  const int per = vt.elements_per_block * vt.num_scalars;

  std::vector<uint128> seeds(n), cws(static_cast<size_t>(L) * n);
  std::vector<uint8_t> cbs(n), ccl(cws.size()), ccr(cws.size());
  std::vector<int8_t> party(n);
  std::vector<uint128> corr(static_cast<size_t>(H) * n * per), tmp;
  for (int64_t i = 0; i < n; ++i) {
    const DpfKey& k = keys[i]->key();
    seeds[i] = MakeUint128(k.seed().high(), k.seed().low());
    cbs[i] = static_cast<uint8_t>(k.party() != 0);
    party[i] = static_cast<int8_t>(k.party());
    for (int a = 0; a < L; ++a) {
      const CorrectionWord& cw = k.correction_words(a);
      cws[a * n + i] = MakeUint128(cw.seed().high(), cw.seed().low());
      ccl[a * n + i] = cw.control_left();
      ccr[a * n + i] = cw.control_right();
    }
    for (int h = 0; h < H; ++h) {
      DPF_RETURN_IF_ERROR(dpf.ValueCorrectionWords(k, h, &tmp));
      if (static_cast<int>(tmp.size()) != per) return InternalError("value correction size");
      std::copy(tmp.begin(), tmp.end(), corr.begin() + (static_cast<size_t>(h) * n + i) * per);
    }
  }
  hipStream_t s = ThreadStream();
  DeviceBuffer dseeds, dcbs, dparty, dpoints, dcws, dccl, dccr, dcorr, dout;
  DPF_RETURN_IF_ERROR(dseeds.Upload(seeds.data(), 16 * n, s));
  DPF_RETURN_IF_ERROR(dcbs.Upload(cbs.data(), n, s));
  DPF_RETURN_IF_ERROR(dparty.Upload(party.data(), n, s));
  DPF_RETURN_IF_ERROR(dpoints.Upload(evaluation_points.data(), 16 * n, s));
  DPF_RETURN_IF_ERROR(dcws.Upload(cws.data(), 16 * cws.size(), s));
  DPF_RETURN_IF_ERROR(dccl.Upload(ccl.data(), ccl.size(), s));
  DPF_RETURN_IF_ERROR(dccr.Upload(ccr.data(), ccr.size(), s));
  DPF_RETURN_IF_ERROR(dcorr.Upload(corr.data(), 16 * corr.size(), s));
  DPF_RETURN_IF_ERROR(dout.Alloc(n * vt.out_stride, s));
  DPF_RETURN_IF_ERROR(ClearPadding(vt, dout.get(), n * vt.out_stride, s));
  DPF_RETURN_IF_ERROR(
      HipStatus(hipMemsetAsync(dout.get(), 0, n * vt.out_stride, s), "memset"));
  DPF_RETURN_IF_ERROR(AbiStatus(dpf_amd_dcf_evaluate(
      n, dseeds.get(), dcbs.as<uint8_t>(), dparty.as<int8_t>(), dpoints.get(), H, tree_of.data(),
      dcws.get(), dccl.as<uint8_t>(), dccr.as<uint8_t>(), &vt, dcorr.get(), dout.get(), s)));
  return CopyToHostSync(out, dout.get(), n * vt.out_stride, s);
}

}  // namespace distributed_point_functions
