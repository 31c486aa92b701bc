// capi.cc — Tier-2 C ABI (include/dpf_amd.h): the reference's public objects
// behind opaque handles, with protos exchanged in wire format.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "dpf_amd.h"
#include "dpf_amd/cuckoo_hashing_sparse_dpf_pir_server.h"
#include "dpf_amd/dense_dpf_pir_server.h"
#include "dpf_amd/distributed_comparison_function.h"
#include "host_device.h"
#include "dpf_amd/distributed_point_function.h"
#include "internal.h"

using namespace distributed_point_functions;

struct dpf_amd_dpf {
  std::unique_ptr<DistributedPointFunction> dpf;
};
struct dpf_amd_ctx {
  EvaluationContext ctx;
};
struct dpf_amd_dcf {
  std::unique_ptr<DistributedComparisonFunction> dcf;
};
struct dpf_amd_pir_db {
  std::unique_ptr<DenseDpfPirDatabase::Builder> builder =
      std::make_unique<DenseDpfPirDatabase::Builder>();
  std::unique_ptr<DenseDpfPirDatabase::Interface> built;
  const DenseDpfPirDatabase* gpu() const {
    return dynamic_cast<const DenseDpfPirDatabase*>(built.get());
  }
};
struct dpf_amd_pir_server {
  std::unique_ptr<DpfPirServer> server;
};
struct dpf_amd_cuckoo_db {
  std::unique_ptr<CuckooHashedDpfPirDatabase::Builder> builder =
      std::make_unique<CuckooHashedDpfPirDatabase::Builder>();
  std::unique_ptr<CuckooHashedDpfPirDatabase::Interface> built;
};

namespace distributed_point_functions {
namespace dpf_internal {
StatusOr<std::unique_ptr<class DpfState>> MakeDpfState(Span<const DpfParameters>);
}
}  // namespace distributed_point_functions

namespace {

int Fail(const Status& s) { return dpf_amd::SetError(s.raw_code(), s.message()); }
int Fail(int code, const std::string& m) { return dpf_amd::SetError(code, m); }

int ToBuffer(const std::string& s, uint8_t** out, size_t* len) {
  *out = static_cast<uint8_t*>(malloc(s.size() ? s.size() : 1));
  if (!*out) return Fail(DPF_AMD_RESOURCE_EXHAUSTED, "malloc failed");
  if (!s.empty()) memcpy(*out, s.data(), s.size());
  *len = s.size();
  return DPF_AMD_OK;
}

std::vector<uint128> ToU128(const uint64_t* w, int64_t n) {
  std::vector<uint128> r(n);
  for (int64_t i = 0; i < n; ++i) r[i] = MakeUint128(w[2 * i + 1], w[2 * i]);
  return r;
}

int ParseType(const uint8_t* p, size_t n, ValueType* vt) {
  if (!ParseValueType(p, n, vt)) return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed ValueType proto");
  return DPF_AMD_OK;
}

}  // namespace

extern "C" {

int dpf_amd_describe_value_type(const uint8_t* value_type_proto, size_t len,
                                double security_parameter, dpf_amd_value_type* vt) {
  DpfParameters p;
  if (!ParseValueType(value_type_proto, len, p.mutable_value_type()))
    return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed ValueType proto");
  p.set_security_parameter(security_parameter);
  StatusOr<std::unique_ptr<DistributedPointFunction>> d = DistributedPointFunction::Create(p);
  if (!d.ok()) return Fail(d.status());
  *vt = (*d)->value_type_descriptor(0);
  return DPF_AMD_OK;
}

int dpf_amd_dpf_create_incremental(const uint8_t* const* parameters, const size_t* lengths,
                                   int num_parameters, dpf_amd_dpf** out) {
  std::vector<DpfParameters> ps(num_parameters > 0 ? num_parameters : 0);
  for (int i = 0; i < num_parameters; ++i)
    if (!ParseDpfParameters(parameters[i], lengths[i], &ps[i]))
      return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed DpfParameters proto");
  StatusOr<std::unique_ptr<DistributedPointFunction>> d =
      DistributedPointFunction::CreateIncremental(Span<const DpfParameters>(ps.data(), ps.size()));
  if (!d.ok()) return Fail(d.status());
  *out = new dpf_amd_dpf{std::move(*d)};
  return DPF_AMD_OK;
}

void dpf_amd_dpf_destroy(dpf_amd_dpf* dpf) { delete dpf; }

int dpf_amd_dpf_tree_levels_needed(const dpf_amd_dpf* dpf) {
  return dpf->dpf->tree_levels_needed();
}
int dpf_amd_dpf_hierarchy_to_tree(const dpf_amd_dpf* dpf, int level) {
  return dpf->dpf->hierarchy_to_tree(level);
}
int dpf_amd_dpf_value_type(const dpf_amd_dpf* dpf, int level, dpf_amd_value_type* vt) {
  if (level < 0 || level >= dpf->dpf->num_hierarchy_levels())
    return Fail(DPF_AMD_INVALID_ARGUMENT, "level out of range");
  *vt = dpf->dpf->value_type_descriptor(level);
  return DPF_AMD_OK;
}

int dpf_amd_dpf_register_value_type(dpf_amd_dpf* dpf, const uint8_t* value_type_proto,
                                    size_t len) {
  if (!dpf) return Fail(DPF_AMD_INVALID_ARGUMENT, "null handle");
  ValueType vt;
  if (!ParseValueType(value_type_proto, len, &vt))
    return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed ValueType proto");
  Status s = dpf->dpf->RegisterValueTypeProto(vt);
  return s.ok() ? DPF_AMD_OK : Fail(s);
}

int dpf_amd_dcf_register_value_type(dpf_amd_dcf* dcf, const uint8_t* value_type_proto,
                                    size_t len) {
  if (!dcf) return Fail(DPF_AMD_INVALID_ARGUMENT, "null handle");
  ValueType vt;
  if (!ParseValueType(value_type_proto, len, &vt))
    return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed ValueType proto");
  Status s = const_cast<DistributedPointFunction&>(dcf->dcf->dpf()).RegisterValueTypeProto(vt);
  return s.ok() ? DPF_AMD_OK : Fail(s);
}

int dpf_amd_dpf_generate_keys(dpf_amd_dpf* dpf, uint64_t alpha_lo, uint64_t alpha_hi,
                              const uint8_t* const* betas, const size_t* beta_lengths,
                              const uint64_t* seeds, uint8_t** key0, size_t* key0_len,
                              uint8_t** key1, size_t* key1_len) {
  const int n = dpf->dpf->num_hierarchy_levels();
  std::vector<Value> values(n);
  for (int i = 0; i < n; ++i)
    if (!ParseValue(betas[i], beta_lengths[i], &values[i]))
      return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed Value proto");
  const uint128 alpha = MakeUint128(alpha_hi, alpha_lo);
  Span<const Value> span(values.data(), values.size());
  StatusOr<std::pair<DpfKey, DpfKey>> keys =
      seeds ? dpf->dpf->GenerateKeysIncrementalWithSeeds(alpha, span,
                                                         MakeUint128(seeds[1], seeds[0]),
                                                         MakeUint128(seeds[3], seeds[2]))
            : dpf->dpf->GenerateKeysIncremental(alpha, span);
  if (!keys.ok()) return Fail(keys.status());
  int rc = ToBuffer(keys->first.SerializeAsString(), key0, key0_len);
  if (rc != DPF_AMD_OK) return rc;
  rc = ToBuffer(keys->second.SerializeAsString(), key1, key1_len);
  if (rc != DPF_AMD_OK) free(*key0);
  return rc;
}

int dpf_amd_ctx_create(const dpf_amd_dpf* dpf, const uint8_t* key, size_t key_len,
                       dpf_amd_ctx** out) {
  DpfKey k;
  if (!k.ParseFromArray(key, key_len)) return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed DpfKey proto");
  StatusOr<EvaluationContext> ctx = dpf->dpf->CreateEvaluationContext(std::move(k));
  if (!ctx.ok()) return Fail(ctx.status());
  *out = new dpf_amd_ctx{std::move(*ctx)};
  return DPF_AMD_OK;
}

int dpf_amd_ctx_parse(const dpf_amd_dpf* dpf, const uint8_t* data, size_t len,
                      dpf_amd_ctx** out) {
  (void)dpf;
  auto c = std::make_unique<dpf_amd_ctx>();
  if (!c->ctx.ParseFromArray(data, len))
    return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed EvaluationContext proto");
  *out = c.release();
  return DPF_AMD_OK;
}

int dpf_amd_ctx_serialize(const dpf_amd_ctx* ctx, uint8_t** data, size_t* len) {
  return ToBuffer(ctx->ctx.SerializeAsString(), data, len);
}

void dpf_amd_ctx_destroy(dpf_amd_ctx* ctx) { delete ctx; }
int dpf_amd_ctx_previous_hierarchy_level(const dpf_amd_ctx* ctx) {
  return ctx->ctx.previous_hierarchy_level();
}
int dpf_amd_ctx_partial_evaluations_level(const dpf_amd_ctx* ctx) {
  return ctx->ctx.partial_evaluations_level();
}
int64_t dpf_amd_ctx_num_partial_evaluations(const dpf_amd_ctx* ctx) {
  return ctx->ctx.partial_evaluations_size();
}

static int EvaluateUntilImpl(const dpf_amd_dpf* dpf, int hierarchy_level,
                           const uint64_t* prefixes, int64_t num_prefixes,
                           const uint8_t* value_type, size_t value_type_len, dpf_amd_ctx* ctx,
                           void* out, int64_t out_capacity, int64_t* num_outputs,
                           bool out_on_device, void* stream) {
  ValueType t;
  int rc = ParseType(value_type, value_type_len, &t);
  if (rc != DPF_AMD_OK) return rc;
  Status st = dpf->dpf->CheckType(t, hierarchy_level, false);
  if (!st.ok()) return Fail(st);
  std::vector<uint128> p = ToU128(prefixes, num_prefixes);
  const int lvl = (hierarchy_level >= 0 && hierarchy_level < dpf->dpf->num_hierarchy_levels())
                      ? hierarchy_level
                      : 0;
  const dpf_amd_value_type layout = dpf->dpf->value_type_descriptor(lvl);
  // (a negative capacity passes through: the unvalidated size query)
  const int64_t cap = out_capacity < 0 ? -1
                      : layout.out_stride > 0 ? out_capacity / layout.out_stride : 0;
  st = dpf->dpf->EvaluateUntilRaw(hierarchy_level, Span<const uint128>(p.data(), p.size()),
                                  ctx->ctx, layout, out, cap, num_outputs, out_on_device, stream);
  return st.ok() ? DPF_AMD_OK : Fail(st);
}

int dpf_amd_evaluate_until(const dpf_amd_dpf* dpf, int hierarchy_level,
                           const uint64_t* prefixes, int64_t num_prefixes,
                           const uint8_t* value_type, size_t value_type_len, dpf_amd_ctx* ctx,
                           void* out, int64_t out_capacity, int64_t* num_outputs) {
  return EvaluateUntilImpl(dpf, hierarchy_level, prefixes, num_prefixes, value_type,
                           value_type_len, ctx, out, out_capacity, num_outputs, false, nullptr);
}

int dpf_amd_evaluate_until_device(const dpf_amd_dpf* dpf, int hierarchy_level,
                                  const uint64_t* prefixes, int64_t num_prefixes,
                                  const uint8_t* value_type, size_t value_type_len,
                                  dpf_amd_ctx* ctx, void* out_device, int64_t out_capacity,
                                  int64_t* num_outputs, void* stream) {
  return EvaluateUntilImpl(dpf, hierarchy_level, prefixes, num_prefixes, value_type,
                           value_type_len, ctx, out_device, out_capacity, num_outputs, true,
                           stream);
}

int dpf_amd_expand_leaves_on_devices(const dpf_amd_dpf* dpf, const uint8_t* key, size_t key_len,
                                     int num_slices, const int* devices,
                                     const int64_t* leaf_begin, const int64_t* leaf_end,
                                     void* const* outs) {
  DpfKey k;
  if (!k.ParseFromArray(key, key_len)) return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed DpfKey proto");
  if (num_slices < 0) return Fail(DPF_AMD_INVALID_ARGUMENT, "negative number of slices");
  const size_t n = static_cast<size_t>(num_slices);
  const int h = dpf->dpf->num_hierarchy_levels() - 1;
  Status st = dpf->dpf->ExpandLeavesOnDevices(
      k, Span<const int>(devices, n), Span<const int64_t>(leaf_begin, n),
      Span<const int64_t>(leaf_end, n), Span<void* const>(outs, n),
      dpf->dpf->value_type_descriptor(h));
  return st.ok() ? DPF_AMD_OK : Fail(st);
}

int dpf_amd_evaluate_at(const dpf_amd_dpf* dpf, const uint8_t* key, size_t key_len,
                        int hierarchy_level, const uint64_t* points, int64_t num_points,
                        const uint8_t* value_type, size_t value_type_len, void* out) {
  DpfKey k;
  if (!k.ParseFromArray(key, key_len)) return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed DpfKey proto");
  ValueType t;
  int rc = ParseType(value_type, value_type_len, &t);
  if (rc != DPF_AMD_OK) return rc;
  Status st = dpf->dpf->CheckType(t, hierarchy_level, true);
  if (!st.ok()) return Fail(st);
  std::vector<uint128> p = ToU128(points, num_points);
  const int lvl = (hierarchy_level >= 0 && hierarchy_level < dpf->dpf->num_hierarchy_levels())
                      ? hierarchy_level
                      : 0;
  st = dpf->dpf->EvaluateAtRaw(k, hierarchy_level, Span<const uint128>(p.data(), p.size()),
                               nullptr, dpf->dpf->value_type_descriptor(lvl), out);
  return st.ok() ? DPF_AMD_OK : Fail(st);
}

int dpf_amd_evaluate_at_ctx(const dpf_amd_dpf* dpf, int hierarchy_level, const uint64_t* points,
                            int64_t num_points, const uint8_t* value_type, size_t value_type_len,
                            dpf_amd_ctx* ctx, void* out) {
  if (!dpf || !ctx) return Fail(DPF_AMD_INVALID_ARGUMENT, "null handle");
  ValueType t;
  int rc = ParseType(value_type, value_type_len, &t);
  if (rc != DPF_AMD_OK) return rc;
  Status st = dpf->dpf->CheckType(t, hierarchy_level, true);
  if (!st.ok()) return Fail(st);
  std::vector<uint128> p = ToU128(points, num_points);
  const int lvl = (hierarchy_level >= 0 && hierarchy_level < dpf->dpf->num_hierarchy_levels())
                      ? hierarchy_level
                      : 0;
  st = dpf->dpf->EvaluateAtRaw(ctx->ctx.key(), hierarchy_level,
                               Span<const uint128>(p.data(), p.size()), &ctx->ctx,
                               dpf->dpf->value_type_descriptor(lvl), out);
  return st.ok() ? DPF_AMD_OK : Fail(st);
}

int dpf_amd_evaluate_and_apply(const dpf_amd_dpf* dpf, const uint8_t* const* keys,
                               const size_t* key_lengths, int64_t num_keys,
                               const uint64_t* points, int rightshift,
                               const uint8_t* value_type, size_t value_type_len, void* out,
                               dpf_amd_apply_fn op, void* user) {
  // A key buffer passed for several points (same address and length) is
  // parsed once, and the points share one DpfKey object (which the library
  // uploads once).
  std::vector<DpfKey> ks;
  ks.reserve(num_keys);
  std::vector<const DpfKey*> ptrs(num_keys);
  std::vector<int64_t> which(num_keys);
  {
    std::map<std::pair<const uint8_t*, size_t>, int64_t> parsed;
    for (int64_t i = 0; i < num_keys; ++i) {
      auto ins = parsed.emplace(std::make_pair(keys[i], key_lengths[i]),
                                static_cast<int64_t>(ks.size()));
      if (ins.second) {
        ks.emplace_back();
        if (!ks.back().ParseFromArray(keys[i], key_lengths[i]))
          return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed DpfKey proto");
      }
      which[i] = ins.first->second;
    }
  }
  for (int64_t i = 0; i < num_keys; ++i) ptrs[i] = &ks[which[i]];
  ValueType t;
  int rc = ParseType(value_type, value_type_len, &t);
  if (rc != DPF_AMD_OK) return rc;
  Status st = dpf->dpf->CheckType(t, -1, true);
  if (!st.ok()) return Fail(st);
  std::vector<uint128> p = ToU128(points, num_keys);
  int done = 0;
  struct Ctx {
    dpf_amd_apply_fn op;
    void* user;
    const char* out;
    int64_t n;
    int64_t stride;
  } ctx{op, user, static_cast<const char*>(out), num_keys,
        dpf->dpf->value_type_descriptor(0).out_stride};
  auto on_level = [](void* u, int h) -> bool {
    Ctx* c = static_cast<Ctx*>(u);
    return c->op(c->user, h, c->out + h * c->n * c->stride, c->n) != 0;
  };
  st = dpf->dpf->EvaluateAndApplyRaw(Span<const DpfKey* const>(ptrs.data(), ptrs.size()),
                                     Span<const uint128>(p.data(), p.size()), rightshift,
                                     dpf->dpf->value_type_descriptor(0), out, &done,
                                     op ? +on_level : nullptr, &ctx);
  return st.ok() ? DPF_AMD_OK : Fail(st);
}

// --- PIR ---------------------------------------------------------------------

// --- DistributedComparisonFunction (dcf/distributed_comparison_function.h) ---

int dpf_amd_dcf_create(const uint8_t* parameters, size_t len, dpf_amd_dcf** out) {
  DcfParameters p;
  if (!p.ParseFromArray(parameters, len))
    return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed DcfParameters proto");
  StatusOr<std::unique_ptr<DistributedComparisonFunction>> d =
      DistributedComparisonFunction::Create(p);
  if (!d.ok()) return Fail(d.status());
  *out = new dpf_amd_dcf{std::move(*d)};
  return DPF_AMD_OK;
}

void dpf_amd_dcf_destroy(dpf_amd_dcf* dcf) { delete dcf; }

int dpf_amd_dcf_generate_keys(dpf_amd_dcf* dcf, uint64_t alpha_lo, uint64_t alpha_hi,
                              const uint8_t* beta, size_t beta_len, const uint64_t* seeds,
                              uint8_t** key0, size_t* key0_len, uint8_t** key1,
                              size_t* key1_len) {
  Value b;
  if (!ParseValue(beta, beta_len, &b)) return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed Value proto");
  const uint128 alpha = MakeUint128(alpha_hi, alpha_lo);
  StatusOr<std::pair<DcfKey, DcfKey>> keys =
      seeds ? dcf->dcf->GenerateKeysWithSeeds(alpha, b, MakeUint128(seeds[1], seeds[0]),
                                              MakeUint128(seeds[3], seeds[2]))
            : dcf->dcf->GenerateKeys(alpha, b);
  if (!keys.ok()) return Fail(keys.status());
  int rc = ToBuffer(keys->first.SerializeAsString(), key0, key0_len);
  if (rc != DPF_AMD_OK) return rc;
  rc = ToBuffer(keys->second.SerializeAsString(), key1, key1_len);
  if (rc != DPF_AMD_OK) free(*key0);
  return rc;
}

int dpf_amd_dcf_batch_evaluate(const dpf_amd_dcf* dcf, const uint8_t* const* keys,
                               const size_t* key_lengths, int64_t num_keys,
                               const uint64_t* points, int64_t num_points,
                               const uint8_t* value_type, size_t value_type_len, void* out) {
  if (num_keys != num_points)
    return Fail(DPF_AMD_INVALID_ARGUMENT, "`keys` and `evaluation_points` must have the same size");
  std::vector<DcfKey> ks(num_keys);
  std::vector<const DcfKey*> ptrs(num_keys);
  for (int64_t i = 0; i < num_keys; ++i) {
    if (!ks[i].ParseFromArray(keys[i], key_lengths[i]))
      return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed DcfKey proto");
    ptrs[i] = &ks[i];
  }
  ValueType t;
  int rc = ParseType(value_type, value_type_len, &t);
  if (rc != DPF_AMD_OK) return rc;
  const DistributedPointFunction& dpf = dcf->dcf->dpf();
  Status st = dpf.CheckType(t, -1, true);
  if (!st.ok()) return Fail(st);
  std::vector<uint128> p = ToU128(points, num_points);
  st = dcf->dcf->BatchEvaluateRaw(Span<const DcfKey* const>(ptrs.data(), ptrs.size()),
                                  Span<const uint128>(p.data(), p.size()),
                                  dpf.value_type_descriptor(dpf.num_hierarchy_levels() - 1), out);
  return st.ok() ? DPF_AMD_OK : Fail(st);
}

int dpf_amd_pir_db_create(dpf_amd_pir_db** out) {
  *out = new dpf_amd_pir_db();
  return DPF_AMD_OK;
}

int dpf_amd_pir_db_insert(dpf_amd_pir_db* db, const uint8_t* record, size_t len) {
  if (!db->builder) return Fail(DPF_AMD_FAILED_PRECONDITION, "Database already built");
  db->builder->Insert(std::string(reinterpret_cast<const char*>(record), len));
  return DPF_AMD_OK;
}

int dpf_amd_pir_db_insert_fixed(dpf_amd_pir_db* db, const uint8_t* records, int64_t num_records,
                                int64_t record_size) {
  if (!db->builder) return Fail(DPF_AMD_FAILED_PRECONDITION, "Database already built");
  db->builder->InsertFixed(reinterpret_cast<const char*>(records), num_records, record_size);
  return DPF_AMD_OK;
}

int dpf_amd_pir_db_insert_packed(dpf_amd_pir_db* db, const uint8_t* data, const int64_t* sizes,
                                 int64_t num_records) {
  if (!db->builder) return Fail(DPF_AMD_FAILED_PRECONDITION, "Database already built");
  if (num_records < 0 || (num_records > 0 && (sizes == nullptr)))
    return Fail(DPF_AMD_INVALID_ARGUMENT, "bad packed records");
  int64_t total = 0;
  for (int64_t i = 0; i < num_records; ++i) {
    if (sizes[i] < 0) return Fail(DPF_AMD_INVALID_ARGUMENT, "negative record size");
    total += sizes[i];
  }
  if (total > 0 && data == nullptr) return Fail(DPF_AMD_INVALID_ARGUMENT, "bad packed records");
  const char* p = reinterpret_cast<const char*>(data);
  for (int64_t i = 0; i < num_records; ++i) {  // Builder::Insert per record, in order
    db->builder->Insert(std::string(p, static_cast<size_t>(sizes[i])));
    p += sizes[i];
  }
  return DPF_AMD_OK;
}

int dpf_amd_pir_db_build(dpf_amd_pir_db* db) {
  if (!db->builder) return Fail(DPF_AMD_FAILED_PRECONDITION, "Database already built");
  StatusOr<std::unique_ptr<DenseDpfPirDatabase::Interface>> b = db->builder->Build();
  if (!b.ok()) return Fail(b.status());
  db->built = std::move(*b);
  db->builder.reset();
  return DPF_AMD_OK;
}

void dpf_amd_pir_db_destroy(dpf_amd_pir_db* db) { delete db; }

int dpf_amd_release_cached_memory(int64_t* released) {
  auto& pool = dpf_internal_host::DevicePool::Get();
  const size_t before = pool.cached_bytes();
  pool.Release();
  if (released) *released = static_cast<int64_t>(before - pool.cached_bytes());
  return DPF_AMD_OK;
}

int dpf_amd_pir_db_insert_fixed_device(dpf_amd_pir_db* db, const void* records, int device,
                                       int64_t num_records, int64_t record_size) {
  if (!db->builder) return Fail(DPF_AMD_FAILED_PRECONDITION, "Database already built");
  if (num_records < 0 || record_size < 0 || (num_records > 0 && records == nullptr))
    return Fail(DPF_AMD_INVALID_ARGUMENT, "bad device records");
  db->builder->InsertFixedFromDevice(records, device, num_records, record_size);
  return DPF_AMD_OK;
}

int dpf_amd_pir_db_set_devices(dpf_amd_pir_db* db, const int* devices, int num_devices) {
  if (!db->builder) return Fail(DPF_AMD_FAILED_PRECONDITION, "Database already built");
  if (num_devices < 0 || (num_devices > 0 && devices == nullptr))
    return Fail(DPF_AMD_INVALID_ARGUMENT, "bad device list");
  int count = 0;
  if (num_devices > 0 && hipGetDeviceCount(&count) != hipSuccess)
    return Fail(DPF_AMD_INTERNAL, "hipGetDeviceCount failed");
  for (int i = 0; i < num_devices; ++i)
    if (devices[i] < 0 || devices[i] >= count)
      return Fail(DPF_AMD_INVALID_ARGUMENT, "device " + std::to_string(devices[i]) +
                                                " out of range [0, " + std::to_string(count) + ")");
  db->builder->SetDevices(std::vector<int>(devices, devices + num_devices));
  return DPF_AMD_OK;
}

int dpf_amd_pir_db_num_shards(const dpf_amd_pir_db* db) {
  return db->gpu() ? static_cast<int>(db->gpu()->shards().size()) : 0;
}

int dpf_amd_pir_db_shard(const dpf_amd_pir_db* db, int shard, int* device, int64_t* row_begin,
                         int64_t* row_end, const void** records) {
  if (!db->gpu()) return Fail(DPF_AMD_FAILED_PRECONDITION, "database not built");
  const auto& sh = db->gpu()->shards();
  if (shard < 0 || shard >= static_cast<int>(sh.size()))
    return Fail(DPF_AMD_INVALID_ARGUMENT, "shard out of range");
  if (device) *device = sh[shard].device;
  if (row_begin) *row_begin = sh[shard].row_begin;
  if (row_end) *row_end = sh[shard].row_end;
  if (records) *records = sh[shard].records;
  return DPF_AMD_OK;
}

int64_t dpf_amd_pir_db_size(const dpf_amd_pir_db* db) {
  return db->built ? static_cast<int64_t>(db->built->size()) : 0;
}
int64_t dpf_amd_pir_db_max_value_size(const dpf_amd_pir_db* db) {
  return db->gpu() ? static_cast<int64_t>(db->gpu()->max_value_size_in_bytes()) : 0;
}
const void* dpf_amd_pir_db_device_records(const dpf_amd_pir_db* db, int64_t* record_stride) {
  if (!db->gpu()) return nullptr;
  *record_stride = db->gpu()->record_stride();
  return db->gpu()->device_records();
}

int dpf_amd_pir_db_inner_product(const dpf_amd_pir_db* db, const uint64_t* selections,
                                 int64_t selection_blocks, int num_queries, uint8_t* out) {
  if (!db->gpu()) return Fail(DPF_AMD_FAILED_PRECONDITION, "database not built");
  std::vector<std::vector<XorWrapper<uint128>>> sel(num_queries);
  for (int q = 0; q < num_queries; ++q) {
    sel[q].resize(selection_blocks);
    for (int64_t b = 0; b < selection_blocks; ++b) {
      const uint64_t* w = selections + 2 * (q * selection_blocks + b);
      sel[q][b] = XorWrapper<uint128>(MakeUint128(w[1], w[0]));
    }
  }
  StatusOr<std::vector<std::string>> r = db->built->InnerProductWith(
      Span<const std::vector<XorWrapper<uint128>>>(sel.data(), sel.size()));
  if (!r.ok()) return Fail(r.status());
  size_t off = 0;
  for (const std::string& s : *r) {
    memcpy(out + off, s.data(), s.size());
    off += s.size();
  }
  return DPF_AMD_OK;
}

}  // extern "C"

struct dpf_amd_pir_call {
  std::function<void()>* while_waiting = nullptr;
  bool waited = false;
  bool has_response = false;
  std::string response;
};

namespace {

// Shared by the three factories: parses the config, finishes the database.
int PrepareServer(const uint8_t* config, size_t config_len, dpf_amd_pir_db* db, PirConfig* c,
                  std::unique_ptr<DenseDpfPirServer::Database>* d) {
  if (!c->ParseFromArray(config, config_len)) {
    delete db;
    return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed PirConfig proto");
  }
  if (db && !db->built) {
    int rc = dpf_amd_pir_db_build(db);
    if (rc != DPF_AMD_OK) {
      delete db;
      return rc;
    }
  }
  if (db) *d = std::move(db->built);
  delete db;
  return DPF_AMD_OK;
}

template <typename Server>
int Finish(StatusOr<std::unique_ptr<Server>> s, dpf_amd_pir_server** out) {
  if (!s.ok()) return Fail(s.status());
  *out = new dpf_amd_pir_server{std::move(*s)};
  return DPF_AMD_OK;
}

Status CallbackStatus(int rc, const char* what) {
  return Status(static_cast<StatusCode>(rc == DPF_AMD_OK ? DPF_AMD_INTERNAL : rc),
                std::string(what) + " callback failed with status " + std::to_string(rc));
}

DpfPirServer::ForwardHelperRequestFn MakeSender(dpf_amd_pir_forward_fn forward, void* user) {
  DpfPirServer::ForwardHelperRequestFn sender;
  if (forward) {
    sender = [forward, user](const PirRequest& helper_request,
                             std::function<void()> while_waiting) -> StatusOr<PirResponse> {
      const std::string req = helper_request.SerializeAsString();
      dpf_amd_pir_call call;
      call.while_waiting = &while_waiting;
      int frc = forward(reinterpret_cast<const uint8_t*>(req.data()), req.size(), &call, user);
      if (frc != DPF_AMD_OK) return CallbackStatus(frc, "ForwardHelperRequestFn");
      if (!call.has_response)
        return Status(StatusCode::kInternal, "ForwardHelperRequestFn returned no response");
      PirResponse resp;
      if (!resp.ParseFromArray(call.response.data(), call.response.size()))
        return Status(StatusCode::kInternal, "malformed PirResponse from the Helper");
      return resp;
    };
  }
  return sender;
}

DpfPirServer::DecryptHelperRequestFn MakeDecrypter(dpf_amd_pir_decrypt_fn decrypt, void* user) {
  DpfPirServer::DecryptHelperRequestFn decrypter;
  if (decrypt) {
    decrypter = [decrypt, user](const std::string& ciphertext,
                                const std::string& info) -> StatusOr<std::string> {
      dpf_amd_pir_call call;
      int drc = decrypt(reinterpret_cast<const uint8_t*>(ciphertext.data()), ciphertext.size(),
                        reinterpret_cast<const uint8_t*>(info.data()), info.size(), &call, user);
      if (drc != DPF_AMD_OK) return CallbackStatus(drc, "DecryptHelperRequestFn");
      if (!call.has_response)
        return Status(StatusCode::kInternal, "DecryptHelperRequestFn returned no plaintext");
      return call.response;
    };
  }
  return decrypter;
}

}  // namespace

extern "C" {

int dpf_amd_pir_call_while_waiting(dpf_amd_pir_call* call) {
  if (!call || !call->while_waiting)
    return Fail(DPF_AMD_FAILED_PRECONDITION, "no `while_waiting` for this call");
  if (call->waited) return Fail(DPF_AMD_FAILED_PRECONDITION, "`while_waiting` already called");
  call->waited = true;
  (*call->while_waiting)();
  return DPF_AMD_OK;
}

int dpf_amd_pir_call_set_response(dpf_amd_pir_call* call, const uint8_t* data, size_t len) {
  if (!call) return Fail(DPF_AMD_INVALID_ARGUMENT, "null call");
  call->response.assign(reinterpret_cast<const char*>(data), len);
  call->has_response = true;
  return DPF_AMD_OK;
}

int dpf_amd_pir_server_create_plain(const uint8_t* config, size_t config_len, dpf_amd_pir_db* db,
                                    dpf_amd_pir_server** out) {
  PirConfig c;
  std::unique_ptr<DenseDpfPirServer::Database> d;
  int rc = PrepareServer(config, config_len, db, &c, &d);
  if (rc != DPF_AMD_OK) return rc;
  return Finish(DenseDpfPirServer::CreatePlain(c, std::move(d)), out);
}

int dpf_amd_pir_server_create_leader(const uint8_t* config, size_t config_len, dpf_amd_pir_db* db,
                                     dpf_amd_pir_forward_fn forward, void* user,
                                     dpf_amd_pir_server** out) {
  PirConfig c;
  std::unique_ptr<DenseDpfPirServer::Database> d;
  int rc = PrepareServer(config, config_len, db, &c, &d);
  if (rc != DPF_AMD_OK) return rc;
  DpfPirServer::ForwardHelperRequestFn sender = MakeSender(forward, user);
  return Finish(DenseDpfPirServer::CreateLeader(c, std::move(d), std::move(sender)), out);
}

int dpf_amd_pir_server_create_helper(const uint8_t* config, size_t config_len, dpf_amd_pir_db* db,
                                     dpf_amd_pir_decrypt_fn decrypt, void* user,
                                     dpf_amd_pir_server** out) {
  PirConfig c;
  std::unique_ptr<DenseDpfPirServer::Database> d;
  int rc = PrepareServer(config, config_len, db, &c, &d);
  if (rc != DPF_AMD_OK) return rc;
  DpfPirServer::DecryptHelperRequestFn decrypter = MakeDecrypter(decrypt, user);
  return Finish(DenseDpfPirServer::CreateHelper(c, std::move(d), std::move(decrypter)), out);
}

void dpf_amd_pir_server_destroy(dpf_amd_pir_server* server) { delete server; }

int dpf_amd_pir_server_handle_request(const dpf_amd_pir_server* server, const uint8_t* request,
                                      size_t request_len, uint8_t** response,
                                      size_t* response_len) {
  PirRequest r;
  if (!r.ParseFromArray(request, request_len))
    return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed PirRequest proto");
  StatusOr<PirResponse> resp = server->server->HandleRequest(r);
  if (!resp.ok()) return Fail(resp.status());
  return ToBuffer(resp->SerializeAsString(), response, response_len);
}


/* ---- Cuckoo-hashed sparse PIR ---- */

int dpf_amd_sha256_hash(const uint8_t* seed, size_t seed_len, const uint8_t* input,
                        size_t input_len, int upper_bound, int* out) {
  if (upper_bound <= 0) return Fail(DPF_AMD_INVALID_ARGUMENT, "`upper_bound` must be positive");
  SHA256HashFunction h(std::string(reinterpret_cast<const char*>(seed), seed_len));
  *out = h(std::string(reinterpret_cast<const char*>(input), input_len), upper_bound);
  return DPF_AMD_OK;
}

int dpf_amd_hash_family_evaluate(const uint8_t* hash_family_config, size_t config_len,
                                 int num_hash_functions, const uint8_t* input, size_t input_len,
                                 int upper_bound, int* out) {
  HashFamilyConfig c;
  if (!c.ParseFromArray(hash_family_config, config_len))
    return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed HashFamilyConfig proto");
  if (upper_bound <= 0) return Fail(DPF_AMD_INVALID_ARGUMENT, "`upper_bound` must be positive");
  StatusOr<HashFamily> family = CreateHashFamilyFromConfig(c);
  if (!family.ok()) return Fail(family.status());
  StatusOr<std::vector<HashFunction>> fns = CreateHashFunctions(*family, num_hash_functions);
  if (!fns.ok()) return Fail(fns.status());
  const std::string in(reinterpret_cast<const char*>(input), input_len);
  for (int i = 0; i < num_hash_functions; ++i) out[i] = (*fns)[i](in, upper_bound);
  return DPF_AMD_OK;
}

int dpf_amd_cuckoo_generate_params(const uint8_t* config, size_t config_len, uint8_t** params,
                                   size_t* params_len) {
  PirConfig c;
  if (!c.ParseFromArray(config, config_len))
    return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed PirConfig proto");
  StatusOr<CuckooHashingParams> p = CuckooHashingSparseDpfPirServer::GenerateParams(c);
  if (!p.ok()) return Fail(p.status());
  return ToBuffer(p->SerializeAsString(), params, params_len);
}

int dpf_amd_cuckoo_db_create(const uint8_t* params, size_t params_len, dpf_amd_cuckoo_db** out) {
  CuckooHashingParams p;
  if (!p.ParseFromArray(params, params_len))
    return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed CuckooHashingParams proto");
  *out = new dpf_amd_cuckoo_db();
  (*out)->builder->SetParams(std::move(p));
  return DPF_AMD_OK;
}

int dpf_amd_cuckoo_db_insert(dpf_amd_cuckoo_db* db, const uint8_t* key, size_t key_len,
                             const uint8_t* value, size_t value_len) {
  if (db->built) return Fail(DPF_AMD_FAILED_PRECONDITION, "Database already built");
  db->builder->Insert({std::string(reinterpret_cast<const char*>(key), key_len),
                       std::string(reinterpret_cast<const char*>(value), value_len)});
  return DPF_AMD_OK;
}

int dpf_amd_cuckoo_db_place(const dpf_amd_cuckoo_db* db, int64_t* bucket_key_lengths,
                            int64_t num_buckets) {
  StatusOr<std::vector<std::optional<std::string>>> t = db->builder->PlaceKeys();
  if (!t.ok()) return Fail(t.status());
  if (static_cast<int64_t>(t->size()) != num_buckets)
    return Fail(DPF_AMD_INVALID_ARGUMENT, "`num_buckets` does not match the params");
  for (int64_t i = 0; i < num_buckets; ++i)
    bucket_key_lengths[i] = (*t)[i] ? static_cast<int64_t>((*t)[i]->size()) : -1;
  return DPF_AMD_OK;
}

int dpf_amd_cuckoo_db_place_keys(const dpf_amd_cuckoo_db* db, uint8_t* keys, size_t keys_len) {
  StatusOr<std::vector<std::optional<std::string>>> t = db->builder->PlaceKeys();
  if (!t.ok()) return Fail(t.status());
  size_t off = 0;
  for (const auto& b : *t) {
    if (!b) continue;
    if (off + b->size() > keys_len) return Fail(DPF_AMD_INVALID_ARGUMENT, "`keys` too small");
    memcpy(keys + off, b->data(), b->size());
    off += b->size();
  }
  return DPF_AMD_OK;
}

int dpf_amd_cuckoo_db_build(dpf_amd_cuckoo_db* db) {
  StatusOr<std::unique_ptr<CuckooHashedDpfPirDatabase::Interface>> b = db->builder->Build();
  if (!b.ok()) return Fail(b.status());
  db->built = std::move(*b);
  return DPF_AMD_OK;
}

void dpf_amd_cuckoo_db_destroy(dpf_amd_cuckoo_db* db) { delete db; }

int64_t dpf_amd_cuckoo_db_size(const dpf_amd_cuckoo_db* db) {
  return db->built ? static_cast<int64_t>(db->built->size()) : -1;
}

int64_t dpf_amd_cuckoo_db_num_selection_bits(const dpf_amd_cuckoo_db* db) {
  return db->built ? static_cast<int64_t>(db->built->num_selection_bits()) : -1;
}

namespace {
int PrepareCuckoo(const uint8_t* params, size_t params_len, dpf_amd_cuckoo_db* db,
                  CuckooHashingParams* p,
                  std::unique_ptr<CuckooHashingSparseDpfPirServer::Database>* d) {
  if (!p->ParseFromArray(params, params_len)) {
    delete db;
    return Fail(DPF_AMD_INVALID_ARGUMENT, "malformed CuckooHashingParams proto");
  }
  if (db && !db->built) {
    int rc = dpf_amd_cuckoo_db_build(db);
    if (rc != DPF_AMD_OK) {
      delete db;
      return rc;
    }
  }
  if (db) *d = std::move(db->built);
  delete db;
  return DPF_AMD_OK;
}
}  // namespace

int dpf_amd_cuckoo_server_create_plain(const uint8_t* params, size_t params_len,
                                       dpf_amd_cuckoo_db* db, dpf_amd_pir_server** out) {
  CuckooHashingParams p;
  std::unique_ptr<CuckooHashingSparseDpfPirServer::Database> d;
  int rc = PrepareCuckoo(params, params_len, db, &p, &d);
  if (rc != DPF_AMD_OK) return rc;
  return Finish(CuckooHashingSparseDpfPirServer::CreatePlain(std::move(p), std::move(d)), out);
}

int dpf_amd_cuckoo_server_create_leader(const uint8_t* params, size_t params_len,
                                        dpf_amd_cuckoo_db* db, dpf_amd_pir_forward_fn forward,
                                        void* user, dpf_amd_pir_server** out) {
  CuckooHashingParams p;
  std::unique_ptr<CuckooHashingSparseDpfPirServer::Database> d;
  int rc = PrepareCuckoo(params, params_len, db, &p, &d);
  if (rc != DPF_AMD_OK) return rc;
  return Finish(CuckooHashingSparseDpfPirServer::CreateLeader(std::move(p), std::move(d),
                                                             MakeSender(forward, user)),
                out);
}

int dpf_amd_cuckoo_server_create_helper(const uint8_t* params, size_t params_len,
                                        dpf_amd_cuckoo_db* db, dpf_amd_pir_decrypt_fn decrypt,
                                        void* user, dpf_amd_pir_server** out) {
  CuckooHashingParams p;
  std::unique_ptr<CuckooHashingSparseDpfPirServer::Database> d;
  int rc = PrepareCuckoo(params, params_len, db, &p, &d);
  if (rc != DPF_AMD_OK) return rc;
  return Finish(CuckooHashingSparseDpfPirServer::CreateHelper(std::move(p), std::move(d),
                                                             MakeDecrypter(decrypt, user)),
                out);
}

int dpf_amd_pir_server_public_params(const dpf_amd_pir_server* server, uint8_t** params,
                                     size_t* params_len) {
  return ToBuffer(server->server->GetPublicParams().SerializeAsString(), params, params_len);
}

}  // extern "C"
