// pir.cc — dense DPF PIR server and HBM-resident database (see
// include/dpf_amd/dense_dpf_pir_server.h for the reference mapping).
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <cmath>

#include "dpf_amd/dense_dpf_pir_server.h"
#include "host_aes.h"
#include "host_device.h"
#include "internal.h"

namespace distributed_point_functions {
namespace {

Status HipStatus(hipError_t e, const char* what) {
  if (e == hipSuccess) return OkStatus();
  if (e == hipErrorOutOfMemory)
    return ResourceExhaustedError(std::string(what) + ": " + hipGetErrorString(e));
  return InternalError(std::string(what) + ": " + hipGetErrorString(e));
}

Status AbiStatus(int rc) {
  if (rc == DPF_AMD_OK) return OkStatus();
  return Status(static_cast<StatusCode>(rc), dpf_amd::LastError());
}

hipStream_t PirStream() {
  thread_local hipStream_t s = [] {
    hipStream_t x = nullptr;
    if (hipStreamCreateWithFlags(&x, hipStreamNonBlocking) != hipSuccess) x = nullptr;
    return x;
  }();
  return s;
}

// AlignBytes (pir/dense_dpf_pir_database.cc:40-52).
int64_t AlignBytes(int64_t n) { return (n + 15) & ~int64_t{15}; }


}  // namespace

// ---------------------------------------------------------------------------
// DenseDpfPirDatabase
// ---------------------------------------------------------------------------

DenseDpfPirDatabase::Builder::Builder() = default;

DenseDpfPirDatabase::Builder& DenseDpfPirDatabase::Builder::Insert(std::string value) {
  if (fixed_count_ > 0) {  // keep insertion order: materialise bulk records first
    for (int64_t i = 0; i < fixed_count_; ++i)
      values_.emplace_back(fixed_.data() + i * fixed_size_, fixed_size_);
    std::vector<char>().swap(fixed_);
    fixed_count_ = 0;
  }
  total_database_bytes_ += AlignBytes(static_cast<int64_t>(value.size()));
  values_.push_back(std::move(value));
  return *this;
}

DenseDpfPirDatabase::Builder& DenseDpfPirDatabase::Builder::InsertFixed(const char* data,
                                                                        int64_t num,
                                                                        int64_t size) {
  if (fixed_count_ == 0) fixed_size_ = size;
  if (!values_.empty() || size != fixed_size_) {
    for (int64_t i = 0; i < num; ++i) Insert(std::string(data + i * size, size));
    return *this;
  }
  fixed_.insert(fixed_.end(), data, data + num * size);
  fixed_count_ += num;
  total_database_bytes_ += num * AlignBytes(size);
  return *this;
}

std::unique_ptr<DenseDpfPirDatabase::Interface::Builder> DenseDpfPirDatabase::Builder::Clone()
    const {
  auto r = std::make_unique<Builder>();
  r->values_ = values_;
  r->fixed_ = fixed_;
  r->fixed_count_ = fixed_count_;
  r->fixed_size_ = fixed_size_;
  r->total_database_bytes_ = total_database_bytes_;
  r->has_been_built_ = has_been_built_;
  return r;
}

StatusOr<std::unique_ptr<DenseDpfPirDatabase::Interface>> DenseDpfPirDatabase::Builder::Build() {
  if (has_been_built_) return FailedPreconditionError("Database already built");
  has_been_built_ = true;
  std::unique_ptr<DenseDpfPirDatabase> db(new DenseDpfPirDatabase());
  const int64_t n = static_cast<int64_t>(values_.size()) + fixed_count_;
  int64_t max_size = fixed_count_ ? fixed_size_ : 0;
  for (const std::string& v : values_) max_size = std::max<int64_t>(max_size, v.size());
  db->num_records_ = n;
  db->max_value_size_ = max_size;
  // Device row stride: the reference's 16-byte alignment (KPirScanG maps any
  // width onto the wave, so no padding is read or stored).
  db->stride_ = std::max<int64_t>(16, AlignBytes(max_size));
  const int64_t bytes = std::max<int64_t>(16, n * db->stride_);
  hipError_t e = hipMalloc(&db->records_, bytes);
  if (e == hipErrorOutOfMemory) {
    // idle blocks cached by earlier Tier-2 calls go back to the device first
    (void)hipGetLastError();
    dpf_internal_host::DevicePool::Get().Release();
    e = hipMalloc(&db->records_, bytes);
  }
  DPF_RETURN_IF_ERROR(HipStatus(e, "hipMalloc(database)"));
  DPF_RETURN_IF_ERROR(HipStatus(hipMemset(db->records_, 0, bytes), "hipMemset(database)"));
  // Upload in 64 MiB chunks of zero-padded fixed-stride rows.
  const int64_t rows_per_chunk = std::max<int64_t>(1, (64 << 20) / db->stride_);
  std::vector<char> chunk(rows_per_chunk * db->stride_);
  int64_t row = 0;
  auto flush = [&](int64_t rows) -> Status {
    if (rows == 0) return OkStatus();
    Status s = HipStatus(hipMemcpy(static_cast<char*>(db->records_) + (row - rows) * db->stride_,
                                   chunk.data(), rows * db->stride_, hipMemcpyHostToDevice),
                         "upload database");
    std::fill(chunk.begin(), chunk.end(), 0);
    return s;
  };
  int64_t in_chunk = 0;
  for (int64_t i = 0; i < n; ++i) {
    const char* src;
    int64_t len;
    if (i < static_cast<int64_t>(values_.size())) {
      src = values_[i].data();
      len = static_cast<int64_t>(values_[i].size());
    } else {
      const int64_t j = i - static_cast<int64_t>(values_.size());
      src = fixed_.data() + j * fixed_size_;
      len = fixed_size_;
    }
    memcpy(chunk.data() + in_chunk * db->stride_, src, len);
    ++in_chunk;
    ++row;
    if (in_chunk == rows_per_chunk) {
      DPF_RETURN_IF_ERROR(flush(in_chunk));
      in_chunk = 0;
    }
  }
  DPF_RETURN_IF_ERROR(flush(in_chunk));
  std::vector<std::string>().swap(values_);
  std::vector<char>().swap(fixed_);
  return std::unique_ptr<Interface>(std::move(db));
}

DenseDpfPirDatabase::~DenseDpfPirDatabase() {
  if (records_) (void)hipFree(records_);
}

StatusOr<std::vector<std::string>> DenseDpfPirDatabase::InnerProductWithDevice(
    const void* selections_dev, int64_t selection_blocks, int num_queries, void* stream) const {
  if (num_queries == 0) return std::vector<std::string>();
  if (max_value_size_ <= 0) return InvalidArgumentError("`max_value_size` must be positive");
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : PirStream();
  const int64_t ws = dpf_amd_inner_product_workspace_size(num_records_, stride_, num_queries);
  void* work = nullptr;
  void* out = nullptr;
  DPF_RETURN_IF_ERROR(dpf_internal_host::DevicePool::Get().Alloc(std::max<int64_t>(ws, 16), s, &work));
  Status st = dpf_internal_host::DevicePool::Get().Alloc(num_queries * stride_, s, &out);
  std::vector<char> host(num_queries * stride_);
  if (st.ok())
    st = AbiStatus(dpf_amd_inner_product(records_, num_records_, stride_, selections_dev,
                                         selection_blocks, num_queries, work, out, s));
  if (st.ok())
    st = HipStatus(hipMemcpyAsync(host.data(), out, host.size(), hipMemcpyDeviceToHost, s), "d2h");
  dpf_internal_host::DevicePool::Get().Free(work, s);
  if (out) dpf_internal_host::DevicePool::Get().Free(out, s);
  Status sync = HipStatus(hipStreamSynchronize(s), "sync");
  if (!st.ok()) return st;
  if (!sync.ok()) return sync;
  std::vector<std::string> r(num_queries);
  for (int q = 0; q < num_queries; ++q) r[q].assign(host.data() + q * stride_, max_value_size_);
  return r;
}

StatusOr<std::vector<std::string>> DenseDpfPirDatabase::InnerProductWith(
    Span<const std::vector<BlockType>> selections) const {
  // Validation of pir_internal::InnerProduct (inner_product_hwy.cc:300-334).
  if (selections.empty()) return std::vector<std::string>();
  const size_t first = selections[0].size();
  for (size_t i = 0; i < selections.size(); ++i) {
    if (selections[i].size() * 128 < static_cast<size_t>(num_records_))
      return InvalidArgumentError("`selections[" + std::to_string(i) +
                                  "]` contains insufficient number of bits: " +
                                  std::to_string(selections[i].size() * 128) +
                                  ", expected: " + std::to_string(num_records_));
    if (selections[i].size() != first)
      return InvalidArgumentError("`selections[" + std::to_string(i) +
                                  "].size()` does not match `selections[0].size()`: actual" +
                                  std::to_string(selections[i].size()) + ", expected " +
                                  std::to_string(first));
    if (max_value_size_ <= 0) return InvalidArgumentError("`max_value_size` must be positive");
  }
  // Only the blocks that select existing records are read by the scan.
  const int64_t blocks = std::max<int64_t>(1, (num_records_ + 127) / 128);
  const int q = static_cast<int>(selections.size());
  std::vector<uint128> host(static_cast<size_t>(q) * blocks);
  for (int k = 0; k < q; ++k)
    for (int64_t b = 0; b < blocks && b < static_cast<int64_t>(first); ++b)
      host[k * blocks + b] = selections[k][b].value();
  hipStream_t s = PirStream();
  void* dev = nullptr;
  DPF_RETURN_IF_ERROR(dpf_internal_host::DevicePool::Get().Alloc(16 * host.size(), s, &dev));
  Status st = HipStatus(hipMemcpyAsync(dev, host.data(), 16 * host.size(),
                                       hipMemcpyHostToDevice, s), "h2d");
  StatusOr<std::vector<std::string>> r =
      st.ok() ? InnerProductWithDevice(dev, blocks, q, s) : StatusOr<std::vector<std::string>>(st);
  dpf_internal_host::DevicePool::Get().Free(dev, s);
  (void)hipStreamSynchronize(s);
  return r;
}

// ---------------------------------------------------------------------------
// DpfPirServer roles (pir/dpf_pir_server.cc:35-193)
// ---------------------------------------------------------------------------

Status DpfPirServer::MakeLeader(ForwardHelperRequestFn sender) {
  if (sender == nullptr) return InvalidArgumentError("`sender` may not be null");
  sender_ = std::move(sender);
  role_ = Role::kLeader;
  return OkStatus();
}

Status DpfPirServer::MakeHelper(DecryptHelperRequestFn decrypter, std::string info) {
  if (decrypter == nullptr) return InvalidArgumentError("`decrypter` may not be null");
  decrypter_ = std::move(decrypter);
  encryption_context_info_ = std::move(info);
  role_ = Role::kHelper;
  return OkStatus();
}

StatusOr<PirResponse> DpfPirServer::HandleRequest(const PirRequest& request) const {
  switch (role_) {
    case Role::kLeader:
      return HandleLeaderRequest(request);
    case Role::kHelper:
      return HandleHelperRequest(request);
    default:
      return HandlePlainRequest(request);
  }
}

StatusOr<PirResponse> DpfPirServer::HandleLeaderRequest(const PirRequest& request) const {
  if (request.dpf_pir_request().wrapped_request_case() != DpfPirRequest::kLeaderRequest)
    return InvalidArgumentError("`request` must be a valid DpfPirRequest::LeaderRequest");
  const DpfPirRequest::LeaderRequest& leader_request = request.dpf_pir_request().leader_request();
  if (!leader_request.has_plain_request())
    return InvalidArgumentError("`plain_request` must be set");
  if (!leader_request.has_encrypted_helper_request())
    return InvalidArgumentError("`encrypted_helper_request` must be set");
  PirRequest plain_request, helper_request;
  *plain_request.mutable_dpf_pir_request()->mutable_plain_request() = leader_request.plain_request();
  *helper_request.mutable_dpf_pir_request()->mutable_encrypted_helper_request() =
      leader_request.encrypted_helper_request();
  bool has_run = false;
  StatusOr<PirResponse> leader_response = InternalError("not run");
  auto while_waiting = [&] {
    leader_response = this->HandlePlainRequest(plain_request);
    has_run = true;
  };
  StatusOr<PirResponse> helper_response = sender_(helper_request, while_waiting);
  if (!helper_response.ok()) return helper_response.status();
  if (!has_run)
    return FailedPreconditionError(
        "HandleRequest: `while_waiting` was not called from `sender` passed at construction.");
  if (!leader_response.ok()) return leader_response.status();
  const int n = helper_response->dpf_pir_response().masked_response_size();
  if (n != leader_response->dpf_pir_response().masked_response_size())
    return InternalError("Number of responses from Helper (=" + std::to_string(n) +
                         ")  does not match the number of responses from Leader (=" +
                         std::to_string(leader_response->dpf_pir_response().masked_response_size()) +
                         ")");
  for (int i = 0; i < n; ++i) {
    const std::string& h = helper_response->dpf_pir_response().masked_response(i);
    std::string& l = *leader_response->mutable_dpf_pir_response()->mutable_masked_response(i);
    if (h.size() != l.size())
      return InternalError("Response size mismatch at index " + std::to_string(i) + ": Got " +
                           std::to_string(h.size()) + " (Helper) vs. " +
                           std::to_string(l.size()) + " (Leader)");
    for (size_t j = 0; j < h.size(); ++j) l[j] ^= h[j];
  }
  return leader_response;
}

StatusOr<PirResponse> DpfPirServer::HandleHelperRequest(const PirRequest& request) const {
  if (request.dpf_pir_request().wrapped_request_case() != DpfPirRequest::kEncryptedHelperRequest)
    return InvalidArgumentError("`request` must be a valid EncryptedHelperRequest");
  StatusOr<std::string> decrypted = decrypter_(
      request.dpf_pir_request().encrypted_helper_request().encrypted_request(),
      encryption_context_info_);
  if (!decrypted.ok()) return decrypted.status();
  DpfPirRequest::HelperRequest inner;
  if (!inner.ParseFromString(*decrypted))
    return InvalidArgumentError(
        "`request` does not encrypt a valid DpfPirRequest::HelperRequest");
  PirRequest plain_request;
  *plain_request.mutable_dpf_pir_request()->mutable_plain_request() = inner.plain_request();
  StatusOr<PirResponse> response = this->HandlePlainRequest(plain_request);
  if (!response.ok()) return response.status();
  const std::string& seed = inner.one_time_pad_seed();
  if (seed.size() != 16)
    return InvalidArgumentError("seed must be 16 bytes, supplied seed is " +
                                std::to_string(seed.size()) + " bytes.");
  size_t offset = 0;
  for (int i = 0; i < response->dpf_pir_response().masked_response_size(); ++i) {
    std::string& r = *response->mutable_dpf_pir_response()->mutable_masked_response(i);
    const std::string pad = dpf_amd::AesCtrKeystream(seed, offset, r.size());
    offset += r.size();
    for (size_t j = 0; j < r.size(); ++j) r[j] ^= pad[j];
  }
  return response;
}

std::string AesCtrOneTimePad(const std::string& seed, size_t offset, size_t length) {
  return dpf_amd::AesCtrKeystream(seed, offset, length);
}

// ---------------------------------------------------------------------------
// DenseDpfPirServer (pir/dense_dpf_pir_server.cc:39-127)
// ---------------------------------------------------------------------------

DenseDpfPirServer::DenseDpfPirServer(std::unique_ptr<DistributedPointFunction> dpf,
                                     std::unique_ptr<Database> database)
    : dpf_(std::move(dpf)), database_(std::move(database)) {}

StatusOr<std::unique_ptr<DenseDpfPirServer>> DenseDpfPirServer::CreateLeader(
    const PirConfig& config, std::unique_ptr<Database> database, ForwardHelperRequestFn sender) {
  StatusOr<std::unique_ptr<DenseDpfPirServer>> s = CreatePlain(config, std::move(database));
  if (!s.ok()) return s.status();
  DPF_RETURN_IF_ERROR((*s)->MakeLeader(std::move(sender)));
  return s;
}

StatusOr<std::unique_ptr<DenseDpfPirServer>> DenseDpfPirServer::CreateHelper(
    const PirConfig& config, std::unique_ptr<Database> database,
    DecryptHelperRequestFn decrypter) {
  StatusOr<std::unique_ptr<DenseDpfPirServer>> s = CreatePlain(config, std::move(database));
  if (!s.ok()) return s.status();
  DPF_RETURN_IF_ERROR((*s)->MakeHelper(std::move(decrypter), kEncryptionContextInfo));
  return s;
}

StatusOr<std::unique_ptr<DenseDpfPirServer>> DenseDpfPirServer::CreatePlain(
    const PirConfig& config, std::unique_ptr<Database> database) {
  if (config.wrapped_pir_config_case() != PirConfig::kDenseDpfPirConfig)
    return InvalidArgumentError("`config` does not contain a valid DenseDpfPirConfig");
  if (database == nullptr) return InvalidArgumentError("`database` cannot be null");
  if (config.dense_dpf_pir_config().num_elements() <= 0)
    return InvalidArgumentError("`num_elements` must be positive");
  if (static_cast<int64_t>(database->size()) != config.dense_dpf_pir_config().num_elements())
    return InvalidArgumentError("Database size does not match the config size");
  DpfParameters parameters;
  parameters.set_log_domain_size(static_cast<int>(
      std::ceil(std::log2(static_cast<double>(config.dense_dpf_pir_config().num_elements())))));
  parameters.mutable_value_type()->mutable_xor_wrapper()->set_bitsize(128);
  StatusOr<std::unique_ptr<DistributedPointFunction>> dpf =
      DistributedPointFunction::Create(parameters);
  if (!dpf.ok()) return dpf.status();
  return std::unique_ptr<DenseDpfPirServer>(
      new DenseDpfPirServer(std::move(*dpf), std::move(database)));
}

const PirServerPublicParams& DenseDpfPirServer::GetPublicParams() const {
  return PirServerPublicParams::default_instance();
}

StatusOr<PirResponse> DenseDpfPirServer::HandlePlainRequest(const PirRequest& request) const {
  if (request.wrapped_pir_request_case() != PirRequest::kDpfPirRequest)
    return InvalidArgumentError("`request` does not contain a valid DpfPirRequest");
  if (request.dpf_pir_request().wrapped_request_case() != DpfPirRequest::kPlainRequest)
    return InvalidArgumentError(
        "`request` does not contain a valid DpfPirRequest::PlainRequest");
  const DpfPirRequest::PlainRequest& plain = request.dpf_pir_request().plain_request();
  if (plain.dpf_key_size() == 0) return InvalidArgumentError("`dpf_key` must not be empty");
  const int q = plain.dpf_key_size();
  std::vector<std::string> inner_products;
  const auto* gpu_db = dynamic_cast<const DenseDpfPirDatabase*>(database_.get());
  if (gpu_db != nullptr) {
    // Fused path: expand only the ceil(N/128) selection blocks the scan
    // reads, straight into HBM, then scan.
    for (int i = 0; i < q; ++i) {
      StatusOr<EvaluationContext> ctx = dpf_->CreateEvaluationContext(plain.dpf_key(i));
      if (!ctx.ok()) return ctx.status();
    }
    const int64_t n = static_cast<int64_t>(database_->size());
    const int64_t blocks = std::max<int64_t>(1, (n + 127) / 128);
    hipStream_t s = PirStream();
    void* sel = nullptr;
    DPF_RETURN_IF_ERROR(dpf_internal_host::DevicePool::Get().Alloc(16 * blocks * q, s, &sel));
    const dpf_amd_value_type layout = dpf_internal::HostLayoutOf<XorWrapper<uint128>>();
    std::vector<const DpfKey*> keys(q);
    for (int i = 0; i < q; ++i) keys[i] = &plain.dpf_key(i);
    Status st = dpf_->ExpandLeavesOnDeviceBatched(
        Span<const DpfKey* const>(keys.data(), keys.size()), blocks, layout, sel, s);
    StatusOr<std::vector<std::string>> r =
        st.ok() ? gpu_db->InnerProductWithDevice(sel, blocks, q, s)
                : StatusOr<std::vector<std::string>>(st);
    dpf_internal_host::DevicePool::Get().Free(sel, s);
    (void)hipStreamSynchronize(s);
    if (!r.ok()) return r.status();
    inner_products = std::move(*r);
  } else {
    std::vector<std::vector<XorWrapper<uint128>>> selections(q);
    for (int i = 0; i < q; ++i) {
      StatusOr<EvaluationContext> ctx = dpf_->CreateEvaluationContext(plain.dpf_key(i));
      if (!ctx.ok()) return ctx.status();
      StatusOr<std::vector<XorWrapper<uint128>>> sel =
          dpf_->EvaluateNext<XorWrapper<uint128>>({}, *ctx);
      if (!sel.ok()) return sel.status();
      selections[i] = std::move(*sel);
    }
    StatusOr<std::vector<std::string>> r = database_->InnerProductWith(
        Span<const std::vector<XorWrapper<uint128>>>(selections.data(), selections.size()));
    if (!r.ok()) return r.status();
    inner_products = std::move(*r);
  }
  PirResponse response;
  for (std::string& s : inner_products)
    *response.mutable_dpf_pir_response()->add_masked_response() = std::move(s);
  return response;
}

}  // namespace distributed_point_functions
