// cuckoo_pir.cc — SHA-256 hash family, cuckoo hash table, cuckoo-hashed
// sparse PIR database and server (see
// include/dpf_amd/cuckoo_hashing_sparse_dpf_pir_server.h for the reference
// mapping).  Everything here is host-side bookkeeping except the two HBM
// scans, which reuse DenseDpfPirDatabase (k_pir.hip).
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <fstream>

#include "dpf_amd/cuckoo_hashing_sparse_dpf_pir_server.h"
#include "host_device.h"
#include "internal.h"

namespace distributed_point_functions {
namespace {

// ---------------------------------------------------------------------------
// SHA-256 (FIPS 180-4). The reference calls OpenSSL's SHA256_* (BoringSSL
// @6347808f, sha256_hash_family.cc:33-60); the digest is a fixed standard,
// pinned in tests by the reference's NIST CAVP vector
// (sha256_hash_family_test.cc:36-59).
// ---------------------------------------------------------------------------
constexpr uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
    0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
    0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
    0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
    0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
    0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
    0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
    0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};

inline uint32_t Rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

void Sha256Compress(uint32_t h[8], const uint8_t* block) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i)
    w[i] = (uint32_t{block[4 * i]} << 24) | (uint32_t{block[4 * i + 1]} << 16) |
           (uint32_t{block[4 * i + 2]} << 8) | block[4 * i + 3];
  for (int i = 16; i < 64; ++i) {
    const uint32_t s0 = Rotr(w[i - 15], 7) ^ Rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
    const uint32_t s1 = Rotr(w[i - 2], 17) ^ Rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; ++i) {
    const uint32_t t1 =
        hh + (Rotr(e, 6) ^ Rotr(e, 11) ^ Rotr(e, 25)) + ((e & f) ^ (~e & g)) + kSha256K[i] + w[i];
    const uint32_t t2 = (Rotr(a, 2) ^ Rotr(a, 13) ^ Rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
  h[5] += f;
  h[6] += g;
  h[7] += hh;
}

void Sha256(const std::string& a, const std::string& b, uint8_t out[32]) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint8_t buf[64];
  size_t fill = 0;
  uint64_t total = 0;
  for (const std::string* part : {&a, &b}) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(part->data());
    size_t n = part->size();
    total += n;
    while (n > 0) {
      const size_t take = std::min(n, 64 - fill);
      memcpy(buf + fill, p, take);
      fill += take;
      p += take;
      n -= take;
      if (fill == 64) {
        Sha256Compress(h, buf);
        fill = 0;
      }
    }
  }
  buf[fill++] = 0x80;
  if (fill > 56) {
    memset(buf + fill, 0, 64 - fill);
    Sha256Compress(h, buf);
    fill = 0;
  }
  memset(buf + fill, 0, 56 - fill);
  const uint64_t bits = total * 8;
  for (int i = 0; i < 8; ++i) buf[56 + i] = static_cast<uint8_t>(bits >> (56 - 8 * i));
  Sha256Compress(h, buf);
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 4; ++j) out[4 * i + j] = static_cast<uint8_t>(h[i] >> (24 - 8 * j));
}

hipStream_t CuckooStream() { return dpf_internal_host::ThreadStream(); }

Status HipStatus(hipError_t e, const char* what) {
  if (e == hipSuccess) return OkStatus();
  if (e == hipErrorOutOfMemory)
    return ResourceExhaustedError(std::string(what) + ": " + hipGetErrorString(e));
  return InternalError(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

std::string Sha256Digest(const std::string& data) {
  uint8_t out[32];
  Sha256(data, std::string(), out);
  return std::string(reinterpret_cast<const char*>(out), 32);
}

int SHA256HashFunction::operator()(const std::string& input, int upper_bound) const {
  uint8_t d[32];
  Sha256(seed_, input, d);
  // The digest as a 256-bit little-endian integer mod upper_bound: the
  // reference's three-step long division over hi = d[16..32), lo = d[0..16)
  // (sha256_hash_family.cc:66-85) is exactly this Horner reduction.
  const uint64_t m = static_cast<uint64_t>(upper_bound);
  unsigned __int128 r = 0;
  for (int i = 31; i >= 0; --i) r = ((r << 8) | d[i]) % m;
  return static_cast<int>(r);
}

HashFamily WrapWithSeed(HashFamily family, std::string family_seed) {
  return [family = std::move(family), family_seed = std::move(family_seed)](
             const std::string& seed) { return family(family_seed + seed); };
}

StatusOr<std::vector<HashFunction>> CreateHashFunctions(HashFamily family,
                                                        int num_hash_functions) {
  if (num_hash_functions < 0)
    return InvalidArgumentError("num_hash_functions must not be negative");
  std::vector<HashFunction> result;
  result.reserve(num_hash_functions);
  for (int i = 0; i < num_hash_functions; ++i) result.push_back(family(std::to_string(i)));
  return result;
}

StatusOr<HashFamily> CreateHashFamilyFromConfig(const HashFamilyConfig& config) {
  if (config.seed().empty()) return InvalidArgumentError("`seed` must not be empty");
  switch (config.hash_family()) {
    case HashFamilyConfig::HASH_FAMILY_SHA256:
      return WrapWithSeed(SHA256HashFamily(), config.seed());
    case HashFamilyConfig::HASH_FAMILY_UNSPECIFIED:
      return InvalidArgumentError("Hash family unspecified");
    default:
      return InvalidArgumentError("Unknown hash family specified");
  }
}

// ---------------------------------------------------------------------------
// CuckooHashTable (pir/hashing/cuckoo_hash_table.cc)
// ---------------------------------------------------------------------------

CuckooHashTable::CuckooHashTable(std::vector<HashFunction> hash_functions, int num_buckets,
                                 int max_relocations, std::optional<int> max_stash_size)
    : num_buckets_(num_buckets),
      max_relocations_(max_relocations),
      max_stash_size_(max_stash_size),
      hash_functions_(std::move(hash_functions)),
      table_(num_buckets) {
  if (max_stash_size) stash_.reserve(*max_stash_size);
}

StatusOr<std::unique_ptr<CuckooHashTable>> CuckooHashTable::Create(
    std::vector<HashFunction> hash_functions, int num_buckets, int max_relocations,
    std::optional<int> max_stash_size) {
  if (num_buckets <= 0) return InvalidArgumentError("num_buckets must be positive");
  if (hash_functions.size() < 2)
    return InvalidArgumentError("hash_functions.size() must be at least 2");
  if (max_relocations < 0) return InvalidArgumentError("max_relocations must be non-negative");
  if (max_stash_size && *max_stash_size < 0)
    return InvalidArgumentError("max_stash_size must be non-negative");
  return std::unique_ptr<CuckooHashTable>(new CuckooHashTable(
      std::move(hash_functions), num_buckets, max_relocations, max_stash_size));
}

StatusOr<std::unique_ptr<CuckooHashTable>> CuckooHashTable::Create(
    HashFamily hash_family, int num_buckets, int num_hash_functions, int max_relocations,
    std::optional<int> max_stash_size) {
  StatusOr<std::vector<HashFunction>> fns =
      CreateHashFunctions(std::move(hash_family), num_hash_functions);
  if (!fns.ok()) return fns.status();
  return Create(std::move(*fns), num_buckets, max_relocations, max_stash_size);
}

int CuckooHashTable::RandomHashFunction() {
  // absl::uniform_int_distribution<int>(0, k-1): range R = k-1 as uint32;
  // FastUniformBits<uint32_t> over a 2^64-range engine takes the low 32 bits
  // of one draw; power-of-two lengths mask, others use the fixed-point
  // multiply with rejection below -Lim % Lim.
  const uint32_t range = static_cast<uint32_t>(hash_functions_.size() - 1);
  const uint32_t lim = range + 1;
  uint32_t bits = static_cast<uint32_t>(rng_());
  if ((range & lim) == 0) return static_cast<int>(bits & range);
  uint64_t product = static_cast<uint64_t>(bits) * lim;
  if (static_cast<uint32_t>(product) < lim) {
    const uint32_t threshold = (0u - lim) % lim;
    while (static_cast<uint32_t>(product) < threshold) {
      bits = static_cast<uint32_t>(rng_());
      product = static_cast<uint64_t>(bits) * lim;
    }
  }
  return static_cast<int>(product >> 32);
}

Status CuckooHashTable::Insert(const std::string& input) {
  std::string current(input);
  for (int i = 0; i < max_relocations_; ++i) {
    const int hash = hash_functions_[RandomHashFunction()](current, num_buckets_);
    if (table_[hash]) {
      std::swap(current, *table_[hash]);  // evict and re-insert the occupant
    } else {
      table_[hash] = std::move(current);
      return OkStatus();
    }
  }
  if (max_stash_size_ && static_cast<int>(stash_.size()) >= *max_stash_size_)
    return InternalError("Cannot insert element: stash is full");
  stash_.push_back(std::move(current));
  return OkStatus();
}

// ---------------------------------------------------------------------------
// CuckooHashedDpfPirDatabase (pir/cuckoo_hashed_dpf_pir_database.cc)
// ---------------------------------------------------------------------------

CuckooHashedDpfPirDatabase::Builder::Builder() = default;

CuckooHashedDpfPirDatabase::Builder& CuckooHashedDpfPirDatabase::Builder::Insert(
    RecordType key_value) {
  records_.insert(std::move(key_value));  // first insert of a key wins, as btree_map
  return *this;
}

std::unique_ptr<CuckooHashedDpfPirDatabase::Interface::Builder>
CuckooHashedDpfPirDatabase::Builder::Clone() const {
  auto r = std::make_unique<Builder>();
  r->params_ = params_;
  if (key_database_builder_) r->key_database_builder_ = key_database_builder_->Clone();
  if (value_database_builder_) r->value_database_builder_ = value_database_builder_->Clone();
  r->records_ = records_;
  r->has_been_built_ = has_been_built_;
  return r;
}

CuckooHashedDpfPirDatabase::Builder& CuckooHashedDpfPirDatabase::Builder::SetParams(
    CuckooHashingParams params) {
  params_ = std::move(params);
  return *this;
}

CuckooHashedDpfPirDatabase::Builder& CuckooHashedDpfPirDatabase::Builder::SetKeyDatabaseBuilder(
    std::unique_ptr<DenseDatabase::Builder> builder) {
  key_database_builder_ = std::move(builder);
  return *this;
}

CuckooHashedDpfPirDatabase::Builder&
CuckooHashedDpfPirDatabase::Builder::SetValueDatabaseBuilder(
    std::unique_ptr<DenseDatabase::Builder> builder) {
  value_database_builder_ = std::move(builder);
  return *this;
}

StatusOr<std::vector<std::optional<std::string>>>
CuckooHashedDpfPirDatabase::Builder::PlaceKeys() const {
  if (params_.num_buckets() <= 0) return InvalidArgumentError("`num_buckets` must be positive");
  if (params_.num_hash_functions() <= 0)
    return InvalidArgumentError("`num_hash_functions` must be positive");
  StatusOr<HashFamily> family = CreateHashFamilyFromConfig(params_.hash_family_config());
  if (!family.ok()) return family.status();
  // max_relocations = number of records, unlimited stash (.cc:117-122):
  // keys left on the stash are not served, as in the reference.
  StatusOr<std::unique_ptr<CuckooHashTable>> table = CuckooHashTable::Create(
      std::move(*family), static_cast<int>(params_.num_buckets()),
      params_.num_hash_functions(), static_cast<int>(records_.size()));
  if (!table.ok()) return table.status();
  for (const auto& kv : records_) {
    if (kv.first.empty()) return InvalidArgumentError("Key cannot be empty");
    DPF_RETURN_IF_ERROR((*table)->Insert(kv.first));
  }
  return (*table)->GetTable();
}

StatusOr<std::unique_ptr<CuckooHashedDpfPirDatabase::Interface>>
CuckooHashedDpfPirDatabase::Builder::Build() {
  if (has_been_built_) return FailedPreconditionError("Database already built");
  has_been_built_ = true;
  StatusOr<std::vector<std::optional<std::string>>> table = PlaceKeys();
  if (!table.ok()) return table.status();
  if (!key_database_builder_) key_database_builder_ = std::make_unique<DenseDpfPirDatabase::Builder>();
  if (!value_database_builder_)
    value_database_builder_ = std::make_unique<DenseDpfPirDatabase::Builder>();
  const size_t num_records = records_.size();
  for (std::optional<std::string>& bucket : *table) {
    if (bucket) {
      auto it = records_.find(*bucket);
      std::string value = std::move(it->second);
      records_.erase(it);
      key_database_builder_->Insert(std::move(*bucket));
      value_database_builder_->Insert(std::move(value));
    } else {  // dummy strings for empty buckets
      key_database_builder_->Insert(std::string());
      value_database_builder_->Insert(std::string());
    }
  }
  StatusOr<std::unique_ptr<DenseDatabase>> keys = key_database_builder_->Build();
  if (!keys.ok()) return keys.status();
  StatusOr<std::unique_ptr<DenseDatabase>> values = value_database_builder_->Build();
  if (!values.ok()) return values.status();
  const size_t bits = (*keys)->num_selection_bits();
  if (bits != (*values)->num_selection_bits() ||
      bits != static_cast<size_t>(params_.num_buckets()))
    return InternalError("Number of selection bits in underlying databases doesn't match");
  return std::unique_ptr<Interface>(new CuckooHashedDpfPirDatabase(
      std::move(*keys), std::move(*values), num_records, bits));
}

CuckooHashedDpfPirDatabase::CuckooHashedDpfPirDatabase(
    std::unique_ptr<DenseDatabase> key_database, std::unique_ptr<DenseDatabase> value_database,
    size_t size, size_t num_selection_bits)
    : key_database_(std::move(key_database)),
      value_database_(std::move(value_database)),
      size_(size),
      num_selection_bits_(num_selection_bits) {}

namespace {
StatusOr<std::vector<CuckooHashedDpfPirDatabase::RecordType>> Zip(
    StatusOr<std::vector<std::string>> keys, StatusOr<std::vector<std::string>> values,
    size_t expected) {
  if (!keys.ok()) return keys.status();
  if (!values.ok()) return values.status();
  if (keys->size() != values->size() || keys->size() != expected)
    return InternalError("Result sizes do not match. This should not happen.");
  std::vector<CuckooHashedDpfPirDatabase::RecordType> result;
  result.reserve(keys->size());
  for (size_t i = 0; i < keys->size(); ++i)
    result.emplace_back(std::move((*keys)[i]), std::move((*values)[i]));
  return result;
}
}  // namespace

StatusOr<std::vector<CuckooHashedDpfPirDatabase::RecordType>>
CuckooHashedDpfPirDatabase::InnerProductWith(Span<const std::vector<BlockType>> selections) const {
  return Zip(key_database_->InnerProductWith(selections),
             value_database_->InnerProductWith(selections), selections.size());
}

bool CuckooHashedDpfPirDatabase::device_resident() const {
  return dynamic_cast<const DenseDpfPirDatabase*>(key_database_.get()) != nullptr &&
         dynamic_cast<const DenseDpfPirDatabase*>(value_database_.get()) != nullptr;
}

StatusOr<std::vector<CuckooHashedDpfPirDatabase::RecordType>>
CuckooHashedDpfPirDatabase::InnerProductWithDevice(const void* selections_dev,
                                                   int64_t selection_blocks, int num_queries,
                                                   void* stream) const {
  const auto* k = dynamic_cast<const DenseDpfPirDatabase*>(key_database_.get());
  const auto* v = dynamic_cast<const DenseDpfPirDatabase*>(value_database_.get());
  if (!k || !v) return FailedPreconditionError("tables are not HBM-resident");
  return Zip(k->InnerProductWithDevice(selections_dev, selection_blocks, num_queries, stream),
             v->InnerProductWithDevice(selections_dev, selection_blocks, num_queries, stream),
             static_cast<size_t>(num_queries));
}

// ---------------------------------------------------------------------------
// CuckooHashingSparseDpfPirServer (pir/cuckoo_hashing_sparse_dpf_pir_server.cc)
// ---------------------------------------------------------------------------

StatusOr<CuckooHashingParams> CuckooHashingSparseDpfPirServer::GenerateParams(
    const PirConfig& config) {
  if (config.wrapped_pir_config_case() != PirConfig::kCuckooHashingSparseDpfPirConfig)
    return InvalidArgumentError("`config` must be a valid CuckooHashingSparseDpfPirConfig");
  std::string seed(kHashFunctionSeedLengthBytes, '\0');
  {
    std::ifstream urandom("/dev/urandom", std::ios::binary);
    if (!urandom.read(&seed[0], seed.size()))
      return InternalError("failed to read random bytes for the hash family seed");
  }
  CuckooHashingParams params;
  params.mutable_hash_family_config()->set_seed(std::move(seed));
  params.mutable_hash_family_config()->set_hash_family(
      config.cuckoo_hashing_sparse_dpf_pir_config().hash_family());
  params.set_num_hash_functions(3);  // kNumHashFunctions
  // kBucketsPerElement (1.5) * num_elements, truncated as the int64 setter does.
  params.set_num_buckets(static_cast<int64_t>(
      1.5 * static_cast<double>(config.cuckoo_hashing_sparse_dpf_pir_config().num_elements())));
  return params;
}

CuckooHashingSparseDpfPirServer::CuckooHashingSparseDpfPirServer(
    PirServerPublicParams params, std::unique_ptr<DistributedPointFunction> dpf,
    std::unique_ptr<Database> database)
    : params_(std::move(params)), dpf_(std::move(dpf)), database_(std::move(database)) {}

StatusOr<std::unique_ptr<CuckooHashingSparseDpfPirServer>>
CuckooHashingSparseDpfPirServer::CreatePlain(CuckooHashingParams params,
                                             std::unique_ptr<Database> database) {
  if (params.num_buckets() <= 0) return InvalidArgumentError("`num_buckets` must be positive");
  if (params.num_hash_functions() <= 0)
    return InvalidArgumentError("`num_hash_functions` must be positive");
  if (params.hash_family_config().hash_family() == HashFamilyConfig::HASH_FAMILY_UNSPECIFIED)
    return InvalidArgumentError("params.hash_family_config.hash_family must be set");
  if (database == nullptr) return InvalidArgumentError("`database` cannot be null");
  if (database->num_selection_bits() != static_cast<size_t>(params.num_buckets()))
    return InvalidArgumentError(
        "Number of selection bits in the database does not match `params.num_buckets`");
  DpfParameters dpf_parameters;
  dpf_parameters.set_log_domain_size(
      static_cast<int>(std::ceil(std::log2(static_cast<double>(params.num_buckets())))));
  dpf_parameters.mutable_value_type()->mutable_xor_wrapper()->set_bitsize(128);
  StatusOr<std::unique_ptr<DistributedPointFunction>> dpf =
      DistributedPointFunction::Create(dpf_parameters);
  if (!dpf.ok()) return dpf.status();
  PirServerPublicParams server_params;
  *server_params.mutable_cuckoo_hashing_sparse_dpf_pir_server_params() = std::move(params);
  return std::unique_ptr<CuckooHashingSparseDpfPirServer>(new CuckooHashingSparseDpfPirServer(
      std::move(server_params), std::move(*dpf), std::move(database)));
}

StatusOr<std::unique_ptr<CuckooHashingSparseDpfPirServer>>
CuckooHashingSparseDpfPirServer::CreateLeader(CuckooHashingParams params,
                                              std::unique_ptr<Database> database,
                                              ForwardHelperRequestFn sender) {
  StatusOr<std::unique_ptr<CuckooHashingSparseDpfPirServer>> s =
      CreatePlain(std::move(params), std::move(database));
  if (!s.ok()) return s.status();
  DPF_RETURN_IF_ERROR((*s)->MakeLeader(std::move(sender)));
  return s;
}

StatusOr<std::unique_ptr<CuckooHashingSparseDpfPirServer>>
CuckooHashingSparseDpfPirServer::CreateHelper(CuckooHashingParams params,
                                              std::unique_ptr<Database> database,
                                              DecryptHelperRequestFn decrypter) {
  StatusOr<std::unique_ptr<CuckooHashingSparseDpfPirServer>> s =
      CreatePlain(std::move(params), std::move(database));
  if (!s.ok()) return s.status();
  DPF_RETURN_IF_ERROR((*s)->MakeHelper(std::move(decrypter), kEncryptionContextInfo));
  return s;
}

StatusOr<PirResponse> CuckooHashingSparseDpfPirServer::HandlePlainRequest(
    const PirRequest& request) const {
  if (request.wrapped_pir_request_case() != PirRequest::kDpfPirRequest)
    return InvalidArgumentError("`request` does not contain a valid DpfPirRequest");
  if (request.dpf_pir_request().wrapped_request_case() != DpfPirRequest::kPlainRequest)
    return InvalidArgumentError(
        "`request` does not contain a valid DpfPirRequest::PlainRequest");
  const DpfPirRequest::PlainRequest& plain = request.dpf_pir_request().plain_request();
  if (plain.dpf_key_size() == 0) return InvalidArgumentError("`dpf_key` must not be empty");
  const int q = plain.dpf_key_size();
  for (int i = 0; i < q; ++i) {  // key validation, as EvaluateNext would
    StatusOr<EvaluationContext> ctx = dpf_->CreateEvaluationContext(plain.dpf_key(i));
    if (!ctx.ok()) return ctx.status();
  }
  std::vector<Database::RecordType> inner_products;
  const auto* gpu_db = dynamic_cast<const CuckooHashedDpfPirDatabase*>(database_.get());
  if (gpu_db != nullptr && gpu_db->device_resident()) {
    // One device expansion per key into the ceil(B/128) selection blocks the
    // scans read; both tables are scanned from that buffer.
    const int64_t buckets = static_cast<int64_t>(database_->num_selection_bits());
    const int64_t blocks = std::max<int64_t>(1, (buckets + 127) / 128);
    hipStream_t s = CuckooStream();
    void* sel = nullptr;
    DPF_RETURN_IF_ERROR(dpf_internal_host::DevicePool::Get().Alloc(16 * blocks * q, s, &sel));
    const dpf_amd_value_type layout = dpf_internal::HostLayoutOf<XorWrapper<uint128>>();
    std::vector<const DpfKey*> keys(q);
    for (int i = 0; i < q; ++i) keys[i] = &plain.dpf_key(i);
    Status st = dpf_->ExpandLeavesOnDeviceBatched(
        Span<const DpfKey* const>(keys.data(), keys.size()), blocks, layout, sel, s);
    StatusOr<std::vector<Database::RecordType>> r =
        st.ok() ? gpu_db->InnerProductWithDevice(sel, blocks, q, s)
                : StatusOr<std::vector<Database::RecordType>>(st);
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
    StatusOr<std::vector<Database::RecordType>> r = database_->InnerProductWith(
        Span<const std::vector<XorWrapper<uint128>>>(selections.data(), selections.size()));
    if (!r.ok()) return r.status();
    inner_products = std::move(*r);
  }
  PirResponse response;
  for (Database::RecordType& kv : inner_products) {
    *response.mutable_dpf_pir_response()->add_masked_response() = std::move(kv.first);
    *response.mutable_dpf_pir_response()->add_masked_response() = std::move(kv.second);
  }
  return response;
}

}  // namespace distributed_point_functions
