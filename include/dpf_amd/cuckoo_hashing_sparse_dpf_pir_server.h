// cuckoo_hashing_sparse_dpf_pir_server.h — keyword (sparse) two-server DPF
// PIR on MI355X: a cuckoo-hashed key/value store served as two dense HBM
// scans sharing one device-resident DPF selection vector.
//   HashFunction / HashFamily        pir/hashing/hash_family.h:27-66
//   SHA256HashFunction / Family      pir/hashing/sha256_hash_family.h, .cc:47-86
//   CreateHashFamilyFromConfig       pir/hashing/hash_family_config.cc:27-45
//   CuckooHashTable                  pir/hashing/cuckoo_hash_table.h:35-110, .cc:34-90
//   CuckooHashedDpfPirDatabase       pir/cuckoo_hashed_dpf_pir_database.h:37-110, .cc:49-192
//   CuckooHashingSparseDpfPirServer  pir/cuckoo_hashing_sparse_dpf_pir_server.h:37-125,
//                                    .cc:35-157
// HandlePlainRequest expands each DPF key once, on the device, into the
// ceil(num_buckets/128) selection blocks both scans read, then XOR-scans the
// key table and the value table (k_pir.hip) from that same buffer.
#ifndef DPF_AMD_CUCKOO_HASHING_SPARSE_DPF_PIR_SERVER_H_
#define DPF_AMD_CUCKOO_HASHING_SPARSE_DPF_PIR_SERVER_H_

#include <stdint.h>

#include <functional>
#include <map>
#include <memory>
#include <optional>
#include <random>
#include <string>
#include <utility>
#include <vector>

#include "dpf_amd/dense_dpf_pir_server.h"

namespace distributed_point_functions {

// A hash function maps (input, upper_bound) to [0, upper_bound).
using HashFunction = std::function<int(const std::string& input, int upper_bound)>;
// A hash family maps a seed to a hash function.
using HashFamily = std::function<HashFunction(const std::string& seed)>;

// SHA256(seed || input) read as a 256-bit little-endian integer, mod
// upper_bound (sha256_hash_family.cc:59-86).
class SHA256HashFunction {
 public:
  explicit SHA256HashFunction(std::string seed) : seed_(std::move(seed)) {}
  int operator()(const std::string& input, int upper_bound) const;

 private:
  std::string seed_;
};

struct SHA256HashFamily {
  HashFunction operator()(const std::string& seed) const { return SHA256HashFunction(seed); }
};

// hash_family.h:45-53: prefixes every per-function seed with `family_seed`.
HashFamily WrapWithSeed(HashFamily family, std::string family_seed);
// hash_family.cc:27-39: function i is family(StrCat(i)).
StatusOr<std::vector<HashFunction>> CreateHashFunctions(HashFamily family,
                                                        int num_hash_functions);
// hash_family_config.cc:27-45.
StatusOr<HashFamily> CreateHashFamilyFromConfig(const HashFamilyConfig& config);

// Raw SHA-256 digest (FIPS 180-4), exposed for tests.
std::string Sha256Digest(const std::string& data);

class CuckooHashTable {
 public:
  static StatusOr<std::unique_ptr<CuckooHashTable>> Create(
      std::vector<HashFunction> hash_functions, int num_buckets, int max_relocations,
      std::optional<int> max_stash_size = std::nullopt);
  static StatusOr<std::unique_ptr<CuckooHashTable>> Create(
      HashFamily hash_family, int num_buckets, int num_hash_functions, int max_relocations,
      std::optional<int> max_stash_size = std::nullopt);

  // cuckoo_hash_table.cc:62-90: random-walk insertion with at most
  // max_relocations evictions, then the stash.
  Status Insert(const std::string& input);
  const std::vector<std::optional<std::string>>& GetTable() const { return table_; }
  const std::vector<std::string>& GetStash() const { return stash_; }

 private:
  CuckooHashTable(std::vector<HashFunction> hash_functions, int num_buckets,
                  int max_relocations, std::optional<int> max_stash_size);
  // absl::uniform_int_distribution<int>(0, k-1) over std::mt19937_64
  // (cuckoo_hash_table.h:106-107), restated.
  int RandomHashFunction();

  const int num_buckets_;
  const int max_relocations_;
  const std::optional<int> max_stash_size_;
  std::vector<HashFunction> hash_functions_;
  std::vector<std::optional<std::string>> table_;
  std::vector<std::string> stash_;
  std::mt19937_64 rng_;
};

class CuckooHashedDpfPirDatabase
    : public PirDatabaseInterface<XorWrapper<uint128>, std::pair<std::string, std::string>> {
 public:
  using Interface = PirDatabaseInterface;
  using DenseDatabase = PirDatabaseInterface<XorWrapper<uint128>, std::string>;

  class Builder : public PirDatabaseInterface::Builder {
   public:
    Builder();
    Builder& Insert(RecordType key_value) override;
    std::unique_ptr<PirDatabaseInterface::Builder> Clone() const override;
    Builder& SetParams(CuckooHashingParams params);
    Builder& SetKeyDatabaseBuilder(std::unique_ptr<DenseDatabase::Builder> builder);
    Builder& SetValueDatabaseBuilder(std::unique_ptr<DenseDatabase::Builder> builder);
    StatusOr<std::unique_ptr<PirDatabaseInterface>> Build() override;

    // The host half of Build(): validation and cuckoo placement, returning
    // the bucket table (nullopt = empty bucket). No device work.
    StatusOr<std::vector<std::optional<std::string>>> PlaceKeys() const;

   private:
    CuckooHashingParams params_;
    std::unique_ptr<DenseDatabase::Builder> key_database_builder_;
    std::unique_ptr<DenseDatabase::Builder> value_database_builder_;
    std::map<std::string, std::string> records_;  // absl::btree_map order
    bool has_been_built_ = false;
  };

  size_t size() const override { return size_; }
  size_t num_selection_bits() const override { return num_selection_bits_; }
  StatusOr<std::vector<RecordType>> InnerProductWith(
      Span<const std::vector<BlockType>> selections) const override;

  // Both scans from one device-resident selection buffer (num_queries *
  // selection_blocks blocks). Null when a table is not HBM-resident.
  StatusOr<std::vector<RecordType>> InnerProductWithDevice(const void* selections_dev,
                                                           int64_t selection_blocks,
                                                           int num_queries, void* stream) const;
  bool device_resident() const;
  const DenseDatabase& key_database() const { return *key_database_; }
  const DenseDatabase& value_database() const { return *value_database_; }

 private:
  CuckooHashedDpfPirDatabase(std::unique_ptr<DenseDatabase> key_database,
                             std::unique_ptr<DenseDatabase> value_database, size_t size,
                             size_t num_selection_bits);
  std::unique_ptr<DenseDatabase> key_database_;
  std::unique_ptr<DenseDatabase> value_database_;
  size_t size_;
  size_t num_selection_bits_;
};

class CuckooHashingSparseDpfPirServer : public DpfPirServer {
 public:
  using Database =
      PirDatabaseInterface<XorWrapper<uint128>, std::pair<std::string, std::string>>;
  static constexpr const char* kEncryptionContextInfo = "CuckooHashingSparseDpfPirServer";
  static constexpr int kHashFunctionSeedLengthBytes = 16;

  // cuckoo_hashing_sparse_dpf_pir_server.cc:46-65: 3 hash functions,
  // 1.5 buckets per element, fresh random 16-byte seed.
  static StatusOr<CuckooHashingParams> GenerateParams(const PirConfig& config);

  static StatusOr<std::unique_ptr<CuckooHashingSparseDpfPirServer>> CreatePlain(
      CuckooHashingParams params, std::unique_ptr<Database> database);
  static StatusOr<std::unique_ptr<CuckooHashingSparseDpfPirServer>> CreateLeader(
      CuckooHashingParams params, std::unique_ptr<Database> database,
      ForwardHelperRequestFn sender);
  static StatusOr<std::unique_ptr<CuckooHashingSparseDpfPirServer>> CreateHelper(
      CuckooHashingParams params, std::unique_ptr<Database> database,
      DecryptHelperRequestFn decrypter);

  const PirServerPublicParams& GetPublicParams() const override { return params_; }
  const Database& database() const { return *database_; }

 protected:
  StatusOr<PirResponse> HandlePlainRequest(const PirRequest& request) const override;

 private:
  CuckooHashingSparseDpfPirServer(PirServerPublicParams params,
                                  std::unique_ptr<DistributedPointFunction> dpf,
                                  std::unique_ptr<Database> database);
  PirServerPublicParams params_;
  std::unique_ptr<DistributedPointFunction> dpf_;
  std::unique_ptr<Database> database_;
};

}  // namespace distributed_point_functions

#endif  // DPF_AMD_CUCKOO_HASHING_SPARSE_DPF_PIR_SERVER_H_
