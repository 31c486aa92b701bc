// dense_dpf_pir_server.h — dense two-server DPF PIR on MI355X.
//   PirDatabaseInterface        pir/pir_database_interface.h:31-74
//   DenseDpfPirDatabase         pir/dense_dpf_pir_database.h:45-112 (records in HBM)
//   DpfPirServer roles          pir/dpf_pir_server.h:75-174
//   DenseDpfPirServer           pir/dense_dpf_pir_server.h:37-112
// HandlePlainRequest expands each DPF key on the device straight into the
// selection buffer (only the ceil(N/128) leaves the scan reads) and runs the
// HBM-streaming XOR scan; nothing crosses PCIe but the keys and responses.
#ifndef DPF_AMD_DENSE_DPF_PIR_SERVER_H_
#define DPF_AMD_DENSE_DPF_PIR_SERVER_H_

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "dpf_amd/distributed_point_function.h"
#include "dpf_amd/protos.h"
#include "dpf_amd/status.h"
#include "dpf_amd/value_types.h"

namespace distributed_point_functions {

template <typename BlockTypeT, typename RecordTypeT>
class PirDatabaseInterface {
 public:
  using BlockType = BlockTypeT;
  using RecordType = RecordTypeT;
  class Builder {
   public:
    Builder() = default;
    virtual ~Builder() = default;
    Builder(Builder&) = delete;
    Builder& operator=(Builder&) = delete;
    virtual Builder& Insert(RecordType) = 0;
    virtual std::unique_ptr<Builder> Clone() const = 0;
    virtual StatusOr<std::unique_ptr<PirDatabaseInterface>> Build() = 0;
  };
  virtual ~PirDatabaseInterface() {}
  virtual StatusOr<std::vector<RecordType>> InnerProductWith(
      Span<const std::vector<BlockType>> selections) const = 0;
  virtual size_t size() const = 0;
  virtual size_t num_selection_bits() const = 0;
};

// HBM-resident dense database.  Records are stored with a fixed stride
// (max record size rounded up to 16 bytes), zero padded, so the scan is a
// pure coalesced stream; results are identical to the reference's packed
// layout because padding bytes are zero and responses are truncated to the
// maximum record size.
class DenseDpfPirDatabase : public PirDatabaseInterface<XorWrapper<uint128>, std::string> {
 public:
  using Interface = PirDatabaseInterface;

  class Builder : public PirDatabaseInterface::Builder {
   public:
    Builder();
    Builder& Insert(std::string value) override;
    // Bulk insert of `num` records of `size` bytes each (fast path).
    Builder& InsertFixed(const char* data, int64_t num, int64_t size);
    // Bulk insert of `num` records of `size` bytes each that already live in
    // device memory on `device` (consecutive, `size` bytes apart): Build()
    // copies them device-to-device (peer copies for shards elsewhere) and
    // never stages them through the host.  Must be the only insert.
    Builder& InsertFixedFromDevice(const void* records, int device, int64_t num, int64_t size);
    std::unique_ptr<PirDatabaseInterface::Builder> Clone() const override;
    StatusOr<std::unique_ptr<PirDatabaseInterface>> Build() override;
    int64_t total_database_bytes() const { return total_database_bytes_; }
    // Devices the records are sharded over: contiguous row ranges aligned to
    // the 128-record selection blocks, one per entry, in order (entries may
    // repeat: {0, 0, 0, 0} is four shards on device 0).  Empty (default):
    // one shard on the current device.
    Builder& SetDevices(std::vector<int> devices);

   private:
    std::vector<std::string> values_;
    std::vector<char> fixed_;
    int64_t fixed_count_ = 0, fixed_size_ = 0;
    int64_t total_database_bytes_ = 0;
    bool has_been_built_ = false;
    std::vector<int> devices_;
    const void* device_records_ = nullptr;  // InsertFixedFromDevice
    int device_of_records_ = 0;
    bool mixed_inserts_ = false;
  };

  // Rows [row_begin, row_end) on `device` (selection blocks row_begin / 128
  // up to ceil(row_end / 128)), stored at `records` with the database stride.
  struct Shard {
    int device;
    int64_t row_begin, row_end;
    void* records;
  };

  ~DenseDpfPirDatabase() override;
  size_t size() const override { return static_cast<size_t>(num_records_); }
  size_t num_selection_bits() const override { return size(); }
  StatusOr<std::vector<std::string>> InnerProductWith(
      Span<const std::vector<BlockType>> selections) const override;
  size_t max_value_size_in_bytes() const { return static_cast<size_t>(max_value_size_); }

  // Device-side inner product of a single-shard database: `selections_dev`
  // holds num_queries * selection_blocks 128-bit blocks in HBM; returns host
  // strings.
  StatusOr<std::vector<std::string>> InnerProductWithDevice(const void* selections_dev,
                                                            int64_t selection_blocks,
                                                            int num_queries,
                                                            void* stream) const;
  // Sharded inner product: for every shard, `fill(shard, block_begin,
  // block_end, selections_dev, stream)` writes the num_queries x (block_end -
  // block_begin) selection blocks of the shard's rows (query-major) into
  // device memory on the shard's device, stream-ordered on `stream` (that
  // device's stream of the calling thread); each shard is scanned there, and
  // the num_queries x record partials of all shards are copied to the first
  // shard's device (peer copies over xGMI) and XOR-folded (KXorFold).
  using FillSelectionsFn = std::function<Status(const Shard& shard, int64_t block_begin,
                                                int64_t block_end, void* selections_dev,
                                                void* stream)>;
  StatusOr<std::vector<std::string>> InnerProductSharded(const FillSelectionsFn& fill,
                                                         int num_queries) const;
  const std::vector<Shard>& shards() const { return shards_; }
  const void* device_records() const { return shards_.empty() ? nullptr : shards_[0].records; }
  int64_t record_stride() const { return stride_; }

 private:
  DenseDpfPirDatabase() = default;
  std::vector<Shard> shards_;
  int64_t num_records_ = 0;
  int64_t stride_ = 16;
  int64_t max_value_size_ = 0;
};

class PirServer {
 public:
  virtual ~PirServer() = default;
  virtual const PirServerPublicParams& GetPublicParams() const = 0;
  virtual StatusOr<PirResponse> HandleRequest(const PirRequest& request) const = 0;
};

class DpfPirServer : public PirServer {
 public:
  enum class Role { kPlain = 0, kLeader, kHelper };
  using ForwardHelperRequestFn = std::function<StatusOr<PirResponse>(
      const PirRequest& helper_request, std::function<void()> while_waiting)>;
  using DecryptHelperRequestFn = std::function<StatusOr<std::string>(
      const std::string& encrypted_helper_request, const std::string& encryption_context_info)>;

  Role role() const { return role_; }
  StatusOr<PirResponse> HandleRequest(const PirRequest& request) const final;

 protected:
  DpfPirServer() = default;
  virtual StatusOr<PirResponse> HandlePlainRequest(const PirRequest& request) const = 0;
  Status MakeLeader(ForwardHelperRequestFn sender);
  Status MakeHelper(DecryptHelperRequestFn decrypter, std::string encryption_context_info);

 private:
  StatusOr<PirResponse> HandleLeaderRequest(const PirRequest& request) const;
  StatusOr<PirResponse> HandleHelperRequest(const PirRequest& request) const;
  Role role_ = Role::kPlain;
  ForwardHelperRequestFn sender_;
  DecryptHelperRequestFn decrypter_;
  std::string encryption_context_info_;
};

class DenseDpfPirServer : public DpfPirServer {
 public:
  using Database = PirDatabaseInterface<XorWrapper<uint128>, std::string>;
  static constexpr const char* kEncryptionContextInfo = "DenseDpfPirServer";

  static StatusOr<std::unique_ptr<DenseDpfPirServer>> CreateLeader(
      const PirConfig& config, std::unique_ptr<Database> database, ForwardHelperRequestFn sender);
  static StatusOr<std::unique_ptr<DenseDpfPirServer>> CreateHelper(
      const PirConfig& config, std::unique_ptr<Database> database,
      DecryptHelperRequestFn decrypter);
  static StatusOr<std::unique_ptr<DenseDpfPirServer>> CreatePlain(
      const PirConfig& config, std::unique_ptr<Database> database);

  const Database& database() const { return *database_; }
  const DistributedPointFunction& dpf() const { return *dpf_; }
  const PirServerPublicParams& GetPublicParams() const override;

 protected:
  StatusOr<PirResponse> HandlePlainRequest(const PirRequest& request) const override;

 private:
  DenseDpfPirServer(std::unique_ptr<DistributedPointFunction> dpf,
                    std::unique_ptr<Database> database);
  std::unique_ptr<DistributedPointFunction> dpf_;
  std::unique_ptr<Database> database_;
};

// Aes128CtrSeededPrng one-time pad (pir/prng/aes_128_ctr_seeded_prng.cc):
// bytes [offset, offset + length) of the key stream of `seed` (16 bytes).
std::string AesCtrOneTimePad(const std::string& seed, size_t offset, size_t length);

}  // namespace distributed_point_functions

#endif  // DPF_AMD_DENSE_DPF_PIR_SERVER_H_
