// pir.cc — dense DPF PIR server and HBM-resident database (see
// include/dpf_amd/dense_dpf_pir_server.h for the reference mapping).
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <functional>
#include <map>

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

hipStream_t PirStream() { return dpf_internal_host::ThreadStream(); }

// AlignBytes (pir/dense_dpf_pir_database.cc:40-52).
int64_t AlignBytes(int64_t n) { return (n + 15) & ~int64_t{15}; }

// Device row stride: the reference's 16-byte alignment (KPirScanG maps any
// width onto the wave, so no padding is read), except that rows are padded
// to a whole number of 128-byte cache lines when that costs at most 1/16
// more bytes (rows of ~1.8 KiB and up): a row then starts on a line, and
// the scans' slices of neighbouring rows never share one.  2^20 x 16 KiB
// rows (16,400 -> 16,512 B): FETCH 18.9 -> 17.3 GB, Q = 1 / 10 / 100 2.92 /
// 4.11 / 6.07 -> 2.71 / 3.16 / 5.73 ms; 2 KiB rows (2,064 -> 2,176 B)
// 0.42 / 0.52 / 0.99 -> 0.36 / 0.41 / 0.95 ms (profiles/ab_grid_align_r06q/).
int64_t DeviceRowStride(int64_t max_size) {
  const int64_t s16 = std::max<int64_t>(16, AlignBytes(max_size));
  const int64_t s128 = (s16 + 127) & ~int64_t{127};
  return (s128 - s16) * 16 <= s16 ? s128 : s16;
}


}  // namespace

// ---------------------------------------------------------------------------
// DenseDpfPirDatabase
// ---------------------------------------------------------------------------

DenseDpfPirDatabase::Builder::Builder() = default;

DenseDpfPirDatabase::Builder& DenseDpfPirDatabase::Builder::Insert(std::string value) {
  if (device_records_ != nullptr) {
    mixed_inserts_ = true;
    return *this;
  }
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
  if (device_records_ != nullptr) {
    mixed_inserts_ = true;
    return *this;
  }
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
  r->devices_ = devices_;
  r->device_records_ = device_records_;
  r->device_of_records_ = device_of_records_;
  r->mixed_inserts_ = mixed_inserts_;
  return r;
}

DenseDpfPirDatabase::Builder& DenseDpfPirDatabase::Builder::InsertFixedFromDevice(
    const void* records, int device, int64_t num, int64_t size) {
  if (!values_.empty() || fixed_count_ > 0 || device_records_ != nullptr) mixed_inserts_ = true;
  device_records_ = records;
  device_of_records_ = device;
  fixed_count_ = num;
  fixed_size_ = size;
  total_database_bytes_ += num * AlignBytes(size);
  return *this;
}

DenseDpfPirDatabase::Builder& DenseDpfPirDatabase::Builder::SetDevices(std::vector<int> devices) {
  devices_ = std::move(devices);
  return *this;
}

namespace {

// Device allocation that first returns the pool's idle blocks on failure.
Status MallocOrRelease(void** p, int64_t bytes) {
  hipError_t e = hipMalloc(p, bytes);
  if (e == hipErrorOutOfMemory) {
    // idle blocks cached by earlier Tier-2 calls go back to the device first
    (void)hipGetLastError();
    dpf_internal_host::DevicePool::Get().Release();
    e = hipMalloc(p, bytes);
  }
  return HipStatus(e, "hipMalloc(database)");
}

// Shard g of G over `blocks` 128-record selection blocks: blocks
// [g * blocks / G, (g + 1) * blocks / G).
int64_t ShardBlock(int64_t blocks, int64_t g, int64_t num) { return blocks * g / num; }

}  // namespace

StatusOr<std::unique_ptr<DenseDpfPirDatabase::Interface>> DenseDpfPirDatabase::Builder::Build() {
  if (has_been_built_) return FailedPreconditionError("Database already built");
  if (mixed_inserts_)
    return InvalidArgumentError("InsertFixedFromDevice must be the only insert of a database");
  has_been_built_ = true;
  std::unique_ptr<DenseDpfPirDatabase> db(new DenseDpfPirDatabase());
  const int64_t n = static_cast<int64_t>(values_.size()) + fixed_count_;
  int64_t max_size = fixed_count_ ? fixed_size_ : 0;
  for (const std::string& v : values_) max_size = std::max<int64_t>(max_size, v.size());
  db->num_records_ = n;
  db->max_value_size_ = max_size;
  db->stride_ = DeviceRowStride(max_size);
  std::vector<int> devices = devices_;
  if (devices.empty()) {
    int cur = 0;
    DPF_RETURN_IF_ERROR(HipStatus(hipGetDevice(&cur), "hipGetDevice"));
    devices.push_back(cur);
  }
  for (int d : devices) DPF_RETURN_IF_ERROR(dpf_internal_host::CheckDevice(d));
  if (device_records_ != nullptr)
    DPF_RETURN_IF_ERROR(dpf_internal_host::CheckDevice(device_of_records_));
  const bool force_peer = dpf_amd::ForcePeerCopies();
  const int64_t blocks = (n + 127) / 128;
  const int64_t num = static_cast<int64_t>(devices.size());
  for (int64_t g = 0; g < num; ++g) {
    const int64_t r0 = std::min(n, 128 * ShardBlock(blocks, g, num));
    const int64_t r1 = std::min(n, 128 * ShardBlock(blocks, g + 1, num));
    if (r1 > r0 || (g == 0 && n == 0)) db->shards_.push_back(Shard{devices[g], r0, r1, nullptr});
  }
  // Peer access between shard devices (the partials' combine copies) and
  // from every shard device to the device holding the source rows (the
  // build's row copies).
  auto enable_peer = [](int from, int to) {
    if (from == to) return;
    dpf_internal_host::DeviceGuard g(from);
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, from, to) == hipSuccess && can)
      (void)hipDeviceEnablePeerAccess(to, 0);
    (void)hipGetLastError();  // "already enabled" is not an error here
  };
  for (const Shard& a : db->shards_) {
    for (const Shard& b : db->shards_) enable_peer(a.device, b.device);
    if (device_records_ != nullptr) enable_peer(a.device, device_of_records_);
  }
  // Upload each shard in 64 MiB chunks of zero-padded fixed-stride rows.
  const int64_t rows_per_chunk = std::max<int64_t>(1, (64 << 20) / db->stride_);
  std::vector<char> chunk(rows_per_chunk * db->stride_);
  auto record = [&](int64_t i, const char** src, int64_t* len) {
    if (i < static_cast<int64_t>(values_.size())) {
      *src = values_[i].data();
      *len = static_cast<int64_t>(values_[i].size());
    } else {
      *src = fixed_.data() + (i - static_cast<int64_t>(values_.size())) * fixed_size_;
      *len = fixed_size_;
    }
  };
  if (device_records_ != nullptr) {
    // every kernel or copy that writes the source rows was issued before
    // Build, on whatever stream: drain the source device first
    dpf_internal_host::DeviceGuard g(device_of_records_);
    DPF_RETURN_IF_ERROR(HipStatus(hipDeviceSynchronize(), "hipDeviceSynchronize"));
  }
  for (Shard& sh : db->shards_) {
    dpf_internal_host::DeviceGuard g(sh.device);
    const int64_t bytes = std::max<int64_t>(16, (sh.row_end - sh.row_begin) * db->stride_);
    DPF_RETURN_IF_ERROR(MallocOrRelease(&sh.records, bytes));
    DPF_RETURN_IF_ERROR(HipStatus(hipMemset(sh.records, 0, bytes), "hipMemset(database)"));
    if (device_records_ != nullptr) {
      // records already in HBM: one (peer) copy per shard, rows re-strided
      // to 16-byte alignment when the record size is not a multiple of 16
      const char* src = static_cast<const char*>(device_records_) + sh.row_begin * fixed_size_;
      const int64_t rows = sh.row_end - sh.row_begin;
      if (rows == 0) continue;
      const bool peer = sh.device != device_of_records_ || force_peer;
      if (fixed_size_ == db->stride_ && peer) {
        DPF_RETURN_IF_ERROR(HipStatus(hipMemcpyPeer(sh.records, sh.device, src,
                                                    device_of_records_, rows * fixed_size_),
                                      "database peer copy"));
      } else if (peer) {
        // rows to re-stride on another device: one peer copy of the packed
        // rows into the shard's device, then the strided copy there
        void* packed = nullptr;
        DPF_RETURN_IF_ERROR(MallocOrRelease(&packed, rows * fixed_size_));
        Status cs = HipStatus(hipMemcpyPeer(packed, sh.device, src, device_of_records_,
                                            rows * fixed_size_),
                              "database peer copy");
        if (cs.ok())
          cs = HipStatus(hipMemcpy2D(sh.records, db->stride_, packed, fixed_size_, fixed_size_,
                                     rows, hipMemcpyDeviceToDevice),
                         "database device copy");
        (void)hipFree(packed);
        DPF_RETURN_IF_ERROR(cs);
      } else {
        DPF_RETURN_IF_ERROR(HipStatus(
            hipMemcpy2D(sh.records, db->stride_, src, fixed_size_, fixed_size_, rows,
                        hipMemcpyDeviceToDevice),
            "database device copy"));
      }
      continue;
    }
    for (int64_t r = sh.row_begin; r < sh.row_end; r += rows_per_chunk) {
      const int64_t rows = std::min(rows_per_chunk, sh.row_end - r);
      std::fill(chunk.begin(), chunk.end(), 0);
      for (int64_t k = 0; k < rows; ++k) {
        const char* src;
        int64_t len;
        record(r + k, &src, &len);
        memcpy(chunk.data() + k * db->stride_, src, len);
      }
      DPF_RETURN_IF_ERROR(HipStatus(
          hipMemcpy(static_cast<char*>(sh.records) + (r - sh.row_begin) * db->stride_,
                    chunk.data(), rows * db->stride_, hipMemcpyHostToDevice),
          "upload database"));
    }
  }
  // The copies above run on the null stream; the scans run on the library's
  // non-blocking streams, which do not wait for it: the rows are complete
  // on every shard device before the database is handed out.
  for (const Shard& sh : db->shards_) {
    dpf_internal_host::DeviceGuard g(sh.device);
    DPF_RETURN_IF_ERROR(HipStatus(hipDeviceSynchronize(), "hipDeviceSynchronize"));
  }
  std::vector<std::string>().swap(values_);
  std::vector<char>().swap(fixed_);
  device_records_ = nullptr;
  return std::unique_ptr<Interface>(std::move(db));
}

DenseDpfPirDatabase::~DenseDpfPirDatabase() {
  for (Shard& sh : shards_)
    if (sh.records) {
      dpf_internal_host::DeviceGuard g(sh.device);
      (void)hipFree(sh.records);
    }
}

StatusOr<std::vector<std::string>> DenseDpfPirDatabase::InnerProductWithDevice(
    const void* selections_dev, int64_t selection_blocks, int num_queries, void* stream) const {
  if (num_queries == 0) return std::vector<std::string>();
  if (max_value_size_ <= 0) return InvalidArgumentError("`max_value_size` must be positive");
  if (shards_.size() != 1)
    return FailedPreconditionError("InnerProductWithDevice needs a single-shard database");
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : PirStream();
  const int64_t ws = dpf_amd_inner_product_workspace_size(num_records_, stride_, num_queries);
  void* work = nullptr;
  void* out = nullptr;
  DPF_RETURN_IF_ERROR(dpf_internal_host::DevicePool::Get().Alloc(std::max<int64_t>(ws, 16), s, &work));
  Status st = dpf_internal_host::DevicePool::Get().Alloc(num_queries * stride_, s, &out);
  std::vector<char> host(num_queries * stride_);
  if (st.ok())
    st = AbiStatus(dpf_amd_inner_product(shards_[0].records, num_records_, stride_,
                                         selections_dev, selection_blocks, num_queries, work, out,
                                         s));
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

StatusOr<std::vector<std::string>> DenseDpfPirDatabase::InnerProductSharded(
    const FillSelectionsFn& fill, int num_queries) const {
  using dpf_internal_host::DeviceGuard;
  using dpf_internal_host::DevicePool;
  if (num_queries == 0) return std::vector<std::string>();
  if (max_value_size_ <= 0) return InvalidArgumentError("`max_value_size` must be positive");
  const int64_t part_bytes = static_cast<int64_t>(num_queries) * stride_;
  // Device groups: consecutive shards on one device with adjacent rows share
  // one selection expansion (the group's block range), one workspace (the
  // scans' partials side by side, or one set of atomic fold slots) and one
  // fold — shards are per device, so on a node this is one group per GPU.
  // With forced peer copies every shard is its own group, as if each sat on
  // a device of its own (the rehearsal of the cross-device combine).
  struct Piece {
    Shard sh;
    dpf_amd::ScanPlan plan;
    int64_t ws_off = 0;
  };
  struct Group {
    int device = 0;
    int stream_index = 0;
    int64_t b0 = 0, b1 = 0;
    std::vector<Piece> pieces;
    hipStream_t s = nullptr;
    bool slots = true;
    dpf_internal_host::FoldSlots::Entry* slot_entry = nullptr;
    bool fold_cleared = false;  // the clearing fold was enqueued on `s`
    int fold_parts = 0;
    void* buf = nullptr;
    char* sel = nullptr;
    char* ws = nullptr;
    char* part = nullptr;
    hipEvent_t done = nullptr;
  };
  const bool force_peer = dpf_amd::ForcePeerCopies();
  std::vector<Group> w;
  {
    std::map<int, int> next_index;
    for (const Shard& sh : shards_) {
      const int64_t b0 = sh.row_begin / 128, b1 = (sh.row_end + 127) / 128;
      if (force_peer || w.empty() || w.back().device != sh.device || w.back().b1 != b0) {
        Group g;
        g.device = sh.device;
        g.b0 = b0;
        g.b1 = b0;
        g.stream_index = next_index[sh.device]++;
        g.s = dpf_internal_host::ThreadStreamOn(sh.device, g.stream_index);
        w.push_back(g);
      }
      Group& g = w.back();
      g.b1 = std::max(g.b1, b1);
      Piece pc;
      pc.sh = sh;
      pc.plan = dpf_amd::PlanScan(sh.row_end - sh.row_begin, stride_, num_queries);
      g.slots &= pc.plan.slots;
      g.pieces.push_back(pc);
    }
  }
  const size_t G = w.size();
  dpf_internal_host::HostTrace trace("InnerProductSharded");
  const int dev0 = w[0].device;
  hipStream_t s0 = w[0].s;
  void* gather = nullptr;
  void* folded = nullptr;
  std::vector<char> host;
  Status st = OkStatus();
  // The last fold writes the answer straight into pinned host memory mapped
  // into the device (no D2H copy behind it) when it is small.
  void* hout = nullptr;
  void* kout = nullptr;
  if (part_bytes <= static_cast<int64_t>(dpf_internal_host::HostOutMax()))
    st = dpf_internal_host::ThreadRecycled<dpf_internal_host::PinnedOut>::Get().Get(
        part_bytes, &hout, &kout);
  if (!kout) host.resize(part_bytes);
  auto align = [](int64_t b) { return (b + 255) & ~int64_t{255}; };
  // 1. every group: one allocation, its selection blocks, its scans and its
  // fold, back to back on its own stream
  for (size_t gi = 0; gi < G && st.ok(); ++gi) {
    Group& g = w[gi];
    DeviceGuard dg(g.device);
    if (g.s == nullptr) {
      st = InternalError("no stream on device " + std::to_string(g.device));
      break;
    }
    const int64_t nb = std::max<int64_t>(1, g.b1 - g.b0);
    int64_t ws_bytes = 0;
    if (g.slots) {
      g.fold_parts = dpf_amd::ScanFoldParts(g.pieces[0].plan);
      ws_bytes = g.fold_parts * part_bytes;
    } else {
      for (Piece& pc : g.pieces) {
        pc.plan.slots = false;
        pc.ws_off = ws_bytes;
        ws_bytes += dpf_amd::ScanFoldParts(pc.plan) * part_bytes;
      }
      g.fold_parts = static_cast<int>(ws_bytes / part_bytes);
    }
    // atomic fold slots live in the thread's zeroed FoldSlots, per-block
    // partials in the request's allocation
    const int64_t sel_bytes = align(16 * nb * num_queries);
    const int64_t ws_own = g.slots ? 0 : align(std::max<int64_t>(16, ws_bytes));
    const int64_t total = sel_bytes + ws_own + part_bytes;
    st = DevicePool::Get().Alloc(total, g.s, &g.buf);
    if (!st.ok()) break;
    g.sel = static_cast<char*>(g.buf);
    g.ws = g.sel + sel_bytes;
    g.part = g.ws + ws_own;
    if (g.slots)
      st = dpf_internal_host::ThreadRecycled<dpf_internal_host::FoldSlots>::Get().Acquire(
          g.device, g.stream_index, ws_bytes, g.s, &g.ws, &g.slot_entry);
    if (st.ok()) st = fill(g.pieces[0].sh, g.b0, g.b0 + nb, g.sel, g.s);
    for (size_t k = 0; k < g.pieces.size() && st.ok(); ++k) {
      const Piece& pc = g.pieces[k];
      const int64_t rows = pc.sh.row_end - pc.sh.row_begin;
      const int64_t pb0 = pc.sh.row_begin / 128 - g.b0;
      // query q's blocks of this piece: row q of the group's [query][nb]
      st = AbiStatus(dpf_amd::ScanPiece(pc.sh.records, rows, stride_, g.sel + 16 * pb0, nb,
                                        num_queries, pc.plan, g.ws + (g.slots ? 0 : pc.ws_off),
                                        g.s));
    }
    if (st.ok()) {
      void* fold_out = G == 1 && kout ? kout : g.part;
      if (g.slots) {
        st = AbiStatus(dpf_amd::XorFoldClear(g.ws, g.fold_parts, part_bytes, fold_out, g.s));
        g.fold_cleared = st.ok();  // clean only once the request has synchronized OK
      } else {
        st = AbiStatus(dpf_amd_xor_fold(g.ws, g.fold_parts, part_bytes, fold_out, g.s));
      }
    }
    if (st.ok() && G > 1) {
      st = HipStatus(hipEventCreateWithFlags(&g.done, hipEventDisableTiming), "hipEventCreate");
      if (st.ok()) st = HipStatus(hipEventRecord(g.done, g.s), "hipEventRecord");
    }
  }
  trace.Mark("selections+scan_launch");
  // 2. combine on the first group's device: (peer) copies of the partials,
  // one XOR fold, one D2H
  const void* result = nullptr;
  if (st.ok()) {
    DeviceGuard dg(dev0);
    if (G == 1) {
      result = w[0].part;
    } else {
      st = DevicePool::Get().Alloc(part_bytes * G, s0, &gather);
      if (st.ok()) st = DevicePool::Get().Alloc(part_bytes, s0, &folded);
      for (size_t g = 0; g < G && st.ok(); ++g) {
        char* dst = static_cast<char*>(gather) + g * part_bytes;
        st = HipStatus(hipStreamWaitEvent(s0, w[g].done, 0), "hipStreamWaitEvent");
        if (!st.ok()) break;
        if (w[g].device == dev0 && !force_peer)
          st = HipStatus(hipMemcpyAsync(dst, w[g].part, part_bytes, hipMemcpyDeviceToDevice, s0),
                         "partials copy");
        else
          st = HipStatus(hipMemcpyPeerAsync(dst, dev0, w[g].part, w[g].device, part_bytes, s0),
                         "partials peer copy");
      }
      if (st.ok())
        st = AbiStatus(dpf_amd_xor_fold(gather, static_cast<int>(G), part_bytes,
                                        kout ? kout : folded, s0));
      result = folded;
    }
    if (st.ok() && !kout)
      st = HipStatus(hipMemcpyAsync(host.data(), result, part_bytes, hipMemcpyDeviceToHost, s0),
                     "d2h");
  }
  trace.Mark("combine_launch");
  // 3. drain every stream used, then return the buffers (no copy still reads them)
  for (size_t g = 0; g < G; ++g) {
    if (!w[g].s) continue;
    DeviceGuard dg(w[g].device);
    Status sy = HipStatus(hipStreamSynchronize(w[g].s), "sync");
    if (st.ok()) st = sy;
  }
  {
    DeviceGuard dg(dev0);
    Status sy = HipStatus(hipStreamSynchronize(s0), "sync");
    if (st.ok()) st = sy;
    if (gather) DevicePool::Get().Free(gather, s0);
    if (folded) DevicePool::Get().Free(folded, s0);
  }
  // The fold slots count as zeroed only when the fold that cleared them ran
  // and every stream of the request synchronized without error; otherwise
  // the next request on them zeroes them first.
  for (size_t g = 0; g < G; ++g)
    if (st.ok() && w[g].fold_cleared) dpf_internal_host::FoldSlots::MarkClean(w[g].slot_entry);
  for (size_t g = 0; g < G; ++g) {
    DeviceGuard dg(w[g].device);
    if (w[g].buf) DevicePool::Get().Free(w[g].buf, w[g].s);
    if (w[g].done) (void)hipEventDestroy(w[g].done);
  }
  trace.Mark("sync+free");
  if (!st.ok()) return st;
  const char* answer = kout ? static_cast<const char*>(hout) : host.data();
  std::vector<std::string> r(num_queries);
  for (int q = 0; q < num_queries; ++q) r[q].assign(answer + q * stride_, max_value_size_);
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
  // Only the blocks that select existing records are read by the scan: each
  // shard gets its own blocks of every query, query-major.
  const int q = static_cast<int>(selections.size());
  auto fill = [&](const Shard&, int64_t b0, int64_t b1, void* dev, void* stream) -> Status {
    const int64_t nb = std::max<int64_t>(1, b1 - b0);
    std::vector<uint128> host(static_cast<size_t>(q) * nb);
    for (int k = 0; k < q; ++k)
      for (int64_t b = b0; b < b1 && b < static_cast<int64_t>(first); ++b)
        host[k * nb + (b - b0)] = selections[k][b].value();
    // host is a local: copied through the pinned ring (async, safe to return)
    return dpf_internal_host::ThreadUploadRing().Copy(dev, host.data(), 16 * host.size(),
                                                     static_cast<hipStream_t>(stream));
  };
  return InnerProductSharded(fill, q);
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
  dpf_internal_host::HostTrace trace("HandlePlainRequest");
  const auto* gpu_db = dynamic_cast<const DenseDpfPirDatabase*>(database_.get());
  if (gpu_db != nullptr) {
    // Fused path: expand only the selection blocks the scan reads, straight
    // into HBM, then scan; a sharded database expands each shard's blocks
    // (a leaf range of every key) on the shard's device.
    for (int i = 0; i < q; ++i) {
      StatusOr<EvaluationContext> ctx = dpf_->CreateEvaluationContext(plain.dpf_key(i));
      if (!ctx.ok()) return ctx.status();
    }
    const dpf_amd_value_type layout = dpf_internal::HostLayoutOf<XorWrapper<uint128>>();
    std::vector<const DpfKey*> keys(q);
    for (int i = 0; i < q; ++i) keys[i] = &plain.dpf_key(i);
    trace.Mark("validate");
    auto fill = [&](const DenseDpfPirDatabase::Shard&, int64_t b0, int64_t b1, void* sel,
                    void* stream) -> Status {
      return dpf_->ExpandLeavesOnDeviceBatched(Span<const DpfKey* const>(keys.data(), keys.size()),
                                               b0, std::max(b1, b0 + 1), layout, sel, stream);
    };
    StatusOr<std::vector<std::string>> r = gpu_db->InnerProductSharded(fill, q);
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
  trace.Mark("inner_products+response");
  return response;
}

}  // namespace distributed_point_functions
