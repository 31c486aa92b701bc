// host_device.h — host-side HIP plumbing shared by the Tier-2 objects
// (csrc/dpf.cc, csrc/dcf.cc): status mapping, the per-thread stream and a
// stream-ordered device buffer.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <thread>
#include <map>
#include <mutex>
#include <unordered_map>
#include <utility>
#include <vector>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "dpf_amd.h"
#include "dpf_amd/status.h"
#include "internal.h"

namespace distributed_point_functions {
namespace dpf_internal_host {


inline Status HipStatus(hipError_t e, const char* what) {
  if (e == hipSuccess) return OkStatus();
  if (e == hipErrorOutOfMemory)
    return ResourceExhaustedError(std::string(what) + ": " + hipGetErrorString(e));
  return InternalError(std::string(what) + ": " + hipGetErrorString(e));
}

inline Status AbiStatus(int rc) {
  if (rc == DPF_AMD_OK) return OkStatus();
  return Status(static_cast<StatusCode>(rc), dpf_amd::LastError());
}

// Per-thread host resources (streams, pinned staging buffers, events) are
// recycled through a process-wide free list when their thread exits instead
// of being destroyed: a server answering from many short-lived threads pays
// for stream / pinned-memory creation once per concurrent thread, not once
// per thread, and no HIP call runs in a thread-exit handler.  (Round 3's
// 128-thread test crashed in the runtime while per-thread objects were
// destroyed in exit handlers and other threads launched work; that run's
// output was not kept, so the exit handlers are the suspected, not the
// proven, cause — DESIGN.md §5.)  Every recycled object waits for its own
// in-flight work before it reuses a buffer, so a new owner thread inherits it
// safely.  At most ThreadCacheCap() idle objects of a kind are kept; an exit
// handler parks the surplus, and the next thread to take an object (in its
// first Get, a live thread) destroys it.
template <class T>
class ThreadRecycled {
 public:
  static T& Get() {
    thread_local Holder h;
    return *h.p;
  }
  // Idle objects kept for future threads, and surplus awaiting destruction.
  static std::pair<size_t, size_t> Idle() {
    std::lock_guard<std::mutex> l(P().mu);
    return {P().free.size(), P().surplus.size()};
  }

 private:
  struct Pool {
    std::mutex mu;
    std::vector<T*> free;
    std::vector<T*> surplus;
  };
  static Pool& P() {
    static Pool* p = new Pool();
    return *p;
  }
  struct Holder {
    T* p = nullptr;
    Holder() {
      std::vector<T*> drop;
      {
        std::lock_guard<std::mutex> l(P().mu);
        if (!P().free.empty()) {
          p = P().free.back();
          P().free.pop_back();
        }
        drop.swap(P().surplus);
      }
      for (T* x : drop) delete x;  // outside the lock, in a live thread
      if (p == nullptr) p = new T();
    }
    ~Holder() {
      std::lock_guard<std::mutex> l(P().mu);
      const size_t cap = static_cast<size_t>(std::max(0, dpf_amd::ThreadCacheCap()));
      (P().free.size() < cap ? P().free : P().surplus).push_back(p);
    }
  };
};

// Makes `device` current for the guard's scope (the HIP runtime's current
// device is per thread) and restores the previous one.
class DeviceGuard {
 public:
  explicit DeviceGuard(int device) {
    if (hipGetDevice(&prev_) != hipSuccess) {
      prev_ = -1;
      (void)hipGetLastError();
    }
    if (device >= 0 && device != prev_) {
      if (hipSetDevice(device) == hipSuccess) {
        set_ = true;
      } else {
        ok_ = false;
        (void)hipGetLastError();  // not left sticky for the next launch check
      }
    }
  }
  ~DeviceGuard() {
    if (set_ && prev_ >= 0) (void)hipSetDevice(prev_);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
  // false when the device could not be made current
  bool ok() const { return ok_; }

 private:
  int prev_ = -1;
  bool set_ = false;
  bool ok_ = true;
};

// INVALID_ARGUMENT unless 0 <= device < the number of visible devices.
inline Status CheckDevice(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    n = 0;
  }
  if (device < 0 || device >= n)
    return InvalidArgumentError("invalid device id " + std::to_string(device) + " (" +
                                std::to_string(n) + " visible)");
  return OkStatus();
}

// The calling thread's stream number `index` on `device` (sharded
// databases and multi-GPU expansions issue each device's work on its own
// stream from one thread; pieces of work on one device that should overlap
// take different indices).
struct ThreadStreams {
  std::map<std::pair<int, int>, hipStream_t> s;
};
inline hipStream_t ThreadStreamOn(int device, int index = 0) {
  ThreadStreams& h = ThreadRecycled<ThreadStreams>::Get();
  const std::pair<int, int> key(device, index);
  auto it = h.s.find(key);
  if (it != h.s.end()) return it->second;
  DeviceGuard g(device);
  if (!g.ok()) return nullptr;  // never file a stream of another device under `device`
  hipStream_t st = nullptr;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  h.s[key] = st;
  return st;
}

// The calling thread's stream on its current device.
inline hipStream_t ThreadStream() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  return ThreadStreamOn(dev);
}

// Host-side phase timer: with DPF_AMD_TRACE_HOST set, Mark(name) prints the
// wall time since the previous mark to stderr (the reference has no tracing;
// this is how the Tier-2 host overhead is attributed).
class HostTrace {
 public:
  explicit HostTrace(const char* scope)
      : scope_(scope), on_(std::getenv("DPF_AMD_TRACE_HOST") != nullptr),
        t_(std::chrono::steady_clock::now()) {}
  void Mark(const char* phase) {
    if (!on_) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[dpf_amd] %s/%s %.3f ms\n", scope_, phase,
                 std::chrono::duration<double, std::milli>(now - t_).count());
    t_ = now;
  }

 private:
  const char* scope_;
  bool on_;
  std::chrono::steady_clock::time_point t_;
};

// Device-to-host copy on `s`.  DPF_AMD_SYNC_D2H=1 drains the stream before
// the copy is issued (diagnostics of kernel -> copy ordering).
inline Status CopyToHost(void* dst, const void* src, size_t bytes, hipStream_t s) {
  static const bool drain = std::getenv("DPF_AMD_SYNC_D2H") != nullptr;
  if (drain) DPF_RETURN_IF_ERROR(HipStatus(hipStreamSynchronize(s), "sync"));
  return HipStatus(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s), "d2h");
}

// Drains `s` when it goes out of scope unless dismissed: an early error
// return must not leave an async D2H copy in flight into host memory the
// returning function owns (locals, unique_ptr arrays).
class StreamSyncGuard {
 public:
  explicit StreamSyncGuard(hipStream_t s) : s_(s) {}
  StreamSyncGuard(const StreamSyncGuard&) = delete;
  StreamSyncGuard& operator=(const StreamSyncGuard&) = delete;
  ~StreamSyncGuard() {
    if (s_) (void)hipStreamSynchronize(s_);
  }
  void Dismiss() { s_ = nullptr; }

 private:
  hipStream_t s_;
};

// A few persistent host worker threads for the Tier-2 paths' data-parallel
// host loops: Run(parts, fn) calls fn(0..parts-1) spread over the workers
// and the caller and returns when all are done (one Run in flight at a
// time; fn must not call Run).  One thread copies from pinned into pageable
// memory at ~8 GB/s, below the PCIe DMA rate, and the incremental path's
// per-prefix loops (2^16 per level at c3) are memory-bound the same way.
class HostPool {
 public:
  static constexpr size_t kWorkers = 7;
  static HostPool& Get() {
    static HostPool* pool = new HostPool();  // never destroyed: workers live to exit
    return *pool;
  }
  template <typename Fn>
  void Run(size_t parts, const Fn& fn) {
    if (parts <= 1) {
      if (parts == 1) fn(size_t{0});
      return;
    }
    // Another thread's job holds the workers: run this one inline rather
    // than queue behind it (a many-thread server's host loops and pinned
    // copies then proceed side by side instead of one Run at a time).
    std::unique_lock<std::mutex> one(call_mu_, std::try_to_lock);
    if (!one.owns_lock()) {
      for (size_t i = 0; i < parts; ++i) fn(i);
      return;
    }
    Job job{&fn, [](const void* f, size_t i) { (*static_cast<const Fn*>(f))(i); }};
    {
      std::lock_guard<std::mutex> l(mu_);
      job_ = job;
      next_ = 1;
      parts_ = parts;
      pending_ = parts - 1;
      ++gen_;
    }
    cv_.notify_all();
    fn(size_t{0});  // part 0 on the caller
    std::unique_lock<std::mutex> l(mu_);
    done_cv_.wait(l, [&] { return pending_ == 0; });
  }
  // Splits [0, n) into at most kWorkers + 1 ranges of at least `grain`.
  // Returns the number of ranges (range i is fn's first argument).
  template <typename Fn>
  int ParallelRanges(int64_t n, int64_t grain, const Fn& fn) {
    const int64_t parts =
        std::max<int64_t>(1, std::min<int64_t>(kWorkers + 1, n / std::max<int64_t>(grain, 1)));
    const int64_t per = (n + parts - 1) / parts;
    Run(static_cast<size_t>(parts), [&](size_t i) {
      const int64_t b = static_cast<int64_t>(i) * per;
      fn(static_cast<int>(i), std::min(b, n), std::min(b + per, n));
    });
    return static_cast<int>(parts);
  }
  // memcpy split over the pool in pieces of at least `grain` bytes
  void Copy(char* dst, const char* src, size_t bytes, size_t grain = size_t{1} << 20) {
    const size_t parts = std::min<size_t>(kWorkers + 1, std::max<size_t>(1, bytes / grain));
    const size_t per = (bytes + parts - 1) / parts;
    Run(parts, [&](size_t i) {
      const size_t off = i * per;
      if (off < bytes) std::memcpy(dst + off, src + off, std::min(per, bytes - off));
    });
  }

 private:
  struct Job {
    const void* fn;
    void (*call)(const void*, size_t);
  };
  HostPool() {
    for (size_t i = 0; i < kWorkers; ++i) std::thread([this] { Work(); }).detach();
  }
  void Work() {
    uint64_t seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> l(mu_);
      cv_.wait(l, [&] { return gen_ != seen && next_ < parts_; });
      seen = gen_;
      while (next_ < parts_) {
        const size_t i = next_++;
        const Job job = job_;
        l.unlock();
        job.call(job.fn, i);
        l.lock();
        if (--pending_ == 0) done_cv_.notify_one();
      }
    }
  }
  std::mutex call_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  Job job_{nullptr, nullptr};
  size_t next_ = 0, parts_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
};

// Largest D2H copy into pageable memory left to the runtime's own path
// (DPF_AMD_D2H_DIRECT_KB, default 1024; A/B of the staging threshold).
inline size_t D2HDirectMax() {
  static const size_t v = [] {
    const char* e = std::getenv("DPF_AMD_D2H_DIRECT_KB");
    return (e ? std::strtoull(e, nullptr, 10) : 1024ull) << 10;
  }();
  return v;
}

// Small results written by the kernel straight into pinned host memory
// (up to DPF_AMD_HOST_OUT_KB, default 1024): one EvaluateAt's outputs then
// reach the host without a copy-engine transfer and its completion wait —
// the kernel's stores cross PCIe as it retires, and the call copies the
// block into the caller's buffer after one stream sync.
inline size_t HostOutMax() {
  static const size_t v = [] {
    const char* e = std::getenv("DPF_AMD_HOST_OUT_KB");
    return (e ? std::strtoull(e, nullptr, 10) : 1024ull) << 10;
  }();
  return v;
}
class PinnedOut {
 public:
  PinnedOut() = default;
  PinnedOut(const PinnedOut&) = delete;
  PinnedOut& operator=(const PinnedOut&) = delete;
  ~PinnedOut() {
    if (p_) (void)hipHostFree(p_);
  }
  // A block of at least `bytes` (host pointer, and the pointer kernels
  // write through); the previous user has synchronized.
  Status Get(size_t bytes, void** host, void** dev) {
    if (cap_ < bytes) {
      if (p_) (void)hipHostFree(p_);
      p_ = d_ = nullptr;
      cap_ = 0;
      size_t cap = 64u << 10;
      while (cap < bytes) cap <<= 1;
      DPF_RETURN_IF_ERROR(HipStatus(
          hipHostMalloc(&p_, cap, hipHostMallocMapped | hipHostMallocPortable), "hipHostMalloc"));
      DPF_RETURN_IF_ERROR(HipStatus(hipHostGetDevicePointer(&d_, p_, 0), "hipHostGetDevicePointer"));
      cap_ = cap;
    }
    *host = p_;
    *dev = d_;
    return OkStatus();
  }

 private:
  void* p_ = nullptr;
  void* d_ = nullptr;
  size_t cap_ = 0;
};

// The masked scan's atomic fold slots, kept zeroed between requests per
// (device, stream index): the fold that reads them writes them back to zero
// (dpf_amd::XorFoldClear), so a request needs no memset — one dispatch and
// its dependent gap, ~10 us of a 0.4 ms shard request — in front of its
// selection expansion.  A buffer is dirty from Acquire until the clearing
// fold has run and the request's streams synchronized without error
// (MarkClean); a dirty one (a request that stopped or failed between its
// scan and the end of its fold, a new or grown buffer) is zeroed whole by
// the next Acquire.  DPF_AMD_FOLD_CLEAR=0 zeroes on every Acquire (A/B).  The
// previous user has synchronized.
class FoldSlots {
 public:
  FoldSlots() = default;
  FoldSlots(const FoldSlots&) = delete;
  FoldSlots& operator=(const FoldSlots&) = delete;
  ~FoldSlots() {
    for (auto& e : m_)
      if (e.second.p) (void)hipFree(e.second.p);
  }
  struct Entry {
    void* p = nullptr;
    size_t cap = 0;
    bool clean = false;
  };
  // Zeroed slots of at least `bytes` on the current device, ordered on `s`.
  Status Acquire(int device, int index, size_t bytes, hipStream_t s, char** p, Entry** entry) {
    static const bool always_zero = [] {
      const char* e = std::getenv("DPF_AMD_FOLD_CLEAR");
      return e != nullptr && std::strcmp(e, "0") == 0;
    }();
    Entry& e = m_[{device, index}];
    if (e.cap < bytes) {
      if (e.p) (void)hipFree(e.p);  // idle: its last user synchronized
      e.p = nullptr;
      e.cap = 0;
      size_t cap = 64u << 10;
      while (cap < bytes) cap <<= 1;
      DPF_RETURN_IF_ERROR(HipStatus(hipMalloc(&e.p, cap), "hipMalloc(fold slots)"));
      e.cap = cap;
      e.clean = false;
    }
    if (!e.clean || always_zero)
      DPF_RETURN_IF_ERROR(HipStatus(hipMemsetAsync(e.p, 0, e.cap, s), "scan slots memset"));
    e.clean = false;
    *p = static_cast<char*>(e.p);
    *entry = &e;
    return OkStatus();
  }
  static void MarkClean(Entry* e) { e->clean = true; }

 private:
  std::map<std::pair<int, int>, Entry> m_;
};

// Device-to-host copy into pageable `dst`, complete on return.  A plain
// hipMemcpy into pageable memory stages through the runtime's own small
// pinned buffers one after the other; copies above 1 MiB here go through two
// pinned 4 MiB chunks per thread, the DMA of chunk i + 1 overlapping the
// host memcpy of chunk i (c3: 128 MiB per level).
class D2HStaging {
 public:
  static constexpr size_t kChunk = 4u << 20;
  D2HStaging() = default;
  D2HStaging(const D2HStaging&) = delete;
  D2HStaging& operator=(const D2HStaging&) = delete;
  ~D2HStaging() {
    for (int i = 0; i < 2; ++i) {
      if (ev_[i]) {
        (void)hipEventSynchronize(ev_[i]);
        (void)hipEventDestroy(ev_[i]);
      }
      if (pin_[i]) (void)hipHostFree(pin_[i]);
    }
  }
  Status Copy(char* dst, const char* src, size_t bytes, hipStream_t s) {
    int dev = 0;
    DPF_RETURN_IF_ERROR(HipStatus(hipGetDevice(&dev), "hipGetDevice"));
    for (int i = 0; i < 2; ++i) {
      if (!pin_[i])
        DPF_RETURN_IF_ERROR(HipStatus(hipHostMalloc(&pin_[i], kChunk, 0), "hipHostMalloc"));
      if (ev_[i] && dev_[i] != dev) {  // events are recorded on streams of their device
        (void)hipEventDestroy(ev_[i]);  // idle: every copy below ends synchronized
        ev_[i] = nullptr;
      }
      if (!ev_[i]) {
        DPF_RETURN_IF_ERROR(
            HipStatus(hipEventCreateWithFlags(&ev_[i], hipEventDisableTiming), "hipEventCreate"));
        dev_[i] = dev;
      }
    }
    const size_t n = (bytes + kChunk - 1) / kChunk;
    auto len = [&](size_t i) { return std::min(kChunk, bytes - i * kChunk); };
    for (size_t i = 0; i <= n; ++i) {
      if (i < n) {
        DPF_RETURN_IF_ERROR(HipStatus(hipMemcpyAsync(pin_[i & 1], src + i * kChunk, len(i),
                                                     hipMemcpyDeviceToHost, s),
                                      "d2h"));
        DPF_RETURN_IF_ERROR(HipStatus(hipEventRecord(ev_[i & 1], s), "hipEventRecord"));
      }
      if (i >= 1) {
        const size_t j = i - 1;
        DPF_RETURN_IF_ERROR(HipStatus(hipEventSynchronize(ev_[j & 1]), "d2h"));
        HostPool::Get().Copy(dst + j * kChunk, static_cast<const char*>(pin_[j & 1]), len(j));
      }
    }
    return OkStatus();
  }

 private:
  void* pin_[2] = {nullptr, nullptr};
  hipEvent_t ev_[2] = {nullptr, nullptr};
  int dev_[2] = {-1, -1};
};

// Host-to-device copy of pageable `src` through two pinned chunks per
// thread: the host memcpy of chunk i + 1 (split over HostPool) overlaps the
// DMA of chunk i.  Returns once `src` has been read; the DMAs stay ordered on
// `s` (a chunk buffer is refilled only after the event behind its last DMA).
class H2DStaging {
 public:
  static constexpr size_t kChunk = 4u << 20;
  H2DStaging() = default;
  H2DStaging(const H2DStaging&) = delete;
  H2DStaging& operator=(const H2DStaging&) = delete;
  ~H2DStaging() {
    for (int i = 0; i < 2; ++i) {
      if (ev_[i]) {
        (void)hipEventSynchronize(ev_[i]);
        (void)hipEventDestroy(ev_[i]);
      }
      if (pin_[i]) (void)hipHostFree(pin_[i]);
    }
  }
  Status Copy(char* dst, const char* src, size_t bytes, hipStream_t s) {
    int dev = 0;
    DPF_RETURN_IF_ERROR(HipStatus(hipGetDevice(&dev), "hipGetDevice"));
    for (int i = 0; i < 2; ++i) {
      if (!pin_[i])
        DPF_RETURN_IF_ERROR(HipStatus(hipHostMalloc(&pin_[i], kChunk, 0), "hipHostMalloc"));
      if (ev_[i] && dev_[i] != dev) {  // events are recorded on streams of their device
        DPF_RETURN_IF_ERROR(HipStatus(hipEventSynchronize(ev_[i]), "h2d"));
        (void)hipEventDestroy(ev_[i]);
        ev_[i] = nullptr;
      }
      if (!ev_[i]) {
        DPF_RETURN_IF_ERROR(
            HipStatus(hipEventCreateWithFlags(&ev_[i], hipEventDisableTiming), "hipEventCreate"));
        dev_[i] = dev;
        used_[i] = false;
      }
    }
    for (size_t off = 0; off < bytes; off += kChunk) {
      const size_t n = std::min(kChunk, bytes - off);
      const int b = next_;
      next_ ^= 1;
      if (used_[b]) DPF_RETURN_IF_ERROR(HipStatus(hipEventSynchronize(ev_[b]), "h2d"));
      HostPool::Get().Copy(static_cast<char*>(pin_[b]), src + off, n);
      DPF_RETURN_IF_ERROR(
          HipStatus(hipMemcpyAsync(dst + off, pin_[b], n, hipMemcpyHostToDevice, s), "h2d"));
      DPF_RETURN_IF_ERROR(HipStatus(hipEventRecord(ev_[b], s), "hipEventRecord"));
      used_[b] = true;
    }
    return OkStatus();
  }

 private:
  void* pin_[2] = {nullptr, nullptr};
  hipEvent_t ev_[2] = {nullptr, nullptr};
  int dev_[2] = {-1, -1};
  bool used_[2] = {false, false};
  int next_ = 0;
};

inline H2DStaging& ThreadH2DStaging() { return ThreadRecycled<H2DStaging>::Get(); }

inline Status CopyToHostSync(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes <= D2HDirectMax()) {
    DPF_RETURN_IF_ERROR(CopyToHost(dst, src, bytes, s));
    return HipStatus(hipStreamSynchronize(s), "sync");
  }
  return ThreadRecycled<D2HStaging>::Get().Copy(static_cast<char*>(dst), static_cast<const char*>(src), bytes, s);
}

// Host layouts with holes (e.g. {uint32_t, uint64_t}: 16 bytes, 4 unused):
// the kernels write only the scalars, so a buffer whose rows reach the caller
// is cleared first and stale device memory never shows up in the padding.
inline bool HasPadding(const dpf_amd_value_type& vt) {
  int used = 0;
  for (int i = 0; i < vt.num_scalars; ++i) used += vt.scalars[i].bytes;
  return used < vt.out_stride;
}

inline Status ClearPadding(const dpf_amd_value_type& vt, void* p, size_t bytes, hipStream_t s) {
  if (bytes == 0 || !HasPadding(vt)) return OkStatus();
  return HipStatus(hipMemsetAsync(p, 0, bytes, s), "hipMemsetAsync");
}

// Pinned staging for host-to-device uploads: the Tier-2 paths upload locals
// that go out of scope before the stream drains, so every upload is first
// copied into a pinned slot (then a true async DMA); a slot is reused only
// after the event recorded behind its copy.  Uploads above kMaxSlotBytes
// (EvaluateAndApply's 2^20 points, DCF BatchEvaluate's per-key correction
// words) do not grow a slot: they go through the thread's two pinned
// H2DStaging chunks, so no thread keeps more than 16 + 8 MiB of pinned
// memory for the life of the process.
class UploadRing {
 public:
  UploadRing() = default;
  UploadRing(const UploadRing&) = delete;
  UploadRing& operator=(const UploadRing&) = delete;
  ~UploadRing() {
    for (Slot& sl : slots_) {
      if (sl.done) {
        (void)hipEventSynchronize(sl.done);
        (void)hipEventDestroy(sl.done);
      }
      if (sl.host) (void)hipHostFree(sl.host);
    }
    for (PlaceSlot& pl : places_) {
      if (pl.done) {
        (void)hipEventSynchronize(pl.done);
        (void)hipEventDestroy(pl.done);
      }
      if (pl.dev) (void)hipFree(pl.dev);
    }
  }
  Status Copy(void* dst, const void* src, size_t bytes, hipStream_t s) {
    const HostPart part{src, bytes};
    return CopyPacked(dst, &part, 1, bytes, nullptr, s);
  }
  // Several host arrays in one slot and one DMA: part i lands at dst +
  // off[i] (16-byte aligned; PackedLayout computes the offsets and total).
  struct HostPart {
    const void* p;
    size_t bytes;
  };
  static size_t PackedLayout(const HostPart* parts, int k, size_t* off) {
    size_t at = 0;
    for (int i = 0; i < k; ++i) {
      if (off) off[i] = at;
      at += (parts[i].bytes + 15) & ~size_t{15};
    }
    return at;
  }
  Status CopyPacked(void* dst, const HostPart* parts, int k, size_t bytes, const size_t* off,
                    hipStream_t s) {
    if (bytes == 0) return OkStatus();
    if (bytes > kMaxSlotBytes) {
      for (int i = 0; i < k; ++i)
        if (parts[i].bytes)
          DPF_RETURN_IF_ERROR(ThreadH2DStaging().Copy(static_cast<char*>(dst) + (off ? off[i] : 0),
                                                      static_cast<const char*>(parts[i].p),
                                                      parts[i].bytes, s));
      return OkStatus();
    }
    Slot& sl = slots_[next_];
    next_ = (next_ + 1) % kSlots;
    int dev = 0;
    DPF_RETURN_IF_ERROR(HipStatus(hipGetDevice(&dev), "hipGetDevice"));
    if (sl.done != nullptr && sl.device != dev) {
      // the slot's event belongs to the device its last copy ran on; events
      // are recorded on streams of their own device (s is on the current one)
      DPF_RETURN_IF_ERROR(HipStatus(hipEventSynchronize(sl.done), "upload slot"));
      (void)hipEventDestroy(sl.done);
      sl.done = nullptr;
    }
    sl.device = dev;
    if (sl.done == nullptr)
      DPF_RETURN_IF_ERROR(HipStatus(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming),
                                    "hipEventCreate"));
    else
      DPF_RETURN_IF_ERROR(HipStatus(hipEventSynchronize(sl.done), "upload slot"));
    DPF_RETURN_IF_ERROR(EnsureCapacity(sl, bytes));
    for (int i = 0; i < k; ++i)
      if (parts[i].bytes)
        std::memcpy(static_cast<char*>(sl.host) + (off ? off[i] : 0), parts[i].p, parts[i].bytes);
    if (Mode() == kSdma || Mode() == kSdmaSync) {
      DPF_RETURN_IF_ERROR(
          HipStatus(hipMemcpyAsync(dst, sl.host, bytes, hipMemcpyHostToDevice, s), "upload"));
      if (Mode() == kSdmaSync) DPF_RETURN_IF_ERROR(HipStatus(hipStreamSynchronize(s), "sync"));
    } else {
      DPF_RETURN_IF_ERROR(AbiStatus(dpf_amd::CopyFromMappedHost(dst, sl.dev, bytes, s)));
    }
    return HipStatus(hipEventRecord(sl.done, s), "hipEventRecord");
  }

  // Zero-copy staging: the parts are packed into a slot mapped as
  // fine-grained (uncached) memory and a kernel reads them in place through
  // *dev; Release(slot, s) must follow the last launch that reads them (it
  // records the slot's reuse event behind it).  Returns false in *staged
  // (nothing done) when the upload mode does not map slots coherently or the
  // parts do not fit a slot; the caller then uploads with CopyPacked.
  Status Stage(const HostPart* parts, int k, size_t bytes, const size_t* off, bool* staged,
               int* slot, const char** dev) {
    *staged = false;
    static const bool disabled = [] {  // DPF_AMD_ZERO_COPY=0: always copy (A/B)
      const char* e = std::getenv("DPF_AMD_ZERO_COPY");
      return e != nullptr && std::strcmp(e, "0") == 0;
    }();
    if (disabled || bytes == 0 || bytes > kMaxSlotBytes || Mode() != kKernelCoherent) return OkStatus();
    const int i = next_;
    Slot& sl = slots_[i];
    next_ = (next_ + 1) % kSlots;
    int d = 0;
    DPF_RETURN_IF_ERROR(HipStatus(hipGetDevice(&d), "hipGetDevice"));
    if (sl.done != nullptr) {
      DPF_RETURN_IF_ERROR(HipStatus(hipEventSynchronize(sl.done), "upload slot"));
      if (sl.device != d) {
        (void)hipEventDestroy(sl.done);
        sl.done = nullptr;
      }
    }
    sl.device = d;
    if (sl.done == nullptr)
      DPF_RETURN_IF_ERROR(HipStatus(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming),
                                    "hipEventCreate"));
    DPF_RETURN_IF_ERROR(EnsureCapacity(sl, bytes));
    for (int j = 0; j < k; ++j)
      if (parts[j].bytes)
        std::memcpy(static_cast<char*>(sl.host) + (off ? off[j] : 0), parts[j].p, parts[j].bytes);
    *staged = true;
    *slot = i;
    *dev = static_cast<const char*>(sl.dev);
    return OkStatus();
  }
  Status Release(int slot, hipStream_t s) {
    return HipStatus(hipEventRecord(slots_[slot].done, s), "hipEventRecord");
  }

  // Small parts written by the host straight into fine-grained device memory
  // (a large-BAR device maps its VRAM into the process), so the kernel that
  // reads them needs no copy kernel in front of it — 2.3 us plus a 6 us
  // dependent-dispatch gap per call on the per-call EvaluateAt path
  // (tools/experiments/host_write_probe.hip: 2.3 KiB written and checked by a
  // kernel in 12.9 us per round against 19.3 us with a copy kernel and 12.3
  // us for the check kernel alone).  Fine-grained memory is kept coherent, so
  // a kernel never reads a stale line of a reused slot.  ReleasePlaced(slot,
  // s) must follow the last launch that reads the slot.  *placed = false
  // (nothing done) when the device is not large-BAR, the one-time check of
  // the path failed, DPF_AMD_HOST_WRITE=0, or the parts exceed a slot.
  // `max_bytes`: the largest upload placed (default: small key parts; c3's
  // prefix lists pass kMaxPlaceLargeBytes).
  Status Place(const HostPart* parts, int k, size_t bytes, const size_t* off, bool* placed,
               int* slot, char** dev, size_t max_bytes = kMaxPlaceBytes) {
    *placed = false;
    if (bytes == 0 || bytes > max_bytes) return OkStatus();
    int d = 0;
    DPF_RETURN_IF_ERROR(HipStatus(hipGetDevice(&d), "hipGetDevice"));
    if (!HostWritable(d)) return OkStatus();
    const int i = place_next_;
    PlaceSlot& pl = places_[i];
    place_next_ = (place_next_ + 1) % kSlots;
    if (pl.done != nullptr) DPF_RETURN_IF_ERROR(HipStatus(hipEventSynchronize(pl.done), "place slot"));
    if (pl.device != d || pl.cap < bytes) {
      if (pl.dev) (void)hipFree(pl.dev);  // idle: its event has completed
      pl.dev = nullptr;
      pl.cap = 0;
      if (pl.done) (void)hipEventDestroy(pl.done);
      pl.done = nullptr;
      size_t cap = 4096;
      while (cap < bytes) cap <<= 1;
      DPF_RETURN_IF_ERROR(HipStatus(hipExtMallocWithFlags(&pl.dev, cap, hipDeviceMallocFinegrained),
                                    "hipExtMallocWithFlags"));
      pl.cap = cap;
      pl.device = d;
    }
    if (pl.done == nullptr)
      DPF_RETURN_IF_ERROR(HipStatus(hipEventCreateWithFlags(&pl.done, hipEventDisableTiming),
                                    "hipEventCreate"));
    char* base = static_cast<char*>(pl.dev);
    for (int j = 0; j < k; ++j)
      if (parts[j].bytes) std::memcpy(base + (off ? off[j] : 0), parts[j].p, parts[j].bytes);
    std::atomic_thread_fence(std::memory_order_seq_cst);  // writes before the launch's doorbell
    *placed = true;
    *slot = i;
    *dev = base;
    return OkStatus();
  }
  Status ReleasePlaced(int slot, hipStream_t s) {
    return HipStatus(hipEventRecord(places_[slot].done, s), "hipEventRecord");
  }

 private:
  // DPF_AMD_UPLOAD = kernel_coherent (default: a copy kernel on the
  // caller's stream reading the slot, mapped as fine-grained uncached memory)
  // | kernel (the slot mapped non-coherent) | sdma (hipMemcpyAsync from the
  // slot) | sdma_sync.  The copy kernel needs no copy-engine hand-off before
  // the consumer kernel: 64 C++ EvaluateAt calls 7.74-7.88 ms against
  // 7.84-8.38 with sdma on one box, 7.72-7.86 against 8.29-8.35 on another
  // (profiles/ab_upload_r05n.log; the other C++ configs and the c4/8 request
  // within noise).
  enum UploadMode { kKernel, kKernelCoherent, kSdma, kSdmaSync };
  static UploadMode Mode() {
    static const UploadMode m = [] {
      const char* e = std::getenv("DPF_AMD_UPLOAD");
      if (!e) return kKernelCoherent;
      if (!std::strcmp(e, "kernel")) return kKernel;
      if (!std::strcmp(e, "sdma")) return kSdma;
      if (!std::strcmp(e, "sdma_sync")) return kSdmaSync;
      return kKernelCoherent;
    }();
    return m;
  }
  static constexpr int kSlots = 16;
  static constexpr size_t kMaxSlotBytes = size_t{1} << 20;
  struct Slot {
    void* host = nullptr;
    void* dev = nullptr;  // device address of `host`
    size_t cap = 0;
    hipEvent_t done = nullptr;
    int device = -1;  // device of `done`
  };
  Slot slots_[kSlots];
  int next_ = 0;
  static constexpr size_t kMaxPlaceBytes = size_t{64} << 10;

 public:
  static constexpr size_t kMaxPlaceLargeBytes = size_t{1} << 20;  // c3's 2^16 prefixes

 private:
  struct PlaceSlot {
    void* dev = nullptr;  // fine-grained device memory, written by the host
    size_t cap = 0;
    hipEvent_t done = nullptr;
    int device = -1;
  };
  PlaceSlot places_[kSlots];
  int place_next_ = 0;

  // Whether the host can write `device`'s fine-grained memory directly:
  // large BAR, and the case Place() relies on — a kernel reading a slot,
  // the host rewriting it, a kernel reading it again — returns the new bytes
  // both times (the copy kernel reads the slot into ordinary VRAM, checked
  // through hipMemcpy; once per device; DPF_AMD_HOST_WRITE=0 turns it off).
  // Called with `device` current.
  static bool HostWritable(int device) {
    static std::mutex mu;
    static int state[64];  // 0 unknown, 1 yes, 2 no
    if (device < 0 || device >= 64) return false;
    std::lock_guard<std::mutex> l(mu);
    if (state[device] == 0) {
      state[device] = 2;
      const char* e = std::getenv("DPF_AMD_HOST_WRITE");
      int large = 0;
      void* p = nullptr;
      void* q = nullptr;
      if (!(e && std::strcmp(e, "0") == 0) &&
          hipDeviceGetAttribute(&large, hipDeviceAttributeIsLargeBar, device) == hipSuccess &&
          large && hipExtMallocWithFlags(&p, 4096, hipDeviceMallocFinegrained) == hipSuccess &&
          hipMalloc(&q, 4096) == hipSuccess) {
        uint32_t w[1024], r[1024];
        bool ok = true;
        for (int round = 0; round < 2 && ok; ++round) {
          for (int i = 0; i < 1024; ++i) w[i] = 0x9e3779b9u * (uint32_t)(i + 1) + (uint32_t)round;
          std::memcpy(p, w, sizeof(w));
          std::atomic_thread_fence(std::memory_order_seq_cst);
          ok = dpf_amd::CopyFromMappedHost(q, p, sizeof(w), nullptr) == DPF_AMD_OK &&
               hipMemcpy(r, q, sizeof(r), hipMemcpyDeviceToHost) == hipSuccess &&
               std::memcmp(w, r, sizeof(w)) == 0;
        }
        if (ok) state[device] = 1;
      }
      if (p) (void)hipFree(p);
      if (q) (void)hipFree(q);
      (void)hipGetLastError();  // a refused attribute / allocation is not a launch error
    }
    return state[device] == 1;
  }

  static Status EnsureCapacity(Slot& sl, size_t bytes) {
    if (sl.cap >= bytes) return OkStatus();
    if (sl.host) (void)hipHostFree(sl.host);
    sl.host = nullptr;
    sl.cap = 0;
    size_t cap = 4096;
    while (cap < bytes) cap <<= 1;
    const unsigned flags = Mode() == kKernelCoherent
                               ? (hipHostMallocMapped | hipHostMallocCoherent)
                               : hipHostMallocMapped;
    DPF_RETURN_IF_ERROR(HipStatus(hipHostMalloc(&sl.host, cap, flags), "hipHostMalloc"));
    DPF_RETURN_IF_ERROR(
        HipStatus(hipHostGetDevicePointer(&sl.dev, sl.host, 0), "hipHostGetDevicePointer"));
    sl.cap = cap;
    return OkStatus();
  }
};

inline UploadRing& ThreadUploadRing() { return ThreadRecycled<UploadRing>::Get(); }

// Caching device allocator with stream-ordered reuse, on top of hipMalloc.
// The library does not use hipMallocAsync: under ROCm 7.2's runtime
// (70226015) a device-to-host hipMemcpyAsync out of pool memory that was
// freed with hipFreeAsync and handed out again returns wrong bytes, while
// kernels on the same stream see the right contents.  tools/
// malloc_async_repro.cc reproduces it without the library — one stream, the
// allocation pattern of a c3 level: from the first reused 128 MiB block on,
// 100 % of the copied elements are wrong on the host and 0 on the device
// (profiles/malloc_async_repro_r03.log); hipMalloc: 0 wrong.  The library
// with DPF_AMD_MALLOC_ASYNC=1 fails c3 the same way (level 2 share sum,
// gather-offset check).
// A freed block keeps an event recorded on the freeing stream; it is handed
// out again at once on that stream (stream order covers the reuse) and on
// any other stream once the event has completed.  Sizes are rounded to
// powers of two up to 1 MiB and to 2 MiB multiples above; a request may take
// an idle block up to 25 % larger than its bucket.  Idle blocks are bounded:
// above DPF_AMD_POOL_CACHE_MB (default 4096) of idle memory the least
// recently freed blocks go back to the device, and an allocation that fails
// (here or in a caller, through dpf_amd_release_cached_memory) releases all
// idle blocks and retries.
class DevicePool {
 public:
  static DevicePool& Get() {
    static DevicePool* pool = new DevicePool();  // never destroyed: no HIP calls at exit
    return *pool;
  }

  Status Alloc(size_t bytes, hipStream_t s, void** out) {
    const size_t size = Bucket(bytes);
    int dev = 0;
    DPF_RETURN_IF_ERROR(HipStatus(hipGetDevice(&dev), "hipGetDevice"));
    {
      std::lock_guard<std::mutex> l(mu_);
      const size_t limit = size + size / 4;
      for (auto it = free_.lower_bound(std::make_pair(dev, size));
           it != free_.end() && it->first.first == dev && it->first.second <= limit; ++it) {
        Block& b = it->second;
        if (b.stream != s && hipEventQuery(b.ready) != hipSuccess) {
          // not-ready is the expected answer; clear it so the next launch
          // check (hipGetLastError) does not report it as its own failure
          (void)hipGetLastError();
          continue;
        }
        *out = b.p;
        events_[dev].push_back(b.ready);
        live_[b.p] = std::make_pair(b.size, dev);
        cached_ -= b.size;
        free_.erase(it);
        return OkStatus();
      }
    }
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, size);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      Release();
      e = hipMalloc(&p, size);
    }
    DPF_RETURN_IF_ERROR(HipStatus(e, "hipMalloc"));
    std::lock_guard<std::mutex> l(mu_);
    live_[p] = std::make_pair(size, dev);
    *out = p;
    return OkStatus();
  }

  void Free(void* p, hipStream_t s) {
    if (p == nullptr) return;
    std::vector<Evicted> evict;
    {
      std::lock_guard<std::mutex> l(mu_);
      FreeLocked(p, s, &evict);
    }
    Drop(evict);  // GPU syncs and hipFree without the pool lock
  }

  // Returns every idle cached block to the device.
  void Release() {
    std::vector<Evicted> evict;
    {
      std::lock_guard<std::mutex> l(mu_);
      TakeLocked(0, &evict);
    }
    Drop(evict);
  }

  size_t cached_bytes() {
    std::lock_guard<std::mutex> l(mu_);
    return cached_;
  }

 private:
  struct Block {
    void* p;
    size_t size;
    hipStream_t stream;
    hipEvent_t ready;
    uint64_t seq;  // free order (least recently freed is trimmed first)
  };
  struct Evicted {
    int device;
    Block b;
  };
  void FreeLocked(void* p, hipStream_t s, std::vector<Evicted>* evict) {
    auto it = live_.find(p);
    if (it == live_.end()) return;
    Block b{p, it->second.first, s, nullptr, ++seq_};
    const int dev = it->second.second;
    live_.erase(it);
    DeviceGuard g(dev);  // events belong to the block's (and its stream's) device
    std::vector<hipEvent_t>& evs = events_[dev];
    if (!evs.empty()) {
      b.ready = evs.back();
      evs.pop_back();
    } else if (hipEventCreateWithFlags(&b.ready, hipEventDisableTiming) != hipSuccess) {
      b.ready = nullptr;
    }
    if (b.ready == nullptr || hipEventRecord(b.ready, s) != hipSuccess) {
      // no event: drain the stream so the block is idle
      (void)hipGetLastError();
      (void)hipStreamSynchronize(s);
      if (b.ready == nullptr) (void)hipEventCreateWithFlags(&b.ready, hipEventDisableTiming);
    }
    free_.emplace(std::make_pair(dev, b.size), b);
    cached_ += b.size;
    if (cached_ > CacheLimit()) TakeLocked(CacheLimit(), evict);
  }
  static size_t CacheLimit() {
    static const size_t lim = [] {
      const char* e = std::getenv("DPF_AMD_POOL_CACHE_MB");
      return (e ? std::strtoull(e, nullptr, 10) : 4096ull) << 20;
    }();
    return lim;
  }
  // Takes idle blocks out of the cache, least recently freed first, until at
  // most `keep` bytes stay cached (caller holds mu_); Drop frees them.
  void TakeLocked(size_t keep, std::vector<Evicted>* out) {
    if (cached_ <= keep) return;
    std::vector<std::multimap<std::pair<int, size_t>, Block>::iterator> order;
    order.reserve(free_.size());
    for (auto it = free_.begin(); it != free_.end(); ++it) order.push_back(it);
    std::sort(order.begin(), order.end(),
              [](const auto& x, const auto& y) { return x->second.seq < y->second.seq; });
    for (auto it : order) {
      if (cached_ <= keep) break;
      out->push_back(Evicted{it->first.first, it->second});
      cached_ -= it->second.size;
      free_.erase(it);
    }
  }
  // Waits for each evicted block's last use and frees it (no lock held),
  // then returns the events to the per-device free lists.
  void Drop(const std::vector<Evicted>& evict) {
    if (evict.empty()) return;
    for (const Evicted& e : evict) {
      DeviceGuard g(e.device);
      if (e.b.ready) (void)hipEventSynchronize(e.b.ready);
      (void)hipFree(e.b.p);
    }
    std::lock_guard<std::mutex> l(mu_);
    for (const Evicted& e : evict)
      if (e.b.ready) events_[e.device].push_back(e.b.ready);
  }
  static size_t Bucket(size_t n) {
    if (n <= (size_t{1} << 20)) {
      size_t b = 512;
      while (b < n) b <<= 1;
      return b;
    }
    const size_t g = size_t{2} << 20;
    return (n + g - 1) / g * g;
  }
  std::mutex mu_;
  std::unordered_map<void*, std::pair<size_t, int>> live_;  // block -> (size, device)
  std::multimap<std::pair<int, size_t>, Block> free_;        // (device, size) -> idle block
  std::map<int, std::vector<hipEvent_t>> events_;            // recycled, per device
  size_t cached_ = 0;
  uint64_t seq_ = 0;
};

// DPF_AMD_DEBUG_ALLOC=1: every live DeviceBuffer range is registered and a
// new allocation overlapping a live one is reported on stderr (diagnostics
// for the stream-ordered pool).
struct LiveRanges {
  std::mutex mu;
  std::map<uintptr_t, size_t> live;
  static LiveRanges& Get() {
    static LiveRanges r;
    return r;
  }
  static bool On() {
    static const bool on = std::getenv("DPF_AMD_DEBUG_ALLOC") != nullptr;
    return on;
  }
  void Add(void* p, size_t n) {
    std::lock_guard<std::mutex> l(mu);
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    auto it = live.upper_bound(a);
    if (it != live.end() && it->first < a + n)
      std::fprintf(stderr, "[dpf_amd] alloc %p+%zu overlaps live %p+%zu\n", p, n,
                   reinterpret_cast<void*>(it->first), it->second);
    if (it != live.begin()) {
      --it;
      if (it->first + it->second > a)
        std::fprintf(stderr, "[dpf_amd] alloc %p+%zu overlaps live %p+%zu\n", p, n,
                     reinterpret_cast<void*>(it->first), it->second);
    }
    live[a] = n;
  }
  void Remove(void* p) {
    std::lock_guard<std::mutex> l(mu);
    live.erase(reinterpret_cast<uintptr_t>(p));
  }
};

class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  ~DeviceBuffer() { Reset(); }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  Status Alloc(size_t bytes, hipStream_t s) {
    Reset();
    stream_ = s;
    if (bytes == 0) bytes = 16;
    Status st = MallocAsync() ? HipStatus(hipMallocAsync(&p_, bytes, s), "hipMallocAsync")
                : NoPool()    ? HipStatus(hipMalloc(&p_, bytes), "hipMalloc")
                              : DevicePool::Get().Alloc(bytes, s, &p_);
    if (st.ok() && LiveRanges::On()) LiveRanges::Get().Add(p_, bytes);
    return st;
  }
  Status Upload(const void* src, size_t bytes, hipStream_t s) {
    DPF_RETURN_IF_ERROR(Alloc(bytes, s));
    if (bytes == 0) return OkStatus();
    return ThreadUploadRing().Copy(p_, src, bytes, s);
  }
  void Reset() {
    if (p_) {
      if (LiveRanges::On()) LiveRanges::Get().Remove(p_);
      if (MallocAsync()) {
        (void)hipFreeAsync(p_, stream_);
      } else if (NoPool()) {
        (void)hipStreamSynchronize(stream_);
        (void)hipFree(p_);
      } else {
        DevicePool::Get().Free(p_, stream_);
      }
    }
    p_ = nullptr;
  }
  void* get() const { return p_; }
  // DPF_AMD_NO_POOL=1 (diagnostics): synchronous hipMalloc / hipFree instead
  // of the caching pool.
  static bool NoPool() {
    static const bool on = std::getenv("DPF_AMD_NO_POOL") != nullptr;
    return on;
  }
  // DPF_AMD_MALLOC_ASYNC=1 (diagnostics): the runtime's stream-ordered
  // allocator (hipMallocAsync / hipFreeAsync on the buffer's stream), the
  // allocator the DevicePool replaced (tools/malloc_async_repro.cc).
  static bool MallocAsync() {
    static const bool on = std::getenv("DPF_AMD_MALLOC_ASYNC") != nullptr;
    return on;
  }
  template <typename T>
  T* as() const {
    return static_cast<T*>(p_);
  }

 private:
  void* p_ = nullptr;
  hipStream_t stream_ = nullptr;
};

}  // namespace dpf_internal_host
}  // namespace distributed_point_functions
