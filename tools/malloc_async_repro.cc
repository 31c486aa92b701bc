// malloc_async_repro.cc — standalone check of hipMallocAsync / hipFreeAsync
// under the allocation pattern of one c3 EvaluateNext level (csrc/dpf.cc
// EvaluateUntilRaw), without the library: per level, on one non-blocking
// stream, stream-ordered allocations of the walk inputs, a 128 MiB expansion
// staging buffer, the gather offsets and a 128 MiB result; an "expand" kernel
// writes a deterministic value per element, a gather kernel copies each
// prefix's 256-element segment through the uploaded offsets (flagging an
// offset out of range, as KGatherRows does), the result comes back through a
// pinned buffer and is compared element by element; everything is freed
// stream-ordered before the next level.  Run with `async` (hipMallocAsync),
// `malloc` (hipMalloc / hipFree) or `async2` (allocations on a second stream
// that waits on the first through an event — the cross-stream reuse case).
//
// Built by hand on the GPU box:
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/malloc_async_repro tools/malloc_async_repro.cc
//   /tmp/malloc_async_repro async 4
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                   \
    }                                                                                 \
  } while (0)

__host__ __device__ inline uint64_t Mix(uint64_t level, uint64_t i) {
  uint64_t z = (level << 40) ^ i ^ 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__global__ void KExpandLike(uint64_t* out, int64_t n, uint64_t level, const uint64_t* roots,
                            int64_t num_roots) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
    // reads the uploaded roots like the expansion reads its root seeds
    const uint64_t r = roots[(i >> 8) % num_roots];
    out[i] = Mix(level, i) ^ (r - r);
  }
}

__global__ void KGather(const int64_t* src, int64_t n, int64_t opp, const uint64_t* in,
                        int64_t in_rows, uint64_t* out, int* err) {
  const int64_t total = n * opp;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < total; w += step) {
    const int64_t p = w / opp, k = w - p * opp;
    const int64_t r = src[p];
    if (r < 0 || r > in_rows - opp) {
      *err = 1;
      continue;
    }
    out[w] = in[r + k];
  }
}

// Device-side check of the gathered result (tells a kernel-visible error
// from one only the copy engine sees).
__global__ void KVerify(const uint64_t* out, const int64_t* src, int64_t n, int64_t opp,
                        uint64_t level, unsigned long long* bad) {
  const int64_t total = n * opp;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  unsigned long long mine = 0;
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < total; w += step) {
    const int64_t p = w / opp, k = w - p * opp;
    if (out[w] != Mix(level, src[p] + k)) ++mine;
  }
  if (mine) atomicAdd(bad, mine);
}

struct Alloc {
  enum Mode { kAsync, kMalloc, kAsync2 } mode;
  hipStream_t s, s2;
  hipEvent_t ev;
  void* Get(size_t bytes) {
    void* p = nullptr;
    if (mode == kMalloc) {
      CHECK(hipMalloc(&p, bytes));
    } else if (mode == kAsync) {
      CHECK(hipMallocAsync(&p, bytes, s));
    } else {  // allocate on s2, then make s wait for s2
      CHECK(hipMallocAsync(&p, bytes, s2));
      CHECK(hipEventRecord(ev, s2));
      CHECK(hipStreamWaitEvent(s, ev, 0));
    }
    return p;
  }
  void Put(void* p) {
    if (mode == kMalloc) {
      CHECK(hipStreamSynchronize(s));
      CHECK(hipFree(p));
    } else {
      CHECK(hipFreeAsync(p, s));
    }
  }
};

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "async";
  const int reps = argc > 2 ? std::atoi(argv[2]) : 4;
  int rt = 0, drv = 0;
  CHECK(hipRuntimeGetVersion(&rt));
  CHECK(hipDriverGetVersion(&drv));
  Alloc a;
  a.mode = mode == "malloc" ? Alloc::kMalloc : mode == "async2" ? Alloc::kAsync2 : Alloc::kAsync;
  CHECK(hipStreamCreateWithFlags(&a.s, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&a.s2, hipStreamNonBlocking));
  CHECK(hipEventCreateWithFlags(&a.ev, hipEventDisableTiming));
  std::printf("runtime %d driver %d mode %s reps %d\n", rt, drv, mode.c_str(), reps);

  const int64_t opp = 256;  // outputs per prefix (8-bit hierarchy step)
  const int64_t max_prefixes = 1 << 16;
  const int64_t max_elems = max_prefixes * opp;  // 2^24 uint64 = 128 MiB
  uint64_t* pin_out = nullptr;
  int64_t* pin_src = nullptr;
  uint64_t* pin_roots = nullptr;
  int* pin_err = nullptr;
  CHECK(hipHostMalloc((void**)&pin_out, max_elems * 8, 0));
  CHECK(hipHostMalloc((void**)&pin_src, max_prefixes * 8, 0));
  CHECK(hipHostMalloc((void**)&pin_roots, max_prefixes * 16, 0));
  CHECK(hipHostMalloc((void**)&pin_err, sizeof(int), 0));
  std::mt19937_64 rng(1);
  int64_t bad_total = 0, err_total = 0;
  for (int rep = 0; rep < reps; ++rep) {
    for (int level = 0; level < 16; ++level) {
      // level 0: one root; level 1: 256 prefixes; then 2^16 prefixes whose
      // tree indices are unique (expanded = prefixes * opp)
      const int64_t n = level == 0 ? 1 : level == 1 ? 256 : max_prefixes;
      const int64_t rows = n * opp;
      // walk inputs (seeds + control bits + paths + cws packed)
      const size_t in_bytes = size_t(n) * 33 + 16 * 8 + 64;
      char* inputs = (char*)a.Get(in_bytes);
      for (int64_t i = 0; i < 2 * n; ++i) pin_roots[i] = rng();
      CHECK(hipMemcpyAsync(inputs, pin_roots, 16 * n, hipMemcpyHostToDevice, a.s));
      uint64_t* staging = (uint64_t*)a.Get(rows * 8);
      hipLaunchKernelGGL(KExpandLike, dim3(2048), dim3(256), 0, a.s, staging, rows,
                         (uint64_t)level, (const uint64_t*)inputs, 2 * n);
      CHECK(hipGetLastError());
      // prefixes in shuffled order: segment p of the result is tree index
      // perm[p] of the staging buffer
      std::vector<int64_t> perm(n);
      for (int64_t i = 0; i < n; ++i) perm[i] = i;
      std::shuffle(perm.begin(), perm.end(), rng);
      for (int64_t i = 0; i < n; ++i) pin_src[i] = perm[i] * opp;
      int64_t* src = (int64_t*)a.Get(8 * n);
      CHECK(hipMemcpyAsync(src, pin_src, 8 * n, hipMemcpyHostToDevice, a.s));
      uint64_t* result = (uint64_t*)a.Get(rows * 8);
      int* err = (int*)a.Get(sizeof(int));
      CHECK(hipMemsetAsync(err, 0, sizeof(int), a.s));
      hipLaunchKernelGGL(KGather, dim3(2048), dim3(256), 0, a.s, (const int64_t*)src, n, opp,
                         (const uint64_t*)staging, rows, result, err);
      CHECK(hipGetLastError());
      unsigned long long* dbad = (unsigned long long*)a.Get(sizeof(unsigned long long));
      CHECK(hipMemsetAsync(dbad, 0, sizeof(unsigned long long), a.s));
      hipLaunchKernelGGL(KVerify, dim3(2048), dim3(256), 0, a.s, (const uint64_t*)result,
                         (const int64_t*)src, n, opp, (uint64_t)level, dbad);
      CHECK(hipGetLastError());
      unsigned long long dev_bad = 0;
      CHECK(hipMemcpyAsync(pin_out, result, rows * 8, hipMemcpyDeviceToHost, a.s));
      CHECK(hipMemcpyAsync(pin_roots, dbad, 8, hipMemcpyDeviceToHost, a.s));
      CHECK(hipMemcpyAsync(pin_err, err, sizeof(int), hipMemcpyDeviceToHost, a.s));
      CHECK(hipStreamSynchronize(a.s));
      dev_bad = pin_roots[0];
      int64_t bad = 0;
      for (int64_t p = 0; p < n; ++p)
        for (int64_t k = 0; k < opp; ++k)
          if (pin_out[p * opp + k] != Mix(level, perm[p] * opp + k)) ++bad;
      auto overlap = [](const void* x, size_t nx, const void* y, size_t ny) {
        const char *a0 = (const char*)x, *b0 = (const char*)y;
        return a0 < b0 + ny && b0 < a0 + nx;
      };
      const bool alias = overlap(staging, rows * 8, result, rows * 8) ||
                         overlap(inputs, in_bytes, staging, rows * 8) ||
                         overlap(inputs, in_bytes, result, rows * 8) ||
                         overlap(src, 8 * n, staging, rows * 8) ||
                         overlap(src, 8 * n, result, rows * 8);
      if (bad || *pin_err || dev_bad || alias)
        std::printf("rep %d level %d: %lld of %lld elements wrong on the host, %llu on the "
                    "device, gather flag %d; staging %p result %p inputs %p src %p%s\n",
                    rep, level, (long long)bad, (long long)rows, dev_bad, *pin_err,
                    (void*)staging, (void*)result, (void*)inputs, (void*)src,
                    alias ? " OVERLAP" : "");
      bad_total += bad;
      err_total += *pin_err;
      a.Put(dbad);
      a.Put(err);
      a.Put(result);
      a.Put(src);
      a.Put(staging);
      a.Put(inputs);
    }
    std::printf("rep %d done\n", rep);
    std::fflush(stdout);
  }
  CHECK(hipStreamSynchronize(a.s));
  std::printf("RESULT mode %s: %lld wrong elements, %lld gather flags over %d reps x 16 levels\n",
              mode.c_str(), (long long)bad_total, (long long)err_total, reps);
  return bad_total || err_total ? 1 : 0;
}
