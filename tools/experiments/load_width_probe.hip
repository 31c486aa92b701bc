// Streaming-read probe (round 5): does the load width hold the Four-Russians
// scan (KPirScanM4, one buffer_load_dword per lane per record) below the
// masked scan's 16-byte loads?  Reads 16 GiB (c4: 2^26 x 256 B) once, XOR-
// reducing into a per-wave value, with (a) 4-byte loads, lane j = dword j of
// a 256-byte record, 4 records per step, and (b) 16-byte loads, 4 records per
// wave-instruction; grid-stride over 128-record tiles as the scans do.
//   hipcc --offload-arch=gfx950 -O3 load_width_probe.hip -o load_width_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int64_t kRecords = int64_t{1} << 26;
constexpr int kRec = 256;

template <int PF>
__global__ __launch_bounds__(256) void KLoad4(const uint32_t* __restrict__ db, int64_t tiles,
                                              uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t waves = (int64_t)gridDim.x * 4;
  uint32_t acc = 0;
  for (int64_t t = wave; t < tiles; t += waves) {
    const uint32_t* base = db + t * 128 * 64 + lane;
#pragma unroll 4
    for (int r = 0; r < 128; r += PF) {
      uint32_t v[PF];
#pragma unroll
      for (int i = 0; i < PF; ++i) v[i] = __builtin_nontemporal_load(base + (r + i) * 64);
#pragma unroll
      for (int i = 0; i < PF; ++i) acc ^= v[i];
    }
  }
  out[wave * 64 + lane] = acc;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void KLoad16(const u32x4* __restrict__ db, int64_t tiles,
                                               uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t waves = (int64_t)gridDim.x * 4;
  uint32_t acc = 0;
  for (int64_t t = wave; t < tiles; t += waves) {
    const u32x4* base = db + t * 128 * 16 + lane;  // 4 records per wave-instruction
#pragma unroll 4
    for (int r = 0; r < 128; r += 4 * 8) {
      u32x4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = __builtin_nontemporal_load(base + (r / 4 + i) * 64);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    }
  }
  out[wave * 64 + lane] = acc;
}

template <class F>
float Time(F f, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  (void)hipEventRecord(a);
  for (int r = 0; r < reps; ++r) f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const size_t bytes = kRecords * kRec;
  void* db = nullptr;
  if (hipMalloc(&db, bytes) != hipSuccess) return 1;
  (void)hipMemset(db, 1, bytes);
  uint32_t* out = nullptr;
  const int blocks = 8192;
  (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
  const int64_t tiles = kRecords / 128;
  const float t4a = Time([&] { hipLaunchKernelGGL(KLoad4<4>, dim3(blocks), dim3(256), 0, 0, (const uint32_t*)db, tiles, out); }, 5);
  const float t4b = Time([&] { hipLaunchKernelGGL(KLoad4<8>, dim3(blocks), dim3(256), 0, 0, (const uint32_t*)db, tiles, out); }, 5);
  const float t4c = Time([&] { hipLaunchKernelGGL(KLoad4<16>, dim3(blocks), dim3(256), 0, 0, (const uint32_t*)db, tiles, out); }, 5);
  const float t16 = Time([&] { hipLaunchKernelGGL(KLoad16, dim3(blocks), dim3(256), 0, 0, (const u32x4*)db, tiles, out); }, 5);
  auto tbs = [&](float ms) { return bytes / (ms * 1e-3) / 1e12; };
  printf("{\"bytes\": %zu, \"load4_pf4\": [%.3f, %.2f], \"load4_pf8\": [%.3f, %.2f], "
         "\"load4_pf16\": [%.3f, %.2f], \"load16_pf8\": [%.3f, %.2f], \"unit\": \"[ms, TB/s]\"}\n",
         bytes, t4a, tbs(t4a), t4b, tbs(t4b), t4c, tbs(t4c), t16, tbs(t16));
  return 0;
}
