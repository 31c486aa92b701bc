// Host pool dispatch latency vs serial loops (tools/pool_latency.cc)
#include "host_device.h"
#include <chrono>
#include <cstdio>
namespace dpf_amd { int ThreadCacheCap() { return 64; } }
using namespace distributed_point_functions::dpf_internal_host;
using clk = std::chrono::steady_clock;
int main() {
  HostPool& p = HostPool::Get();
  std::vector<uint64_t> v(1 << 16, 1);
  volatile uint64_t sink = 0;
  for (int warm = 0; warm < 100; ++warm) p.ParallelRanges(1 << 16, 8192, [&](int, int64_t, int64_t) {});
  for (int grain : {8192, 16384, 32768, 65536}) {
    for (int gap_us : {0, 300}) {
      double tot = 0;
      const int N = 300;
      for (int it = 0; it < N; ++it) {
        if (gap_us) std::this_thread::sleep_for(std::chrono::microseconds(gap_us));
        auto t0 = clk::now();
        uint64_t sums[8] = {};
        p.ParallelRanges(1 << 16, grain, [&](int r, int64_t b, int64_t e) {
          uint64_t s = 0;
          for (int64_t i = b; i < e; ++i) s += v[i] * (uint64_t)i;
          sums[r] = s;
        });
        sink = sink + sums[0];
        tot += std::chrono::duration<double, std::micro>(clk::now() - t0).count();
      }
      std::printf("2^16 elements, grain %d (%d parts), gap %d us: %.1f us\n", grain,
                  (1 << 16) / grain, gap_us, tot / N);
    }
  }
  std::printf("hardware_concurrency %u\n", std::thread::hardware_concurrency());
}
