// cpp_api_bench.cc — wall-clock cost of the reference's C++ API on the
// BASELINE configs c1-c3, called exactly as a C++ caller of
// dpf/distributed_point_function.h would (host std::vector results), linked
// against libdpf_amd.so.  One JSON line per config on stdout.
//
//   c1  EvaluateNext<uint64_t> full domain, log_domain_size 20
//   c2  EvaluateAt<uint128> of 16384 random points for each of 64 keys,
//       log_domain_size 128 (2^20 points)
//   c2a the same 2^20 (key, point) pairs through EvaluateAndApply<uint128>
//       (h:1072-1198, 64 distinct keys each repeated for its 16384 points)
//   c3  16 hierarchy levels of 8 bits, uint64, EvaluateNext on 2^16 distinct
//       surviving prefixes per level (distributed_point_function_benchmark.cc:
//       154-191 shape)
//   c4  (only when asked: 16 GiB of host records) DenseDpfPirServer::
//       HandleRequest over 2^26 records x 256 B for Q = 1, 8, 64 keys per
//       request (pir/dense_dpf_pir_database_benchmark.cc:37-157 batch shapes;
//       pir/dense_dpf_pir_server.cc:92-127), both parties, reconstruction
//       checked
//
// Built by distributed_point_functions_amd/build_native.py next to the
// library; run on the GPU box: _native/cpp_api_bench [reps] [c1,c2,c2a,c3,c4].
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>
#include <vector>

#include <cstring>
#include <string>

#include "dpf_amd/dense_dpf_pir_server.h"
#include "dpf_amd/distributed_point_function.h"

using namespace distributed_point_functions;

namespace {

double Now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

#define OK_OR_DIE(expr)                                                            \
  do {                                                                             \
    if (!(expr).ok()) {                                                            \
      std::fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__,                      \
                   (expr).status().ToString().c_str());                            \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

void C1(int reps) {
  DpfParameters p;
  p.set_log_domain_size(20);
  p.mutable_value_type()->mutable_integer()->set_bitsize(64);
  auto dpf = DistributedPointFunction::Create(p);
  OK_OR_DIE(dpf);
  auto keys = (*dpf)->GenerateKeys(uint128{777777}, uint128{123456789123ull});
  OK_OR_DIE(keys);
  double best = 1e30, total = 0;
  bool ok = true;
  for (int r = 0; r <= reps; ++r) {
    auto ctx = (*dpf)->CreateEvaluationContext(keys->first);
    OK_OR_DIE(ctx);
    const double t0 = Now();
    auto out = (*dpf)->EvaluateNext<uint64_t>(Span<const uint128>(), *ctx);
    const double t = Now() - t0;
    OK_OR_DIE(out);
    ok &= out->size() == (size_t{1} << 20);
    if (r > 0) {  // the first call warms up
      best = std::min(best, t);
      total += t;
    }
  }
  std::printf("{\"config\": \"c1\", \"api\": \"C++ EvaluateNext<uint64_t> -> std::vector\", "
              "\"leaves\": %d, \"best_ms\": %.4f, \"mean_ms\": %.4f, "
              "\"leaves_per_s\": %.4g, \"correct\": %s}\n",
              1 << 20, 1e3 * best, 1e3 * total / reps, (1 << 20) / best, ok ? "true" : "false");
}

void C2(int reps) {
  DpfParameters p;
  p.set_log_domain_size(128);
  p.mutable_value_type()->mutable_integer()->set_bitsize(128);
  auto dpf = DistributedPointFunction::Create(p);
  OK_OR_DIE(dpf);
  std::mt19937_64 rng(2);
  const int nkeys = 64, per = 1 << 14;
  std::vector<DpfKey> k0s, k1s;
  std::vector<std::vector<uint128>> pts(nkeys);
  std::vector<uint128> betas;
  for (int k = 0; k < nkeys; ++k) {
    const uint128 alpha = MakeUint128(rng(), rng()), beta = MakeUint128(rng(), rng());
    auto keys = (*dpf)->GenerateKeys(alpha, beta);
    OK_OR_DIE(keys);
    k0s.push_back(keys->first);
    k1s.push_back(keys->second);
    betas.push_back(beta);
    pts[k].resize(per);
    for (auto& x : pts[k]) x = MakeUint128(rng(), rng());
    pts[k][0] = alpha;
  }
  double best = 1e30;
  for (int r = 0; r <= reps; ++r) {
    const double t0 = Now();
    for (int k = 0; k < nkeys; ++k) {
      auto out = (*dpf)->EvaluateAt<uint128>(k0s[k], 0, pts[k]);
      OK_OR_DIE(out);
    }
    const double t = Now() - t0;
    if (r > 0) best = std::min(best, t);
  }
  bool ok = true;
  for (int k = 0; k < nkeys; k += 9) {
    auto a = (*dpf)->EvaluateAt<uint128>(k0s[k], 0, pts[k]);
    auto b = (*dpf)->EvaluateAt<uint128>(k1s[k], 0, pts[k]);
    OK_OR_DIE(a);
    OK_OR_DIE(b);
    ok &= uint128((*a)[0] + (*b)[0]) == betas[k] && uint128((*a)[1] + (*b)[1]) == 0;
  }
  std::printf("{\"config\": \"c2\", \"api\": \"C++ EvaluateAt<uint128>, 64 keys x 16384 points\", "
              "\"points\": %d, \"best_ms\": %.3f, \"points_per_s\": %.4g, \"correct\": %s}\n",
              nkeys * per, 1e3 * best, nkeys * per / best, ok ? "true" : "false");
}

void C2Apply(int reps) {
  DpfParameters p;
  p.set_log_domain_size(128);
  p.mutable_value_type()->mutable_integer()->set_bitsize(128);
  auto dpf = DistributedPointFunction::Create(p);
  OK_OR_DIE(dpf);
  std::mt19937_64 rng(2);
  const int nkeys = 64, per = 1 << 14;
  std::vector<DpfKey> k0s, k1s;
  std::vector<uint128> betas, alphas;
  for (int k = 0; k < nkeys; ++k) {
    const uint128 alpha = MakeUint128(rng(), rng()), beta = MakeUint128(rng(), rng());
    auto keys = (*dpf)->GenerateKeys(alpha, beta);
    OK_OR_DIE(keys);
    k0s.push_back(keys->first);
    k1s.push_back(keys->second);
    betas.push_back(beta);
    alphas.push_back(alpha);
  }
  // key i / per at point i: each key's first point is its alpha
  std::vector<const DpfKey*> kp0(nkeys * per), kp1(nkeys * per);
  std::vector<uint128> pts(nkeys * per);
  for (int i = 0; i < nkeys * per; ++i) {
    kp0[i] = &k0s[i / per];
    kp1[i] = &k1s[i / per];
    pts[i] = (i % per == 0) ? alphas[i / per] : MakeUint128(rng(), rng());
  }
  std::vector<uint128> a(pts.size()), b(pts.size());
  double best = 1e30;
  for (int r = 0; r <= reps; ++r) {
    const double t0 = Now();
    Status st = (*dpf)->EvaluateAndApply<uint128>(
        Span<const DpfKey* const>(kp0.data(), kp0.size()), pts, [&](Span<const uint128> v) {
          std::memcpy(a.data(), v.data(), 16 * v.size());
          return true;
        });
    const double t = Now() - t0;
    if (!st.ok()) {
      std::fprintf(stderr, "EvaluateAndApply: %s\n", st.ToString().c_str());
      std::exit(1);
    }
    if (r > 0) best = std::min(best, t);
  }
  Status st = (*dpf)->EvaluateAndApply<uint128>(
      Span<const DpfKey* const>(kp1.data(), kp1.size()), pts, [&](Span<const uint128> v) {
        std::memcpy(b.data(), v.data(), 16 * v.size());
        return true;
      });
  bool ok = st.ok();
  for (int i = 0; i < nkeys * per && ok; ++i)
    ok = uint128(a[i] + b[i]) == (i % per == 0 ? betas[i / per] : uint128{0});
  std::printf("{\"config\": \"c2a\", \"api\": \"C++ EvaluateAndApply<uint128>, 2^20 (key, point) "
              "pairs over 64 keys\", \"points\": %d, \"best_ms\": %.3f, \"points_per_s\": %.4g, "
              "\"correct\": %s}\n",
              nkeys * per, 1e3 * best, nkeys * per / best, ok ? "true" : "false");
}

void C4(int reps) {
  const int64_t n = int64_t{1} << 26;
  const int rec = 256;
  std::vector<char> data(static_cast<size_t>(n) * rec);
  uint64_t x = 0x9e3779b97f4a7c15ull;
  for (size_t i = 0; i < data.size(); i += 8) {  // splitmix64 records
    uint64_t z = (x += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    z ^= z >> 31;
    std::memcpy(&data[i], &z, 8);
  }
  PirConfig cfg;
  cfg.mutable_dense_dpf_pir_config()->set_num_elements(n);
  std::unique_ptr<DenseDpfPirServer> servers[2];
  double build_s = 0;
  for (int s = 0; s < 2; ++s) {
    const double t0 = Now();
    DenseDpfPirDatabase::Builder b;
    b.InsertFixed(data.data(), n, rec);
    auto db = b.Build();
    OK_OR_DIE(db);
    auto server = DenseDpfPirServer::CreatePlain(cfg, std::move(*db));
    OK_OR_DIE(server);
    servers[s] = std::move(*server);
    build_s = Now() - t0;
  }
  DpfParameters p;
  p.set_log_domain_size(26);
  p.mutable_value_type()->mutable_xor_wrapper()->set_bitsize(128);
  auto dpf = DistributedPointFunction::Create(p);
  OK_OR_DIE(dpf);
  std::mt19937_64 rng(4);
  for (int q : {1, 8, 64, 100}) {
    PirRequest req[2];
    std::vector<int64_t> idx(q);
    for (int k = 0; k < q; ++k) {
      idx[k] = static_cast<int64_t>(rng() % n);
      auto keys = (*dpf)->GenerateKeys(
          uint128(idx[k] / 128), XorWrapper<uint128>(uint128{1} << (idx[k] % 128)));
      OK_OR_DIE(keys);
      *req[0].mutable_dpf_pir_request()->mutable_plain_request()->add_dpf_key() = keys->first;
      *req[1].mutable_dpf_pir_request()->mutable_plain_request()->add_dpf_key() = keys->second;
    }
    double best = 1e30, total = 0;
    for (int r = 0; r <= reps; ++r) {
      const double t0 = Now();
      auto resp = servers[0]->HandleRequest(req[0]);
      const double t = Now() - t0;
      OK_OR_DIE(resp);
      if (r > 0) {
        best = std::min(best, t);
        total += t;
      }
    }
    auto r0 = servers[0]->HandleRequest(req[0]);
    auto r1 = servers[1]->HandleRequest(req[1]);
    OK_OR_DIE(r0);
    OK_OR_DIE(r1);
    bool ok = true;
    for (int k = 0; k < q; ++k) {
      const std::string& a = r0->dpf_pir_response().masked_response(k);
      const std::string& b = r1->dpf_pir_response().masked_response(k);
      for (int j = 0; j < rec && ok; ++j) ok = (a[j] ^ b[j]) == data[idx[k] * rec + j];
    }
    std::printf("{\"config\": \"c4\", \"api\": \"C++ DenseDpfPirServer::HandleRequest\", "
                "\"records\": %lld, \"record_bytes\": %d, \"queries\": %d, \"best_ms\": %.3f, "
                "\"mean_ms\": %.3f, \"db_GBps\": %.1f, \"build_s\": %.2f, \"correct\": %s}\n",
                static_cast<long long>(n), rec, q, 1e3 * best, 1e3 * total / reps,
                n * rec / best / 1e9, build_s, ok ? "true" : "false");
    std::fflush(stdout);
  }
}

void C3(int reps) {
  const int H = 16;
  std::vector<DpfParameters> ps(H);
  for (int i = 0; i < H; ++i) {
    ps[i].set_log_domain_size(8 * (i + 1));
    ps[i].mutable_value_type()->mutable_integer()->set_bitsize(64);
  }
  auto dpf = DistributedPointFunction::CreateIncremental(ps);
  OK_OR_DIE(dpf);
  std::mt19937_64 rng(3);
  const uint128 alpha = MakeUint128(rng(), rng());
  std::vector<uint128> betas(H);
  for (auto& b : betas) b = rng();
  auto keys = (*dpf)->GenerateKeysIncremental(alpha, betas);
  OK_OR_DIE(keys);
  // prefixes[i]: 2^16 distinct children of level i-1's prefixes, sorted,
  // alpha's prefix included
  std::vector<std::vector<uint128>> prefixes(H);
  for (int i = 1; i < H; ++i) {
    std::set<uint128> cur;
    const uint128 ap = alpha >> (128 - 8 * i);
    cur.insert(ap);
    if (i == 1) {
      for (int j = 0; j < 256; ++j) cur.insert(j);
    } else {
      const auto& prev = prefixes[i - 1];
      while (cur.size() < (size_t{1} << 16))
        cur.insert((prev[rng() % prev.size()] << 8) | (rng() & 255));
    }
    prefixes[i].assign(cur.begin(), cur.end());
  }
  if (const char* dump = std::getenv("DPF_AMD_BENCH_DUMP")) {
    // keys + prefixes, for replaying this case elsewhere (tools/replay_c3.py)
    FILE* f = std::fopen(dump, "wb");
    if (f) {
      for (const DpfKey* k : {&keys->first, &keys->second}) {
        const std::string b = k->SerializeAsString();
        const uint64_t n = b.size();
        std::fwrite(&n, 8, 1, f);
        std::fwrite(b.data(), 1, n, f);
      }
      const uint64_t a[2] = {static_cast<uint64_t>(alpha), static_cast<uint64_t>(alpha >> 64)};
      std::fwrite(a, 8, 2, f);
      for (int i = 0; i < H; ++i) {
        const uint64_t b = static_cast<uint64_t>(betas[i]), n = prefixes[i].size();
        std::fwrite(&b, 8, 1, f);
        std::fwrite(&n, 8, 1, f);
        std::fwrite(prefixes[i].data(), 16, n, f);
      }
      std::fclose(f);
    }
  }
  std::vector<double> best(H, 1e30);
  double best_total = 1e30;
  size_t leaves = 0;
  bool ok = true;
  for (int r = 0; r <= reps; ++r) {
    auto c0 = (*dpf)->CreateEvaluationContext(keys->first);
    auto c1 = (*dpf)->CreateEvaluationContext(keys->second);
    OK_OR_DIE(c0);
    OK_OR_DIE(c1);
    double total = 0;
    leaves = 0;
    for (int i = 0; i < H; ++i) {
      const double t0 = Now();
      auto a = (*dpf)->EvaluateNext<uint64_t>(prefixes[i], *c0);
      const double t = Now() - t0;
      OK_OR_DIE(a);
      total += t;
      leaves += a->size();
      if (r > 0) best[i] = std::min(best[i], t);
      if (r == 0) {  // check the share sum once
        auto b = (*dpf)->EvaluateNext<uint64_t>(prefixes[i], *c1);
        OK_OR_DIE(b);
        size_t nonzero = 0;
        for (size_t x = 0; x < a->size(); ++x) {
          const uint64_t s = (*a)[x] + (*b)[x];
          if (s != 0) {
            ++nonzero;
            if (s != static_cast<uint64_t>(betas[i]) && ok)
              std::fprintf(stderr, "c3 level %d: share sum %llu at %zu, beta %llu\n", i,
                           static_cast<unsigned long long>(s), x,
                           static_cast<unsigned long long>(betas[i]));
            ok &= s == static_cast<uint64_t>(betas[i]);
          }
        }
        if (nonzero != 1 && ok)
          std::fprintf(stderr, "c3 level %d: %zu non-zero share sums of %zu\n", i, nonzero,
                       a->size());
        ok &= nonzero == 1;
      }
    }
    if (r > 0) best_total = std::min(best_total, total);
  }
  // The result container alone: a fresh std::vector<uint64_t>(2^24) (what
  // EvaluateNext<uint64_t> returns per level at 2^16 prefixes) value-
  // initialises 128 MiB of freshly mapped pages — the floor of this API path
  // on this host, paid by the reference's own result vector too.
  double vec_best = 1e30;
  for (int r = 0; r < 5; ++r) {
    const double t0 = Now();
    std::vector<uint64_t> v(size_t{1} << 24);
    const double t = Now() - t0;
    vec_best = std::min(vec_best, t);
    if (v[12345] != 0) std::printf(" ");
  }
  std::printf("{\"config\": \"c3\", \"api\": \"C++ EvaluateNext<uint64_t> per level -> "
              "std::vector\", \"levels\": %d, \"returned_leaves\": %zu, \"best_total_ms\": %.3f, "
              "\"leaves_per_s\": %.4g, \"vector_2e24_alloc_ms\": %.3f, \"best_ms_per_level\": [",
              H, leaves, 1e3 * best_total, leaves / best_total, 1e3 * vec_best);
  for (int i = 0; i < H; ++i) std::printf("%s%.3f", i ? ", " : "", 1e3 * best[i]);
  std::printf("], \"correct\": %s}\n", ok ? "true" : "false");
}

}  // namespace

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
  const std::string only = argc > 2 ? argv[2] : "c1,c2,c2a,c3";
  auto want = [&](const char* c) { return ("," + only + ",").find("," + std::string(c) + ",") != std::string::npos; };
  if (want("c1")) C1(reps);
  if (want("c2")) C2(std::max(1, reps / 2));
  if (want("c2a")) C2Apply(std::max(1, reps / 2));
  if (want("c3")) C3(std::max(1, reps / 2));
  if (want("c4")) C4(reps);
  return 0;
}
