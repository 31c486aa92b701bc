// api_test.cc — the reference's C++ API used as a drop-in: this file is
// written against include/dpf_amd/*.h exactly as a caller of
// dpf/distributed_point_function.h and dcf/distributed_comparison_function.h
// would write it (templates, StatusOr, Span), and links libdpf_amd.so.
// Checks mirror the reference's tests:
//   distributed_point_function_test.cc:1015-1042 (full-domain share-sum),
//   :1044-1079 (EvaluateAt share-sum), :652-696 (incremental),
//   distributed_comparison_function_test.cc:106-133 (GenEval),
//   pir/dense_dpf_pir_server_test.cc (plain requests reconstruct records),
//   here over a database sharded with Builder::SetDevices.
// Exit status 0 = all checks passed.  Built and run by tests/test_cpp_api.py.
#include <algorithm>
#include <cstdio>
#include <memory>
#include <string>
#include <set>
#include <vector>

#include "dpf_amd/dense_dpf_pir_server.h"
#include "dpf_amd/distributed_comparison_function.h"
#include "dpf_amd/distributed_point_function.h"

using namespace distributed_point_functions;

static int failures = 0;
#define CHECK(cond)                                                                  \
  do {                                                                               \
    if (!(cond)) {                                                                   \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                                    \
    }                                                                                \
  } while (0)
#define CHECK_OK(expr)                                                \
  do {                                                                \
    if (!(expr).ok()) {                                               \
      std::fprintf(stderr, "%s:%d: not OK: %s\n", __FILE__, __LINE__, \
                   (expr).status().ToString().c_str());               \
      return 1;                                                       \
    }                                                                 \
  } while (0)

static int FullDomainUint64() {
  DpfParameters p;
  p.set_log_domain_size(10);
  p.mutable_value_type()->mutable_integer()->set_bitsize(64);
  auto dpf = DistributedPointFunction::Create(p);
  CHECK_OK(dpf);
  const uint128 alpha = 123;
  auto keys = (*dpf)->GenerateKeys(alpha, uint128{42});
  CHECK_OK(keys);
  auto c0 = (*dpf)->CreateEvaluationContext(keys->first);
  auto c1 = (*dpf)->CreateEvaluationContext(keys->second);
  CHECK_OK(c0);
  CHECK_OK(c1);
  auto r0 = (*dpf)->EvaluateNext<uint64_t>(Span<const uint128>(), *c0);
  auto r1 = (*dpf)->EvaluateNext<uint64_t>(Span<const uint128>(), *c1);
  CHECK_OK(r0);
  CHECK_OK(r1);
  CHECK(r0->size() == 1024 && r1->size() == 1024);
  for (size_t x = 0; x < r0->size(); ++x)
    CHECK(uint64_t((*r0)[x] + (*r1)[x]) == (x == alpha ? 42u : 0u));
  // EvaluateAt on a few points of the same keys.
  std::vector<uint128> pts = {0, 122, 123, 124, 1023};
  auto a0 = (*dpf)->EvaluateAt<uint64_t>(keys->first, 0, pts);
  auto a1 = (*dpf)->EvaluateAt<uint64_t>(keys->second, 0, pts);
  CHECK_OK(a0);
  CHECK_OK(a1);
  for (size_t i = 0; i < pts.size(); ++i)
    CHECK(uint64_t((*a0)[i] + (*a1)[i]) == (pts[i] == alpha ? 42u : 0u));
  return 0;
}

using P64 = IntModN<uint64_t, 18446744073709551557ull>;
using C5 = Tuple<uint32_t, P64>;

static int IncrementalTuple() {
  // Two hierarchy levels of the c5 value type (security_parameter = 48).
  std::vector<DpfParameters> ps(2);
  ps[0].set_log_domain_size(6);
  ps[1].set_log_domain_size(12);
  for (auto& p : ps) {
    *p.mutable_value_type() = ToValueType<C5>();
    p.set_security_parameter(48);
  }
  auto dpf = DistributedPointFunction::CreateIncremental(ps);
  CHECK_OK(dpf);
  const uint128 alpha = 0xabc;
  std::vector<C5> betas = {C5(7u, P64(11)), C5(13u, P64(17))};
  auto keys = (*dpf)->GenerateKeysIncremental<C5>(alpha, Span<const C5>(betas.data(), 2));
  CHECK_OK(keys);
  auto c0 = (*dpf)->CreateEvaluationContext(keys->first);
  auto c1 = (*dpf)->CreateEvaluationContext(keys->second);
  CHECK_OK(c0);
  CHECK_OK(c1);
  auto l0a = (*dpf)->EvaluateNext<C5>(Span<const uint128>(), *c0);
  auto l0b = (*dpf)->EvaluateNext<C5>(Span<const uint128>(), *c1);
  CHECK_OK(l0a);
  CHECK_OK(l0b);
  for (size_t x = 0; x < 64; ++x)
    CHECK(((*l0a)[x] + (*l0b)[x]) == ((x == (alpha >> 6)) ? betas[0] : C5()));
  std::vector<uint128> prefixes = {1, alpha >> 6, 60};
  auto l1a = (*dpf)->EvaluateNext<C5>(prefixes, *c0);
  auto l1b = (*dpf)->EvaluateNext<C5>(prefixes, *c1);
  CHECK_OK(l1a);
  CHECK_OK(l1b);
  CHECK(l1a->size() == 3 * 64);
  for (size_t i = 0; i < l1a->size(); ++i) {
    const uint128 x = (prefixes[i / 64] << 6) | (i % 64);
    CHECK(((*l1a)[i] + (*l1b)[i]) == (x == alpha ? betas[1] : C5()));
  }
  return 0;
}

// distributed_point_function_test.cc:190-235 (TestSinglePointPartialEvaluation):
// EvaluateAt<uint32_t>(0, {prefix}, ctx) at a 108-bit level, then
// EvaluateUntil<uint32_t>(1, {prefix}, ctx) from the stored evaluation.
static int SinglePointPartialEvaluation() {
  std::vector<DpfParameters> ps(2);
  ps[0].set_log_domain_size(108);
  ps[1].set_log_domain_size(128);
  for (auto& p : ps) p.mutable_value_type()->mutable_integer()->set_bitsize(32);
  auto dpf = DistributedPointFunction::CreateIncremental(ps);
  CHECK_OK(dpf);
  const uint128 prefix = 0xdeadbeef, suffix = 23;
  const uint128 alpha = (prefix << 20) + suffix;
  const uint32_t beta = 42;
  auto keys = (*dpf)->GenerateKeysIncremental(alpha, std::vector<uint128>{beta, beta});
  CHECK_OK(keys);
  auto ca = (*dpf)->CreateEvaluationContext(keys->first);
  auto cb = (*dpf)->CreateEvaluationContext(keys->second);
  CHECK_OK(ca);
  CHECK_OK(cb);
  std::vector<uint128> pre = {prefix};
  auto ra = (*dpf)->EvaluateAt<uint32_t>(0, pre, *ca);
  auto rb = (*dpf)->EvaluateAt<uint32_t>(0, pre, *cb);
  CHECK_OK(ra);
  CHECK_OK(rb);
  CHECK(uint32_t((*ra)[0] + (*rb)[0]) == beta);
  CHECK(ca->previous_hierarchy_level() == 0 && ca->partial_evaluations_size() == 1);
  auto ua = (*dpf)->EvaluateUntil<uint32_t>(1, pre, *ca);
  auto ub = (*dpf)->EvaluateUntil<uint32_t>(1, pre, *cb);
  CHECK_OK(ua);
  CHECK_OK(ub);
  CHECK(ua->size() == (size_t{1} << 20) && ub->size() == ua->size());
  for (size_t i = 0; i < ua->size(); ++i)
    CHECK(uint32_t((*ua)[i] + (*ub)[i]) == (i == suffix ? beta : 0u));
  return 0;
}

// A context after EvaluateNext with prefixes (its list held on the device):
// the reference's field accessors see the list, a copy sees the same list, a
// serialize / parse round trip keeps it, and a parsed context (list on the
// host) continues to the same outputs; writing the field takes it to the host.
static int ContextListAccessors() {
  std::vector<DpfParameters> ps(3);
  ps[0].set_log_domain_size(8);
  ps[1].set_log_domain_size(16);
  ps[2].set_log_domain_size(24);
  for (auto& p : ps) p.mutable_value_type()->mutable_integer()->set_bitsize(64);
  auto dpf = DistributedPointFunction::CreateIncremental(ps);
  CHECK_OK(dpf);
  const uint128 alpha = 0xabcdef;
  auto keys = (*dpf)->GenerateKeysIncremental(alpha, std::vector<uint128>{1, 2, 3});
  CHECK_OK(keys);
  auto ctx = (*dpf)->CreateEvaluationContext(keys->first);
  CHECK_OK(ctx);
  CHECK_OK((*dpf)->EvaluateNext<uint64_t>(Span<const uint128>(), *ctx));
  std::vector<uint128> p1 = {3, 7, 8, 0xab, 0xab, 200};  // sorted, one duplicate
  CHECK_OK((*dpf)->EvaluateNext<uint64_t>(p1, *ctx));
  // tree indices of level 0 (8 bits, uint64: 2 elements per block): p >> 1
  const std::vector<uint64_t> want = {1, 3, 4, 0x55, 100};
  CHECK(ctx->partial_evaluations_size() == 5);
  if (ctx->partial_evaluations_size() != 5) return 1;
  for (int i = 0; i < 5; ++i)
    CHECK(ctx->partial_evaluations(i).prefix().low() == want[i] &&
          ctx->partial_evaluations(i).prefix().high() == 0);
  EvaluationContext copy = *ctx;
  CHECK(copy.partial_evaluations_size() == 5 &&
        copy.partial_evaluations(4).seed().low() == ctx->partial_evaluations(4).seed().low());
  EvaluationContext parsed;
  CHECK(parsed.ParseFromString(ctx->SerializeAsString()));
  CHECK(parsed.SerializeAsString() == ctx->SerializeAsString());
  std::vector<uint128> p2 = {(uint128{0xab} << 8) | 0xcd, (uint128{0xab} << 8) | 0xef,
                             (uint128{200} << 8) | 1};
  auto a = (*dpf)->EvaluateNext<uint64_t>(p2, *ctx);
  auto b = (*dpf)->EvaluateNext<uint64_t>(p2, parsed);
  CHECK_OK(a);
  CHECK_OK(b);
  CHECK(*a == *b);
  CHECK(ctx->SerializeAsString() == parsed.SerializeAsString());
  // a write takes the (device-held) list of `copy` to the host first
  copy.mutable_partial_evaluations(0)->set_control_bit(!copy.partial_evaluations(0).control_bit());
  CHECK(copy.partial_evaluations_size() == 5 &&
        copy.partial_evaluations(1).prefix().low() == want[1]);
  return 0;
}

static int DcfGenEval() {
  DcfParameters p;
  p.mutable_parameters()->set_log_domain_size(5);
  p.mutable_parameters()->mutable_value_type()->mutable_integer()->set_bitsize(32);
  auto dcf = DistributedComparisonFunction::Create(p);
  CHECK_OK(dcf);
  for (uint128 alpha = 0; alpha < 32; alpha += 5) {
    auto keys = (*dcf)->GenerateKeys<uint32_t>(alpha, 42u);
    CHECK_OK(keys);
    std::vector<DcfKey> k0(32, keys->first), k1(32, keys->second);
    std::vector<uint128> xs(32);
    for (int x = 0; x < 32; ++x) xs[x] = x;
    auto r0 = (*dcf)->BatchEvaluate<uint32_t>(k0, xs);
    auto r1 = (*dcf)->BatchEvaluate<uint32_t>(k1, xs);
    CHECK_OK(r0);
    CHECK_OK(r1);
    for (int x = 0; x < 32; ++x)
      CHECK(uint32_t((*r0)[x] + (*r1)[x]) == (uint128(x) < alpha ? 42u : 0u));
  }
  // Error path with the reference's message.
  DcfParameters bad;
  bad.mutable_parameters()->set_log_domain_size(0);
  auto e = DistributedComparisonFunction::Create(bad);
  CHECK(!e.ok() && e.status().message() == "A DCF must have log_domain_size >= 1");
  return 0;
}

// KeyGenerationFailsIfValueTypeNotRegistered (distributed_point_function_
// test.cc:148-167) and the templated overload registering T (:130-146).
static int Registration() {
  DpfParameters p;
  p.set_log_domain_size(10);
  p.mutable_value_type()->mutable_tuple()->add_elements()->mutable_integer()->set_bitsize(32);
  auto dpf = DistributedPointFunction::Create(p);
  CHECK_OK(dpf);
  Value beta;
  beta.mutable_tuple()->add_elements()->mutable_integer()->set_value_uint64(42);
  auto bad = (*dpf)->GenerateKeys(23, beta);
  CHECK(!bad.ok() && bad.status().code() == StatusCode::kFailedPrecondition);
  CHECK(!bad.ok() && bad.status().message().rfind("No value correction function known", 0) == 0);
  auto good = (*dpf)->GenerateKeys(23, Tuple<uint32_t>(42u));  // ToValue<T> registers T
  CHECK_OK(good);
  auto again = (*dpf)->GenerateKeys(23, beta);
  CHECK_OK(again);
  return 0;
}

// EvaluateAndApply stops evaluating when op returns false (h:1190-1196).
static int EvaluateAndApplyStops() {
  std::vector<DpfParameters> ps(3);
  for (int h = 0; h < 3; ++h) {
    ps[h].set_log_domain_size(8 * (h + 1));
    ps[h].mutable_value_type()->mutable_integer()->set_bitsize(64);
  }
  auto dpf = DistributedPointFunction::CreateIncremental(ps);
  CHECK_OK(dpf);
  auto keys = (*dpf)->GenerateKeysIncremental(uint128{0x123456},
                                              std::vector<uint128>{1, 2, 3});
  CHECK_OK(keys);
  std::vector<DpfKey> ks = {keys->first, keys->second};
  std::vector<uint128> pts = {0x123456, 0x123456};
  int calls = 0;
  auto st = (*dpf)->EvaluateAndApply<uint64_t>(
      Span<const DpfKey>(ks.data(), ks.size()), Span<const uint128>(pts.data(), pts.size()),
      [&calls](Span<const uint64_t> v) {
        ++calls;
        return v.size() == 2 && calls < 2;  // stop after the second level
      });
  CHECK(st.ok());
  CHECK(calls == 2);
  int all = 0;
  std::vector<uint64_t> sums;
  st = (*dpf)->EvaluateAndApply<uint64_t>(
      Span<const DpfKey>(ks.data(), ks.size()), Span<const uint128>(pts.data(), pts.size()),
      [&](Span<const uint64_t> v) {
        ++all;
        sums.push_back(v[0] + v[1]);
        return true;
      });
  CHECK(st.ok() && all == 3);
  CHECK(sums == std::vector<uint64_t>({1, 2, 3}));
  return 0;
}

// Incremental evaluation with many surviving prefixes per level (the c3
// heavy-hitters shape, smaller): share sums at every level.  Run under the
// ROCm runtime in /opt/rocm (not torch's), this is the case that exposed the
// hipMallocAsync pool issue host_device.h's DevicePool works around.
static int IncrementalManyPrefixes() {
  const int H = 8;
  std::vector<DpfParameters> ps(H);
  for (int i = 0; i < H; ++i) {
    ps[i].set_log_domain_size(8 * (i + 1));
    ps[i].mutable_value_type()->mutable_integer()->set_bitsize(64);
  }
  auto dpf = DistributedPointFunction::CreateIncremental(ps);
  CHECK_OK(dpf);
  const uint128 alpha = 0x0123456789abcdefull;
  std::vector<uint128> betas(H);
  for (int i = 0; i < H; ++i) betas[i] = 1000 + i;
  auto keys = (*dpf)->GenerateKeysIncremental(alpha, betas);
  CHECK_OK(keys);
  auto c0 = (*dpf)->CreateEvaluationContext(keys->first);
  auto c1 = (*dpf)->CreateEvaluationContext(keys->second);
  CHECK_OK(c0);
  CHECK_OK(c1);
  std::vector<uint128> prefixes;
  uint64_t x = 88172645463325252ull;  // xorshift64
  for (int i = 0; i < H; ++i) {
    auto a = (*dpf)->EvaluateNext<uint64_t>(prefixes, *c0);
    auto b = (*dpf)->EvaluateNext<uint64_t>(prefixes, *c1);
    CHECK_OK(a);
    CHECK_OK(b);
    size_t nonzero = 0;
    for (size_t j = 0; j < a->size(); ++j) {
      const uint64_t s = (*a)[j] + (*b)[j];
      if (s) {
        ++nonzero;
        CHECK(s == 1000u + i);
      }
    }
    CHECK(nonzero == 1);
    if (i + 1 == H) break;
    // next level's candidates: 2^14 distinct children of these prefixes,
    // alpha's included
    std::set<uint128> next;
    next.insert(alpha >> (64 - 8 * (i + 1)));
    while (next.size() < (i == 0 ? size_t{256} : size_t{1} << 14)) {
      x ^= x << 13;
      x ^= x >> 7;
      x ^= x << 17;
      const uint128 parent = prefixes.empty() ? 0 : prefixes[x % prefixes.size()];
      next.insert(prefixes.empty() ? uint128(x & 255) : (parent << 8) | ((x >> 32) & 255));
    }
    prefixes.assign(next.begin(), next.end());
  }
  return 0;
}

// EvaluateAndApply over many points that share a few key objects (the
// reference takes one key per point; callers pass the same key repeatedly):
// every share pair sums to beta at alpha and to 0 elsewhere, per level.
static int EvaluateAndApplyRepeatedKeys() {
  std::vector<DpfParameters> ps(2);
  ps[0].set_log_domain_size(10);
  ps[1].set_log_domain_size(20);
  for (auto& p : ps) p.mutable_value_type()->mutable_integer()->set_bitsize(32);
  auto dpf = DistributedPointFunction::CreateIncremental(ps);
  CHECK_OK(dpf);
  const uint128 alphas[3] = {0x12345, 0xfffff, 0};
  std::vector<std::pair<DpfKey, DpfKey>> pairs;
  for (int k = 0; k < 3; ++k) {
    auto kp = (*dpf)->GenerateKeysIncremental(alphas[k], std::vector<uint128>{7u + k, 100u + k});
    CHECK_OK(kp);
    pairs.push_back(*kp);
  }
  const int n = 3000;
  std::vector<DpfKey> k0, k1;
  std::vector<uint128> pts;
  for (int i = 0; i < n; ++i) {
    const int k = (i / 7) % 3;  // runs of one key, then switches
    k0.push_back(pairs[k].first);
    k1.push_back(pairs[k].second);
    pts.push_back(i % 5 == 0 ? alphas[k] : uint128((i * 2654435761u) & 0xfffff));
  }
  std::vector<std::vector<uint32_t>> a, b;
  auto sa = (*dpf)->EvaluateAndApply<uint32_t>(
      Span<const DpfKey>(k0.data(), k0.size()), Span<const uint128>(pts.data(), pts.size()),
      [&a](Span<const uint32_t> v) {
        a.emplace_back(v.begin(), v.end());
        return true;
      });
  auto sb = (*dpf)->EvaluateAndApply<uint32_t>(
      Span<const DpfKey>(k1.data(), k1.size()), Span<const uint128>(pts.data(), pts.size()),
      [&b](Span<const uint32_t> v) {
        b.emplace_back(v.begin(), v.end());
        return true;
      });
  CHECK(sa.ok() && sb.ok());
  CHECK(a.size() == 2 && b.size() == 2);
  if (a.size() != 2 || b.size() != 2) return 1;
  for (int h = 0; h < 2; ++h) {
    CHECK(a[h].size() == size_t(n) && b[h].size() == size_t(n));
    const int shift = h == 0 ? 10 : 0;
    for (int i = 0; i < n; ++i) {
      const int k = (i / 7) % 3;
      const bool hit = (pts[i] >> shift) == (alphas[k] >> shift);
      const uint32_t want = hit ? (h == 0 ? 7u + k : 100u + k) : 0u;
      if (uint32_t(a[h][i] + b[h][i]) != want) {
        CHECK(uint32_t(a[h][i] + b[h][i]) == want);
        return 1;
      }
    }
  }
  return 0;
}

// Two plain DenseDpfPirServers over the same records, one database on one
// shard and one split into three shards with Builder::SetDevices (all on
// device 0 here; the same code path peer-copies partials across GPUs): the
// XOR of their responses is each requested record, zero padded to the
// longest record (dense_dpf_pir_client.cc:124-161).
static int PirShardedPlainRequests() {
  const int64_t n = 1000;  // not a multiple of the 128-record block
  std::vector<std::string> recs(n);
  for (int64_t i = 0; i < n; ++i) {
    recs[i].resize(1 + (i * 7) % 40);
    for (size_t j = 0; j < recs[i].size(); ++j) recs[i][j] = char((i * 31 + j * 17 + 5) & 255);
  }
  size_t max_len = 0;
  for (auto& r : recs) max_len = std::max(max_len, r.size());
  PirConfig cfg;
  cfg.mutable_dense_dpf_pir_config()->set_num_elements(n);
  auto make = [&](std::vector<int> devices) -> std::unique_ptr<DenseDpfPirServer> {
    DenseDpfPirDatabase::Builder b;
    for (auto& r : recs) b.Insert(r);
    if (!devices.empty()) b.SetDevices(devices);
    auto db = b.Build();
    if (!db.ok()) return nullptr;
    auto s = DenseDpfPirServer::CreatePlain(cfg, std::move(*db));
    return s.ok() ? std::move(*s) : nullptr;
  };
  auto s0 = make({});
  auto s1 = make({0, 0, 0});
  CHECK(s0 && s1);
  if (!s0 || !s1) return 1;
  // the client's DPF (dense_dpf_pir_client.cc:50-75): ceil(log2 n) levels,
  // XorWrapper<uint128> values
  DpfParameters cp;
  cp.set_log_domain_size(10);
  cp.mutable_value_type()->mutable_xor_wrapper()->set_bitsize(128);
  auto client = DistributedPointFunction::Create(cp);
  CHECK_OK(client);
  const int64_t idx[] = {0, 127, 128, 517, 999, 517};
  PirRequest r0, r1;
  for (int64_t i : idx) {
    auto kp = (*client)->GenerateKeys(uint128(i / 128),
                                     XorWrapper<uint128>(uint128(1) << (i % 128)));
    CHECK_OK(kp);
    *r0.mutable_dpf_pir_request()->mutable_plain_request()->add_dpf_key() = kp->first;
    *r1.mutable_dpf_pir_request()->mutable_plain_request()->add_dpf_key() = kp->second;
  }
  auto a = s0->HandleRequest(r0);
  auto b = s1->HandleRequest(r1);
  CHECK_OK(a);
  CHECK_OK(b);
  const auto& ma = a->dpf_pir_response();
  const auto& mb = b->dpf_pir_response();
  CHECK(ma.masked_response_size() == 6 && mb.masked_response_size() == 6);
  if (ma.masked_response_size() != 6 || mb.masked_response_size() != 6) return 1;
  for (int q = 0; q < 6; ++q) {
    const std::string& x = ma.masked_response(q);
    const std::string& y = mb.masked_response(q);
    CHECK(x.size() == max_len && y.size() == max_len);
    std::string want = recs[idx[q]];
    want.resize(max_len, '\0');
    std::string got(max_len, '\0');
    for (size_t j = 0; j < max_len && j < x.size() && j < y.size(); ++j) got[j] = x[j] ^ y[j];
    CHECK(got == want);
  }
  return 0;
}

int main() {
  if (FullDomainUint64() || IncrementalTuple() || SinglePointPartialEvaluation() ||
      ContextListAccessors() ||
      DcfGenEval() || Registration() ||
      EvaluateAndApplyStops() || IncrementalManyPrefixes() || EvaluateAndApplyRepeatedKeys() ||
      PirShardedPlainRequests())
    return 2;
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("cpp api: all checks passed\n");
  return 0;
}
