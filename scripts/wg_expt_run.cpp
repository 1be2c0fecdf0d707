// wg_expt_run.cpp — phase experiments on wg_kernel (C3: 5,000 nodes, 100k-pod batches), for one
// build of the library given on the command line (scripts/wg_expt.sh builds the variants: the
// product source with -DMSH_STAMPS and an MSH_WG_EXPT mask; never the product library).
//   wg_expt_run <lib.so> <tag> [batches per launch = 8] [clock]
// "clock" (a -DMSH_CLOCK_STAMPS build): about 2 s of back-to-back launches first, then one launch whose
// persistent waves stamp the shader clock (s_memtime) and the 100 MHz clock (s_memrealtime) at start
// and end; prints the median in-kernel clock over the waves (MI355X_MICROARCH.md, DVFS item 6).
// Prints one JSON line: the kernel duration per launch (msh_timing_*: the kernel's own start / stop)
// and, from the stamps of one launch, the per-wave phase durations (entry -> after the table copy and
// barrier -> after the scan -> after the stores; percentiles in microseconds) and the wave start spread.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <vector>

#include "minisched_hip.h"

#define CHECK(x)                                   \
  do {                                             \
    int rc_ = (int)(x);                            \
    if (rc_ != 0) {                                \
      fprintf(stderr, "%s failed: %d\n", #x, rc_); \
      return 1;                                    \
    }                                              \
  } while (0)

template <typename F>
F sym(void* h, const char* n) {
  void* p = dlsym(h, n);
  if (!p) {
    fprintf(stderr, "missing %s\n", n);
    exit(2);
  }
  return reinterpret_cast<F>(p);
}

static double pct(std::vector<double> v, double q) {
  if (v.empty()) return -1;
  std::sort(v.begin(), v.end());
  return v[(size_t)(q * (v.size() - 1))];
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    fprintf(stderr, "%s\n", dlerror());
    return 2;
  }
  const int NB = argc > 3 ? atoi(argv[3]) : 8;
  auto create = sym<int (*)(int, msh_ctx**)>(h, "msh_create");
  auto upload = sym<int (*)(msh_ctx*, int32_t, const uint8_t*, const int8_t*)>(h, "msh_upload_nodes");
  auto batches = sym<int (*)(msh_ctx*, int32_t, const msh_batch*, void*)>(h, "msh_schedule_batches_device");
  auto tbegin = sym<int (*)(msh_ctx*, int32_t)>(h, "msh_timing_begin");
  auto tend = sym<int (*)(msh_ctx*, int32_t*, double*, double*)>(h, "msh_timing_end");
  auto stamps_set = reinterpret_cast<int (*)(void*)>(dlsym(h, "msh_stamps_set"));
  const int N = 5000, P = 100000;
  uint64_t x = 0x6d696e69;
  auto rnd = [&]() {
    x += 0x9e3779b97f4a7c15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  };
  std::vector<uint8_t> u(N), pt(P);
  std::vector<int8_t> d(N), pd(P);
  for (int i = 0; i < N; ++i) {
    u[i] = rnd() % 10 == 0;
    d[i] = (int8_t)(i % 10);
  }
  for (int j = 0; j < P; ++j) {
    pd[j] = (int8_t)(rnd() % 100 == 0 ? -1 : rnd() % 10);
    pt[j] = rnd() % 20 == 0;
  }
  msh_ctx* ctx = nullptr;
  CHECK(create(0, &ctx));
  if (const char* nm = getenv("MSH_RUN_NORM")) {  // NodeNumber's normalize mode (3 = MIN-MAX: the KX kernel)
    auto setp = sym<int (*)(msh_ctx*, const int32_t*, int32_t, const int32_t*, int32_t, const int32_t*, const int64_t*,
                            const int32_t*, int32_t)>(h, "msh_set_plugins_ex");
    const int32_t f[1] = {MSH_PLUGIN_NODE_UNSCHEDULABLE}, pre[1] = {MSH_PLUGIN_NODE_NUMBER},
                  sc[1] = {MSH_PLUGIN_NODE_NUMBER}, norm[1] = {atoi(nm)};
    const int64_t w[1] = {1};
    CHECK(setp(ctx, f, 1, pre, 1, sc, w, norm, 1));
  }
  CHECK(upload(ctx, N, u.data(), d.data()));
  std::vector<msh_batch> desc(NB);
  for (int b = 0; b < NB; ++b) {
    int8_t* dpd;
    uint8_t* dpt;
    int32_t *doi, *dst;
    int64_t* dsc;
    CHECK(hipMalloc(&dpd, P));
    CHECK(hipMalloc(&dpt, P));
    CHECK(hipMalloc(&doi, P * 4));
    CHECK(hipMalloc(&dst, P * 4));
    CHECK(hipMalloc(&dsc, (size_t)P * 8));
    CHECK(hipMemcpy(dpd, pd.data(), P, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dpt, pt.data(), P, hipMemcpyHostToDevice));
    desc[b] = msh_batch{P, 0, dpd, dpt, doi, dsc, dst};
  }
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  for (int i = 0; i < 10; ++i) CHECK(batches(ctx, NB, desc.data(), st));
  CHECK(hipStreamSynchronize(st));
  const int R = 30;
  CHECK(tbegin(ctx, R));
  for (int i = 0; i < R; ++i) CHECK(batches(ctx, NB, desc.data(), st));
  int32_t n = 0;
  double tot = 0, mx = 0;
  CHECK(tend(ctx, &n, &tot, &mx));
  printf("{\"tag\": \"%s\", \"batches_per_launch\": %d, \"kernel_us\": %.3f, \"us_per_batch\": %.3f", argv[2], NB,
         tot * 1e3 / n, tot * 1e3 / n / NB);
  const bool clock_mode = argc > 4 && std::string(argv[4]) == "clock";
  if (argc > 4 && std::string(argv[4]) == "region") {
    // the bench's K = NB region from C: device synchronize, clock, one launch of NB batches, device
    // synchronize, clock; 200 repetitions after 1 ms idle each; median and p10 / p90 in microseconds
    std::vector<double> us;
    for (int rep = 0; rep < 200; ++rep) {
      CHECK(hipDeviceSynchronize());
      const auto idle = std::chrono::steady_clock::now() + std::chrono::microseconds(1000);
      while (std::chrono::steady_clock::now() < idle) {
      }
      const auto t0 = std::chrono::steady_clock::now();
      CHECK(batches(ctx, NB, desc.data(), st));
      CHECK(hipDeviceSynchronize());
      us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    printf(", \"region_us\": [%.2f, %.2f, %.2f]", pct(us, 0.1), pct(us, 0.5), pct(us, 0.9));
  }
  if (stamps_set && clock_mode) {
    const size_t slots = (size_t)4096 * 16 * 8;
    unsigned long long* d_st;
    CHECK(hipMalloc(&d_st, slots * 8));
    CHECK(hipMemset(d_st, 0, slots * 8));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0, st));
    int warm = 0;
    for (float ms = 0; ms < 2000.f; ++warm) {
      for (int i = 0; i < 50; ++i) CHECK(batches(ctx, NB, desc.data(), st));
      warm += 49;
      CHECK(hipEventRecord(e1, st));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
    }
    CHECK(stamps_set(d_st));
    CHECK(tbegin(ctx, 1));
    CHECK(batches(ctx, NB, desc.data(), st));
    CHECK(tend(ctx, &n, &tot, &mx));
    std::vector<unsigned long long> hs(slots);
    CHECK(hipMemcpy(hs.data(), d_st, slots * 8, hipMemcpyDeviceToHost));
    std::vector<double> ghz, life, beg, fin;
    unsigned long long r_min = ~0ull;
    for (size_t w = 0; w < slots / 8; ++w)
      if (hs[w * 8 + 1]) r_min = std::min(r_min, hs[w * 8 + 1]);
    // waves per CU (xcc, se, sh, cu from HW_ID / XCC_ID) and the per-CU mean end time
    std::map<unsigned, std::pair<int, double>> cu;
    std::map<int, int> items;
    FILE* dump = getenv("CLOCK_DUMP") ? fopen(getenv("CLOCK_DUMP"), "w") : nullptr;
    for (size_t w = 0; w < slots / 8; ++w) {
      const unsigned long long* t = &hs[w * 8];
      if (!t[1] || t[3] <= t[1]) continue;
      const unsigned hw = (unsigned)t[4], xcc = (unsigned)t[5] & 0xf;
      const unsigned key = (xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xf);
      cu[key].first++;
      cu[key].second += (t[3] - r_min) * 0.01;
      items[(int)t[6]]++;
      if (dump) fprintf(dump, "%u %u %u %.2f %.2f %d %d\n", xcc, (hw >> 13) & 7, ((hw >> 12) & 1) * 16 + ((hw >> 8) & 0xf),
                        (t[1] - r_min) * 0.01, (t[3] - r_min) * 0.01, (int)t[6], (int)t[7]);
    }
    if (dump) fclose(dump);
    std::map<int, std::pair<int, double>> by_waves;  // waves on the CU -> (CUs, mean end)
    for (auto& kv : cu) {
      by_waves[kv.second.first].first++;
      by_waves[kv.second.first].second += kv.second.second / kv.second.first;
    }
    printf(", \"cus\": %zu, \"waves_per_cu\": {", cu.size());
    bool first = true;
    for (auto& kv : by_waves) {
      printf("%s\"%d\": [%d, %.2f]", first ? "" : ", ", kv.first, kv.second.first, kv.second.second / kv.second.first);
      first = false;
    }
    printf("}, \"items_per_wave\": {");
    first = true;
    for (auto& kv : items) {
      printf("%s\"%d\": %d", first ? "" : ", ", kv.first, kv.second);
      first = false;
    }
    printf("}");
    for (size_t w = 0; w < slots / 8; ++w) {
      const unsigned long long* t = &hs[w * 8];
      if (!t[1] || t[3] <= t[1]) continue;
      ghz.push_back((double)(t[2] - t[0]) / (double)(t[3] - t[1]) * 0.1);
      life.push_back((t[3] - t[1]) * 0.01);
      beg.push_back((t[1] - r_min) * 0.01);
      fin.push_back((t[3] - r_min) * 0.01);
    }
    printf(", \"clock\": {\"warm_launches\": %d, \"stamped_kernel_us\": %.3f, \"waves\": %zu, \"ghz\": [%.3f, %.3f, %.3f], "
           "\"wave_life_us\": [%.2f, %.2f, %.2f], \"start_us\": [%.2f, %.2f, %.2f, %.2f], \"end_us\": [%.2f, %.2f, %.2f, %.2f, %.2f]}",
           warm, tot * 1e3, ghz.size(), pct(ghz, 0.1), pct(ghz, 0.5), pct(ghz, 0.9), pct(life, 0.1), pct(life, 0.5),
           pct(life, 0.9), pct(beg, 0.1), pct(beg, 0.5), pct(beg, 0.9), pct(beg, 1.0), pct(fin, 0.0), pct(fin, 0.1),
           pct(fin, 0.5), pct(fin, 0.9), pct(fin, 1.0));
  } else if (stamps_set) {
    const int blocks = (P + 255) / 256;
    const size_t slots = (size_t)blocks * NB * 4 * 4;
    unsigned long long* d_st;
    CHECK(hipMalloc(&d_st, slots * 8));
    CHECK(hipMemset(d_st, 0, slots * 8));
    CHECK(stamps_set(d_st));
    CHECK(batches(ctx, NB, desc.data(), st));
    CHECK(hipStreamSynchronize(st));
    std::vector<unsigned long long> hs(slots);
    CHECK(hipMemcpy(hs.data(), d_st, slots * 8, hipMemcpyDeviceToHost));
    unsigned long long t_min = ~0ull, t_max = 0;
    for (size_t w = 0; w < slots / 4; ++w)
      if (hs[w * 4]) {
        t_min = std::min(t_min, hs[w * 4]);
        t_max = std::max(t_max, hs[w * 4 + 3]);
      }
    std::vector<double> start, pro, scan, tail, life;
    for (size_t w = 0; w < slots / 4; ++w) {
      const unsigned long long* t = &hs[w * 4];
      if (!t[0] || !t[3]) continue;
      start.push_back((t[0] - t_min) * 0.01);
      pro.push_back((t[1] - t[0]) * 0.01);
      scan.push_back((t[2] - t[1]) * 0.01);
      tail.push_back((t[3] - t[2]) * 0.01);
      life.push_back((t[3] - t[0]) * 0.01);
    }
    printf(", \"waves\": %zu, \"span_us\": %.2f, \"start_us\": [%.2f, %.2f, %.2f, %.2f], \"prologue_us\": [%.2f, %.2f, %.2f], "
           "\"scan_us\": [%.2f, %.2f, %.2f], \"tail_us\": [%.2f, %.2f, %.2f], \"life_us\": [%.2f, %.2f, %.2f]",
           start.size(), (t_max - t_min) * 0.01, pct(start, 0.1), pct(start, 0.5), pct(start, 0.9), pct(start, 1.0),
           pct(pro, 0.1), pct(pro, 0.5), pct(pro, 0.9), pct(scan, 0.1), pct(scan, 0.5), pct(scan, 0.9), pct(tail, 0.1),
           pct(tail, 0.5), pct(tail, 0.9), pct(life, 0.1), pct(life, 0.5), pct(life, 0.9));
  }
  printf("}\n");
  return 0;
}
