// stamps_run.hip — wave timeline of one C3 batch launch (rows_kernel), from the stamps build of the
// library (scripts/stamps.sh: msh_kernels.hip with -DMSH_STAMPS; never the product library). Per
// wave the kernel records the 100 MHz wall clock at entry, after the prologue's loads, after the
// scan and before the stores; this prints, per launch, the spread of wave start times and the
// phase durations (percentiles over waves, in microseconds) next to the launch's HIP-event time.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "minisched_hip.h"

extern "C" int msh_stamps_set(void* p);

#define CHECK(x)                                   \
  do {                                             \
    int rc_ = (int)(x);                            \
    if (rc_ != 0) {                                \
      fprintf(stderr, "%s failed: %d\n", #x, rc_); \
      return 1;                                    \
    }                                              \
  } while (0)

static double pct(std::vector<double> v, double q) {
  if (v.empty()) return -1;
  std::sort(v.begin(), v.end());
  return v[(size_t)(q * (v.size() - 1))];
}

int main(int argc, char** argv) {
  const int N = 5000, P = argc > 1 ? atoi(argv[1]) : 100000;
  const size_t slots = ((size_t)P / 64 + 1) * 16 * 4;
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
  CHECK(msh_create(0, &ctx));
  CHECK(msh_upload_nodes(ctx, N, u.data(), d.data()));
  int8_t* d_pd;
  uint8_t* d_pt;
  int32_t *d_oi, *d_os;
  int64_t* d_sc;
  unsigned long long* d_st;
  CHECK(hipMalloc(&d_pd, P));
  CHECK(hipMalloc(&d_pt, P));
  CHECK(hipMalloc(&d_oi, P * 4));
  CHECK(hipMalloc(&d_os, P * 4));
  CHECK(hipMalloc(&d_sc, (size_t)P * 8));
  CHECK(hipMalloc(&d_st, slots * 8));
  CHECK(hipMemcpy(d_pd, pd.data(), P, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_pt, pt.data(), P, hipMemcpyHostToDevice));
  CHECK(msh_stamps_set(d_st));
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 10; ++i) CHECK(msh_schedule_batch_device(ctx, P, d_pd, d_pt, d_oi, d_sc, d_os, st));
  CHECK(hipStreamSynchronize(st));
  std::vector<unsigned long long> h(slots);
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipMemset(d_st, 0, slots * 8));
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0, st));
    CHECK(msh_schedule_batch_device(ctx, P, d_pd, d_pt, d_oi, d_sc, d_os, st));
    CHECK(hipEventRecord(e1, st));
    CHECK(hipStreamSynchronize(st));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipMemcpy(h.data(), d_st, slots * 8, hipMemcpyDeviceToHost));
    unsigned long long t_min = ~0ull, t_max = 0;
    std::vector<double> start, pro, scan, merge;
    for (size_t w = 0; w < slots / 4; ++w) {
      const unsigned long long* t = &h[w * 4];
      if (!t[0]) continue;
      t_min = std::min(t_min, t[0]);
      t_max = std::max(t_max, std::max(t[2], t[3]));
    }
    for (size_t w = 0; w < slots / 4; ++w) {
      const unsigned long long* t = &h[w * 4];
      if (!t[0]) continue;
      start.push_back((t[0] - t_min) * 0.01);
      pro.push_back((t[1] - t[0]) * 0.01);
      scan.push_back((t[2] - t[1]) * 0.01);
      if (t[3]) merge.push_back((t[3] - t[2]) * 0.01);
    }
    printf("{\"pods\": %d, \"rep\": %d, \"event_us\": %.2f, \"waves\": %zu, \"span_us\": %.2f, "
           "\"start_us\": [%.2f, %.2f, %.2f, %.2f], \"prologue_us\": [%.2f, %.2f, %.2f], "
           "\"scan_us\": [%.2f, %.2f, %.2f], \"merge_us\": [%.2f, %.2f, %.2f]}\n",
           P, rep, ms * 1e3, start.size(), (t_max - t_min) * 0.01, pct(start, 0.1), pct(start, 0.5), pct(start, 0.9),
           pct(start, 1.0), pct(pro, 0.1), pct(pro, 0.5), pct(pro, 0.9), pct(scan, 0.1), pct(scan, 0.5),
           pct(scan, 0.9), pct(merge, 0.1), pct(merge, 0.5), pct(merge, 0.9));
    fflush(stdout);
  }
  msh_destroy(ctx);
  return 0;
}
