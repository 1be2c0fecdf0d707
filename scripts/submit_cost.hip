// submit_cost.hip — host-side cost of one C3 batch submission through the C ABI, with no Python in
// between (what a cgo caller pays): an empty kernel's hipLaunchKernelGGL for scale, then
// msh_schedule_batch_device (submit time per call, and completed calls per second with 1 and 2
// streams in flight), then msh_schedule_batch on msh_host_alloc buffers (one synchronous call).
// One JSON line per measurement.
// Build: hipcc --offload-arch=gfx950 -O2 -Iinclude scripts/submit_cost.hip -Lmini-kube-scheduler_amd
//        -lminisched_hip -Wl,-rpath,'$ORIGIN/../mini-kube-scheduler_amd' -o scripts/submit_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "minisched_hip.h"

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1024) p[0] = 0;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CHECK(x)                                                 \
  do {                                                           \
    int rc_ = (int)(x);                                          \
    if (rc_ != 0) {                                              \
      fprintf(stderr, "%s failed: %d\n", #x, rc_);               \
      return 1;                                                  \
    }                                                            \
  } while (0)

int main() {
  const int N = 5000, P = 100000, K = 2000;
  hipStream_t st[2];
  CHECK(hipStreamCreateWithFlags(&st[0], hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&st[1], hipStreamNonBlocking));
  {  // empty kernel
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st[0], nullptr);
    CHECK(hipStreamSynchronize(st[0]));
    const double t0 = now_us();
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st[0], nullptr);
    const double t1 = now_us();
    CHECK(hipStreamSynchronize(st[0]));
    const double t2 = now_us();
    printf("{\"what\": \"empty kernel hipLaunchKernelGGL\", \"submit_us\": %.3f, \"wall_us\": %.3f}\n",
           (t1 - t0) / K, (t2 - t0) / K);
  }
  msh_ctx* ctx = nullptr;
  CHECK(msh_create(0, &ctx));
  // the default plugin set: the reference's (filter NodeUnschedulable, NodeNumber w=1, NONE)
  std::vector<uint8_t> u(N);
  std::vector<int8_t> d(N);
  uint64_t x = 0x6d696e69;
  auto rnd = [&]() {
    x += 0x9e3779b97f4a7c15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  };
  for (int i = 0; i < N; ++i) {
    u[i] = rnd() % 10 == 0;
    d[i] = (int8_t)(i % 10);
  }
  CHECK(msh_upload_nodes(ctx, N, u.data(), d.data()));
  std::vector<int8_t> pd(P);
  std::vector<uint8_t> pt(P);
  for (int j = 0; j < P; ++j) {
    pd[j] = (int8_t)(rnd() % 100 == 0 ? -1 : rnd() % 10);
    pt[j] = rnd() % 20 == 0;
  }
  int8_t* d_pd[2];
  uint8_t* d_pt[2];
  int32_t *d_oi[2], *d_os[2];
  int64_t* d_sc[2];
  for (int b = 0; b < 2; ++b) {
    CHECK(hipMalloc(&d_pd[b], P));
    CHECK(hipMalloc(&d_pt[b], P));
    CHECK(hipMalloc(&d_oi[b], P * 4));
    CHECK(hipMalloc(&d_os[b], P * 4));
    CHECK(hipMalloc(&d_sc[b], P * 8));
    CHECK(hipMemcpy(d_pd[b], pd.data(), P, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_pt[b], pt.data(), P, hipMemcpyHostToDevice));
  }
  for (int ns = 1; ns <= 2; ++ns) {
    for (int i = 0; i < 50; ++i)
      CHECK(msh_schedule_batch_device(ctx, P, d_pd[i % ns], d_pt[i % ns], d_oi[i % ns], d_sc[i % ns], d_os[i % ns],
                                      st[i % ns]));
    CHECK(hipDeviceSynchronize());
    const double t0 = now_us();
    for (int i = 0; i < K; ++i)
      CHECK(msh_schedule_batch_device(ctx, P, d_pd[i % ns], d_pt[i % ns], d_oi[i % ns], d_sc[i % ns], d_os[i % ns],
                                      st[i % ns]));
    const double t1 = now_us();
    CHECK(hipDeviceSynchronize());
    const double t2 = now_us();
    printf("{\"what\": \"msh_schedule_batch_device C3\", \"streams\": %d, \"submit_us\": %.3f, \"wall_us_per_batch\": %.3f}\n",
           ns, (t1 - t0) / K, (t2 - t0) / K);
  }
  {  // synchronous host-buffer call on page-locked buffers
    void *hpd, *hpt, *hoi, *hsc, *hos;
    CHECK(msh_host_alloc(P, &hpd));
    CHECK(msh_host_alloc(P, &hpt));
    CHECK(msh_host_alloc((size_t)P * 4, &hoi));
    CHECK(msh_host_alloc((size_t)P * 8, &hsc));
    CHECK(msh_host_alloc((size_t)P * 4, &hos));
    memcpy(hpd, pd.data(), P);
    memcpy(hpt, pt.data(), P);
    const int KH = 500;
    std::vector<double> ts;
    for (int i = 0; i < KH + 20; ++i) {
      const double t0 = now_us();
      CHECK(msh_schedule_batch(ctx, P, (int8_t*)hpd, (uint8_t*)hpt, (int32_t*)hoi, (int64_t*)hsc, (int32_t*)hos));
      if (i >= 20) ts.push_back(now_us() - t0);
    }
    std::sort(ts.begin(), ts.end());
    printf("{\"what\": \"msh_schedule_batch C3 pinned\", \"us_median\": %.3f, \"us_min\": %.3f}\n", ts[ts.size() / 2],
           ts[0]);
    std::vector<int32_t> poi(P), pos(P);
    std::vector<int64_t> psc(P);
    ts.clear();
    for (int i = 0; i < KH + 20; ++i) {
      const double t0 = now_us();
      CHECK(msh_schedule_batch(ctx, P, pd.data(), pt.data(), poi.data(), psc.data(), pos.data()));
      if (i >= 20) ts.push_back(now_us() - t0);
    }
    std::sort(ts.begin(), ts.end());
    printf("{\"what\": \"msh_schedule_batch C3 pageable\", \"us_median\": %.3f, \"us_min\": %.3f}\n", ts[ts.size() / 2],
           ts[0]);
    for (void* p : {hpd, hpt, hoi, hsc, hos}) msh_host_free(p);
  }
  msh_destroy(ctx);
  return 0;
}
