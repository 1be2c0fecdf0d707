// submit_mt.hip — does the HIP launch path scale over host threads? C3 batches submitted through
// msh_schedule_batch_device from T host threads at once, each thread with its own ctx (the ABI's
// one-ctx-per-thread rule), its own stream and its own pod/output buffers; and, for scale, an empty
// kernel launched the same way (one workgroup, and the C3 batch's grid: 1,563 workgroups of 256
// threads), and the batch entry point on a 64-pod batch. One JSON line per (what, T): wall time per
// launch over all threads
// (submit phase, and up to the device synchronize), every thread's launches counted.
// Build: hipcc --offload-arch=gfx950 -O2 -Iinclude scripts/submit_mt.hip -Lmini-kube-scheduler_amd
//        -lminisched_hip -Wl,-rpath,'$ORIGIN/../mini-kube-scheduler_amd' -pthread -o scripts/submit_mt
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <thread>
#include <vector>

#include "minisched_hip.h"

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1024) p[0] = 0;
}
struct Args120 {  // the size of the batch kernel's argument block (msh::BatchArgs)
  int* p;
  uint64_t pad[14];
};
__global__ void empty_kernel_120(Args120 a) {
  if (a.p && threadIdx.x == 1024) a.p[0] = (int)a.pad[3];
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CHECK(x)                                   \
  do {                                             \
    int rc_ = (int)(x);                            \
    if (rc_ != 0) {                                \
      fprintf(stderr, "%s failed: %d\n", #x, rc_); \
      return 1;                                    \
    }                                              \
  } while (0)

struct Lane {
  msh_ctx* ctx = nullptr;
  hipStream_t st = nullptr;
  int8_t* pd = nullptr;
  uint8_t* pt = nullptr;
  int32_t *oi = nullptr, *os = nullptr;
  int64_t* sc = nullptr;
};

int main() {
  const int N = 5000, P = 100000, K = 4000, TMAX = 4;
  std::vector<uint8_t> u(N);
  std::vector<int8_t> d(N), pd(P);
  std::vector<uint8_t> pt(P);
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
  for (int j = 0; j < P; ++j) {
    pd[j] = (int8_t)(rnd() % 100 == 0 ? -1 : rnd() % 10);
    pt[j] = rnd() % 20 == 0;
  }
  std::vector<Lane> lanes(TMAX);
  for (auto& l : lanes) {
    CHECK(msh_create(0, &l.ctx));
    CHECK(msh_upload_nodes(l.ctx, N, u.data(), d.data()));
    CHECK(hipStreamCreateWithFlags(&l.st, hipStreamNonBlocking));
    CHECK(hipMalloc(&l.pd, P));
    CHECK(hipMalloc(&l.pt, P));
    CHECK(hipMalloc(&l.oi, P * 4));
    CHECK(hipMalloc(&l.os, P * 4));
    CHECK(hipMalloc(&l.sc, P * 8));
    CHECK(hipMemcpy(l.pd, pd.data(), P, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(l.pt, pt.data(), P, hipMemcpyHostToDevice));
  }
  const char* names[5] = {"empty kernel hipLaunchKernelGGL", "msh_schedule_batch_device C3",
                          "empty kernel, C3 grid (1563 x 256)", "msh_schedule_batch_device 64 pods",
                          "empty kernel, 120-byte arguments"};
  for (int what = 0; what < 5; ++what) {
    for (int T = 1; T <= TMAX; ++T) {
      for (int rep = 0; rep < 2; ++rep) {
        std::atomic<int> ready{0}, go{0}, bad{0};
        std::vector<double> t_end(T);
        auto body = [&](int t) {
          Lane& l = lanes[t];
          const int k = K / T;
          auto launch = [&]() {
            if (what == 0)
              hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, l.st, nullptr);
            else if (what == 2)
              hipLaunchKernelGGL(empty_kernel, dim3((P + 63) / 64), dim3(256), 0, l.st, nullptr);
            else if (what == 4)
              hipLaunchKernelGGL(empty_kernel_120, dim3(1), dim3(64), 0, l.st, Args120{});
            else if (msh_schedule_batch_device(l.ctx, what == 1 ? P : 64, l.pd, l.pt, l.oi, l.sc, l.os, l.st))
              bad = 1;
          };
          for (int i = 0; i < 20; ++i) launch();  // warm the thread's own launch path
          if (hipStreamSynchronize(l.st)) bad = 1;
          ready.fetch_add(1);
          while (!go.load(std::memory_order_acquire)) {
          }
          for (int i = 0; i < k; ++i) launch();
          t_end[t] = now_us();
        };
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) th.emplace_back(body, t);
        while (ready.load() < T) {
        }
        const double t0 = now_us();
        go.store(1, std::memory_order_release);
        for (auto& h : th) h.join();
        double t1 = 0;
        for (double v : t_end) t1 = v > t1 ? v : t1;
        CHECK(hipDeviceSynchronize());
        const double t2 = now_us();
        if (bad) {
          fprintf(stderr, "a launch failed\n");
          return 1;
        }
        const double launches = (double)(K / T) * T;
        printf("{\"what\": \"%s\", \"threads\": %d, \"rep\": %d, \"submit_us_per_launch\": %.3f, "
               "\"wall_us_per_launch\": %.3f}\n",
               names[what], T, rep,
               (t1 - t0) / launches, (t2 - t0) / launches);
        fflush(stdout);
      }
    }
  }
  for (auto& l : lanes) {
    hipFree(l.pd);
    hipFree(l.pt);
    hipFree(l.oi);
    hipFree(l.os);
    hipFree(l.sc);
    hipStreamDestroy(l.st);
    msh_destroy(l.ctx);
  }
  return 0;
}
