// launch_floor.hip — the fixed cost of a bench region on MI355X, from C: device synchronize, clock,
// ONE launch, device synchronize, clock (the shape of the driver's K = 20 region, which is one
// persistent launch), for kernels that do nothing:
//   1wg       one workgroup of 64 threads, 8-byte arguments
//   grid      2,048 workgroups of 256 threads with 17 KB of dynamic LDS (the persistent batch
//             kernel's grid at C3), 8-byte arguments
//   grid_arg  the same with a 1,928-byte argument block (the multi-batch kernel's)
// 200 repetitions each after 1 ms idle; median / p10 / p90 in microseconds, one JSON line per case.
//   hipcc --offload-arch=gfx950 -O3 scripts/launch_floor.hip -o scripts/launch_floor
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                       \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
      return 1;                                                        \
    }                                                                  \
  } while (0)

struct Big {
  unsigned long long w[241];  // 1,928 bytes
};

__global__ void k_small(int* p) {
  if (p && threadIdx.x == 1000000) p[0] = 1;
}
__global__ void k_big(Big b) {
  extern __shared__ int s[];
  if (threadIdx.x == 1000000) s[0] = (int)b.w[3];
}

template <typename F>
static void region(const char* name, F launch) {
  std::vector<double> us;
  for (int rep = 0; rep < 220; ++rep) {
    (void)hipDeviceSynchronize();
    const auto idle = std::chrono::steady_clock::now() + std::chrono::microseconds(1000);
    while (std::chrono::steady_clock::now() < idle) {
    }
    const auto t0 = std::chrono::steady_clock::now();
    launch();
    (void)hipDeviceSynchronize();
    if (rep >= 20) us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  std::sort(us.begin(), us.end());
  printf("{\"case\": \"%s\", \"region_us\": [%.2f, %.2f, %.2f]}\n", name, us[us.size() / 10], us[us.size() / 2],
         us[us.size() * 9 / 10]);
}

int main() {
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  Big b{};
  region("1wg", [&] { hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, st, nullptr); });
  region("grid", [&] { hipLaunchKernelGGL(k_small, dim3(2048), dim3(256), 17 * 1024, st, nullptr); });
  region("grid_arg", [&] { hipLaunchKernelGGL(k_big, dim3(2048), dim3(256), 17 * 1024, st, b); });
  region("grid_arg_null_stream", [&] { hipLaunchKernelGGL(k_big, dim3(2048), dim3(256), 17 * 1024, 0, b); });
  return 0;
}
