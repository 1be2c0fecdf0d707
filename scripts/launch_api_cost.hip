// launch_api_cost.hip — host cost of one kernel launch through each HIP launch API on gfx950
// (empty kernel, one workgroup, K launches back to back on one stream): hipLaunchKernelGGL,
// hipLaunchKernel, hipModuleLaunchKernel on a hipFunction_t from hipGetFuncBySymbol, and
// hipExtLaunchKernel. One JSON line per API: submit us per launch and wall us per launch.
// Build: hipcc --offload-arch=gfx950 -O2 scripts/launch_api_cost.hip -o scripts/launch_api_cost
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

struct Args {
  int* p;
  int n;
  long long pad[12];  // a kernel-argument block the size of BatchArgs (~110 bytes)
};

__global__ void empty_kernel(Args a) {
  if (a.p && threadIdx.x == 1024) a.p[0] = a.n;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <typename F>
void measure(const char* name, F launch, hipStream_t s) {
  const int K = 4000;
  for (int i = 0; i < 200; ++i) launch();
  (void)hipStreamSynchronize(s);
  const double t0 = now_us();
  for (int i = 0; i < K; ++i) launch();
  const double t1 = now_us();
  (void)hipStreamSynchronize(s);
  const double t2 = now_us();
  printf("{\"api\": \"%s\", \"submit_us\": %.3f, \"wall_us\": %.3f, \"err\": \"%s\"}\n", name, (t1 - t0) / K,
         (t2 - t0) / K, hipGetErrorName(hipGetLastError()));
}

int main() {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  Args a{};
  measure("hipLaunchKernelGGL", [&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, a); }, s);
  void* kargs[] = {&a};
  measure("hipLaunchKernel", [&] {
    (void)hipLaunchKernel(reinterpret_cast<const void*>(empty_kernel), dim3(1), dim3(64), kargs, 0, s);
  }, s);
  hipFunction_t f = nullptr;
  if (hipGetFuncBySymbol(&f, reinterpret_cast<const void*>(empty_kernel)) == hipSuccess) {
    size_t sz = sizeof(a);
    void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
    measure("hipModuleLaunchKernel(extra)", [&] {
      (void)hipModuleLaunchKernel(f, 1, 1, 1, 64, 1, 1, 0, s, nullptr, cfg);
    }, s);
    measure("hipModuleLaunchKernel(params)", [&] {
      (void)hipModuleLaunchKernel(f, 1, 1, 1, 64, 1, 1, 0, s, kargs, nullptr);
    }, s);
  }
  measure("hipExtLaunchKernel", [&] {
    (void)hipExtLaunchKernel(reinterpret_cast<const void*>(empty_kernel), dim3(1), dim3(64), kargs, 0, s, nullptr,
                             nullptr, 0);
  }, s);
  return 0;
}
