// stream_isolation.hip — which HIP operations on stream A wait for unrelated work queued on
// stream B (both non-blocking streams of one device)? Stream B gets a ~20 ms spin kernel; then each
// candidate operation of a table upload runs on A followed by hipStreamSynchronize(A), and the host
// time of the pair is printed with whether B was still running when it returned.
// Build: hipcc --offload-arch=gfx950 -O2 scripts/stream_isolation.hip -o scripts/stream_isolation
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_));      \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void spin(long long cycles, int* out) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

__global__ void touch(int* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1;
}

int main() {
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  int *d_spin, *d_buf;
  CK(hipMalloc(&d_spin, 1024 * sizeof(int)));
  CK(hipMalloc(&d_buf, 1 << 20));
  unsigned char *h_pin, *h_page = new unsigned char[1 << 20];
  CK(hipHostMalloc(reinterpret_cast<void**>(&h_pin), 1 << 20, hipHostMallocDefault));
  std::memset(h_page, 1, 1 << 20);
  std::memset(h_pin, 1, 1 << 20);
  hipEvent_t done_b;
  CK(hipEventCreateWithFlags(&done_b, hipEventDisableTiming));
  CK(hipDeviceSynchronize());
  const char* names[] = {"kernel", "memcpy_h2d_pinned_10k", "memcpy_h2d_pageable_10k", "memset_async_20k",
                         "memset_d32_async_20k", "memcpy_h2d_pinned_8B", "memcpy_h2d_pageable_8B", "event_sync_only"};
  for (int op = 0; op < 8; ++op) {
    spin<<<8, 64, 0, b>>>(2'400'000LL * 20, d_spin);  // ~20 ms at 2.4 GHz
    CK(hipEventRecord(done_b, b));
    CK(hipStreamSynchronize(a));
    const auto t0 = std::chrono::steady_clock::now();
    switch (op) {
      case 0: touch<<<40, 256, 0, a>>>(d_buf, 10240); break;
      case 1: CK(hipMemcpyAsync(d_buf, h_pin, 10000, hipMemcpyHostToDevice, a)); break;
      case 2: CK(hipMemcpyAsync(d_buf, h_page, 10000, hipMemcpyHostToDevice, a)); break;
      case 3: CK(hipMemsetAsync(d_buf, 0, 20480, a)); break;
      case 4: CK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_buf), 0, 5120, a)); break;
      case 5: CK(hipMemcpyAsync(d_buf, h_pin, 8, hipMemcpyHostToDevice, a)); break;
      case 6: CK(hipMemcpyAsync(d_buf, h_page, 8, hipMemcpyHostToDevice, a)); break;
      default: break;
    }
    CK(hipStreamSynchronize(a));
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    const bool b_running = hipEventQuery(done_b) == hipErrorNotReady;
    std::printf("{\"op\": \"%s\", \"host_us\": %.1f, \"b_still_running\": %s}\n", names[op], us,
                b_running ? "true" : "false");
    CK(hipStreamSynchronize(b));
  }
  CK(hipHostFree(h_pin));
  delete[] h_page;
  CK(hipFree(d_spin));
  CK(hipFree(d_buf));
  return 0;
}
