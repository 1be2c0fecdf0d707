// ubench_valu.hip — gfx950 issue-rate microbenchmark for the instructions on the hot path.
// Each wave runs `iters` blocks of 16 instructions of one kind on 8 independent chains
// (inline asm, so the exact instruction is what is timed). Reports wave-instructions per
// cycle per SIMD (full rate for a wave64 VALU op on a SIMD32 = 0.5) at several occupancies.
// Build: hipcc --offload-arch=gfx950 -O3 ubench_valu.hip -o ubench_valu
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define BLOCK16(INS)                                                                    \
  asm volatile(INS " %0, %8, %0\n\t" INS " %1, %8, %1\n\t" INS " %2, %8, %2\n\t" INS  \
               " %3, %8, %3\n\t" INS " %4, %8, %4\n\t" INS " %5, %8, %5\n\t" INS       \
               " %6, %8, %6\n\t" INS " %7, %8, %7\n\t" INS " %0, %8, %0\n\t" INS       \
               " %1, %8, %1\n\t" INS " %2, %8, %2\n\t" INS " %3, %8, %3\n\t" INS       \
               " %4, %8, %4\n\t" INS " %5, %8, %5\n\t" INS " %6, %8, %6\n\t" INS       \
               " %7, %8, %7"                                                           \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), \
                 "+v"(a7)                                                              \
               : "s"(k))

// VOP3 with two VGPR sources + SGPR (sad / min3 forms)
#define BLOCK16_3(INS)                                                                       \
  asm volatile(INS " %0, %0, %8, %1\n\t" INS " %1, %1, %8, %2\n\t" INS " %2, %2, %8, %3\n\t" \
               INS " %3, %3, %8, %4\n\t" INS " %4, %4, %8, %5\n\t" INS " %5, %5, %8, %6\n\t" \
               INS " %6, %6, %8, %7\n\t" INS " %7, %7, %8, %0\n\t" INS " %0, %0, %8, %1\n\t" \
               INS " %1, %1, %8, %2\n\t" INS " %2, %2, %8, %3\n\t" INS " %3, %3, %8, %4\n\t" \
               INS " %4, %4, %8, %5\n\t" INS " %5, %5, %8, %6\n\t" INS " %6, %6, %8, %7\n\t" \
               INS " %7, %7, %8, %0"                                                         \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),      \
                 "+v"(a7)                                                                   \
               : "s"(k))

template <int KIND>
__global__ void kern(uint32_t* out, int iters, uint32_t k) {
  // small non-negative values: finite f16 bit patterns for the pk_minimum3 kind
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
           a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < iters; ++i) {
    if (KIND == 0) BLOCK16("v_add_u32");
    if (KIND == 1) BLOCK16("v_xor_b32");
    if (KIND == 2) BLOCK16("v_min_u32");
    if (KIND == 3) BLOCK16("v_pk_min_u16");
    if (KIND == 4) BLOCK16_3("v_sad_u32");
    if (KIND == 5) BLOCK16_3("v_min3_u32");
    if (KIND == 6) {  // the former IDENT inner pattern: xor then pk_min, 8 chains
      BLOCK16("v_xor_b32");
      BLOCK16("v_pk_min_u16");
    }
    if (KIND == 7) {  // the IDENT inner pattern: two xors per pk_minimum3, 8 chains
      BLOCK16("v_xor_b32");
      BLOCK16("v_xor_b32");
      BLOCK16_3("v_pk_minimum3_f16");
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

int main() {
  const char* names[] = {"v_add_u32", "v_xor_b32", "v_min_u32", "v_pk_min_u16", "v_sad_u32",
                         "v_min3_u32", "xor+pk_min", "2xor+pk_minimum3"};
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const int iters = 20000;
  uint32_t* out;
  hipMalloc(&out, (size_t)cus * 8 * 1024 * sizeof(uint32_t));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int clk_khz = 0;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  for (int kind = 0; kind < 8; ++kind) {
    for (int waves_per_simd : {1, 2, 4, 8}) {
      const int threads = 256;  // 4 waves = 1 per SIMD per block
      const int blocks = cus * waves_per_simd;
      auto launch = [&]() {
        switch (kind) {
          case 0: hipLaunchKernelGGL(kern<0>, dim3(blocks), dim3(threads), 0, 0, out, iters, 3u); break;
          case 1: hipLaunchKernelGGL(kern<1>, dim3(blocks), dim3(threads), 0, 0, out, iters, 3u); break;
          case 2: hipLaunchKernelGGL(kern<2>, dim3(blocks), dim3(threads), 0, 0, out, iters, 3u); break;
          case 3: hipLaunchKernelGGL(kern<3>, dim3(blocks), dim3(threads), 0, 0, out, iters, 3u); break;
          case 4: hipLaunchKernelGGL(kern<4>, dim3(blocks), dim3(threads), 0, 0, out, iters, 3u); break;
          case 5: hipLaunchKernelGGL(kern<5>, dim3(blocks), dim3(threads), 0, 0, out, iters, 3u); break;
          case 6: hipLaunchKernelGGL(kern<6>, dim3(blocks), dim3(threads), 0, 0, out, iters, 3u); break;
          case 7: hipLaunchKernelGGL(kern<7>, dim3(blocks), dim3(threads), 0, 0, out, iters, 3u); break;
        }
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(e0, 0);
      launch();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double instr_per_wave = 16.0 * iters * (kind == 6 ? 2 : kind == 7 ? 3 : 1);
      const double total_wave_instr = instr_per_wave * blocks * 4;
      const double simd_cycles = ms * 1e-3 * 2.4e9;  // nominal 2.4 GHz
      const double ipc_simd = total_wave_instr / (cus * 4) / simd_cycles;
      printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"wave_instr_per_simd_cycle@2.4GHz\": %.4f, "
             "\"lane_ops_per_s\": %.4g}\n",
             names[kind], waves_per_simd, ms, ipc_simd, total_wave_instr * 64 / (ms * 1e-3));
    }
  }
  printf("{\"clock_khz_attr\": %d}\n", clk_khz);
  return 0;
}
