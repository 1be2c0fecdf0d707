// ubench_bitop3.hip — gfx950 issue rate of bits_kernel's scan instruction mix (msh_kernels.hip):
// per 32-node word and pod, v_and_b32 (SGPR, VGPR) + 4 x v_bitop3_b32 (VGPR, SGPR, VGPR), and one
// v_bitop3_b32 (3 VGPR) AND per two words; 8 independent word chains per block (as the unrolled
// group). Also each form alone. Reports wave-instructions per SIMD-cycle at 2.4 GHz nominal, at
// 1 / 2 / 4 / 8 waves per SIMD, one JSON line per (op, occupancy).
// Build: hipcc --offload-arch=gfx950 -O3 ubench_bitop3.hip -o ubench_bitop3
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

// one word: t = (X & nT); t = t | (Dk ^ Pk) for k = 0..3
#define WORD(T)                                              \
  "v_and_b32 " T ", %[x], %[nt]\n\t"                         \
  "v_bitop3_b32 " T ", " T ", %[d0], %[p0] bitop3:0xf6\n\t"  \
  "v_bitop3_b32 " T ", " T ", %[d1], %[p1] bitop3:0xf6\n\t"  \
  "v_bitop3_b32 " T ", " T ", %[d2], %[p2] bitop3:0xf6\n\t"  \
  "v_bitop3_b32 " T ", " T ", %[d3], %[p3] bitop3:0xf6\n\t"
#define AND3(A, X, Y) "v_bitop3_b32 " A ", " A ", " X ", " Y " bitop3:0x80\n\t"
#define MIX                                                                                   \
  WORD("%[t0]") WORD("%[t1]") WORD("%[t2]") WORD("%[t3]") WORD("%[t4]") WORD("%[t5]")         \
  WORD("%[t6]") WORD("%[t7]") AND3("%[a0]", "%[t0]", "%[t1]") AND3("%[a1]", "%[t2]", "%[t3]") \
  AND3("%[a2]", "%[t4]", "%[t5]") AND3("%[a3]", "%[t6]", "%[t7]")
#define B3ONLY(T) "v_bitop3_b32 " T ", " T ", %[d0], %[p0] bitop3:0xf6\n\t"
#define B3BLOCK B3ONLY("%[t0]") B3ONLY("%[t1]") B3ONLY("%[t2]") B3ONLY("%[t3]") B3ONLY("%[t4]") \
  B3ONLY("%[t5]") B3ONLY("%[t6]") B3ONLY("%[t7]")
#define ANDONLY(T) "v_and_b32 " T ", %[x], " T "\n\t"
#define ANDBLOCK ANDONLY("%[t0]") ANDONLY("%[t1]") ANDONLY("%[t2]") ANDONLY("%[t3]") ANDONLY("%[t4]") \
  ANDONLY("%[t5]") ANDONLY("%[t6]") ANDONLY("%[t7]")

#define OPS                                                                                        \
  [t0] "+v"(t0), [t1] "+v"(t1), [t2] "+v"(t2), [t3] "+v"(t3), [t4] "+v"(t4), [t5] "+v"(t5),       \
      [t6] "+v"(t6), [t7] "+v"(t7), [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3)
#define INS                                                                                     \
  [x] "s"(x), [d0] "s"(d0), [d1] "s"(d1), [d2] "s"(d2), [d3] "s"(d3), [nt] "v"(nt), [p0] "v"(p0), \
      [p1] "v"(p1), [p2] "v"(p2), [p3] "v"(p3)

struct Kind {
  const char* name;
  int instr_per_iter;
};
static const Kind kinds[] = {{"bits scan mix", 44}, {"v_bitop3_b32 vsv", 8}, {"v_and_b32 sv", 8}};

template <int KIND>
__global__ __launch_bounds__(256) void kern(uint32_t* out, int iters, uint32_t x, uint32_t d0, uint32_t d1,
                                            uint32_t d2, uint32_t d3) {
  uint32_t t0 = threadIdx.x, t1 = t0 * 3, t2 = t0 * 5, t3 = t0 * 7, t4 = t0 ^ 9, t5 = t0 ^ 11, t6 = t0 + 13,
           t7 = t0 + 15, a0 = ~0u, a1 = ~0u, a2 = ~0u, a3 = ~0u;
  const uint32_t nt = 0u - (threadIdx.x & 1), p0 = 0u - ((threadIdx.x >> 1) & 1), p1 = 0u - ((threadIdx.x >> 2) & 1),
                 p2 = 0u - ((threadIdx.x >> 3) & 1), p3 = 0u - ((threadIdx.x >> 4) & 1);
  for (int i = 0; i < iters; ++i) {
    if (KIND == 0) asm volatile(MIX : OPS : INS);
    if (KIND == 1) asm volatile(B3BLOCK : OPS : INS);
    if (KIND == 2) asm volatile(ANDBLOCK : OPS : INS);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = t0 ^ t1 ^ t2 ^ t3 ^ t4 ^ t5 ^ t6 ^ t7 ^ a0 ^ a1 ^ a2 ^ a3;
}

template <int KIND>
void run(uint32_t* d_out, int cus) {
  const int iters = 4000;
  for (int wps : {1, 2, 4, 8}) {
    const int blocks = cus * wps;  // 256-thread blocks: one wave per SIMD per block
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern<KIND>, dim3(blocks), dim3(256), 0, 0, d_out, 10, 1u, 2u, 3u, 4u, 5u);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(kern<KIND>, dim3(blocks), dim3(256), 0, 0, d_out, iters, 1u, 2u, 3u, 4u, 5u);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double wave_instr = (double)blocks * 4 * iters * kinds[KIND].instr_per_iter;
    const double per_simd_cycle = wave_instr / (cus * 4.0) / (ms * 1e-3 * 2.4e9);
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"wave_instr_per_simd_cycle@2.4GHz\": %.4f}\n",
           kinds[KIND].name, wps, ms, per_simd_cycle);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
  }
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* d_out = nullptr;
  hipMalloc(&d_out, (size_t)cus * 8 * 256 * sizeof(uint32_t));
  run<0>(d_out, cus);
  run<1>(d_out, cus);
  run<2>(d_out, cus);
  hipFree(d_out);
  return 0;
}
