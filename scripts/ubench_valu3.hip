// ubench_valu3.hip — gfx950 issue rate of all-VGPR operand forms (VOP2 vv, VOP3 vvv, VOP3P) vs the
// SGPR-operand forms: ubench_valu2 found v_sub_f32 v,v at ~0.38 wave-instr/SIMD-cycle vs ~0.21 with an
// SGPR source. Each wave runs `iters` blocks of 16 instructions on 8
// independent chains (inline asm). Reports wave-instructions per SIMD-cycle at 2.4 GHz.
// Build: hipcc --offload-arch=gfx950 -O3 ubench_valu3.hip -o ubench_valu3
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CH8(F) F(0, 1) F(1, 2) F(2, 3) F(3, 4) F(4, 5) F(5, 6) F(6, 7) F(7, 0)
#define OUTS "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)

// dst = op(k, dst)  (VOP2, SGPR first source)
#define V2(INS) INS " %0, %8, %0\n\t" INS " %1, %8, %1\n\t" INS " %2, %8, %2\n\t" INS " %3, %8, %3\n\t" \
                INS " %4, %8, %4\n\t" INS " %5, %8, %5\n\t" INS " %6, %8, %6\n\t" INS " %7, %8, %7\n\t"
// dst = op(next, dst)  (VOP2, two VGPR sources)
#define VV2(INS) INS " %0, %1, %0\n\t" INS " %1, %2, %1\n\t" INS " %2, %3, %2\n\t" INS " %3, %4, %3\n\t" \
                 INS " %4, %5, %4\n\t" INS " %5, %6, %5\n\t" INS " %6, %7, %6\n\t" INS " %7, %0, %7\n\t"
// dst = op(dst, next, k) (VOP3, two VGPR + one SGPR)
#define V3(INS) INS " %0, %0, %1, %8\n\t" INS " %1, %1, %2, %8\n\t" INS " %2, %2, %3, %8\n\t" \
                INS " %3, %3, %4, %8\n\t" INS " %4, %4, %5, %8\n\t" INS " %5, %5, %6, %8\n\t" \
                INS " %6, %6, %7, %8\n\t" INS " %7, %7, %0, %8\n\t"
// dst = op(dst, |next|, |next2|) (VOP3, three VGPR, abs modifiers: the fp32 min3 scan form)
#define V3ABS(INS) INS " %0, %0, |%1|, |%2|\n\t" INS " %1, %1, |%2|, |%3|\n\t" INS " %2, %2, |%3|, |%4|\n\t" \
                   INS " %3, %3, |%4|, |%5|\n\t" INS " %4, %4, |%5|, |%6|\n\t" INS " %5, %5, |%6|, |%7|\n\t" \
                   INS " %6, %6, |%7|, |%0|\n\t" INS " %7, %7, |%0|, |%1|\n\t"
// dst = op(dst, next, next2) three VGPR (the v_pk_minimum3_f16 scan form)
#define V3V(INS) INS " %0, %0, %1, %2\n\t" INS " %1, %1, %2, %3\n\t" INS " %2, %2, %3, %4\n\t" \
                 INS " %3, %3, %4, %5\n\t" INS " %4, %4, %5, %6\n\t" INS " %5, %5, %6, %7\n\t" \
                 INS " %6, %6, %7, %0\n\t" INS " %7, %7, %0, %1\n\t"

#define RUN32(BODY) asm volatile(BODY BODY : OUTS : "s"(k))
#define RUN64(BODY) asm volatile(BODY BODY : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) : "s"(k64))

struct Kind {
  const char* name;
  int instr_per_block;
};
static const Kind kinds[] = {
    {"v_xor_b32 vv", 16},
    {"v_xor_b32 sv", 16},
    {"v_add_u32 vv", 16},
    {"v_min_u32 vv", 16},
    {"v_and_b32 vv", 16},
    {"v_sub_f32 vv", 16},
    {"v_min_f32 vv", 16},
    {"v_pk_min_u16 vv", 16},
    {"v_pk_min_f16 vv", 16},
    {"v_min3_u32 vvv", 16},
    {"v_min3_f32 vvv", 16},
    {"v_pk_minimum3_f16 vvv", 16},
    {"v_xor_b32 vv x2 + v_pk_minimum3_f16", 24},
    {"v_xor_b32 vv + v_pk_min_u16 vv", 16},
    {"v_sub_f32 vv + v_min_f32 vv", 16},
    {"v_xor_b32 vv x2 + v_min3_u32 vvv", 24},
    {"v_xor_b32 vv x2 + v_min3_f32 vvv", 24},
    {"v_sub_f32 vv x2 + v_min3_f32 |abs|", 24},
    {"v_xor_b32 e64 vv", 16},
    {"v_pk_fma_f32 vvv", 16},
};
constexpr int NKINDS = sizeof(kinds) / sizeof(kinds[0]);

template <int KIND>
__global__ void kern(uint32_t* out, int iters, uint32_t k) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7;
  uint64_t b0 = a0, b1 = a1, b2 = a2, b3 = a3, b4 = a4, b5 = a5, b6 = a6, b7 = a7;
  for (int i = 0; i < iters; ++i) {
    if (KIND == 0) { RUN32(VV2("v_xor_b32")); }
    if (KIND == 1) { RUN32(V2("v_xor_b32")); }
    if (KIND == 2) { RUN32(VV2("v_add_u32")); }
    if (KIND == 3) { RUN32(VV2("v_min_u32")); }
    if (KIND == 4) { RUN32(VV2("v_and_b32")); }
    if (KIND == 5) { RUN32(VV2("v_sub_f32")); }
    if (KIND == 6) { RUN32(VV2("v_min_f32")); }
    if (KIND == 7) { RUN32(VV2("v_pk_min_u16")); }
    if (KIND == 8) { RUN32(VV2("v_pk_min_f16")); }
    if (KIND == 9) { RUN32(V3V("v_min3_u32")); }
    if (KIND == 10) { RUN32(V3V("v_min3_f32")); }
    if (KIND == 11) { RUN32(V3V("v_pk_minimum3_f16")); }
    if (KIND == 12) { asm volatile(VV2("v_xor_b32") VV2("v_xor_b32") V3V("v_pk_minimum3_f16") : OUTS : "s"(k)); }
    if (KIND == 13) { asm volatile(VV2("v_xor_b32") VV2("v_pk_min_u16") : OUTS : "s"(k)); }
    if (KIND == 14) { asm volatile(VV2("v_sub_f32") VV2("v_min_f32") : OUTS : "s"(k)); }
    if (KIND == 15) { asm volatile(VV2("v_xor_b32") VV2("v_xor_b32") V3V("v_min3_u32") : OUTS : "s"(k)); }
    if (KIND == 16) { asm volatile(VV2("v_xor_b32") VV2("v_xor_b32") V3V("v_min3_f32") : OUTS : "s"(k)); }
    if (KIND == 17) { asm volatile(VV2("v_sub_f32") VV2("v_sub_f32") V3ABS("v_min3_f32") : OUTS : "s"(k)); }
    if (KIND == 18) { RUN32(VV2("v_xor_b32_e64")); }
    if (KIND == 19) { asm volatile(
          "v_pk_fma_f32 %0, %1, %0, %2\n\tv_pk_fma_f32 %1, %2, %1, %3\n\tv_pk_fma_f32 %2, %3, %2, %4\n\tv_pk_fma_f32 %3, %4, %3, %5\n\t"
          "v_pk_fma_f32 %4, %5, %4, %6\n\tv_pk_fma_f32 %5, %6, %5, %7\n\tv_pk_fma_f32 %6, %7, %6, %0\n\tv_pk_fma_f32 %7, %0, %7, %1\n\t"
          "v_pk_fma_f32 %0, %1, %0, %2\n\tv_pk_fma_f32 %1, %2, %1, %3\n\tv_pk_fma_f32 %2, %3, %2, %4\n\tv_pk_fma_f32 %3, %4, %3, %5\n\t"
          "v_pk_fma_f32 %4, %5, %4, %6\n\tv_pk_fma_f32 %5, %6, %5, %7\n\tv_pk_fma_f32 %6, %7, %6, %0\n\tv_pk_fma_f32 %7, %0, %7, %1\n\t"
          : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7)); }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] =
      a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(b0 ^ b1 ^ b2 ^ b3 ^ b4 ^ b5 ^ b6 ^ b7);
}
template <int K>
void launch(int kind, int blocks, uint32_t* out, int iters) {
  if (kind == K) hipLaunchKernelGGL(kern<K>, dim3(blocks), dim3(256), 0, 0, out, iters, 0x3c003c00u);
  if constexpr (K + 1 < NKINDS) launch<K + 1>(kind, blocks, out, iters);
}

int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const int iters = 40000;
  uint32_t* out;
  hipMalloc(&out, (size_t)cus * 8 * 1024 * sizeof(uint32_t));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int kind = 0; kind < NKINDS; ++kind) {
    for (int wps : {2, 4, 8}) {
      const int blocks = cus * wps;  // 256 threads = 1 wave per SIMD per block
      launch<0>(kind, blocks, out, iters);
      hipDeviceSynchronize();
      hipEventRecord(e0, 0);
      launch<0>(kind, blocks, out, iters);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const int per_iter = kinds[kind].instr_per_block;
      const double wave_instr = (double)per_iter * iters * blocks * 4;
      const double ipc = wave_instr / (cus * 4) / (ms * 1e-3 * 2.4e9);
      printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"wave_instr_per_simd_cycle@2.4GHz\": %.4f}\n",
             kinds[kind].name, wps, ms, ipc);
    }
  }
  return 0;
}
