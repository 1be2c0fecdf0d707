// ubench_valu2.hip — gfx950 issue rate of FP32 / packed-FP32 / packed-16 VALU forms next to the
// integer forms of ubench_valu.hip: is a wave64 VALU instruction 2 cycles on a SIMD32 (guide) for
// some opcode classes and 4 for others? Each wave runs `iters` blocks of 16 instructions on 8
// independent chains (inline asm). Reports wave-instructions per SIMD-cycle at 2.4 GHz.
// Build: hipcc --offload-arch=gfx950 -O3 ubench_valu2.hip -o ubench_valu2
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
    {"v_xor_b32", 16},           // 0 integer reference
    {"v_add_f32", 16},           // 1
    {"v_min_f32", 16},           // 2
    {"v_fma_f32", 16},           // 3
    {"v_min3_f32", 16},          // 4
    {"v_min3_f32|abs|", 16},     // 5
    {"v_pk_add_f32", 16},        // 6 (64-bit operand pairs)
    {"v_pk_fma_f32", 16},        // 7
    {"v_pk_add_f16", 16},        // 8
    {"v_pk_min_f16", 16},        // 9
    {"v_sub_f32+v_min3_f32|abs|", 24},  // 10: 16 subs + 8 min3 (the fp32 scan form)
    {"v_pk_add_f32+v_min3_f32|abs|", 24},  // 11: 8 pk_add (16 subs) + 16 min3? see body
    {"v_mov_b32", 16},           // 12
    {"v_pk_minimum3_f16", 16},   // 13
    {"v_xor_b32+v_min3_f32", 32},  // 14 int and fp32 interleaved 1:1
    {"v_sub_f32", 16},             // 15
    {"v_add_f32+v_min3_f32|abs|", 24},   // 16
    {"v_sub_f32+v_min3_f32", 24},        // 17
    {"v_xor_b32+v_min3_f32|abs|", 24},   // 18
    {"v_sub_f32+v_pk_minimum3_f16", 24}, // 19
    {"v_xor_b32+v_pk_minimum3_f16", 24}, // 20
    {"v_sub_u32+v_min3_u32", 24},        // 21
    {"v_sub_f32(vv)", 16},               // 22 two VGPR sources
    {"v_sub_f32+v_min3_f32|abs| (again)", 24},  // 23 = kind 10
};
constexpr int NKINDS = sizeof(kinds) / sizeof(kinds[0]);

template <int KIND>
__global__ void kern(uint32_t* out, int iters, uint32_t k) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7;
  uint64_t b0 = a0, b1 = a1, b2 = a2, b3 = a3, b4 = a4, b5 = a5, b6 = a6, b7 = a7;
  const uint64_t k64 = ((uint64_t)k << 32) | k;
  for (int i = 0; i < iters; ++i) {
    if (KIND == 0) RUN32(V2("v_xor_b32"));
    if (KIND == 1) RUN32(V2("v_add_f32"));
    if (KIND == 2) RUN32(V2("v_min_f32"));
    if (KIND == 3) RUN32(V3("v_fma_f32"));
    if (KIND == 4) RUN32(V3("v_min3_f32"));
    if (KIND == 5) RUN32(V3ABS("v_min3_f32"));
    if (KIND == 6) {
      asm volatile(
          "v_pk_add_f32 %0, %8, %0\n\tv_pk_add_f32 %1, %8, %1\n\tv_pk_add_f32 %2, %8, %2\n\tv_pk_add_f32 %3, %8, %3\n\t"
          "v_pk_add_f32 %4, %8, %4\n\tv_pk_add_f32 %5, %8, %5\n\tv_pk_add_f32 %6, %8, %6\n\tv_pk_add_f32 %7, %8, %7\n\t"
          "v_pk_add_f32 %0, %8, %0\n\tv_pk_add_f32 %1, %8, %1\n\tv_pk_add_f32 %2, %8, %2\n\tv_pk_add_f32 %3, %8, %3\n\t"
          "v_pk_add_f32 %4, %8, %4\n\tv_pk_add_f32 %5, %8, %5\n\tv_pk_add_f32 %6, %8, %6\n\tv_pk_add_f32 %7, %8, %7\n\t"
          : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7)
          : "s"(k64));
    }
    if (KIND == 7) {
      asm volatile(
          "v_pk_fma_f32 %0, %8, %0, %1\n\tv_pk_fma_f32 %1, %8, %1, %2\n\tv_pk_fma_f32 %2, %8, %2, %3\n\tv_pk_fma_f32 %3, %8, %3, %4\n\t"
          "v_pk_fma_f32 %4, %8, %4, %5\n\tv_pk_fma_f32 %5, %8, %5, %6\n\tv_pk_fma_f32 %6, %8, %6, %7\n\tv_pk_fma_f32 %7, %8, %7, %0\n\t"
          "v_pk_fma_f32 %0, %8, %0, %1\n\tv_pk_fma_f32 %1, %8, %1, %2\n\tv_pk_fma_f32 %2, %8, %2, %3\n\tv_pk_fma_f32 %3, %8, %3, %4\n\t"
          "v_pk_fma_f32 %4, %8, %4, %5\n\tv_pk_fma_f32 %5, %8, %5, %6\n\tv_pk_fma_f32 %6, %8, %6, %7\n\tv_pk_fma_f32 %7, %8, %7, %0\n\t"
          : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7)
          : "s"(k64));
    }
    if (KIND == 8) RUN32(V2("v_pk_add_f16"));
    if (KIND == 9) RUN32(V2("v_pk_min_f16"));
    if (KIND == 10) {
      asm volatile(V2("v_sub_f32") V2("v_sub_f32") V3ABS("v_min3_f32") : OUTS : "s"(k));
    }
    if (KIND == 11) {
      // 8 v_pk_add_f32 (on the 64-bit chains) + 16 v_min3_f32 |abs| on the 32-bit chains
      asm volatile(
          "v_pk_add_f32 %0, %8, %0\n\tv_pk_add_f32 %1, %8, %1\n\tv_pk_add_f32 %2, %8, %2\n\tv_pk_add_f32 %3, %8, %3\n\t"
          "v_pk_add_f32 %4, %8, %4\n\tv_pk_add_f32 %5, %8, %5\n\tv_pk_add_f32 %6, %8, %6\n\tv_pk_add_f32 %7, %8, %7\n\t"
          : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7)
          : "s"(k64));
      RUN32(V3ABS("v_min3_f32"));
    }
    if (KIND == 12) {
      asm volatile(
          "v_mov_b32 %0, %8\n\tv_mov_b32 %1, %8\n\tv_mov_b32 %2, %8\n\tv_mov_b32 %3, %8\n\t"
          "v_mov_b32 %4, %8\n\tv_mov_b32 %5, %8\n\tv_mov_b32 %6, %8\n\tv_mov_b32 %7, %8\n\t"
          "v_mov_b32 %0, %8\n\tv_mov_b32 %1, %8\n\tv_mov_b32 %2, %8\n\tv_mov_b32 %3, %8\n\t"
          "v_mov_b32 %4, %8\n\tv_mov_b32 %5, %8\n\tv_mov_b32 %6, %8\n\tv_mov_b32 %7, %8\n\t"
          : OUTS : "s"(k));
    }
    if (KIND == 13) RUN32(V3V("v_pk_minimum3_f16"));
    if (KIND == 15) RUN32(V2("v_sub_f32"));
    if (KIND == 16) asm volatile(V2("v_add_f32") V2("v_add_f32") V3ABS("v_min3_f32") : OUTS : "s"(k));
    if (KIND == 17) asm volatile(V2("v_sub_f32") V2("v_sub_f32") V3V("v_min3_f32") : OUTS : "s"(k));
    if (KIND == 18) asm volatile(V2("v_xor_b32") V2("v_xor_b32") V3ABS("v_min3_f32") : OUTS : "s"(k));
    if (KIND == 19) asm volatile(V2("v_sub_f32") V2("v_sub_f32") V3V("v_pk_minimum3_f16") : OUTS : "s"(k));
    if (KIND == 20) asm volatile(V2("v_xor_b32") V2("v_xor_b32") V3V("v_pk_minimum3_f16") : OUTS : "s"(k));
    if (KIND == 21) asm volatile(V2("v_sub_u32") V2("v_sub_u32") V3V("v_min3_u32") : OUTS : "s"(k));
    if (KIND == 22) RUN32(VV2("v_sub_f32"));
    if (KIND == 23) asm volatile(V2("v_sub_f32") V2("v_sub_f32") V3ABS("v_min3_f32") : OUTS : "s"(k));
    if (KIND == 14) {
      RUN32(V2("v_xor_b32"));
      RUN32(V3("v_min3_f32"));
    }
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
    for (int wps : {1, 2, 4, 8}) {
      const int blocks = cus * wps;  // 256 threads = 1 wave per SIMD per block
      launch<0>(kind, blocks, out, iters);
      hipDeviceSynchronize();
      hipEventRecord(e0, 0);
      launch<0>(kind, blocks, out, iters);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      // every kind's asm block is issued twice per iteration where RUN32/RUN64 double BODY
      int per_iter = kinds[kind].instr_per_block;
      if (kind <= 5 || kind == 8 || kind == 9 || kind == 12 || kind == 13) per_iter = 16;
      const double wave_instr = (double)per_iter * iters * blocks * 4;
      const double ipc = wave_instr / (cus * 4) / (ms * 1e-3 * 2.4e9);
      printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"wave_instr_per_simd_cycle@2.4GHz\": %.4f}\n",
             kinds[kind].name, wps, ms, ipc);
    }
  }
  return 0;
}
