// ubench_valu_r4.hip — what sets the wave64 integer VALU issue rate on MI355X (gfx950). Round 3's
// ubench_valu_peak.hip found v_bitop3_b32 with three VGPR operands and v_add_u32 at ~0.4 wave64
// instructions per SIMD-cycle but v_bitop3 with an SGPR operand, v_or3, v_min_u32 and v_and_b32 at
// ~0.21. The forms there differ in two ways at once: an SGPR operand or not, and whether the
// accumulator's value converges (a = a | x stops changing) or keeps toggling (a = a + b). This
// separates the two: the same operation with an SGPR or a VGPR operand, on toggling (XOR) and on
// converging (OR) data, 16 independent chains per lane, 1 / 4 / 8 waves per SIMD.
// Rate = instructions per SIMD / (launch duration x 2.4 GHz), the fastest of three launches.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_valu_r4.hip -o scripts/ubench_valu_r4
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define R16(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)
#define OP_XOR3_S(i) "v_bitop3_b32 %[a" #i "], %[a" #i "], %[s], %[b] bitop3:0x96\n\t"
#define OP_XOR3_V(i) "v_bitop3_b32 %[a" #i "], %[a" #i "], %[c], %[b] bitop3:0x96\n\t"
#define OP_ORXOR_S(i) "v_bitop3_b32 %[a" #i "], %[a" #i "], %[s], %[b] bitop3:0xf6\n\t"
#define OP_ORXOR_V(i) "v_bitop3_b32 %[a" #i "], %[a" #i "], %[c], %[b] bitop3:0xf6\n\t"
#define OP_XOR_S(i) "v_xor_b32_e32 %[a" #i "], %[s], %[a" #i "]\n\t"
#define OP_XOR_V(i) "v_xor_b32_e32 %[a" #i "], %[c], %[a" #i "]\n\t"
#define OP_OR_S(i) "v_or_b32_e32 %[a" #i "], %[s], %[a" #i "]\n\t"
#define OP_OR_V(i) "v_or_b32_e32 %[a" #i "], %[c], %[a" #i "]\n\t"
#define OP_ADD_V(i) "v_add_u32_e32 %[a" #i "], %[c], %[a" #i "]\n\t"
#define OP_ADD_S(i) "v_add_u32_e32 %[a" #i "], %[s], %[a" #i "]\n\t"
#define OUTS(i) [a##i] "+v"(a[i]),
#define BODY(OPM) asm volatile(R16(OPM) : R16(OUTS)[d] "+v"(d) : [b] "v"(b), [c] "v"(c), [s] "s"(sc))

static const char* kNames[] = {"bitop3 xor3 SGPR (toggling)", "bitop3 xor3 VGPR (toggling)",
                               "bitop3 or_xor SGPR (converging)", "bitop3 or_xor VGPR (converging)",
                               "v_xor SGPR (toggling)", "v_xor VGPR (toggling)", "v_or SGPR (converging)",
                               "v_or VGPR (converging)", "v_add_u32 VGPR (toggling)", "v_add_u32 SGPR (toggling)"};
constexpr int kN = 10;

template <int F>
__global__ __launch_bounds__(256) void kern(uint32_t* out, int iters, uint32_t sc) {
  uint32_t a[16];
  for (int i = 0; i < 16; ++i) a[i] = threadIdx.x * (i + 3) + blockIdx.x;
  uint32_t b = threadIdx.x ^ 0x5a5a5a5au, c = ~threadIdx.x * 0x9e3779b9u, d = 0;
  for (int it = 0; it < iters; ++it) {
    if constexpr (F == 0) BODY(OP_XOR3_S);
    if constexpr (F == 1) BODY(OP_XOR3_V);
    if constexpr (F == 2) BODY(OP_ORXOR_S);
    if constexpr (F == 3) BODY(OP_ORXOR_V);
    if constexpr (F == 4) BODY(OP_XOR_S);
    if constexpr (F == 5) BODY(OP_XOR_V);
    if constexpr (F == 6) BODY(OP_OR_S);
    if constexpr (F == 7) BODY(OP_OR_V);
    if constexpr (F == 8) BODY(OP_ADD_V);
    if constexpr (F == 9) BODY(OP_ADD_S);
  }
  uint32_t x = d;
  for (int i = 0; i < 16; ++i) x ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int F>
void run(int blocks, uint32_t* out, int iters) {
  hipLaunchKernelGGL(kern<F>, dim3(blocks), dim3(256), 0, 0, out, iters, 0x3c3c5a5au);
}
void run_form(int f, int blocks, uint32_t* out, int iters) {
  switch (f) {
    case 0: run<0>(blocks, out, iters); break;
    case 1: run<1>(blocks, out, iters); break;
    case 2: run<2>(blocks, out, iters); break;
    case 3: run<3>(blocks, out, iters); break;
    case 4: run<4>(blocks, out, iters); break;
    case 5: run<5>(blocks, out, iters); break;
    case 6: run<6>(blocks, out, iters); break;
    case 7: run<7>(blocks, out, iters); break;
    case 8: run<8>(blocks, out, iters); break;
    default: run<9>(blocks, out, iters); break;
  }
}

int main() {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess || cus <= 0) return 2;
  uint32_t* d_out = nullptr;
  if (hipMalloc(&d_out, (size_t)cus * 8 * 256 * sizeof(uint32_t)) != hipSuccess) return 2;
  const int iters = 8000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int order = 0; order < 2; ++order) {  // both orders: a drift with time shows as a difference
    for (int k = 0; k < kN; ++k) {
      const int f = order == 0 ? k : kN - 1 - k;
      for (int wps : {1, 4, 8}) {
        const int blocks = cus * wps;
        run_form(f, blocks, d_out, iters / 4);
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
          (void)hipEventRecord(e0, 0);
          run_form(f, blocks, d_out, iters);
          (void)hipEventRecord(e1, 0);
          (void)hipEventSynchronize(e1);
          float ms = 0;
          (void)hipEventElapsedTime(&ms, e0, e1);
          best = ms < best ? ms : best;
        }
        const double ipc = (double)wps * iters * 16 / (best * 1e-3 * 2.4e9);
        printf("{\"form\": \"%s\", \"order\": %d, \"waves_per_simd\": %d, \"ms\": %.4f, "
               "\"wave_instr_per_simd_cycle_at_2p4\": %.4f}\n", kNames[f], order, wps, best, ipc);
      }
    }
  }
  return 0;
}
