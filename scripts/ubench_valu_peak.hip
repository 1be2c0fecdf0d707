// ubench_valu_peak.hip — the wave64 VALU issue rate of one SIMD on MI355X (gfx950), per instruction
// form, with 16 independent accumulator chains per lane (no dependency stalls) at 1, 2, 4 and 8
// waves per SIMD. It settles the peak bench.py's VALU roofline uses: whether the integer forms the
// batch kernels issue (v_bitop3_b32, v_or3_b32, v_and_b32, v_min_u32, v_lshl_or_b32) issue every 2
// cycles like v_fma_f32 / v_add_f32 (MI355X_MICROARCH.md: SIMD-32, a wave64 instruction over two
// cycles) or every 4.
//
// Rate = instructions per SIMD / (the launch's event duration x the clock the chip held, measured
// inside the kernel: s_memtime / s_memrealtime of lane 0 of block 0 around its loop), the fastest of
// three launches after a warm-up. Launch overhead is <1% at these durations (1-8 ms).
// Prints one JSON line per (form, waves per SIMD), then a summary line:
//   {"int_valu_wave_instr_per_simd_cycle": ..., "fp32_valu_wave_instr_per_simd_cycle": ...}
// Build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_valu_peak.hip -o scripts/ubench_valu_peak
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define R16(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)

// one instruction per chain; %[a<i>] the chain's accumulator, b / c / s loop-invariant operands
#define OP_BITOP3(i) "v_bitop3_b32 %[a" #i "], %[a" #i "], %[b], %[c] bitop3:0x70\n\t"
#define OP_BITOP3S(i) "v_bitop3_b32 %[a" #i "], %[a" #i "], %[s], %[c] bitop3:0xf6\n\t"
#define OP_OR3(i) "v_or3_b32 %[a" #i "], %[a" #i "], %[b], %[c]\n\t"
#define OP_AND(i) "v_and_b32_e32 %[a" #i "], %[s], %[a" #i "]\n\t"
#define OP_MIN(i) "v_min_u32_e32 %[a" #i "], %[b], %[a" #i "]\n\t"
#define OP_LSHLOR(i) "v_lshl_or_b32 %[a" #i "], %[a" #i "], 1, %[c]\n\t"
#define OP_ADDU(i) "v_add_u32_e32 %[a" #i "], %[b], %[a" #i "]\n\t"
#define OP_ADDF(i) "v_add_f32_e32 %[a" #i "], %[b], %[a" #i "]\n\t"
#define OP_FMAF(i) "v_fma_f32 %[a" #i "], %[a" #i "], %[b], %[c]\n\t"

#define OUTS(i) [a##i] "+v"(a[i]),
#define ASM_BODY(OPM)                                                                                     \
  asm volatile(R16(OPM)                                                                                   \
               : R16(OUTS)[dummy] "+v"(dummy)                                                              \
               : [b] "v"(b), [c] "v"(c), [s] "s"(sc))

struct Form {
  const char* name;
  bool integer;
};
static const Form kForms[] = {{"v_bitop3_b32 (3 VGPR)", true}, {"v_bitop3_b32 (SGPR operand)", true},
                              {"v_or3_b32", true},             {"v_and_b32 (SGPR operand)", true},
                              {"v_min_u32", true},             {"v_lshl_or_b32", true},
                              {"v_add_u32", true},             {"v_add_f32", false},
                              {"v_fma_f32", false}};
constexpr int kNForms = sizeof(kForms) / sizeof(kForms[0]);

template <int F>
__global__ __launch_bounds__(256) void kern(uint32_t* out, unsigned long long* clk, int iters, uint32_t sc) {
  uint32_t a[16];
  for (int i = 0; i < 16; ++i) a[i] = threadIdx.x * (i + 3) + blockIdx.x;
  uint32_t b = threadIdx.x ^ 0x5a5a5a5au, c = ~threadIdx.x, dummy = 0;
  if (F >= 7) {  // finite floats for the f32 forms
    b = __float_as_uint(1.0e-7f);
    c = __float_as_uint(0.5f);
    for (int i = 0; i < 16; ++i) a[i] = __float_as_uint((float)(threadIdx.x + i));
  }
  unsigned long long t0 = 0, r0 = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int it = 0; it < iters; ++it) {
    if constexpr (F == 0) ASM_BODY(OP_BITOP3);
    if constexpr (F == 1) ASM_BODY(OP_BITOP3S);
    if constexpr (F == 2) ASM_BODY(OP_OR3);
    if constexpr (F == 3) ASM_BODY(OP_AND);
    if constexpr (F == 4) ASM_BODY(OP_MIN);
    if constexpr (F == 5) ASM_BODY(OP_LSHLOR);
    if constexpr (F == 6) ASM_BODY(OP_ADDU);
    if constexpr (F == 7) ASM_BODY(OP_ADDF);
    if constexpr (F == 8) ASM_BODY(OP_FMAF);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  uint32_t x = dummy;
  for (int i = 0; i < 16; ++i) x ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int F>
void launch(int blocks, uint32_t* out, unsigned long long* clk, int iters) {
  hipLaunchKernelGGL(kern<F>, dim3(blocks), dim3(256), 0, 0, out, clk, iters, 0x0f0f0f0fu);
}

void launch_form(int f, int blocks, uint32_t* out, unsigned long long* clk, int iters) {
  switch (f) {
    case 0: launch<0>(blocks, out, clk, iters); break;
    case 1: launch<1>(blocks, out, clk, iters); break;
    case 2: launch<2>(blocks, out, clk, iters); break;
    case 3: launch<3>(blocks, out, clk, iters); break;
    case 4: launch<4>(blocks, out, clk, iters); break;
    case 5: launch<5>(blocks, out, clk, iters); break;
    case 6: launch<6>(blocks, out, clk, iters); break;
    case 7: launch<7>(blocks, out, clk, iters); break;
    default: launch<8>(blocks, out, clk, iters); break;
  }
}

int main() {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess || cus <= 0) {
    fprintf(stderr, "no device\n");
    return 2;
  }
  uint32_t* d_out = nullptr;
  unsigned long long* d_clk = nullptr;
  if (hipMalloc(&d_out, (size_t)cus * 8 * 256 * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&d_clk, 2 * sizeof(unsigned long long)) != hipSuccess)
    return 2;
  const int iters = 16000;  // 256,000 instructions per wave per launch
  std::vector<double> int8w, fp8w, scan8w;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int f = 0; f < kNForms; ++f) {
    for (int wps : {1, 2, 4, 8}) {
      const int blocks = cus * wps;  // 256-thread blocks: one wave per SIMD per block
      launch_form(f, blocks, d_out, d_clk, iters / 4);  // warm-up (clock ramp, code load)
      float best = 1e30f;
      double ghz = 0.0;
      for (int rep = 0; rep < 3; ++rep) {  // the fastest of three: the launch's whole duration (events)
        (void)hipEventRecord(e0, 0);
        launch_form(f, blocks, d_out, d_clk, iters);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        unsigned long long clk[2] = {0, 0};
        (void)hipMemcpy(clk, d_clk, sizeof(clk), hipMemcpyDeviceToHost);
        if (ms < best) {
          best = ms;
          ghz = clk[1] ? (double)clk[0] / ((double)clk[1] * 10.0) : 2.4;  // memrealtime: 100 MHz
        }
      }
      // every SIMD runs wps waves of iters x 16 instructions; cycles = the launch's duration at the
      // clock block 0 measured (s_memtime over s_memrealtime)
      const double instr_per_simd = (double)wps * iters * 16;
      const double ipc = instr_per_simd / (best * 1e-3 * ghz * 1e9);
      printf("{\"form\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"clock_ghz_in_kernel\": %.3f, "
             "\"wave_instr_per_simd_cycle\": %.4f, \"cycles_per_wave_instr\": %.2f}\n",
             kForms[f].name, wps, best, ghz, ipc, 1.0 / ipc);
      if (wps == 8) {
        (kForms[f].integer ? int8w : fp8w).push_back(ipc);
        if (f == 0 || f == 2 || f == 4 || f == 5) scan8w.push_back(ipc);  // the forms wg_kernel's scan issues
      }
    }
  }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
  };
  printf("{\"int_valu_wave_instr_per_simd_cycle\": %.4f, \"scan_forms_wave_instr_per_simd_cycle\": %.4f, "
         "\"fp32_valu_wave_instr_per_simd_cycle\": %.4f, \"note\": \"median over the forms at 8 waves per SIMD; "
         "cycles = the fastest of three launches' event duration x the in-kernel clock (s_memtime / "
         "s_memrealtime); scan forms = v_bitop3 (VGPR), v_or3, v_min_u32, v_lshl_or\"}\n",
         med(int8w), med(scan8w), med(fp8w));
  (void)hipFree(d_out);
  (void)hipFree(d_clk);
  return 0;
}
