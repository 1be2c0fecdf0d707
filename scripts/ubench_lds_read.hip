// ubench_lds_read.hip — ds_read_b128 rate on MI355X for the address patterns of the persistent batch
// kernel (wgp_kernel): every lane of a wave reads 16 B per instruction from a 15 KB LDS table.
//   pattern 0: 16 entries, lane l entry l mod 16 (every 16-B bank slot once: conflict-free)
//   pattern 1: 11 entries shared by the lanes (a pod's class row, non-tolerating pods only)
//   pattern 2: 22 entries (tolerating pods 1 in 20, as in BASELINE C3's synthetic pods)
//   pattern 3: every lane the same entry (broadcast)
// Reads are issued four per step (two groups of two entries, as in the scan), ORed into an
// accumulator (v_bitop3 OR3 chains, 6 VALU per step); 8 waves per SIMD (8 workgroups of 4 waves per CU).
// Prints one JSON line per pattern: bytes read per CU-cycle at the in-kernel clock.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_lds_read.hip -o scripts/ubench_lds_read
#include <hip/hip_runtime.h>

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

constexpr int STEPS = 2000;
constexpr int GQL = 44;      // entries per group (16 B each)
constexpr int GROUPS = 20;   // C3's table

__device__ __forceinline__ uint32_t or3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xfe);
}

__global__ __launch_bounds__(256) void k_read(int pattern, uint32_t* out, unsigned long long* clk) {
  __shared__ uint4 tab[GROUPS * GQL];
  for (int i = threadIdx.x; i < GROUPS * GQL; i += 256) tab[i] = make_uint4(i, i * 3, i * 5, i * 7);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  // splitmix of the global thread id: the lane's class
  unsigned long long z = (blockIdx.x * 256ull + threadIdx.x) * 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z ^= z >> 27;
  uint32_t ra;
  if (pattern == 0) ra = lane % 16;
  else if (pattern == 1) ra = (uint32_t)(z % 11);
  else if (pattern == 2) ra = (uint32_t)(z % 11) + ((z >> 20) % 20 == 0 ? 11u : 0u);
  else ra = 3;
  uint32_t acc = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int s = 0; s < STEPS; ++s) {
    const int g = (GROUPS - 2) - 2 * (s % (GROUPS / 2));
    const uint4* t1 = tab + (g + 1) * GQL + ra;
    const uint4* t0p = tab + g * GQL + ra;
    const uint4 a = t1[0], b = t1[22], c = t0p[0], d = t0p[22];
    acc = or3(acc, or3(or3(a.x, a.y, a.z), or3(a.w, b.x, b.y), or3(b.z, b.w, c.x)),
              or3(or3(c.y, c.z, c.w), or3(d.x, d.y, d.z), d.w));
  }
  const unsigned long long t1c = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if (threadIdx.x == 0) {
    clk[blockIdx.x * 2] = t1c - t0;
    clk[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount, blocks = cus * 8;
  uint32_t* out;
  unsigned long long* clk;
  CHECK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  CHECK(hipMalloc(&clk, (size_t)blocks * 16));
  std::vector<unsigned long long> h(blocks * 2);
  for (int pattern = 0; pattern < 4; ++pattern) {
    for (int rep = 0; rep < 3; ++rep) k_read<<<blocks, 256>>>(pattern, out, clk);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0));
    k_read<<<blocks, 256>>>(pattern, out, clk);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost));
    double cyc = 0, real = 0;
    for (int b = 0; b < blocks; ++b) {
      cyc += h[b * 2];
      real += h[b * 2 + 1];
    }
    cyc /= blocks;
    real /= blocks;
    const double ghz = cyc / real * 0.1;
    // bytes per CU over the loop: 8 workgroups x 4 waves x STEPS x 4 reads x 1 KiB, in the mean loop cycles
    const double bytes_cu = 8.0 * 4 * STEPS * 4 * 1024;
    printf("{\"pattern\": %d, \"kernel_ms\": %.4f, \"loop_cycles\": %.0f, \"ghz\": %.3f, \"bytes_per_cu_cycle\": %.1f, "
           "\"tb_per_s_chip\": %.1f}\n",
           pattern, ms, cyc, ghz, bytes_cu / cyc, bytes_cu * cus / (cyc / (ghz * 1e9)) / 1e12);
  }
  return 0;
}
