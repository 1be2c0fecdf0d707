// msh_kernels.hip — gfx950 (MI355X, CDNA4) kernels for the batched pods x nodes hot path.
//
// Reference path (shopetan/mini-kube-scheduler, Go): for ONE pod per cycle,
//   RunFilterPlugins   minisched/minisched.go:115-151  (NodeUnschedulable, upstream v1.22.0)
//   RunPreScorePlugins minisched/minisched.go:153-162  (NodeNumber.PreScore, nodenumber.go:50-64)
//   RunScorePlugins    minisched/minisched.go:164-199  (NodeNumber.Score, nodenumber.go:73-95)
//   selectHost         minisched/minisched.go:304-325  (argmax; ties -> lowest index here)
//
// Layout (msh_internal.h): per group of 256 List-order nodes, the digit rows ER[r] (bit i of row r:
// node i is feasible-relevant and scores 10 for a digit-r pod; row 10 all zero), the X words
// (NodeUnschedulable verdict for non-tolerating pods) and, for REVERSE / MINMAX, the V words (real
// node), plus the bit planes of the node codes the sequential / A/B kernels read. The batched kernels
// put one POD per lane: a lane's hit word for 32 nodes is ER[row] & ~(X & nT), one v_bitop3, so every
// VALU operation evaluates 32 (pod, node) pairs.
// Stages (north_star):
//   1. feasibility bitmask with wavefront __ballot (X / V words, first feasible per class) -> node_prep_kernel
//   2. int64 score with the plugin weight fused                    -> decode_pod / decode_ident
//   3. per-pod normalisation (DEFAULT / REVERSE / MINMAX need the extent of the raw scores over the
//      feasible list: first feasible match / non-match)             -> wgp_kernel / wg_kernel<KX> + decode
//   4. argmax with a fixed lowest-index tie-break: the lowest group with a hit, then its first set
//      bit (v_ffbl) in List order                                   -> wgp_kernel / wg_kernel
//   5. node-table tiles staged in LDS once per workgroup and reused by every pod it serves
//                                                                   -> wgp_kernel / wg_kernel
//   generic_kernel does stages 1-5 with an explicit int64 score per pair, for any score-plugin list
//   (score-column plugins; a real LDS min/max reduction and a wave-shuffle argmax).
//
// Kernels, by entry point:
//   node_prep_kernel (+ prep_reset_kernel)  every upload / patch / plugin change
//   wgp_kernel           msh_schedule_batch*, msh_schedule_batches_device on tables up to 8,192 nodes
//                        (BASELINE C2 / C3): persistent grid, the pod-class rows copied once per workgroup
//   wg_kernel            the same entry points on larger tables (chunk-streamed), and msh_shard_keys_device
//   generic_kernel       the batch entry points when the score list names a score-column plugin
//   rows_kernel          A/B (MSH_BATCH_KERNEL=slices): the round-2 slice kernel
//   bits_kernel          A/B (MSH_KX_BITS=1): REVERSE / MINMAX on the code planes
//   decode_keys_kernel   node-sharded mode: decode the merged int32 shard keys
//   seq_kernel           sequential commit, one pod at a time, one workgroup
//   export_kernel        per-pair result export (simulator result store)
// See DESIGN.md for the roofline / instruction budget of each kernel.
#include "msh_internal.h"

#include <hip/hip_ext.h>

#include <type_traits>

namespace msh {

// Kernel start / stop events for the next hot-kernel launch on this thread (msh_timing_begin):
// hipExtLaunchKernelGGL records them at the kernel's own start and completion, the interval
// rocprofv3's kernel trace reports, not around the launch like events recorded on the stream.
namespace {
thread_local hipEvent_t t_ev_start = nullptr, t_ev_stop = nullptr;
}
void set_launch_events(hipEvent_t start, hipEvent_t stop) {
  t_ev_start = start;
  t_ev_stop = stop;
}
bool launch_events_pending() { return t_ev_start != nullptr; }
#define MSH_TIMED_LAUNCH(kern, grid, block, lds, stream, ...)                                                   \
  do {                                                                                                          \
    if (t_ev_start) {                                                                                           \
      hipExtLaunchKernelGGL(kern, grid, block, lds, stream, t_ev_start, t_ev_stop, 0, __VA_ARGS__);             \
      t_ev_start = t_ev_stop = nullptr;                                                                         \
    } else {                                                                                                    \
      hipLaunchKernelGGL(kern, grid, block, lds, stream, __VA_ARGS__);                                          \
    }                                                                                                           \
  } while (0)

__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

// ---------------------------------------------------------------------------------------
// Stage 1: node table preparation + feasibility bitmask (once per upload / plugin change).
// For the only filter, NodeUnschedulable (upstream v1.22.0), feasibility depends on the pod
// only through "tolerates the unschedulable taint", so there are exactly two pod classes:
// 0 = does not tolerate, 1 = tolerates (feasible on every real node). Per 64-node wave, the
// ballots of the code bits, of X (infeasible for class 0) and of V (real node) are the planes of
// two words; the first feasible node of each class goes to ball[c] as a key (KMAX - idx, 0 =
// none), one atomicMax per class per 1,024-node block.
// ---------------------------------------------------------------------------------------
constexpr int PREP_THREADS = 1024;  // n_pad is a multiple of 1024: every block is whole
__global__ __launch_bounds__(PREP_THREADS) void node_prep_kernel(const uint8_t* __restrict__ unsched,
                                                                 const int8_t* __restrict__ digit,
                                                                 int32_t n, int32_t has_nu,
                                                                 uint32_t* __restrict__ ball,
                                                                 uint32_t* __restrict__ planes,
                                                                 uint32_t* __restrict__ erows,
                                                                 uint32_t* __restrict__ hrows) {
  constexpr int NWV = PREP_THREADS / WAVE;
  __shared__ uint32_t s_k0[NWV], s_k1[NWV];
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const bool valid = i < n;
  const bool u = valid && unsched[i] != 0;
  const int d = valid ? (int)digit[i] : -1;
  // NodeUnschedulable.Filter: Spec.Unschedulable && !tolerates -> UnschedulableAndUnresolvable
  const bool feas0 = valid && !(has_nu && u);
  const bool has_digit = d >= 0 && d <= 9;
  const uint32_t code = has_digit ? (uint32_t)d : CODE_NONE_NODE;  // NodeNumber: Atoi of the last byte
  const unsigned long long pm[PLANE_N] = {__ballot(code & 1u), __ballot(code & 2u), __ballot(code & 4u),
                                          __ballot(code & 8u), __ballot(valid && !feas0), __ballot(valid)};
  // this wave's 64 nodes are words 2t and 2t + 1 of the PLANE_* layout: lanes 0..11 write them
  if (lane < 2 * PLANE_N) {
    const int k = lane >> 1, half = lane & 1;
    unsigned long long m = pm[0];
#pragma unroll
    for (int q = 1; q < PLANE_N; ++q) m = (k == q) ? pm[q] : m;
    const uint32_t word = ((uint32_t)(i - lane) >> 5) + (uint32_t)half;  // i - lane: the wave's first node
    planes[((word / PLANE_GW) * PLANE_N + k) * PLANE_GW + word % PLANE_GW] = (uint32_t)(m >> (32 * half));
  }
  // the digit rows of the same two words (ER_* layout): row r = real nodes with digit r; lanes
  // 0..21 write rows 0..10 (row 10, pods without a digit, stays zero)
  unsigned long long em[ER_ROWS - 1];
#pragma unroll
  for (int r = 0; r < ER_ROWS - 1; ++r) em[r] = __ballot(code == (uint32_t)r);  // padding: code 15
  if (lane < 2 * ER_ROWS) {
    const int r = lane >> 1, half = lane & 1;
    unsigned long long m = 0;
#pragma unroll
    for (int q = 0; q < ER_ROWS - 1; ++q) m = (r == q) ? em[q] : m;
    const uint32_t word = ((uint32_t)(i - lane) >> 5) + (uint32_t)half;
    const uint32_t g = word / PLANE_GW, c = (word / 4) & 1u, k = word & 3u;
    erows[(size_t)g * ER_GD + (c * ER_ROWS + (uint32_t)r) * 4 + k] = (uint32_t)(m >> (32 * half));
  } else if (lane < 2 * ER_ROWS + 2) {  // lanes 22, 23: the X words behind the rows
    const int half = lane & 1;
    const uint32_t word = ((uint32_t)(i - lane) >> 5) + (uint32_t)half;
    erows[(size_t)(word / PLANE_GW) * ER_GD + ER_Q * 4 + word % PLANE_GW] = (uint32_t)(pm[PLANE_X] >> (32 * half));
  }
  // the class rows of the same two words (HR_* layout): lanes 0..43 write H[t][r] (row 10 zero),
  // lanes 44..47 F[t]
  {
    const unsigned long long x0 = ~pm[PLANE_X];  // class 0 passes NodeUnschedulable where X is clear
    if (lane < 4 * ER_ROWS) {
      const int r = lane >> 2, t = (lane >> 1) & 1, half = lane & 1;
      unsigned long long m = 0;
#pragma unroll
      for (int q = 0; q < ER_ROWS - 1; ++q) m = (r == q) ? em[q] : m;
      if (t == 0) m &= x0;
      const uint32_t word = ((uint32_t)(i - lane) >> 5) + (uint32_t)half;  // i - lane: the wave's first node
      const uint32_t g = word / PLANE_GW, c = (word / 4) & 1u, k = word & 3u;
      hrows[(size_t)g * HR_GD + hr_entry(c, (uint32_t)t, (uint32_t)r) * 4 + k] = (uint32_t)(m >> (32 * half));
    } else if (lane < 4 * ER_ROWS + 4) {
      const int t = (lane >> 1) & 1, half = lane & 1;
      const unsigned long long m = t == 0 ? (pm[PLANE_V] & x0) : pm[PLANE_V];
      const uint32_t word = ((uint32_t)(i - lane) >> 5) + (uint32_t)half;
      hrows[(size_t)(word / PLANE_GW) * HR_GD + (HR_F + 2 * t) * 4 + word % PLANE_GW] = (uint32_t)(m >> (32 * half));
    }
  }
  const unsigned long long m0 = pm[PLANE_V] & ~pm[PLANE_X], m1 = pm[PLANE_V];
  if (lane == 0) {
    s_k0[wv] = m0 ? KMAX - (uint32_t)(i + __builtin_ctzll(m0)) : 0u;
    s_k1[wv] = m1 ? KMAX - (uint32_t)(i + __builtin_ctzll(m1)) : 0u;
  }
  __syncthreads();
  // one first-feasible update per class per BLOCK: device-scope atomics on one address serialise
  if (threadIdx.x == 0) {
    uint32_t k0 = 0, k1 = 0;
    for (int w = 0; w < NWV; ++w) {
      k0 = umax(k0, s_k0[w]);
      k1 = umax(k1, s_k1[w]);
    }
    if (k0) atomicMax(&ball[0], k0);
    if (k1) atomicMax(&ball[1], k1);
  }
}

// ---------------------------------------------------------------------------------------
// Stage 2+3 epilogue: status / selected node / int64 score for one pod.
// im / ix / ia: first feasible match / first feasible non-match / first feasible of any
// class (node index, -1 = none). ix is only read by the modes that need it (needs_kx).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void decode_pod(int64_t im, int64_t ix, int64_t ia, bool pd_valid,
                                           const PluginParams& pp, int32_t* out_idx,
                                           int64_t* out_score, int32_t* out_status) {
  int64_t sel = -1, sc = 0;
  int32_t st = 0;
  if (ia < 0) {
    st = 1;  // FitError: no feasible node (minisched.go:143-148)
  } else if (pp.has_nn_score && (!pp.nn_prescore || !pd_valid)) {
    st = 2;  // NodeNumber.Score: state.Read -> ErrNotFound (nodenumber.go:74-77), F > 0
  } else if (!pp.has_nn_score) {
    sel = ia;  // all totals 0: first feasible
  } else {
    const int64_t w = pp.weight;
    switch (pp.mode) {
      case 1:  // DefaultNormalizeScore: match -> 100, rest 0 (max 10), or all 0 (max 0)
        sel = im >= 0 ? im : ia;
        sc = im >= 0 ? 100 * w : 0;
        break;
      case 2:  // DefaultNormalizeScore reverse: non-match -> 100, match -> 0 (or all 100)
        sel = ix >= 0 ? ix : im;
        sc = ix >= 0 ? 100 * w : 0;
        break;
      case 3:  // min-max: (s-min)*100/(max-min); 0 when only one class is feasible
        sel = im >= 0 ? im : ix;
        sc = (im >= 0 && ix >= 0) ? 100 * w : 0;
        break;
      default:  // NONE (the reference): raw 10 on match, 0 otherwise, times weight
        sel = im >= 0 ? im : ia;
        sc = im >= 0 ? 10 * w : 0;
        break;
    }
  }
  *out_idx = (int32_t)sel;
  *out_score = sc;
  *out_status = st;
}

// Shard keys (int32): GKEY_MAX - global node index, 0 = none. The slot-1 keys of the
// identity-like modes are per pod CLASS (first feasible node of that class), written once per
// launch by the first workgroup: keys[n_pods + c], c = 0 non-tolerating, 1 tolerating.
__device__ __forceinline__ int32_t shard_key(int64_t node_base, uint32_t local_idx) {
  return GKEY_MAX - (int32_t)(node_base + (int64_t)local_idx);
}
__device__ __forceinline__ void write_class_keys(const BatchArgs& a) {
  if (blockIdx.x == 0 && threadIdx.x < 2) {
    const uint32_t b = a.ball[threadIdx.x];
    a.keys[(size_t)a.n_pods + threadIdx.x] = b ? shard_key(a.node_base, KMAX - b) : 0;
  }
}

// decode_pod for the identity-like modes (NONE, DEFAULT: everything that does not need the
// first feasible non-match), as selects on launch-constant flags instead of a branch per mode.
struct IdentDecode {
  bool err_all;      // NodeNumber scores without its PreScore state: every feasible pod errors
  bool err_nodigit;  // ... with it: pods whose name has no digit suffix error
  bool use_im;       // NodeNumber scores at all (otherwise every total is 0: first feasible)
  int64_t sm;        // total score of a match: weight x (10 raw, or 100 normalized)
};
__device__ __forceinline__ IdentDecode make_ident_decode(const PluginParams& pp) {
  IdentDecode d;
  d.err_all = pp.has_nn_score && !pp.nn_prescore;
  d.err_nodigit = pp.has_nn_score && pp.nn_prescore;
  d.use_im = pp.has_nn_score != 0;
  d.sm = (pp.mode == 1 ? 100 : 10) * pp.weight;
  return d;
}
__device__ __forceinline__ void decode_ident(int64_t im, int64_t ia, bool pd_valid, const IdentDecode& d,
                                             int32_t* out_idx, int64_t* out_score, int32_t* out_status) {
  const bool fit = ia < 0;                                         // FitError (minisched.go:143)
  const bool serr = !fit && (d.err_all || (d.err_nodigit && !pd_valid));  // Score error (nodenumber.go:74-77)
  const bool hit = d.use_im && im >= 0;
  *out_status = fit ? 1 : (serr ? 2 : 0);
  *out_idx = (fit || serr) ? -1 : (int32_t)(hit ? im : ia);
  *out_score = (fit || serr || !hit) ? 0 : d.sm;
}

__device__ __forceinline__ int64_t key_to_idx(uint32_t k) {
  return k ? (int64_t)(KMAX - k) : (int64_t)-1;
}

// ---------------------------------------------------------------------------------------
// Bit-sliced batched kernel: stages 1-4 for every normalize mode (the default batch path).
//
// "Lanes = pods": lane l of the workgroup's waves holds pod 64 b + l. The node table is the
// bit-sliced PLANE_* layout (msh_internal.h): one 32-bit word per plane covers 32 nodes, and the
// planes of a word are wave-uniform, so they arrive by scalar loads and sit in SGPRs. Per lane
// and word, with the pod's code bits as all-ones / all-zero masks P0..P3 and nT = ~tolerates:
//   miss = (X & nT) | (D0 ^ P0) | (D1 ^ P1) | (D2 ^ P2) | (D3 ^ P3)      1 v_and + 4 v_bitop3
// has a zero bit exactly at each node that passes NodeUnschedulable for this pod AND whose suffix
// digit equals the pod's (NodeNumber.Score = 10): 32 (pod, node) pairs evaluated per lane-op
// chain, 5 VALU per 32 x 64 pairs. Padding slots carry code 15, pods without a digit code 14: they
// never match. Pairs of words AND into a per-group accumulator (v_bitop3, 3 inputs); a group of
// PLANE_GW words with a zero bit is remembered (groups are walked in DESCENDING List order, so the
// last one remembered is the first); the exact node is the first word of that group with a zero
// bit, then its lowest zero bit (see below for where the words come from). No
// cross-lane reduction at all: the first maximum of selectHost (minisched.go:304-325) falls out of
// the List order of words and bits.
//
// KX (REVERSE / MINMAX normalizers) also needs the first feasible NON-match:
//   nmiss = ~dm | (X & nT) | ~V,  dm = (D0 ^ P0) | ... | (D3 ^ P3)
// (8 VALU per word). The first feasible node of the pod's class comes from the prep (ball).
//
// S slice waves per workgroup split the groups of the table for the same 64 pods (small batches
// against large tables keep the chip busy); their firsts meet in LDS (slices ascend in List
// order, so the minimum is the first).
// ---------------------------------------------------------------------------------------
// t | (d ^ p) in one v_bitop3_b32 (truth table over S0 = t, S1 = d, S2 = p), d wave-uniform.
// Written as asm: the backend prefers v_xor + v_or3 pairs, 7.75 VALU per word instead of 5.
__device__ __forceinline__ uint32_t or_xor_s(uint32_t t, uint32_t d, uint32_t p) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xf6" : "=v"(r) : "v"(t), "s"(d), "v"(p));
  return r;
}
// x & m in one v_and_b32, x wave-uniform (SGPR), m a per-lane mask: left to itself the backend
// rewrites `x & (tol ? 0 : ~0)` as v_mov + v_cndmask on the lane condition, two VALU per word.
__device__ __forceinline__ uint32_t and_s(uint32_t x, uint32_t m) {
  uint32_t r;
  asm("v_and_b32_e32 %0, %1, %2" : "=v"(r) : "s"(x), "v"(m));
  return r;
}
// ~dm | xi | ~v (truth table over S0 = dm, S1 = xi, S2 = v), v wave-uniform
__device__ __forceinline__ uint32_t nmiss_s(uint32_t dm, uint32_t xi, uint32_t v) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xdf" : "=v"(r) : "v"(dm), "v"(xi), "s"(v));
  return r;
}

typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

// NPL planes of one group (PLANE_GW dwords each, contiguous) into SGPRs: NPL s_load_dwordx8 in
// flight, then ONE s_waitcnt that takes the loaded registers as operands, so that no use of them
// can be scheduled in front of it (the backend does not count asm-issued scalar loads).
template <int NPL>
__device__ __forceinline__ void sload_group(u32x8 (&pl)[NPL], const uint32_t* src) {
#pragma unroll
  for (int k = 0; k < NPL; ++k)
    asm volatile("s_load_dwordx8 %0, %1, %2" : "=s"(pl[k]) : "s"(src), "n"(k * PLANE_GW * 4));
  if constexpr (NPL == 5)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(pl[0]), "+s"(pl[1]), "+s"(pl[2]), "+s"(pl[3]), "+s"(pl[4]));
  else
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(pl[0]), "+s"(pl[1]), "+s"(pl[2]), "+s"(pl[3]), "+s"(pl[4]),
                 "+s"(pl[5]));
}

constexpr uint32_t NO_GROUP = 0xFFFFFFFFu;

// The lane's first node in group g (per-lane vector loads of the group's planes): the first word
// with a zero bit in the miss word, then its lowest zero bit. NONMATCH: the first feasible
// non-match instead of the first feasible match. Returns a node index (g has one by construction).
template <bool NONMATCH>
__device__ __forceinline__ uint32_t group_first(const uint32_t* __restrict__ planes, uint32_t g, uint32_t P0,
                                                uint32_t P1, uint32_t P2, uint32_t P3, uint32_t nT) {
  const uint4* q = reinterpret_cast<const uint4*>(planes + (size_t)g * GROUP_DWORDS);
  constexpr int NP = NONMATCH ? PLANE_N : PLANE_V;
  uint32_t pl[NP][PLANE_GW];
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const uint4 lo = q[k * 2], hi = q[k * 2 + 1];
    pl[k][0] = lo.x; pl[k][1] = lo.y; pl[k][2] = lo.z; pl[k][3] = lo.w;
    pl[k][4] = hi.x; pl[k][5] = hi.y; pl[k][6] = hi.z; pl[k][7] = hi.w;
  }
  uint32_t bw = 0;
  int32_t bj = 0;
#pragma unroll
  for (int c = PLANE_GW - 1; c >= 0; --c) {
    const uint32_t dm = (pl[0][c] ^ P0) | (pl[1][c] ^ P1) | (pl[2][c] ^ P2) | (pl[3][c] ^ P3);
    const uint32_t xi = pl[PLANE_X][c] & nT;
    uint32_t hit;
    if constexpr (NONMATCH) hit = dm & ~xi & pl[PLANE_N - 1][c];
    else hit = ~(dm | xi);
    bj = hit ? c : bj;
    bw = hit ? hit : bw;
  }
  return (g * PLANE_GW + (uint32_t)bj) * 32u + (uint32_t)__builtin_ctz(bw);
}

// The first node with a zero bit among the 8 kept miss words of group g (words ascend in List
// order, and bits within a word): descending selects, then the lowest zero bit.
__device__ __forceinline__ uint32_t kept_first(const uint32_t (&k)[PLANE_GW], uint32_t g) {
  uint32_t bw = 0;
  int32_t bj = 0;
#pragma unroll
  for (int c = PLANE_GW - 1; c >= 0; --c) {
    const uint32_t hit = ~k[c];
    bj = hit ? c : bj;
    bw = hit ? hit : bw;
  }
  return (g * PLANE_GW + (uint32_t)bj) * 32u + (uint32_t)__builtin_ctz(bw);
}

// The lowest group of a slice is scanned last (groups descend) and its miss words are still in
// registers: a lane whose first hit lies there (nearly every lane: a 256-node group almost always
// holds a feasible node of each digit) reads it off them (kept_first). Only a lane whose first hit
// lies in a higher group re-reads that group's planes (group_first, vector loads), behind an
// exec-mask branch the wave skips when no lane needs it. The groups above the lowest only track
// the first group with a hit: 5 VALU per word, the pair ANDs and one select per group.
template <int S, bool KX, bool SHARD>
__global__ __launch_bounds__(S * WAVE) void bits_kernel(BatchArgs a) {
  __shared__ uint32_t s_res[S][KX ? 2 : 1][WAVE];
  const int lane = threadIdx.x & (WAVE - 1);
  const int s = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int32_t j = (int32_t)blockIdx.x * WAVE + lane;
  const bool act = j < a.n_pods;
  uint32_t code = CODE_NONE_POD, tol = 0;
  if (act) {
    const int d = a.pod_digit[j];
    code = (d >= 0 && d <= 9) ? (uint32_t)d : CODE_NONE_POD;
    tol = a.pod_tol[j] ? 1u : 0u;
  }
  const uint32_t P0 = 0u - (code & 1u), P1 = 0u - ((code >> 1) & 1u), P2 = 0u - ((code >> 2) & 1u),
                 P3 = 0u - (code >> 3);
  const uint32_t nT = tol ? 0u : 0xFFFFFFFFu;
  const int32_t g_lo = min(s * a.gps, a.n_groups), g_hi = min(g_lo + a.gps, a.n_groups);
  constexpr int NPL = KX ? PLANE_N : PLANE_V;  // planes the scan reads
  // One group: the miss words (gm; KX: gx, the non-match miss words) and whether any has a zero bit.
  auto scan_group = [&](int32_t g, uint32_t (&gm)[PLANE_GW], uint32_t (&gx)[PLANE_GW], bool& hm, bool& hx) {
    // the group's planes, wave-uniform: one s_load_dwordx8 per plane, all in flight together,
    // one wait (left to itself the backend interleaves single-dword scalar loads with the
    // bitop3 chain, one lgkmcnt wait every few instructions)
    u32x8 pl[NPL];
    sload_group<NPL>(pl, a.planes + (size_t)g * GROUP_DWORDS);
    uint32_t pg[NPL * PLANE_GW];
#pragma unroll
    for (int k = 0; k < NPL; ++k)
#pragma unroll
      for (int c = 0; c < PLANE_GW; ++c) pg[k * PLANE_GW + c] = pl[k][c];
    uint32_t am = 0xFFFFFFFFu, ax = 0xFFFFFFFFu;
#pragma unroll
    for (int w = 0; w < PLANE_GW; w += 2) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int c = w + q;
        const uint32_t xi = and_s(pg[PLANE_X * PLANE_GW + c], nT);
        if constexpr (KX) {
          uint32_t dm = pg[c] ^ P0;
          dm = or_xor_s(dm, pg[PLANE_GW + c], P1);
          dm = or_xor_s(dm, pg[2 * PLANE_GW + c], P2);
          dm = or_xor_s(dm, pg[3 * PLANE_GW + c], P3);
          gm[c] = dm | xi;
          gx[c] = nmiss_s(dm, xi, pg[PLANE_V * PLANE_GW + c]);
        } else {
          uint32_t t = or_xor_s(xi, pg[c], P0);
          t = or_xor_s(t, pg[PLANE_GW + c], P1);
          t = or_xor_s(t, pg[2 * PLANE_GW + c], P2);
          gm[c] = or_xor_s(t, pg[3 * PLANE_GW + c], P3);
        }
      }
      am &= gm[w] & gm[w + 1];
      if constexpr (KX) ax &= gx[w] & gx[w + 1];
    }
    hm = am != 0xFFFFFFFFu;
    hx = KX && ax != 0xFFFFFFFFu;
  };
  uint32_t fm = NO_GROUP, fx = NO_GROUP;  // first group above the lowest with a feasible match / non-match
  uint32_t gm[PLANE_GW], gx[PLANE_GW];
  bool hm = false, hx = false;
  for (int32_t g = g_hi - 1; g > g_lo; --g) {
    scan_group(g, gm, gx, hm, hx);
    fm = hm ? (uint32_t)g : fm;
    if constexpr (KX) fx = hx ? (uint32_t)g : fx;
  }
  uint32_t rm = NOFIT, rx = NOFIT;  // node index of the first feasible match / non-match
  if (g_lo < g_hi) {
    scan_group(g_lo, gm, gx, hm, hx);
    if (hm) rm = kept_first(gm, (uint32_t)g_lo);
    if (KX && hx) rx = kept_first(gx, (uint32_t)g_lo);
    if (!hm && fm != NO_GROUP) rm = group_first<false>(a.planes, fm, P0, P1, P2, P3, nT);
    if (KX && !hx && fx != NO_GROUP) rx = group_first<true>(a.planes, fx, P0, P1, P2, P3, nT);
  }
  if constexpr (S > 1) {
    s_res[s][0][lane] = rm;
    if constexpr (KX) s_res[s][1][lane] = rx;
    __syncthreads();
    if (s != 0) return;
#pragma unroll
    for (int k = 1; k < S; ++k) {
      rm = umin(rm, s_res[k][0][lane]);
      if constexpr (KX) rx = umin(rx, s_res[k][1][lane]);
    }
  }
  // after the scan: a store in front of it would keep the backend from proving the planes
  // unclobbered, and the scalar loads would become vector loads
  if (SHARD && !KX) write_class_keys(a);
  if (!act) return;
  if constexpr (SHARD) {
    a.keys[j] = rm != NOFIT ? shard_key(a.node_base, rm) : 0;
    if constexpr (KX) a.keys[(size_t)a.n_pods + j] = rx != NOFIT ? shard_key(a.node_base, rx) : 0;
  } else {
    const int64_t ia = key_to_idx(a.ball[tol]);
    const int64_t im = rm != NOFIT ? (int64_t)rm : -1;
    int32_t oi, ost;
    int64_t osc;
    if constexpr (KX)
      decode_pod(im, rx != NOFIT ? (int64_t)rx : -1, ia, code != CODE_NONE_POD, a.pp, &oi, &osc, &ost);
    else
      decode_ident(im, ia, code != CODE_NONE_POD, make_ident_decode(a.pp), &oi, &osc, &ost);
    a.out_idx[j] = oi;
    if (a.out_score) a.out_score[j] = osc;  // optional output (NULL: not written)
    a.out_status[j] = ost;
  }
}

// ---------------------------------------------------------------------------------------
// Digit-row batched kernel: stages 1-4 for every normalize mode, the default batch path.
//
// Lanes = pods as in bits_kernel, but the node side is the digit-row bitmap index (ER_* layout,
// msh_internal.h): for a word of 32 nodes, row r holds the nodes whose suffix digit is r, so a pod
// reads the ONE row of its own digit instead of combining four code planes. Per lane and word:
//   hit = E[row] & ~(X & nT)          one v_bitop3_b32
// is set exactly at the nodes that pass NodeUnschedulable for this pod AND score 10 for it
// (NodeNumber.Score, digit equal): 32 (pod, node) pairs per lane-op. The KX modes (REVERSE,
// MINMAX) also need the first feasible non-match, nm = V & ~E[row] & ~(X & nT), two more VALU.
// Each wave stages its slice's rows and X words in LDS tiles of ER_TG groups (16-byte copies,
// wave-private, no barrier; KX: the V words too, from the code planes), and per group a lane reads
// its row of each 4-word chunk with one ds_read_b128 (lanes of one digit share the address and
// broadcast; the 11 rows of a chunk occupy distinct banks) and the group's X words at one address.
// The group's hits are ORed (v_or3) and a group with one is remembered; groups are walked in
// DESCENDING List order, so the last remembered is the first, and the lowest group of the slice,
// scanned last, keeps its hit words in registers for the exact node (first word with a hit, its
// lowest set bit). A lane whose first hit lies in a higher group re-reads that group from memory
// behind an exec-mask branch (rare: 256 nodes almost always hold a match). ~2 VALU and two
// ds_read_b128 per 32 x 64 pairs (bits_kernel: 5.75 VALU); at C3 the launches are bound by VALU
// issue with the LDS array about half busy. Slices and the LDS merge of their
// firsts as in bits_kernel.
// ---------------------------------------------------------------------------------------

// The first node among 8 hit words of group g (words ascend in List order, bits within a word):
// v_ffbl_b32 gives each word's lowest set bit, all-ones for an empty word, which ORed with the
// word's offset (32 c) stays all-ones; the unsigned minimum over the words is the first hit.
// 19 VALU (selects per word: ~30). The group must hold a hit.
__device__ __forceinline__ uint32_t lowbit(uint32_t x) {  // v_ffbl_b32: all-ones for 0 (ctz's 0 is UB)
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
__device__ __forceinline__ uint32_t hits_first(const uint32_t (&h)[PLANE_GW], uint32_t g) {
  uint32_t t[PLANE_GW];
#pragma unroll
  for (int c = 0; c < PLANE_GW; ++c) t[c] = lowbit(h[c]) | (uint32_t)(32 * c);
  const uint32_t m = umin(umin(umin(t[0], t[1]), umin(t[2], t[3])), umin(umin(t[4], t[5]), umin(t[6], t[7])));
  return g * GROUP_NODES + m;
}

// The lane's first feasible match in group g, from memory (its row words and the X plane).
__device__ __forceinline__ uint32_t rows_group_first(const BatchArgs& a, uint32_t g, uint32_t row, uint32_t nT) {
  const uint4* er = reinterpret_cast<const uint4*>(a.erows) + (size_t)g * ER_GQ;
  const uint4 e0 = er[row], e1 = er[ER_ROWS + row], x0 = er[ER_Q], x1 = er[ER_Q + 1];
  const uint32_t e[PLANE_GW] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
  const uint32_t x[PLANE_GW] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
  uint32_t h[PLANE_GW];
#pragma unroll
  for (int k = 0; k < PLANE_GW; ++k) h[k] = e[k] & ~(x[k] & nT);
  return hits_first(h, g);
}

// e & ~(x & m) in one v_bitop3_b32, all three in VGPRs (x: the same in every lane)
__device__ __forceinline__ uint32_t hit_v(uint32_t e, uint32_t x, uint32_t m) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x70" : "=v"(r) : "v"(e), "v"(x), "v"(m));
  return r;
}

// One group's hits: the lane's row words of both chunks and the group's X words (four
// ds_read_b128 of the staged tile, the X reads at one address for all lanes); returns whether any
// word has a hit.
__device__ __forceinline__ bool rows_hits(const uint4& e0, const uint4& e1, const uint4& x0, const uint4& x1,
                                          uint32_t nT, uint32_t (&h)[PLANE_GW]) {
  const uint32_t e[PLANE_GW] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
  const uint32_t x[PLANE_GW] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
  for (int k = 0; k < PLANE_GW; ++k) h[k] = hit_v(e[k], x[k], nT);
  return ((h[0] | h[1] | h[2]) | (h[3] | h[4] | h[5]) | (h[6] | h[7])) != 0u;
}

#if defined(MSH_STAMPS) || defined(MSH_CLOCK_STAMPS)
// Timeline / clock A/B builds only (scripts/stamps.sh, scripts/ab_build.sh; never in
// libminisched_hip.so): per wave, the 100 MHz wall clock at entry, after the prologue's loads, after
// the scan and before the stores (MSH_STAMPS); or the shader and 100 MHz clocks at a persistent
// wave's start and end (MSH_CLOCK_STAMPS, wgp_kernel).
__device__ unsigned long long* g_stamps;
#endif
#ifdef MSH_STAMPS
#define MSH_STAMP(i) (__builtin_amdgcn_s_waitcnt(0), stamp_t[i] = wall_clock64())
#else
#define MSH_STAMP(i) ((void)0)
#endif

// One group's feasible non-matches (KX modes): nm = V & ~E & ~(X & nT), two VALU per word
// (xm = X & nT, then one v_bitop3 with truth table 0x10 = S0 & ~S1 & ~S2).
__device__ __forceinline__ uint32_t nonmatch_v(uint32_t v, uint32_t e, uint32_t xm) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x10" : "=v"(r) : "v"(v), "v"(e), "v"(xm));
  return r;
}
__device__ __forceinline__ bool rows_nonmatch(const uint4& e0, const uint4& e1, const uint4& x0, const uint4& x1,
                                              const uint4& v0, const uint4& v1, uint32_t nT,
                                              uint32_t (&n)[PLANE_GW]) {
  const uint32_t e[PLANE_GW] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
  const uint32_t x[PLANE_GW] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
  const uint32_t v[PLANE_GW] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
  for (int k = 0; k < PLANE_GW; ++k) n[k] = nonmatch_v(v[k], e[k], x[k] & nT);
  return ((n[0] | n[1] | n[2]) | (n[3] | n[4] | n[5]) | (n[6] | n[7])) != 0u;
}
// The lane's first feasible non-match in group g, from memory (rare path of the KX modes): the
// rows and X from the digit rows, V from the code planes.
__device__ __forceinline__ uint32_t rows_group_first_nm(const BatchArgs& a, uint32_t g, uint32_t row, uint32_t nT) {
  const uint4* er = reinterpret_cast<const uint4*>(a.erows) + (size_t)g * ER_GQ;
  const uint4* vp = reinterpret_cast<const uint4*>(a.planes + (size_t)g * GROUP_DWORDS + PLANE_V * PLANE_GW);
  uint32_t n[PLANE_GW];
  rows_nonmatch(er[row], er[ER_ROWS + row], er[ER_Q], er[ER_Q + 1], vp[0], vp[1], nT, n);
  return hits_first(n, g);
}

template <int S, bool KX, bool SHARD, int PPL>
__global__ __launch_bounds__(S * WAVE) void rows_kernel(BatchArgs a) {
#ifdef MSH_STAMPS
  unsigned long long stamp_t[4] = {0, 0, 0, 0};
  MSH_STAMP(0);
  auto stamps_out = [&]() {
    if ((threadIdx.x & (WAVE - 1)) == 0)
      for (int i = 0; i < 4; ++i) g_stamps[((size_t)blockIdx.x * S + (threadIdx.x >> 6)) * 4 + i] = stamp_t[i];
  };
#endif
  constexpr int NR = KX ? 2 : 1;  // results per pod: first feasible match (+ first feasible non-match)
  __shared__ uint4 s_tile[S][ER_TG * ER_GQ];
  __shared__ uint4 s_vw[KX ? S : 1][KX ? 2 * ER_TG : 1];  // KX: the tile's V words (from the code planes)
  __shared__ uint32_t s_res[S][NR][PPL][WAVE];
  const int lane = threadIdx.x & (WAVE - 1);
  const int s = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  // PPL pods per lane: lane l holds pods base + q * 64 + l (q < PPL); the group's X words and the
  // staged row tile serve all of them
  const int32_t block0 = (int32_t)blockIdx.x * (PPL * WAVE);
  const int32_t base = block0 + lane;
  const int32_t g_lo = min(s * a.gps, a.n_groups), g_hi = min(g_lo + a.gps, a.n_groups);
  const int32_t ng = g_hi - g_lo;
  const uint4* __restrict__ er = reinterpret_cast<const uint4*>(a.erows);
  uint4* tile = s_tile[s];
  // This wave's tile, read only by this wave: a whole ER_TG-group tile is copied, three 16-byte
  // copies per lane (the table carries padding, so no copy needs a clamp; rows past the slice are
  // never read), and in the KX modes the tile's V words from the code planes (16 lanes, one group
  // half each, clamped to the table). Loads and stores are separate so that the prologue can put
  // the pod-byte loads between them.
  static_assert(ER_TG * ER_GQ == 3 * WAVE, "fill: three 16-byte copies per lane");
  uint4 f0, f1, f2, fv;
  uint4* vtile = s_vw[KX ? s : 0];
  auto fill_load = [&](int32_t t_lo) {
    const uint4* src = er + (uint32_t)(t_lo * ER_GQ);  // wave-uniform base, 32-bit lane offsets
    f0 = src[(uint32_t)lane];
    f1 = src[(uint32_t)(lane + WAVE)];
    f2 = src[(uint32_t)(lane + 2 * WAVE)];
    if constexpr (KX) {
      const int32_t gv = min(t_lo + (lane >> 1) % ER_TG, a.n_groups - 1);
      fv = reinterpret_cast<const uint4*>(a.planes + (size_t)gv * GROUP_DWORDS + PLANE_V * PLANE_GW)[lane & 1];
    }
  };
  auto fill_store = [&]() {
    tile[lane] = f0;
    tile[lane + WAVE] = f1;
    tile[lane + 2 * WAVE] = f2;
    if (KX && lane < 2 * ER_TG) vtile[lane] = fv;
    __builtin_amdgcn_wave_barrier();
  };
  // Prologue: the top tile's row words, the pod bytes (clamped offset: no branch, so nothing waits
  // for them yet) and the class firsts are all requested before the first use of any of them.
  const int32_t t_top = ng > 0 ? (ng - 1) / ER_TG : -1;
  fill_load(g_lo + max(t_top, 0) * ER_TG);  // (an empty slice copies a padding tile it never reads)
  int dq[PPL];
  uint8_t tq[PPL];
  const uint32_t last = (uint32_t)(a.n_pods - 1 - block0);  // n_pods > block0 (empty batches never launch)
  const int8_t* pdb = a.pod_digit + block0;                   // wave-uniform bases, 32-bit lane offsets
  const uint8_t* ptb = a.pod_tol + block0;
#pragma unroll
  for (int q = 0; q < PPL; ++q) {
    const uint32_t off = min((uint32_t)(lane + q * WAVE), last);
    dq[q] = pdb[off];
    tq[q] = ptb[off];
  }
  const uint32_t ball0 = a.ball[0], ball1 = a.ball[1];
  fill_store();
  bool act[PPL];
  uint32_t code[PPL], tol[PPL], nT[PPL], row[PPL];
  const uint4* lrow[PPL];  // the lane's row in chunk 0 of a tile's first group
#pragma unroll
  for (int q = 0; q < PPL; ++q) {
    act[q] = base + q * WAVE < a.n_pods;
    code[q] = (act[q] && dq[q] >= 0 && dq[q] <= 9) ? (uint32_t)dq[q] : CODE_NONE_POD;
    tol[q] = (act[q] && tq[q]) ? 1u : 0u;
    nT[q] = tol[q] ? 0u : 0xFFFFFFFFu;
    row[q] = code[q] <= 9u ? code[q] : (uint32_t)(ER_ROWS - 1);  // no digit: the zero row
    lrow[q] = tile + row[q];
  }
  MSH_STAMP(1);
  uint32_t h[PPL][PLANE_GW], hn[PPL][PLANE_GW];
  // first group above the lowest with a feasible match / non-match (NO_GROUP - 1: in h / hn)
  uint32_t fm[PPL], fx[PPL];
#pragma unroll
  for (int q = 0; q < PPL; ++q) fm[q] = fx[q] = NO_GROUP;
  // One group g of the tile for pod q: hits into hq (and non-matches into nq); returns the flags.
  auto group = [&](int32_t g, int32_t t_lo, int q, uint32_t (&hq)[PLANE_GW], uint32_t (&nq)[PLANE_GW], bool& am,
                   bool& ax) {
    const uint4* tg = tile + (g - t_lo) * ER_GQ;
    const uint4* r0 = lrow[q] + (g - t_lo) * ER_GQ;
    const uint4 e0 = r0[0], e1 = r0[ER_ROWS], x0 = tg[ER_Q], x1 = tg[ER_Q + 1];
    am = rows_hits(e0, e1, x0, x1, nT[q], hq);
    if constexpr (KX) {
      const uint4* vg = vtile + 2 * (g - t_lo);
      ax = rows_nonmatch(e0, e1, x0, x1, vg[0], vg[1], nT[q], nq);
    }
  };
  // Tiles from the top down, each one's groups descending; the lowest group of the slice last.
  for (int32_t t = t_top; t >= 0; --t) {
    const int32_t t_lo = g_lo + t * ER_TG, t_hi = min(t_lo + ER_TG, g_hi);
    if (t != t_top) {
      fill_load(t_lo);
      fill_store();
    }
    const int32_t g_end = t == 0 ? g_lo + 1 : t_lo;  // tile 0: all but the lowest group
    int32_t g = t_hi - 1;
    for (; g - 1 >= g_end; g -= 2) {  // two groups per step
#pragma unroll
      for (int q = 0; q < PPL; ++q) {
        uint32_t h1[PLANE_GW], h2[PLANE_GW], n1[PLANE_GW], n2[PLANE_GW];  // (only the lowest group's are kept)
        bool m1, m2, x1 = false, x2 = false;
        group(g, t_lo, q, h1, n1, m1, x1);
        group(g - 1, t_lo, q, h2, n2, m2, x2);
        fm[q] = m1 ? (uint32_t)g : fm[q];
        fm[q] = m2 ? (uint32_t)(g - 1) : fm[q];
        if constexpr (KX) {
          fx[q] = x1 ? (uint32_t)g : fx[q];
          fx[q] = x2 ? (uint32_t)(g - 1) : fx[q];
        }
      }
    }
    if (g >= g_end) {
#pragma unroll
      for (int q = 0; q < PPL; ++q) {
        uint32_t h1[PLANE_GW], n1[PLANE_GW];
        bool m1, x1 = false;
        group(g, t_lo, q, h1, n1, m1, x1);
        fm[q] = m1 ? (uint32_t)g : fm[q];
        if constexpr (KX) fx[q] = x1 ? (uint32_t)g : fx[q];
      }
    }
    if (t == 0) {  // the lowest group: its hit (and non-match) words stay in registers
#pragma unroll
      for (int q = 0; q < PPL; ++q) {
        bool m1, x1 = false;
        group(g_lo, t_lo, q, h[q], hn[q], m1, x1);
        fm[q] = m1 ? NO_GROUP - 1 : fm[q];
        if constexpr (KX) fx[q] = x1 ? NO_GROUP - 1 : fx[q];
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  uint32_t rm[PPL], rx[PPL];  // node index of the first feasible match / non-match
  MSH_STAMP(2);
#pragma unroll
  for (int q = 0; q < PPL; ++q) {
    rm[q] = rx[q] = NOFIT;
    if (fm[q] == NO_GROUP - 1) rm[q] = hits_first(h[q], (uint32_t)g_lo);
    else if (fm[q] != NO_GROUP) rm[q] = rows_group_first(a, fm[q], row[q], nT[q]);
    if constexpr (KX) {
      if (fx[q] == NO_GROUP - 1) rx[q] = hits_first(hn[q], (uint32_t)g_lo);
      else if (fx[q] != NO_GROUP) rx[q] = rows_group_first_nm(a, fx[q], row[q], nT[q]);
    }
  }
  if constexpr (S > 1) {
#pragma unroll
    for (int q = 0; q < PPL; ++q) {
      s_res[s][0][q][lane] = rm[q];
      if constexpr (KX) s_res[s][NR - 1][q][lane] = rx[q];
    }
    __syncthreads();
#ifdef MSH_STAMPS
    if (s != 0) {
      stamps_out();
      return;
    }
#else
    if (s != 0) return;
#endif
#pragma unroll
    for (int k = 1; k < S; ++k)
#pragma unroll
      for (int q = 0; q < PPL; ++q) {
        rm[q] = umin(rm[q], s_res[k][0][q][lane]);
        if constexpr (KX) rx[q] = umin(rx[q], s_res[k][NR - 1][q][lane]);
      }
  }
  if (SHARD && !KX) write_class_keys(a);
#ifdef MSH_STAMPS
  MSH_STAMP(3);
  stamps_out();
#endif
#pragma unroll
  for (int q = 0; q < PPL; ++q) {
    if (!act[q]) continue;
    const int32_t j = base + q * WAVE;
    if constexpr (SHARD) {
      a.keys[j] = rm[q] != NOFIT ? shard_key(a.node_base, rm[q]) : 0;
      if constexpr (KX) a.keys[(size_t)a.n_pods + j] = rx[q] != NOFIT ? shard_key(a.node_base, rx[q]) : 0;
    } else {
      int32_t oi, ost;
      int64_t osc;
      const int64_t im = rm[q] != NOFIT ? (int64_t)rm[q] : -1, ia = key_to_idx(tol[q] ? ball1 : ball0);
      if constexpr (KX)
        decode_pod(im, rx[q] != NOFIT ? (int64_t)rx[q] : -1, ia, code[q] != CODE_NONE_POD, a.pp, &oi, &osc, &ost);
      else
        decode_ident(im, ia, code[q] != CODE_NONE_POD, make_ident_decode(a.pp), &oi, &osc, &ost);
      a.out_idx[j] = oi;
      if (a.out_score) a.out_score[j] = osc;  // optional output (NULL: not written)
      a.out_status[j] = ost;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Workgroup-table batched kernel (the default batch path since round 3).
//
// Lanes = pods, as in rows_kernel, but the node side is staged ONCE per workgroup: the W waves of a
// workgroup (W x 64 pods) copy the digit rows and X words (KX: and the V words) of up to WG_CHUNK
// groups into LDS together, and every wave then scans every group of the table for its own 64 pods.
// No slices, so no slice merge and no per-wave tile copies. Per lane and 256-node group the scan
// folds the pair evaluation and the group's OR into one v_bitop3 per 32-node word:
//   acc = acc | (E[row] & ~X')        truth table 0xF4 (the first word: E & ~X', 0x44)
// where X' is the group's X words for a pod that does not tolerate the unschedulable taint and a
// zero block staged next to them for one that does (NodeUnschedulable per pair: a tolerating pod
// passes every real node); the lane picks its block once, by address. A group whose acc is non-zero
// holds a feasible digit match: it pushes a 1 into a per-chunk bitmap (bit k = group lo + k; v_min +
// v_lshl_or per group). 11 VALU per group and lane (8 bitop3, the flag, the addresses) against
// rows_kernel's 16; KX also accumulates the feasible non-matches, acc' |= V & ~(E | X') (v_or +
// v_bitop3 per word). Groups are walked in descending List order; the first group with a hit is the
// lowest set bit of the lowest chunk's bitmap that has one, and its hit words are recomputed once per
// lane at the end (from LDS, or from memory when it lies in a chunk no longer staged: more than
// WG_CHUNK groups above the first with a hit, rare). Tables larger than one chunk are streamed chunk
// by chunk, descending: the next chunk's copy is in flight in registers while the current one is
// scanned (two workgroup barriers per chunk).
//
// MULTI: the launch serves up to MULTI_MAX independent batches (msh_schedule_batches_device), each
// with its own pod columns and outputs, described in the kernel arguments; the grid is 2-D, batch =
// blockIdx.y (one scalar load of its descriptor).
// ---------------------------------------------------------------------------------------
// Phase experiments of A/B builds only (scripts/wg_expt.sh, scripts/ab_build.sh; never the product
// library): bit 0 skips the scan loop, bit 1 the output stores, bit 2 the table copy into LDS; bit 4
// (wgp_kernel's quad scan) adds a second reduction tree per pair of groups. MSH_WG_FLAG
// selects the form of the per-group flag (A/B of the same build).
#ifndef MSH_WG_EXPT
#define MSH_WG_EXPT 0
#endif
#ifndef MSH_WG_FLAG
#define MSH_WG_FLAG 0
#endif
constexpr int WG_CHUNK = 32;  // groups per staged chunk (8,192 nodes; 13 KiB, 14 KiB with V words)
// LDS layout of a staged group, in 16-byte entries: the 22 row chunks, X (2), a zero block Z (2) that
// tolerating pods read instead of X, and (KX) V (2)
constexpr int LQ_X = ER_Q, LQ_Z = ER_GQ, LQ_V = ER_GQ + 2;

template <bool MULTI>
struct KArgs {
  using T = BatchArgs;
};
template <>
struct KArgs<true> {
  using T = MultiArgs;
};
__device__ __forceinline__ const BatchArgs& base_args(const BatchArgs& a) { return a; }
__device__ __forceinline__ const BatchArgs& base_args(const MultiArgs& m) { return m.a; }

// acc | (e & ~x), one v_bitop3_b32 (S0 = acc, S1 = e, S2 = x). The builtin, not inline asm: the
// compiler then knows the instruction's hazards (inline asm got a conservative s_nop after each pair).
__device__ __forceinline__ uint32_t acc_andn(uint32_t acc, uint32_t e, uint32_t x) {
  return __builtin_amdgcn_bitop3_b32(acc, e, x, 0xf4);
}
// e & ~x (the first word of a group: S0 is a don't-care)
__device__ __forceinline__ uint32_t andn(uint32_t e, uint32_t x) { return __builtin_amdgcn_bitop3_b32(e, e, x, 0x44); }
__device__ __forceinline__ uint32_t min1(uint32_t x) {  // x != 0 as 0 / 1 in one v_min_u32
  uint32_t r;
  asm("v_min_u32 %0, 1, %1" : "=v"(r) : "v"(x));
  return r;
}
__device__ __forceinline__ uint32_t lshl_or(uint32_t a, uint32_t sh, uint32_t b) {  // (a << sh) | b
  uint32_t r;
  asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "i"(sh), "v"(b));
  return r;
}

// One staged group for one lane: the OR over its 8 words of the feasible digit matches (hit) and, KX,
// of the feasible non-matches (nm). tr: the lane's row entry, tx: the lane's X or Z entry, tv: V.
template <bool KX>
__device__ __forceinline__ void group_acc(const uint4* tr, const uint4* tx, const uint4* tv, uint32_t& hit,
                                          uint32_t& nm) {
  const uint4 e0 = tr[0], e1 = tr[ER_ROWS], x0 = tx[0], x1 = tx[1];
  hit = andn(e0.x, x0.x);
  hit = acc_andn(hit, e0.y, x0.y);
  hit = acc_andn(hit, e0.z, x0.z);
  hit = acc_andn(hit, e0.w, x0.w);
  hit = acc_andn(hit, e1.x, x1.x);
  hit = acc_andn(hit, e1.y, x1.y);
  hit = acc_andn(hit, e1.z, x1.z);
  hit = acc_andn(hit, e1.w, x1.w);
  if constexpr (KX) {
    const uint4 v0 = tv[0], v1 = tv[1];
    nm = andn(v0.x, e0.x | x0.x);
    nm = acc_andn(nm, v0.y, e0.y | x0.y);
    nm = acc_andn(nm, v0.z, e0.z | x0.z);
    nm = acc_andn(nm, v0.w, e0.w | x0.w);
    nm = acc_andn(nm, v1.x, e1.x | x1.x);
    nm = acc_andn(nm, v1.y, e1.y | x1.y);
    nm = acc_andn(nm, v1.z, e1.z | x1.z);
    nm = acc_andn(nm, v1.w, e1.w | x1.w);
  }
}

template <int W, bool KX, bool SHARD, bool MULTI>
__global__ __launch_bounds__(W * WAVE) void wg_kernel(typename KArgs<MULTI>::T ka) {
  static_assert(!(SHARD && MULTI), "shard keys come from single-batch launches");
  constexpr int GQ = KX ? ER_GQ + 2 : ER_GQ;                     // 16-byte entries per group in memory
  constexpr int GQL = KX ? LQ_V + 2 : LQ_Z + 2;                  // ... per staged group in LDS
  constexpr int NT = W * WAVE;                                   // threads per workgroup
  constexpr int EPT = (WG_CHUNK * GQ + NT - 1) / NT;             // staged entries per thread per chunk
  __shared__ uint4 s_tab[WG_CHUNK * GQL];
#ifdef MSH_STAMPS
  unsigned long long stamp_t[4] = {0, 0, 0, 0};
  MSH_STAMP(0);
#endif
  const BatchArgs& A = base_args(ka);
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));

  // ---- this workgroup's batch ----
  int32_t blk = (int32_t)blockIdx.x;
  const int8_t* pod_digit = A.pod_digit;
  const uint8_t* pod_tol = A.pod_tol;
  int32_t* out_idx = A.out_idx;
  int64_t* out_score = A.out_score;
  int32_t* out_status = A.out_status;
  int32_t n_pods = A.n_pods;
  if constexpr (MULTI) {
    const BatchDesc& d = ka.d[blockIdx.y];
    if (blk * NT >= d.n_pods) return;  // past this batch's end (the grid's x extent is the largest batch's)
    pod_digit = d.pod_digit;
    pod_tol = d.pod_tol;
    out_idx = d.out_idx;
    out_score = d.out_score;
    out_status = d.out_status;
    n_pods = d.n_pods;
  }
  const int32_t wbase = blk * NT + wv * WAVE;  // this wave's first pod (may lie past the batch)
  const int32_t j = wbase + lane;

  // ---- staging: chunk c = groups [c * WG_CHUNK, min(+WG_CHUNK, n_groups)) ----
  const int32_t n_groups = A.n_groups;
  const int32_t n_chunks = (n_groups + WG_CHUNK - 1) / WG_CHUNK;  // >= 1 (tables are never empty)
  const uint4* __restrict__ er = reinterpret_cast<const uint4*>(A.erows);
  // Every thread loads EPT (<= 4) entries unconditionally (indices past the chunk clamped to its
  // last entry: no divergent branch around a load, so the copies stay in flight) and stores every
  // slot of the staging array it owns (slots past the chunk are never read). Four named registers,
  // not an array: an array of uint4 captured by the lambdas went to scratch.
  static_assert(EPT <= 4, "wg_kernel stages at most four 16-byte entries per thread and chunk");
  uint4 st0, st1, st2, st3;
  auto st_ref = [&](int k) -> uint4& { return k == 0 ? st0 : k == 1 ? st1 : k == 2 ? st2 : st3; };
  auto chunk_load = [&](int32_t c) {
    if constexpr ((MSH_WG_EXPT & 4) != 0) return;
    const int32_t glo = c * WG_CHUNK, last = min(WG_CHUNK, n_groups - glo) * GQ - 1;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int32_t i = min((int32_t)threadIdx.x + k * NT, last);
      if constexpr (KX) {
        const int32_t gi = i / GQ, q = i - gi * GQ;
        const uint4* src = q < ER_GQ ? er + (size_t)(glo + gi) * ER_GQ + q
                                     : reinterpret_cast<const uint4*>(A.planes + (size_t)(glo + gi) * GROUP_DWORDS +
                                                                      PLANE_V * PLANE_GW) + (q - ER_GQ);
        st_ref(k) = *src;
      } else {
        st_ref(k) = er[(size_t)glo * ER_GQ + i];
      }
    }
  };
  auto chunk_store = [&]() {  // memory entry i of group gi -> LDS entry gi * GQL + q (V past Z)
    if constexpr ((MSH_WG_EXPT & 4) != 0) return;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int32_t i = (int32_t)threadIdx.x + k * NT;
      const int32_t gi = i / GQ, q = i - gi * GQ;
      if ((k + 1) * NT <= WG_CHUNK * GQ || i < WG_CHUNK * GQ) s_tab[gi * GQL + q + (q >= ER_GQ ? 2 : 0)] = st_ref(k);
    }
  };

  // ---- prologue: the top chunk's copy, the pod bytes (clamped offset) and the class firsts in
  // flight together; the zero blocks written once ----
  chunk_load(n_chunks - 1);
  const uint32_t lastp = n_pods > 0 ? (uint32_t)(n_pods - 1) : 0u;
  const uint32_t jj = min((uint32_t)j, lastp);
  const int dq = pod_digit[jj];
  const uint8_t tq = pod_tol[jj];
  const uint32_t ball0 = A.ball[0], ball1 = A.ball[1];
  if (threadIdx.x < 2 * WG_CHUNK) s_tab[(threadIdx.x >> 1) * GQL + LQ_Z + (threadIdx.x & 1)] = make_uint4(0, 0, 0, 0);
  chunk_store();
  const bool act = j < n_pods;
  const uint32_t code = (act && dq >= 0 && dq <= 9) ? (uint32_t)dq : CODE_NONE_POD;
  const uint32_t tol = (act && tq) ? 1u : 0u;
  const uint32_t nT = tol ? 0u : 0xFFFFFFFFu;
  const uint32_t row = code <= 9u ? code : (uint32_t)(ER_ROWS - 1);  // no digit: the zero row
  const uint32_t xq = tol ? (uint32_t)LQ_Z : (uint32_t)LQ_X;           // X, or the zero block
  __syncthreads();
  MSH_STAMP(1);

  uint32_t fm = NO_GROUP, fx = NO_GROUP;  // first group with a feasible match / non-match
  for (int32_t c = n_chunks - 1; c >= 0; --c) {
    const int32_t glo = c * WG_CHUNK, ng = min(WG_CHUNK, n_groups - glo);
    if (c != n_chunks - 1) {
      __syncthreads();  // every wave is done with chunk c + 1
      chunk_store();
      __syncthreads();
    }
    if (c > 0) chunk_load(c - 1);  // in flight during this chunk's scan
    uint32_t bm = 0, bx = 0;        // bit k: group glo + k has a feasible match / non-match
    int32_t k = (MSH_WG_EXPT & 1) ? -1 : ng - 1;
    for (; k >= 1; k -= 2) {  // two groups per step
      const uint4* t1 = s_tab + k * GQL;
      const uint4* t0 = t1 - GQL;
      uint32_t h1, h0, n1 = 0, n0 = 0;
      group_acc<KX>(t1 + row, t1 + xq, t1 + LQ_V, h1, n1);
      group_acc<KX>(t0 + row, t0 + xq, t0 + LQ_V, h0, n0);
#if MSH_WG_FLAG == 1
      bm = (bm << 2) + (h1 != 0 ? 2u : 0u) + (h0 != 0 ? 1u : 0u);
      if constexpr (KX) bx = (bx << 2) + (n1 != 0 ? 2u : 0u) + (n0 != 0 ? 1u : 0u);
#else
      bm = lshl_or(bm, 2, lshl_or(min1(h1), 1, min1(h0)));
      if constexpr (KX) bx = lshl_or(bx, 2, lshl_or(min1(n1), 1, min1(n0)));
#endif
    }
    if (k == 0) {
      uint32_t h0, n0 = 0;
      group_acc<KX>(s_tab + row, s_tab + xq, s_tab + LQ_V, h0, n0);
      bm = lshl_or(bm, 1, min1(h0));
      if constexpr (KX) bx = lshl_or(bx, 1, min1(n0));
    }
    if (bm) fm = (uint32_t)glo + lowbit(bm);
    if constexpr (KX)
      if (bx) fx = (uint32_t)glo + lowbit(bx);
  }
  MSH_STAMP(2);
  // the exact first node of the first group with a hit: chunk 0 is still staged
  uint32_t rm = NOFIT, rx = NOFIT;
  const uint32_t staged_hi = (uint32_t)min(WG_CHUNK, n_groups);
  if (fm != NO_GROUP) {
    if (fm < staged_hi) {
      uint32_t h[PLANE_GW];
      const uint4* tg = s_tab + fm * GQL;
      rows_hits(tg[row], tg[ER_ROWS + row], tg[LQ_X], tg[LQ_X + 1], nT, h);
      rm = hits_first(h, fm);
    } else {
      rm = rows_group_first(A, fm, row, nT);
    }
  }
  if constexpr (KX) {
    if (fx != NO_GROUP) {
      if (fx < staged_hi) {
        uint32_t n[PLANE_GW];
        const uint4* tg = s_tab + fx * GQL;
        rows_nonmatch(tg[row], tg[ER_ROWS + row], tg[LQ_X], tg[LQ_X + 1], tg[LQ_V], tg[LQ_V + 1], nT, n);
        rx = hits_first(n, fx);
      } else {
        rx = rows_group_first_nm(A, fx, row, nT);
      }
    }
  }
  if constexpr (SHARD && !KX) write_class_keys(A);
  if (!act) return;
  if constexpr (SHARD) {
    A.keys[j] = rm != NOFIT ? shard_key(A.node_base, rm) : 0;
    if constexpr (KX) A.keys[(size_t)n_pods + j] = rx != NOFIT ? shard_key(A.node_base, rx) : 0;
  } else {
    int32_t oi, ost;
    int64_t osc;
    const int64_t im = rm != NOFIT ? (int64_t)rm : -1, ia = key_to_idx(tol ? ball1 : ball0);
    if constexpr (KX)
      decode_pod(im, rx != NOFIT ? (int64_t)rx : -1, ia, code != CODE_NONE_POD, A.pp, &oi, &osc, &ost);
    else
      decode_ident(im, ia, code != CODE_NONE_POD, make_ident_decode(A.pp), &oi, &osc, &ost);
    if ((MSH_WG_EXPT & 2) == 0 || oi == 0x7fffffff) {
      out_idx[j] = oi;
      if (out_score) out_score[j] = osc;  // optional output (NULL: not written)
      out_status[j] = ost;
    }
  }
#ifdef MSH_STAMPS
  MSH_STAMP(3);
  if (lane == 0 && g_stamps) {
    const size_t w = ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * W + wv;
    for (int i = 0; i < 4; ++i) g_stamps[w * 4 + i] = stamp_t[i];
  }
#endif
}

// ---------------------------------------------------------------------------------------
// Persistent batch kernel (msh_schedule_batch_device / msh_schedule_batches_device when the table
// has at most WGP_MAX_GROUPS groups, 8,192 nodes: BASELINE C2 and C3). A grid of as many workgroups
// as stay resident (CUs x 8 at C3) copies the table's CLASS ROWS (msh_internal.h HR_*) into LDS once
// per workgroup and then walks the launch's (batch, 256-pod block) space with a stride of the grid;
// after the copy the waves are independent (no barrier per block), and each wave loads the next
// block's pod bytes before it scans the current one.
// Per lane (pod) and 256-node group the pair evaluation is one read of the pod's class row: the two
// 16-byte entries H[t][r] of the group's two 4-word chunks, t = the pod tolerates the unschedulable
// taint, r = its suffix digit (10 = none: the zero row). A set bit is a node that passes
// NodeUnschedulable for the pod and scores 10 for it (NodeNumber). The 8 words are ORed into the
// group's flag (three v_bitop3 OR3 and a v_or, then v_min + v_lshl_or into a per-lane bitmap of
// groups); REVERSE / MINMAX also OR the feasible non-matches F[t] & ~H (one v_bitop3 per word).
// 32 B of LDS per pod and group, 1/8 B per (pod, node) pair: half of wg_kernel's digit rows + X
// words, and the scan is bound by the LDS array's read bandwidth. The first group
// with a hit is the lowest set bit of the bitmap (groups walked in descending List order); its
// exact first node is resolved from the same two entries (v_ffbl), as in wg_kernel.
// ---------------------------------------------------------------------------------------
#ifndef MSH_WGP_W
#define MSH_WGP_W 4  // waves per workgroup of the persistent kernel (A/B builds: 8, 16)
#endif
#ifndef MSH_WGP_AGE_SLOPE
#define MSH_WGP_AGE_SLOPE 100  // per-slot fall of the item share, x 1e-3 (A/B builds)
#endif
#ifndef MSH_WGP_SHARE_MIN
#define MSH_WGP_SHARE_MIN 5  // items per workgroup from which the age-slot shares are used (A/B builds)
#endif
constexpr int WGP_SHARE_MIN = MSH_WGP_SHARE_MIN;
constexpr int WGP_MAX_GROUPS = 32;  // <= 8,192 nodes: 27 KB of LDS (6 workgroups per CU; C3: 17 KB, 8)

__device__ __forceinline__ uint32_t or3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xfe);
}

template <int W, bool KX>
__global__ __launch_bounds__(W * WAVE) void wgp_kernel(MultiArgs ka) {
#ifdef MSH_CLOCK_STAMPS  // diagnostic build only (scripts/ab_build.sh): the in-kernel clock per wave
  const unsigned long long ck_t0 = __builtin_amdgcn_s_memtime(), ck_r0 = __builtin_amdgcn_s_memrealtime();
#endif
  constexpr int GQL = HR_GQ;  // entries staged per group: the whole record (rows, F, first-node offsets)
  constexpr int NT = W * WAVE;
  extern __shared__ uint4 s_tab[];        // n_groups * GQL entries
  const BatchArgs& A = ka.a;
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int32_t n_groups = A.n_groups;  // <= WGP_MAX_GROUPS (the launcher's condition)
  {  // the table copy, once per workgroup: every load in flight before the first store
    constexpr int EPT = (WGP_MAX_GROUPS * GQL + NT - 1) / NT;
    const uint4* __restrict__ hr = reinterpret_cast<const uint4*>(A.hrows);
    const int32_t tot = n_groups * GQL;
    // loads unconditional (index clamped to the last entry: no branch around them, so all are in
    // flight together), then the stores of the slots below tot; named registers, not an array (a
    // uint4 array went to scratch)
    static_assert(EPT <= 7, "wgp_kernel copies at most seven 16-byte entries per thread");
    auto src = [&](int k) { return hr[min((int32_t)threadIdx.x + k * NT, tot - 1)]; };
    const uint4 v0 = src(0), v1 = EPT > 1 ? src(1) : v0, v2 = EPT > 2 ? src(2) : v0, v3 = EPT > 3 ? src(3) : v0,
                v4 = EPT > 4 ? src(4) : v0, v5 = EPT > 5 ? src(5) : v0, v6 = EPT > 6 ? src(6) : v0;
    const uint4 vs[7] = {v0, v1, v2, v3, v4, v5, v6};
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int32_t i = (int32_t)threadIdx.x + k * NT;
      if ((MSH_WG_EXPT & 4) == 0 && i < tot) s_tab[i] = vs[k];
    }
  }
  const uint32_t ball0 = A.ball[0], ball1 = A.ball[1];
  const IdentDecode idd = make_ident_decode(A.pp);
  __syncthreads();
  // ---- the (batch, block) walk: item it = b * bpb + x (pods [NT x, NT x + NT) of batch b, 64 per
  // wave), it = blockIdx.x, blockIdx.x + G, ... Per item a wave: scans the first two groups; issues the
  // PREVIOUS item's output stores and then the NEXT item's pod-byte loads; scans the rest; decodes. The
  // wait for the prefetched bytes (vmcnt counts loads and stores in issue order) thus falls a whole
  // scan after both. Batch, block and descriptor fields are kept wave-uniform (v_readfirstlane), so
  // the descriptor reads are scalar loads and the control flow on them scalar branches.
  // Tried and not kept (profiles/ab/r3_wgp_ab.jsonl): items handed out per wave by an LDS ticket, and
  // issue priority raised by the share of a workgroup's range still ahead. The waves of a CU do not
  // progress at one rate (the issue arbiter favours older waves: a CU's first workgroup ends its 6
  // items in ~13 us, its last in ~23 us), but the CU's LDS stays busy while most of them run, and
  // either remedy cost more than the tail it shortened.
  // Two walks (MultiArgs::walk): with few items per workgroup, items it = g, g + G, g + 2G, ... (the
  // leftover items fall to the low-numbered, oldest workgroups); with many, workgroup g walks the
  // contiguous range the launcher sized for its age slot on the CU (rank_lo). The issue arbiter
  // favours older waves: with equal shares a CU's first workgroup finished in ~60% of the time of
  // its last, and the CU ran its last microseconds on a few workgroups (profiles/ab/r3_wgp_clock.jsonl).
  const int32_t bpb = __builtin_amdgcn_readfirstlane(ka.bpb);
  int32_t it, total, step;
  if (ka.walk == 0) {
    it = (int32_t)blockIdx.x;
    total = ka.nb * bpb;
    step = (int32_t)gridDim.x;
  } else {
    const int32_t rk = (int32_t)blockIdx.x / ka.rank_wgs, rc = (int32_t)blockIdx.x - rk * ka.rank_wgs;
    const int32_t pool_lo = ka.rank_lo[rk], pool = ka.rank_lo[rk + 1] - pool_lo;
    it = pool_lo + (int32_t)((int64_t)pool * rc / ka.rank_wgs);
    total = pool_lo + (int32_t)((int64_t)pool * (rc + 1) / ka.rank_wgs);
    step = 1;
  }
  it = __builtin_amdgcn_readfirstlane(it);
  total = __builtin_amdgcn_readfirstlane(total);
  step = __builtin_amdgcn_readfirstlane(step);
  int32_t b = it / bpb, x = it - b * bpb;
  int dq = 0;
  uint32_t tq = 0;
  auto load_pods = [&]() {  // this wave's pod bytes of item (b, x), clamped offset
    const BatchDesc& d = ka.d[__builtin_amdgcn_readfirstlane(b)];
    const int32_t np = __builtin_amdgcn_readfirstlane(d.n_pods);
    const int32_t w0 = __builtin_amdgcn_readfirstlane(x * NT + wv * WAVE);
    const uint32_t jj = min((uint32_t)(w0 + lane), np > 0 ? (uint32_t)(np - 1) : 0u);
    if (w0 < np) {
      dq = d.pod_digit[jj];
      tq = d.pod_tol[jj];
    }
  };
  struct Item {
    int32_t cb, wbase, j;  // batch, the wave's first pod, the lane's pod
    bool live, act;        // the wave has pods in this item / the lane has a pod
    uint32_t code, tol, cls, e0, e1;  // cls = 11 tol + row; e0 / e1: its class-row entries (hr_entry)
  };
  auto prepare = [&]() {  // the state of item (b, x) from its loaded pod bytes
    Item m;
    const bool in = it < total;
    m.cb = __builtin_amdgcn_readfirstlane(in ? b : 0);
    const int32_t np = __builtin_amdgcn_readfirstlane(in ? ka.d[m.cb].n_pods : 0);
    m.wbase = __builtin_amdgcn_readfirstlane(x * NT + wv * WAVE);
    m.live = __builtin_amdgcn_readfirstlane(m.wbase < np ? 1 : 0) != 0;
    m.j = m.wbase + lane;
    m.act = m.j < np;
    m.code = (m.act && dq >= 0 && dq <= 9) ? (uint32_t)dq : CODE_NONE_POD;
    m.tol = (m.act && tq) ? 1u : 0u;
    const uint32_t row = m.code <= 9u ? m.code : (uint32_t)(ER_ROWS - 1);  // no digit: the zero row
    m.cls = m.tol * ER_ROWS + row;
    m.e0 = hr_entry(0, m.tol, row);
    m.e1 = hr_entry(1, m.tol, row);
    return m;
  };
  auto advance = [&]() {  // to the next item of this workgroup, its pod bytes in flight
    it += step;
    x += step;
    while (x >= bpb) {
      x -= bpb;
      ++b;
    }
    if (it < total) load_pods();
  };
  // the previous item's outputs, stored during the next scan (or after the loop): wave-uniform
  // bases (the wave's first pod) plus the lane's constant offset, so the stores read no VGPR the scan
  // writes (a VGPR an outstanding store still has to read would cost a vmcnt wait inside the scan)
  const uint32_t lo4 = (uint32_t)lane * 4u, lo8 = (uint32_t)lane * 8u;  // the lane's byte offsets
  int32_t s_cb = 0, s_wbase = 0, s_oi = 0, s_ost = 0;
  int64_t s_osc = 0;
  bool s_pending = false;  // the lane holds outputs not yet stored
  // The store addresses too stay live until the scan has ended (pinned below with the values): a
  // register an outstanding store reads may not be rewritten before the store completes, and the
  // compiler would otherwise reuse them at once and wait for the stores (vmcnt) right there.
  int32_t *p_oi = nullptr, *p_ot = nullptr;
  int64_t* p_os = nullptr;
  auto flush = [&]() {
    if ((MSH_WG_EXPT & 2) != 0 && s_oi != 0x7fffffff) s_pending = false;  // phase experiment: no stores
    const BatchDesc& d = ka.d[s_cb];
    const bool has_score = d.out_score != nullptr;
    p_oi = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(d.out_idx + s_wbase) + lo4);
    p_os = reinterpret_cast<int64_t*>(reinterpret_cast<char*>((has_score ? d.out_score : nullptr) + s_wbase) + lo8);
    p_ot = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(d.out_status + s_wbase) + lo4);
    if (s_pending) {
      *p_oi = s_oi;
      if (has_score) *p_os = s_osc;  // optional output (NULL: not written)
      *p_ot = s_ost;
    }
    s_pending = false;
  };
  if (it < total) load_pods();
  Item cur = prepare();
#ifdef MSH_CLOCK_STAMPS
  int n_items = 0;
#endif
  while (it < total) {
#ifdef MSH_CLOCK_STAMPS
    ++n_items;
#endif
    if (!cur.live) {  // this wave's slice lies past its batch's end
      flush();
      advance();
      cur = prepare();
      continue;
    }
    const uint32_t tol = cur.tol;
    const uint32_t e0 = cur.e0, e1 = cur.e1;  // the lane's chunk-0 and chunk-1 class-row entries
    const uint32_t cls = cur.cls;               // its class (first-node tables)
    const uint32_t fa = HR_F + 2 * tol;         // F[tol] (KX)
    // Groups descending, four per step (eight ds_read_b128 in flight; n_groups is a multiple of 4:
    // tables are padded to 1,024-node blocks), one flag per PAIR of groups: bit q of bm = group 2q or
    // 2q + 1 holds a feasible digit match (the 16 words of a pair reduce in 8 VALU: 7 v_bitop3 OR3 and
    // one more), and, KX, bit q of bx = one of them holds a feasible non-match (F[t] & ~H, one v_bitop3
    // per word). The previous item's stores and the next item's loads go after the first step.
    uint32_t bm = 0, bx = 0;
    auto or16 = [](const uint4& a, const uint4& b, const uint4& c, const uint4& d) {
      return or3(or3(or3(a.x, a.y, a.z), or3(a.w, b.x, b.y), or3(b.z, b.w, c.x)),
                 or3(or3(c.y, c.z, c.w), or3(d.x, d.y, d.z), d.w), 0u);
    };
    auto nm16 = [&](const uint4* tg, const uint4& a, const uint4& b, const uint4& c, const uint4& d) {
      const uint4 f0 = tg[fa], f1 = tg[fa + 1], f2 = tg[GQL + fa], f3 = tg[GQL + fa + 1];
      uint32_t n = andn(f0.x, a.x);
      n = acc_andn(n, f0.y, a.y);
      n = acc_andn(n, f0.z, a.z);
      n = acc_andn(n, f0.w, a.w);
      n = acc_andn(n, f1.x, b.x);
      n = acc_andn(n, f1.y, b.y);
      n = acc_andn(n, f1.z, b.z);
      n = acc_andn(n, f1.w, b.w);
      n = acc_andn(n, f2.x, c.x);
      n = acc_andn(n, f2.y, c.y);
      n = acc_andn(n, f2.z, c.z);
      n = acc_andn(n, f2.w, c.w);
      n = acc_andn(n, f3.x, d.x);
      n = acc_andn(n, f3.y, d.y);
      n = acc_andn(n, f3.z, d.z);
      n = acc_andn(n, f3.w, d.w);
      return n;
    };
    auto step = [&](int32_t q) {  // groups q .. q + 3
      const uint4* t = s_tab + q * GQL;
      const uint4 a0 = t[e0], b0 = t[e1], a1 = t[GQL + e0], b1 = t[GQL + e1];
      const uint4 a2 = t[2 * GQL + e0], b2 = t[2 * GQL + e1], a3 = t[3 * GQL + e0], b3 = t[3 * GQL + e1];
      bm = lshl_or(bm, 2, lshl_or(min1(or16(a2, b2, a3, b3)), 1, min1(or16(a0, b0, a1, b1))));
      if constexpr (KX)
        bx = lshl_or(bx, 2, lshl_or(min1(nm16(t + 2 * GQL, a2, b2, a3, b3)), 1, min1(nm16(t, a0, b0, a1, b1))));
    };
    int32_t q = (MSH_WG_EXPT & 1) ? -4 : n_groups - 4;
    if (q >= 0) {
      step(q);
      q -= 4;
    }
    flush();
    advance();
    for (; q >= 0; q -= 4) step(q);
    // the stored values and their addresses live through the scan
    asm volatile("" ::"v"(s_oi), "v"(s_ost), "v"(s_osc), "v"(p_oi), "v"(p_os), "v"(p_ot));
    // the exact first node: the first flagged pair, its first group with one, the offset from the table
    auto first_of = [&](uint32_t bits, uint32_t kind) {
      const uint32_t pq = lowbit(bits);
      const uint16_t* t0 = reinterpret_cast<const uint16_t*>(s_tab + 2 * pq * GQL + HR_FIRST) + kind + cls;
      const uint16_t* t1 = reinterpret_cast<const uint16_t*>(s_tab + (2 * pq + 1) * GQL + HR_FIRST) + kind + cls;
      const uint32_t f0 = *t0, f1 = *t1;
      return f0 != HR_NONE ? 2 * pq * GROUP_NODES + f0 : (2 * pq + 1) * GROUP_NODES + f1;
    };
    uint32_t rm = NOFIT, rx = NOFIT;
    if (bm) rm = first_of(bm, 0);
    if constexpr (KX)
      if (bx) rx = first_of(bx, HR_CLS);
    const int64_t im = rm != NOFIT ? (int64_t)rm : -1, ia = key_to_idx(tol ? ball1 : ball0);
    if constexpr (KX)
      decode_pod(im, rx != NOFIT ? (int64_t)rx : -1, ia, cur.code != CODE_NONE_POD, A.pp, &s_oi, &s_osc, &s_ost);
    else
      decode_ident(im, ia, cur.code != CODE_NONE_POD, idd, &s_oi, &s_osc, &s_ost);
    s_cb = cur.cb;
    s_wbase = cur.wbase;
    s_pending = cur.act;
    cur = prepare();
  }
  flush();
#ifdef MSH_CLOCK_STAMPS
  const unsigned long long ck_t1 = __builtin_amdgcn_s_memtime(), ck_r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0 && g_stamps) {
    unsigned long long* o = g_stamps + ((size_t)blockIdx.x * W + wv) * 8;
    o[0] = ck_t0;
    o[1] = ck_r0;
    o[2] = ck_t1;
    o[3] = ck_r1;
    o[4] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID: cu / sh / se / simd / wave
    o[5] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));  // HW_REG_XCC_ID
    o[6] = (unsigned long long)n_items;
    o[7] = blockIdx.x;
  }
#endif
}

// ---------------------------------------------------------------------------------------
// Generic score pipeline: any score plugin list (NodeNumber and up to four score-column plugins,
// MSH_PLUGIN_SCORE_COLUMN0..3), with the int64 score of every (pod, node) pair computed
// explicitly. The bitmap kernels above are exact only because NodeNumber's raw score takes two
// values; this kernel is the general form of RunScorePlugins (minisched.go:164-199), north_star's
// stages one to one:
//   5. node-table tiles: GEN_TILE nodes (the raw columns and the score columns in use) staged in
//      LDS once per workgroup and reused by its GEN_PB pods;
//   1. feasibility: one node per lane, NodeUnschedulable per pair; the wave's ballot is the
//      feasibility bitmask of its 64 nodes (the feasible count comes from its popcount);
//   3. per-pod extent of every score plugin over the feasible nodes (a pass of its own, only
//      when some plugin normalizes): per-lane max / min, a wave-shuffle reduction, then an LDS
//      reduction across the waves (64-bit LDS atomics);
//   2. the int64 total of each pair: sum over plugins of weight x NormalizeScore(raw) (upstream
//      helper.DefaultNormalizeScore, reverse, or min-max), in Go int64 arithmetic (wrapping);
//   4. selectHost: per lane the first maximum of its nodes (they ascend), then a wave-shuffle
//      argmax on (total desc, index asc) and a cross-wave merge in LDS.
// One workgroup of GEN_THREADS lanes per GEN_PB pods; lanes take nodes i = tid + k * GEN_THREADS
// of each tile. Status as the reference routes it: FitError when no node is feasible, the
// NodeNumber score error (no PreScore state) when some node is.
// ---------------------------------------------------------------------------------------
constexpr int GEN_PB = 8;           // pods per workgroup
constexpr int GEN_TILE = 1024;      // nodes per staged tile (2 KiB + 8 KiB per score column in use)
constexpr int GEN_THREADS = 256;
constexpr int GEN_WAVES = GEN_THREADS / WAVE;
constexpr uint8_t GEN_PAD = 2;      // s_un value of a slot past the table

__device__ __forceinline__ int64_t shfl_xor64(int64_t v, int m) {
  const int lo = __shfl_xor((int)(uint32_t)(uint64_t)v, m), hi = __shfl_xor((int)((uint64_t)v >> 32), m);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo);
}

// NormalizeScore of one raw score given the pod's extent of that plugin over its feasible nodes
// (mx, mn): upstream helper.DefaultNormalizeScore(MaxNodeScore = 100, reverse) — maxCount starts at
// 0, an all-zero list is left alone (reverse: all 100) — or min-max (0 when max == min).
__device__ __forceinline__ int64_t gen_normalize(int64_t raw, int32_t mode, int64_t mx, int64_t mn) {
  switch (mode) {
    case 1: {
      const int64_t m = mx > 0 ? mx : 0;
      return m == 0 ? raw : 100 * raw / m;
    }
    case 2: {
      const int64_t m = mx > 0 ? mx : 0;
      return m == 0 ? 100 : 100 - 100 * raw / m;
    }
    case 3: return mx == mn ? 0 : (raw - mn) * 100 / (mx - mn);
    default: return raw;
  }
}

__global__ __launch_bounds__(GEN_THREADS) void generic_kernel(GenericArgs a) {
  __shared__ uint8_t s_un[GEN_TILE];
  __shared__ int8_t s_dg[GEN_TILE];
  __shared__ int64_t s_col[GEN_COLS][GEN_TILE];
  __shared__ int64_t s_max[GEN_PB][GEN_MAX_SCORE], s_min[GEN_PB][GEN_MAX_SCORE];
  __shared__ int64_t s_btot[GEN_PB][GEN_WAVES];
  __shared__ int32_t s_bidx[GEN_PB][GEN_WAVES];
  const int tid = threadIdx.x, lane = tid & (WAVE - 1);
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int32_t j0 = (int32_t)blockIdx.x * GEN_PB;
  const int npb = min(GEN_PB, a.n_pods - j0);
  // the score columns the plugin list reads (a mask over GEN_COLS)
  int colmask = 0;
  for (int s = 0; s < a.ns; ++s)
    if (a.kind[s] > 0) colmask |= 1 << (a.kind[s] - 1);
  if (tid < GEN_PB * GEN_MAX_SCORE) {
    (&s_max[0][0])[tid] = INT64_MIN;
    (&s_min[0][0])[tid] = INT64_MAX;
  }
  if (tid < GEN_PB * GEN_WAVES) {
    (&s_btot[0][0])[tid] = 0;
    (&s_bidx[0][0])[tid] = -1;
  }
  const int32_t n_tiles = (a.n_nodes + GEN_TILE - 1) / GEN_TILE;
  constexpr int NPT = GEN_TILE / GEN_THREADS;  // nodes per lane and tile
  for (int sweep = a.need_ext ? 0 : 1; sweep < 2; ++sweep) {
    for (int32_t t = 0; t < n_tiles; ++t) {
      __syncthreads();  // the previous tile (or sweep) is done with the staged columns
      const int32_t base = t * GEN_TILE;
      for (int i = tid; i < GEN_TILE; i += GEN_THREADS) {  // coalesced copies of the tile
        const int32_t node = base + i;
        const bool v = node < a.n_nodes;
        s_un[i] = v ? (a.unsched[node] ? 1 : 0) : GEN_PAD;
        s_dg[i] = v ? a.digit[node] : (int8_t)-1;
#pragma unroll
        for (int k = 0; k < GEN_COLS; ++k)
          if (colmask & (1 << k)) s_col[k][i] = v ? a.cols[k * a.col_stride + node] : 0;
      }
      __syncthreads();
      for (int q = 0; q < npb; ++q) {
        const int pd = a.pod_digit[j0 + q];
        const bool tol = a.pod_tol[j0 + q] != 0;
        const bool pd_ok = pd >= 0 && pd <= 9;
        // raw score of plugin s at staged node i (NodeNumber: 10 on a suffix-digit match)
        auto raw = [&](int s, int i) -> int64_t {
          const int kd = a.kind[s];
          if (kd == 0) return (pd_ok && s_dg[i] == pd) ? 10 : 0;
          return s_col[kd - 1][i];
        };
        if (sweep == 0) {  // ---- stage 3: the extent of every score plugin over the feasible nodes
          int64_t lmx[GEN_MAX_SCORE], lmn[GEN_MAX_SCORE];
#pragma unroll
          for (int s = 0; s < GEN_MAX_SCORE; ++s) {
            lmx[s] = INT64_MIN;
            lmn[s] = INT64_MAX;
          }
#pragma unroll
          for (int k = 0; k < NPT; ++k) {
            const int i = tid + k * GEN_THREADS;
            const uint8_t u = s_un[i];
            const bool feas = u != GEN_PAD && !(a.has_nu && u && !tol);  // stage 1: NodeUnschedulable
            if (feas)
#pragma unroll
              for (int s = 0; s < GEN_MAX_SCORE; ++s)
                if (s < a.ns) {
                  const int64_t r = raw(s, i);
                  lmx[s] = r > lmx[s] ? r : lmx[s];
                  lmn[s] = r < lmn[s] ? r : lmn[s];
                }
          }
#pragma unroll
          for (int s = 0; s < GEN_MAX_SCORE; ++s) {
            if (s >= a.ns) break;
#pragma unroll
            for (int m = 32; m > 0; m >>= 1) {  // wave-shuffle reduction
              const int64_t ox = shfl_xor64(lmx[s], m), on = shfl_xor64(lmn[s], m);
              lmx[s] = ox > lmx[s] ? ox : lmx[s];
              lmn[s] = on < lmn[s] ? on : lmn[s];
            }
            if (lane == 0 && lmx[s] != INT64_MIN) {  // LDS reduction across the waves
              atomicMax((long long*)&s_max[q][s], (long long)lmx[s]);
              atomicMin((long long*)&s_min[q][s], (long long)lmn[s]);
            }
          }
        } else {  // ---- stages 1, 2, 4: feasibility, the weighted int64 total, the first maximum
          int64_t mx[GEN_MAX_SCORE], mn[GEN_MAX_SCORE];
#pragma unroll
          for (int s = 0; s < GEN_MAX_SCORE; ++s) {
            mx[s] = s_max[q][s];
            mn[s] = s_min[q][s];
          }
          int64_t btot = 0;
          int32_t bidx = -1;
          uint64_t fmask = 0;  // this wave's feasibility bitmask (stage 1), one tile slice at a time
#pragma unroll
          for (int k = 0; k < NPT; ++k) {
            const int i = tid + k * GEN_THREADS;
            const uint8_t u = s_un[i];
            const bool feas = u != GEN_PAD && !(a.has_nu && u && !tol);
            fmask |= __ballot(feas);
            if (feas) {
              uint64_t tot = 0;  // Go int64: wrapping
#pragma unroll
              for (int s = 0; s < GEN_MAX_SCORE; ++s)
                if (s < a.ns) tot += (uint64_t)gen_normalize(raw(s, i), a.mode[s], mx[s], mn[s]) * (uint64_t)a.weight[s];
              const int64_t ts = (int64_t)tot;
              if (bidx < 0 || ts > btot) {  // nodes ascend per lane: the first maximum
                btot = ts;
                bidx = base + i;
              }
            }
          }
          if (fmask) {  // some node of this wave's slice is feasible for pod q
#pragma unroll
            for (int m = 32; m > 0; m >>= 1) {  // wave-shuffle argmax: total desc, index asc
              const int64_t ot = shfl_xor64(btot, m);
              const int32_t oi = __shfl_xor(bidx, m);
              const bool take = oi >= 0 && (bidx < 0 || ot > btot || (ot == btot && oi < bidx));
              btot = take ? ot : btot;
              bidx = take ? oi : bidx;
            }
            if (lane == 0) {  // this wave's running best across tiles (tiles ascend)
              const int32_t ci = s_bidx[q][wv];
              if (ci < 0 || btot > s_btot[q][wv]) {
                s_btot[q][wv] = btot;
                s_bidx[q][wv] = bidx;
              }
            }
          }
        }
      }
    }
  }
  __syncthreads();
  if (tid < npb) {  // merge the waves' bests (LDS), decode, write
    const int q = tid, j = j0 + q;
    int64_t bt = 0;
    int32_t bi = -1;
#pragma unroll
    for (int w = 0; w < GEN_WAVES; ++w) {
      const int32_t oi = s_bidx[q][w];
      const int64_t ot = s_btot[q][w];
      if (oi >= 0 && (bi < 0 || ot > bt || (ot == bt && oi < bi))) {
        bt = ot;
        bi = oi;
      }
    }
    const int pd = a.pod_digit[j];
    const bool pd_ok = pd >= 0 && pd <= 9;
    int32_t st = 0;
    if (bi < 0) st = 1;                                           // FitError (minisched.go:143-148)
    else if (a.nn_score && (!a.nn_prescore || !pd_ok)) st = 2;    // NodeNumber.Score error (nodenumber.go:74-77)
    a.out_idx[j] = st ? -1 : bi;
    if (a.out_score) a.out_score[j] = st ? 0 : bt;
    a.out_status[j] = st;
  }
}

hipError_t launch_generic(const GenericArgs& a, hipStream_t s) {
  if (a.n_pods <= 0) return hipSuccess;
  MSH_TIMED_LAUNCH(generic_kernel, dim3((unsigned)((a.n_pods + GEN_PB - 1) / GEN_PB)), dim3(GEN_THREADS), 0, s, a);
  return hipGetLastError();
}

// Decode globally merged shard keys (after an element-wise MAX across node shards).
__global__ __launch_bounds__(256) void decode_keys_kernel(const int8_t* __restrict__ pod_digit,
                                                          const uint8_t* __restrict__ pod_tol,
                                                          int32_t p, const int32_t* __restrict__ keys,
                                                          int32_t slot1_any, PluginParams pp,
                                                          int32_t* __restrict__ out_idx,
                                                          int64_t* __restrict__ out_score,
                                                          int32_t* __restrict__ out_status) {
  const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= p) return;
  // slot 1: the pod's class key (identity-like modes) or its own non-match key (KX modes)
  const int32_t k0 = keys[j];
  const int32_t k1 = slot1_any ? keys[(size_t)p + (pod_tol[j] ? 1 : 0)] : keys[(size_t)p + j];
  const int32_t ka = slot1_any ? k1 : (k0 > k1 ? k0 : k1);
  auto idx_of = [](int32_t k) -> int64_t { return k ? (int64_t)(GKEY_MAX - k) : -1; };
  const int d = pod_digit[j];
  int32_t oi, ost;
  int64_t osc;
  decode_pod(idx_of(k0), idx_of(k1), idx_of(ka), d >= 0 && d <= 9, pp, &oi, &osc, &ost);
  out_idx[j] = oi;
  if (out_score) out_score[j] = osc;  // optional output
  out_status[j] = ost;
}

// ---------------------------------------------------------------------------------------
// Sequential-commit kernel (BASELINE C5) on the bit-sliced table: ONE workgroup walks the pods
// in order, one pod at a time, and commits each placement before the next pod is decided.
// Word w of the table lives in registers: q = w / RS, lane q % 64 of wave q / 64, slot w % RS (RS
// consecutive words per lane, lanes and waves in List order), all six planes, plus a FULL plane
// with a capacity. Per pod (its code bits and class are wave-uniform here), every lane evaluates
// its words (5 VALU per 32 pairs), turns its first hit into a node index (v_ffbl_b32: the lowest
// set bit, all-ones when there is none), and the wave's first is its first lane with a hit
// (wave_first). NW > 1 waves meet in a triple-buffered LDS slot
// (atomic min) behind one LDS-only barrier. Then decode, output and commit. With
// max_pods_per_node the commit is per pod: the node's pod count (an LDS table when it fits, device
// memory otherwise) and the owning lane sets the node's FULL bit once the count reaches it, so
// later pods see it infeasible. Without a capacity a commit changes nothing a later pod reads:
// the waves decide U = 4 pods per step (independent scan chains, interleaved word by word; with
// NW > 1 one barrier per step), a dedicated FINALIZER wave (NW > 1) decodes and keeps the outputs
// while the scanners go on, and the counts of a block of 64 placements are committed together
// when the block's outputs leave.
// Nothing inside the per-pod loop waits on memory: the barrier fences LDS only (a plain
// __syncthreads() is a workgroup fence over global memory too, `s_waitcnt vmcnt(0)`); outputs
// collect in lanes (lane jl holds pod j0 + jl, two v_writelane_b32 per pod) and leave as one
// coalesced store per 64 pods; the next 64 pods' bytes are requested one block ahead.
// Issue cost: a wave alone on its SIMD issues one instruction per ~4 cycles of any kind, so the
// per-pod instruction count (VALU and SALU alike) is the latency: 55 per pod at RS = 3 without a
// capacity (profiles/r2_pmc_c3.json, SQ_INSTS_* of the C5 launch).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// The wave's smallest value when lanes hold ascending, disjoint ranges (lane l's candidates all
// precede lane l + 1's): the first lane that has one. One ballot, s_ff1 and a readlane instead of a
// 6-step DPP reduction on the per-pod critical path.
// Branch-free: with no lane holding a value the first lane of (m | lane 63) is lane 63, whose
// value is then "none" too.
__device__ __forceinline__ uint32_t wave_first(uint32_t v) {
  const unsigned long long m = __ballot(v != 0xFFFFFFFFu) | (1ull << 63);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, __builtin_ctzll(m));
}

// t | (d ^ p) and ~(t | (x & m)) in one v_bitop3_b32 each, with the pod's mask p / m wave-uniform
// (SGPR) and the node planes in VGPRs: the sequential kernel's form of or_xor_s.
__device__ __forceinline__ uint32_t or_xor_vs(uint32_t t, uint32_t d, uint32_t p) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xf6" : "=v"(r) : "v"(t), "v"(d), "s"(p));
  return r;
}
__device__ __forceinline__ uint32_t nor_and_vs(uint32_t t, uint32_t x, uint32_t m) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x07" : "=v"(r) : "v"(t), "v"(x), "s"(m));
  return r;
}

// a[lane] = va and b[lane] = vb for ONE lane (wave-uniform values and lane): two v_writelane_b32.
// No builtin for it in this compiler. The lane select goes through M0 (a second SGPR operand
// would break the constant-bus limit); M0 is written by the SALU, and only a VALU-written lane
// select needs wait states before v_writelane.
// (M0 is reserved: the backend never allocates it, and nothing else in this file uses it; the
// clobber stays so that a later M0 user is not silently overwritten.)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
// Compile-time loop: f(integral_constant<int, i>) for i in [B, E) while f returns true.
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    if (f(std::integral_constant<int, B>{})) static_for<B + 1, E>(f);
  }
}
// a lane index plus a compile-time offset, kept compile-time when the index is
template <int D, int L>
__device__ __forceinline__ std::integral_constant<int, L + D> lane_plus(std::integral_constant<int, L>) { return {}; }
template <int D>
__device__ __forceinline__ int32_t lane_plus(int32_t l) { return l + D; }

// v_writelane_b32 with the lane as an inline constant
template <int L>
__device__ __forceinline__ void write_lane1(int32_t& a, int32_t va, std::integral_constant<int, L>) {
  va = __builtin_amdgcn_readfirstlane(va);
  asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(a) : "s"(va), "n"(L));
}
template <int L>
__device__ __forceinline__ void write_lane2(int32_t& a, int32_t& b, int32_t va, int32_t vb,
                                            std::integral_constant<int, L>) {
  va = __builtin_amdgcn_readfirstlane(va);
  vb = __builtin_amdgcn_readfirstlane(vb);
  asm volatile("v_writelane_b32 %0, %2, %4\n\tv_writelane_b32 %1, %3, %4" : "+v"(a), "+v"(b)
               : "s"(va), "s"(vb), "n"(L));
}

// (The values are wave-uniform; readfirstlane puts them in SGPRs where the backend holds them in
// VGPRs, e.g. after a broadcast LDS read.)
__device__ __forceinline__ void write_lane1(int32_t& a, int32_t va, int32_t lane) {
  va = __builtin_amdgcn_readfirstlane(va);
  asm volatile("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(a) : "s"(va), "s"(lane) : "m0");
}
__device__ __forceinline__ void write_lane2(int32_t& a, int32_t& b, int32_t va, int32_t vb, int32_t lane) {
  va = __builtin_amdgcn_readfirstlane(va);
  vb = __builtin_amdgcn_readfirstlane(vb);
  asm volatile("s_mov_b32 m0, %4\n\tv_writelane_b32 %0, %2, m0\n\tv_writelane_b32 %1, %3, m0"
               : "+v"(a), "+v"(b)
               : "s"(va), "s"(vb), "s"(lane)
               : "m0");
}
#pragma clang diagnostic pop

// Lowest set bit (v_ffbl_b32): 0xFFFFFFFF when x == 0, so (base | ffbl(x)) is "no node" then.
__device__ __forceinline__ uint32_t ffbl(uint32_t x) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// U: pods decided per step (U > 1 only for one wave without a capacity; U divides 64).
template <int RS, int NW, bool KX, bool CAP, int U>
__global__ __launch_bounds__((NW + ((!CAP && NW > 1) ? 1 : 0)) * 64) void seq_kernel(SeqArgs a) {
  static_assert(U == 1 || !CAP, "pods are decided ahead of commits only when no commit feeds a decision");
  constexpr bool FIN = !CAP && NW > 1;  // a finalizer wave decodes, keeps the outputs and commits
  constexpr int FINW = FIN ? NW : 0;    // the wave that keeps the outputs
  constexpr bool LDSC = NW <= 4;        // counts in LDS (up to 4 waves x 64 lanes x 4 words x 32
                                        // nodes = 32,768 nodes, 128 KB), else in device memory
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  // per-step exchange slots (NW > 1), triple-buffered: [slot][pod of the step][first match, first
  // feasible, first feasible non-match]
  __shared__ uint32_t xs[3][U][3];
  extern __shared__ int32_t lcnt[];  // [n_pad] per-node pod counts (LDSC)
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = NW == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool scanner = !FIN || wv < NW;

  uint32_t D0[RS], D1[RS], D2[RS], D3[RS], XX[RS], VV[RS], FULL[RS];
#pragma unroll
  for (int r = 0; r < RS; ++r) {
    const int32_t w = (wv * WAVE + lane) * RS + r;
    D0[r] = D1[r] = D2[r] = D3[r] = 0xFFFFFFFFu;  // code 15: never a match
    XX[r] = 0u;
    VV[r] = 0u;
    FULL[r] = 0u;
    if (scanner && w < a.n_words) {
      const uint32_t* g = a.planes + (size_t)(w / PLANE_GW) * GROUP_DWORDS + w % PLANE_GW;
      D0[r] = g[0];
      D1[r] = g[PLANE_GW];
      D2[r] = g[2 * PLANE_GW];
      D3[r] = g[3 * PLANE_GW];
      XX[r] = g[PLANE_X * PLANE_GW];
      VV[r] = g[PLANE_V * PLANE_GW];
      if (CAP) {  // counts carried over from earlier calls: nodes already full
        for (int b = 0; b < 32; ++b)
          FULL[r] |= (a.counts[w * 32 + b] >= a.max_pods ? 1u : 0u) << b;
      }
    }
  }
  if (LDSC)  // ordered before the first commit by the first pod's exchange / barrier
    for (int32_t i = threadIdx.x; i < a.n_words * 32; i += blockDim.x) lcnt[i] = a.counts[i];
  if (threadIdx.x < 9 * U) (&xs[0][0][0])[threadIdx.x] = NONE;
  __syncthreads();
  int sl = 0;
  // Drain the node-state loads here: otherwise the waitcnt pass, unsure they have landed on every
  // path, waits for every outstanding load (the pod prefetch included) inside the loop.
  __builtin_amdgcn_s_waitcnt(0);

  // Pods in lanes, 64 at a time: raw bytes loaded one block ahead (clamped index: no branch around
  // the load), converted only when their block starts, so the loop never waits on them.
  auto load_raw = [&](int32_t j0, int32_t& dr, int32_t& tr) {
    const int32_t jj = min(j0 + lane, a.n_pods - 1);
    dr = a.pod_digit[jj];
    tr = a.pod_tol[jj];
  };
  // Loop-invariant arguments pinned in SGPRs: otherwise the backend re-loads them from the
  // kernel-argument segment inside the loop, and each reload's lgkmcnt wait lands in front of the
  // LDS exchange.
  PluginParams pp = a.pp;
  asm volatile("" : "+s"(pp.has_nu_filter), "+s"(pp.has_nn_score), "+s"(pp.nn_prescore), "+s"(pp.mode),
               "+s"(pp.weight));
  int32_t max_pods = a.max_pods;
  asm volatile("" : "+s"(max_pods));
  const uint32_t ball0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.ball[0]);
  const uint32_t ball1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.ball[1]);
  int32_t* counts = a.counts;
  const IdentDecode idec = make_ident_decode(pp);
  // first feasible node of each pod class (no capacity: constant over the launch), -1 = none
  const int32_t ia0 = ball0 ? (int32_t)(KMAX - ball0) : -1, ia1 = ball1 ? (int32_t)(KMAX - ball1) : -1;
  // A pod's lane word: code | does-not-tolerate << 4 | class status << 5 (bit 4 set for pods that
  // do not tolerate, so one sign-extending bit extract gives the ~tolerates mask), where the class status is
  // decode_ident's status, which without a capacity depends on the pod's class alone (FitError when
  // the class has no feasible node, the NodeNumber score error for a pod without a digit): worked
  // out here once per 64 pods by the lanes, not per pod by the scalar unit.
  auto convert = [&](int32_t j0, int32_t dr, int32_t tr, uint32_t& pk) {
    const bool ok = j0 + lane < a.n_pods;
    const bool dig = ok && dr >= 0 && dr <= 9, tl = ok && tr != 0;
    const bool fit = (tl ? ia1 : ia0) < 0;
    const bool serr = !fit && (idec.err_all || (idec.err_nodigit && !dig));
    const uint32_t st = fit ? 1u : (serr ? 2u : 0u);
    pk = (dig ? (uint32_t)dr : CODE_NONE_POD) | (tl ? 0u : 16u) | (st << 5);
  };
  const uint32_t lane_base = (uint32_t)((wv * WAVE + lane) * RS) << 5;  // node index of bit 0 of slot 0's word
  // the one non-zero score a decode can give (decode_ident: weight x 10 or 100; decode_pod: x 100)
  const int64_t sm = KX ? 100 * pp.weight : idec.sm;
  uint32_t pkv = CODE_NONE_POD;  // lane jl: pod j0 + jl's lane word
  int32_t dn = 0, tn = 0;
  if (a.n_pods > 0) load_raw(0, dn, tn);
  // wave FINW: lane jl holds pod j0 + jl's result, written by v_writelane_b32 as the pod is decided:
  // without a capacity only what the scan found (first match o_a; first non-match o_b in the KX
  // modes), decoded by the lanes together once per 64 pods; with a capacity the decoded node (o_a)
  // and status | scored << 2 (o_b), since every commit needs them at once
  int32_t o_a = -1, o_b = -1;
  auto store_block = [&](int32_t j0, int32_t cnt, uint32_t pk) {  // wave FINW: one coalesced store per array
    if (lane < cnt) {
      int32_t sel, st;
      int64_t sc;
      if constexpr (CAP) {
        sel = o_a;
        st = o_b & 3;
        sc = (o_b & 4) ? sm : 0;
      } else {
        const uint32_t cm = (uint32_t)o_a, tol = ((pk >> 4) & 1u) ^ 1u;
        const int32_t ia = tol ? ia1 : ia0;
        if constexpr (KX) {
          decode_pod(cm != NONE ? (int64_t)cm : -1, (uint32_t)o_b != NONE ? (int64_t)(uint32_t)o_b : -1, ia,
                     (pk & 15u) != CODE_NONE_POD, pp, &sel, &sc, &st);
        } else {  // decode_ident with the class status from the lane word
          st = (int32_t)((pk >> 5) & 3u);
          const bool hit = idec.use_im && cm != NONE;
          sel = st ? -1 : (hit ? (int32_t)cm : ia);
          sc = (hit && st == 0) ? idec.sm : 0;
        }
      }
      a.out_idx[j0 + lane] = sel;
      if (a.out_score) a.out_score[j0 + lane] = sc;  // optional output
      a.out_status[j0 + lane] = st;
      // Without a capacity no decision reads a count, so the block's placements are committed
      // here, one atomic per lane (NodeInfo.AddPod analogue), instead of one per pod.
      if (!CAP && st == 0) {
        if (LDSC) atomicAdd(&lcnt[sel], 1);
        else atomicAdd(&counts[sel], 1);
      }
    }
  };
  // One step: the U pods from pod j on, whose lanes start at jl0 (an int, or without a capacity a
  // compile-time constant: a block's 64 / U steps are unrolled, so readlane and v_writelane take
  // the lane as an inline constant, with no lane arithmetic and no M0). Returns false to end the
  // block early (never; the caller checks the pod count).
  auto step = [&](int32_t j, auto jl0) -> bool {
      // ---- decide: the U pods' scans (U > 1 only without a capacity, where no commit feeds a
      // later decision: independent chains, interleaved word by word) ----
      uint32_t pku[U], p0[U], p1[U], p2[U], p3[U], ntu[U], cmu[U], cau[U], cxu[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        pku[u] = (uint32_t)__builtin_amdgcn_readlane((int)pkv, (int32_t)jl0 + u);
        // the pod's code bits as all-ones / all-zero masks, and ~tolerates: wave-uniform (SGPRs)
        p0[u] = 0u - (pku[u] & 1u);
        p1[u] = 0u - ((pku[u] >> 1) & 1u);
        p2[u] = 0u - ((pku[u] >> 2) & 1u);
        p3[u] = 0u - ((pku[u] >> 3) & 1u);
        ntu[u] = 0u - ((pku[u] >> 4) & 1u);
        cmu[u] = cau[u] = cxu[u] = NONE;  // this lane's first match / feasible / non-match
      }
      if (scanner) {
#pragma unroll
        for (int r = RS - 1; r >= 0; --r) {  // slots ascend in List order per lane
          const uint32_t base = lane_base + (uint32_t)(r * 32);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            uint32_t dm = D0[r] ^ p0[u];
            dm = or_xor_vs(dm, D1[r], p1[u]);
            dm = or_xor_vs(dm, D2[r], p2[u]);
            dm = or_xor_vs(dm, D3[r], p3[u]);
            if constexpr (!CAP && !KX) {
              cmu[u] = umin(cmu[u], base | ffbl(nor_and_vs(dm, XX[r], ntu[u])));
            } else {
              const uint32_t bad = (XX[r] & ntu[u]) | (CAP ? FULL[r] : 0u);
              cmu[u] = umin(cmu[u], base | ffbl(~(dm | bad)));
              if (CAP) cau[u] = umin(cau[u], base | ffbl(VV[r] & ~bad));
              if (KX) cxu[u] = umin(cxu[u], base | ffbl(VV[r] & ~bad & dm));
            }
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          cmu[u] = wave_first(cmu[u]);
          if (CAP) cau[u] = wave_first(cau[u]);
          if (KX) cxu[u] = wave_first(cxu[u]);
        }
      }
      // ---- exchange (NW > 1): lane 0 of every scanning wave folds its wave's results for the step's
      // U pods into their slots; after ONE barrier each pod's result is one broadcast read ----
      if constexpr (NW > 1) {
        if (scanner && lane == 0) {
#pragma unroll
          for (int u = 0; u < U; ++u) {
            atomicMin(&xs[sl][u][0], cmu[u]);
            if (CAP) atomicMin(&xs[sl][u][1], cau[u]);
            if (KX) atomicMin(&xs[sl][u][2], cxu[u]);
          }
        }
        lds_barrier();
        const int sl_now = sl;
        sl = sl == 2 ? 0 : sl + 1;
        if (!CAP && wv != FINW) return true;  // without a capacity only the finalizer finishes a pod
#pragma unroll
        for (int u = 0; u < U; ++u) {
          cmu[u] = xs[sl_now][u][0];
          if (CAP) cau[u] = xs[sl_now][u][1];
          if (KX) cxu[u] = xs[sl_now][u][2];
        }
        // the slot read one step ago is free now (every reader passed this step's barrier) and is
        // next folded into two steps ahead (after the next barrier): wave FINW resets it in between
        if (wv == FINW && lane < 3 * U) (&xs[sl_now == 0 ? 2 : sl_now - 1][0][0])[lane] = NONE;
      }
      // ---- then, in pod order: keep the result in its lane (decoded per 64 pods) or, with a
      // capacity, decode, keep and commit ----
      if constexpr (!CAP) {
        if (wv == FINW) {
          static_for<0, U>([&](auto uc) {
            constexpr int u = decltype(uc)::value;
            const auto jl = lane_plus<u>(jl0);
            if (KX) write_lane2(o_a, o_b, (int32_t)cmu[u], (int32_t)cxu[u], jl);
            else write_lane1(o_a, (int32_t)cmu[u], jl);
            return true;
          });
        }
        return true;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int32_t jl = (int32_t)jl0 + u;
        const uint32_t pc = pku[u] & 15u;
        const uint32_t cm = cmu[u], ca = cau[u], cx = cxu[u];
        const int64_t im = cm != NONE ? (int64_t)cm : -1;
        const int64_t ia = ca != NONE ? (int64_t)ca : -1;
        int32_t sel, st;
        int64_t sc;
        if (KX)
          decode_pod(im, cx != NONE ? (int64_t)cx : -1, ia, pc != CODE_NONE_POD, pp, &sel, &sc, &st);
        else
          decode_ident(im, ia, pc != CODE_NONE_POD, idec, &sel, &sc, &st);
        if (wv == FINW) write_lane2(o_a, o_b, sel, st | (sc != 0 ? 4 : 0), jl);
        if (st == 0) {  // commit, seen by the next pod's decision
          const uint32_t w = (uint32_t)sel >> 5, q = w / RS;
          if ((int)(q / WAVE) == wv) {  // the owning wave
            int32_t old = 0;
            if (lane == 0) old = LDSC ? atomicAdd(&lcnt[sel], 1) : atomicAdd(&counts[sel], 1);
            const bool full = __builtin_amdgcn_readfirstlane(old) + 1 >= max_pods;
            if (full) {
              // the owning lane: the register by a wave-uniform index (scalar branches), the lane
              // by a compare
              const int rs = (int)(w % RS);
              const uint32_t bit = (lane == (int)(q % WAVE)) ? (1u << (sel & 31)) : 0u;
#pragma unroll
              for (int r = 0; r < RS; ++r)
                if (r == rs) FULL[r] |= bit;
            }
          }
        }
      }
      return true;
  };
  for (int32_t jb = 0; jb < a.n_pods; jb += WAVE) {
    // order matters for vmcnt (in-order): the conversion waits only for the loads issued one
    // block ago, then the previous block's results leave, then the next block is requested
    const uint32_t pk_done = pkv;  // the previous block's lane words, for its decode
    convert(jb, dn, tn, pkv);
    if (wv == FINW && jb > 0) store_block(jb - WAVE, WAVE, pk_done);
    load_raw(jb + WAVE, dn, tn);
    if constexpr (!CAP) {
      static_for<0, WAVE / U>([&](auto sc) {
        constexpr int JL = decltype(sc)::value * U;
        if (jb + JL >= a.n_pods) return false;
        return step(jb + JL, std::integral_constant<int, JL>{});
      });
    } else {
      const int32_t je = min(jb + WAVE, a.n_pods);
      for (int32_t j = jb; j < je; j += U) step(j, (int32_t)(j - jb));
    }
  }

  if (wv == FINW && a.n_pods > 0) {
    const int32_t j0 = (a.n_pods - 1) & ~(WAVE - 1);
    store_block(j0, a.n_pods - j0, pkv);
  }
  if (LDSC) {
    __syncthreads();
    for (int32_t i = threadIdx.x; i < a.n_words * 32; i += blockDim.x) a.counts[i] = lcnt[i];
  }
}


// ---------------------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------------------
// Before every prep: reset the first feasible node per class and apply pending msh_patch_nodes
// entries (idx | unsched << 32 | digit << 40). One launch instead of a memset and a scatter.
__global__ __launch_bounds__(256) void prep_reset_kernel(uint32_t* __restrict__ ball,
                                                         const unsigned long long* __restrict__ entries,
                                                         int32_t count, uint8_t* __restrict__ unsched,
                                                         int8_t* __restrict__ digit) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 2) ball[i] = 0;
  if (i < count) {
    const unsigned long long e = entries[i];
    const uint32_t k = (uint32_t)e;
    unsched[k] = (uint8_t)(e >> 32);
    digit[k] = (int8_t)(uint8_t)(e >> 40);
  }
}

// The first-node offsets of every (group, pod class) behind the class rows (msh_internal.h HR_FIRST):
// one thread per (group, kind, class) slot, after node_prep_kernel has written the rows.
__global__ __launch_bounds__(256) void hr_first_kernel(uint32_t* __restrict__ hrows, int32_t n_groups) {
  const int32_t i = (int32_t)(blockIdx.x * 256 + threadIdx.x);
  if (i >= n_groups * 2 * HR_CLS) return;
  const int32_t g = i / (2 * HR_CLS), j = i - g * (2 * HR_CLS);
  const uint32_t kind = (uint32_t)j / HR_CLS, cls = (uint32_t)j - kind * HR_CLS;
  uint16_t* out = reinterpret_cast<uint16_t*>(hrows + (size_t)g * HR_GD + HR_FIRST * 4) + j;
  if (cls >= 2 * ER_ROWS) {
    *out = HR_NONE;
    return;
  }
  const uint32_t t = cls >= ER_ROWS ? 1u : 0u, r = cls - t * ER_ROWS;
  const uint4* tg = reinterpret_cast<const uint4*>(hrows + (size_t)g * HR_GD);
  const uint4 w0 = tg[hr_entry(0, t, r)], w1 = tg[hr_entry(1, t, r)];
  uint32_t h[PLANE_GW] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
  if (kind == 1) {  // the feasible non-matches F[t] & ~H[t][r]
    const uint4 f0 = tg[HR_F + 2 * t], f1 = tg[HR_F + 2 * t + 1];
    const uint32_t f[PLANE_GW] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
#pragma unroll
    for (int k = 0; k < PLANE_GW; ++k) h[k] = f[k] & ~h[k];
  }
  const uint32_t m = hits_first(h, 0);
  *out = (uint16_t)(m < GROUP_NODES ? m : HR_NONE);
}

hipError_t launch_node_prep(const uint8_t* d_unsched, const int8_t* d_digit, int32_t n, int32_t n_pad,
                            int32_t has_nu, uint32_t* d_ball, uint32_t* d_planes, uint32_t* d_erows,
                            uint32_t* d_hrows, hipStream_t s, const unsigned long long* d_patch, int32_t patch_count) {
  hipLaunchKernelGGL(prep_reset_kernel, dim3(patch_count > 0 ? (patch_count + 255) / 256 : 1), dim3(256), 0, s,
                     d_ball, d_patch, patch_count, const_cast<uint8_t*>(d_unsched), const_cast<int8_t*>(d_digit));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (n_pad == 0) return hipSuccess;
  hipLaunchKernelGGL(node_prep_kernel, dim3(n_pad / PREP_THREADS), dim3(PREP_THREADS), 0, s, d_unsched, d_digit, n,
                     has_nu, d_ball, d_planes, d_erows, d_hrows);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const int32_t slots = n_pad / GROUP_NODES * 2 * HR_CLS;
  hipLaunchKernelGGL(hr_first_kernel, dim3((slots + 255) / 256), dim3(256), 0, s, d_hrows, n_pad / GROUP_NODES);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Per-pair plugin results (debug / simulator result store). One workgroup
// per pod: pass 1 ORs "feasible match" / "feasible non-match" over the List to get the
// extent NormalizeScore needs; pass 2 writes, for every node i,
//   filter[i] = 1 passed / 0 rejected by NodeUnschedulable,
//   raw[i]    = NodeNumber.Score (10 on a digit match, else 0),
//   final[i]  = NormalizeScore(raw)[i] * weight,
// with raw/final = EXPORT_NONE where the reference records no score (infeasible node, or the
// pod never reaches Score: no feasible node / PreScore failed / no score plugin).
// Not a hot path: O(P*N) writes of 17 B per pair.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void export_kernel(const uint8_t* __restrict__ unsched,
                                                     const int8_t* __restrict__ digit, int32_t n,
                                                     const int8_t* __restrict__ pod_digit,
                                                     const uint8_t* __restrict__ pod_tol,
                                                     PluginParams pp, uint8_t* __restrict__ filter,
                                                     int64_t* __restrict__ raw,
                                                     int64_t* __restrict__ fin) {
  __shared__ int flags;  // bit0 feasible match, bit1 feasible non-match
  const int32_t j = blockIdx.x;
  const int pd = pod_digit[j];
  const bool pd_valid = pd >= 0 && pd <= 9;
  const bool tol = pod_tol[j] != 0;
  if (threadIdx.x == 0) flags = 0;
  __syncthreads();
  int f = 0;
  for (int32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const bool feas = !(pp.has_nu_filter && unsched[i] && !tol);
    const int d = digit[i];
    if (feas) f |= (pd_valid && d == pd) ? 1 : 2;
  }
  if (f) atomicOr(&flags, f);
  __syncthreads();
  const bool hm = flags & 1, hx = flags & 2;
  const bool scored = (hm || hx) && pp.has_nn_score && pp.nn_prescore && pd_valid;
  const int64_t w = pp.weight;
  const size_t row = (size_t)j * (size_t)n;
  for (int32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const bool feas = !(pp.has_nu_filter && unsched[i] && !tol);
    filter[row + i] = feas ? 1 : 0;
    int64_t r = EXPORT_NONE, o = EXPORT_NONE;
    if (scored && feas) {
      const bool m = digit[i] == pd;
      r = m ? 10 : 0;
      switch (pp.mode) {
        case 1: o = m ? 100 : 0; break;                      // max is 10 whenever a match exists
        case 2: o = hm ? (m ? 0 : 100) : 100; break;         // reverse; max 0 -> all 100
        case 3: o = (hm && hx) ? (m ? 100 : 0) : 0; break;   // min-max; max == min -> 0
        default: o = r; break;
      }
      o *= w;
    }
    raw[row + i] = r;
    fin[row + i] = o;
  }
}

hipError_t launch_export(const uint8_t* d_unsched, const int8_t* d_digit, int32_t n,
                         const int8_t* d_pod_digit, const uint8_t* d_pod_tol, int32_t p,
                         const PluginParams& pp, uint8_t* d_filter, int64_t* d_raw, int64_t* d_fin,
                         hipStream_t s) {
  if (p <= 0 || n <= 0) return hipSuccess;
  hipLaunchKernelGGL(export_kernel, dim3(p), dim3(256), 0, s, d_unsched, d_digit, n, d_pod_digit,
                     d_pod_tol, pp, d_filter, d_raw, d_fin);
  return hipGetLastError();
}

namespace {
// Slice waves per 64-pod block of the bit-sliced kernel: enough waves for ~6 per SIMD, each
// slice at least two groups (512 nodes) so the per-wave fixed cost (pod bytes, the first-node
// decode, the LDS merge) stays small next to the scan.
int bits_slices(int64_t n_pods, int32_t n_groups, const DeviceInfo& dev) {
  if (dev.bits_slices > 0) return dev.bits_slices;
  const int64_t blocks = (n_pods + WAVE - 1) / WAVE;
  const int64_t want = (int64_t)dev.cus * 4 * 6;
  int sl = 1;
  while (sl < 16 && blocks * sl < want && n_groups / (2 * sl) >= 2) sl *= 2;
  return sl;
}

template <int S, bool KX, bool SHARD>
hipError_t launch_bits_s(const BatchArgs& a, hipStream_t s) {
  BatchArgs ka = a;
  ka.gps = (a.n_groups + S - 1) / S;
  const int64_t blocks = ((int64_t)a.n_pods + WAVE - 1) / WAVE;
  MSH_TIMED_LAUNCH((bits_kernel<S, KX, SHARD>), dim3((unsigned)blocks), dim3(S * WAVE), 0, s, ka);
  return hipGetLastError();
}

template <int S, bool KX, bool SHARD, int PPL>
hipError_t launch_rows_s(const BatchArgs& a, hipStream_t s) {
  BatchArgs ka = a;
  ka.gps = (a.n_groups + S - 1) / S;
  const int64_t blocks = ((int64_t)a.n_pods + PPL * WAVE - 1) / (PPL * WAVE);
  MSH_TIMED_LAUNCH((rows_kernel<S, KX, SHARD, PPL>), dim3((unsigned)blocks), dim3(S * WAVE), 0, s, ka);
  return hipGetLastError();
}

template <bool KX, bool SHARD, int PPL>
hipError_t launch_rows_p(const BatchArgs& a, const DeviceInfo& dev, hipStream_t s) {
  // slices for the launch's pod blocks of PPL * 64 pods
  switch (bits_slices((a.n_pods + PPL - 1) / PPL, a.n_groups, dev)) {
    case 1: return launch_rows_s<1, KX, SHARD, PPL>(a, s);
    case 2: return launch_rows_s<2, KX, SHARD, PPL>(a, s);
    case 4: return launch_rows_s<4, KX, SHARD, PPL>(a, s);
    case 8: return launch_rows_s<8, KX, SHARD, PPL>(a, s);
    default: return launch_rows_s<16, KX, SHARD, PPL>(a, s);
  }
}

template <bool KX, bool SHARD>
hipError_t launch_rows_t(const BatchArgs& a, const DeviceInfo& dev, hipStream_t s) {
  if constexpr (KX)  // (two pods per lane, an A/B of the identity modes, would spill here)
    return launch_rows_p<KX, SHARD, 1>(a, dev, s);
  else
    return dev.rows_ppl == 1 ? launch_rows_p<KX, SHARD, 1>(a, dev, s) : launch_rows_p<KX, SHARD, 2>(a, dev, s);
}

// Waves per workgroup of wg_kernel: 4 (one staged copy of the table per 256 pods), or 8 (A/B,
// MSH_WG_WAVES=8).
int wg_waves(int64_t n_pods, const DeviceInfo& dev) {
  (void)n_pods;
  return dev.wg_waves == 8 ? 8 : 4;
}

template <int W, bool KX, bool SHARD>
hipError_t launch_wg_w(const BatchArgs& a, hipStream_t s) {
  const int64_t blocks = ((int64_t)a.n_pods + W * WAVE - 1) / (W * WAVE);
  MSH_TIMED_LAUNCH((wg_kernel<W, KX, SHARD, false>), dim3((unsigned)blocks), dim3(W * WAVE), 0, s, a);
  return hipGetLastError();
}

// The persistent kernel over m.nb batches of m.bpb 256-pod blocks: as many workgroups as stay
// resident (8 per CU: 32 waves, the CU's limit; fewer when the table's LDS copy limits them), never
// more than the launch's blocks.
template <bool KX>
hipError_t launch_persistent(MultiArgs& m, const DeviceInfo& dev, hipStream_t s) {
  constexpr int W = MSH_WGP_W;
  int32_t maxp = 0;
  for (int b = 0; b < m.nb; ++b) maxp = std::max(maxp, m.d[b].n_pods);
  if (maxp == 0) return hipSuccess;
  m.bpb = (maxp + W * WAVE - 1) / (W * WAVE);
  const size_t lds = (size_t)m.a.n_groups * HR_GQ * sizeof(uint4);
  const int64_t per_cu = std::max<int64_t>(1, std::min<int64_t>(32 / W, (int64_t)(160 * 1024 / std::max<size_t>(lds, 1))));
  const int64_t items = (int64_t)m.bpb * m.nb;
  const int64_t grid = std::min<int64_t>(items, (int64_t)dev.cus * per_cu);
  // Item shares by age slot (blockIdx / CUs: the dispatcher fills every CU's slot r before slot r + 1)
  // when the grid fills every slot and each workgroup has at least WGP_SHARE_MIN items: slot r's
  // share falls by MSH_WGP_AGE_SLOPE / 1000 per slot relative to slot 0 (the rates of the slots
  // measured under equal shares); otherwise the strided walk (C3, 32 batches per launch: 0.815 ->
  // 0.777 us per batch; at 8 and 20 batches the strided walk was as fast or faster).
  m.walk = 0;
  if (grid == (int64_t)dev.cus * per_cu && per_cu > 1 && items >= WGP_SHARE_MIN * grid) {
    m.walk = 1;
    m.rank_wgs = dev.cus;
    double wsum = 0, w[RANK_MAX];
    for (int r = 0; r < per_cu; ++r) wsum += (w[r] = 1.0 - MSH_WGP_AGE_SLOPE * 1e-3 * r);
    double acc = 0;
    for (int r = 0; r <= per_cu; ++r) {
      m.rank_lo[r] = (int32_t)std::llround(items * acc / wsum);
      if (r < per_cu) acc += w[r];
    }
    m.rank_lo[per_cu] = (int32_t)items;
  } else {
    m.rank_wgs = (int32_t)grid;
    m.rank_lo[0] = 0;
    m.rank_lo[1] = (int32_t)items;
  }
  MSH_TIMED_LAUNCH((wgp_kernel<W, KX>), dim3((unsigned)grid), dim3(W * WAVE), (unsigned)lds, s, m);
  return hipGetLastError();
}

bool use_persistent(const BatchArgs& a, const DeviceInfo& dev) {
  return a.n_groups <= WGP_MAX_GROUPS && !dev.wg_no_persist;
}

template <bool KX>
hipError_t launch_single_persistent(const BatchArgs& a, const DeviceInfo& dev, hipStream_t s) {
  MultiArgs m{};
  m.a = a;
  m.nb = 1;
  m.d[0] = BatchDesc{a.pod_digit, a.pod_tol, a.out_idx, a.out_score, a.out_status, a.n_pods, 0};
  return launch_persistent<KX>(m, dev, s);
}

template <bool KX, bool SHARD>
hipError_t launch_wg_t(const BatchArgs& a, const DeviceInfo& dev, hipStream_t s) {
  if constexpr (!SHARD) {
    if (use_persistent(a, dev)) return launch_single_persistent<KX>(a, dev, s);
  }
  switch (wg_waves(a.n_pods, dev)) {
    case 8: return launch_wg_w<8, KX, SHARD>(a, s);
    default: return launch_wg_w<4, KX, SHARD>(a, s);
  }
}

template <int W, bool KX>
hipError_t launch_multi_w(MultiArgs& m, const DeviceInfo& dev, hipStream_t s) {
  if (use_persistent(m.a, dev)) return launch_persistent<KX>(m, dev, s);
  int32_t blocks = 0;  // per batch: the largest batch's
  for (int b = 0; b < m.nb; ++b) blocks = std::max(blocks, (m.d[b].n_pods + W * WAVE - 1) / (W * WAVE));
  if (blocks == 0) return hipSuccess;
  m.bpb = blocks;
  MSH_TIMED_LAUNCH((wg_kernel<W, KX, false, true>), dim3((unsigned)blocks, (unsigned)m.nb), dim3(W * WAVE), 0, s, m);
  return hipGetLastError();
}

template <bool KX, bool SHARD>
hipError_t launch_bits_t(const BatchArgs& a, const DeviceInfo& dev, hipStream_t s) {
  switch (bits_slices(a.n_pods, a.n_groups, dev)) {
    case 1: return launch_bits_s<1, KX, SHARD>(a, s);
    case 2: return launch_bits_s<2, KX, SHARD>(a, s);
    case 4: return launch_bits_s<4, KX, SHARD>(a, s);
    case 8: return launch_bits_s<8, KX, SHARD>(a, s);
    default: return launch_bits_s<16, KX, SHARD>(a, s);
  }
}
}  // namespace

hipError_t launch_batch(const BatchArgs& a, bool shard, const DeviceInfo& dev, hipStream_t s) {
  if (a.n_pods == 0) return hipSuccess;
  const bool kx = needs_kx(a.pp);
  // every mode on the digit rows (REVERSE / MINMAX also track the first feasible non-match)
  if (kx && dev.kx_bits)  // A/B: the code-plane kernel for REVERSE / MINMAX
    return shard ? launch_bits_t<true, true>(a, dev, s) : launch_bits_t<true, false>(a, dev, s);
  if (dev.batch_kernel == 1) {  // A/B: the round-2 slice kernel
    if (shard) return kx ? launch_rows_t<true, true>(a, dev, s) : launch_rows_t<false, true>(a, dev, s);
    return kx ? launch_rows_t<true, false>(a, dev, s) : launch_rows_t<false, false>(a, dev, s);
  }
  if (shard) return kx ? launch_wg_t<true, true>(a, dev, s) : launch_wg_t<false, true>(a, dev, s);
  return kx ? launch_wg_t<true, false>(a, dev, s) : launch_wg_t<false, false>(a, dev, s);
}

hipError_t launch_batches(const BatchArgs& a, const BatchDesc* d, int nb, const DeviceInfo& dev, hipStream_t s) {
  if (nb <= 0 || nb > MULTI_MAX) return hipErrorInvalidValue;
  MultiArgs m{};
  m.a = a;
  m.nb = nb;
  int64_t pods = 0;
  for (int b = 0; b < nb; ++b) {
    m.d[b] = d[b];
    pods += d[b].n_pods;
  }
  const bool kx = needs_kx(a.pp);
  switch (wg_waves(pods, dev)) {
    case 8: return kx ? launch_multi_w<8, true>(m, dev, s) : launch_multi_w<8, false>(m, dev, s);
    default: return kx ? launch_multi_w<4, true>(m, dev, s) : launch_multi_w<4, false>(m, dev, s);
  }
}

hipError_t launch_decode_keys(const int8_t* pod_digit, const uint8_t* pod_tol, int32_t p,
                              const int32_t* keys, int32_t slot1_any, PluginParams pp,
                              int32_t* out_idx, int64_t* out_score, int32_t* out_status,
                              hipStream_t s) {
  if (p == 0) return hipSuccess;
  hipLaunchKernelGGL(decode_keys_kernel, dim3((p + 255) / 256), dim3(256), 0, s, pod_digit, pod_tol, p, keys,
                     slot1_any, pp, out_idx, out_score, out_status);
  return hipGetLastError();
}

namespace {
constexpr int SEQ_AHEAD = 4;  // pods decided per step without a capacity

template <int RS, int NW, bool CAP>
hipError_t launch_seq_rs(const SeqArgs& a, hipStream_t s) {
  const dim3 blk((NW + ((!CAP && NW > 1) ? 1 : 0)) * 64);  // + the finalizer wave without a capacity
  const size_t lds = NW <= 4 ? (size_t)a.n_words * 32 * sizeof(int32_t) : 0;  // seq_kernel's LDSC
  constexpr int U = !CAP ? SEQ_AHEAD : 1;
  auto kx = seq_kernel<RS, NW, true, CAP, U>;
  auto id = seq_kernel<RS, NW, false, CAP, U>;
  const void* k = needs_kx(a.pp) ? reinterpret_cast<const void*>(kx) : reinterpret_cast<const void*>(id);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  if (needs_kx(a.pp)) MSH_TIMED_LAUNCH(kx, dim3(1), blk, lds, s, a);
  else MSH_TIMED_LAUNCH(id, dim3(1), blk, lds, s, a);
  return hipGetLastError();
}

template <int NW, bool CAP>
hipError_t launch_seq_nw(const SeqArgs& a, int rs, hipStream_t s) {
  if constexpr (NW == 1) {
    if (rs <= 1) return launch_seq_rs<1, NW, CAP>(a, s);
    if (rs <= 2) return launch_seq_rs<2, NW, CAP>(a, s);
    if (rs <= 3) return launch_seq_rs<3, NW, CAP>(a, s);
    return launch_seq_rs<4, NW, CAP>(a, s);
  } else if constexpr (NW == 4) {
    if (rs <= 2) return launch_seq_rs<2, NW, CAP>(a, s);
    return launch_seq_rs<4, NW, CAP>(a, s);
  } else {
    if (rs <= 4) return launch_seq_rs<4, NW, CAP>(a, s);
    if (CAP || rs <= 8) return launch_seq_rs<8, NW, CAP>(a, s);
    return launch_seq_rs<(CAP ? 8 : 12), NW, CAP>(a, s);  // (CAP at 12 words per lane spills)
  }
}
}  // namespace

// Scanning waves: as few as keep at most 4 words per lane (one wave up to 8,192 nodes, four up to
// 32,768), then 15 (+ the finalizer) waves with up to 12 words per lane without a capacity
// (368,640 nodes; 6 x 12 plane VGPRs per lane), 16 waves with up to 8 with one (262,144 nodes; the
// FULL plane makes 7 per word, and 12 words spill). Per-pod latency is one wave's scan plus one DPP
// reduction; extra waves add an LDS exchange and a barrier.
hipError_t launch_sequential(const SeqArgs& a, const DeviceInfo& dev, hipStream_t s, std::string* err) {
  if (a.n_pods == 0) return hipSuccess;
  const bool cap = a.max_pods > 0;
  const int nw_big = cap ? 16 : 15;
  auto rs_for = [&](int nw) { return (a.n_words + nw * WAVE - 1) / (nw * WAVE); };
  int nw = dev.seq_waves > 0 ? dev.seq_waves : (rs_for(1) <= 4 ? 1 : rs_for(4) <= 4 ? 4 : nw_big);
  if (nw != 1 && nw != 4) nw = nw_big;
  const int rs_max = cap ? 8 : 12;
  if (rs_for(nw) > (nw == nw_big ? rs_max : 4)) nw = nw_big;  // an override too small for the table
  const int rs = rs_for(nw);
  if (rs > rs_max) {
    if (err)
      *err = "sequential mode keeps the node table in registers: at most " +
             std::to_string(nw_big * WAVE * rs_max * 32) + " nodes per device" + (cap ? " with a capacity" : "");
    return hipErrorInvalidValue;
  }
  const SeqArgs& ka = a;
  if (cap) {
    if (nw == 1) return launch_seq_nw<1, true>(ka, rs, s);
    if (nw == 4) return launch_seq_nw<4, true>(ka, rs, s);
    return launch_seq_nw<16, true>(ka, rs, s);
  }
  if (nw == 1) return launch_seq_nw<1, false>(ka, rs, s);
  if (nw == 4) return launch_seq_nw<4, false>(ka, rs, s);
  return launch_seq_nw<15, false>(ka, rs, s);
}

#if defined(MSH_STAMPS) || defined(MSH_CLOCK_STAMPS)
extern "C" int msh_stamps_set(void* p) { return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &p, sizeof(p)); }
#endif

}  // namespace msh
