// msh_kernels.hip — gfx950 (MI355X, CDNA4) kernels for the batched pods x nodes hot path.
//
// Reference path (shopetan/mini-kube-scheduler, Go): for ONE pod per cycle,
//   RunFilterPlugins   minisched/minisched.go:115-151  (NodeUnschedulable, upstream v1.22.0)
//   RunPreScorePlugins minisched/minisched.go:153-162  (NodeNumber.PreScore, nodenumber.go:50-64)
//   RunScorePlugins    minisched/minisched.go:164-199  (NodeNumber.Score, nodenumber.go:73-95)
//   selectHost         minisched/minisched.go:304-325  (argmax; ties -> lowest index here)
//
// Every batch kernel puts one POD per lane and reads the node side wave-uniformly (scalar loads into
// SGPRs), so the node data is read once per 64 pods and the vector unit does per-pair work only.
// Kernels, by entry point:
//   node_prep_kernel (+ prep_reset_kernel)  every upload / patch / filter-list change: the bit planes
//                        (pair_kernel, seq_kernel), the node records (generic_kernel), the class rows
//                        and first-node offsets (the opt-in class-row kernel)
//   pair_kernel          msh_schedule_batch*, msh_schedule_batches_device, msh_shard_keys_device for the
//                        reference plugins, every normalize mode (the default batch path): every (pod,
//                        node) pair's filter verdict and NodeNumber score evaluated from the bit planes,
//                        32 pairs per lane-op
//   generic_kernel       any plugin list with an explicit int64 score per pair (score-column plugins;
//                        the node-sharded msh_generic_* entry points): north_star's five stages literally
//                        (feasibility lane masks, weighted int64 totals, per-pod min/max extents with an
//                        LDS reduction, a running first maximum, node tiles read once per wave)
//   wgp_kernel           the opt-in class-row kernel (MSH_BATCH_KERNEL=classrows, tables <= 8,192 nodes)
//   decode_keys_kernel   node-sharded mode: decode the merged per-pod shard keys
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
                                                                 uint32_t* __restrict__ hrows,
                                                                 uint32_t* __restrict__ nrec) {
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
  // the node record of generic_kernel: the code, and the NodeUnschedulable mask (all-ones: every pod
  // passes; 0: only pods that tolerate the taint pass)
  {
    const uint32_t xm = feas0 ? 0xFFFFFFFFu : 0u;
    reinterpret_cast<uint4*>(nrec)[i] = make_uint4(code, 0u, xm, xm);
  }
  // this wave's 64 nodes are words 2t and 2t + 1 of the PLANE_* layout: lanes 0..11 write them
  if (lane < 2 * PLANE_N) {
    const int k = lane >> 1, half = lane & 1;
    unsigned long long m = pm[0];
#pragma unroll
    for (int q = 1; q < PLANE_N; ++q) m = (k == q) ? pm[q] : m;
    const uint32_t word = ((uint32_t)(i - lane) >> 5) + (uint32_t)half;  // i - lane: the wave's first node
    planes[((word / PLANE_GW) * PLANE_N + k) * PLANE_GW + word % PLANE_GW] = (uint32_t)(m >> (32 * half));
  }
  // per digit r, the real nodes with suffix digit r (padding: code 15), for the class rows below
  unsigned long long em[ER_ROWS - 1];
#pragma unroll
  for (int r = 0; r < ER_ROWS - 1; ++r) em[r] = __ballot(code == (uint32_t)r);
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
__device__ __forceinline__ void sload_group(u32x8* pl, const uint32_t* src) {
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

// ---------------------------------------------------------------------------------------
// Per-pair batch kernel: the default batch path (msh_schedule_batch*, msh_schedule_batches_device,
// msh_shard_keys_device) for the reference's plugins, in every normalize mode.
//
// EVERY (pod, node) pair is evaluated, from the node's own bits and the pod's own bits; no table
// indexed by a pod's class (its digit or tolerates bit) is read. "Lanes = pods": lane l of a wave
// holds one pod; the node table is bit-sliced (msh_internal.h PLANE_*: node i is bit i mod 32 of word
// i / 32), and a group's planes are wave-uniform, so they arrive by scalar loads into SGPRs. Per lane
// and word (32 nodes), with the pod's NodeNumber code bits as all-ones / all-zero masks P0..P3 and
// nT = all-ones unless the pod tolerates the unschedulable taint:
//   xi  = X & nT                                  NodeUnschedulable.Filter rejects the pair
//   dm' = xi | (D0 ^ P0) | (D1 ^ P1) | (D2 ^ P2) | (D3 ^ P3)
//         zero exactly at the feasible pairs whose NodeNumber.Score is 10 (suffix digits equal; node
//         code 15 = no digit or padding and pod code 14 = no digit never match)
//   nm  = dm' & ~xi (& V in a group holding padding)   the feasible pairs whose score is 0
// v_and + 4 v_bitop3 for dm', then the group accumulators am = AND of the dm' words (one v_bitop3
// AND3 per two words) and ax |= nm (one v_bitop3 per word): 6.5 VALU per 32 x 64 pairs.
// Stages 2-4 on NodeNumber's two-valued raw score: every total is weight x NormalizeScore(raw) of 0
// or 10, so selectHost's first maximum is the first feasible pair of the better level. A pod
// therefore needs its first feasible match (im) and its first feasible non-match (ix); its first
// feasible node is min(im, ix); decode_pod turns them into the status, the node and the int64 score
// for the plugin list and normalize mode (minisched.go:50-87, 143-148, 164-199, 304-325).
// Groups are walked in DESCENDING List order and a group with a hit is remembered (the last one
// remembered is the first); the lowest group of the wave's range keeps its words in registers for
// the exact node (v_ffbl of each word); a lane whose first hit lies in a higher group re-reads that
// group (vector loads behind an exec-masked branch: rare, a 256-node group nearly always holds a
// feasible node of each digit). S slice waves share a 64-pod block when a launch has few pods for
// the chip: each scans a contiguous range of groups, and their firsts meet by min in LDS (slices
// ascend in List order). The grid is (workgroup blocks x batches): blockIdx.y = the batch of a
// multi-batch launch, its descriptor read by scalar loads.
// ---------------------------------------------------------------------------------------
constexpr int PAIR_WAVES = 4;  // waves per workgroup

__device__ __forceinline__ uint32_t bop3_andn(uint32_t a, uint32_t b) {  // a & ~b
  return __builtin_amdgcn_bitop3_b32(a, b, b, 0x30);
}
__device__ __forceinline__ uint32_t bop3_and3(uint32_t a, uint32_t b, uint32_t c) {  // a & b & c
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x80);
}
__device__ __forceinline__ uint32_t bop3_or_andn(uint32_t acc, uint32_t a, uint32_t b) {  // acc | (a & ~b)
  return __builtin_amdgcn_bitop3_b32(acc, a, b, 0xf4);
}
__device__ __forceinline__ uint32_t bop3_andn_and(uint32_t a, uint32_t b, uint32_t v) {  // a & ~b & v
  return __builtin_amdgcn_bitop3_b32(a, b, v, 0x20);
}

// t | (d ^ p), d the node plane (SGPR), p the pod's mask. The builtin, not inline asm: the backend
// then knows the instruction's hazards (after inline asm it inserts an s_nop every other VALU).
__device__ __forceinline__ uint32_t bop3_or_xor(uint32_t t, uint32_t d, uint32_t p) {
  return __builtin_amdgcn_bitop3_b32(t, d, p, 0xf6);
}

// dm' of word w of a group's planes (SGPRs) for one lane; xi out
__device__ __forceinline__ uint32_t pair_miss(const u32x8 (&pl)[PLANE_N], int w, uint32_t P0, uint32_t P1,
                                              uint32_t P2, uint32_t P3, uint32_t nT, uint32_t& xi) {
  xi = __builtin_amdgcn_bitop3_b32(pl[PLANE_X][w], nT, nT, 0xc0);  // X & nT
  uint32_t t = bop3_or_xor(xi, pl[0][w], P0);
  t = bop3_or_xor(t, pl[1][w], P1);
  t = bop3_or_xor(t, pl[2][w], P2);
  return bop3_or_xor(t, pl[3][w], P3);
}

// One group above the lowest of the range, accumulated into am (AND of the dm' words: not all-ones
// iff a feasible match) and, KX, ax (OR of the feasible non-match words).
template <bool PAD, bool KX>
__device__ __forceinline__ void pair_group(const u32x8 (&pl)[PLANE_N], uint32_t P0, uint32_t P1, uint32_t P2,
                                           uint32_t P3, uint32_t nT, uint32_t& am, uint32_t& ax) {
#pragma unroll
  for (int w = 0; w < PLANE_GW; w += 2) {
    uint32_t x0, x1;
    const uint32_t t0 = pair_miss(pl, w, P0, P1, P2, P3, nT, x0);
    const uint32_t t1 = pair_miss(pl, w + 1, P0, P1, P2, P3, nT, x1);
    am = bop3_and3(am, t0, t1);
    if constexpr (!KX) {
    } else if constexpr (PAD) {
      ax |= bop3_andn_and(t0, x0, pl[PLANE_V][w]);
      ax |= bop3_andn_and(t1, x1, pl[PLANE_V][w + 1]);
    } else {
      ax = bop3_or_andn(ax, t0, x0);
      ax = bop3_or_andn(ax, t1, x1);
    }
  }
}

// The lowest group of the range: its dm' words (km) and, KX, feasible non-match words (kx) kept.
template <bool PAD, bool KX>
__device__ __forceinline__ void pair_group_keep(const u32x8 (&pl)[PLANE_N], uint32_t P0, uint32_t P1, uint32_t P2,
                                                uint32_t P3, uint32_t nT, uint32_t (&km)[PLANE_GW],
                                                uint32_t (&kx)[PLANE_GW]) {
#pragma unroll
  for (int w = 0; w < PLANE_GW; ++w) {
    uint32_t xi;
    km[w] = pair_miss(pl, w, P0, P1, P2, P3, nT, xi);
    if constexpr (KX) kx[w] = PAD ? bop3_andn_and(km[w], xi, pl[PLANE_V][w]) : bop3_andn(km[w], xi);
  }
}

// NodeUnschedulable's verdict depends on the pod only through its tolerates bit, so the node side of
// "is there a feasible node" is the same for every pod of one tolerates value: V & ~X for a pod that
// does not tolerate the taint, V for one that does. The identity-like modes (NONE, DEFAULT: a pod
// without a feasible match takes its first feasible node) evaluate it here, on the scalar unit, once
// per wave and group, instead of a per-lane OR per word; the lane picks its value by its tolerates bit.
template <bool PAD>
__device__ __forceinline__ void group_feasible_s(const u32x8 (&pl)[PLANE_N], bool& fn, bool& ft) {
  if constexpr (PAD) {
    uint32_t on = 0u, ot = 0u;
#pragma unroll
    for (int w = 0; w < PLANE_GW; ++w) {
      on |= pl[PLANE_V][w] & ~pl[PLANE_X][w];
      ot |= pl[PLANE_V][w];
    }
    fn = on != 0u;
    ft = ot != 0u;
  } else {  // no padding slot: every node is real
    uint32_t ax = 0xFFFFFFFFu;
#pragma unroll
    for (int w = 0; w < PLANE_GW; ++w) ax &= pl[PLANE_X][w];
    fn = ax != 0xFFFFFFFFu;
    ft = true;
  }
}
// The first node of group g (planes pl, all six loaded) feasible for a pod that does not tolerate the
// taint (NT) or that does; NOFIT if none. Scalar.
template <bool NT>
__device__ __forceinline__ uint32_t group_first_feasible_s(const u32x8 (&pl)[PLANE_N], uint32_t g) {
  uint32_t r = NOFIT;
#pragma unroll
  for (int w = PLANE_GW - 1; w >= 0; --w) {
    const uint32_t h = NT ? (pl[PLANE_V][w] & ~pl[PLANE_X][w]) : pl[PLANE_V][w];
    r = h ? (g * PLANE_GW + (uint32_t)w) * 32u + (uint32_t)__builtin_ctz(h) : r;
  }
  return r;
}

// The lane's first feasible match (or, NONMATCH, feasible non-match) in group g, NOFIT if none:
// per-lane vector loads of the group's planes (the rare path: a first hit above the lowest group).
template <bool NONMATCH>
__device__ __forceinline__ uint32_t group_first_or_none(const uint32_t* __restrict__ planes, uint32_t g,
                                                        uint32_t P0, uint32_t P1, uint32_t P2, uint32_t P3,
                                                        uint32_t nT) {
  const uint4* q = reinterpret_cast<const uint4*>(planes + (size_t)g * GROUP_DWORDS);
  uint32_t pl[PLANE_N][PLANE_GW];
#pragma unroll
  for (int k = 0; k < PLANE_N; ++k) {
    const uint4 lo = q[k * 2], hi = q[k * 2 + 1];
    pl[k][0] = lo.x; pl[k][1] = lo.y; pl[k][2] = lo.z; pl[k][3] = lo.w;
    pl[k][4] = hi.x; pl[k][5] = hi.y; pl[k][6] = hi.z; pl[k][7] = hi.w;
  }
  uint32_t h[PLANE_GW];
#pragma unroll
  for (int c = 0; c < PLANE_GW; ++c) {
    const uint32_t dm = (pl[0][c] ^ P0) | (pl[1][c] ^ P1) | (pl[2][c] ^ P2) | (pl[3][c] ^ P3);
    const uint32_t fe = ~(pl[PLANE_X][c] & nT) & pl[PLANE_V][c];
    h[c] = NONMATCH ? (dm & fe) : (~dm & fe);
  }
  const uint32_t m = hits_first(h, 0u);  // all-ones when the group holds none
  return m < GROUP_NODES ? g * GROUP_NODES + m : NOFIT;
}

template <int S, bool SHARD, bool KX>
__global__ __launch_bounds__(PAIR_WAVES * WAVE) void pair_kernel(PairArgs a) {
  constexpr int PB = PAIR_WAVES / S;  // 64-pod blocks per workgroup
  __shared__ uint32_t s_res[S > 1 ? PAIR_WAVES : 1][2][WAVE];
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int sl = wv % S, pb = wv / S;
  const BatchDesc& d = a.d[blockIdx.y];
  const int32_t np = d.n_pods;
  if ((int32_t)blockIdx.x * PB * WAVE >= np) return;  // the whole workgroup lies past its batch's end
  const int32_t wbase = ((int32_t)blockIdx.x * PB + pb) * WAVE;
  const int32_t j = wbase + lane;
  const bool act = j < np;
  uint32_t code = CODE_NONE_POD, tol = 0u;
  if (act) {
    const int dq = d.pod_digit[j];
    code = (dq >= 0 && dq <= 9) ? (uint32_t)dq : CODE_NONE_POD;  // NodeNumber.PreScore: Atoi of the last byte
    tol = d.pod_tol[j] ? 1u : 0u;
  }
  const uint32_t P0 = 0u - (code & 1u), P1 = 0u - ((code >> 1) & 1u), P2 = 0u - ((code >> 2) & 1u),
                 P3 = 0u - (code >> 3);
  const uint32_t nT = tol ? 0u : 0xFFFFFFFFu;
  const bool live = wbase < np;  // wave-uniform: this wave's block holds pods
  const int32_t g_lo = min(sl * a.gps, a.n_groups);
  const int32_t g_hi = live ? min(g_lo + a.gps, a.n_groups) : g_lo;
  const int32_t g_full = a.g_full;  // groups below it hold no padding slot
  // Groups above g_lo, descending, two per step: the pair's flags are one AND / OR over its 16 words,
  // and fm / fx remember the lower group of the lowest pair with a hit (its hit may lie in that group
  // or the one above). Identity-like modes: fn / ft, the lowest group with a node feasible for a pod
  // that does not tolerate / that tolerates the taint (scalar).
  uint32_t fm = NO_GROUP, fx = NO_GROUP;
  uint32_t fn = NO_GROUP, ft = NO_GROUP;
  for (int32_t g = g_hi - 1; g > g_lo; g -= 2) {
    uint32_t am = 0xFFFFFFFFu, ax = 0u;
    const int32_t g2 = g - 1 > g_lo ? g - 1 : g;  // the pair's lower group (g itself when alone)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int32_t gg = h == 0 ? g : g - 1;
      if (h == 1 && gg <= g_lo) break;
      u32x8 pl[PLANE_N];
      bool sn, st;
      if (gg < g_full) {
        sload_group<PLANE_V>(pl, a.planes + (size_t)gg * GROUP_DWORDS);
        pair_group<false, KX>(pl, P0, P1, P2, P3, nT, am, ax);
        if constexpr (!KX) group_feasible_s<false>(pl, sn, st);
      } else {
        sload_group<PLANE_N>(pl, a.planes + (size_t)gg * GROUP_DWORDS);
        pair_group<true, KX>(pl, P0, P1, P2, P3, nT, am, ax);
        if constexpr (!KX) group_feasible_s<true>(pl, sn, st);
      }
      if constexpr (!KX) {
        fn = sn ? (uint32_t)gg : fn;
        ft = st ? (uint32_t)gg : ft;
      }
    }
    fm = am != 0xFFFFFFFFu ? (uint32_t)g2 : fm;
    if constexpr (KX) fx = ax != 0u ? (uint32_t)g2 : fx;
  }
  uint32_t rm = NOFIT, rx = NOFIT;  // first feasible match / KX: non-match, identity-like: feasible node
  if (g_lo < g_hi) {
    uint32_t km[PLANE_GW], kx[PLANE_GW];
    u32x8 pl[PLANE_N];
    sload_group<PLANE_N>(pl, a.planes + (size_t)g_lo * GROUP_DWORDS);
    if (g_lo < g_full) pair_group_keep<false, KX>(pl, P0, P1, P2, P3, nT, km, kx);
    else pair_group_keep<true, KX>(pl, P0, P1, P2, P3, nT, km, kx);
    const uint32_t am = bop3_and3(bop3_and3(km[0], km[1], km[2]), bop3_and3(km[3], km[4], km[5]), km[6] & km[7]);
    if (am != 0xFFFFFFFFu) {
      uint32_t h[PLANE_GW];
#pragma unroll
      for (int w = 0; w < PLANE_GW; ++w) h[w] = ~km[w];
      rm = hits_first(h, (uint32_t)g_lo);
    } else if (fm != NO_GROUP) {  // the lowest hit pair: its lower group, else the one above
      rm = group_first_or_none<false>(a.planes, fm, P0, P1, P2, P3, nT);
      if (rm == NOFIT) rm = group_first_or_none<false>(a.planes, fm + 1, P0, P1, P2, P3, nT);
    }
    if constexpr (KX) {
      const uint32_t ax = (kx[0] | kx[1] | kx[2]) | (kx[3] | kx[4] | kx[5]) | (kx[6] | kx[7]);
      if (ax != 0u) {
        rx = hits_first(kx, (uint32_t)g_lo);
      } else if (fx != NO_GROUP) {
        rx = group_first_or_none<true>(a.planes, fx, P0, P1, P2, P3, nT);
        if (rx == NOFIT) rx = group_first_or_none<true>(a.planes, fx + 1, P0, P1, P2, P3, nT);
      }
    } else {  // the first feasible node for each tolerates value (scalar), then the lane's
      uint32_t an = group_first_feasible_s<true>(pl, (uint32_t)g_lo);
      uint32_t at = group_first_feasible_s<false>(pl, (uint32_t)g_lo);
      if (an == NOFIT && fn != NO_GROUP) {
        u32x8 p2[PLANE_N];
        sload_group<PLANE_N>(p2, a.planes + (size_t)fn * GROUP_DWORDS);
        an = group_first_feasible_s<true>(p2, fn);
      }
      if (at == NOFIT && ft != NO_GROUP) {
        u32x8 p2[PLANE_N];
        sload_group<PLANE_N>(p2, a.planes + (size_t)ft * GROUP_DWORDS);
        at = group_first_feasible_s<false>(p2, ft);
      }
      rx = tol ? at : an;
    }
  }
  if constexpr (S > 1) {
    s_res[wv][0][lane] = rm;
    s_res[wv][1][lane] = rx;
    __syncthreads();
    if (sl != 0) return;
#pragma unroll
    for (int k = 1; k < S; ++k) {
      rm = umin(rm, s_res[wv + k][0][lane]);
      rx = umin(rx, s_res[wv + k][1][lane]);
    }
  }
  if (!act) return;
  if constexpr (SHARD) {  // per-pod keys: the element-wise MAX over node shards is the global first
    a.keys[j] = rm != NOFIT ? shard_key(a.node_base, rm) : 0;
    a.keys[(size_t)np + j] = rx != NOFIT ? shard_key(a.node_base, rx) : 0;
  } else {
    const uint32_t ra = umin(rm, rx);  // the first feasible node (identity-like: rx already is)
    int32_t oi, ost;
    int64_t osc;
    decode_pod(rm != NOFIT ? (int64_t)rm : -1, (KX && rx != NOFIT) ? (int64_t)rx : -1,
               ra != NOFIT ? (int64_t)ra : -1, code != CODE_NONE_POD, a.pp, &oi, &osc, &ost);
    d.out_idx[j] = oi;
    if (d.out_score) d.out_score[j] = osc;  // optional output (NULL: not written)
    d.out_status[j] = ost;
  }
}



// ---------------------------------------------------------------------------------------
// pair_kernel with the node planes staged in LDS (the default for tables up to PAIR_LDS_MAX_GROUPS
// groups and launches that fill the chip). The same per-pair evaluation as pair_kernel, but every
// v_bitop3 reads VGPRs only: an SGPR operand caps a wave64 VALU instruction at ~0.21 issues per
// SIMD-cycle on MI355X where the all-VGPR forms reach 0.30-0.34 (scripts/ubench_valu_r4.hip,
// profiles/r4_ubench_valu.jsonl), and pair_kernel's scan ran at that cap (0.215, profiles/r4_pmc_c3.json).
// A workgroup copies the table's planes into LDS once and its waves then read each group's words as
// wave-uniform ds_read_b128 (every lane the same address: a broadcast, no bank conflict) into VGPRs.
// Each wave evaluates PL_BPW 64-pod blocks together: a group's planes are read from LDS once per wave
// and applied to all of them, and the table copy is amortised over PL_WAVES x PL_BPW blocks.
// Per lane and 32-node word: xi = X & nT, dm' (4 v_bitop3), and per two words one AND3 into the
// group's match flag, plus, KX, one OR of the feasible non-matches (dm' & ~xi), or, identity-like
// modes, one AND3 of two words' xi per two words (the group holds a feasible node iff not all-ones).
// ---------------------------------------------------------------------------------------
constexpr int PL_WAVES = 4;  // waves per workgroup (tables up to PAIR_LDS_MAX_GROUPS groups)
constexpr int PL_WAVES_BIG = 16;  // waves per workgroup for larger tables: one copy of up to 80 KB serves
                                  // 16 waves (two workgroups per CU: 8 waves per SIMD)
constexpr int PAIR_LDS_BIG_GROUPS = 416;  // 106,496 nodes, 78 KB per workgroup
constexpr int PL_BPW_MAX = 4;  // 64-pod blocks per wave (the kernel's PL_BPW: 1-4, DeviceInfo::pair_lds_bpw)
constexpr int PAIR_LDS_MAX_GROUPS = 128;  // 32,768 nodes, 24 KB of LDS per workgroup

// The planes of group g from LDS (NPL planes, 8 words each) into VGPRs.
template <int NPL>
__device__ __forceinline__ void lds_group(uint32_t (&pl)[PLANE_N][PLANE_GW], const uint4* __restrict__ s_tab,
                                          int32_t g) {
  const uint4* q = s_tab + g * (GROUP_DWORDS / 4);
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const uint4 lo = q[2 * k], hi = q[2 * k + 1];
    pl[k][0] = lo.x; pl[k][1] = lo.y; pl[k][2] = lo.z; pl[k][3] = lo.w;
    pl[k][4] = hi.x; pl[k][5] = hi.y; pl[k][6] = hi.z; pl[k][7] = hi.w;
  }
}

__device__ __forceinline__ uint32_t pair_miss_v(const uint32_t (&pl)[PLANE_N][PLANE_GW], int w, uint32_t P0,
                                                uint32_t P1, uint32_t P2, uint32_t P3, uint32_t nT, uint32_t& xi) {
  xi = __builtin_amdgcn_bitop3_b32(pl[PLANE_X][w], nT, nT, 0xc0);  // X & nT
  uint32_t t = bop3_or_xor(xi, pl[0][w], P0);
  t = bop3_or_xor(t, pl[1][w], P1);
  t = bop3_or_xor(t, pl[2][w], P2);
  return bop3_or_xor(t, pl[3][w], P3);
}

// One group: am &= its dm' words; KX: ax |= its feasible non-matches; else af &= its xi words (not
// all-ones iff the group holds a node feasible for the pod; a padding group also ORs ~V into xi).
template <bool PAD, bool KX>
__device__ __forceinline__ void pair_group_v(const uint32_t (&pl)[PLANE_N][PLANE_GW], uint32_t P0, uint32_t P1,
                                             uint32_t P2, uint32_t P3, uint32_t nT, uint32_t& am, uint32_t& ax) {
#pragma unroll
  for (int w = 0; w < PLANE_GW; w += 2) {
    uint32_t x0, x1;
    const uint32_t t0 = pair_miss_v(pl, w, P0, P1, P2, P3, nT, x0);
    const uint32_t t1 = pair_miss_v(pl, w + 1, P0, P1, P2, P3, nT, x1);
    am = bop3_and3(am, t0, t1);
    if constexpr (KX) {
      if constexpr (PAD) {
        ax |= bop3_andn_and(t0, x0, pl[PLANE_V][w]);
        ax |= bop3_andn_and(t1, x1, pl[PLANE_V][w + 1]);
      } else {
        ax = bop3_or_andn(ax, t0, x0);
        ax = bop3_or_andn(ax, t1, x1);
      }
    } else {
      if constexpr (PAD) {  // infeasible: xi or not a real node
        ax = bop3_and3(ax, x0 | ~pl[PLANE_V][w], x1 | ~pl[PLANE_V][w + 1]);
      }
      // (a group without padding: the caller folds nT & AND(X) into ax once per group)
    }
  }
}

// pair_group_v for a block whose 64 pods share their tolerates bit (TY 0: none tolerates, TY 1: every
// one does): the filter term X & nT is X itself or zero, so it folds into the first code compare
// (v_bitop3 X | (D0 ^ P0)), or drops out: 4 VALU per word for dm' instead of 5.
template <bool PAD, bool KX, int TY>
__device__ __forceinline__ void pair_group_ty(const uint32_t (&pl)[PLANE_N][PLANE_GW], uint32_t P0, uint32_t P1,
                                              uint32_t P2, uint32_t P3, uint32_t& am, uint32_t& ax) {
#pragma unroll
  for (int w = 0; w < PLANE_GW; w += 2) {
    uint32_t t[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ww = w + h;
      uint32_t u = TY == 0 ? bop3_or_xor(pl[PLANE_X][ww], pl[0][ww], P0) : (pl[0][ww] ^ P0);
      u = bop3_or_xor(u, pl[1][ww], P1);
      u = bop3_or_xor(u, pl[2][ww], P2);
      t[h] = bop3_or_xor(u, pl[3][ww], P3);
    }
    am = bop3_and3(am, t[0], t[1]);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ww = w + h;
      if constexpr (KX) {  // feasible non-matches: dm' & ~X (TY 0) or dm' (TY 1), & V in a padding group
        if constexpr (TY == 0) ax = PAD ? (ax | bop3_andn_and(t[h], pl[PLANE_X][ww], pl[PLANE_V][ww]))
                                       : bop3_or_andn(ax, t[h], pl[PLANE_X][ww]);
        else ax = PAD ? (ax | (t[h] & pl[PLANE_V][ww])) : (ax | t[h]);
      }
    }
    if constexpr (!KX && PAD) {  // infeasible: X (TY 0) or not a real node
      if constexpr (TY == 0) ax = bop3_and3(ax, pl[PLANE_X][w] | ~pl[PLANE_V][w], pl[PLANE_X][w + 1] | ~pl[PLANE_V][w + 1]);
      else ax = bop3_and3(ax, ~pl[PLANE_V][w], ~pl[PLANE_V][w + 1]);
    }
  }
}

// A full group (no padding slot) with planes 0-2 from LDS (VGPRs) and X, D3 by scalar loads (SGPRs):
// 6 LDS reads per group instead of 10, at the price of two SGPR-operand v_bitop3 per word (the
// "hybrid" form, MSH_PAIR_HYBRID). TY as pair_group_ty (2: mixed tolerates, X & nT per word).
template <bool KX, int TY>
__device__ __forceinline__ void pair_group_hy(const uint32_t (&pl)[PLANE_N][PLANE_GW], const u32x8& X,
                                              const u32x8& D3, uint32_t P0, uint32_t P1, uint32_t P2, uint32_t P3,
                                              uint32_t nT, uint32_t& am, uint32_t& ax) {
#pragma unroll
  for (int w = 0; w < PLANE_GW; w += 2) {
    uint32_t t[2], xi[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ww = w + h;
      uint32_t u;
      if constexpr (TY == 0) {
        u = bop3_or_xor(X[ww], pl[0][ww], P0);
      } else if constexpr (TY == 1) {
        u = pl[0][ww] ^ P0;
      } else {
        xi[h] = __builtin_amdgcn_bitop3_b32(X[ww], nT, nT, 0xc0);  // X & nT
        u = bop3_or_xor(xi[h], pl[0][ww], P0);
      }
      u = bop3_or_xor(u, pl[1][ww], P1);
      u = bop3_or_xor(u, pl[2][ww], P2);
      t[h] = bop3_or_xor(u, D3[ww], P3);
    }
    am = bop3_and3(am, t[0], t[1]);
    if constexpr (KX) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if constexpr (TY == 0) ax = bop3_or_andn(ax, t[h], X[w + h]);
        else if constexpr (TY == 1) ax |= t[h];
        else ax = bop3_or_andn(ax, t[h], xi[h]);
      }
    }
  }
}

// The lane's first feasible node in group g (identity-like modes), NOFIT if none.
__device__ __forceinline__ uint32_t group_first_feasible_v(const uint32_t (&pl)[PLANE_N][PLANE_GW], uint32_t g,
                                                           uint32_t nT) {
  uint32_t h[PLANE_GW];
#pragma unroll
  for (int c = 0; c < PLANE_GW; ++c) h[c] = pl[PLANE_V][c] & ~(pl[PLANE_X][c] & nT);
  const uint32_t m = hits_first(h, 0u);
  return m < GROUP_NODES ? g * GROUP_NODES + m : NOFIT;
}

// The lane's first feasible match (KIND 0), feasible non-match (1) or feasible node (2) in group g
// of the LDS table, NOFIT if none: half a group (four words, 6 x 4 plane words live) at a time.
template <int KIND>
__device__ __forceinline__ uint32_t group_first_lds(const uint4* __restrict__ s_tab, uint32_t g, uint32_t P0,
                                                    uint32_t P1, uint32_t P2, uint32_t P3, uint32_t nT) {
  const uint4* q = s_tab + g * (GROUP_DWORDS / 4);
#pragma unroll 1
  for (int hh = 0; hh < 2; ++hh) {
    uint32_t pl[PLANE_N][4];
#pragma unroll
    for (int k = 0; k < PLANE_N; ++k) {
      const uint4 v = q[2 * k + hh];
      pl[k][0] = v.x; pl[k][1] = v.y; pl[k][2] = v.z; pl[k][3] = v.w;
    }
    uint32_t t[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t fe = ~(pl[PLANE_X][c] & nT) & pl[PLANE_V][c];
      uint32_t h;
      if constexpr (KIND == 2) {
        h = fe;
      } else {
        const uint32_t dm = (pl[0][c] ^ P0) | (pl[1][c] ^ P1) | (pl[2][c] ^ P2) | (pl[3][c] ^ P3);
        h = KIND == 1 ? (dm & fe) : (~dm & fe);
      }
      t[c] = lowbit(h) | (uint32_t)(32 * c);  // all-ones when the word has none
    }
    const uint32_t m = umin(umin(t[0], t[1]), umin(t[2], t[3]));
    if (m < 128u) return g * GROUP_NODES + (uint32_t)(hh * 128) + m;
  }
  return NOFIT;
}

// Both firsts of group g in one pass over its planes (half a group at a time, the upper half only
// when some lane needs it): the first feasible match (rm) and, KX, the first feasible non-match or,
// else, the first feasible node (rx); NOFIT where the group has none. Called by whole waves.
template <bool KX>
__device__ __forceinline__ void group_firsts_lds(const uint4* __restrict__ s_tab, uint32_t g, uint32_t P0,
                                                 uint32_t P1, uint32_t P2, uint32_t P3, uint32_t nT, bool digit,
                                                 uint32_t& rm, uint32_t& rx) {
  const uint4* q = s_tab + g * (GROUP_DWORDS / 4);
  uint32_t bm = 0xFFFFFFFFu, bx = 0xFFFFFFFFu;
#pragma unroll 1
  for (int hh = 0; hh < 2; ++hh) {
    uint32_t pl[PLANE_N][4];
#pragma unroll
    for (int k = 0; k < PLANE_N; ++k) {
      const uint4 v = q[2 * k + hh];
      pl[k][0] = v.x; pl[k][1] = v.y; pl[k][2] = v.z; pl[k][3] = v.w;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t fe = ~(pl[PLANE_X][c] & nT) & pl[PLANE_V][c];
      const uint32_t dm = (pl[0][c] ^ P0) | (pl[1][c] ^ P1) | (pl[2][c] ^ P2) | (pl[3][c] ^ P3);
      const uint32_t off = (uint32_t)(32 * (c + 4 * hh));
      bm = umin(bm, lowbit(~dm & fe) | off);  // all-ones stays all-ones for a word without one
      bx = umin(bx, lowbit(KX ? (dm & fe) : fe) | off);
    }
    // the upper half only when some lane's first match (a pod without a digit has none: its code
    // matches no node's) or first feasible (non-match) is not in the lower one: with random digits
    // almost never, and the scan of group 0 halves
    if (hh == 0 && __ballot((digit && bm == 0xFFFFFFFFu) || bx == 0xFFFFFFFFu) == 0) break;
  }
  rm = bm < GROUP_NODES ? g * GROUP_NODES + bm : NOFIT;
  rx = bx < GROUP_NODES ? g * GROUP_NODES + bx : NOFIT;
}

template <bool SHARD, bool KX, int PL_BPW, int W, bool CMP, int HY>
__device__ __forceinline__ void pair_lds_body(PairArgs a) {
  extern __shared__ uint4 s_tab[];  // n_groups * GROUP_DWORDS / 4
  constexpr int NSL = W * PL_BPW;   // 64-pod slices of the workgroup
  __shared__ uint32_t s_cnt[CMP ? NSL : 1];
  __shared__ uint32_t s_pod[CMP ? NSL * WAVE : 1];
  const BatchDesc& d = a.d[blockIdx.y];
  const int32_t np = d.n_pods;
  const int32_t wg0 = (int32_t)blockIdx.x * NSL * WAVE;  // first pod of this workgroup
  if (wg0 >= np) return;  // the whole workgroup lies past its batch's end
  {
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(a.planes);
    const int32_t nq = a.n_groups * (GROUP_DWORDS / 4);
    for (int32_t i = threadIdx.x; i < nq; i += W * WAVE) s_tab[i] = src[i];
  }
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int32_t n_groups = a.n_groups, g_full = a.g_full;
  // The wave's PL_BPW pod blocks are evaluated together: each group's planes are read from LDS once
  // and applied to all of them (the LDS broadcast reads, ~6 CU-cycles each, would otherwise bound it).
  // CMP: the workgroup's pods are first reordered (stable, through LDS) so that those that do not
  // tolerate the unschedulable taint come first and those that do last: most 64-pod blocks then hold
  // one tolerates value, and their scan folds the filter term into the first code compare
  // (pair_group_ty). Every pair is still evaluated; only the order in which the lanes take the pods
  // changes, and each result is written back to its pod's own index.
  uint32_t pk[PL_BPW];  // per block, the lane's pod: index in the workgroup << 8 | tolerates << 4 | code
#pragma unroll
  for (int b = 0; b < PL_BPW; ++b) {
    const int32_t pos0 = (wv * PL_BPW + b) * WAVE + lane;
    const int32_t j = wg0 + pos0;
    uint32_t c = CODE_NONE_POD, t = 0u;
    if (j < np) {
      const int dq = d.pod_digit[j];
      c = (dq >= 0 && dq <= 9) ? (uint32_t)dq : CODE_NONE_POD;  // NodeNumber.PreScore: Atoi of the last byte
      t = d.pod_tol[j] ? 1u : 0u;
    }
    pk[b] = ((uint32_t)pos0 << 8) | (t << 4) | c;
  }
  if constexpr (CMP) {
    uint64_t mn[PL_BPW];  // per block: the lanes whose pod does not tolerate (padding lanes count here)
#pragma unroll
    for (int b = 0; b < PL_BPW; ++b) {
      mn[b] = __ballot(((pk[b] >> 4) & 1u) == 0u);
      if (lane == 0) s_cnt[wv * PL_BPW + b] = (uint32_t)__builtin_popcountll(mn[b]);
    }
    __syncthreads();
    uint32_t tot = 0, pre[PL_BPW];
#pragma unroll
    for (int k = 0; k < NSL; ++k) {
      const uint32_t c = s_cnt[k];
#pragma unroll
      for (int b = 0; b < PL_BPW; ++b)
        if (k == wv * PL_BPW + b) pre[b] = tot;
      tot += c;
    }
#pragma unroll
    for (int b = 0; b < PL_BPW; ++b) {
      const uint32_t sl = (uint32_t)(wv * PL_BPW + b);
      const bool nt = ((pk[b] >> 4) & 1u) == 0u;
      const uint32_t below = nt ? __builtin_amdgcn_mbcnt_hi((uint32_t)(mn[b] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mn[b], 0u))
                                : __builtin_amdgcn_mbcnt_hi((uint32_t)(~mn[b] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)~mn[b], 0u));
      const uint32_t pos = nt ? pre[b] + below : tot + (sl * WAVE - pre[b]) + below;
      s_pod[pos] = pk[b];
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < PL_BPW; ++b) pk[b] = s_pod[(wv * PL_BPW + b) * WAVE + lane];
  } else {
    __syncthreads();
  }
  uint32_t P0[PL_BPW], P1[PL_BPW], P2[PL_BPW], P3[PL_BPW], nT[PL_BPW], code[PL_BPW];
  int32_t jj[PL_BPW];
  int ty[PL_BPW];  // wave-uniform per block: 0 no pod tolerates, 1 every pod does, 2 mixed
  bool any_act = false;
#pragma unroll
  for (int b = 0; b < PL_BPW; ++b) {
    const uint32_t c = pk[b] & 15u, t = (pk[b] >> 4) & 1u;
    jj[b] = wg0 + (int32_t)(pk[b] >> 8);
    code[b] = c;
    P0[b] = 0u - (c & 1u);
    P1[b] = 0u - ((c >> 1) & 1u);
    P2[b] = 0u - ((c >> 2) & 1u);
    P3[b] = 0u - (c >> 3);
    nT[b] = t ? 0u : 0xFFFFFFFFu;
    const uint64_t tm = __ballot(t != 0u);
    ty[b] = CMP ? (tm == 0 ? 0 : (~tm == 0 ? 1 : 2)) : 2;
    any_act = any_act || __ballot(jj[b] < np) != 0;
  }
  if (!any_act) return;  // wave-uniform; no barrier below
  // Groups above 0, descending, two per step (as pair_kernel): each group's 40 / 48 plane words read
  // into VGPRs at once and applied to every block. fm / fx: the lower group of the lowest pair with a
  // feasible match / KX: feasible non-match, identity-like: feasible node. (Reading half a group at a
  // time, one group per iteration, cut the kernel to 52 VGPRs and 8 waves per SIMD but ran slower:
  // 95.6 against 89.8 us per 32-batch C3 launch, profiles/r4_ab_pair_planes.txt.)
  uint32_t fm[PL_BPW], fx[PL_BPW];
#pragma unroll
  for (int b = 0; b < PL_BPW; ++b) fm[b] = fx[b] = NO_GROUP;
  // Group 0 first: every block's first hits in it (half-group reads; the upper half only when some
  // lane needs it). When every lane already has its first feasible non-match (KX) or first feasible
  // node there, the scan of the groups above needs only the match flags: every pair is still
  // evaluated (dm' per word), but the non-match / feasible reduction, whose answer group 0 has
  // settled, is left out (KX: 5.5 instead of 6.5 VALU per word).
  constexpr int KIND_X = KX ? 1 : 2;  // KX: first feasible non-match; else first feasible node
  uint32_t rm[PL_BPW], rx[PL_BPW];
  auto group0 = [&]() {
#pragma unroll
    for (int b = 0; b < PL_BPW; ++b) group_firsts_lds<KX>(s_tab, 0u, P0[b], P1[b], P2[b], P3[b], nT[b], code[b] != CODE_NONE_POD, rm[b], rx[b]);
  };
  auto scan = [&](auto noax) {
    constexpr bool NOAX = decltype(noax)::value;
    constexpr bool KXS = KX && !NOAX;  // the non-match flags are tracked
    for (int32_t g = n_groups - 1; g > 0; g -= 2) {
      uint32_t am[PL_BPW], ax[PL_BPW];
#pragma unroll
      for (int b = 0; b < PL_BPW; ++b) {
        am[b] = 0xFFFFFFFFu;
        ax[b] = KX ? 0u : 0xFFFFFFFFu;
      }
      const int32_t g2 = g - 1 > 0 ? g - 1 : g;
      u32x8 spp[2][2];  // HY 2: X, D3 of both groups of the step, one wait for the four scalar loads
      if constexpr (HY == 2) {
        asm volatile("s_load_dwordx8 %0, %4, %6\n\ts_load_dwordx8 %1, %4, %7\n\t"
                     "s_load_dwordx8 %2, %5, %6\n\ts_load_dwordx8 %3, %5, %7\n\ts_waitcnt lgkmcnt(0)"
                     : "=&s"(spp[0][0]), "=&s"(spp[0][1]), "=&s"(spp[1][0]), "=&s"(spp[1][1])
                     : "s"(a.planes + (size_t)g * GROUP_DWORDS), "s"(a.planes + (size_t)g2 * GROUP_DWORDS),
                       "n"(PLANE_X * PLANE_GW * 4), "n"(3 * PLANE_GW * 4));
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int32_t gg = h == 0 ? g : g - 1;
        if (h == 1 && gg <= 0) break;
        uint32_t pl[PLANE_N][PLANE_GW];
        if (HY && gg < g_full) {
          u32x8 sp[2];  // X, D3
          if constexpr (HY == 2) {
            sp[0] = spp[h][0];
            sp[1] = spp[h][1];
          } else {
            asm volatile("s_load_dwordx8 %0, %2, %3\n\ts_load_dwordx8 %1, %2, %4\n\ts_waitcnt lgkmcnt(0)"
                         : "=&s"(sp[0]), "=&s"(sp[1])
                         : "s"(a.planes + (size_t)gg * GROUP_DWORDS), "n"(PLANE_X * PLANE_GW * 4), "n"(3 * PLANE_GW * 4));
          }
          lds_group<3>(pl, s_tab, gg);
#pragma unroll
          for (int b = 0; b < PL_BPW; ++b) {
            if (ty[b] == 0) pair_group_hy<KXS, 0>(pl, sp[0], sp[1], P0[b], P1[b], P2[b], P3[b], nT[b], am[b], ax[b]);
            else if (ty[b] == 1) pair_group_hy<KXS, 1>(pl, sp[0], sp[1], P0[b], P1[b], P2[b], P3[b], nT[b], am[b], ax[b]);
            else pair_group_hy<KXS, 2>(pl, sp[0], sp[1], P0[b], P1[b], P2[b], P3[b], nT[b], am[b], ax[b]);
          }
          if constexpr (!KX && !NOAX) {  // nT & AND(X): the AND on the scalar unit
            const uint32_t axg = sp[0][0] & sp[0][1] & sp[0][2] & sp[0][3] & sp[0][4] & sp[0][5] & sp[0][6] & sp[0][7];
#pragma unroll
            for (int b = 0; b < PL_BPW; ++b) ax[b] = bop3_and3(ax[b], nT[b], axg);
          }
        } else if (gg < g_full) {
          lds_group<PLANE_V>(pl, s_tab, gg);
#pragma unroll
          for (int b = 0; b < PL_BPW; ++b) {
            if (ty[b] == 0) pair_group_ty<false, KXS, 0>(pl, P0[b], P1[b], P2[b], P3[b], am[b], ax[b]);
            else if (ty[b] == 1) pair_group_ty<false, KXS, 1>(pl, P0[b], P1[b], P2[b], P3[b], am[b], ax[b]);
            else pair_group_v<false, KXS>(pl, P0[b], P1[b], P2[b], P3[b], nT[b], am[b], ax[b]);
          }
          if constexpr (!KX && !NOAX) {  // no padding: the AND of the group's xi words is nT & AND(X), X shared
            const uint32_t axg = bop3_and3(bop3_and3(pl[PLANE_X][0], pl[PLANE_X][1], pl[PLANE_X][2]),
                                           bop3_and3(pl[PLANE_X][3], pl[PLANE_X][4], pl[PLANE_X][5]),
                                           pl[PLANE_X][6] & pl[PLANE_X][7]);
#pragma unroll
            for (int b = 0; b < PL_BPW; ++b) ax[b] = bop3_and3(ax[b], nT[b], axg);
          }
        } else {
          lds_group<PLANE_N>(pl, s_tab, gg);
#pragma unroll
          for (int b = 0; b < PL_BPW; ++b) {
            if (ty[b] == 0) pair_group_ty<true, KXS, 0>(pl, P0[b], P1[b], P2[b], P3[b], am[b], ax[b]);
            else if (ty[b] == 1) pair_group_ty<true, KXS, 1>(pl, P0[b], P1[b], P2[b], P3[b], am[b], ax[b]);
            else pair_group_v<true, KXS>(pl, P0[b], P1[b], P2[b], P3[b], nT[b], am[b], ax[b]);
          }
        }
      }
#pragma unroll
      for (int b = 0; b < PL_BPW; ++b) {
        fm[b] = am[b] != 0xFFFFFFFFu ? (uint32_t)g2 : fm[b];
        if constexpr (!NOAX) fx[b] = (KX ? ax[b] != 0u : ax[b] != 0xFFFFFFFFu) ? (uint32_t)g2 : fx[b];
      }
    }
  };
  if (a.noax) {
    group0();
    bool xdone = true;
#pragma unroll
    for (int b = 0; b < PL_BPW; ++b) xdone = xdone && __ballot(rx[b] == NOFIT) == 0;
    if (xdone) scan(std::true_type{});
    else scan(std::false_type{});
  } else {  // group 0 after the scan (its registers free during it)
    scan(std::false_type{});
    group0();
  }
  // then the rare re-reads of a higher pair, then the decode
#pragma unroll
  for (int b = 0; b < PL_BPW; ++b) {
    const int32_t j = jj[b];
    if (__ballot(j < np) == 0) continue;  // wave-uniform: a block of padding lanes only
    if (rm[b] == NOFIT && fm[b] != NO_GROUP) {  // the lowest hit pair: its lower group, else the one above
      rm[b] = group_first_lds<0>(s_tab, fm[b], P0[b], P1[b], P2[b], P3[b], nT[b]);
      if (rm[b] == NOFIT) rm[b] = group_first_lds<0>(s_tab, fm[b] + 1, P0[b], P1[b], P2[b], P3[b], nT[b]);
    }
    if (rx[b] == NOFIT && fx[b] != NO_GROUP) {
      rx[b] = group_first_lds<KIND_X>(s_tab, fx[b], P0[b], P1[b], P2[b], P3[b], nT[b]);
      if (rx[b] == NOFIT) rx[b] = group_first_lds<KIND_X>(s_tab, fx[b] + 1, P0[b], P1[b], P2[b], P3[b], nT[b]);
    }
    if (j < np) {
      if constexpr (SHARD) {
        a.keys[j] = rm[b] != NOFIT ? shard_key(a.node_base, rm[b]) : 0;
        a.keys[(size_t)np + j] = rx[b] != NOFIT ? shard_key(a.node_base, rx[b]) : 0;
      } else {
        const uint32_t ra = umin(rm[b], rx[b]);
        int32_t oi, ost;
        int64_t osc;
        decode_pod(rm[b] != NOFIT ? (int64_t)rm[b] : -1, (KX && rx[b] != NOFIT) ? (int64_t)rx[b] : -1,
                   ra != NOFIT ? (int64_t)ra : -1, code[b] != CODE_NONE_POD, a.pp, &oi, &osc, &ost);
        d.out_idx[j] = oi;
        if (d.out_score) d.out_score[j] = osc;
        d.out_status[j] = ost;
      }
    }
  }
}

// (the body is a device function so that A/B builds can wrap it with other register budgets: a
// 7-waves-per-SIMD build, 72 VGPRs with a few spilled, ran 1-5% slower, profiles/r4_ab_pair_planes.txt)
template <bool SHARD, bool KX, int PL_BPW, int W = PL_WAVES, bool CMP = false, int HY = 0>
__global__ __launch_bounds__(W * WAVE) void pair_lds_kernel(PairArgs a) {
  pair_lds_body<SHARD, KX, PL_BPW, W, CMP, HY>(a);
}

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


// ---------------------------------------------------------------------------------------
// The opt-in class-row kernel (MSH_BATCH_KERNEL=classrows; tables up to WGP_MAX_GROUPS groups, 8,192
// nodes). NOT a per-pair evaluation: a pod's verdicts come from rows indexed by its class (tolerates,
// digit) that the prep built per upload; kept for what it is, a placement path specialised to the
// reference plugins, and reported apart from the per-pair kernels. A persistent grid of as many
// workgroups as the runtime reports resident copies the table's class rows (msh_internal.h HR_*) into
// LDS once per workgroup and then walks the launch's (batch, 256-pod block) space; after the copy the
// waves are independent (no barrier per block), and each wave loads the next block's pod bytes before
// it scans the current one.
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
      if (i < tot) s_tab[i] = vs[k];
    }
  }
  const uint32_t ball0 = A.ball[0], ball1 = A.ball[1];
  const IdentDecode idd = make_ident_decode(A.pp);
  constexpr int GQ16 = GQL * 8;  // a group's stride in uint16
  __shared__ uint32_t s_xb[KX ? HR_CLS : 1];
  __syncthreads();
  if constexpr (KX) {
    // REVERSE / MIN-MAX: per pod class, bit g = group g holds a feasible non-match (its first-node
    // offset, hr_first_kernel, is not HR_NONE), once per workgroup from the staged table: 8 lanes per
    // class, four groups each (<= 32 groups), OR-reduced over the 8 lanes. The scan then reads one word
    // per pod instead of a 2-byte offset per group (4 ds_read_u16 and ~10 VALU per four groups).
    static_assert(NT >= HR_CLS * 8 && WGP_MAX_GROUPS <= 32, "one lane per (class, four groups)");
    const int32_t t = (int32_t)threadIdx.x, c = t >> 3, g0 = (t & 7) * 4;
    uint32_t bits = 0;
    if (c < HR_CLS) {
      const uint16_t* o = reinterpret_cast<const uint16_t*>(s_tab + HR_FIRST) + HR_CLS + c;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (g0 + k < n_groups && o[(g0 + k) * GQ16] != HR_NONE) bits |= 1u << (g0 + k);
    }
    bits |= __shfl_xor(bits, 1);
    bits |= __shfl_xor(bits, 2);
    bits |= __shfl_xor(bits, 4);
    if (c < HR_CLS && (t & 7) == 0) s_xb[c] = bits;
    __syncthreads();
  }
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
  while (it < total) {
    if (!cur.live) {  // this wave's slice lies past its batch's end
      flush();
      advance();
      cur = prepare();
      continue;
    }
    const uint32_t tol = cur.tol;
    const uint32_t e0 = cur.e0, e1 = cur.e1;  // the lane's chunk-0 and chunk-1 class-row entries
    const uint32_t cls = cur.cls;               // its class (first-node tables)
    // Groups descending, four per step (eight ds_read_b128 in flight; n_groups is a multiple of 4:
    // tables are padded to 1,024-node blocks), one flag per PAIR of groups: bit q of bm = group 2q or
    // 2q + 1 holds a feasible digit match (the 16 words of a pair reduce in 8 VALU: 7 v_bitop3 OR3 and
    // one more); KX takes the first feasible non-match from the class's group bitmap (s_xb). The
    // previous item's stores and the next item's loads go after the first step.
    uint32_t bm = 0;
    auto or16 = [](const uint4& a, const uint4& b, const uint4& c, const uint4& d) {
      return or3(or3(or3(a.x, a.y, a.z), or3(a.w, b.x, b.y), or3(b.z, b.w, c.x)),
                 or3(or3(c.y, c.z, c.w), or3(d.x, d.y, d.z), d.w), 0u);
    };
    auto step = [&](int32_t q) {  // groups q .. q + 3
      const uint4* t = s_tab + q * GQL;
      const uint4 a0 = t[e0], b0 = t[e1], a1 = t[GQL + e0], b1 = t[GQL + e1];
      const uint4 a2 = t[2 * GQL + e0], b2 = t[2 * GQL + e1], a3 = t[3 * GQL + e0], b3 = t[3 * GQL + e1];
      bm = lshl_or(bm, 2, lshl_or(min1(or16(a2, b2, a3, b3)), 1, min1(or16(a0, b0, a1, b1))));
    };
    int32_t q = n_groups - 4;
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
    if constexpr (KX) {
      const uint32_t xb = s_xb[cls];  // the class's groups with a feasible non-match
      if (xb) {
        const uint32_t g = lowbit(xb);
        rx = g * GROUP_NODES + reinterpret_cast<const uint16_t*>(s_tab + g * GQL + HR_FIRST)[HR_CLS + cls];
      }
    }
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
}

// ---------------------------------------------------------------------------------------
// Generic score pipeline: any score plugin list (NodeNumber and up to four score-column plugins,
// MSH_PLUGIN_SCORE_COLUMN0..3) with the int64 total of EVERY (pod, node) pair computed explicitly:
// the general form of RunFilterPlugins + RunScorePlugins + selectHost (minisched.go:115-199,
// 304-325), north_star's stages one to one.
// "Lanes = pods": lane l of a wave holds one pod; the node side is wave-uniform and arrives by scalar
// loads (GEN_CH nodes per chunk: node words, and the columns in use), so everything that depends on
// the node alone runs on the scalar unit once per wave, and the vector unit does per-pair work only.
//   1. feasibility: NodeUnschedulable per pair, from the node word (X: Spec.Unschedulable with the
//      filter listed; V: a real node) and the lane's tolerates bit: a lane mask per node (the wave's
//      ballot of its 64 pods), built by the scalar unit;
//   3. per-pod extent (max, min) of every normalizing plugin's raw score over the pod's feasible
//      nodes: a sweep of its own, only when some plugin normalizes; slice waves meet in an LDS
//      reduction;
//   2. the int64 total of each pair: the sum over the plugins of weight x NormalizeScore(raw) in Go
//      int64 arithmetic (wrapping). NodeNumber: per pod, its two weighted normalized values (raw 10 on
//      a digit match, else 0), selected per pair by one compare. A column plugin without a normalizer:
//      weight x column, node-only, summed by the scalar unit. A normalizing column: per pair
//      q = (100 raw - b) x r with the pod's reciprocal r = (1 / m)(1 + 2^-49) (b, m from its extent),
//      truncated toward zero: exactly Go's int64 100 raw / m (|100 raw| < 2^39; the bias makes an
//      exact quotient come out at or just above the integer, and keeps every other quotient below
//      the next one);
//   4. selectHost: per lane a running first maximum over the nodes in List order (strict '>', the
//      first feasible node always taken), the node index kept as a chunk-relative inline constant;
//      slice waves meet in LDS (slices ascend in List order).
//   5. the node table is read once per wave through the scalar cache and reused by its 64 pods.
// MODE 0: the whole batch (status, node, score per pod). Node-sharded mode (msh_generic_*): MODE 1
// writes each pod's extents over this shard's nodes (ext, mins negated: one all-reduce MAX merges
// them), MODE 2 takes the merged extents and writes each pod's best (total, global node index) over
// the shard.
// ---------------------------------------------------------------------------------------
constexpr int GEN_WAVES = 4;   // waves per workgroup
constexpr double GEN_RCP_BIAS = 1.0 + 0x1p-49;

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

template <int S, int NCOL, int MODE>
__global__ __launch_bounds__(GEN_WAVES * WAVE) void generic_kernel(GenericArgs a) {
  static_assert(MODE == 0 || S == 1, "the node-sharded modes run one wave per 64-pod block");
  constexpr int PB = GEN_WAVES / S;  // 64-pod blocks per workgroup
  constexpr int NE = 1 + NCOL;       // extents: [0] NodeNumber, [1 + c] column c of the list
  constexpr int NC = NCOL > 0 ? NCOL : 1;
  constexpr int SW = S > 1 ? GEN_WAVES : 1;
  __shared__ int64_t s_mx[SW][NE][WAVE], s_mn[SW][NE][WAVE];
  __shared__ int64_t s_bt[SW][WAVE];
  __shared__ int32_t s_bi[SW][WAVE];
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int sl = wv % S, pb = wv / S;
  const BatchDesc& d = a.d[blockIdx.y];
  const int32_t np = d.n_pods;
  if ((int32_t)blockIdx.x * PB * WAVE >= np) return;  // the whole workgroup lies past its batch's end
  const int32_t wbase = ((int32_t)blockIdx.x * PB + pb) * WAVE;
  const int32_t j = wbase + lane;
  const bool act = j < np;
  int pdg = -1;
  bool tol = false;
  if (act) {
    pdg = d.pod_digit[j];
    tol = d.pod_tol[j] != 0;
  }
  const bool pd_ok = pdg >= 0 && pdg <= 9;  // NodeNumber.PreScore: Atoi of the last byte
  const uint32_t pcode = pd_ok ? (uint32_t)pdg : CODE_NONE_POD;
  const bool live = wbase < np;  // wave-uniform
  const int32_t c_lo = min(sl * a.cps, a.n_chunks);
  const int32_t c_hi = live ? min(c_lo + a.cps, a.n_chunks) : c_lo;
  const int32_t n_nodes = a.n_nodes;
  const uint32_t* __restrict__ nrec = a.nrec;
  // Lane masks are kept explicitly (the wave's ballot of its pods): the scalar unit builds and
  // combines them, and a select reads one through inverse_ballot (the SGPR pair as the lane
  // condition, no VALU). NodeUnschedulable.Filter per pair: the node record's mask is all-ones unless
  // the node is Spec.Unschedulable (with the filter listed), when only the tolerating lanes pass.
  const uint64_t tolm = __ballot(tol);
  auto lanes = [](uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); };
  // Per column of the list (wave-uniform): its raw values as int64 (a column without a normalizer) or
  // as the exact double 100 x raw (a normalizing one), each read 8 nodes at a time by scalar loads.
  struct Chunk {
    uint32_t code[GEN_CH];
    uint64_t fm[GEN_CH];      // NodeUnschedulable: the lanes that pass the node
    uint64_t cv[NC][GEN_CH];  // column values (raw bits: int64 or double)
  };
  auto load_chunk = [&](int32_t i0, auto cnt, Chunk& ch) {
    const uint32_t* __restrict__ r = nrec + (size_t)i0 * NREC;
#pragma unroll
    for (int k = 0; k < GEN_CH; ++k) {
      if (k >= cnt) break;
      ch.code[k] = r[k * NREC];
      ch.fm[k] = tolm | ((uint64_t)r[k * NREC + 3] << 32 | r[k * NREC + 2]);
    }
#pragma unroll
    for (int cc = 0; cc < NCOL; ++cc) {
      const size_t off = (size_t)a.ccol[cc] * a.col_stride + i0;
      const uint64_t* __restrict__ cb = a.cmode[cc] == 0 ? reinterpret_cast<const uint64_t*>(a.cols + off)
                                                         : reinterpret_cast<const uint64_t*>(a.cols100 + off);
#pragma unroll
      for (int k = 0; k < GEN_CH; ++k) {
        if (k >= cnt) break;
        ch.cv[cc][k] = cb[k];
      }
    }
  };
  auto for_chunks = [&](auto&& body) {
    for (int32_t c = c_lo; c < c_hi; ++c) {
      const int32_t i0 = c * GEN_CH;
      const int32_t cnt = min(GEN_CH, n_nodes - i0);
      if (cnt == GEN_CH) body(i0, std::integral_constant<int, GEN_CH>{});
      else body(i0, cnt);
    }
  };
  auto as_f64 = [](uint64_t v) { return __builtin_bit_cast(double, v); };
  // bit cc: column cc of the list normalizes (wave-uniform, in an SGPR)
  int32_t nmask = 0;
#pragma unroll
  for (int cc = 0; cc < NCOL; ++cc) nmask |= a.cmode[cc] != 0 ? 1 << cc : 0;
  nmask = __builtin_amdgcn_readfirstlane(nmask);
  auto norm_col = [&](int cc) { return ((nmask >> cc) & 1) != 0; };

  // ---- stage 3: extents over the feasible nodes (normalizing plugins only) ----
  // NodeNumber's raw scores are 10 / 0: its extent is which of the two a feasible node gives. A
  // normalizing column's extent is a running f64 max / min of 100 x raw (exact) over the lanes that
  // pass the node: one v_max_f64 / v_min_f64 each, under the feasibility mask as the exec mask.
  int64_t emx[NE], emn[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    emx[e] = INT64_MIN;
    emn[e] = INT64_MAX;
  }
  if (MODE != 2 && a.need_ext) {
    uint64_t fmm = 0, fxm = 0;  // NodeNumber: lanes with a feasible match / non-match seen
    double dmx[NC], dmn[NC];
#pragma unroll
    for (int cc = 0; cc < NC; ++cc) {
      dmx[cc] = -__builtin_inf();
      dmn[cc] = __builtin_inf();
    }
    const bool nn_ext = a.nn_score && a.nn_mode != 0;
    for_chunks([&](int32_t i0, auto cnt) {
      Chunk ch;
      load_chunk(i0, cnt, ch);
#pragma unroll
      for (int k = 0; k < GEN_CH; ++k) {
        if (k >= cnt) break;
        const uint64_t f = ch.fm[k];
        if (nn_ext) {
          const uint64_t m = __ballot(ch.code[k] == pcode);
          fmm |= f & m;
          fxm |= f & ~m;
        }
#pragma unroll
        for (int cc = 0; cc < NCOL; ++cc) {
          if (!norm_col(cc)) continue;
          const double v = as_f64(ch.cv[cc][k]);
          // v_max_f64 / v_min_f64 (inline: fmax adds a NaN canonicalisation per operand; no NaN
          // here): every lane passes a schedulable node (f all-ones, the common case), only the
          // tolerating lanes an unschedulable one (their update kept by a select)
          const double hi = dmx[cc], lo = dmn[cc];
          double h2, l2;
          asm("v_max_f64 %0, %1, %2" : "=v"(h2) : "v"(hi), "s"(v));
          asm("v_min_f64 %0, %1, %2" : "=v"(l2) : "v"(lo), "s"(v));
          if (~f == 0) {
            dmx[cc] = h2;
            dmn[cc] = l2;
          } else {
            dmx[cc] = lanes(f) ? h2 : hi;
            dmn[cc] = lanes(f) ? l2 : lo;
          }
        }
      }
    });
    const bool fm = lanes(fmm), fx = lanes(fxm);
    emx[0] = fm ? 10 : (fx ? 0 : INT64_MIN);  // NodeNumber's raw scores are 10 / 0
    emn[0] = fx ? 0 : (fm ? 10 : INT64_MAX);
#pragma unroll
    for (int cc = 0; cc < NCOL; ++cc) {
      if (a.cmode[cc] == 0) continue;
      if (dmx[cc] != -__builtin_inf()) {  // 100 x raw / 100: exact (|raw| <= 2^31)
        emx[1 + cc] = (int64_t)(dmx[cc] * 0.01);
        emn[1 + cc] = (int64_t)(dmn[cc] * 0.01);
      }
    }
    if constexpr (S > 1) {  // the slices' partial extents meet in LDS
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        s_mx[wv][e][lane] = emx[e];
        s_mn[wv][e][lane] = emn[e];
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < S; ++k) {
        const int ow = pb * S + k;
#pragma unroll
        for (int e = 0; e < NE; ++e) {
          const int64_t ox = s_mx[ow][e][lane], on = s_mn[ow][e][lane];
          emx[e] = ox > emx[e] ? ox : emx[e];
          emn[e] = on < emn[e] ? on : emn[e];
        }
      }
    }
    if constexpr (MODE == 1) {  // node-sharded: this shard's extents, mins negated (one MAX merges both)
      if (act) {
#pragma unroll
        for (int e = 0; e < NE; ++e) {
          a.ext[(size_t)(2 * e) * np + j] = emx[e];
          a.ext[(size_t)(2 * e + 1) * np + j] = -emn[e];  // emn <= INT64_MAX: no overflow
        }
      }
      return;
    }
  }
  if constexpr (MODE == 1) return;
  if (MODE == 2 && a.need_ext && act) {  // the extents merged over every shard
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      emx[e] = a.ext[(size_t)(2 * e) * np + j];
      emn[e] = -a.ext[(size_t)(2 * e + 1) * np + j];
    }
  }

  // ---- per pod: NodeNumber's two weighted values, each normalizing column's reciprocal ----
  int64_t c1 = 0, c0 = 0;
  if (a.nn_score && a.nn_mode != 0 && emx[0] != INT64_MIN) {
    c1 = (int64_t)((uint64_t)gen_normalize(10, a.nn_mode, emx[0], emn[0]) * (uint64_t)a.nn_weight);
    c0 = (int64_t)((uint64_t)gen_normalize(0, a.nn_mode, emx[0], emn[0]) * (uint64_t)a.nn_weight);
  } else if (a.nn_score) {
    c1 = (int64_t)((uint64_t)10 * (uint64_t)a.nn_weight);  // NONE: raw x weight
  }
  double rr[NC], bb[NC];
#pragma unroll
  for (int cc = 0; cc < NC; ++cc) {
    rr[cc] = 0.0;
    bb[cc] = 0.0;
  }
#pragma unroll
  for (int cc = 0; cc < NCOL; ++cc) {
    const int32_t md = a.cmode[cc];
    const int64_t mx = emx[1 + cc], mn = emn[1 + cc];
    if (md == 0 || mx == INT64_MIN) continue;  // no normalizer, or no feasible node
    if (md == 3) {  // min-max: (raw - mn) x 100 / (mx - mn), 0 when mx == mn
      if (mx != mn) {
        rr[cc] = (1.0 / (double)(mx - mn)) * GEN_RCP_BIAS;
        bb[cc] = 100.0 * (double)mn;
      }
    } else {  // DefaultNormalizeScore: 100 raw / max(mx, 0); DEFAULT leaves an all-zero list (m = 100 -> raw)
      const int64_t m = mx > 0 ? mx : 0;
      if (m != 0) rr[cc] = (1.0 / (double)m) * GEN_RCP_BIAS;
      else if (md == 1) rr[cc] = 0.01 * GEN_RCP_BIAS;
      // REVERSE with m == 0: r = 0, 100 - 0 = 100 for every node
    }
  }
  // Wave-uniform: the normalizing columns' signed weights (REVERSE adds 100 w - n w: the 100 w of every
  // REVERSE column is a constant of the total, summed once), and whether all of them fit 31 bits
  // (then n x w + total is one v_mad_i64_i32).
  int64_t cws[NC];
  uint64_t tot0 = 0;
  bool wsmall = true;
#pragma unroll
  for (int cc = 0; cc < NCOL; ++cc) {
    const int32_t md = a.cmode[cc];
    const int64_t w = a.cweight[cc];
    cws[cc] = md == 2 ? -w : w;
    if (md == 2) tot0 += (uint64_t)100 * (uint64_t)w;
    if (md != 0) wsmall = wsmall && w < ((int64_t)1 << 31);
    if (md != 3) bb[cc] = 0.0;  // (100 raw - b) with b = 0: one v_add_f64 for every mode, exact
  }
  // the fast path's per-column modes as one uniform bit set: bit cc = MIN-MAX (its numerator is never
  // negative on a feasible pair)
  int32_t mmask = 0;
#pragma unroll
  for (int cc = 0; cc < NCOL; ++cc) mmask |= a.cmode[cc] == 3 ? 1 << cc : 0;
  mmask = __builtin_amdgcn_readfirstlane(mmask);
  const int32_t wsm = __builtin_amdgcn_readfirstlane(wsmall ? 1 : 0);

  // ---- stages 1, 2, 4: feasibility, the total, the first maximum ----
  uint64_t best = 0x8000000000000000ull;  // INT64_MIN; the first feasible node is always taken
  int32_t bidx = -1;
  uint64_t fdm = 0;  // lanes with a feasible node seen
  const uint64_t cw1 = (uint64_t)c1, cw0 = (uint64_t)c0;
  for_chunks([&](int32_t i0, auto cnt) {
    Chunk ch;
    load_chunk(i0, cnt, ch);
    int32_t bk = 0;
    uint64_t took = 0;  // lanes whose maximum moved in this chunk
#pragma unroll
    for (int k = 0; k < GEN_CH; ++k) {
      if (k >= cnt) break;
      const uint64_t f = ch.fm[k];
      // the node-only part (scalar unit): weight x column of the columns without a normalizer
      uint64_t ts = tot0;
#pragma unroll
      for (int cc = 0; cc < NCOL; ++cc)
        if (!norm_col(cc)) ts += ch.cv[cc][k] * (uint64_t)a.cweight[cc];
      // NodeNumber: 10 on a suffix-digit match (c1 = c0 = 0 when it does not score)
      uint64_t tot = ts + ((ch.code[k] == pcode) ? cw1 : cw0);
#pragma unroll
      for (int cc = 0; cc < NCOL; ++cc) {
        if (!norm_col(cc)) continue;
        const uint64_t bits = ch.cv[cc][k];
        const double q = (as_f64(bits) - bb[cc]) * rr[cc];  // (100 raw - b) x r: both operations exact
        // the numerator's sign from the node value's top dword (scalar unit): MIN-MAX numerators of
        // feasible pairs are never negative
        // (the sign bit by a scalar shift in asm: as C the test folds to a 64-bit compare, which the
        // scalar unit lacks, and became a VALU v_cmp_lt_i64 per pair)
        uint32_t sgn;
        asm("s_lshr_b32 %0, %1, 31" : "=s"(sgn) : "s"((uint32_t)(bits >> 32)));
        const bool nonneg = ((mmask >> cc) & 1) != 0 || sgn == 0;
        if (nonneg && wsm) {
          // |q| <= 100 on a feasible pair: v_cvt_i32_f64 (saturating in hardware: the value of an
          // infeasible pair converts without a fault and is never taken), then n x w + total in one
          // v_mad_i64_i32
          const int32_t n = (int32_t)q;
          tot = (uint64_t)((int64_t)n * (int64_t)(int32_t)cws[cc] + (int64_t)tot);
        } else {
          const int64_t n = (int64_t)__builtin_fmin(__builtin_fmax(q, -0x1p62), 0x1p62);  // |q| < 2^40 if feasible
          tot += (uint64_t)n * (uint64_t)cws[cc];
        }
      }
      const uint64_t take = f & (~fdm | __ballot((int64_t)tot > (int64_t)best));  // strict '>': the first max
      best = lanes(take) ? tot : best;
      bk = lanes(take) ? k : bk;
      took |= take;
      fdm |= f;
    }
    bidx = lanes(took) ? i0 + bk : bidx;
  });
  bool found = lanes(fdm);
  if constexpr (S > 1) {  // slices ascend in List order: a later slice wins only with a larger total
    s_bt[wv][lane] = (int64_t)best;
    s_bi[wv][lane] = found ? bidx : -1;
    __syncthreads();
    if (sl != 0) return;
#pragma unroll
    for (int k = 1; k < S; ++k) {
      const int32_t oi = s_bi[wv + k][lane];
      const int64_t ot = s_bt[wv + k][lane];
      if (oi >= 0 && (!found || ot > (int64_t)best)) {
        best = (uint64_t)ot;
        bidx = oi;
        found = true;
      }
    }
  }
  if (!act) return;
  if constexpr (MODE == 2) {  // this shard's best: merged by MAX total, then MIN global index
    a.best_total[j] = found ? (int64_t)best : INT64_MIN;
    a.best_idx[j] = found ? (int32_t)(a.node_base + bidx) : INT32_MAX;
  } else {
    int32_t st = 0;
    if (!found) st = 1;                                          // FitError (minisched.go:143-148)
    else if (a.nn_score && (!a.nn_prescore || !pd_ok)) st = 2;   // NodeNumber.Score error (nodenumber.go:74-77)
    d.out_idx[j] = st ? -1 : bidx;
    if (d.out_score) d.out_score[j] = st ? 0 : (int64_t)best;
    d.out_status[j] = st;
  }
}

// The decode of the node-sharded generic path, after the merge (msh_generic_decode_device).
__global__ __launch_bounds__(256) void generic_decode_kernel(const int8_t* __restrict__ pod_digit, int32_t p,
                                                             const int64_t* __restrict__ best_total,
                                                             const int32_t* __restrict__ best_idx,
                                                             int32_t nn_score, int32_t nn_prescore,
                                                             int32_t* __restrict__ out_idx,
                                                             int64_t* __restrict__ out_score,
                                                             int32_t* __restrict__ out_status) {
  const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= p) return;
  const int pd = pod_digit[j];
  const bool pd_ok = pd >= 0 && pd <= 9;
  const int32_t bi = best_idx[j];
  int32_t st = 0;
  if (bi == INT32_MAX) st = 1;                          // no shard has a feasible node: FitError
  else if (nn_score && (!nn_prescore || !pd_ok)) st = 2;  // NodeNumber.Score error
  out_idx[j] = st ? -1 : bi;
  if (out_score) out_score[j] = st ? 0 : best_total[j];
  out_status[j] = st;
}

// Per pod of a shard: its best index if its best total equals the merged maximum, else INT32_MAX
// (the second, MIN, all-reduce then yields the lowest global index among the maxima).
__global__ __launch_bounds__(256) void generic_candidate_kernel(int32_t p, const int64_t* __restrict__ local_total,
                                                                const int64_t* __restrict__ merged_total,
                                                                int32_t* __restrict__ idx) {
  const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= p) return;
  if (idx[j] != INT32_MAX && local_total[j] != merged_total[j]) idx[j] = INT32_MAX;
}

namespace {
int gen_slices(int64_t waves, int32_t n_chunks, int mode, const DeviceInfo& dev) {
  if (mode != 0) return 1;
  if (dev.bits_slices > 0) return dev.bits_slices;
  const int64_t want = (int64_t)dev.cus * 4 * 4;
  int sl = 1;
  while (sl < GEN_WAVES && waves * sl < want && n_chunks >= 64 * sl) sl *= 2;
  return sl;
}

template <int S, int NCOL, int MODE>
hipError_t launch_gen_k(GenericArgs& a, int32_t bx, hipStream_t s) {
  a.cps = (a.n_chunks + S - 1) / S;
  MSH_TIMED_LAUNCH((generic_kernel<S, NCOL, MODE>), dim3((unsigned)bx, (unsigned)a.nb), dim3(GEN_WAVES * WAVE), 0, s,
                   a);
  return hipGetLastError();
}

template <int NCOL>
hipError_t launch_gen_n(GenericArgs& a, int mode, int S, int32_t blocks, hipStream_t s) {
  auto bx = [&](int sl) { return (blocks * sl + GEN_WAVES - 1) / GEN_WAVES; };
  if (mode == 1) return launch_gen_k<1, NCOL, 1>(a, bx(1), s);
  if (mode == 2) return launch_gen_k<1, NCOL, 2>(a, bx(1), s);
  switch (S) {
    case 1: return launch_gen_k<1, NCOL, 0>(a, bx(1), s);
    case 2: return launch_gen_k<2, NCOL, 0>(a, bx(2), s);
    default: return launch_gen_k<4, NCOL, 0>(a, bx(4), s);
  }
}
}  // namespace

hipError_t launch_generic(GenericArgs& a, int mode, const DeviceInfo& dev, hipStream_t s) {
  if (a.nb <= 0 || a.nb > MULTI_MAX || a.ncol < 0 || a.ncol > GEN_COLS || (mode != 0 && a.nb != 1))
    return hipErrorInvalidValue;
  int32_t maxp = 0;
  int64_t waves = 0;
  for (int b = 0; b < a.nb; ++b) {
    maxp = std::max(maxp, a.d[b].n_pods);
    waves += (a.d[b].n_pods + WAVE - 1) / WAVE;
  }
  if (maxp == 0) return hipSuccess;
  const int32_t blocks = (maxp + WAVE - 1) / WAVE;
  const int S = gen_slices(waves, a.n_chunks, mode, dev);
  switch (a.ncol) {
    case 0: return launch_gen_n<0>(a, mode, S, blocks, s);
    case 1: return launch_gen_n<1>(a, mode, S, blocks, s);
    case 2: return launch_gen_n<2>(a, mode, S, blocks, s);
    case 3: return launch_gen_n<3>(a, mode, S, blocks, s);
    default: return launch_gen_n<4>(a, mode, S, blocks, s);
  }
}

hipError_t launch_generic_candidates(int32_t p, const int64_t* local_total, const int64_t* merged_total, int32_t* idx,
                                     hipStream_t s) {
  if (p <= 0) return hipSuccess;
  hipLaunchKernelGGL(generic_candidate_kernel, dim3((p + 255) / 256), dim3(256), 0, s, p, local_total, merged_total,
                     idx);
  return hipGetLastError();
}

hipError_t launch_generic_decode(const int8_t* pod_digit, int32_t p, const int64_t* best_total, const int32_t* best_idx,
                                 int32_t nn_score, int32_t nn_prescore, int32_t* out_idx, int64_t* out_score,
                                 int32_t* out_status, hipStream_t s) {
  if (p <= 0) return hipSuccess;
  hipLaunchKernelGGL(generic_decode_kernel, dim3((p + 255) / 256), dim3(256), 0, s, pod_digit, p, best_total, best_idx,
                     nn_score, nn_prescore, out_idx, out_score, out_status);
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
  // The first feasible node for a pod that does not tolerate the unschedulable taint (V & ~X) and for
  // one that does (V), evaluated here from the register-resident planes once per launch (lanes and
  // waves hold ascending word ranges: the first lane with one, then the smallest over the waves).
  __shared__ uint32_t s_first[NW + 1][2];
  {
    uint32_t fn = NONE, ft = NONE;
#pragma unroll
    for (int r = RS - 1; r >= 0; --r) {
      const uint32_t base = (uint32_t)((wv * WAVE + lane) * RS + r) << 5;
      const uint32_t hn = VV[r] & ~XX[r], ht = VV[r];
      fn = hn ? base + (uint32_t)__builtin_ctz(hn) : fn;
      ft = ht ? base + (uint32_t)__builtin_ctz(ht) : ft;
    }
    fn = wave_first(fn);
    ft = wave_first(ft);
    if (lane == 0) {
      s_first[wv][0] = fn;
      s_first[wv][1] = ft;
    }
  }
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
  int32_t* counts = a.counts;
  const IdentDecode idec = make_ident_decode(pp);
  // the first feasible node for each tolerates value (no capacity: constant over the launch), -1 = none
  uint32_t fa0 = NONE, fa1 = NONE;
#pragma unroll
  for (int w = 0; w < NW + (FIN ? 1 : 0); ++w) {
    fa0 = umin(fa0, s_first[w][0]);
    fa1 = umin(fa1, s_first[w][1]);
  }
  const int32_t ia0 = fa0 != NONE ? (int32_t)__builtin_amdgcn_readfirstlane((int)fa0) : -1;
  const int32_t ia1 = fa1 != NONE ? (int32_t)__builtin_amdgcn_readfirstlane((int)fa1) : -1;
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
                            int32_t has_nu, uint32_t* d_ball, uint32_t* d_planes, uint32_t* d_hrows,
                            uint32_t* d_nrec, hipStream_t s, const unsigned long long* d_patch, int32_t patch_count) {
  hipLaunchKernelGGL(prep_reset_kernel, dim3(patch_count > 0 ? (patch_count + 255) / 256 : 1), dim3(256), 0, s,
                     d_ball, d_patch, patch_count, const_cast<uint8_t*>(d_unsched), const_cast<int8_t*>(d_digit));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (n_pad == 0) return hipSuccess;
  hipLaunchKernelGGL(node_prep_kernel, dim3(n_pad / PREP_THREADS), dim3(PREP_THREADS), 0, s, d_unsched, d_digit, n,
                     has_nu, d_ball, d_planes, d_hrows, d_nrec);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const int32_t slots = n_pad / GROUP_NODES * 2 * HR_CLS;
  hipLaunchKernelGGL(hr_first_kernel, dim3((slots + 255) / 256), dim3(256), 0, s, d_hrows, n_pad / GROUP_NODES);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void cols100_kernel(const int64_t* __restrict__ cols, double* __restrict__ cols100,
                                                     int64_t stride, int32_t n, int32_t n_pad, uint32_t col_mask) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const int k = blockIdx.y;
  if (i >= n_pad || !((col_mask >> k) & 1u)) return;
  cols100[(size_t)k * stride + i] = i < n ? 100.0 * (double)cols[(size_t)k * stride + i] : 0.0;
}

hipError_t launch_cols100(const int64_t* cols, double* cols100, int64_t stride, int32_t n, int32_t n_pad,
                          uint32_t col_mask, hipStream_t s) {
  if (n_pad <= 0 || !col_mask) return hipSuccess;
  hipLaunchKernelGGL(cols100_kernel, dim3((n_pad + 255) / 256, GEN_COLS), dim3(256), 0, s, cols, cols100, stride, n,
                     n_pad, col_mask);
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
// Occupancy of a kernel at a block size and dynamic LDS, from the runtime (workgroups per CU).
int resident_per_cu(const void* kern, int threads, size_t lds) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, threads, lds) != hipSuccess) {
    (void)hipGetLastError();
    return 1;
  }
  return std::max(nb, 1);
}

// The class-row kernel over m.nb batches of m.bpb 256-pod blocks (MSH_BATCH_KERNEL=classrows, an
// opt-in): as many workgroups as the runtime reports resident (its occupancy query for this kernel,
// block size and LDS: 8 per CU for the identity-like form at C3, 6 for the REVERSE / MINMAX form and
// its 78 VGPRs), never more than the launch's blocks; a launch larger than what stays resident would
// run its extra workgroups after the persistent ones and break the age-slot shares below.
template <bool KX>
hipError_t launch_persistent(MultiArgs& m, const DeviceInfo& dev, hipStream_t s) {
  constexpr int W = MSH_WGP_W;
  int32_t maxp = 0;
  for (int b = 0; b < m.nb; ++b) maxp = std::max(maxp, m.d[b].n_pods);
  if (maxp == 0) return hipSuccess;
  m.bpb = (maxp + W * WAVE - 1) / (W * WAVE);
  const size_t lds = (size_t)m.a.n_groups * HR_GQ * sizeof(uint4);
  const int64_t per_cu = std::min<int64_t>(
      RANK_MAX, resident_per_cu(reinterpret_cast<const void*>(wgp_kernel<W, KX>), W * WAVE, lds));
  const int64_t items = (int64_t)m.bpb * m.nb;
  const int64_t grid = std::min<int64_t>(items, (int64_t)dev.cus * per_cu);
  // Item shares by age slot (blockIdx / CUs: the dispatcher fills every CU's slot r before slot r + 1)
  // when the grid fills every resident slot and each workgroup has at least WGP_SHARE_MIN items: slot
  // r's share falls by MSH_WGP_AGE_SLOPE / 1000 per slot relative to slot 0 (the rates of the slots
  // measured under equal shares); otherwise the strided walk.
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

// Slice waves per 64-pod block of pair_kernel: one, unless the launch has fewer than ~4 waves per
// SIMD; then 2 or 4, while each slice keeps at least two groups.
int pair_slices(int64_t waves, int32_t n_groups, const DeviceInfo& dev) {
  if (dev.bits_slices > 0) return dev.bits_slices;
  const int64_t want = (int64_t)dev.cus * 4 * 4;
  int sl = 1;
  while (sl < PAIR_WAVES && waves * sl < want && n_groups >= 4 * sl) sl *= 2;
  return sl;
}

template <int S, bool SHARD, bool KX>
hipError_t launch_pair_s(PairArgs& a, int32_t bx, hipStream_t s) {
  a.gps = (a.n_groups + S - 1) / S;
  MSH_TIMED_LAUNCH((pair_kernel<S, SHARD, KX>), dim3((unsigned)bx, (unsigned)a.nb), dim3(PAIR_WAVES * WAVE), 0, s,
                   a);
  return hipGetLastError();
}

template <bool SHARD, bool KX>
hipError_t launch_pair_t(PairArgs& a, const DeviceInfo& dev, hipStream_t s) {
  int32_t maxp = 0;
  int64_t waves = 0;
  for (int b = 0; b < a.nb; ++b) {
    maxp = std::max(maxp, a.d[b].n_pods);
    waves += (a.d[b].n_pods + WAVE - 1) / WAVE;
  }
  if (maxp == 0) return hipSuccess;
  // LDS-staged planes when the table fits and the launch fills the chip with whole workgroups (the
  // copy is amortised over PL_WAVES x PL_BPW blocks); scalar-loaded planes (with slice waves) otherwise
  // (auto: every normalize mode; per 32-batch C3 launch NONE 96.5 -> 85.0 us and MINMAX 95.4 -> 91.5 us
  // against scalar-loaded planes, profiles/r4_ab_pair_planes.txt)
  const bool fits = a.n_groups <= PAIR_LDS_MAX_GROUPS;
  const bool big = !fits && a.n_groups <= PAIR_LDS_BIG_GROUPS;  // 16-wave workgroups, two blocks per wave
  // (big: two 16-wave workgroups per CU fill it from 32 blocks per CU on)
  const int64_t min_waves = (int64_t)dev.cus * (big ? 2 * PL_WAVES_BIG : 4 * 4 * PL_BPW_MAX);
  const bool lds = (fits || big) && (dev.pair_planes == 2 ||
                                     (dev.pair_planes == 0 && waves >= min_waves && dev.bits_slices == 0));
  if (lds) {
    const int bpw = big ? 2 : (dev.pair_lds_bpw >= 1 && dev.pair_lds_bpw <= 4 ? dev.pair_lds_bpw : 2);
    const int w = big ? PL_WAVES_BIG : PL_WAVES;
    const int32_t blocks = (maxp + WAVE - 1) / WAVE;
    const int32_t bx = (blocks + w * bpw - 1) / (w * bpw);
    const size_t bytes = (size_t)a.n_groups * GROUP_DWORDS * sizeof(uint32_t);
    const dim3 grid((unsigned)bx, (unsigned)a.nb), blk(w * WAVE);
    const bool cmp = dev.pair_compact < 0 ? KX : dev.pair_compact != 0;
    const int hy = dev.pair_hybrid >= 0 && dev.pair_hybrid <= 2 ? dev.pair_hybrid : (KX ? 2 : 1);
    a.noax = dev.pair_noax >= 0 ? dev.pair_noax : (KX ? 1 : 0);
    // (bpw, compaction, hybrid) -> instance: 1 block per wave in the plain LDS form only
    using PairKernel = void (*)(PairArgs);
    // (bpw, compaction, hybrid) -> instance: 1, 3 and 4 blocks per wave in the plain LDS form only (with
    // hybrid planes they measured slower, profiles/r4_ab_pair_planes.txt)
    auto pick = [&](auto bpw_c, auto w_c) -> PairKernel {
      constexpr int B = decltype(bpw_c)::value, WW = decltype(w_c)::value;
      if constexpr (B != 2) {
        return pair_lds_kernel<SHARD, KX, B, WW>;
      } else {
        const PairKernel t[2][3] = {
            {pair_lds_kernel<SHARD, KX, B, WW, false, 0>,
             pair_lds_kernel<SHARD, KX, B, WW, false, 1>,
             pair_lds_kernel<SHARD, KX, B, WW, false, 2>},
            {pair_lds_kernel<SHARD, KX, B, WW, true, 0>,
             pair_lds_kernel<SHARD, KX, B, WW, true, 1>,
             pair_lds_kernel<SHARD, KX, B, WW, true, 2>}};
        return t[cmp ? 1 : 0][hy];
      }
    };
    PairKernel k;
    if (big) k = pick(std::integral_constant<int, 2>{}, std::integral_constant<int, PL_WAVES_BIG>{});
    else if (bpw == 1) k = pick(std::integral_constant<int, 1>{}, std::integral_constant<int, PL_WAVES>{});
    else if (bpw == 3) k = pick(std::integral_constant<int, 3>{}, std::integral_constant<int, PL_WAVES>{});
    else if (bpw == 4) k = pick(std::integral_constant<int, 4>{}, std::integral_constant<int, PL_WAVES>{});
    else k = pick(std::integral_constant<int, 2>{}, std::integral_constant<int, PL_WAVES>{});
    if (bytes > 64 * 1024) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
      if (e != hipSuccess) return e;
    }
    MSH_TIMED_LAUNCH(k, grid, blk, (unsigned)bytes, s, a);
    return hipGetLastError();
  }
  const int S = pair_slices(waves, a.n_groups, dev);
  const int32_t blocks = (maxp + WAVE - 1) / WAVE;  // 64-pod blocks of the largest batch
  auto bx = [&](int sl) { return (blocks * sl + PAIR_WAVES - 1) / PAIR_WAVES; };
  switch (S) {
    case 1: return launch_pair_s<1, SHARD, KX>(a, bx(1), s);
    case 2: return launch_pair_s<2, SHARD, KX>(a, bx(2), s);
    default: return launch_pair_s<4, SHARD, KX>(a, bx(4), s);
  }
}
}  // namespace

hipError_t launch_pairs(PairArgs& a, bool shard, const DeviceInfo& dev, hipStream_t s) {
  if (a.nb <= 0 || a.nb > MULTI_MAX || (shard && a.nb != 1)) return hipErrorInvalidValue;
  // KX: the normalize mode needs each pod's first feasible non-match (REVERSE, MINMAX)
  if (needs_kx(a.pp)) return shard ? launch_pair_t<true, true>(a, dev, s) : launch_pair_t<false, true>(a, dev, s);
  return shard ? launch_pair_t<true, false>(a, dev, s) : launch_pair_t<false, false>(a, dev, s);
}

bool classrows_fit(int32_t n_groups) { return n_groups <= WGP_MAX_GROUPS; }

hipError_t launch_classrows(const BatchArgs& a, const BatchDesc* d, int nb, const DeviceInfo& dev, hipStream_t s) {
  if (nb <= 0 || nb > MULTI_MAX || !classrows_fit(a.n_groups)) return hipErrorInvalidValue;
  MultiArgs m{};
  m.a = a;
  m.nb = nb;
  for (int b = 0; b < nb; ++b) m.d[b] = d[b];
  return needs_kx(a.pp) ? launch_persistent<true>(m, dev, s) : launch_persistent<false>(m, dev, s);
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


}  // namespace msh
