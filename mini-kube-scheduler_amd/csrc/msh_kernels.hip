// msh_kernels.hip — gfx950 (MI355X, CDNA4) kernels for the batched pods x nodes hot path.
//
// Reference path (shopetan/mini-kube-scheduler, Go): for ONE pod per cycle,
//   RunFilterPlugins   minisched/minisched.go:115-151  (NodeUnschedulable, upstream v1.22.0)
//   RunPreScorePlugins minisched/minisched.go:153-162  (NodeNumber.PreScore, nodenumber.go:50-64)
//   RunScorePlugins    minisched/minisched.go:164-199  (NodeNumber.Score, nodenumber.go:73-95)
//   selectHost         minisched/minisched.go:304-325  (argmax; ties -> lowest index here)
//
// Layout: "lanes = nodes". A wave holds 64 consecutive nodes of a chunk in its lanes and a
// group of up to G pods in scalar registers; every (pod, node) pair is evaluated by lane ops.
// Stages (north_star):
//   1. feasibility bitmask per pod class with wavefront __ballot      -> node_prep_kernel
//   2. int64 score with the plugin weight fused                        -> decode_pod
//   3. per-pod normalisation (DEFAULT / REVERSE / MINMAX need the per-pod extent of the
//      raw scores over the feasible list: first feasible match / non-match) -> KX path + decode
//   4. argmax with a fixed lowest-index tie-break, wave-wide DPP reduction -> wave_reduce
//   5. node-table tile staged in LDS once per workgroup and re-read for every pod group
//
// The score of a pair under the reference plugin set is 10*w if the node is feasible and
// its suffix digit equals the pod's, else 0, so selectHost's first max is "first feasible
// match, else first feasible". The IDENT path keeps one node per 16-bit half of a word,
// duplicated in both halves: (code << 10) | (chunk mod 1008), code = the node's digit if it
// is feasible for non-tolerating pods, else 15. A pod pair sits in one VGPR (the all-VGPR
// v_xor_b32 issues at twice the rate of the SGPR form) as (codeB << 26) | (codeA << 10); per
// word and pair
//     x = W ^ PP      (v_xor_b32)  -> a half is < 1024 iff that node matches that pod
// and two such words fold into the running first match of both pods with ONE
//     bm = v_pk_minimum3_f16(bm, x_r, x_r+1)
// (every half is a non-negative finite f16, so its f16 order is its integer order): 0.75
// lane-ops per (pod, node) evaluation. Nodes feasible only for tolerating pods are corrected
// afterwards from a short list (ulist). The KX path (batch_kernel) serves the REVERSE /
// MINMAX normalizers, which also need the first feasible non-match.
//
// Kernels, by entry point:
//   node_prep_kernel (+ prep_reset_kernel)  every upload / patch / plugin change
//   ident_wave_kernel    batch, IDENT modes, single-tile tables (default, up to 64 rounds of
//                        8 pairs per wave): one contiguous pod-pair range per wave,
//                        XCD-contiguous wave ranks
//   ident_dyn_kernel     batch, IDENT modes: per-CU work queue of 8-pod units (larger batches);
//                        MULTI form for tables of several 64,512-node compute tiles
//   ident_split_kernel   batch, IDENT modes, few pods against a large table: teams of waves
//                        share a unit over table slices
//   batch_kernel         batch, REVERSE / MINMAX (compare/select, LDS-staged tiles)
//   ident_kernel         batch, static pod ranges (A/B only: MSH_BATCH_KERNEL=2 / 0)
//   decode_keys_kernel   node-sharded mode: decode the merged int32 shard keys
//   seq_kernel           sequential commit, one pod at a time, one workgroup
//   export_kernel        per-pair result export (simulator result store)
// See DESIGN.md for the roofline / instruction budget of each kernel.
#include "msh_internal.h"

namespace msh {

__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

// |d - p| + c in ONE v_sad_u32 (p wave-uniform, read from an SGPR). Written as asm: the
// backend does match the generic form, but reassociates it into min/max/sub/add (4 VALU)
// whenever c is loop-invariant.
__device__ __forceinline__ uint32_t sad(uint32_t d, uint32_t p, uint32_t c) {
  uint32_t r;
  asm("v_sad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(d), "s"(p), "v"(c));
  return r;
}

template <bool IS_MIN, int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_step(uint32_t v) {
  // Lanes whose row is masked off keep `old`: the identity of the reduction.
  const int ident = IS_MIN ? -1 : 0;
  const uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp(ident, (int)v, CTRL, ROW_MASK, 0xF, false);
  return IS_MIN ? umin(v, t) : umax(v, t);
}

// Wave-wide unsigned max (IS_MIN=false) / min (IS_MIN=true); result is wave-uniform.
template <bool IS_MIN>
__device__ __forceinline__ uint32_t wave_reduce(uint32_t v) {
  v = dpp_step<IS_MIN, 0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
  v = dpp_step<IS_MIN, 0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
  v = dpp_step<IS_MIN, 0x141, 0xF>(v);  // row_half_mirror
  v = dpp_step<IS_MIN, 0x140, 0xF>(v);  // row_mirror   -> each 16-lane row holds its result
  v = dpp_step<IS_MIN, 0x142, 0xA>(v);  // row_bcast:15 -> rows 1,3 fold in rows 0,2
  v = dpp_step<IS_MIN, 0x143, 0xC>(v);  // row_bcast:31 -> rows 2,3 fold in row 1 (= rows 0..1)
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) { return wave_reduce<false>(v); }
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) { return wave_reduce<true>(v); }

#ifdef MSH_STAMPS
// Diagnostic build only (-DMSH_STAMPS): per-wave s_memrealtime / s_memtime stamps of the
// IDENT kernel phases. Never compiled into the product library.
constexpr int STAMPS_PER_WAVE = 8;
constexpr int STAMP_WAVES = 16384;
__device__ unsigned long long msh_stamp_buf[STAMP_WAVES * STAMPS_PER_WAVE * 2];
#define MSH_STAMP(slot)                                                                   \
  do {                                                                                    \
    if (lane == 0 && gw < STAMP_WAVES) {                                                  \
      msh_stamp_buf[((size_t)gw * STAMPS_PER_WAVE + (slot)) * 2] = __builtin_amdgcn_s_memrealtime(); \
      msh_stamp_buf[((size_t)gw * STAMPS_PER_WAVE + (slot)) * 2 + 1] = __builtin_amdgcn_s_memtime(); \
    }                                                                                     \
  } while (0)
#else
#define MSH_STAMP(slot) \
  do {                  \
  } while (0)
#endif

// first-match cost (idx, or >= 2^24 when none) -> key (KMAX - idx, 0 when none)
__device__ __forceinline__ uint32_t cost_to_key(uint32_t c) { return c < MATCH_LIMIT ? KMAX - c : 0u; }

// ---------------------------------------------------------------------------------------
// Stage 1: node table preparation + feasibility bitmask (once per upload / plugin change).
// For the only filter, NodeUnschedulable (upstream v1.22.0), feasibility depends on the
// pod only through "tolerates the unschedulable taint", so there are exactly two pod
// classes: 0 = does not tolerate, 1 = tolerates. Class 1 is feasible on every node.
//   c0[i]  = i if node i is feasible for class 0, else NOFIT
//   dig[i] = NodeNumber node digit (Atoi of the last byte, nodenumber.go:81-87) or 0xFF
//   w0[i]  = packed-16 first-match word (see msh_internal.h); ulist = class-1-only nodes
//   mask[c][chunk] = __ballot(feasible for class c)   (64-node feasibility bitmask)
//   ball[c] = key (KMAX - idx) of the first feasible node of class c (0 = none)
// ---------------------------------------------------------------------------------------
constexpr int PREP_THREADS = 1024;  // n_pad is a multiple of 1024: every block is whole
__global__ __launch_bounds__(PREP_THREADS) void node_prep_kernel(const uint8_t* __restrict__ unsched,
                                                                 const int8_t* __restrict__ digit,
                                                                 int32_t n, int32_t n_pad, int32_t has_nu,
                                                                 uint32_t* __restrict__ c0,
                                                                 uint8_t* __restrict__ dig,
                                                                 uint32_t* __restrict__ w0,
                                                                 uint32_t* __restrict__ ulist,
                                                                 uint32_t* __restrict__ ucount,
                                                                 unsigned long long* __restrict__ mask,
                                                                 uint32_t* __restrict__ ball,
                                                                 uint32_t* __restrict__ planes) {
  constexpr int NWV = PREP_THREADS / WAVE;
  __shared__ uint32_t s_cnt[NWV], s_k0[NWV], s_k1[NWV];
  __shared__ uint32_t s_base;
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const bool valid = i < n;
  const bool u = valid && unsched[i] != 0;
  const int d = valid ? (int)digit[i] : -1;
  // NodeUnschedulable.Filter: Spec.Unschedulable && !tolerates -> UnschedulableAndUnresolvable
  const bool feas0 = valid && !(has_nu && u);
  const bool feas1 = valid;
  const bool has_digit = d >= 0 && d <= 9;
  c0[i] = feas0 ? (uint32_t)i : NOFIT;
  dig[i] = has_digit ? (uint8_t)d : (uint8_t)DIGIT_NONE;
  const uint32_t local_chunk = (uint32_t)(i >> 6) % (uint32_t)TILE_CHUNKS;
  const uint32_t wd0 = ((feas0 && has_digit ? (uint32_t)d : CODE_NONE_NODE) << CODE_SHIFT) | local_chunk;
  w0[word_pos(i)] = wd0 | (wd0 << 16);
  const unsigned long long m0 = __ballot(feas0);
  const unsigned long long m1 = __ballot(feas1);
  // nodes whose feasibility differs between the classes -> ulist (order irrelevant: min search)
  const bool diff = feas1 && !feas0;
  const unsigned long long md = __ballot(diff);
  {
    // bit-sliced table: this wave's 64 nodes are words 2t and 2t + 1 of the PLANE_* layout
    const uint32_t code = has_digit ? (uint32_t)d : CODE_NONE_NODE;
    const unsigned long long pm[PLANE_N] = {__ballot(code & 1u), __ballot(code & 2u), __ballot(code & 4u),
                                            __ballot(code & 8u), __ballot(valid && !feas0), __ballot(valid)};
    if (lane < 2 * PLANE_N) {
      const int k = lane >> 1, half = lane & 1;
      unsigned long long m = pm[0];
#pragma unroll
      for (int q = 1; q < PLANE_N; ++q) m = (k == q) ? pm[q] : m;
      const uint32_t word = ((uint32_t)(i - lane) >> 5) + (uint32_t)half;  // i - lane: the wave's first node
      planes[((word / PLANE_GW) * PLANE_N + k) * PLANE_GW + word % PLANE_GW] = (uint32_t)(m >> (32 * half));
    }
  }
  if (lane == 0) {
    const int32_t chunk = i >> 6;
    const int32_t n_chunks = n_pad >> 6;
    mask[chunk] = m0;
    mask[n_chunks + chunk] = m1;
    s_cnt[wv] = (uint32_t)__builtin_popcountll(md);
    s_k0[wv] = m0 ? KMAX - (uint32_t)(i + __builtin_ctzll(m0)) : 0u;
    s_k1[wv] = m1 ? KMAX - (uint32_t)(i + __builtin_ctzll(m1)) : 0u;
  }
  __syncthreads();
  // one ulist reservation and one first-feasible update per class per BLOCK: device-scope
  // atomics on one address serialise (~86 M/s), so per-wave atomics made the 100k-node prep ~60 us
  if (threadIdx.x == 0) {
    uint32_t tot = 0, k0 = 0, k1 = 0;
    for (int w = 0; w < NWV; ++w) {
      tot += s_cnt[w];
      k0 = umax(k0, s_k0[w]);
      k1 = umax(k1, s_k1[w]);
    }
    s_base = tot ? atomicAdd(ucount, tot) : 0u;
    if (k0) atomicMax(&ball[0], k0);
    if (k1) atomicMax(&ball[1], k1);
  }
  __syncthreads();
  if (diff) {
    uint32_t base = s_base;
    for (int w = 0; w < wv; ++w) base += s_cnt[w];
    const uint32_t rank = (uint32_t)__builtin_popcountll(md & ((1ull << lane) - 1ull));
    ulist[base + rank] = ((has_digit ? (uint32_t)d : CODE_NONE_NODE) << 24) | (uint32_t)i;
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
// last one remembered is the first); afterwards the lane re-reads its own first group (vector
// loads) and finds the exact node: first word with a zero bit, then its lowest zero bit. No
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
  uint32_t fm = NO_GROUP, fx = NO_GROUP;  // first group with a feasible match / non-match
  constexpr int NPL = KX ? PLANE_N : PLANE_V;  // planes the scan reads
  for (int32_t g = g_hi - 1; g >= g_lo; --g) {
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
      uint32_t mm[2], mx[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int c = w + q;
        const uint32_t xi = pg[PLANE_X * PLANE_GW + c] & nT;
        if constexpr (KX) {
          uint32_t dm = pg[c] ^ P0;
          dm = or_xor_s(dm, pg[PLANE_GW + c], P1);
          dm = or_xor_s(dm, pg[2 * PLANE_GW + c], P2);
          dm = or_xor_s(dm, pg[3 * PLANE_GW + c], P3);
          mm[q] = dm | xi;
          mx[q] = nmiss_s(dm, xi, pg[PLANE_V * PLANE_GW + c]);
        } else {
          uint32_t t = or_xor_s(xi, pg[c], P0);
          t = or_xor_s(t, pg[PLANE_GW + c], P1);
          t = or_xor_s(t, pg[2 * PLANE_GW + c], P2);
          mm[q] = or_xor_s(t, pg[3 * PLANE_GW + c], P3);
        }
      }
      am &= mm[0] & mm[1];
      if constexpr (KX) ax &= mx[0] & mx[1];
    }
    fm = am != 0xFFFFFFFFu ? (uint32_t)g : fm;
    if constexpr (KX) fx = ax != 0xFFFFFFFFu ? (uint32_t)g : fx;
  }
  uint32_t rm = NOFIT, rx = NOFIT;  // node index of the first feasible match / non-match
  if (fm != NO_GROUP) rm = group_first<false>(a.planes, fm, P0, P1, P2, P3, nT);
  if (KX && fx != NO_GROUP) rx = group_first<true>(a.planes, fx, P0, P1, P2, P3, nT);
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
    if constexpr (KX)
      decode_pod(im, rx != NOFIT ? (int64_t)rx : -1, ia, code != CODE_NONE_POD, a.pp, &a.out_idx[j],
                 &a.out_score[j], &a.out_status[j]);
    else
      decode_ident(im, ia, code != CODE_NONE_POD, make_ident_decode(a.pp), &a.out_idx[j], &a.out_score[j],
                   &a.out_status[j]);
  }
}

// ---------------------------------------------------------------------------------------
// Batched kernel. Workgroup = 4 waves; the node table (or a tile of it) is staged in LDS
// once per tile and re-read by every pod group of every wave. Each wave owns a contiguous
// pod range, walked in windows of 64 pods (one pod per lane). Within a window the pods are
// split by class with __ballot (class = tolerates the unschedulable taint), and each class
// is processed in groups of up to G pods whose digits sit in SGPRs. For every R-chunk
// sub-tile the wave loads R node records per lane from LDS, then for every pod of the group
//   IDENT:  bm = min3(bm, sad(D0, pd, C0), sad(D1, pd, C1))       [1.5 VALU / 64 pairs]
//   KX:     m = (D == pd); bm = max(bm, m ? K : 0); bx = max(bx, m ? 0 : K)   [5 VALU]
// Results land in the pod's lane (lane select) and are decoded and stored once per window.
// ---------------------------------------------------------------------------------------
template <int R, int G, bool NEED_KX, bool SHARD>
__global__ __launch_bounds__(BATCH_THREADS) void batch_kernel(BatchArgs a, int32_t tile_chunks) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  uint32_t* lds_c = reinterpret_cast<uint32_t*>(lds_raw);
  uint8_t* lds_d = lds_raw + (size_t)tile_chunks * WAVE * sizeof(uint32_t);

  constexpr int WPG = BATCH_THREADS / WAVE;
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t W = (int64_t)gridDim.x * WPG;
  const int64_t gw = (int64_t)blockIdx.x * WPG + wv;
  const int32_t p0 = (int32_t)((int64_t)a.n_pods * gw / W);
  const int32_t p1 = (int32_t)((int64_t)a.n_pods * (gw + 1) / W);
  const int32_t ntiles = (a.n_chunks + tile_chunks - 1) / tile_chunks;
  if (SHARD && !NEED_KX) write_class_keys(a);
  const uint32_t ball0 = a.ball[0], ball1 = a.ball[1];

  for (int32_t t = 0; t < ntiles; ++t) {
    // ---- stage node tile t in LDS (stage 5) ----
    const int32_t c0t = t * tile_chunks;
    const int32_t nc = min(tile_chunks, a.n_chunks - c0t);  // multiple of 16 (host pads)
    if (t > 0) __syncthreads();
    {
      const uint4* src = reinterpret_cast<const uint4*>(a.c0 + (size_t)c0t * WAVE);
      uint4* dst = reinterpret_cast<uint4*>(lds_c);
      for (int32_t i = threadIdx.x; i < nc * (WAVE / 4); i += BATCH_THREADS) dst[i] = src[i];
      const uint4* srcd = reinterpret_cast<const uint4*>(a.dig + (size_t)c0t * WAVE);
      uint4* dstd = reinterpret_cast<uint4*>(lds_d);
      for (int32_t i = threadIdx.x; i < nc * (WAVE / 16); i += BATCH_THREADS) dstd[i] = srcd[i];
    }
    __syncthreads();
    const uint32_t idx_base = (uint32_t)(c0t * WAVE + lane);  // global node index of chunk 0
    const bool last_tile = (t == ntiles - 1);

    for (int32_t w0 = p0; w0 < p1; w0 += WAVE) {
      const int32_t nwin = min((int32_t)WAVE, p1 - w0);
      const bool act = lane < nwin;
      uint32_t pdv = POD_DIGIT_NONE, tolv = 0;
      if (act) {
        const int d = a.pod_digit[w0 + lane];
        pdv = (d >= 0 && d <= 9) ? (uint32_t)d : POD_DIGIT_NONE;
        tolv = a.pod_tol[w0 + lane] ? 1u : 0u;
      }
      uint32_t res_m = 0u, res_x = 0u;  // keys (KMAX - idx, 0 = none)
      if (t > 0 && act) {
        res_m = a.partial[w0 + lane];
        if (NEED_KX) res_x = a.partial[(size_t)a.n_pods + w0 + lane];
      }
      const unsigned long long cls_mask[2] = {__ballot(act && tolv == 0u), __ballot(act && tolv != 0u)};

#pragma unroll
      for (int cls = 0; cls < 2; ++cls) {
        unsigned long long mask = cls_mask[cls];
        while (mask) {
          // ---- form a class-homogeneous group of up to G pods (scalar) ----
          uint32_t spd[G];
          int32_t lsel[G];
          int32_t cnt = 0;
#pragma unroll
          for (int g = 0; g < G; ++g) {
            if (mask) {
              const int32_t l = (int32_t)__builtin_ctzll(mask);
              mask &= mask - 1;
              lsel[g] = l;
              spd[g] = (uint32_t)__builtin_amdgcn_readlane((int)pdv, l);
              cnt = g + 1;
            } else {
              lsel[g] = 0;
              spd[g] = POD_DIGIT_NONE;
            }
          }
          uint32_t bm[G], bx[G];
#pragma unroll
          for (int g = 0; g < G; ++g) {
            bm[g] = NEED_KX ? 0u : 0xFFFFFFFFu;
            bx[g] = 0u;
          }
          const uint32_t* pc = lds_c + lane;
          const uint8_t* pdg = lds_d + lane;
          for (int32_t c0 = 0; c0 < nc; c0 += R) {
            uint32_t D[R], C[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
              const int32_t c = c0 + r;
              const uint32_t d = pdg[c * WAVE];
              // class 0: staged cost; class 1 (tolerates): every real node is feasible.
              // Padding nodes carry digit 0xFF and never match.
              const uint32_t cost = (cls == 0) ? pc[c * WAVE] : idx_base + (uint32_t)(c * WAVE);
              if (NEED_KX) {
                D[r] = d;
                const bool feas = (cls == 0) ? cost < MATCH_LIMIT : (cost < (uint32_t)a.n_nodes);
                C[r] = feas ? KMAX - cost : 0u;  // class key
              } else {
                D[r] = d << 24;
                C[r] = cost;
              }
            }
#pragma unroll
            for (int g = 0; g < G; ++g) {
              if (g < cnt) {
                if (NEED_KX) {
                  const uint32_t pd = spd[g];
#pragma unroll
                  for (int r = 0; r < R; r += 2) {
                    uint32_t t0 = (D[r] == pd) ? C[r] : 0u;
                    uint32_t t1 = (D[r + 1] == pd) ? C[r + 1] : 0u;
                    uint32_t x0 = (D[r] == pd) ? 0u : C[r];
                    uint32_t x1 = (D[r + 1] == pd) ? 0u : C[r + 1];
                    asm("" : "+v"(t0), "+v"(t1), "+v"(x0), "+v"(x1));
                    bm[g] = umax(umax(bm[g], t0), t1);
                    bx[g] = umax(umax(bx[g], x0), x1);
                  }
                } else {
                  const uint32_t pd = spd[g] << 24;
#pragma unroll
                  for (int r = 0; r < R; r += 2)
                    bm[g] = umin(umin(bm[g], sad(D[r], pd, C[r])), sad(D[r + 1], pd, C[r + 1]));
                }
              }
            }
          }
          // ---- stage 4: wave-wide first-max, result into the pod's lane ----
#pragma unroll
          for (int g = 0; g < G; ++g) {
            if (g < cnt) {
              const uint32_t vm = NEED_KX ? wave_max_u32(bm[g]) : cost_to_key(wave_min_u32(bm[g]));
              res_m = (lane == lsel[g]) ? umax(vm, res_m) : res_m;
              if (NEED_KX) {
                const uint32_t vx = wave_max_u32(bx[g]);
                res_x = (lane == lsel[g]) ? umax(vx, res_x) : res_x;
              }
            }
          }
        }
      }

      if (!act) continue;
      const int32_t j = w0 + lane;
      if (!last_tile) {
        a.partial[j] = res_m;
        if (NEED_KX) a.partial[(size_t)a.n_pods + j] = res_x;
        continue;
      }
      const uint32_t ball = tolv ? ball1 : ball0;
      if (SHARD) {
        a.keys[j] = res_m ? shard_key(a.node_base, KMAX - res_m) : 0;
        if (NEED_KX) a.keys[(size_t)a.n_pods + j] = res_x ? shard_key(a.node_base, KMAX - res_x) : 0;
      } else {
        decode_pod(key_to_idx(res_m), key_to_idx(res_x), key_to_idx(ball), pdv != POD_DIGIT_NONE,
                   a.pp, &a.out_idx[j], &a.out_score[j], &a.out_status[j]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// IDENT batched kernel (normalize NONE / DEFAULT, i.e. the reference plugin set): packed-16.
// Workgroup = 8 waves. Each wave owns a contiguous pod range, walked in windows of 64 pods,
// processed in groups of G2 pod PAIRS. A pair's two pod codes sit in one SGPR
//   PP = (code_B << 26) | (code_A << 10)
// and every node word holds (code << 10 | chunk) in both 16-bit halves, so
//   x = W ^ PP        -> low half: (pod A, node) pair, high half: (pod B, node) pair;
//                        a half is < 1024 exactly when the node is feasible and its digit
//                        equals the pod's, and then it IS the node's chunk in the tile
//   bm = v_pk_minimum3_f16(bm, x_r, x_r+1) -> per lane, the first matching chunk for both pods
// = 3 VALU per 4 x 64 (pod, node) pairs. At the end of a tile the
// lane is folded in (chunk << 6 | lane = node index) and one packed DPP min per pair gives
// both pods' first feasible match. Node words come from LDS (staged once per workgroup,
// 4 B/node) or, DIRECT, straight from L1/L2. Pods that tolerate the unschedulable taint
// additionally scan `ulist` (the nodes only they may use), so every pair is evaluated once;
// pods whose name has no digit suffix get SCORE_ERROR whenever a node is feasible (the
// reference's Score fails on the first feasible node), so they skip the scan.
// ---------------------------------------------------------------------------------------
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
  const u16x2 x = __builtin_bit_cast(u16x2, a), y = __builtin_bit_cast(u16x2, b);
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(x, y));
}

__device__ __forceinline__ uint32_t pk_shl6(uint32_t a) {
  const u16x2 x = __builtin_bit_cast(u16x2, a);
  return __builtin_bit_cast(uint32_t, (u16x2)(x << (u16x2){6, 6}));
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_pkmin(uint32_t v) {
  // Rows masked off by ROW_MASK (row_bcast steps) get an undefined `t`; the min then leaves
  // garbage only in rows whose values never reach lane 63, the one lane read at the end.
  const uint32_t t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, ROW_MASK, 0xF, false);
  return pk_min_u16(v, t);
}

// chunk << 6 | lane in both halves, "no match" halves (>= 1024) saturated to chunk 1023 first
// (-> 0xFFC0 | lane, >= NOMATCH16): v_pk_min_u16 + v_pk_mad_u16 (bm * 64 + lane). Plain vector
// arithmetic, not asm: the permlane swaps that read the result need the compiler to see the
// VALU write (hazard wait states).
__device__ __forceinline__ uint32_t pk_fold_lane(uint32_t bm, uint32_t lane2) {
  const u16x2 c = __builtin_bit_cast(u16x2, pk_min_u16(bm, 0x03FF03FFu));
  const u16x2 l = __builtin_bit_cast(u16x2, lane2);
  const u16x2 k = {64, 64};
  return __builtin_bit_cast(uint32_t, (u16x2)(c * k + l));
}

// Wave-wide packed u16 min of FOUR registers at once. v_permlane32_swap folds a and b into one
// register (a's 32-lane partial in lanes 0..31, b's in 32..63), likewise c and d; one
// v_permlane16_swap folds those two into one register whose rows hold a, c, b, d; four in-row
// DPP steps finish all four: 14 VALU for four pairs where four DPP trees take 48.
// Row r of the result (any lane of it) holds: r=0 a, r=1 c, r=2 b, r=3 d.
__device__ __forceinline__ uint32_t wave_pkmin_u16_x4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const auto ab = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  const auto cd = __builtin_amdgcn_permlane32_swap(c, d, false, false);
  const uint32_t x = pk_min_u16(ab[0], ab[1]);
  const uint32_t y = pk_min_u16(cd[0], cd[1]);
  const auto xy = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  uint32_t v = pk_min_u16(xy[0], xy[1]);
  v = dpp_pkmin<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
  v = dpp_pkmin<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
  v = dpp_pkmin<0x141, 0xF>(v);  // row_half_mirror
  v = dpp_pkmin<0x140, 0xF>(v);  // row_mirror: every lane of a row holds the row's min
  return v;
}

constexpr int ULIST_STEP = 256;  // ulist entries per block of independent loads (divides NODE_PAD)
constexpr int IDENT_THREADS = 512;
#ifndef MSH_UNIT
#define MSH_UNIT 8
#endif
constexpr int IDENT_UNIT = MSH_UNIT;  // pods per work-queue unit (ident_dyn_kernel): 2*QB
#ifndef MSH_QB
#define MSH_QB 4
#endif
constexpr int QB = MSH_QB;  // pod pairs per interleaved block (independent v_pk_min chains)
constexpr uint32_t NOMATCH16 = 0xFFC0u;  // (1023 << 6): above every chunk<<6|lane of a tile

// R chunks of node words (one dword per lane each) starting at chunk c0 of the slice (c0 and
// R multiples of 4). The table is laid out in 4-chunk groups, lane-major (word_pos), so one
// 16-byte load per lane brings 4 chunks. DIRECT: buffer_load_dwordx4 off a wave-uniform
// descriptor; the per-lane offsets are loop-invariant VGPRs and the block offset an SGPR, so
// the scan loop spends no VALU on addressing.
template <bool DIRECT, int R>
__device__ __forceinline__ void load_words(uint32_t (&w)[R], const uint32_t* __restrict__ words,
                                           __amdgpu_buffer_rsrc_t rs, int32_t c0, int lane) {
  static_assert(R % 4 == 0, "whole 4-chunk groups");
#pragma unroll
  for (int g = 0; g < R / 4; ++g) {
    uint4 v;
    if constexpr (DIRECT) {
      const auto t = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16 + g * (4 * WAVE * 4),
                                                           c0 * (WAVE * 4), 0);
      v = __builtin_bit_cast(uint4, t);
    } else {
      v = reinterpret_cast<const uint4*>(words)[(c0 / 4 + g) * WAVE + lane];
    }
    w[4 * g + 0] = v.x;
    w[4 * g + 1] = v.y;
    w[4 * g + 2] = v.z;
    w[4 * g + 3] = v.w;
  }
}

#ifndef MSH_MIN3
#define MSH_MIN3 1
#endif
// Largest finite f16 in both halves: "no match yet", and never a NaN for v_pk_minimum3_f16.
constexpr uint32_t BM_INIT = 0x7BFF7BFFu;

// Packed IEEE minimum of three f16 pairs, used as an integer min: every operand is a
// non-negative finite f16 (see the w16 layout in msh_internal.h), whose order is its bit order.
__device__ __forceinline__ uint32_t pk_min3_f16bits(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_pk_minimum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// v_xor_b32 with both sources in VGPRs. gfx950 issues the all-VGPR VOP2 form of xor / add / and
// at ~2 cycles per wave64 instruction on a SIMD32, but every form with an SGPR (or constant)
// source, and v_min*/VOP3/VOP3P, at ~4 (scripts/ubench_valu3.hip, profiles/r1_ubench_valu3.jsonl):
// the pod-pair code is therefore held in a VGPR (same value in every lane), not an SGPR.
#ifndef MSH_XOR_VV
#define MSH_XOR_VV 1
#endif
__device__ __forceinline__ uint32_t xor_vv(uint32_t a, uint32_t b) {
  uint32_t r;
  if (MSH_XOR_VV)
    asm("v_xor_b32_e32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  else
    r = a ^ b;
  return r;
}

// A wave-uniform value copied into a VGPR (one v_mov per group, outside the scan loop).
__device__ __forceinline__ uint32_t to_vgpr(uint32_t s) {
  uint32_t r;
  if (MSH_XOR_VV)
    asm("v_mov_b32_e32 %0, %1" : "=v"(r) : "s"(s));
  else
    r = s;
  return r;
}

// Per pod pair (PP, held in a VGPR) and two node words: x = W ^ PP (v_xor_b32, a half is < 1024
// iff that node matches that pod), bm = min3(bm, x_r, x_r+1) -> 3 VALU per 4 x 64 pairs (0.75
// lane-op per pair). MSH_MIN3=0: bm = pk_min_u16(bm, x), 1.0 lane-op per pair.
template <int R, int GQ>
__device__ __forceinline__ void scan_words(const uint32_t (&w)[R], const uint32_t (&pp)[GQ],
                                           uint32_t (&bm)[GQ], int32_t cnt) {
  static_assert(R % 2 == 0, "chunks are folded two at a time");
#pragma unroll
  for (int qb = 0; qb < GQ; qb += QB) {
    constexpr int QB_ = QB;  // the last block may be partial when GQ is not a multiple of QB
    if (qb < cnt) {
#pragma unroll
      for (int r = 0; r < R; r += 2) {
        uint32_t x[QB_], y[QB_];
#pragma unroll
        for (int q = 0; q < QB_; ++q) {
          if (qb + q >= GQ) break;
          x[q] = xor_vv(w[r], pp[qb + q]);
          y[q] = xor_vv(w[r + 1], pp[qb + q]);
        }
#pragma unroll
        for (int q = 0; q < QB_; ++q) {
          if (qb + q >= GQ) break;
          if (MSH_MIN3) {
            bm[qb + q] = pk_min3_f16bits(bm[qb + q], x[q], y[q]);
          } else {
            bm[qb + q] = pk_min_u16(pk_min_u16(bm[qb + q], x[q]), y[q]);
          }
        }
      }
    }
  }
}

// One group of up to GQ pod pairs taken from `mask` (lanes of the window), scanned against
// node words [0, nc) chunks of the current tile slice; results min-merged into `res`.
// `node_base` = global index of chunk 0 of the compute tile the slice belongs to.
// nc is a multiple of 2R: two register blocks alternate (load one, scan the other) with no
// copies between them.
template <int R, int GQ, bool DIRECT>
__device__ __forceinline__ void ident_group(unsigned long long& mask, uint32_t pcv, uint32_t& res,
                                            const uint32_t* __restrict__ words,
                                            __amdgpu_buffer_rsrc_t rs, int32_t nc,
                                            uint32_t node_base, int lane) {
  static_assert(GQ % QB == 0, "GQ must be a multiple of QB");
  static_assert(GQ % 4 == 0, "pairs are reduced four at a time");
  uint32_t pp[GQ];
  int32_t la[GQ], lb[GQ];
  int32_t cnt = 0;
#pragma unroll
  for (int q = 0; q < GQ; ++q) {
    uint32_t ca = CODE_NONE_POD, cb = CODE_NONE_POD;
    la[q] = -1;
    lb[q] = -1;
    if (mask) {
      la[q] = (int32_t)__builtin_ctzll(mask);
      mask &= mask - 1;
      ca = (uint32_t)__builtin_amdgcn_readlane((int)pcv, la[q]);
      cnt = q + 1;
      if (mask) {
        lb[q] = (int32_t)__builtin_ctzll(mask);
        mask &= mask - 1;
        cb = (uint32_t)__builtin_amdgcn_readlane((int)pcv, lb[q]);
      }
    }
    pp[q] = to_vgpr((cb << (16 + CODE_SHIFT)) | (ca << CODE_SHIFT));
  }
  uint32_t bm[GQ];
#pragma unroll
  for (int q = 0; q < GQ; ++q) bm[q] = BM_INIT;
  uint32_t wa[R], wb[R];
  load_words<DIRECT>(wa, words, rs, 0, lane);
#ifdef MSH_DIAG_REUSE  // timing diagnostic only (wrong results): no node-word loads in the loop
  load_words<DIRECT>(wb, words, rs, R, lane);
  for (int32_t c0 = 0; c0 < nc; c0 += 2 * R) {
    scan_words<R, GQ>(wa, pp, bm, cnt);
    scan_words<R, GQ>(wb, pp, bm, cnt);
    wa[c0 & (R - 1)] += 1u;
  }
#else
  for (int32_t c0 = 0; c0 < nc; c0 += 2 * R) {
    load_words<DIRECT>(wb, words, rs, c0 + R, lane);
    scan_words<R, GQ>(wa, pp, bm, cnt);
    // DIRECT: the next block's load is issued unconditionally; past the slice the buffer
    // descriptor's range check returns zeros, which are never scanned. A branch around it
    // would merge two vmcnt states and make the wait before scan(wb) cover this load too.
    if (DIRECT || c0 + 2 * R < nc) load_words<DIRECT>(wa, words, rs, c0 + 2 * R, lane);
    scan_words<R, GQ>(wb, pp, bm, cnt);
  }
#endif
  // ---- stage 4: fold in the lane, then one transposed cross-lane min per 4 pairs ----
  const uint32_t lane2 = (uint32_t)lane | ((uint32_t)lane << 16);
#pragma unroll
  for (int q0 = 0; q0 < GQ; q0 += 4) {
    if (q0 < cnt) {
      const uint32_t x = wave_pkmin_u16_x4(pk_fold_lane(bm[q0], lane2), pk_fold_lane(bm[q0 + 1], lane2),
                                           pk_fold_lane(bm[q0 + 2], lane2), pk_fold_lane(bm[q0 + 3], lane2));
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (q0 + k < cnt) {
          // pair k's two results sit in row {0, 2, 1, 3}[k]
          const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)x, 16 * ((k & 1) * 2 + (k >> 1)));
          const uint32_t lo = v & 0xFFFFu, hi = v >> 16;
          const uint32_t ga = lo < NOMATCH16 ? node_base + lo : NOFIT;
          const uint32_t gb = hi < NOMATCH16 ? node_base + hi : NOFIT;
          res = (lane == la[q0 + k]) ? umin(res, ga) : res;
          res = (lane == lb[q0 + k]) ? umin(res, gb) : res;
        }
      }
    }
  }
}

// Tolerating pods (set bits of `mt`): a pass over ulist, the nodes feasible for
// them alone. The list is read in whole ULIST_STEP-entry blocks (sentinel-padded, no bounds
// check), ULIST_WIN blocks at a time into registers: each window is loaded ONCE for all the
// tolerating pods of the wave (the entries do not depend on the pod), which then take it two at
// a time with two independent wave reductions in flight. Entry ^ (digit << 24) is < 2^24
// exactly on a digit match, and then it is the node index; a window's per-pod minimum folds
// into `res` by min, so windows and the main scan combine in any order.
constexpr int ULIST_WIN = 2;
__device__ __forceinline__ uint32_t ulist_pass(unsigned long long mt, uint32_t pcv, uint32_t res,
                                               const uint32_t* __restrict__ ulist, uint32_t ucnt,
                                               int lane) {
  constexpr int NL = ULIST_STEP / WAVE;
  const uint32_t nblk = (ucnt + ULIST_STEP - 1) / ULIST_STEP;
  // wave-uniform descriptor: block offset in an SGPR, lane offset one loop-invariant VGPR
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)ulist, (short)0, (int32_t)(nblk * ULIST_STEP * sizeof(uint32_t)), 0x00020000);
#pragma unroll 1
  for (uint32_t b0 = 0; b0 < nblk; b0 += ULIST_WIN) {
    uint32_t x[ULIST_WIN * NL];
#pragma unroll
    for (int b = 0; b < ULIST_WIN; ++b)
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        const uint32_t v = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(
            rs, lane * 4 + i * WAVE * 4, (int)((b0 + b) * ULIST_STEP * 4), 0);
        x[b * NL + i] = b0 + b < nblk ? v : 0xFFFFFFFFu;  // past the list: never a match
      }
    unsigned long long m = mt;
#pragma unroll 1
    while (m) {
      const int32_t l0 = (int32_t)__builtin_ctzll(m);
      m &= m - 1;
      const int32_t l1 = m ? (int32_t)__builtin_ctzll(m) : l0;  // an odd last pod goes twice
      if (m) m &= m - 1;
      const uint32_t p0 = (uint32_t)__builtin_amdgcn_readlane((int)pcv, l0) << 24;
      const uint32_t p1 = (uint32_t)__builtin_amdgcn_readlane((int)pcv, l1) << 24;
      uint32_t u0 = 0xFFFFFFFFu, u1 = 0xFFFFFFFFu;
#pragma unroll
      for (int i = 0; i < ULIST_WIN * NL; i += 2) {
        u0 = umin(u0, umin(x[i] ^ p0, x[i + 1] ^ p0));
        u1 = umin(u1, umin(x[i] ^ p1, x[i + 1] ^ p1));
      }
      const uint32_t v0 = wave_min_u32(u0), v1 = wave_min_u32(u1);
      if (v0 < MATCH_LIMIT) res = (lane == l0) ? umin(res, v0) : res;
      if (v1 < MATCH_LIMIT) res = (lane == l1) ? umin(res, v1) : res;
    }
  }
  return res;
}

// DIRECT: node words are read straight from global memory (L1/L2-resident: 4 B/node) with no
// LDS staging and no workgroup barrier; otherwise staged in LDS slices of STAGE_CHUNKS.
template <int R, int G2, bool SHARD, bool DIRECT>
__global__ __launch_bounds__(IDENT_THREADS) void ident_kernel(BatchArgs a, int32_t stage_chunks) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  uint32_t* lw0 = reinterpret_cast<uint32_t*>(lds_raw);

  constexpr int WPG = IDENT_THREADS / WAVE;
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t W = (int64_t)gridDim.x * WPG;
  const int64_t gw = (int64_t)blockIdx.x * WPG + wv;
  const int32_t p0 = (int32_t)((int64_t)a.n_pods * gw / W);
  const int32_t p1 = (int32_t)((int64_t)a.n_pods * (gw + 1) / W);
  // stage_chunks divides TILE_CHUNKS, so a stage never straddles two compute tiles
  const int32_t nstages = (a.n_chunks + stage_chunks - 1) / stage_chunks;
  if (SHARD) write_class_keys(a);
  const uint32_t ball0 = a.ball[0], ball1 = a.ball[1];
  const uint32_t ucnt = *a.ucount;
  MSH_STAMP(0);

  for (int32_t st = 0; st < nstages; ++st) {
    const int32_t s0 = st * stage_chunks;
    const int32_t nc = min(stage_chunks, a.n_chunks - s0);  // multiple of 16
    // global index of chunk 0 of this stage's compute tile (words hold tile-relative chunks)
    const uint32_t tile_node_base = (uint32_t)(s0 / TILE_CHUNKS) * (uint32_t)TILE_NODES;
    const uint32_t* words;
    if (DIRECT) {
      words = a.w0 + (size_t)s0 * WAVE;
    } else {
      if (st > 0) __syncthreads();
      const uint4* src0 = reinterpret_cast<const uint4*>(a.w0 + (size_t)s0 * WAVE);
      uint4* dst0 = reinterpret_cast<uint4*>(lw0);
      const int32_t n0 = nc * (WAVE / 4);
      for (int32_t i = threadIdx.x; i < n0; i += 4 * IDENT_THREADS) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (i + k * IDENT_THREADS < n0) v[k] = src0[i + k * IDENT_THREADS];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (i + k * IDENT_THREADS < n0) dst0[i + k * IDENT_THREADS] = v[k];
      }
      __syncthreads();
      words = lw0;
    }
    MSH_STAMP(1);
    const bool last_stage = (st == nstages - 1);
    // wave-uniform descriptor over this slice's words (DIRECT); unused for the LDS variant
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)words, (short)0, DIRECT ? nc * WAVE * (int32_t)sizeof(uint32_t) : 0, 0x00020000);

    for (int32_t w0 = p0; w0 < p1; w0 += WAVE) {
      const int32_t nwin = min((int32_t)WAVE, p1 - w0);
      const bool act = lane < nwin;
      uint32_t pcv = CODE_NONE_POD, tolv = 0;
      if (act) {
        const int d = a.pod_digit[w0 + lane];
        pcv = (d >= 0 && d <= 9) ? (uint32_t)d : CODE_NONE_POD;
        tolv = a.pod_tol[w0 + lane] ? 1u : 0u;
      }
      uint32_t res = NOFIT;  // global index of the first feasible match, NOFIT = none
      if (st > 0 && act) res = a.partial[w0 + lane];
      unsigned long long m = __ballot(act && pcv != CODE_NONE_POD);
      MSH_STAMP(2);
      while (m) ident_group<R, G2, DIRECT>(m, pcv, res, words, rs, nc, tile_node_base, lane);
      MSH_STAMP(3);

      // tolerating pods: the class-1-only nodes (ulist), once (first stage)
      const unsigned long long mt = __ballot(act && tolv != 0u && pcv != CODE_NONE_POD);
      if (st == 0 && mt) res = ulist_pass(mt, pcv, res, a.ulist, ucnt, lane);
      MSH_STAMP(4);

      if (!act) continue;
      const int32_t j = w0 + lane;
      if (!last_stage) {
        a.partial[j] = res;
        continue;
      }
      const uint32_t ball = tolv ? ball1 : ball0;
      if (SHARD) {
        a.keys[j] = res != NOFIT ? shard_key(a.node_base, res) : 0;
      } else {
        decode_ident(res != NOFIT ? (int64_t)res : -1, key_to_idx(ball), pcv != CODE_NONE_POD,
                     make_ident_decode(a.pp), &a.out_idx[j], &a.out_score[j], &a.out_status[j]);
      }
    }
  }
  MSH_STAMP(5);
#ifdef MSH_STAMPS
  if (lane == 0 && gw < STAMP_WAVES) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    msh_stamp_buf[((size_t)gw * STAMPS_PER_WAVE + 7) * 2] = hw;
    msh_stamp_buf[((size_t)gw * STAMPS_PER_WAVE + 7) * 2 + 1] = xcc;
  }
#endif
}

// ---------------------------------------------------------------------------------------
// Work-queue IDENT kernel (default for single-tile node tables, DIRECT reads). Same per-pair
// arithmetic as ident_kernel; the difference is how pods reach waves. With a static pod range
// per wave, age-priority issue leaves the youngest wave of every SIMD running alone at the end
// of the launch (per-wave stamps at C3: 18k..58k cycles for equal work), and a wave's last
// partial group wastes pair slots. Here one workgroup of 16 waves per CU (4 per SIMD) owns a
// contiguous pod range and its waves draw IDENT_UNIT-pod units (one QB block of pod pairs) from
// an LDS counter until the range is spent: the SIMDs of a CU drain together, the tail is one
// unit, and no global atomics or cross-launch state are involved.
// ---------------------------------------------------------------------------------------
constexpr int DYN_THREADS = 1024;
// LDS size class of the LDS-resident variant: 288 chunks (18,432 nodes incl. the pad) = 72 KiB,
// two 1024-thread workgroups per CU
constexpr int DYN_LDS_CHUNKS = 288;
#ifndef MSH_DYN_LDS_DEFAULT
#define MSH_DYN_LDS_DEFAULT 0
#endif

// One 8-pod unit of the work-queue kernel, pods in lanes 0..7 with FIXED pairs: pair q = lanes
// 2q (low half) and 2q+1 (high half), pods without a digit included (their code 14 never
// matches; decode turns them into SCORE_ERROR). Compared with ident_group (pairs formed from a
// ballot mask, each pod's result picked out by readlane + compare + select), the pair codes come
// from one DPP step and four readlanes, and the four reduced pairs reach their pods' lanes with
// ONE ds_bpermute. Returns, in lanes 0..7, the pod's first feasible matching node index in the
// tile, or NOFIT.
#ifndef MSH_UNIT8
#define MSH_UNIT8 1
#endif
// R chunks of node words from the workgroup's LDS copy of the table (same lane-major 4-chunk
// groups as in global memory): one conflict-free ds_read_b128 per lane per 4 chunks.
template <int R>
__device__ __forceinline__ void load_words_lds(uint32_t (&w)[R], const uint4* lw, int32_t c0, int lane) {
  static_assert(R % 4 == 0, "whole 4-chunk groups");
#pragma unroll
  for (int g = 0; g < R / 4; ++g) {
    const uint4 v = lw[(c0 / 4 + g) * WAVE + lane];
    w[4 * g + 0] = v.x;
    w[4 * g + 1] = v.y;
    w[4 * g + 2] = v.z;
    w[4 * g + 3] = v.w;
  }
}

// `wa` holds chunks [0, R) on entry (requested by the caller together with the pod bytes).
// NP pod pairs (1..8; IDENT_UNIT / 2 for the work queue): pair q = lanes 2q (low half) and
// 2q+1 (high half).
template <int R, bool LDSW, int NP = IDENT_UNIT / 2>
__device__ __forceinline__ uint32_t ident_unit8(uint32_t pcv, uint32_t (&wa)[R], const uint32_t* __restrict__ words,
                                                __amdgpu_buffer_rsrc_t rs, const uint4* lw, int32_t nc,
                                                int lane) {
  static_assert(NP >= 1 && NP <= 8 && QB == 4, "1..8 pod pairs, scanned in blocks of 4");
  const uint32_t c = pcv << CODE_SHIFT;
  // quad_perm [1,0,3,2]: lane 2q receives lane 2q+1's code
  const uint32_t partner = (uint32_t)__builtin_amdgcn_mov_dpp((int)c, 0xB1, 0xF, 0xF, false);
  const uint32_t ppl = c | (partner << 16);  // pair code, valid in even lanes
  uint32_t pp[NP], bm[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    pp[q] = to_vgpr((uint32_t)__builtin_amdgcn_readlane((int)ppl, 2 * q));
    bm[q] = BM_INIT;
  }
  uint32_t wb[R];
#ifdef MSH_DIAG_NOLOAD  // timing diagnostic only (wrong results): node words loaded once
  load_words<true>(wb, words, rs, R, lane);
  for (int32_t c0 = 0; c0 < nc; c0 += 2 * R) {
    scan_words<R, NP>(wa, pp, bm, NP);
    scan_words<R, NP>(wb, pp, bm, NP);
    wa[0] += 1u;
  }
#else
  if (LDSW) {
    for (int32_t c0 = 0; c0 < nc; c0 += 2 * R) {
      load_words_lds<R>(wb, lw, c0 + R, lane);
      scan_words<R, NP>(wa, pp, bm, NP);
      load_words_lds<R>(wa, lw, c0 + 2 * R, lane);  // past the table: the LDS pad, never scanned
      scan_words<R, NP>(wb, pp, bm, NP);
    }
  } else {
    for (int32_t c0 = 0; c0 < nc; c0 += 2 * R) {
      load_words<true>(wb, words, rs, c0 + R, lane);
      scan_words<R, NP>(wa, pp, bm, NP);
      load_words<true>(wa, words, rs, c0 + 2 * R, lane);  // past the slice: zeros, never scanned
      scan_words<R, NP>(wb, pp, bm, NP);
    }
  }
#endif
  const uint32_t lane2 = (uint32_t)lane | ((uint32_t)lane << 16);
  // pair q's two results sit in row {0, 2, 1, 3}[q % 4] of the reduction of its group of four;
  // every lane of a row holds them, so one ds_bpermute per group brings them to the pods' lanes
  const int q = (lane >> 1) & 3;
  const int row = ((q & 1) << 1) | (q >> 1);
  uint32_t v = 0;
  auto bmq = [&](int q) -> uint32_t { return q < NP ? pk_fold_lane(bm[q < NP ? q : 0], lane2) : 0xFFFFFFFFu; };
#pragma unroll
  for (int g = 0; g < (NP + 3) / 4; ++g) {
    const uint32_t x = wave_pkmin_u16_x4(bmq(4 * g), bmq(4 * g + 1), bmq(4 * g + 2), bmq(4 * g + 3));
    const uint32_t vg = (uint32_t)__builtin_amdgcn_ds_bpermute(row * 16 * 4, (int)x);
    v = (lane >> 3) == g ? vg : v;
  }
  const uint32_t h = (lane & 1) ? (v >> 16) : (v & 0xFFFFu);
  return h < NOMATCH16 ? h : NOFIT;
}

// MULTI: the node table spans several 64,512-node compute tiles (word halves hold tile-relative
// chunks). A unit scans the tiles in List order and keeps the first tile with a match: the whole
// table per unit, no running results in memory between launches or stages.
template <int R, bool SHARD, int NT = DYN_THREADS, bool LDSW = false, bool MULTI = false>
__global__ __launch_bounds__(NT) void ident_dyn_kernel(BatchArgs a) {
  __shared__ uint32_t next_unit;
  // LDSW: the workgroup's copy of the node words (nc + R chunks, the last R a zero pad that the
  // scan loop's one-block-ahead read may touch but never scans)
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_words[];
  const int lane = threadIdx.x & (WAVE - 1);
#ifdef MSH_STAMPS
  // diagnostic stamps: 0 entry, 1 first unit fetched, 2 its pods loaded, 3 its groups scanned,
  // 4 its ulist scanned, 5 exit; slot 6 = units taken by this wave; 7 = hardware ids
  const int64_t gw = (int64_t)blockIdx.x * (NT / WAVE) + (threadIdx.x >> 6);
  uint32_t n_taken = 0;
#endif
  MSH_STAMP(0);
  // tile 0 (the whole table unless MULTI)
  const int32_t nc = MULTI ? min(a.n_chunks, (int32_t)TILE_CHUNKS) : a.n_chunks;
  const uint32_t* words = a.w0;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)words, (short)0, nc * WAVE * (int32_t)sizeof(uint32_t), 0x00020000);
  // Per-launch scalars written by the prep kernel, requested as VECTOR loads so that nothing
  // waits for them before the first unit: a scalar load would share lgkmcnt with the LDS work
  // counter and put two dependent round trips in front of every wave's first claim.
  const uint32_t bvec = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(
      __builtin_amdgcn_make_buffer_rsrc((void*)a.ball, (short)0, 8, 0x00020000), (lane & 1) * 4, 0, 0);
  const uint32_t uvec = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(
      __builtin_amdgcn_make_buffer_rsrc((void*)a.ucount, (short)0, 4, 0x00020000), 0, 0, 0);
  if (SHARD) write_class_keys(a);
  // this workgroup's contiguous unit range (host-computed quotient/remainder: no 64-bit division)
  const int32_t b = (int32_t)blockIdx.x;
  const int32_t ub = b * a.unit_q + min(b, a.unit_r);
  const int32_t n_units = a.unit_q + (b < a.unit_r ? 1 : 0);
  const int32_t g0 = ub * IDENT_UNIT;
  const int32_t g1 = min(g0 + n_units * IDENT_UNIT, a.n_pods);
  const uint4* lw = reinterpret_cast<const uint4*>(lds_words);
  if (LDSW) {
    const uint4* src = reinterpret_cast<const uint4*>(words);
    uint4* dst = reinterpret_cast<uint4*>(lds_words);
    const int32_t n16 = nc * (WAVE / 4), pad16 = (nc + R) * (WAVE / 4);
    for (int32_t i = threadIdx.x; i < pad16; i += NT) dst[i] = i < n16 ? src[i] : make_uint4(0, 0, 0, 0);
  }
  if (threadIdx.x == 0) next_unit = 0;
  __syncthreads();
  auto claim = [&]() -> uint32_t {
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(&next_unit, 1u);
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
  };
  // (claiming the next unit and requesting its pod bytes before scanning the current one was
  // measured 1 us slower isolated at C3, and no faster pipelined)
  for (uint32_t u = claim(); u < (uint32_t)n_units; u = claim()) {
#ifdef MSH_STAMPS
    const bool first_unit = n_taken++ == 0;
    if (first_unit) MSH_STAMP(1);
#endif
    const int32_t w0 = g0 + (int32_t)u * IDENT_UNIT;
    const int32_t nwin = min((int32_t)IDENT_UNIT, g1 - w0);
    const bool act = lane < nwin;
    // the unit's first block of node words is requested before the pod bytes are waited for
    uint32_t wa[R];
    if (LDSW)
      load_words_lds<R>(wa, lw, 0, lane);
    else
      load_words<true>(wa, words, rs, 0, lane);
    uint32_t pcv = CODE_NONE_POD, tolv = 0;
    if (act) {
      const int d = a.pod_digit[w0 + lane];
      pcv = (d >= 0 && d <= 9) ? (uint32_t)d : CODE_NONE_POD;
      tolv = a.pod_tol[w0 + lane] ? 1u : 0u;
    }
    uint32_t res = NOFIT;
    unsigned long long m = __ballot(act && pcv != CODE_NONE_POD);
#ifdef MSH_STAMPS
    if (first_unit) MSH_STAMP(2);
#endif
    if (MSH_UNIT8) {
      if (m) res = ident_unit8<R, LDSW>(pcv, wa, words, rs, lw, nc, lane);
      if (MULTI && m) {
        for (int32_t t0 = TILE_CHUNKS; t0 < a.n_chunks; t0 += TILE_CHUNKS) {
          const int32_t nct = min(a.n_chunks - t0, (int32_t)TILE_CHUNKS);
          const uint32_t* wt = a.w0 + (size_t)t0 * WAVE;
          const __amdgpu_buffer_rsrc_t rst = __builtin_amdgcn_make_buffer_rsrc(
              (void*)wt, (short)0, nct * WAVE * (int32_t)sizeof(uint32_t), 0x00020000);
          load_words<true>(wa, wt, rst, 0, lane);
          const uint32_t rt = ident_unit8<R, false>(pcv, wa, wt, rst, lw, nct, lane);
          // tiles ascend in List order: an earlier tile's match is always the smaller index
          if (res == NOFIT && rt != NOFIT) res = (uint32_t)(t0 / TILE_CHUNKS) * (uint32_t)TILE_NODES + rt;
        }
      }
    } else {
      while (m) ident_group<R, IDENT_UNIT / 2, true>(m, pcv, res, words, rs, nc, 0u, lane);
    }
#ifdef MSH_STAMPS
    if (first_unit) MSH_STAMP(3);
#endif
    const unsigned long long mt = __ballot(act && tolv != 0u && pcv != CODE_NONE_POD);
    if (mt) res = ulist_pass(mt, pcv, res, a.ulist, (uint32_t)__builtin_amdgcn_readfirstlane((int)uvec), lane);
#ifdef MSH_STAMPS
    if (first_unit) MSH_STAMP(4);
#endif
    if (act) {
      const int32_t j = w0 + lane;
      const uint32_t ball = tolv ? (uint32_t)__builtin_amdgcn_readlane((int)bvec, 1)
                                 : (uint32_t)__builtin_amdgcn_readlane((int)bvec, 0);
      if (SHARD) {
        a.keys[j] = res != NOFIT ? shard_key(a.node_base, res) : 0;
      } else {
        decode_ident(res != NOFIT ? (int64_t)res : -1, key_to_idx(ball), pcv != CODE_NONE_POD,
                     make_ident_decode(a.pp), &a.out_idx[j], &a.out_score[j], &a.out_status[j]);
      }
    }
  }
  MSH_STAMP(5);
#ifdef MSH_STAMPS
  if (lane == 0 && gw < STAMP_WAVES) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    msh_stamp_buf[((size_t)gw * STAMPS_PER_WAVE + 6) * 2] = n_taken;
    msh_stamp_buf[((size_t)gw * STAMPS_PER_WAVE + 7) * 2] = hw;
    msh_stamp_buf[((size_t)gw * STAMPS_PER_WAVE + 7) * 2 + 1] = xcc;
  }
#endif
}

// ---------------------------------------------------------------------------------------
// One-range-per-wave IDENT kernel: when the batch gives every wave of a full chip at most 8
// pod PAIRS, each wave takes ONE contiguous range of q or q + 1 pairs and scans the table once
// for all of them: no work-queue claims, no workgroup barrier, one cross-lane reduction per 4
// pairs. Pairs, not pods, are dealt out so that no wave pads a half-empty pair slot, and the
// r = Q mod W waves that take one more pair are spread across workgroups (wave rank =
// wave-in-workgroup x grid + workgroup), so every CU gets the same work to within a pair per
// workgroup. NP = the longest range, in pairs; the shorter ranges run the NP - 1 body.
// ---------------------------------------------------------------------------------------
template <int R, bool SHARD, int NP, int WT>
__global__ __launch_bounds__(WT) __attribute__((amdgpu_waves_per_eu(8))) void ident_wave_kernel(BatchArgs a,
                                                                                      int32_t rounds,
                                                                                      int32_t xcd) {
  const int lane = threadIdx.x & (WAVE - 1);
  const int32_t wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int32_t gd = (int32_t)gridDim.x, b = (int32_t)blockIdx.x;
  int32_t g, np, ps;
  if (xcd) {
    // XCD-contiguous ranks: workgroups are dispatched round-robin over the 8 XCDs (b mod 8), so
    // XCD x's workgroups take one contiguous block of ranks and neighbouring ranges (whose output
    // cache lines they share) are written through the same L2. The +1 pairs are spread evenly in
    // rank order (Bresenham): rank g takes pairs [g q + floor(g r / W), (g + 1) q + floor((g + 1) r / W)).
    const int32_t x = b & 7, base = gd >> 3, extra = gd & 7;
    g = (x * base + min(x, extra) + (b >> 3)) * (WT / WAVE) + wv;
    const uint32_t W = (uint32_t)a.unit_w, r = (uint32_t)a.unit_r;
    const int32_t lo = (int32_t)((uint32_t)g * r / W), hi = (int32_t)((uint32_t)(g + 1) * r / W);
    np = a.unit_q + (hi - lo);
    ps = g * a.unit_q + lo;
  } else {
    g = wv * gd + b;
    np = a.unit_q + (g < a.unit_r ? 1 : 0);
    ps = g * a.unit_q + min(g, a.unit_r);
  }
  const int32_t nc = a.n_chunks;  // one compute tile
  const uint32_t* words = a.w0;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)words, (short)0, nc * WAVE * (int32_t)sizeof(uint32_t), 0x00020000);
  const uint32_t bvec = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(
      __builtin_amdgcn_make_buffer_rsrc((void*)a.ball, (short)0, 8, 0x00020000), (lane & 1) * 4, 0, 0);
  const uint32_t uvec = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(
      __builtin_amdgcn_make_buffer_rsrc((void*)a.ucount, (short)0, 4, 0x00020000), 0, 0, 0);
  if (SHARD) write_class_keys(a);
  // (xcd = 0, A/B: rank g = wave-in-workgroup x grid + workgroup takes pairs [g q + min(g, r),
  // +q (+1 if g < r)); q / r / W host-computed: unit_q / unit_r / unit_w)
  // ranks past the W-th start at or past P (2 (g q + r) >= 2 (W q + r) = 2Q >= P)
  if (2 * ps >= a.n_pods) return;  // whole waves only; no barrier follows
  // the range in `rounds` rounds of np * j / rounds .. np * (j + 1) / rounds pairs: NP or NP - 1
  // each (the host picks rounds and NP so; one round unless the batch exceeds 8 pairs per wave)
#pragma unroll 1
  for (int32_t j = 0; j < rounds; ++j) {
    const int32_t r0 = np * j / rounds, r1 = np * (j + 1) / rounds;
    const int32_t w0 = 2 * (ps + r0);
    if (r1 == r0 || w0 >= a.n_pods) continue;
    const int32_t nwin = min(2 * (r1 - r0), a.n_pods - w0);
    const bool act = lane < nwin;
    uint32_t wa[R];
    load_words<true>(wa, words, rs, 0, lane);  // requested before the pod bytes are waited for
    uint32_t pcv = CODE_NONE_POD, tolv = 0;
    if (act) {
      const int d = a.pod_digit[w0 + lane];
      pcv = (d >= 0 && d <= 9) ? (uint32_t)d : CODE_NONE_POD;
      tolv = a.pod_tol[w0 + lane] ? 1u : 0u;
    }
    // the tolerating pods' ulist pass first: its load latency overlaps the first node words'
    // (already in flight); its per-pod minimum joins the scan's by min
    uint32_t res = NOFIT;
    const unsigned long long mt = __ballot(act && tolv != 0u && pcv != CODE_NONE_POD);
    if (mt) res = ulist_pass(mt, pcv, res, a.ulist, (uint32_t)__builtin_amdgcn_readfirstlane((int)uvec), lane);
    if (__ballot(act && pcv != CODE_NONE_POD)) {
      uint32_t rsc;
      if (NP == 1 || r1 - r0 == NP)
        rsc = ident_unit8<R, false, NP>(pcv, wa, words, rs, nullptr, nc, lane);
      else
        rsc = ident_unit8<R, false, (NP > 1 ? NP - 1 : 1)>(pcv, wa, words, rs, nullptr, nc, lane);
      res = umin(res, rsc);
    }
    if (act) {
      const int32_t jp = w0 + lane;
      if (SHARD) {
        a.keys[jp] = res != NOFIT ? shard_key(a.node_base, res) : 0;
      } else {
        const uint32_t ball = tolv ? (uint32_t)__builtin_amdgcn_readlane((int)bvec, 1)
                                   : (uint32_t)__builtin_amdgcn_readlane((int)bvec, 0);
        decode_ident(res != NOFIT ? (int64_t)res : -1, key_to_idx(ball), pcv != CODE_NONE_POD,
                     make_ident_decode(a.pp), &a.out_idx[jp], &a.out_score[jp], &a.out_status[jp]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Node-split IDENT kernel: few pods against a large table. The work-queue kernel gives each
// 8-pod unit to ONE wave, which then scans the whole table: with 512 pods and 100k nodes, 64
// waves scan 1,563 chunks each while the rest of the chip idles (71 us for 5e7 evaluations).
// Here a TEAM of SPLIT waves of one workgroup shares a unit: wave k scans the k-th slice of
// `slice_chunks` chunks (a multiple of 16, cut at compute-tile boundaries as needed), the
// team's per-pod firsts meet in LDS by atomicMin (slices ascend in List order, so the min is
// the first match of the whole table), and the team's first wave runs the tolerating-pod pass
// and the decode. 16 / SPLIT units per workgroup round, two barriers per round; no global
// scratch, so launches on different streams stay independent.
// ---------------------------------------------------------------------------------------
template <int R, bool SHARD, int SPLIT>
__global__ __launch_bounds__(DYN_THREADS) void ident_split_kernel(BatchArgs a, int32_t slice_chunks) {
  constexpr int WPG = DYN_THREADS / WAVE;
  constexpr int TEAMS = WPG / SPLIT;
  static_assert(SPLIT >= 2 && WPG % SPLIT == 0, "SPLIT divides the workgroup's 16 waves");
  __shared__ uint32_t slot[TEAMS][IDENT_UNIT];
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int team = wv / SPLIT, k = wv % SPLIT;
  const uint32_t bvec = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(
      __builtin_amdgcn_make_buffer_rsrc((void*)a.ball, (short)0, 8, 0x00020000), (lane & 1) * 4, 0, 0);
  const uint32_t uvec = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(
      __builtin_amdgcn_make_buffer_rsrc((void*)a.ucount, (short)0, 4, 0x00020000), 0, 0, 0);
  if (SHARD) write_class_keys(a);
  const int32_t b = (int32_t)blockIdx.x;
  const int32_t ub = b * a.unit_q + min(b, a.unit_r);
  const int32_t n_units = a.unit_q + (b < a.unit_r ? 1 : 0);
  const int32_t g0 = ub * IDENT_UNIT;
  const int32_t g1 = min(g0 + n_units * IDENT_UNIT, a.n_pods);
  // this wave's slice of the table, in global chunks
  const int32_t c_lo = min(k * slice_chunks, a.n_chunks);
  const int32_t c_hi = min(c_lo + slice_chunks, a.n_chunks);
  if (threadIdx.x < TEAMS * IDENT_UNIT) slot[threadIdx.x / IDENT_UNIT][threadIdx.x % IDENT_UNIT] = NOFIT;
  __syncthreads();
  for (int32_t r0 = 0; r0 < n_units; r0 += TEAMS) {  // uniform over the workgroup
    const int32_t u = r0 + team;
    const bool has = u < n_units;
    const int32_t w0 = g0 + u * IDENT_UNIT;
    const int32_t nwin = has ? min((int32_t)IDENT_UNIT, g1 - w0) : 0;
    const bool act = lane < nwin;
    uint32_t pcv = CODE_NONE_POD, tolv = 0;
    if (act) {
      const int d = a.pod_digit[w0 + lane];
      pcv = (d >= 0 && d <= 9) ? (uint32_t)d : CODE_NONE_POD;
      tolv = a.pod_tol[w0 + lane] ? 1u : 0u;
    }
    const unsigned long long m = __ballot(act && pcv != CODE_NONE_POD);
    uint32_t res = NOFIT;
    if (m) {
      // the slice's pieces, one per compute tile it touches (word halves are tile-relative)
      for (int32_t c = c_lo; c < c_hi;) {
        const int32_t t0 = c / TILE_CHUNKS * TILE_CHUNKS;
        const int32_t hi = min(c_hi, t0 + TILE_CHUNKS);
        const uint32_t* wt = a.w0 + (size_t)c * WAVE;
        const __amdgpu_buffer_rsrc_t rst = __builtin_amdgcn_make_buffer_rsrc(
            (void*)wt, (short)0, (hi - c) * WAVE * (int32_t)sizeof(uint32_t), 0x00020000);
        uint32_t wa[R];
        load_words<true>(wa, wt, rst, 0, lane);
        const uint32_t rt = ident_unit8<R, false>(pcv, wa, wt, rst, nullptr, hi - c, lane);
        // pieces ascend in List order: the first piece with a match holds the slice's first
        if (res == NOFIT && rt != NOFIT) res = (uint32_t)(t0 / TILE_CHUNKS) * (uint32_t)TILE_NODES + rt;
        c = hi;
      }
      if (act && res != NOFIT) atomicMin(&slot[team][lane], res);
    }
    __syncthreads();
    if (k == 0 && has) {
      res = act ? slot[team][lane] : NOFIT;
      const unsigned long long mt = __ballot(act && tolv != 0u && pcv != CODE_NONE_POD);
      if (mt) res = ulist_pass(mt, pcv, res, a.ulist, (uint32_t)__builtin_amdgcn_readfirstlane((int)uvec), lane);
      if (act) {
        const int32_t j = w0 + lane;
        if (SHARD) {
          a.keys[j] = res != NOFIT ? shard_key(a.node_base, res) : 0;
        } else {
          const uint32_t ball = tolv ? (uint32_t)__builtin_amdgcn_readlane((int)bvec, 1)
                                     : (uint32_t)__builtin_amdgcn_readlane((int)bvec, 0);
          decode_ident(res != NOFIT ? (int64_t)res : -1, key_to_idx(ball), pcv != CODE_NONE_POD,
                       make_ident_decode(a.pp), &a.out_idx[j], &a.out_score[j], &a.out_status[j]);
        }
        slot[team][lane] = NOFIT;  // ready for the next round (ordered by the barrier below)
      }
    }
    __syncthreads();
  }
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
  decode_pod(idx_of(k0), idx_of(k1), idx_of(ka), d >= 0 && d <= 9, pp, &out_idx[j],
             &out_score[j], &out_status[j]);
}

// ---------------------------------------------------------------------------------------
// Sequential-commit kernel: ONE workgroup of NW waves walks the pods in order; node state
// lives in registers (chunk c is owned by wave c % NW, slot c / NW). Per pod: every wave
// scans its chunks -- first-match cost (v_sad_u32, as the compare/select-free IDENT form),
// first-feasible cost, and the non-match key when the normalize mode needs it --, reduces
// across lanes with DPP, and lane 0 folds the wave's result into the pod's LDS slot with LDS
// atomics (min / max; slots triple-buffered). After one barrier the pod's result is a single
// broadcast read, decoded and committed: count += 1 and, with a capacity, the owning lane
// retires a full node. The per-pod latency (scan + 1 reduction + 1 barrier + decode), not
// throughput, bounds it, so nothing else may wait on memory inside the loop:
//   * the barrier fences LDS only (a plain __syncthreads() is a workgroup fence over global
//     memory too: `s_waitcnt vmcnt(0)`, i.e. every pod would wait for the previous pod's stores);
//   * results collect in lanes (lane jl of wave 0 holds pod j0 + jl) and leave as one coalesced
//     store per 64 pods;
//   * the next 64 pods are prefetched one block ahead.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// CAP (max_pods_per_node > 0): a commit can make a node infeasible, so every wave reads each
// pod's result and the owning lane updates its registers before the next pod. Without a
// capacity a commit changes nothing the next pod reads: only wave 0 reads the result, decodes,
// keeps the output and adds the commit to a per-node count table held in LDS; the other waves
// go straight on to the next pod's scan (the barrier per pod still orders every commit before
// the next pod is decided).
// NW = scanning waves (chunk c is owned by wave c % NW). Without a capacity one more wave, the
// FINALIZER (wave NW), does no scanning: after each pod's barrier it reads the pod's result,
// decodes it, keeps the output and commits, while the scanners already scan the next pod.
template <int RS, int NW, bool NEED_KX, bool CAP>
__global__ __launch_bounds__((NW + (CAP ? 0 : 1)) * 64) void seq_kernel(SeqArgs a) {
  constexpr int FINW = CAP ? 0 : NW;  // the wave that decodes, keeps the output and commits
  // per-pod exchange slots, triple-buffered: [slot][first-match cost, first-feasible cost,
  // non-match key]
  __shared__ uint32_t xs[3][3];
  extern __shared__ int32_t lcnt[];  // !CAP: [n_chunks * 64] per-node pod counts
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool scanner = CAP || wv < NW;

  uint32_t D[RS], C0[RS], C1[RS];
  int32_t CNT[RS];
#pragma unroll
  for (int r = 0; r < RS; ++r) {
    const int32_t c = wv + NW * r;
    D[r] = DIGIT_NONE << 24;
    C0[r] = NOFIT;
    C1[r] = NOFIT;
    CNT[r] = 0;
    if (scanner && c < a.n_chunks) {
      const int32_t i = c * WAVE + lane;
      D[r] = (uint32_t)a.dig[i] << 24;
      C0[r] = a.c0[i];
      C1[r] = i < a.n_nodes ? (uint32_t)i : NOFIT;
      if (CAP) {
        CNT[r] = a.counts[i];
        if (CNT[r] >= a.max_pods) {
          C0[r] = NOFIT;
          C1[r] = NOFIT;
        }
      }
    }
  }
  if (!CAP) {  // ordered before the finalizer's first commit by the first pod's barrier
    for (int32_t i = threadIdx.x; i < a.n_chunks * WAVE; i += blockDim.x) lcnt[i] = a.counts[i];
  }
  if (threadIdx.x < 9) xs[threadIdx.x / 3][threadIdx.x % 3] = (threadIdx.x % 3 == 2) ? 0u : 0xFFFFFFFFu;
  __syncthreads();  // the slots' identities before any wave's first fold
  int sl = 0;

  // Drain the node-state loads here: otherwise the waitcnt pass, unsure they have landed on the
  // loop's class-0 path, waits for every outstanding load (the pod prefetch included) there.
  __builtin_amdgcn_s_waitcnt(0);
  // Pods in lanes, 64 at a time: raw bytes are loaded one block ahead (clamped index, so the
  // load needs no branch) and converted only when their block starts, so the loop never waits
  // on them.
  auto load_raw = [&](int32_t j0, int32_t& dr, int32_t& tr) {
    const int32_t jj = min(j0 + lane, a.n_pods - 1);
    dr = a.pod_digit[jj];
    tr = a.pod_tol[jj];
  };
  auto convert = [&](int32_t j0, int32_t dr, int32_t tr, uint32_t& pdl, uint32_t& tll) {
    const bool ok = j0 + lane < a.n_pods;
    pdl = (ok && dr >= 0 && dr <= 9) ? (uint32_t)dr : POD_DIGIT_NONE;
    tll = (ok && tr != 0) ? 1u : 0u;
  };
  // Loop-invariant arguments pinned in SGPRs: otherwise the backend re-loads them from the
  // kernel-argument segment inside the per-pod loop, and each reload's lgkmcnt wait lands in
  // front of the LDS exchange.
  PluginParams pp = a.pp;
  asm volatile("" : "+s"(pp.has_nu_filter), "+s"(pp.has_nn_score), "+s"(pp.nn_prescore), "+s"(pp.mode),
               "+s"(pp.weight));
  int32_t max_pods = a.max_pods;
  asm volatile("" : "+s"(max_pods));
  const IdentDecode idec = make_ident_decode(pp);
  uint32_t pdv = POD_DIGIT_NONE, tolv = 0;
  int32_t dn = 0, tn = 0;
  if (a.n_pods > 0) load_raw(0, dn, tn);
  int32_t o_idx = -1, o_st = 0;  // wave FINW: lane jl holds pod j0 + jl of the current block
  int64_t o_sc = 0;
  auto store_block = [&](int32_t j0, int32_t cnt) {  // wave FINW: one coalesced store per array
    if (lane < cnt) {
      a.out_idx[j0 + lane] = o_idx;
      a.out_score[j0 + lane] = o_sc;
      a.out_status[j0 + lane] = o_st;
    }
  };
#ifdef MSH_STAMPS  // diagnostic build only: per-wave cycles spent in each phase of the pod loop
  uint64_t ph[6] = {0, 0, 0, 0, 0, 0};
  uint64_t t_prev = __builtin_amdgcn_s_memtime();
#define SEQ_PH(k)                                        \
  do {                                                   \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();    \
    ph[k] += t_ - t_prev;                                \
    t_prev = t_;                                         \
  } while (0)
#else
#define SEQ_PH(k) \
  do {            \
  } while (0)
#endif
  for (int32_t j = 0; j < a.n_pods; ++j) {
    const int jl = j & (WAVE - 1);
    SEQ_PH(5);
    if (jl == 0) {
      // order matters for vmcnt (in-order): the conversion waits only for the loads issued one
      // block ago, then the previous block's results leave, then the next block is requested
      convert(j, dn, tn, pdv, tolv);
      if (wv == FINW && j > 0) store_block(j - WAVE, WAVE);
      load_raw(j + WAVE, dn, tn);  // one block ahead (clamped: no branch around it)
    }
    const uint32_t pd = (uint32_t)__builtin_amdgcn_readlane((int)pdv, jl);
    const uint32_t tol = (uint32_t)__builtin_amdgcn_readlane((int)tolv, jl);
    const uint32_t pds = pd << 24;
    // two independent min chains per cost (even / odd registers): half the dependent depth
    uint32_t bm = 0xFFFFFFFFu, ba = 0xFFFFFFFFu, bx = 0u;
    if (scanner) {
      uint32_t bm1 = 0xFFFFFFFFu, ba1 = 0xFFFFFFFFu;
      if (tol) {
#pragma unroll
        for (int r = 0; r < RS; ++r) {
          if (r & 1) {
            bm1 = umin(bm1, sad(D[r], pds, C1[r]));
            ba1 = umin(ba1, C1[r]);
          } else {
            bm = umin(bm, sad(D[r], pds, C1[r]));
            ba = umin(ba, C1[r]);
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < RS; ++r) {
          if (r & 1) {
            bm1 = umin(bm1, sad(D[r], pds, C0[r]));
            ba1 = umin(ba1, C0[r]);
          } else {
            bm = umin(bm, sad(D[r], pds, C0[r]));
            ba = umin(ba, C0[r]);
          }
        }
      }
      bm = umin(bm, bm1);
      ba = umin(ba, ba1);
    }
    if (NEED_KX && scanner) {
#pragma unroll
      for (int r = 0; r < RS; ++r) {
        const uint32_t cst = tol ? C1[r] : C0[r];
        const uint32_t k = cst < MATCH_LIMIT ? KMAX - cst : 0u;
        bx = umax(bx, D[r] == pds ? 0u : k);
      }
    }
    SEQ_PH(0);
    // Cross-wave exchange: lane 0 of every wave folds its wave's result into this pod's slot with
    // LDS atomics (min of the two costs, max of the non-match key), so after the barrier the pod's
    // result is ONE broadcast read: no second reduction on the critical path.
    uint32_t wm = 0xFFFFFFFFu, wa = 0xFFFFFFFFu, wx = 0u;
    if (scanner) {
      wm = wave_min_u32(bm);
      wa = wave_min_u32(ba);
      wx = NEED_KX ? wave_max_u32(bx) : 0u;
    }
    SEQ_PH(1);
    if (scanner && lane == 0) {
      atomicMin(&xs[sl][0], wm);
      atomicMin(&xs[sl][1], wa);
      if (NEED_KX) atomicMax(&xs[sl][2], wx);
    }
    lds_barrier();
    SEQ_PH(2);
    const int sl_now = sl;
    sl = sl == 2 ? 0 : sl + 1;
    if (!CAP && wv != FINW) continue;  // without a capacity only the finalizer finishes a pod
    const uint32_t gm = xs[sl_now][0], ga = xs[sl_now][1];
    const uint32_t gx = NEED_KX ? xs[sl_now][2] : 0u;
    // the slot read one pod ago is free now (every reader passed this pod's barrier) and is next
    // folded into two pods ahead (after the next barrier): wave FINW resets it in between
    if (wv == FINW && lane == 0) {
      const int sr = sl_now == 0 ? 2 : sl_now - 1;
      xs[sr][0] = 0xFFFFFFFFu;
      xs[sr][1] = 0xFFFFFFFFu;
      xs[sr][2] = 0u;
    }
    const int64_t im = gm < MATCH_LIMIT ? (int64_t)gm : -1;  // costs: node index, or >= 2^24 = none
    const int64_t ia = ga < MATCH_LIMIT ? (int64_t)ga : -1;
    const int64_t ix = NEED_KX ? key_to_idx(gx) : -1;
    int32_t sel, st;
    int64_t sc;
    SEQ_PH(3);
    if (NEED_KX)
      decode_pod(im, ix, ia, pd != POD_DIGIT_NONE, pp, &sel, &sc, &st);
    else
      decode_ident(im, ia, pd != POD_DIGIT_NONE, idec, &sel, &sc, &st);
    if (wv == FINW) {
      const bool mine = lane == jl;
      o_idx = mine ? sel : o_idx;
      o_sc = mine ? sc : o_sc;
      o_st = mine ? st : o_st;
    }
    if (st == 0) {  // commit (NodeInfo.AddPod analogue)
      if (!CAP) {
        if (lane == 0) atomicAdd(&lcnt[sel], 1);  // the finalizer; no return value waited for
      } else {
        const int32_t c = sel >> 6;
        if ((c % NW) == wv) {
          // the owning lane: the register by a wave-uniform index (scalar branches), the lane
          // by a compare (an unrolled `if (r == rs && mine)` became RS exec-mask branches)
          const int rs = __builtin_amdgcn_readfirstlane(c / NW);
          const bool mine = lane == (sel & (WAVE - 1));
#pragma unroll
          for (int r = 0; r < RS; ++r) {
            if (r == rs) {  // wave-uniform: a scalar branch to the one register, 4 VALU there
              CNT[r] += mine ? 1 : 0;
              const bool full = mine && CNT[r] >= max_pods;
              C0[r] = full ? NOFIT : C0[r];
              C1[r] = full ? NOFIT : C1[r];
            }
          }
        }
      }
    }
  }

  if (wv == FINW && a.n_pods > 0) {
    const int32_t j0 = (a.n_pods - 1) & ~(WAVE - 1);
    store_block(j0, a.n_pods - j0);
  }
#ifdef MSH_STAMPS
  if (lane == 0 && wv < 16) {
    for (int k = 0; k < 6; ++k) msh_stamp_buf[wv * 8 + k] = ph[k];
    msh_stamp_buf[wv * 8 + 6] = (unsigned long long)a.n_pods;
  }
#endif
#undef SEQ_PH
  if (CAP) {
#pragma unroll
    for (int r = 0; r < RS; ++r) {
      const int32_t c = wv + NW * r;
      if (c < a.n_chunks) a.counts[c * WAVE + lane] = CNT[r];
    }
  } else {
    __syncthreads();
    for (int32_t i = threadIdx.x; i < a.n_chunks * WAVE; i += blockDim.x) a.counts[i] = lcnt[i];
  }
}

// ---------------------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------------------
// Before every prep: reset the per-launch scalars (first feasible per class, ulist count), fill
// ulist with the never-matching entry (CODE_NONE_NODE << 24: the batch kernels read whole
// ULIST_STEP-entry blocks with no bounds check; count <= n <= n_pad, and n_pad is a multiple of
// ULIST_STEP), and apply pending msh_patch_nodes entries (idx | unsched << 32 | digit << 40).
// One launch instead of three memsets and a scatter kernel.
__global__ __launch_bounds__(256) void prep_reset_kernel(uint32_t* __restrict__ ball, uint32_t* __restrict__ ucount,
                                                         uint32_t* __restrict__ ulist, int32_t n_pad,
                                                         const unsigned long long* __restrict__ entries,
                                                         int32_t count, uint8_t* __restrict__ unsched,
                                                         int8_t* __restrict__ digit) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_pad) ulist[i] = CODE_NONE_NODE << 24;
  if (i < 2) ball[i] = 0;
  if (i == 0) *ucount = 0;
  if (i < count) {
    const unsigned long long e = entries[i];
    const uint32_t k = (uint32_t)e;
    unsched[k] = (uint8_t)(e >> 32);
    digit[k] = (int8_t)(uint8_t)(e >> 40);
  }
}

hipError_t launch_node_prep(const uint8_t* d_unsched, const int8_t* d_digit, int32_t n,
                            int32_t n_pad, int32_t has_nu, uint32_t* d_c0, uint8_t* d_dig,
                            uint32_t* d_w0, uint32_t* d_ulist, uint32_t* d_ucount,
                            unsigned long long* d_mask, uint32_t* d_ball, uint32_t* d_planes,
                            hipStream_t s, const unsigned long long* d_patch, int32_t patch_count) {
  const int32_t span = n_pad > patch_count ? n_pad : patch_count;
  hipLaunchKernelGGL(prep_reset_kernel, dim3((span > 0 ? span + 255 : 256) / 256), dim3(256), 0, s, d_ball,
                     d_ucount, d_ulist, n_pad, d_patch, patch_count, const_cast<uint8_t*>(d_unsched),
                     const_cast<int8_t*>(d_digit));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (n_pad == 0) return hipSuccess;
  const int blocks = (n_pad + PREP_THREADS - 1) / PREP_THREADS;
  hipLaunchKernelGGL(node_prep_kernel, dim3(blocks), dim3(PREP_THREADS), 0, s, d_unsched, d_digit, n, n_pad,
                     has_nu, d_c0, d_dig, d_w0, d_ulist, d_ucount, d_mask, d_ball, d_planes);
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
// Occupancy is a pure function of (kernel, block size, LDS bytes): query once per triple.
// The query costs microseconds of host time, which would otherwise sit between the caller's
// start event and the kernel on every launch.
int cached_occupancy(const void* kern, int threads, size_t lds) {
  struct Entry { const void* k; int t; size_t l; int occ; };
  static Entry cache[32];
  static int n = 0;
  for (int i = 0; i < n; ++i)
    if (cache[i].k == kern && cache[i].t == threads && cache[i].l == lds) return cache[i].occ;
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return -1;
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, threads, lds) != hipSuccess) return -1;
  if (n < 32) cache[n++] = Entry{kern, threads, lds, occ};
  return occ;
}

constexpr int BATCH_R = 8;
constexpr int BATCH_G = 32;
constexpr size_t LDS_BYTES_PER_NODE = sizeof(uint32_t) + sizeof(uint8_t);
constexpr size_t BATCH_LDS_MAX = 80 * 1024;  // 2 workgroups per CU at the largest tile

template <bool NEED_KX, bool SHARD>
hipError_t launch_batch_t(const BatchArgs& a, const DeviceInfo& dev, hipStream_t s,
                          std::string* err) {
  auto kern = batch_kernel<BATCH_R, BATCH_G, NEED_KX, SHARD>;
  const int32_t tile_chunks = batch_tile_chunks(a.n_chunks);
  if (tile_chunks < a.n_chunks && a.partial == nullptr) {
    if (err) *err = "batch kernel: multi-tile node table needs partial-key scratch";
    return hipErrorInvalidValue;
  }
  const size_t lds = (size_t)tile_chunks * WAVE * LDS_BYTES_PER_NODE;
  const int occ = cached_occupancy(reinterpret_cast<const void*>(kern), BATCH_THREADS, lds);
  if (occ < 1) {
    if (err) *err = "batch kernel: zero occupancy";
    return hipErrorInvalidConfiguration;
  }
  // Grid: enough waves for ~one pod group each, capped at what is resident at once, and a
  // whole number of workgroups per CU when it exceeds one round (balanced CU load).
  const int64_t waves_wanted = ((int64_t)a.n_pods + BATCH_G - 1) / BATCH_G;
  int64_t grid = (waves_wanted + 3) / 4;
  const int64_t cap = (int64_t)dev.cus * occ;
  if (const char* env = getenv("MSH_BATCH_WG_PER_CU")) {
    const int k = atoi(env);
    if (k > 0) grid = (int64_t)dev.cus * (k < occ ? k : occ);
  } else if (grid > cap) {
    grid = cap;
  } else if (grid > dev.cus) {
    grid = ((grid + dev.cus - 1) / dev.cus) * dev.cus;
    if (grid > cap) grid = cap;
  }
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(BATCH_THREADS), lds, s, a, tile_chunks);
  return hipGetLastError();
}

int32_t ident_stage_chunks(int32_t n_chunks, bool direct);

constexpr int IDENT_R = 8;
constexpr int IDENT_G2 = 8;   // pod pairs per group
constexpr size_t IDENT_LDS_BYTES_PER_NODE = sizeof(uint32_t);

int32_t ident_stage_chunks(int32_t n_chunks, bool direct) {
  // DIRECT: one compute tile per pass; LDS: whole table if it fits a stage, else stages
  const int32_t cap = direct ? TILE_CHUNKS : STAGE_CHUNKS;
  return n_chunks <= cap ? n_chunks : cap;
}

template <bool SHARD, bool DIRECT>
hipError_t launch_ident_t(const BatchArgs& a, const DeviceInfo& dev, hipStream_t s,
                          std::string* err) {
  auto kern = ident_kernel<IDENT_R, IDENT_G2, SHARD, DIRECT>;
  const int32_t lds_chunks = ident_stage_chunks(a.n_chunks, DIRECT);
  if (lds_chunks < a.n_chunks && a.partial == nullptr) {
    if (err) *err = "ident kernel: multi-stage node table needs partial scratch";
    return hipErrorInvalidValue;
  }
  const size_t lds = DIRECT ? 0 : (size_t)lds_chunks * WAVE * IDENT_LDS_BYTES_PER_NODE;
  const int occ = cached_occupancy(reinterpret_cast<const void*>(kern), IDENT_THREADS, lds);
  if (occ < 1) {
    if (err) *err = "ident kernel: zero occupancy";
    return hipErrorInvalidConfiguration;
  }
  constexpr int WPG = IDENT_THREADS / WAVE;
  // ~two full groups of G2 pod pairs per wave: enough pods per wave to amortise the per-group
  // costs, enough waves (>= 4 per SIMD at C3) to keep the VALU fed
  const int64_t waves_wanted = ((int64_t)a.n_pods + 4 * IDENT_G2 - 1) / (4 * IDENT_G2);
  int64_t grid = (waves_wanted + WPG - 1) / WPG;
  const int64_t cap = (int64_t)dev.cus * occ;
  if (const char* env = getenv("MSH_BATCH_WG_PER_CU")) {
    const int k = atoi(env);
    if (k > 0) grid = (int64_t)dev.cus * (k < occ ? k : occ);
  } else if (grid > cap) {
    grid = cap;
  } else if (grid > dev.cus) {
    grid = ((grid + dev.cus - 1) / dev.cus) * dev.cus;
    if (grid > cap) grid = cap;
  }
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(IDENT_THREADS), lds, s, a, lds_chunks);
  return hipGetLastError();
}
template <bool SHARD, int NT, bool LDSW, bool MULTI = false>
hipError_t launch_ident_dyn_nt(const BatchArgs& a, const DeviceInfo& dev, hipStream_t s, std::string* err) {
  auto kern = ident_dyn_kernel<IDENT_R, SHARD, NT, LDSW, MULTI>;
  // LDSW: a fixed per-launch LDS size class (occupancy is cached per size)
  const size_t lds = LDSW ? (size_t)DYN_LDS_CHUNKS * WAVE * sizeof(uint32_t) : 0;
  const int occ = cached_occupancy(reinterpret_cast<const void*>(kern), NT, lds);
  if (occ < 1) {
    if (err) *err = "ident work-queue kernel: zero occupancy";
    return hipErrorInvalidConfiguration;
  }
  // 32 waves per CU (8 per SIMD) measured ~3% faster than 16 at C3; fewer workgroups when the
  // batch is too small to give every wave a unit
  constexpr int WPG = NT / WAVE;
  const int wg_per_cu = 32 / WPG;
  const int64_t n_units = ((int64_t)a.n_pods + IDENT_UNIT - 1) / IDENT_UNIT;
  int64_t grid = (int64_t)dev.cus * (occ < wg_per_cu ? occ : wg_per_cu);
  if (const char* env = getenv("MSH_BATCH_WG_PER_CU")) {
    const int k = atoi(env);
    if (k > 0) grid = (int64_t)dev.cus * (k < occ ? k : occ);
  }
  if (const char* env = getenv("MSH_BATCH_GRID")) {  // tuning / A-B only: explicit workgroup count
    const int k = atoi(env);
    if (k > 0) grid = k;
  }
  const int64_t grid_units = (n_units + WPG - 1) / WPG;
  if (grid > grid_units) grid = grid_units;
  if (grid < 1) grid = 1;
  BatchArgs ka = a;
  ka.unit_q = (int32_t)(n_units / grid);
  ka.unit_r = (int32_t)(n_units % grid);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), lds, s, ka);
  return hipGetLastError();
}

template <bool SHARD, int SPLIT>
hipError_t launch_ident_split_t(const BatchArgs& a, const DeviceInfo& dev, hipStream_t s, int32_t slice_chunks) {
  auto kern = ident_split_kernel<IDENT_R, SHARD, SPLIT>;
  const int occ = cached_occupancy(reinterpret_cast<const void*>(kern), DYN_THREADS, 0);
  constexpr int TEAMS = DYN_THREADS / WAVE / SPLIT;
  const int64_t n_units = ((int64_t)a.n_pods + IDENT_UNIT - 1) / IDENT_UNIT;
  int64_t grid = (n_units + TEAMS - 1) / TEAMS;
  const int64_t cap = (int64_t)dev.cus * (occ < 2 ? (occ < 1 ? 1 : occ) : 2);
  if (grid > cap) grid = cap;
  if (grid < 1) grid = 1;
  BatchArgs ka = a;
  ka.unit_q = (int32_t)(n_units / grid);
  ka.unit_r = (int32_t)(n_units % grid);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(DYN_THREADS), 0, s, ka, slice_chunks);
  return hipGetLastError();
}

// Waves per unit for the node-split kernel: enough (unit, slice) pairs to put ~4096 waves to
// work, slices of at least 64 chunks (4096 nodes) so the per-unit reduction stays small next to
// the scan. 1 = the work-queue kernel (one wave per unit). MSH_SPLIT overrides (A/B).
int choose_split(int64_t n_pods, int32_t n_chunks, const DeviceInfo& dev) {
  if (const char* env = getenv("MSH_SPLIT")) return atoi(env);
  const int64_t n_units = (n_pods + IDENT_UNIT - 1) / IDENT_UNIT;
  const int64_t want = (int64_t)dev.cus * 16;
  int split = 1;
  while (split < 16 && n_units * split < want && n_chunks / (2 * split) >= 64) split *= 2;
  return split;
}

template <bool SHARD, int NP, int WT>
hipError_t launch_ident_wave_wt(const BatchArgs& a, int64_t waves, int32_t rounds, hipStream_t s) {
  constexpr int WPG = WT / WAVE;
  const int64_t pairs = ((int64_t)a.n_pods + 1) / 2;
  BatchArgs ka = a;  // pairs per wave: unit_q, and one more for the first unit_r wave ranks
  ka.unit_q = (int32_t)(pairs / waves);
  ka.unit_r = (int32_t)(pairs % waves);
  ka.unit_w = (int32_t)waves;
  const int64_t grid = (waves + WPG - 1) / WPG;
  // MSH_WAVE_XCD (A/B only): 1 = XCD-contiguous wave ranks (default), 0 = ranks interleaved
  // across workgroups
  const char* env = getenv("MSH_WAVE_XCD");
  const int32_t xcd = env ? (atoi(env) != 0) : 1;
  hipLaunchKernelGGL((ident_wave_kernel<IDENT_R, SHARD, NP, WT>), dim3((unsigned)grid), dim3(WT), 0, s, ka,
                     rounds, xcd);
  return hipGetLastError();
}

// Workgroup size of the wave-range kernel: small workgroups free their CU slot as soon as
// their own few waves end, so the next launch (another stream) fills the chip sooner.
// MSH_WAVE_THREADS (256 / 512 / 1024) is for A/B only.
template <bool SHARD, int NP>
hipError_t launch_ident_wave_np(const BatchArgs& a, int64_t waves, int32_t rounds, hipStream_t s) {
  const char* env = getenv("MSH_WAVE_THREADS");
  const int wt = env ? atoi(env) : 256;
  if (wt == 1024) return launch_ident_wave_wt<SHARD, NP, 1024>(a, waves, rounds, s);
  if (wt == 512) return launch_ident_wave_wt<SHARD, NP, 512>(a, waves, rounds, s);
  return launch_ident_wave_wt<SHARD, NP, 256>(a, waves, rounds, s);
}

// Waves for one contiguous pair range per wave: at most every wave of a full chip (8 per
// SIMD), fewer when there are fewer than 4 or 7 pairs per wave (below); 0 = the work queue
// takes over (a multi-tile table, or more than MSH_WAVE_MAX_ROUNDS rounds of 8 pairs per wave;
// default 64). MSH_WAVE_RANGE=0 disables it (A/B).
int64_t wave_range_waves(int64_t n_pods, int32_t n_chunks, const DeviceInfo& dev) {
  if (const char* env = getenv("MSH_WAVE_RANGE"))
    if (atoi(env) == 0) return 0;
  if (n_chunks > TILE_CHUNKS || n_pods <= 0) return 0;
  const char* env = getenv("MSH_WAVE_MAX_ROUNDS");
  const int64_t max_rounds = env ? atoi(env) : 64;
  const int64_t full = (int64_t)dev.cus * 32;
  const int64_t pairs = (n_pods + 1) / 2;
  if (pairs > 8 * max_rounds * full) return 0;
  // pairs per wave at least mp (MSH_WAVE_MIN_PAIRS, A/B only). Batches that fill the chip at 4
  // pairs per wave take 7: a wave's fixed costs (prologue, reduction, decode) and each node-word
  // load are shared by more pairs; at C3 that leaves 7,143 of 8,192 wave slots busy and measured
  // 1.5-2.7% faster pipelined than 6.1 pairs on all 8,192. Smaller batches take 4: shorter waves,
  // lower latency (16k pods: 5.6 vs 6.9 us). profiles/ab/wave_min_pairs.jsonl
  const char* menv = getenv("MSH_WAVE_MIN_PAIRS");
  const int64_t mp = menv ? std::max(1, atoi(menv)) : pairs < 4 * full ? 4 : 7;
  return std::min(full, (pairs + mp - 1) / mp);
}

template <bool SHARD>
hipError_t launch_ident_dyn_t(const BatchArgs& a, const DeviceInfo& dev, hipStream_t s,
                              std::string* err) {
  const int split = choose_split(a.n_pods, a.n_chunks, dev);
  if (split > 1) {
    const int sp = split >= 16 ? 16 : split >= 8 ? 8 : split >= 4 ? 4 : 2;
    const int32_t sc = ((a.n_chunks + sp - 1) / sp + 15) / 16 * 16;  // multiple of 2R chunks
    if (sp == 2) return launch_ident_split_t<SHARD, 2>(a, dev, s, sc);
    if (sp == 4) return launch_ident_split_t<SHARD, 4>(a, dev, s, sc);
    if (sp == 8) return launch_ident_split_t<SHARD, 8>(a, dev, s, sc);
    return launch_ident_split_t<SHARD, 16>(a, dev, s, sc);
  }
  if (const int64_t waves = wave_range_waves(a.n_pods, a.n_chunks, dev)) {
    const int64_t longest = (((int64_t)a.n_pods + 1) / 2 + waves - 1) / waves;  // in pairs
    const int32_t rounds = (int32_t)((longest + 7) / 8);
    switch ((longest + rounds - 1) / rounds) {  // the longest round, in pairs
      case 1: return launch_ident_wave_np<SHARD, 1>(a, waves, rounds, s);
      case 2: return launch_ident_wave_np<SHARD, 2>(a, waves, rounds, s);
      case 3: return launch_ident_wave_np<SHARD, 3>(a, waves, rounds, s);
      case 4: return launch_ident_wave_np<SHARD, 4>(a, waves, rounds, s);
      case 5: return launch_ident_wave_np<SHARD, 5>(a, waves, rounds, s);
      case 6: return launch_ident_wave_np<SHARD, 6>(a, waves, rounds, s);
      case 7: return launch_ident_wave_np<SHARD, 7>(a, waves, rounds, s);
      default: return launch_ident_wave_np<SHARD, 8>(a, waves, rounds, s);
    }
  }
  // MSH_DYN_THREADS (tuning / A-B only): workgroup size of the work-queue kernel
  const char* env = getenv("MSH_DYN_THREADS");
  const int nt = env ? atoi(env) : DYN_THREADS;
  // node words from an LDS copy when the table fits the size class (MSH_DYN_LDS=0: L1/L2 reads)
  const char* lenv = getenv("MSH_DYN_LDS");
  const bool ldsw = (lenv ? atoi(lenv) : MSH_DYN_LDS_DEFAULT) != 0 && a.n_chunks + IDENT_R <= DYN_LDS_CHUNKS;
  if (a.n_chunks > TILE_CHUNKS) return launch_ident_dyn_nt<SHARD, 1024, false, true>(a, dev, s, err);
  if (ldsw) return launch_ident_dyn_nt<SHARD, 1024, true>(a, dev, s, err);
  if (nt == 256) return launch_ident_dyn_nt<SHARD, 256, false>(a, dev, s, err);
  if (nt == 512) return launch_ident_dyn_nt<SHARD, 512, false>(a, dev, s, err);
  return launch_ident_dyn_nt<SHARD, 1024, false>(a, dev, s, err);
}
// Slice waves per 64-pod block of the bit-sliced kernel: enough waves for ~6 per SIMD, each
// slice at least two groups (512 nodes) so the per-wave fixed cost (pod bytes, the first-group
// re-read, the LDS merge) stays small next to the scan.
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
  hipLaunchKernelGGL((bits_kernel<S, KX, SHARD>), dim3((unsigned)blocks), dim3(S * WAVE), 0, s, ka);
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

int32_t batch_tile_chunks(int32_t n_chunks) {
  const int32_t max_tile = (int32_t)(BATCH_LDS_MAX / (LDS_BYTES_PER_NODE * WAVE)) / 16 * 16;
  return n_chunks <= max_tile ? n_chunks : max_tile;
}

bool batch_needs_partial(int32_t n_chunks) {
  return batch_tile_chunks(n_chunks) < n_chunks || ident_stage_chunks(n_chunks, false) < n_chunks;
}

// MSH_BATCH_KERNEL (tuning / A-B only): 3 = IDENT work queue (default), 2 = IDENT direct
// static, 0 = IDENT LDS-staged, 1 = compare/select kernel
int batch_kernel_choice() {
  const char* kenv = getenv("MSH_BATCH_KERNEL");
  return kenv ? atoi(kenv) : 3;
}

bool batch_uses_partial(const PluginParams& pp, int32_t n_chunks, const DeviceInfo& dev) {
  if (!dev.legacy_batch) return false;  // the bit-sliced kernel keeps no running results
  const int kv = batch_kernel_choice();
  if (!needs_kx(pp) && kv == 3) return false;  // the work queue scans every tile per unit
  if (!needs_kx(pp) && kv != 1) return ident_stage_chunks(n_chunks, kv != 0) < n_chunks;
  return batch_tile_chunks(n_chunks) < n_chunks;
}

hipError_t launch_batch(const BatchArgs& a, bool shard, const DeviceInfo& dev, hipStream_t s,
                        std::string* err) {
  if (a.n_pods == 0) return hipSuccess;
  const bool kx = needs_kx(a.pp);
  if (!dev.legacy_batch) {
    if (shard) return kx ? launch_bits_t<true, true>(a, dev, s) : launch_bits_t<false, true>(a, dev, s);
    return kx ? launch_bits_t<true, false>(a, dev, s) : launch_bits_t<false, false>(a, dev, s);
  }
  const int kv = batch_kernel_choice();
  if (!kx && kv == 3)
    return shard ? launch_ident_dyn_t<true>(a, dev, s, err) : launch_ident_dyn_t<false>(a, dev, s, err);
  if (!kx && kv != 1) {
    if (kv == 0)
      return shard ? launch_ident_t<true, false>(a, dev, s, err) : launch_ident_t<false, false>(a, dev, s, err);
    return shard ? launch_ident_t<true, true>(a, dev, s, err) : launch_ident_t<false, true>(a, dev, s, err);
  }
  if (shard) return kx ? launch_batch_t<true, true>(a, dev, s, err) : launch_batch_t<false, true>(a, dev, s, err);
  return kx ? launch_batch_t<true, false>(a, dev, s, err) : launch_batch_t<false, false>(a, dev, s, err);
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
template <int RS, int NW, bool CAP>
hipError_t launch_seq_rs(const SeqArgs& a, hipStream_t s) {
  const dim3 blk((NW + (CAP ? 0 : 1)) * 64);  // + the finalizer wave without a capacity
  const size_t lds = CAP ? 0 : (size_t)a.n_chunks * WAVE * sizeof(int32_t);  // !CAP count table
  if (needs_kx(a.pp)) hipLaunchKernelGGL((seq_kernel<RS, NW, true, CAP>), dim3(1), blk, lds, s, a);
  else hipLaunchKernelGGL((seq_kernel<RS, NW, false, CAP>), dim3(1), blk, lds, s, a);
  return hipGetLastError();
}

// Register-resident node state: RS chunks per lane. Spill-free on gfx950 up to RS = 24 at
// 4 waves, 16 at 8 waves, 12 at 16 waves, 16 at 15 scanners + the finalizer (checked with
// -Rpass-analysis=kernel-resource-usage).
template <int NW, int RS_MAX, bool CAP>
hipError_t launch_seq_nw(const SeqArgs& a, hipStream_t s) {
  const int rs = (a.n_chunks + NW - 1) / NW;
  if (rs <= 1) return launch_seq_rs<1, NW, CAP>(a, s);
  if (rs <= 2) return launch_seq_rs<2, NW, CAP>(a, s);
  if (rs <= 3) return launch_seq_rs<3, NW, CAP>(a, s);
  if (rs <= 4) return launch_seq_rs<4, NW, CAP>(a, s);
  if (rs <= 6) return launch_seq_rs<6, NW, CAP>(a, s);
  if (rs <= 8) return launch_seq_rs<8, NW, CAP>(a, s);
  if (rs <= 12 || RS_MAX <= 12) return launch_seq_rs<12, NW, CAP>(a, s);
  if (rs <= 16 || RS_MAX <= 16) return launch_seq_rs<(RS_MAX < 16 ? RS_MAX : 16), NW, CAP>(a, s);
  return launch_seq_rs<(RS_MAX < 24 ? RS_MAX : 24), NW, CAP>(a, s);
}
}  // namespace

hipError_t launch_sequential(const SeqArgs& a, hipStream_t s, std::string* err) {
  if (a.n_pods == 0) return hipSuccess;
  // Scanning waves: MSH_SEQ_WAVES (4, 8 or 16) for tuning; default 8 with a capacity, 4 without
  // (scripts/sweep_seq.py at 5k nodes: 4 scanners + the finalizer 0.35 us per pod, 8 + 1 0.38),
  // raised until the table fits the registers. Without a capacity a finalizer wave comes on
  // top (16 -> 15 scanners + 1: the 1024-thread workgroup limit).
  const char* env = getenv("MSH_SEQ_WAVES");
  int nw = env ? atoi(env) : (a.max_pods > 0 ? 8 : 4);
  if (nw == 4 && a.n_chunks > 4 * 24) nw = 8;
  if (nw == 8 && a.n_chunks > 8 * 16) nw = 16;
  if (nw != 4 && nw != 8) nw = 16;
  if (a.n_chunks > 16 * 12) {
    if (err) *err = "sequential mode supports at most 12288 nodes per device";
    return hipErrorInvalidValue;
  }
  if (a.max_pods > 0) {
    if (nw == 4) return launch_seq_nw<4, 24, true>(a, s);
    if (nw == 8) return launch_seq_nw<8, 16, true>(a, s);
    return launch_seq_nw<16, 12, true>(a, s);
  }
  if (nw == 4) return launch_seq_nw<4, 24, false>(a, s);
  if (nw == 8) return launch_seq_nw<8, 16, false>(a, s);
  return launch_seq_nw<15, 16, false>(a, s);
}

}  // namespace msh

#ifdef MSH_STAMPS
extern "C" int msh_debug_read_stamps(unsigned long long* out, int n_waves) {
  if (n_waves > msh::STAMP_WAVES) n_waves = msh::STAMP_WAVES;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(msh::msh_stamp_buf),
                                  sizeof(unsigned long long) * 2 * msh::STAMPS_PER_WAVE * n_waves, 0,
                                  hipMemcpyDeviceToHost);
}
extern "C" int msh_debug_clear_stamps(void) {
  static unsigned long long zero[msh::STAMP_WAVES * msh::STAMPS_PER_WAVE * 2];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(msh::msh_stamp_buf), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
}
#endif
