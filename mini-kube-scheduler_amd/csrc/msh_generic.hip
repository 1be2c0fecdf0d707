// msh_generic.hip — the generic score pipeline (gfx950): any score plugin list (NodeNumber and up to four
// score-column plugins, MSH_PLUGIN_SCORE_COLUMN0..3) with the int64 total of EVERY (pod, node) pair
// computed explicitly — the general form of RunFilterPlugins + RunScorePlugins + selectHost
// (minisched/minisched.go:115-199, 304-325) and north_star's five stages one to one.
//
// "Lanes = pods": lane l of a wave holds one pod of each of its two 64-pod blocks. The node table is
// streamed through LDS in tiles shared by the workgroup's waves (stage 5): per node a record {code, xm}
// (the NodeNumber code — suffix digit, or 10 — and xm = all-ones when NodeUnschedulable rejects the node
// for pods that do not tolerate the taint), the node-only sum of the columns without a normalizer, and
// 100 x raw as an exact double per normalizing column; the waves read them as wave-uniform ds_read_b128
// broadcasts into VGPRs. Per pair, everything is VGPR-only vector work:
//   1. feasibility: NodeUnschedulable's verdict, infeasible = xm & ~tolerates, clears the pair's key
//      (one v_bitop3): an infeasible pair never becomes a pod's maximum;
//   3. extents (max, min) of every normalizing plugin's raw score over the pod's feasible nodes, only
//      when some plugin normalizes. The filter list is [NodeUnschedulable] or empty, so a pod's feasible
//      nodes are those of its tolerates class (all nodes, or the schedulable ones): the workgroup reduces
//      the table once per class (a strided pass, wave shuffles, an LDS reduction over the waves) and each
//      pod takes its class's extents — NodeNumber's from the codes present in the class;
//   2. the total of each pair: Σ weight x NormalizeScore(raw) in Go int64 arithmetic. NodeNumber is one
//      compare + select between the pod's two weighted values; a normalizing column is
//      q = (100 raw - b) x r with the pod's exact reciprocal r, truncated; the
//      columns without a normalizer are the staged node-only sum;
//   4. selectHost: the total as a key (total + 2^31 or total ^ 2^63 unsigned, 0 = infeasible; or the
//      total itself as a double, NaN = infeasible), a running v_max per lane, and per 16-node chunk the
//      chunk where the maximum last rose; after the scan the winner's chunk is re-evaluated for the first
//      node with that key (the first maximum in List order: strict '>' as selectHost's scan,
//      minisched.go:311-315).
// Key type KT: 0, 32-bit totals, when the host has bounded every feasible pair's |total| below 2^31 - 1
// from the weights, the modes and the uploaded columns' range; 2, doubles, when below 2^53 (every term
// and partial sum is an integer a double holds exactly); else 1, 64-bit (Go's wrapping int64).
// MODE 0: the whole batch (status, node, score per pod). Node-sharded mode (msh_generic_*): MODE 1 writes
// each pod's extents over this shard's nodes (ext, mins negated: one all-reduce MAX merges them), MODE 2
// takes the merged extents and writes each pod's best (total, global node index) over the shard.
#include "msh_device.h"

namespace msh {

constexpr int GEN_W = 8;       // waves per workgroup
constexpr int GEN_BPW = 2;     // 64-pod blocks per wave: one LDS read of a node serves both
constexpr int GEN_CHUNK = 16;  // nodes per first-maximum chunk
constexpr uint32_t GEN_CODE_NONE = 10u;  // a node name without a suffix digit (matches no pod's code)
constexpr double GEN_RCP_BIAS = 1.0 + 0x1p-49;
// two nodes' staged values per LDS read: ds_read_b128 moves 16 B per lane in 4 LDS cycles, where the
// ds_read2_b64 the compiler forms from two 8-B reads takes 8 (MI355X_MICROARCH.md §LDS)
typedef uint32_t gen_u4 __attribute__((ext_vector_type(4)));
typedef double gen_d2 __attribute__((ext_vector_type(2)));
constexpr uint32_t GEN_NONE = 0xFFFFFFFFu;

// NormalizeScore of one raw score given the pod's extent of that plugin over its feasible nodes
// (mx, mn): upstream helper.DefaultNormalizeScore(MaxNodeScore = 100, reverse) — maxCount starts at 0,
// an all-zero list is left alone (reverse: all 100) — or min-max (0 when max == min).
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

// v_max_f64 as the instruction (fmax adds a NaN canonicalisation per operand): IEEE mode,
// a quiet NaN operand yields the other one
__device__ __forceinline__ double vmax_f64(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// v with its high dword ORed with m: m all-ones turns it into a quiet NaN (exponent and quiet bit set)
__device__ __forceinline__ double nan_if(double v, uint32_t x, uint32_t nt) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t hi = bop3_or_and((uint32_t)(b >> 32), x, nt);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | (uint32_t)b);
}

// Per-pair key of the main pass (KT): uint32_t (32-bit totals, biased by 2^31) or uint64_t (biased by
// 2^63), 0 = infeasible; or double (the total, |total| < 2^53), NaN = infeasible (v_max_f64 skips it).
template <int KT>
using GKey = typename std::conditional<KT == 0, uint32_t,
                                       typename std::conditional<KT == 1, uint64_t, double>::type>::type;

template <int KT>
__device__ __forceinline__ GKey<KT> key_mask(GKey<KT> t, uint32_t xm, uint32_t nt) {
  if constexpr (KT == 2) {
    return nan_if(t, xm, nt);
  } else if constexpr (KT == 1) {
    const uint32_t lo = bop3_andn_of_and((uint32_t)t, xm, nt), hi = bop3_andn_of_and((uint32_t)(t >> 32), xm, nt);
    return ((uint64_t)hi << 32) | lo;
  } else {
    return bop3_andn_of_and(t, xm, nt);
  }
}

// One lane's scoring state of one 64-pod block (main pass): NodeNumber's weighted normalized value on a
// digit match / otherwise, biased (the score columns' part is the node's class term, staged per tile).
template <int KT>
struct GLane {
  GKey<KT> k1, k0;
};

// The contribution of normalizing column c to a pair's total: w x trunc((v - b) x r), v = 100 x raw.
template <int KT, bool SUB>
__device__ __forceinline__ GKey<KT> col_term(double v, double b, double r, GKey<KT> cw) {
  const double q = (SUB ? v - b : v) * r;
  if constexpr (KT == 2) {
    // |trunc(q) x w| is within the host's 2^53 bound on a feasible pair: exact (the others are masked)
    return __builtin_trunc(q) * cw;
  } else if constexpr (KT == 1) {
    // |q| < 2^40 on a feasible pair; an infeasible pair's value is clamped, converted and masked out
    const int64_t n = (int64_t)__builtin_fmin(__builtin_fmax(q, -0x1p62), 0x1p62);
    return (uint64_t)n * cw;
  } else {
    // |n| and |w| below 2^23 on a feasible pair (the host's bound, GenericArgs::w64): the signed 24-bit
    // multiply (full rate, where v_mul_lo_u32 is quarter rate); v_cvt_i32_f64 saturates on the others.
    // That operand range is guaranteed ONLY by generic_args' c24 check (msh_capi.cpp): every normalizing
    // column's weight and normalized-score bound below 2^23, else the launch takes 64-bit keys. A new term
    // multiplied here must be added to that check.
    const int32_t n = (int32_t)q;
    return (uint32_t)__mul24(n, (int32_t)cw);
  }
}

template <int MODE, int KT, bool TS, int NNC, bool MMX>
__global__ __launch_bounds__(GEN_W * WAVE) void generic_kernel(GenericArgs a) {
  using Key = GKey<KT>;
  constexpr bool W64 = KT != 0;  // 8-byte keys
  // the node-only sum of the columns without a normalizer (exact in int64 for the double keys, whose
  // host bound keeps every term and the sum below 2^53)
  auto node_sum = [&](int32_t i) -> Key {
    if constexpr (KT == 2) {
      int64_t t = 0;
      for (int c = 0; c < a.nts; ++c) t += a.cols[(size_t)a.tcc[c] * a.col_stride + i] * a.tw[c];
      return (double)t;
    } else {
      Key t = 0;
      for (int c = 0; c < a.nts; ++c) t += (Key)a.cols[(size_t)a.tcc[c] * a.col_stride + i] * (Key)a.tw[c];
      return t;
    }
  };
  constexpr int NC = NNC > 0 ? NNC : 1;
  extern __shared__ uint4 s_dyn[];
  __shared__ uint32_t s_ffs;  // the first node NodeUnschedulable passes for every pod (GEN_NONE: none)
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int S = a.slices;           // waves per pod group (1, 2, 4, 8), each scanning a slice of every tile
  const int sl = wv % S, pg = wv / S;
  const int pgs = GEN_W / S;        // pod groups per workgroup
  const BatchDesc& d = a.d[blockIdx.y];
  const int32_t np = d.n_pods;
  const int32_t wg0 = (int32_t)blockIdx.x * pgs * GEN_BPW * WAVE;
  if (wg0 >= np) return;  // the whole workgroup lies past its batch's end
  const int32_t n = a.n_nodes, TN = a.tile;
  const int nnc = NNC == 4 ? a.nnc : NNC;  // normalizing columns (the general instance: a runtime count)
  // The score columns' part of a pair's total depends on the node and on the pod's tolerates class alone
  // (stage 3: the class fixes the extents, hence every normalized value): the CLASS TERM of node i for
  // class k, Σ over the columns of weight x NormalizeScore(raw), is staged with the node, once per class.
  constexpr bool CT = TS || NNC > 0;
  // staged terms per node: one per class with a normalizing column; without one the columns' part is the
  // node-only sum, the same for both classes: one
  constexpr int NCT = NNC > 0 ? 2 : (TS ? 1 : 0);
  // dynamic LDS: the tile (records, then [TN][NCT] class terms), then the slice-merge area
  uint2* s_cx = reinterpret_cast<uint2*>(s_dyn);
  Key* s_ct = reinterpret_cast<Key*>(s_cx + TN);
  char* s_merge = reinterpret_cast<char*>(s_ct + NCT * (size_t)TN);
  // per class (0: pods that do not tolerate the unschedulable taint, 1: pods that do) and normalizing
  // column: the reciprocal and the min-max offset of its NormalizeScore
  __shared__ double s_crr[2][NC], s_cbb[2][NC];
  if (threadIdx.x == 0) s_ffs = GEN_NONE;
  if (threadIdx.x < 2 * NC) {
    (&s_crr[0][0])[threadIdx.x] = 0.0;
    (&s_cbb[0][0])[threadIdx.x] = 0.0;
  }
  __syncthreads();

  // ---- the lane's pods ----
  uint32_t pcode[GEN_BPW], ntol[GEN_BPW];
  int32_t jj[GEN_BPW];
  bool pdok[GEN_BPW];
  const int32_t pbase = wg0 + pg * GEN_BPW * WAVE;
#pragma unroll
  for (int b = 0; b < GEN_BPW; ++b) {
    const int32_t j = pbase + b * WAVE + lane;
    jj[b] = j;
    int dq = -1, tq = 0;
    if (j < np) {
      dq = d.pod_digit[j];
      tq = d.pod_tol[j];
    }
    pdok[b] = dq >= 0 && dq <= 9;  // NodeNumber.PreScore: Atoi of the last byte
    pcode[b] = pdok[b] ? (uint32_t)dq : CODE_NONE_POD;
    ntol[b] = tq ? 0u : 0xFFFFFFFFu;
  }

  const int n_tiles = n > 0 ? (n + TN - 1) / TN : 0;
  // the wave's slice of a tile of tn nodes: [lo, hi)
  auto slice_of = [&](int32_t tn, int32_t& lo, int32_t& hi) {
    const int32_t L = (((tn + S - 1) / S) + GEN_CHUNK - 1) & ~(GEN_CHUNK - 1);
    lo = min(sl * L, tn);
    hi = min(lo + L, tn);
  };

  // ---- stage 3: extents over the feasible nodes (normalizing plugins only) ----
  int64_t emx[GEN_BPW][1 + NC], emn[GEN_BPW][1 + NC];  // [0] NodeNumber, [1 + c] normalizing column c
#pragma unroll
  for (int b = 0; b < GEN_BPW; ++b)
#pragma unroll
    for (int e = 0; e < 1 + NC; ++e) {
      emx[b][e] = INT64_MIN;
      emn[b][e] = INT64_MAX;
    }
  const bool nn_ext = a.nn_score && a.nn_mode != 0;
  bool staged = false;  // the main pass stages each tile (a single-tile table once)
  if (MODE != 2 && a.need_ext) {
    // A pod's feasible nodes are one of two sets: the filter list is [NodeUnschedulable] or empty, so they
    // are every node for a pod that tolerates the unschedulable taint and the schedulable ones for a pod
    // that does not. Every extent a pod needs is therefore its tolerates class's: the workgroup reduces
    // the (shard's) table once per class, in LDS, instead of each pod scanning every node:
    //  * each normalizing column's (max, min) raw score over the class's nodes;
    //  * NodeNumber: the codes present among the class's nodes (bit code, 10 = no digit); a pod of code d
    //    has a feasible match iff bit d is set, a feasible non-match iff any other bit is.
    __shared__ int64_t s_cext[GEN_W][2][2][GEN_COLS];  // [wave][class: 0 schedulable, 1 all][max, -min][column]
    __shared__ uint32_t s_cpres[GEN_W][2];
    int64_t cmx[2][NC], cmn[2][NC];
    uint32_t pres[2] = {0u, 0u};
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      cmx[0][c] = cmx[1][c] = INT64_MIN;
      cmn[0][c] = cmn[1][c] = INT64_MAX;
    }
    for (int32_t i = threadIdx.x; i < n; i += GEN_W * WAVE) {
      const int dg = a.digit[i];
      const bool sched = !(a.has_nu && a.unsched[i]);
      const uint32_t bit = 1u << ((dg >= 0 && dg <= 9) ? (uint32_t)dg : GEN_CODE_NONE);
      pres[1] |= bit;
      pres[0] |= sched ? bit : 0u;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if (c >= nnc) break;
        const int64_t v = a.cols[(size_t)a.ncc[c] * a.col_stride + i];
        cmx[1][c] = max(cmx[1][c], v);
        cmn[1][c] = min(cmn[1][c], v);
        if (sched) {
          cmx[0][c] = max(cmx[0][c], v);
          cmn[0][c] = min(cmn[0][c], v);
        }
      }
    }
    // the wave's, then the workgroup's
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        pres[k] |= (uint32_t)__shfl_xor((int)pres[k], off);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          if (c >= nnc) break;
          cmx[k][c] = max(cmx[k][c], (int64_t)__shfl_xor((long long)cmx[k][c], off));
          cmn[k][c] = min(cmn[k][c], (int64_t)__shfl_xor((long long)cmn[k][c], off));
        }
      }
    }
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        s_cpres[wv][k] = pres[k];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          if (c >= nnc) break;
          s_cext[wv][k][0][c] = cmx[k][c];
          s_cext[wv][k][1][c] = -cmn[k][c];  // negated: one max merges both (cmn <= INT64_MAX)
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      pres[k] = 0u;
#pragma unroll
      for (int c = 0; c < NC; ++c) cmx[k][c] = cmn[k][c] = INT64_MIN;  // cmn negated here
      for (int w = 0; w < GEN_W; ++w) {
        pres[k] |= s_cpres[w][k];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          if (c >= nnc) break;
          cmx[k][c] = max(cmx[k][c], s_cext[w][k][0][c]);
          cmn[k][c] = max(cmn[k][c], s_cext[w][k][1][c]);
        }
      }
    }
    // every pod takes its class's extents
#pragma unroll
    for (int b = 0; b < GEN_BPW; ++b) {
      const int k = ntol[b] ? 0 : 1;
      if (nn_ext) {  // NodeNumber's raw scores over the feasible nodes: 10 on a match, 0 otherwise
        const uint32_t pb = pcode[b] <= 9 ? 1u << pcode[b] : 0u;
        const bool fm = (pres[k] & pb) != 0, fnm = (pres[k] & ~pb) != 0;
        if (fm || fnm) {
          emx[b][0] = fm ? 10 : 0;
          emn[b][0] = fnm ? 0 : 10;
        }
      }
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if (c >= nnc) break;
        if (cmx[k][c] != INT64_MIN) {
          emx[b][1 + c] = cmx[k][c];
          emn[b][1 + c] = MMX ? -cmn[k][c] : INT64_MAX;
        }
      }
    }
    if constexpr (MODE == 1) {  // node-sharded: this shard's extents, mins negated (one MAX merges both)
      if (sl == 0) {
        const int ne = 1 + a.ncol;
#pragma unroll
        for (int b = 0; b < GEN_BPW; ++b) {
          const int32_t j = jj[b];
          if (j >= np) continue;
          for (int e = 0; e < ne; ++e) {  // list positions without a normalizer: no extent
            a.ext[(size_t)(2 * e) * np + j] = INT64_MIN;
            a.ext[(size_t)(2 * e + 1) * np + j] = -INT64_MAX;
          }
          a.ext[j] = emx[b][0];
          a.ext[(size_t)np + j] = -emn[b][0];  // emn <= INT64_MAX: no overflow
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            if (c >= nnc) break;
            const int e = 1 + a.npos[c];
            a.ext[(size_t)(2 * e) * np + j] = emx[b][1 + c];
            a.ext[(size_t)(2 * e + 1) * np + j] = -emn[b][1 + c];
          }
        }
      }
      return;
    }
  }
  if constexpr (MODE == 1) return;
  if (MODE == 2 && a.need_ext) {  // the extents merged over every shard
#pragma unroll
    for (int b = 0; b < GEN_BPW; ++b) {
      const int32_t j = jj[b];
      if (j >= np) continue;
      emx[b][0] = a.ext[j];
      emn[b][0] = -a.ext[(size_t)np + j];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if (c >= nnc) break;
        const int e = 1 + a.npos[c];
        emx[b][1 + c] = a.ext[(size_t)(2 * e) * np + j];
        emn[b][1 + c] = -a.ext[(size_t)(2 * e + 1) * np + j];
      }
    }
  }

  // ---- per pod: NodeNumber's two weighted values, each normalizing column's reciprocal ----
  Key cw[NC];  // the normalizing columns' weights, negated for REVERSE (its 100 w is in the keys' base)
  uint64_t tot0 = 0;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    cw[c] = 0;
    if (c >= nnc) break;
    const bool rev = a.nmode[c] == 2;
    if constexpr (KT == 2) cw[c] = rev ? -(double)a.nw[c] : (double)a.nw[c];
    else cw[c] = rev ? (Key)(0 - (uint64_t)a.nw[c]) : (Key)a.nw[c];
    if (rev) tot0 += (uint64_t)100 * (uint64_t)a.nw[c];
  }
  GLane<KT> L[GEN_BPW];
#pragma unroll
  for (int b = 0; b < GEN_BPW; ++b) {
    int64_t c1 = 0, c0 = 0;
    if (a.nn_score && a.nn_mode != 0 && emx[b][0] != INT64_MIN) {
      c1 = (int64_t)((uint64_t)gen_normalize(10, a.nn_mode, emx[b][0], emn[b][0]) * (uint64_t)a.nn_weight);
      c0 = (int64_t)((uint64_t)gen_normalize(0, a.nn_mode, emx[b][0], emn[b][0]) * (uint64_t)a.nn_weight);
    } else if (a.nn_score) {
      c1 = (int64_t)((uint64_t)10 * (uint64_t)a.nn_weight);  // NONE: raw x weight
    }
    if constexpr (KT == 2) {
      L[b].k1 = (double)(c1 + (int64_t)tot0);
      L[b].k0 = (double)(c0 + (int64_t)tot0);
    } else if constexpr (KT == 1) {
      L[b].k1 = ((uint64_t)c1 + tot0) ^ 0x8000000000000000ull;
      L[b].k0 = ((uint64_t)c0 + tot0) ^ 0x8000000000000000ull;
    } else {
      L[b].k1 = (uint32_t)((uint64_t)c1 + tot0) + 0x80000000u;
      L[b].k0 = (uint32_t)((uint64_t)c0 + tot0) + 0x80000000u;
    }
    // the class's NormalizeScore parameters: every pod of a class has the same extents, so the lanes of
    // a class write the same values (a class without a pod in the workgroup keeps r = 0: never read)
    if (jj[b] >= np) continue;
    const int kc = ntol[b] ? 0 : 1;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (c >= nnc) break;
      const int32_t md = a.nmode[c];
      const int64_t mx = emx[b][1 + c], mn = emn[b][1 + c];
      if (mx == INT64_MIN) continue;  // no feasible node
      double rr = 0.0, bb = 0.0;
      if (md == 3) {                  // min-max: (raw - mn) x 100 / (mx - mn), 0 when mx == mn
        if (mx != mn) {
          rr = (1.0 / (double)(mx - mn)) * GEN_RCP_BIAS;
          bb = 100.0 * (double)mn;
        }
      } else {  // DefaultNormalizeScore: 100 raw / max(mx, 0); DEFAULT leaves an all-zero list (m = 0 -> raw)
        const int64_t m = mx > 0 ? mx : 0;
        if (m != 0) rr = (1.0 / (double)m) * GEN_RCP_BIAS;
        else if (md == 1) rr = 0.01 * GEN_RCP_BIAS;
        // REVERSE with m == 0: r = 0, 100 - 0 = 100 for every node
      }
      s_crr[kc][c] = rr;
      s_cbb[kc][c] = bb;
    }
  }
  __syncthreads();  // the class parameters, before any class term is staged
  // The class term of node i for class kc from the uploaded columns: the node-only sum of the columns
  // without a normalizer, plus weight x trunc((100 raw - b) x r) per normalizing column (the exact
  // truncation of DESIGN.md §4.3). The staged tiles and the re-evaluation of the winning chunk use it alike.
  auto class_term = [&](int kc, int32_t i) -> Key {
    Key t = 0;
    if constexpr (TS) t = node_sum(i);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (c >= nnc) break;
      const double v = 100.0 * (double)a.cols[(size_t)a.ncc[c] * a.col_stride + i];
      t += col_term<KT, MMX>(v, s_cbb[kc][c], s_crr[kc][c], cw[c]);
    }
    return t;
  };

  // ---- stage 5: tiles of the node table through LDS, shared by the workgroup's waves ----
  auto stage = [&](int32_t t0) {
    const int32_t tn = min(TN, n - t0);
    for (int32_t k = threadIdx.x; k < ((tn + WAVE - 1) & ~(WAVE - 1)); k += GEN_W * WAVE) {
      const int32_t i = t0 + k;
      const bool in = k < tn;
      uint32_t xm = 0u;
      if (in) {
        const int dg = a.digit[i];
        xm = (a.has_nu && a.unsched[i]) ? 0xFFFFFFFFu : 0u;
        s_cx[k] = make_uint2((dg >= 0 && dg <= 9) ? (uint32_t)dg : GEN_CODE_NONE, xm);
        if constexpr (NCT == 2) {
          s_ct[2 * k] = class_term(0, i);
          s_ct[2 * k + 1] = class_term(1, i);
        } else if constexpr (NCT == 1) {
          s_ct[k] = class_term(0, i);
        }
      }
      const uint64_t m = __ballot(in && xm == 0u);
      if (m && lane == 0) atomicMin(&s_ffs, (uint32_t)(i - lane) + (uint32_t)__builtin_ctzll(m));
    }
  };
  // NodeNumber's key without a compare (32-bit keys, |c1 - c0| < 2^24: a.nn24): base + bit x delta, the bit
  // (v_bfe_u32) of the pod's one-hot code set at the node's code, base / delta ordered so that delta >= 0,
  // so the product and the add are one v_mad_u32_u24 and no lane mask (VCC) is written per pair
  uint32_t nsel[GEN_BPW], nbase[GEN_BPW], ndelta[GEN_BPW];
#pragma unroll
  for (int b = 0; b < GEN_BPW; ++b) {
    const uint32_t k1 = (uint32_t)L[b].k1, k0 = (uint32_t)L[b].k0, one = 1u << pcode[b];
    const bool up = k1 >= k0;
    nsel[b] = up ? one : ~one;
    nbase[b] = up ? k0 : k1;
    ndelta[b] = (up ? k1 - k0 : k0 - k1) & 0xFFFFFFu;
  }
  // the key of one pair, from a node's staged (or re-read) values: NodeNumber's part, plus the node's
  // class term for the pod's class (ct0: pods that do not tolerate the taint, ct1: pods that do)
  auto pair_key = [&](int b, uint32_t code, uint32_t xm, Key ct0, Key ct1, auto nnfast) -> Key {
    Key t;
    if constexpr (decltype(nnfast)::value && !W64)
      t = nbase[b] + __builtin_amdgcn_ubfe(nsel[b], code, 1) * ndelta[b];
    else
      t = code == pcode[b] ? L[b].k1 : L[b].k0;
    if constexpr (NCT == 2) t += ntol[b] ? ct0 : ct1;
    else if constexpr (NCT == 1) t += ct0;
    return key_mask<KT>(t, xm, ntol[b]);
  };

  // ---- stages 1, 2, 4: feasibility, the total, the first maximum ----
  Key best[GEN_BPW];
  int32_t cidx[GEN_BPW];
#pragma unroll
  for (int b = 0; b < GEN_BPW; ++b) {
    best[b] = KT == 2 ? Key(-__builtin_inf()) : Key(0);  // below every feasible key
    cidx[b] = -1;
  }
  auto main_pass = [&](auto nnfast) {
    for (int t = 0; t < n_tiles; ++t) {
      const int32_t t0 = t * TN, tn = min(TN, n - t0);
      if (n_tiles > 1 || !staged) {
        __syncthreads();
        stage(t0);
        __syncthreads();
        staged = true;
      }
      int32_t lo, hi;
      slice_of(tn, lo, hi);
      auto node_v = [&](uint2 cx, Key ct0, Key ct1) {
#pragma unroll
        for (int b = 0; b < GEN_BPW; ++b) {
          const Key key = pair_key(b, cx.x, cx.y, ct0, ct1, nnfast);
          if constexpr (KT == 2) best[b] = vmax_f64(best[b], key);  // an infeasible (NaN) key is skipped
          else best[b] = key > best[b] ? key : best[b];
        }
      };
      auto node = [&](int32_t k) {
        Key ct0 = 0, ct1 = 0;
        if constexpr (NCT == 2) {
          ct0 = s_ct[2 * k];
          ct1 = s_ct[2 * k + 1];
        } else if constexpr (NCT == 1) {
          ct0 = ct1 = s_ct[k];
        }
        node_v(s_cx[k], ct0, ct1);
      };
      // two nodes per LDS read (k even: a chunk starts at a multiple of GEN_CHUNK)
      auto node_pair = [&](int32_t k2) {  // nodes 2 k2, 2 k2 + 1
        const gen_u4 c2 = reinterpret_cast<const gen_u4*>(s_cx)[k2];
        Key ct[4] = {0, 0, 0, 0};  // node 2 k2's class terms, then node 2 k2 + 1's
        if constexpr (NCT == 2 && !W64) {
          const gen_u4 t4 = reinterpret_cast<const gen_u4*>(s_ct)[k2];
          ct[0] = t4.x;
          ct[1] = t4.y;
          ct[2] = t4.z;
          ct[3] = t4.w;
        } else if constexpr (NCT == 2) {
#pragma unroll
          for (int q = 0; q < 4; ++q) ct[q] = s_ct[4 * k2 + q];
        } else if constexpr (NCT == 1) {  // one term per node: both classes read it
          ct[0] = ct[1] = s_ct[2 * k2];
          ct[2] = ct[3] = s_ct[2 * k2 + 1];
        }
        node_v(make_uint2(c2.x, c2.y), ct[0], ct[1]);
        node_v(make_uint2(c2.z, c2.w), ct[2], ct[3]);
      };
      int32_t k = lo;
      for (; k + GEN_CHUNK <= hi; k += GEN_CHUNK) {
        Key prev[GEN_BPW];
#pragma unroll
        for (int b = 0; b < GEN_BPW; ++b) prev[b] = best[b];
#pragma unroll
        for (int q = 0; q < GEN_CHUNK / 2; ++q) {
          // with score columns two nodes' records per ds_read_b128 (4.30 against 4.43 ms per 32-batch C3
          // launch on NodeNumber + a DEFAULT column, one box); NodeNumber alone keeps the compiler's
          // ds_read2_b64 pairs (1.54 against 1.57 ms on the reference list; profiles/ab/r5_MSH_GEN_LDS128_*)
          if constexpr (CT) {
            node_pair((k >> 1) + q);
          } else {
            node(k + 2 * q);
            node(k + 2 * q + 1);
          }
        }

#pragma unroll
        for (int b = 0; b < GEN_BPW; ++b) cidx[b] = best[b] > prev[b] ? t0 + k : cidx[b];
      }
      if (k < hi) {  // the slice's last, partial chunk
        Key prev[GEN_BPW];
#pragma unroll
        for (int b = 0; b < GEN_BPW; ++b) prev[b] = best[b];
        for (int32_t q = k; q < hi; ++q) node(q);
#pragma unroll
        for (int b = 0; b < GEN_BPW; ++b) cidx[b] = best[b] > prev[b] ? t0 + k : cidx[b];
      }
    }
  };
  if (!W64 && a.nn24) main_pass(std::true_type{});
  else main_pass(std::false_type{});
  // the exact node: the first of the winning chunk whose key is the maximum (re-read from the uploaded
  // columns, the same arithmetic as the staged values)
  int32_t bidx[GEN_BPW];
#pragma unroll
  for (int b = 0; b < GEN_BPW; ++b) {
    bidx[b] = INT32_MAX;
    if (best[b] == (KT == 2 ? Key(-__builtin_inf()) : Key(0)) || jj[b] >= np) continue;
    const int32_t e = min(cidx[b] + GEN_CHUNK, n);
    for (int32_t i = cidx[b]; i < e; ++i) {
      const int dg = a.digit[i];
      const uint32_t code = (dg >= 0 && dg <= 9) ? (uint32_t)dg : GEN_CODE_NONE;
      const uint32_t xm = (a.has_nu && a.unsched[i]) ? 0xFFFFFFFFu : 0u;
      Key ct = 0;
      if constexpr (CT) ct = class_term(ntol[b] ? 0 : 1, i);
      if (pair_key(b, code, xm, ct, ct, std::false_type{}) == best[b]) {
        bidx[b] = i;
        break;
      }
    }
  }
  // slice waves of a pod group meet in LDS: the larger key, then the lower index (slices of one tile
  // ascend in List order, but a later tile's first slice follows an earlier tile's last)
  if (S > 1) {
    Key* m_key = reinterpret_cast<Key*>(s_merge);                                      // [GEN_W][BPW][64]
    int32_t* m_idx = reinterpret_cast<int32_t*>(s_merge + GEN_W * GEN_BPW * WAVE * sizeof(Key));
    __syncthreads();
#pragma unroll
    for (int b = 0; b < GEN_BPW; ++b) {
      m_key[(wv * GEN_BPW + b) * WAVE + lane] = best[b];
      m_idx[(wv * GEN_BPW + b) * WAVE + lane] = bidx[b];
    }
    __syncthreads();
    if (sl != 0) return;
    for (int k = 1; k < S; ++k) {
      const int ow = pg * S + k;
#pragma unroll
      for (int b = 0; b < GEN_BPW; ++b) {
        const Key ok = m_key[(ow * GEN_BPW + b) * WAVE + lane];
        const int32_t oi = m_idx[(ow * GEN_BPW + b) * WAVE + lane];
        if (ok > best[b] || (ok == best[b] && oi < bidx[b])) {
          best[b] = ok;
          bidx[b] = oi;
        }
      }
    }
  }
  const uint32_t ffs = s_ffs;  // complete: every tile has been staged (barriers above)
#pragma unroll
  for (int b = 0; b < GEN_BPW; ++b) {
    const int32_t j = jj[b];
    if (j >= np) continue;
    // the first feasible node: node 0 for a pod that tolerates the taint, else the first one the filter
    // passes for every pod
    const uint32_t ff = n == 0 ? GEN_NONE : (ntol[b] == 0u ? 0u : ffs);
    const bool found = ff != GEN_NONE;
    int64_t total;
    int32_t idx;
    if constexpr (KT == 2) {  // a found pod has a finite best total
      total = found ? (int64_t)best[b] : 0;
      idx = bidx[b];
    } else if (best[b] == 0) {  // every feasible total is INT64_MIN (64-bit totals only): the first feasible node
      total = INT64_MIN;
      idx = (int32_t)ff;
    } else {
      total = W64 ? (int64_t)((uint64_t)best[b] ^ 0x8000000000000000ull)
                  : (int64_t)(int32_t)((uint32_t)best[b] - 0x80000000u);
      idx = bidx[b];
    }
    if constexpr (MODE == 2) {  // this shard's best: merged by MAX total, then MIN global index
      a.best_total[j] = found ? total : INT64_MIN;
      a.best_idx[j] = found ? (int32_t)(a.node_base + idx) : INT32_MAX;
    } else {
      int32_t st = 0;
      if (!found) st = 1;                                             // FitError (minisched.go:143-148)
      else if (a.nn_score && (!a.nn_prescore || !pdok[b])) st = 2;    // NodeNumber.Score error (nodenumber.go:74-77)
      d.out_idx[j] = st ? -1 : idx;
      if (d.out_score) d.out_score[j] = st ? 0 : total;
      d.out_status[j] = st;
    }
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
  if (bi == INT32_MAX) st = 1;                            // no shard has a feasible node: FitError
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
constexpr size_t GEN_LDS_BUDGET = 40 * 1024;  // tile bytes per workgroup (4 workgroups per CU)

// Slice waves per pod group: one, unless the launch has fewer than ~2 pod groups per SIMD.
int gen_slices(int64_t groups, int32_t n, const DeviceInfo& dev) {
  if (dev.bits_slices > 0) return std::min(dev.bits_slices, GEN_W);
  const int64_t want = (int64_t)dev.cus * 4 * 2;
  int sl = 1;
  while (sl < GEN_W && groups * sl < want && n >= 256 * sl) sl *= 2;
  return sl;
}

template <int MODE, int KT, bool TS, int NNC, bool MMX>
hipError_t launch_gen_k(GenericArgs& a, int32_t bx, size_t lds, hipStream_t s) {
  auto k = generic_kernel<MODE, KT, TS, NNC, MMX>;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
  }
  MSH_TIMED_LAUNCH(k, dim3((unsigned)bx, (unsigned)a.nb), dim3(GEN_W * WAVE), (unsigned)lds, s, a);
  return hipGetLastError();
}

// At most one normalizing column, each key type: {a node-only sum or not} x {no normalizing column, one
// DEFAULT / REVERSE column, one MIN-MAX column}
template <int MODE, int KT>
hipError_t launch_gen_w(GenericArgs& a, int32_t bx, size_t lds, hipStream_t s) {
  const bool ts = a.nts > 0;
  if (a.nnc == 0) return ts ? launch_gen_k<MODE, KT, true, 0, false>(a, bx, lds, s)
                            : launch_gen_k<MODE, KT, false, 0, false>(a, bx, lds, s);
  const bool mm = a.nmode[0] == 3;
  if (ts) return mm ? launch_gen_k<MODE, KT, true, 1, true>(a, bx, lds, s)
                    : launch_gen_k<MODE, KT, true, 1, false>(a, bx, lds, s);
  return mm ? launch_gen_k<MODE, KT, false, 1, true>(a, bx, lds, s)
            : launch_gen_k<MODE, KT, false, 1, false>(a, bx, lds, s);
}

template <int MODE>
hipError_t launch_gen_mode(GenericArgs& a, int32_t bx, size_t lds, hipStream_t s) {
  // two or more normalizing columns: the general form (8-byte keys, a runtime column count): doubles when
  // the host bounds the totals below 2^53, else uint64_t (the extents mode computes no key)
  if (a.nnc > 1) {
    // exactly two normalizing columns under the 32-bit bound: 32-bit keys, a compile-time count
    if (a.nnc == 2 && !a.w64) return launch_gen_k<MODE, 0, true, 2, true>(a, bx, lds, s);
    if constexpr (MODE != 1) {
      // exactly two normalizing columns (compile-time count) or up to four (a runtime count)
      if (a.f53) return a.nnc == 2 ? launch_gen_k<MODE, 2, true, 2, true>(a, bx, lds, s)
                                   : launch_gen_k<MODE, 2, true, 4, true>(a, bx, lds, s);
    }
    return launch_gen_k<MODE, 1, true, 4, true>(a, bx, lds, s);
  }
  if (!a.w64) return launch_gen_w<MODE, 0>(a, bx, lds, s);
  // 8-byte keys: doubles when the host bounds the totals below 2^53, else uint64_t; the extents mode
  // computes no key (the 8-byte staging is the same), so it shares the uint64_t instances
  if constexpr (MODE != 1) {
    if (a.f53) return launch_gen_w<MODE, 2>(a, bx, lds, s);
  }
  return launch_gen_w<MODE, 1>(a, bx, lds, s);
}
}  // namespace

hipError_t launch_generic(GenericArgs& a, int mode, const DeviceInfo& dev, hipStream_t s) {
  if (a.nb <= 0 || a.nb > MULTI_MAX || a.nnc < 0 || a.nnc > GEN_COLS || a.nts < 0 || a.nts > GEN_COLS ||
      (mode != 0 && a.nb != 1))
    return hipErrorInvalidValue;
  int32_t maxp = 0;
  int64_t groups = 0;
  for (int b = 0; b < a.nb; ++b) {
    maxp = std::max(maxp, a.d[b].n_pods);
    groups += (a.d[b].n_pods + GEN_BPW * WAVE - 1) / (GEN_BPW * WAVE);
  }
  if (maxp == 0) return hipSuccess;
  const bool general = a.nnc > 1;  // launch_gen_mode's forms for two or more normalizing columns
  const size_t key = (a.w64 || (general && a.nnc > 2)) ? 8 : 4;  // launch_gen_mode's key type
  // bytes per staged node: the record, and the kernel's NCT terms: one per class with a normalizing column
  // (the general form included), one node-only sum otherwise, none for NodeNumber alone
  const size_t per_node = 8 + ((general || a.nnc > 0) ? 2 * key : (a.nts > 0 ? key : 0));
  int32_t tile = (int32_t)(GEN_LDS_BUDGET / per_node) & ~(GEN_CHUNK - 1);
  tile = std::max<int32_t>(GEN_CHUNK, std::min<int32_t>(tile, (a.n_nodes + GEN_CHUNK - 1) & ~(GEN_CHUNK - 1)));
  a.tile = tile;
  a.slices = gen_slices(groups, a.n_nodes, dev);
  // the slice merge (S > 1): (key, index) per pod
  const size_t merge = a.slices > 1 ? (size_t)GEN_W * GEN_BPW * WAVE * (key + 4) : 0;
  const size_t lds = (size_t)tile * per_node + merge;
  const int pgs = GEN_W / a.slices;
  const int32_t bx = (maxp + pgs * GEN_BPW * WAVE - 1) / (pgs * GEN_BPW * WAVE);
  if (mode == 1) return launch_gen_mode<1>(a, bx, lds, s);
  if (mode == 2) return launch_gen_mode<2>(a, bx, lds, s);
  return launch_gen_mode<0>(a, bx, lds, s);
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

}  // namespace msh
