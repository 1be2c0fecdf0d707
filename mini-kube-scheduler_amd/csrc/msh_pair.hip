// msh_pair.hip — the per-pair batch kernels (gfx950): pair_kernel (node planes by scalar loads) and
// pair_lds_kernel (planes staged in LDS), the default batch path of the reference plugin list in every
// normalize mode: msh_schedule_batch*, msh_schedule_batches_device and msh_shard_keys_device.
//
// Reference path (shopetan/mini-kube-scheduler, Go): for ONE pod per cycle,
//   RunFilterPlugins   minisched/minisched.go:115-151  (NodeUnschedulable, upstream v1.22.0)
//   RunPreScorePlugins minisched/minisched.go:153-162  (NodeNumber.PreScore, nodenumber.go:50-64)
//   RunScorePlugins    minisched/minisched.go:164-199  (NodeNumber.Score, nodenumber.go:73-95)
//   selectHost         minisched/minisched.go:304-325  (argmax; ties -> lowest index here)
// EVERY (pod, node) pair's filter verdict and NodeNumber score is evaluated from the bit planes, 32 pairs
// per lane-op. See DESIGN.md §4.2 for the instruction budget and the A/B record behind each choice.
#include "msh_device.h"

namespace msh {

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

// NPL planes of group g: by scalar loads (LDSP false), or (LDSP) from the workgroup's LDS copy of the
// table as wave-uniform ds_read_b128 (a broadcast) into VGPRs.
template <int NPL, bool LDSP>
__device__ __forceinline__ void get_group(u32x8* pl, const uint32_t* planes, const uint4* s_tab, int32_t g) {
  if constexpr (LDSP) {
    const uint4* q = s_tab + g * (GROUP_DWORDS / 4);
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const uint4 lo = q[2 * k], hi = q[2 * k + 1];
      pl[k] = u32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    }
  } else {
    sload_group<NPL>(pl, planes + (size_t)g * GROUP_DWORDS);
  }
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

template <int S, bool SHARD, bool KX, bool CNT, int NB, bool LDSP>
__global__ __launch_bounds__(PAIR_WAVES * WAVE) void pair_kernel(PairArgsN<NB> a) {
  constexpr int PB = PAIR_WAVES / S;  // 64-pod blocks per workgroup
  __shared__ uint32_t s_res[S > 1 ? PAIR_WAVES : 1][2][WAVE];
  extern __shared__ uint4 s_tabp[];  // LDSP: the table's planes (n_groups x GROUP_DWORDS)
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int sl = wv % S, pb = wv / S;
  const BatchDesc& d = a.d[NB == 1 ? 0 : blockIdx.y];
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
  if constexpr (LDSP) {  // the table into LDS, its loads in flight together with the pod loads above
    const uint4* src = reinterpret_cast<const uint4*>(a.planes);
    const int32_t n4 = a.n_groups * (GROUP_DWORDS / 4);
    for (int32_t i = (int32_t)threadIdx.x; i < n4; i += PAIR_WAVES * WAVE) s_tabp[i] = src[i];
    __syncthreads();
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
        get_group<PLANE_V, LDSP>(pl, a.planes, s_tabp, gg);
        pair_group<false, KX>(pl, P0, P1, P2, P3, nT, am, ax);
        if constexpr (!KX) group_feasible_s<false>(pl, sn, st);
      } else {
        get_group<PLANE_N, LDSP>(pl, a.planes, s_tabp, gg);
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
    get_group<PLANE_N, LDSP>(pl, a.planes, s_tabp, g_lo);
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
        get_group<PLANE_N, LDSP>(p2, a.planes, s_tabp, (int32_t)fn);
        an = group_first_feasible_s<true>(p2, fn);
      }
      if (at == NOFIT && ft != NO_GROUP) {
        u32x8 p2[PLANE_N];
        get_group<PLANE_N, LDSP>(p2, a.planes, s_tabp, (int32_t)ft);
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
    if constexpr (CNT) {
      // sequential mode without a capacity (msh_schedule_sequential_device): the commit of every placed
      // pod, NodeInfo.AddPod's count (minisched.go:89-112 binds it), one device atomic per distinct node
      // of the wave (a digit's pods all land on its first feasible match), into count replica
      // (block mod SEQ_COUNT_REPLICAS) so that the atomics of many waves do not queue on one address (all
      // waves reach it at about the same time: 16 replicas cost 8.5 us per C5 launch, 64 cost 1.5)
      const uint32_t node = ost == 0 ? (uint32_t)oi : NOFIT;
      uint64_t pend = __ballot(ost == 0);
      int32_t* cnt = a.counts + (size_t)((((int32_t)blockIdx.x * PB + pb)) % SEQ_COUNT_REPLICAS) * a.count_stride;
      while (pend) {
        const int ld = (int)__builtin_ctzll(pend);
        const uint32_t n = (uint32_t)__builtin_amdgcn_readlane((int)node, ld);
        const uint64_t same = __ballot(node == n);
        if (lane == ld) atomicAdd(cnt + n, (int32_t)__popcll(same));
        pend &= ~same;
      }
    }
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
// Each wave evaluates PL_BPW = 2 64-pod blocks together: a group's planes are read from LDS once per
// wave and applied to both, and the table copy is amortised over W x 2 blocks.
// Per lane and 32-node word: xi = X & nT, dm' (4 v_bitop3), and per two words one AND3 into the
// group's match flag, plus, KX, one OR of the feasible non-matches (dm' & ~xi), or, identity-like
// modes, one AND3 of two words' xi per two words (the group holds a feasible node iff not all-ones).
// The forms that lost their A/B (profiles/r4_ab_pair_planes.txt) are no longer built:
// one, three and four blocks per wave; the pure-LDS full-group form (a full group always takes hybrid
// planes: X and D3 by scalar loads, D0-D2 from LDS); compaction in the identity-like modes and hybrid
// form 1 in REVERSE / MINMAX. What is left per (SHARD, KX) is the launcher's choice at 4 and 16 waves.
// ---------------------------------------------------------------------------------------
constexpr int PL_WAVES = 4;  // waves per workgroup (tables up to PAIR_LDS_MAX_GROUPS groups)
constexpr int PL_WAVES_BIG = 16;  // waves per workgroup for larger tables: one copy of up to 78 KB serves
                                  // 16 waves (two workgroups per CU: 8 waves per SIMD)
constexpr int PAIR_LDS_BIG_GROUPS = 416;  // 106,496 nodes, 78 KB per workgroup
constexpr int PL_BPW = 2;                 // 64-pod blocks per wave
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

// W waves per workgroup (PL_WAVES or PL_WAVES_BIG). REVERSE / MINMAX (KX) compact the tolerates bit in
// 4-wave workgroups (2% faster; in 16-wave ones its 8.3 KB of static LDS on top of a table of up to 78 KB
// would leave one workgroup per CU) and load both groups' scalar planes of a step under one wait (HY 2,
// 3% faster); the identity-like modes wait per group (HY 1).
// (Two attempts to hide the LDS broadcast latency lost their A/B, DESIGN.md §4.2: a software-pipelined
// scan — group g-1's LDS and scalar planes requested by one asm block before group g's v_bitop3 chains,
// one explicit wait per group — ran 81.4 against 76.7 us per 32-batch C3 launch in the identity-like
// modes, 80.3 against 80.0 in MINMAX; the identity-like 4-wave form compiled for 8 waves per SIMD
// (amdgpu_waves_per_eu(8): 64 VGPRs, 36 B of spills outside the scan loop, against 78 VGPRs and 6 waves)
// ran 78.1 against 78.0 at w=3 DEFAULT and 78.6 against 78.2 at w=1 NONE.)
template <bool SHARD, bool KX, int W>
__global__ __launch_bounds__(W * WAVE) void pair_lds_kernel(PairArgs a) {
  constexpr bool CMP = KX && W == PL_WAVES;
  constexpr int HY = KX ? 2 : 1;
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
        if (gg < g_full) {  // a full group: hybrid planes
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

namespace {
// Slice waves per 64-pod block of pair_kernel: one, unless the launch has fewer than ~4 waves per
// SIMD; then 2 or 4, while each slice keeps at least two groups.
int pair_slices(int64_t waves, int32_t n_groups, const DeviceInfo& dev) {
  if (dev.bits_slices > 0) return dev.bits_slices;
  const int64_t want = (int64_t)dev.cus * 4 * 4;
  int sl = 1;
  while (sl < PAIR_WAVES && waves * sl < want && n_groups >= 4 * sl) sl *= 2;
  return sl;
}

template <int S, bool SHARD, bool KX, bool LDSP>
hipError_t launch_pair_l(PairArgs& a, int32_t bx, hipStream_t s) {
  a.gps = (a.n_groups + S - 1) / S;
  const dim3 grid((unsigned)bx, (unsigned)a.nb), blk(PAIR_WAVES * WAVE);
  const unsigned lds = LDSP ? (unsigned)(a.n_groups * GROUP_DWORDS * sizeof(uint32_t)) : 0u;
  if (a.nb == 1) {  // one descriptor's worth of kernel arguments (shard-key and counting launches: always)
    PairArgsN<1> b;
    static_cast<PairCommon&>(b) = a;
    b.d[0] = a.d[0];
    if (a.counts) {
      if constexpr (SHARD) return hipErrorInvalidValue;  // (launch_pairs rejects it first)
      else MSH_TIMED_LAUNCH((pair_kernel<S, false, KX, true, 1, LDSP>), grid, blk, lds, s, b);
    } else {
      MSH_TIMED_LAUNCH((pair_kernel<S, SHARD, KX, false, 1, LDSP>), grid, blk, lds, s, b);
    }
    return hipGetLastError();
  }
  if constexpr (SHARD) return hipErrorInvalidValue;  // shard keys: one batch (launch_pairs rejects more first)
  else MSH_TIMED_LAUNCH((pair_kernel<S, false, KX, false, MULTI_MAX, LDSP>), grid, blk, lds, s, a);
  return hipGetLastError();
}

// Planes from LDS for tables up to PAIR_SLICE_LDS_GROUPS groups (msh_options.pair_planes = 1 keeps scalar
// loads): a one-batch C3 launch waited on five dependent scalar-load round trips per wave.
constexpr int PAIR_SLICE_LDS_GROUPS = 128;  // 32,768 nodes, 24 KB per workgroup
template <int S, bool SHARD, bool KX>
hipError_t launch_pair_s(PairArgs& a, int32_t bx, const DeviceInfo& dev, hipStream_t s) {
  if (dev.pair_planes != 1 && a.n_groups <= PAIR_SLICE_LDS_GROUPS) return launch_pair_l<S, SHARD, KX, true>(a, bx, s);
  return launch_pair_l<S, SHARD, KX, false>(a, bx, s);
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
  // (big: two 16-wave workgroups per CU fill it from 32 blocks per CU on; 4-wave workgroups from 64 waves
  // per CU)
  const int64_t min_waves = (int64_t)dev.cus * (big ? 2 * PL_WAVES_BIG : 64);
  // (counting launches, sequential mode: always scalar-loaded planes, whose kernel has the commit epilogue)
  const bool lds = !a.counts && (fits || big) && (dev.pair_planes == 2 ||
                                     (dev.pair_planes == 0 && waves >= min_waves && dev.bits_slices == 0));
  if (lds) {
    const int w = big ? PL_WAVES_BIG : PL_WAVES;
    const int32_t blocks = (maxp + WAVE - 1) / WAVE;
    const int32_t bx = (blocks + w * PL_BPW - 1) / (w * PL_BPW);
    const size_t bytes = (size_t)a.n_groups * GROUP_DWORDS * sizeof(uint32_t);
    const dim3 grid((unsigned)bx, (unsigned)a.nb), blk(w * WAVE);
    a.noax = dev.pair_noax >= 0 ? dev.pair_noax : (KX ? 1 : 0);
    using PairKernel = void (*)(PairArgs);
    const PairKernel k = big ? pair_lds_kernel<SHARD, KX, PL_WAVES_BIG> : pair_lds_kernel<SHARD, KX, PL_WAVES>;
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
    case 1: return launch_pair_s<1, SHARD, KX>(a, bx(1), dev, s);
    case 2: return launch_pair_s<2, SHARD, KX>(a, bx(2), dev, s);
    default: return launch_pair_s<4, SHARD, KX>(a, bx(4), dev, s);
  }
}
}  // namespace

hipError_t launch_pairs(PairArgs& a, bool shard, const DeviceInfo& dev, hipStream_t s) {
  if (a.nb <= 0 || a.nb > MULTI_MAX || (shard && a.nb != 1) || (a.counts && (shard || a.nb != 1)))
    return hipErrorInvalidValue;
  // KX: the normalize mode needs each pod's first feasible non-match (REVERSE, MINMAX)
  if (needs_kx(a.pp)) return shard ? launch_pair_t<true, true>(a, dev, s) : launch_pair_t<false, true>(a, dev, s);
  return shard ? launch_pair_t<true, false>(a, dev, s) : launch_pair_t<false, false>(a, dev, s);
}

}  // namespace msh
