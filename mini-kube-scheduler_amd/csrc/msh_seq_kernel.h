// msh_seq_kernel.h — the sequential-commit kernel template (BASELINE C5, gfx950): one workgroup walks the
// pods in order and commits each placement before a later decision reads it, the reference's strictly
// sequential scheduleOne loop (minisched/minisched.go:28-30, 32-113) with NodeInfo.AddPod as the commit.
// Instantiated by msh_seq.hip (no capacity) and msh_seq_cap.hip (with one): two translation units that
// compile in parallel.
#pragma once

#include "msh_device.h"

namespace msh {

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

// Threads of a seq_kernel workgroup: NW scanning waves (+ the finalizer wave without a capacity), or PW
// pod waves (one scanning wave each, pod blocks).
constexpr int seq_threads(int nw, bool cap, int pw) { return (pw > 1 ? pw : nw + ((!cap && nw > 1) ? 1 : 0)) * 64; }

// U: pods decided per step (U > 1 only for one wave without a capacity; U divides 64).
// PW: pod waves per workgroup (one scanning wave, pod blocks): each wave holds the whole table and walks
// 64 / PW consecutive pods of the workgroup's 64-pod block in order; the waves share the block's LDS
// counts. PW = 1: one wave walks the whole block.
template <int RS, int NW, bool KX, bool CAP, int U, int PW = 1>
__global__ __launch_bounds__(seq_threads(NW, CAP, PW)) void seq_kernel(SeqArgs a0) {
  static_assert(U == 1 || !CAP, "pods are decided ahead of commits only when no commit feeds a decision");
  static_assert(PW == 1 || (NW == 1 && !CAP), "pod waves: one scanning wave, no capacity");
  constexpr bool FIN = !CAP && NW > 1;  // a finalizer wave decodes, keeps the outputs and commits
  constexpr int FINW = FIN ? NW : 0;    // the wave that keeps the outputs
  // Without a capacity no commit feeds a later decision, so the launcher may split the pods into
  // 64-pod blocks of consecutive pods, one workgroup each (as ranks split them in pod-sharded
  // sequential mode): each walks its block in order against the whole table, and its commits are
  // added to the device counts, which then equal the serial loop's. With a capacity: one workgroup.
  const bool split = !CAP && gridDim.x > 1;
  SeqArgs a = a0;
  if (split) {
    // this wave's pods: sub-block pw of the workgroup's block (PW = 1: the whole block)
    const int pw = PW > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
    const int32_t sub = a0.pods_per_block / PW;
    const int32_t j0 = (int32_t)blockIdx.x * a0.pods_per_block + pw * sub;
    a.n_pods = max(0, min(sub, a0.n_pods - j0));
    a.pod_digit += j0;
    a.pod_tol += j0;
    a.out_idx += j0;
    if (a.out_score) a.out_score += j0;
    a.out_status += j0;
  }
  // Counts in LDS (up to 4 waves x 64 lanes x 4 words x 32 nodes = 32,768 nodes, 128 KB), else
  // device-memory atomics (one workgroup only). Split: a block counts its 64 commits in LDS and adds
  // one device atomic per node it reached, into count replica blockIdx % SEQ_COUNT_REPLICAS. A digit's
  // pods all land on its first feasible match, so device atomics from every block onto one array queue
  // on about ten addresses. Per C5 launch (1,563 blocks): one atomic per commit 149 us, one per block
  // and node 26 us, the same over 16 replicas 11.6 us (11.3 without any add; 64 replicas since the
  // pair form's epilogue needs them, msh_internal.h). (Merging 32 blocks'
  // counts through staging rows and a last-block ticket needs an agent-scope release per block, an L2
  // write-back on MI355X: 52 us.)
  constexpr bool LDSC = NW <= 4;
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  // per-step exchange slots (NW > 1), triple-buffered: [slot][pod of the step][first match, first
  // feasible, first feasible non-match]
  __shared__ uint32_t xs[3][U][3];
  extern __shared__ int32_t lcnt[];  // [n_pad] per-node pod counts (LDSC)
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = NW == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool scanner = !FIN || wv < NW;

  if (a0.fold && !split) {  // one workgroup: the replicas' counts into replica 0 first
    for (int32_t i = threadIdx.x; i < a.n_words * 32; i += blockDim.x) {
      int32_t sum = 0;
      for (int k = 1; k < a.count_replicas; ++k) {
        sum += a.counts[k * a.count_stride + i];
        a.counts[k * a.count_stride + i] = 0;
      }
      a.counts[i] += sum;
    }
    __syncthreads();
  }
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
  if (LDSC) {  // ordered before the first commit by the first pod's exchange / barrier
    if (split) {
      for (int32_t i = threadIdx.x; i < a.n_words * 8; i += blockDim.x)
        reinterpret_cast<int4*>(lcnt)[i] = make_int4(0, 0, 0, 0);
    } else {
      for (int32_t i = threadIdx.x; i < a.n_words * 32; i += blockDim.x) lcnt[i] = a.counts[i];
    }
  }
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
        if (LDSC) {
          const int32_t old = atomicAdd(&lcnt[sel], 1);
          if (PW == 1 && split && old == 0) {  // split: the lane that counted a node first for this 64-pod block
            // moves the block's count of it (every lane's add has landed: one wave, LDS in order) to
            // the device counts and clears it for the next block
            const int32_t c = lcnt[sel];
            lcnt[sel] = 0;
            atomicAdd(&counts[(int64_t)(blockIdx.x % SEQ_COUNT_REPLICAS) * a0.count_stride + sel], c);
          }
        } else {
          atomicAdd(&counts[sel], 1);  // one workgroup (the launcher splits LDS-count tables only)
        }
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
  if (LDSC && !split) {
    __syncthreads();
    for (int32_t i = threadIdx.x; i < a.n_words * 32; i += blockDim.x) a.counts[i] = lcnt[i];
  }
  if (PW > 1 && split) {  // the block's counts (every wave's commits) to its device count replica
    __syncthreads();
    int32_t* rep = counts + (int64_t)(blockIdx.x % SEQ_COUNT_REPLICAS) * a0.count_stride;
    for (int32_t i = threadIdx.x; i < a.n_words * 32; i += blockDim.x) {
      const int32_t c = lcnt[i];
      if (c) atomicAdd(&rep[i], c);
    }
  }
}

namespace seqlaunch {
constexpr int SEQ_AHEAD = 4;  // pods decided per step without a capacity

// PW: pod waves per workgroup (one scanning wave, pod blocks), else 1
template <int RS, int NW, bool CAP, int PW>
hipError_t launch_seq_rs(const SeqArgs& a, int32_t blocks, hipStream_t s) {
  const dim3 blk(seq_threads(NW, CAP, PW));  // + the finalizer wave without a capacity
  const size_t lds = NW <= 4 ? (size_t)a.n_words * 32 * sizeof(int32_t) : 0;  // seq_kernel's LDSC
  constexpr int U = !CAP ? SEQ_AHEAD : 1;
  auto kx = seq_kernel<RS, NW, true, CAP, U, PW>;
  auto id = seq_kernel<RS, NW, false, CAP, U, PW>;
  const void* k = needs_kx(a.pp) ? reinterpret_cast<const void*>(kx) : reinterpret_cast<const void*>(id);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  if (needs_kx(a.pp)) MSH_TIMED_LAUNCH(kx, dim3((unsigned)blocks), blk, lds, s, a);
  else MSH_TIMED_LAUNCH(id, dim3((unsigned)blocks), blk, lds, s, a);
  return hipGetLastError();
}

template <int NW, bool CAP, int PW>
hipError_t launch_seq_nw(const SeqArgs& a, int rs, int32_t blocks, hipStream_t s) {
  if constexpr (NW == 1) {
    if (rs <= 1) return launch_seq_rs<1, NW, CAP, PW>(a, blocks, s);
    if (rs <= 2) return launch_seq_rs<2, NW, CAP, PW>(a, blocks, s);
    if (rs <= 3) return launch_seq_rs<3, NW, CAP, PW>(a, blocks, s);
    return launch_seq_rs<4, NW, CAP, PW>(a, blocks, s);
  } else if constexpr (NW == 4) {
    if (rs <= 2) return launch_seq_rs<2, NW, CAP, PW>(a, blocks, s);
    return launch_seq_rs<4, NW, CAP, PW>(a, blocks, s);
  } else {
    if (rs <= 4) return launch_seq_rs<4, NW, CAP, PW>(a, blocks, s);
    if (CAP || rs <= 8) return launch_seq_rs<8, NW, CAP, PW>(a, blocks, s);
    return launch_seq_rs<(CAP ? 8 : 12), NW, CAP, PW>(a, blocks, s);  // (CAP at 12 words per lane spills)
  }
}
}  // namespace seqlaunch


}  // namespace msh
