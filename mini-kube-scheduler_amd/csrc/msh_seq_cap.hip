// msh_seq_cap.hip — the capacity form of the sequential-commit kernel: one workgroup walks the whole batch
// in order and a commit that fills a node makes it infeasible for the next pod (msh_schedule_sequential with
// max_pods_per_node > 0; the reference's serial loop, minisched/minisched.go:28-30, with a node-state commit
// between placements). A translation unit of its own so that the kernel families compile in parallel.
#include "msh_seq_kernel.h"

namespace msh {

// ---------------------------------------------------------------------------------------
// seq_cap1_kernel: the capacity form on ONE wave (tables up to 8,192 nodes: RS <= 4 words per lane).
// The general seq_kernel<..., CAP> decides a pod, then commits it and waits for the LDS count to come
// back before the next pod may scan (the FULL bit it may set is read by that scan), and scans a second
// first-hit chain (the first feasible node) per pod. Here:
//  * per tolerates class, an availability plane AV = V & ~FULL (& ~X for pods that do not tolerate the
//    unschedulable taint) per word: a pod's first available match is its code compare (4 VALU per word)
//    ANDed into AV and one first-hit step;
//  * the first available node of each class (the fallback of a pod without a match, and its FitError
//    when there is none) is kept as two wave-uniform scalars, recomputed only when that very node fills;
//  * the commit's count update (an LDS atomic) is resolved one pod LATE: pod j + 1 scans while pod j's
//    atomic is in flight, and only then reads the old count back. A node that fills removes ONE candidate,
//    which changes pod j + 1's choice only if pod j + 1 chose that node: then (rarely) its scan is redone.
//    The decisions are exactly the serial loop's.
// ---------------------------------------------------------------------------------------
template <int RS, bool KX>
__global__ __launch_bounds__(64) void seq_cap1_kernel(SeqArgs a) {
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  extern __shared__ int32_t lcnt[];  // [n_words * 32] pods per node: carried in, updated, written back
  const int lane = threadIdx.x;
  const int32_t slots = a.n_words * 32;
  // the counts (with the replicas of earlier pod-block launches folded in, a.fold) into LDS
  for (int32_t i = lane; i < slots; i += WAVE) {
    int32_t c = a.counts[i];
    if (a.fold) {
      for (int k = 1; k < a.count_replicas; ++k) {
        c += a.counts[k * a.count_stride + i];
        a.counts[k * a.count_stride + i] = 0;
      }
    }
    lcnt[i] = c;
  }
  __syncthreads();
  int32_t max_pods = a.max_pods;
  asm volatile("" : "+s"(max_pods));
  // the table in registers: lane l holds words l * RS .. l * RS + RS - 1 (List order across lanes)
  const uint32_t lane_base = (uint32_t)(lane * RS) << 5;  // node index of bit 0 of slot 0's word
  uint32_t D0[RS], D1[RS], D2[RS], D3[RS], AV0[RS], AV1[RS];
#pragma unroll
  for (int r = 0; r < RS; ++r) {
    const int32_t w = lane * RS + r;
    D0[r] = D1[r] = D2[r] = D3[r] = 0xFFFFFFFFu;  // code 15: never a match
    AV0[r] = AV1[r] = 0u;
    if (w < a.n_words) {
      const uint32_t* g = a.planes + (size_t)(w / PLANE_GW) * GROUP_DWORDS + w % PLANE_GW;
      D0[r] = g[0];
      D1[r] = g[PLANE_GW];
      D2[r] = g[2 * PLANE_GW];
      D3[r] = g[3 * PLANE_GW];
      uint32_t full = 0;
      for (int b = 0; b < 32; ++b) full |= (lcnt[w * 32 + b] >= max_pods ? 1u : 0u) << b;
      AV1[r] = g[PLANE_V * PLANE_GW] & ~full;
      AV0[r] = AV1[r] & ~g[PLANE_X * PLANE_GW];
    }
  }
  // The first available node of a class: the lanes' first (slots ascend), then the wave's first lane.
  auto first_avail = [&](const uint32_t (&av)[RS]) -> uint32_t {
    uint32_t f = NONE;
#pragma unroll
    for (int r = RS - 1; r >= 0; --r) f = umin(f, (lane_base + (uint32_t)(32 * r)) | ffbl(av[r]));
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_first(f));
  };
  uint32_t ca0 = first_avail(AV0), ca1 = first_avail(AV1);
  __builtin_amdgcn_s_waitcnt(0);  // the table loads drained here, not inside the loop

  PluginParams pp = a.pp;
  asm volatile("" : "+s"(pp.has_nu_filter), "+s"(pp.has_nn_score), "+s"(pp.nn_prescore), "+s"(pp.mode),
               "+s"(pp.weight));
  const IdentDecode idec = make_ident_decode(pp);
  const int64_t sm = KX ? 100 * pp.weight : idec.sm;  // the one non-zero score a decode gives
  // pods in lanes, 64 at a time: raw bytes loaded one block ahead, then one lane word per pod:
  // code | does-not-tolerate << 4
  auto load_raw = [&](int32_t j0, int32_t& dr, int32_t& tr) {
    const int32_t jj = min(j0 + lane, a.n_pods - 1);
    dr = a.pod_digit[jj];
    tr = a.pod_tol[jj];
  };
  int32_t dn = 0, tn = 0;
  if (a.n_pods > 0) load_raw(0, dn, tn);
  // lane jl of the block's outputs: the selected node (o_a) and status | scored << 2 (o_b)
  int32_t o_a = -1, o_b = 0;
  auto store_block = [&](int32_t j0, int32_t cnt) {
    if (lane < cnt) {
      a.out_idx[j0 + lane] = o_a;
      if (a.out_score) a.out_score[j0 + lane] = (o_b & 4) ? sm : 0;
      a.out_status[j0 + lane] = o_b & 3;
    }
  };
  // The previous pod's commit, resolved after the next pod's scan: its node (-1: none) and the node's count
  // before it (an LDS read in flight). The wave alone owns the counts, so the commit is a plain read, then
  // (one pod later) a write of count + 1: LDS operations of a wave complete in order, so a later pod's read
  // of the same node, issued after that write, sees it.
  int32_t pend = -1, pend_cnt = 0;
  uint32_t pkv = 0;
  for (int32_t jb = 0; jb < a.n_pods; jb += WAVE) {
    if (jb > 0) store_block(jb - WAVE, WAVE);
    {
      // lane word: code | does-not-tolerate << 4 | score error << 5. The identity-like decode is folded in
      // here, once per 64 pods by the lanes: a pod whose NodeNumber score errors (no PreScore state, or a
      // name without a digit; decode_ident) or is not scored at all never takes a match, so its code
      // becomes CODE_NONE_POD and its scan finds none; per pod the scalar unit then only picks the match
      // or the class's first available node.
      const bool ok = jb + lane < a.n_pods;
      const bool dig = ok && dn >= 0 && dn <= 9, tl = ok && tn != 0;
      const bool serr = !KX && (idec.err_all || (idec.err_nodigit && !dig));
      const bool code = KX ? dig : (dig && idec.use_im && !serr);
      pkv = (code ? (uint32_t)dn : CODE_NONE_POD) | (tl ? 0u : 16u) | (serr ? 32u : 0u);
    }
    load_raw(jb + WAVE, dn, tn);
    const int32_t je = min(jb + WAVE, a.n_pods);
    for (int32_t j = jb; j < je; ++j) {
      const int32_t jl = j - jb;
      const uint32_t pk = (uint32_t)__builtin_amdgcn_readlane((int)pkv, jl);
      const uint32_t p0 = 0u - (pk & 1u), p1 = 0u - ((pk >> 1) & 1u), p2 = 0u - ((pk >> 2) & 1u),
                     p3 = 0u - ((pk >> 3) & 1u);
      const bool tol = ((pk >> 4) & 1u) == 0;
      uint32_t cm = NONE, cx = NONE;  // the first available match / non-match (KX)
      auto scan = [&](const uint32_t (&av)[RS]) {
        cm = cx = NONE;
#pragma unroll
        for (int r = RS - 1; r >= 0; --r) {
          const uint32_t base = lane_base + (uint32_t)(32 * r);
          uint32_t dm = D0[r] ^ p0;
          dm = or_xor_vs(dm, D1[r], p1);
          dm = or_xor_vs(dm, D2[r], p2);
          dm = or_xor_vs(dm, D3[r], p3);
          cm = umin(cm, base | ffbl(bop3_andn(av[r], dm)));
          if (KX) cx = umin(cx, base | ffbl(av[r] & dm));
        }
        cm = (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_first(cm));
        if (KX) cx = (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_first(cx));
      };
      if (tol) scan(AV1);
      else scan(AV0);
      // the previous pod's commit: did its node just fill?
      const int32_t c = __builtin_amdgcn_readfirstlane(pend_cnt) + 1;
      if (pend >= 0) {
        lcnt[pend] = c;  // every lane stores the same value
        if (c >= max_pods) {
          const uint32_t w = (uint32_t)pend >> 5, q = w / RS, rs = w % RS;
          const uint32_t m = (uint32_t)lane == q ? (1u << (pend & 31)) : 0u;
#pragma unroll
          for (int r = 0; r < RS; ++r)
            if ((uint32_t)r == rs) {
              AV0[r] &= ~m;
              AV1[r] &= ~m;
            }
          if (cm == (uint32_t)pend || (KX && cx == (uint32_t)pend)) {  // this pod chose it: decide again
            if (tol) scan(AV1);
            else scan(AV0);
          }
          if (ca0 == (uint32_t)pend) ca0 = first_avail(AV0);
          if (ca1 == (uint32_t)pend) ca1 = first_avail(AV1);
        }
      }
      const uint32_t ca = tol ? ca1 : ca0;
      int32_t sel, st;
      if constexpr (KX) {
        int64_t sc;
        decode_pod(cm != NONE ? (int64_t)cm : -1, cx != NONE ? (int64_t)cx : -1, ca != NONE ? (int64_t)ca : -1,
                   (pk & 15u) != CODE_NONE_POD, pp, &sel, &sc, &st);
        st |= sc != 0 ? 4 : 0;
      } else {  // decode_ident with the score error from the lane word (a pod with one has no match)
        const bool fit = ca == NONE, serr = (pk >> 5) & 1u, hit = cm != NONE;
        st = fit ? 1 : (serr ? 2 : (hit ? 4 : 0));
        sel = st & 3 ? -1 : (int32_t)(hit ? cm : ca);
      }
      // wave-uniform by construction (every input is): kept in SGPRs, so the commit and the next pod's
      // resolve branch on the scalar unit instead of masking lanes
      sel = __builtin_amdgcn_readfirstlane(sel);
      st = __builtin_amdgcn_readfirstlane(st);
      write_lane2(o_a, o_b, sel, st, jl);
      st &= 3;
      // commit (NodeInfo.AddPod): the node's count is read now and used after the next scan; the read is
      // issued for every pod (of node 0 when there is no commit), so that exactly one read is in flight
      // at the resolve and the compiler's wait for it lands there, not earlier
      pend = st == 0 ? sel : -1;
      pend_cnt = lcnt[st == 0 ? sel : 0];
    }
  }
  if (pend >= 0) lcnt[pend] = __builtin_amdgcn_readfirstlane(pend_cnt) + 1;  // the last pod's commit
  if (a.n_pods > 0) {
    const int32_t j0 = (a.n_pods - 1) & ~(WAVE - 1);
    store_block(j0, a.n_pods - j0);
  }
  __syncthreads();  // every count update has landed
  for (int32_t i = lane; i < slots; i += WAVE) a.counts[i] = lcnt[i];
}

namespace {
template <int RS>
hipError_t launch_cap1_rs(const SeqArgs& a, hipStream_t s) {
  const size_t lds = (size_t)a.n_words * 32 * sizeof(int32_t);  // <= 32 KB (8,192 nodes)
  if (needs_kx(a.pp)) MSH_TIMED_LAUNCH((seq_cap1_kernel<RS, true>), dim3(1), dim3(WAVE), lds, s, a);
  else MSH_TIMED_LAUNCH((seq_cap1_kernel<RS, false>), dim3(1), dim3(WAVE), lds, s, a);
  return hipGetLastError();
}
}  // namespace

hipError_t launch_seq_capacity(const SeqArgs& a, int nw, int rs, hipStream_t s) {
  using seqlaunch::launch_seq_nw;
  if (nw == 1) {
    if (rs <= 1) return launch_cap1_rs<1>(a, s);
    if (rs <= 2) return launch_cap1_rs<2>(a, s);
    if (rs <= 3) return launch_cap1_rs<3>(a, s);
    return launch_cap1_rs<4>(a, s);
  }
  if (nw == 4) return launch_seq_nw<4, true, 1>(a, rs, 1, s);
  return launch_seq_nw<16, true, 1>(a, rs, 1, s);
}

}  // namespace msh
