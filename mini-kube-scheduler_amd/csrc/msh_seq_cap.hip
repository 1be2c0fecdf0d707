// msh_seq_cap.hip — the capacity form of the sequential-commit kernel: one workgroup walks the whole batch
// in order and a commit that fills a node makes it infeasible for the next pod (msh_schedule_sequential with
// max_pods_per_node > 0; the reference's serial loop, minisched/minisched.go:28-30, with a node-state commit
// between placements). A translation unit of its own so that the kernel families compile in parallel.
#include "msh_seq_kernel.h"

namespace msh {

// ---------------------------------------------------------------------------------------
// seq_capu_kernel: the capacity form on ONE wave, U pods per step. A commit changes a later decision only
// when it FILLS a node (the node leaves the availability planes), and then only for a pod whose first
// available match (or non-match) or class fallback was that very node. So the U pods of a step are
// scanned together against the state at the step's start (U independent chains, interleaved word by
// word), then resolved in order on the scalar unit:
//  * a pod whose scan result is a node an earlier pod of the step filled is scanned again (rare: a fill is
//    one commit in max_pods), the class fallbacks are the current scalars;
//  * the count of the committed node was read for the step's predicted placements in one batch of LDS
//    reads; a pod adds the commits of earlier pods of the step to the same node (their writes follow the
//    read), and reads again only when its placement differs from the prediction.
// The decisions are exactly the serial loop's. Per pod the scalar unit only picks the placement and
// commits; the identity-like decode (status, score) is done by the lanes once per 64 pods from the
// scan's first match and the class fallback kept in each pod's lane.
// ---------------------------------------------------------------------------------------
template <int RS, bool KX, int U>
__global__ __launch_bounds__(64) void seq_capu_kernel(SeqArgs a) {
  static_assert(WAVE % U == 0, "a step never straddles a 64-pod block");
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  // [n_words * 32 + 1] pods per node: carried in, updated, written back; the extra slot is the read target
  // of a placement without a commit (an index min(node, slots), no branch)
  extern __shared__ int32_t lcnt[];
  const int lane = threadIdx.x;
  const int32_t slots = a.n_words * 32;
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
  if (lane == 0) lcnt[slots] = 0;
  __syncthreads();
  int32_t max_pods = a.max_pods;
  asm volatile("" : "+s"(max_pods));
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
  auto first_avail = [&](const uint32_t (&av)[RS]) -> uint32_t {
    uint32_t f = NONE;
#pragma unroll
    for (int r = RS - 1; r >= 0; --r) f = umin(f, (lane_base + (uint32_t)(32 * r)) | ffbl(av[r]));
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_first(f));
  };
  uint32_t ca0 = first_avail(AV0), ca1 = first_avail(AV1);  // each class's first available node
  uint32_t cax = ca0 ^ ca1;  // a pod's fallback is ca1 ^ (cax & ~tolerates): two scalar ops, no compare
  __builtin_amdgcn_s_waitcnt(0);

  PluginParams pp = a.pp;
  asm volatile("" : "+s"(pp.has_nu_filter), "+s"(pp.has_nn_score), "+s"(pp.nn_prescore), "+s"(pp.mode),
               "+s"(pp.weight));
  const IdentDecode idec = make_ident_decode(pp);
  const int64_t sm = KX ? 100 * pp.weight : idec.sm;
  auto load_raw = [&](int32_t j0, int32_t& dr, int32_t& tr) {
    const int32_t jj = min(j0 + lane, a.n_pods - 1);
    dr = a.pod_digit[jj];
    tr = a.pod_tol[jj];
  };
  int32_t dn = 0, tn = 0;
  if (a.n_pods > 0) load_raw(0, dn, tn);
  // Per lane (pod jl of the block): the code bits as all-ones / all-zero masks, ~tolerates, and FL: in the
  // KX modes flags (bit 0: no commit — past the batch's end; bit 1: the pod's code is a digit), in the
  // identity-like modes the no-commit mask (all-ones for a score error or a pod past the batch's end).
  uint32_t P0 = 0, P1 = 0, P2 = 0, P3 = 0, NT = 0, FL = 0;
  // The block's outputs, lane jl = pod jl: identity-like modes keep the scan's first available match (o_a)
  // and the class fallback at the decision (o_b), decoded by the lanes at the store; KX modes keep the
  // decoded node (o_a) and status | scored << 2 (o_b).
  int32_t o_a = -1, o_b = 0;
  uint32_t fl_done = 0;  // the stored block's flags
  auto store_block = [&](int32_t j0, int32_t cnt) {
    if (lane < cnt) {
      int32_t sel, st;
      int64_t sc;
      if constexpr (KX) {
        sel = o_a;
        st = o_b & 3;
        sc = (o_b & 4) ? sm : 0;
      } else {  // decode_ident: FitError when the class had no available node, then the score error
        const bool fit = (uint32_t)o_b == NONE, hit = (uint32_t)o_a != NONE;
        st = fit ? 1 : ((fl_done & 1u) ? 2 : 0);
        sel = st ? -1 : (hit ? o_a : o_b);
        sc = (st == 0 && hit) ? sm : 0;
      }
      a.out_idx[j0 + lane] = sel;
      if (a.out_score) a.out_score[j0 + lane] = sc;
      a.out_status[j0 + lane] = st;
    }
  };
  for (int32_t jb = 0; jb < a.n_pods; jb += WAVE) {
    if (jb > 0) store_block(jb - WAVE, WAVE);
    {
      const bool ok = jb + lane < a.n_pods;
      const bool dig = ok && dn >= 0 && dn <= 9, tl = ok && tn != 0;
      // KX: decode_pod reads the code (the score error is its own); identity-like: a pod that cannot take
      // a match (its score errors, or NodeNumber does not score) scans with the code that matches nothing
      const bool serr = !ok || (!KX && (idec.err_all || (idec.err_nodigit && !dig)));
      const bool code = KX ? dig : (dig && idec.use_im && !serr);
      const uint32_t c = code ? (uint32_t)dn : CODE_NONE_POD;
      P0 = 0u - (c & 1u);
      P1 = 0u - ((c >> 1) & 1u);
      P2 = 0u - ((c >> 2) & 1u);
      P3 = 0u - ((c >> 3) & 1u);
      NT = tl ? 0u : 0xFFFFFFFFu;
      // KX: flags (bit 0 no commit, bit 1 a digit); identity-like: the no-commit mask, ORed into the placement
      FL = KX ? ((serr ? 1u : 0u) | (dig ? 2u : 0u)) : (serr ? NONE : 0u);
    }
    fl_done = FL;
    load_raw(jb + WAVE, dn, tn);
    const int32_t je = min(jb + WAVE, a.n_pods);
    for (int32_t j0 = jb; j0 < je; j0 += U) {
      const int32_t jl0 = j0 - jb;
      // ---- the U pods' masks (wave-uniform, SGPRs) and scans against the step's starting state ----
      uint32_t p0[U], p1[U], p2[U], p3[U], nt[U], fl[U], cm[U], cx[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        p0[u] = (uint32_t)__builtin_amdgcn_readlane((int)P0, jl0 + u);
        p1[u] = (uint32_t)__builtin_amdgcn_readlane((int)P1, jl0 + u);
        p2[u] = (uint32_t)__builtin_amdgcn_readlane((int)P2, jl0 + u);
        p3[u] = (uint32_t)__builtin_amdgcn_readlane((int)P3, jl0 + u);
        nt[u] = (uint32_t)__builtin_amdgcn_readlane((int)NT, jl0 + u);
        fl[u] = (uint32_t)__builtin_amdgcn_readlane((int)FL, jl0 + u);
        cm[u] = cx[u] = NONE;
      }
      // one pod's first available match (and non-match) in this lane's words: the class's availability by
      // a select on ~tolerates (nt ? AV0 : AV1), the code compare ORed over the four code planes
      auto scan_word = [&](int r, int u, uint32_t& m, uint32_t& x) {
        const uint32_t base = lane_base + (uint32_t)(32 * r);
        uint32_t dm = D0[r] ^ p0[u];
        dm = bop3_or_xor(dm, D1[r], p1[u]);
        dm = bop3_or_xor(dm, D2[r], p2[u]);
        dm = bop3_or_xor(dm, D3[r], p3[u]);
        const uint32_t av = __builtin_amdgcn_bitop3_b32(AV1[r], AV0[r], nt[u], 0xD8);  // nt ? AV0 : AV1
        m = umin(m, base | ffbl(bop3_andn(av, dm)));
        if (KX) x = umin(x, base | ffbl(av & dm));
      };
#pragma unroll
      for (int r = RS - 1; r >= 0; --r)
#pragma unroll
        for (int u = 0; u < U; ++u) scan_word(r, u, cm[u], cx[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        cm[u] = (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_first(cm[u]));
        if (KX) cx[u] = (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_first(cx[u]));
      }
      // ---- the placement of pod u from its scan and the current class fallback: node (NONE: no commit);
      // lane values: identity-like modes the scan's first match and the fallback (decoded per block), KX
      // modes the decoded node and status | scored << 2 ----
      auto decide = [&](int u, int32_t& va, int32_t& vb) -> uint32_t {
        const uint32_t ca = ca1 ^ (cax & nt[u]);
        if constexpr (KX) {
          int32_t sel, st;
          int64_t sc;
          decode_pod(cm[u] != NONE ? (int64_t)cm[u] : -1, cx[u] != NONE ? (int64_t)cx[u] : -1,
                     ca != NONE ? (int64_t)ca : -1, (fl[u] & 2u) != 0, pp, &sel, &sc, &st);
          sel = __builtin_amdgcn_readfirstlane(sel);
          st = __builtin_amdgcn_readfirstlane(st);
          va = sel;
          vb = st | (sc != 0 ? 4 : 0);
          return (st == 0 && !(fl[u] & 1u)) ? (uint32_t)sel : NONE;
        } else {
          va = (int32_t)cm[u];
          vb = (int32_t)ca;
          return (cm[u] != NONE ? cm[u] : ca) | fl[u];  // ca NONE: FitError; fl all-ones: no commit
        }
      };
      // the placements at the step's start (final unless an earlier pod of the step fills a node), and
      // their counts (one batch of LDS reads)
      uint32_t node[U], ci[U];
      int32_t va[U], vb[U], cnt[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        node[u] = decide(u, va[u], vb[u]);
        ci[u] = umin(node[u], (uint32_t)slots);  // NONE reads the spare slot
        cnt[u] = lcnt[ci[u]];
      }
      // ---- in pod order: the commit, and a fill's effect on the later pods ----
      bool filled[U];
      bool any_fill = false;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        filled[u] = false;
        bool fresh = false;  // the placement changed since the count was read
        if (any_fill) {
          // a scan result an earlier pod of this step filled: scan again against the current planes; the
          // class fallback may have moved too, so the placement is decided again
          bool redo = false;
#pragma unroll
          for (int v = 0; v < u; ++v)
            redo = redo || (filled[v] && (node[v] == cm[u] || (KX && node[v] == cx[u])));
          if (redo) {
            uint32_t m = NONE, x = NONE;
#pragma unroll
            for (int r = RS - 1; r >= 0; --r) scan_word(r, u, m, x);
            cm[u] = (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_first(m));
            if (KX) cx[u] = (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_first(x));
          }
          const uint32_t n2 = decide(u, va[u], vb[u]);
          fresh = n2 != node[u];
          node[u] = n2;
        }
        write_lane2(o_a, o_b, va[u], vb[u], jl0 + u);
        const uint32_t n = node[u];
        if (n == NONE) continue;
        // the node's count before this commit (NodeInfo.AddPod): the step's read plus the earlier pods of
        // the step that committed to it (their writes follow the read)
        int32_t c;
        if (!fresh) {
          c = __builtin_amdgcn_readfirstlane(cnt[u]);
#pragma unroll
          for (int v = 0; v < u; ++v) c += node[v] == n ? 1 : 0;
        } else {
          ci[u] = n;
          c = __builtin_amdgcn_readfirstlane(lcnt[n]);  // after every earlier commit's write (LDS in order)
        }
        lcnt[ci[u]] = c + 1;  // every lane stores the same value (ci[u] == n here)
        if (c + 1 >= max_pods) {  // the node is full: out of both classes' availability
          filled[u] = true;
          any_fill = true;
          const uint32_t w = n >> 5, q = w / RS, rs = w % RS;
          const uint32_t bit = (uint32_t)lane == q ? (1u << (n & 31)) : 0u;
#pragma unroll
          for (int r = 0; r < RS; ++r)
            if ((uint32_t)r == rs) {
              AV0[r] &= ~bit;
              AV1[r] &= ~bit;
            }
          if (ca0 == n) ca0 = first_avail(AV0);
          if (ca1 == n) ca1 = first_avail(AV1);
          cax = ca0 ^ ca1;
        }
      }
    }
  }
  if (a.n_pods > 0) {
    const int32_t j0 = (a.n_pods - 1) & ~(WAVE - 1);
    store_block(j0, a.n_pods - j0);
  }
  __syncthreads();  // every count update has landed
  for (int32_t i = lane; i < slots; i += WAVE) a.counts[i] = lcnt[i];
}

namespace {
constexpr int SEQ_CAP_AHEAD = 4;  // pods per step of seq_capu_kernel

template <int RS>
hipError_t launch_capu_rs(const SeqArgs& a, hipStream_t s) {
  const size_t lds = ((size_t)a.n_words * 32 + 1) * sizeof(int32_t);  // <= 128 KB + 4 B (32,768 nodes)
  auto kx = seq_capu_kernel<RS, true, SEQ_CAP_AHEAD>;
  auto id = seq_capu_kernel<RS, false, SEQ_CAP_AHEAD>;
  if (lds > 64 * 1024) {
    const void* k = needs_kx(a.pp) ? reinterpret_cast<const void*>(kx) : reinterpret_cast<const void*>(id);
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  if (needs_kx(a.pp)) MSH_TIMED_LAUNCH(kx, dim3(1), dim3(WAVE), lds, s, a);
  else MSH_TIMED_LAUNCH(id, dim3(1), dim3(WAVE), lds, s, a);
  return hipGetLastError();
}
}  // namespace

hipError_t launch_seq_capacity(const SeqArgs& a, int nw, int rs, hipStream_t s) {
  using seqlaunch::launch_seq_nw;
  if (nw == 1) {
    if (rs <= 1) return launch_capu_rs<1>(a, s);
    if (rs <= 2) return launch_capu_rs<2>(a, s);
    if (rs <= 3) return launch_capu_rs<3>(a, s);
    if (rs <= 4) return launch_capu_rs<4>(a, s);
    if (rs <= 6) return launch_capu_rs<6>(a, s);
    if (rs <= 8) return launch_capu_rs<8>(a, s);
    if (rs <= 12) return launch_capu_rs<12>(a, s);
    return launch_capu_rs<16>(a, s);
  }
  if (nw == 4) return launch_seq_nw<4, true, 1>(a, rs, 1, s);
  return launch_seq_nw<16, true, 1>(a, rs, 1, s);
}

}  // namespace msh
