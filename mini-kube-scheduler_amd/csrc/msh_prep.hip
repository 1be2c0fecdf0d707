// msh_prep.hip — gfx950 kernels around the hot path: the node table's bit planes (every upload and
// filter-list change), their O(change) update for msh_patch_nodes, the decode of merged node-shard keys,
// and the per-pair result export (f4). The hot kernels live in msh_pair.hip (per-pair batch kernels),
// msh_generic.hip (explicit int64 score pipeline) and msh_seq.hip (sequential commit).
#include "msh_device.h"

namespace msh {

thread_local hipEvent_t t_ev_start = nullptr, t_ev_stop = nullptr;

void set_launch_events(hipEvent_t start, hipEvent_t stop) {
  t_ev_start = start;
  t_ev_stop = stop;
}
bool launch_events_pending() { return t_ev_start != nullptr; }

// NodeUnschedulable.Filter rejects node i for a pod that does not tolerate the unschedulable taint
// (upstream v1.22.0: Spec.Unschedulable && !tolerates -> UnschedulableAndUnresolvable), and
// NodeNumber reads the suffix digit of its name (nodenumber.go:50-64, 80-95): code = digit, or
// CODE_NONE_NODE without one (and for padding slots).
__device__ __forceinline__ uint32_t node_code(int32_t d) {
  return (d >= 0 && d <= 9) ? (uint32_t)d : CODE_NONE_NODE;
}

// ---------------------------------------------------------------------------------------
// Stage 1, node side: the bit planes (msh_internal.h PLANE_*), once per upload / filter-list change.
// One thread per node; per 64-node wave the six ballots (code bits, X, V) are the planes of two words,
// written by 12 lanes. O(N), a few microseconds; nothing here depends on a pod.
// ---------------------------------------------------------------------------------------
constexpr int PREP_THREADS = 1024;  // n_pad is a multiple of 1024: every block is whole
__global__ __launch_bounds__(PREP_THREADS) void node_prep_kernel(const uint8_t* __restrict__ unsched,
                                                                 const int8_t* __restrict__ digit,
                                                                 int32_t n, int32_t has_nu,
                                                                 uint32_t* __restrict__ planes) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const bool valid = i < n;
  const bool x = valid && has_nu && unsched[i] != 0;
  const uint32_t code = valid ? node_code(digit[i]) : CODE_NONE_NODE;
  const unsigned long long pm[PLANE_N] = {__ballot(code & 1u), __ballot(code & 2u), __ballot(code & 4u),
                                          __ballot(code & 8u), __ballot(x), __ballot(valid)};
  // this wave's 64 nodes are words 2t and 2t + 1 of the PLANE_* layout: lanes 0..11 write them
  if (lane < 2 * PLANE_N) {
    const int k = lane >> 1, half = lane & 1;
    unsigned long long m = pm[0];
#pragma unroll
    for (int q = 1; q < PLANE_N; ++q) m = (k == q) ? pm[q] : m;
    const uint32_t word = ((uint32_t)(i - lane) >> 5) + (uint32_t)half;  // i - lane: the wave's first node
    planes[((word / PLANE_GW) * PLANE_N + k) * PLANE_GW + word % PLANE_GW] = (uint32_t)(m >> (32 * half));
  }
}

hipError_t launch_node_prep(const uint8_t* d_unsched, const int8_t* d_digit, int32_t n, int32_t n_pad,
                            int32_t has_nu, uint32_t* d_planes, hipStream_t s) {
  if (n_pad == 0) return hipSuccess;
  hipLaunchKernelGGL(node_prep_kernel, dim3(n_pad / PREP_THREADS), dim3(PREP_THREADS), 0, s, d_unsched, d_digit, n,
                     has_nu, d_planes);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// A table rewrite builds the unpublished version from the published one (msh_capi.cpp rewrite): one
// thread per 32-node word copies the word's uploaded columns (32 + 32 bytes) and its six plane words.
// msh_patch_nodes (an informer Update, eventhandler.go:45-65) rides on the same launch when it changes at
// most PATCH_INLINE nodes: their entries (idx | unsched << 32 | (uint8)digit << 40) travel in the kernel
// arguments, and the thread of a word that holds one writes the patched bytes and rebuilds the word's
// planes from them instead of copying. A cordon flip is then one launch, O(N / 32) threads of a few
// loads each, and no O(N) prep. Larger patches scatter their entries after the copy and re-run the prep.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void table_copy_kernel(TableCopyArgs a) {
  const int32_t w = (int32_t)(blockIdx.x * 256 + threadIdx.x);
  if (w >= a.n_words) return;
  const size_t g = (size_t)(w / PLANE_GW) * GROUP_DWORDS + w % PLANE_GW;  // plane 0 of word w
  bool patched = false;
  for (int e = 0; e < a.count; ++e) patched = patched || (int32_t)((uint32_t)a.inl[e] >> 5) == w;
  const uint4* su = reinterpret_cast<const uint4*>(a.src_unsched) + 2 * w;
  const uint4* sd = reinterpret_cast<const uint4*>(a.src_digit) + 2 * w;
  uint4* du = reinterpret_cast<uint4*>(a.dst_unsched) + 2 * w;
  uint4* dd = reinterpret_cast<uint4*>(a.dst_digit) + 2 * w;
  if (!patched) {
    du[0] = su[0];
    du[1] = su[1];
    dd[0] = sd[0];
    dd[1] = sd[1];
#pragma unroll
    for (int k = 0; k < PLANE_N; ++k) a.dst_planes[g + k * PLANE_GW] = a.src_planes[g + k * PLANE_GW];
    return;
  }
  // the word's 32 unsched and 32 digit bytes as 8 + 8 dwords (compile-time indices throughout: no
  // scratch), the entries of this word overlaid, the planes rebuilt
  uint32_t uw[8], dw[8];
  {
    const uint4 u0 = su[0], u1 = su[1], d0 = sd[0], d1 = sd[1];
    uw[0] = u0.x; uw[1] = u0.y; uw[2] = u0.z; uw[3] = u0.w; uw[4] = u1.x; uw[5] = u1.y; uw[6] = u1.z; uw[7] = u1.w;
    dw[0] = d0.x; dw[1] = d0.y; dw[2] = d0.z; dw[3] = d0.w; dw[4] = d1.x; dw[5] = d1.y; dw[6] = d1.z; dw[7] = d1.w;
  }
  for (int e = 0; e < a.count; ++e) {
    const unsigned long long x = a.inl[e];
    const uint32_t i = (uint32_t)x;
    if ((int32_t)(i >> 5) != w) continue;
    const uint32_t q = (i & 31u) >> 2, sh = (i & 3u) * 8u, keep = ~(0xFFu << sh);
    const uint32_t nu = (uint32_t)(uint8_t)(x >> 32) << sh, nd = (uint32_t)(uint8_t)(x >> 40) << sh;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uw[k] = (uint32_t)k == q ? (uw[k] & keep) | nu : uw[k];
      dw[k] = (uint32_t)k == q ? (dw[k] & keep) | nd : dw[k];
    }
  }
  uint32_t pl[PLANE_N] = {};
#pragma unroll
  for (int b = 0; b < 32; ++b) {
    const bool real = w * 32 + b < a.n;
    const uint32_t code = real ? node_code((int8_t)(uint8_t)(dw[b >> 2] >> (8 * (b & 3)))) : CODE_NONE_NODE;
    const uint32_t bit = 1u << b;
#pragma unroll
    for (int k = 0; k < 4; ++k) pl[k] |= ((code >> k) & 1u) ? bit : 0u;
    pl[PLANE_X] |= (real && a.has_nu && ((uw[b >> 2] >> (8 * (b & 3))) & 0xFFu)) ? bit : 0u;
    pl[PLANE_V] |= real ? bit : 0u;
  }
  du[0] = make_uint4(uw[0], uw[1], uw[2], uw[3]);
  du[1] = make_uint4(uw[4], uw[5], uw[6], uw[7]);
  dd[0] = make_uint4(dw[0], dw[1], dw[2], dw[3]);
  dd[1] = make_uint4(dw[4], dw[5], dw[6], dw[7]);
#pragma unroll
  for (int k = 0; k < PLANE_N; ++k) a.dst_planes[g + k * PLANE_GW] = pl[k];
}

hipError_t launch_table_copy(const TableCopyArgs& a, hipStream_t s) {
  if (a.n_words <= 0) return hipSuccess;
  if (a.count < 0 || a.count > PATCH_INLINE) return hipErrorInvalidValue;
  hipLaunchKernelGGL(table_copy_kernel, dim3((a.n_words + 255) / 256), dim3(256), 0, s, a);
  return hipGetLastError();
}

// A patch of more than PATCH_INLINE nodes: its entries scattered into the copied columns (the prep
// re-runs after it).
__global__ __launch_bounds__(256) void patch_scatter_kernel(const unsigned long long* __restrict__ entries,
                                                            int32_t count, uint8_t* __restrict__ unsched,
                                                            int8_t* __restrict__ digit) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const unsigned long long e = entries[i];
  const uint32_t k = (uint32_t)e;
  unsched[k] = (uint8_t)(e >> 32);
  digit[k] = (int8_t)(uint8_t)(e >> 40);
}

hipError_t launch_patch_scatter(const unsigned long long* d_entries, int32_t count, uint8_t* d_unsched,
                                int8_t* d_digit, hipStream_t s) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(patch_scatter_kernel, dim3((count + 255) / 256), dim3(256), 0, s, d_entries, count, d_unsched,
                     d_digit);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Node-sharded mode: decode the merged per-pod shard keys (after the element-wise MAX across shards).
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void decode_keys_kernel(const int8_t* __restrict__ pod_digit, int32_t p,
                                                          const int32_t* __restrict__ keys, PluginParams pp,
                                                          int32_t* __restrict__ out_idx,
                                                          int64_t* __restrict__ out_score,
                                                          int32_t* __restrict__ out_status) {
  const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= p) return;
  // slot 0: the pod's first feasible match; slot 1: its first feasible non-match
  const int32_t k0 = keys[j], k1 = keys[(size_t)p + j];
  const int32_t ka = k0 > k1 ? k0 : k1;  // the first feasible node
  auto idx_of = [](int32_t k) -> int64_t { return k ? (int64_t)(GKEY_MAX - k) : -1; };
  const int d = pod_digit[j];
  int32_t oi, ost;
  int64_t osc;
  decode_pod(idx_of(k0), idx_of(k1), idx_of(ka), d >= 0 && d <= 9, pp, &oi, &osc, &ost);
  out_idx[j] = oi;
  if (out_score) out_score[j] = osc;  // optional output
  out_status[j] = ost;
}

hipError_t launch_decode_keys(const int8_t* pod_digit, int32_t p, const int32_t* keys, PluginParams pp,
                              int32_t* out_idx, int64_t* out_score, int32_t* out_status, hipStream_t s) {
  if (p == 0) return hipSuccess;
  hipLaunchKernelGGL(decode_keys_kernel, dim3((p + 255) / 256), dim3(256), 0, s, pod_digit, p, keys, pp, out_idx,
                     out_score, out_status);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Device groups (msh_group_*): the cross-shard merge on the home device. Every shard's per-pod result
// stays in its own HBM; one thread per pod loads it from each shard through the peer mapping (xGMI reads,
// coalesced: consecutive pods, consecutive addresses), merges, and decodes. The merge replaces the
// all-reduce of the one-process-per-GPU form; the reduction is the same (MAX of the keys / extents; MAX
// total then MIN index), so the decisions are the same.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void group_keys_decode_kernel(GroupPtrs g, const int8_t* __restrict__ pod_digit,
                                                                int32_t p, PluginParams pp,
                                                                int32_t* __restrict__ out_idx,
                                                                int64_t* __restrict__ out_score,
                                                                int32_t* __restrict__ out_status) {
  const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= p) return;
  int32_t k0 = 0, k1 = 0;  // 0 = no node (every real key is positive)
  for (int s = 0; s < g.n; ++s) {
    const int32_t* k = g.keys[s];
    k0 = max(k0, k[j]);
    k1 = max(k1, k[(size_t)p + j]);
  }
  const int32_t ka = k0 > k1 ? k0 : k1;
  auto idx_of = [](int32_t k) -> int64_t { return k ? (int64_t)(GKEY_MAX - k) : -1; };
  const int d = pod_digit[j];
  int32_t oi, ost;
  int64_t osc;
  decode_pod(idx_of(k0), idx_of(k1), idx_of(ka), d >= 0 && d <= 9, pp, &oi, &osc, &ost);
  out_idx[j] = oi;
  if (out_score) out_score[j] = osc;
  out_status[j] = ost;
}

__global__ __launch_bounds__(256) void group_max_i64_kernel(GroupPtrs g, int64_t len, int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= len) return;
  int64_t m = INT64_MIN;
  for (int s = 0; s < g.n; ++s) m = max(m, g.v[s][i]);
  out[i] = m;
}

// Per pod: the largest total over the shards, the lowest global index among the shards that hold it
// (selectHost's first maximum across shards); INT64_MIN / INT32_MAX when no shard has a feasible node.
__global__ __launch_bounds__(256) void group_best_merge_kernel(GroupPtrs g, int32_t p, int64_t* __restrict__ out_total,
                                                               int32_t* __restrict__ out_idx) {
  const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= p) return;
  int64_t best = INT64_MIN;
  int32_t bi = INT32_MAX;
  for (int s = 0; s < g.n; ++s) {
    const int32_t i = g.idx[s][j];
    const int64_t t = g.v[s][j];
    if (i != INT32_MAX && (bi == INT32_MAX || t > best || (t == best && i < bi))) {
      best = t;
      bi = i;
    }
  }
  out_total[j] = best;
  out_idx[j] = bi;
}

hipError_t launch_group_keys_decode(const GroupPtrs& g, const int8_t* pod_digit, int32_t p, PluginParams pp,
                                    int32_t* out_idx, int64_t* out_score, int32_t* out_status, hipStream_t s) {
  if (p <= 0) return hipSuccess;
  if (g.n < 1 || g.n > GROUP_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(group_keys_decode_kernel, dim3((p + 255) / 256), dim3(256), 0, s, g, pod_digit, p, pp, out_idx,
                     out_score, out_status);
  return hipGetLastError();
}

hipError_t launch_group_max_i64(const GroupPtrs& g, int64_t len, int64_t* out, hipStream_t s) {
  if (len <= 0) return hipSuccess;
  if (g.n < 1 || g.n > GROUP_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(group_max_i64_kernel, dim3((unsigned)((len + 255) / 256)), dim3(256), 0, s, g, len, out);
  return hipGetLastError();
}

hipError_t launch_group_best_merge(const GroupPtrs& g, int32_t p, int64_t* out_total, int32_t* out_idx,
                                   hipStream_t s) {
  if (p <= 0) return hipSuccess;
  if (g.n < 1 || g.n > GROUP_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(group_best_merge_kernel, dim3((p + 255) / 256), dim3(256), 0, s, g, p, out_total, out_idx);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Per-pair plugin results (debug / simulator result store). One workgroup per pod:
// pass 1 ORs "feasible match" / "feasible non-match" over the List to get the extent NormalizeScore
// needs; pass 2 writes, for every node i,
//   filter[i] = 1 passed / 0 rejected by NodeUnschedulable,
//   raw[i]    = NodeNumber.Score (10 on a digit match, else 0),
//   final[i]  = NormalizeScore(raw)[i] * weight,
// with raw/final = EXPORT_NONE where the reference records no score (infeasible node, or the pod never
// reaches Score: no feasible node / PreScore failed / no score plugin). Not a hot path: O(P*N) writes of
// 17 B per pair.
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
        case 1: o = m ? 100 : 0; break;                     // max is 10 whenever a match exists
        case 2: o = hm ? (m ? 0 : 100) : 100; break;        // reverse; max 0 -> all 100
        case 3: o = (hm && hx) ? (m ? 100 : 0) : 0; break;  // min-max; max == min -> 0
        default: o = r; break;
      }
      o *= w;
    }
    raw[row + i] = r;
    fin[row + i] = o;
  }
}

hipError_t launch_export(const uint8_t* d_unsched, const int8_t* d_digit, int32_t n, const int8_t* d_pod_digit,
                         const uint8_t* d_pod_tol, int32_t p, const PluginParams& pp, uint8_t* d_filter,
                         int64_t* d_raw, int64_t* d_fin, hipStream_t s) {
  if (p <= 0 || n <= 0) return hipSuccess;
  hipLaunchKernelGGL(export_kernel, dim3(p), dim3(256), 0, s, d_unsched, d_digit, n, d_pod_digit, d_pod_tol, pp,
                     d_filter, d_raw, d_fin);
  return hipGetLastError();
}

}  // namespace msh
