// msh_device.h — device-side helpers shared by the gfx950 kernel translation units (msh_prep.hip,
// msh_pair.hip, msh_generic.hip, msh_seq.hip). Not part of the public ABI.
#pragma once

#include "msh_internal.h"

#include <hip/hip_ext.h>

#include <type_traits>

namespace msh {

// Kernel start / stop events for the next hot-kernel launch on this thread (msh_timing_begin, defined in
// msh_prep.hip): hipExtLaunchKernelGGL records them at the kernel's own start and completion, the
// interval rocprofv3's kernel trace reports, not around the launch like events recorded on the stream.
extern thread_local hipEvent_t t_ev_start, t_ev_stop;
#define MSH_TIMED_LAUNCH(kern, grid, block, lds, stream, ...)                                                   \
  do {                                                                                                          \
    if (::msh::t_ev_start) {                                                                                    \
      hipExtLaunchKernelGGL(kern, grid, block, lds, stream, ::msh::t_ev_start, ::msh::t_ev_stop, 0, __VA_ARGS__); \
      ::msh::t_ev_start = ::msh::t_ev_stop = nullptr;                                                           \
    } else {                                                                                                    \
      hipLaunchKernelGGL(kern, grid, block, lds, stream, __VA_ARGS__);                                          \
    }                                                                                                           \
  } while (0)

__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

// ---------------------------------------------------------------------------------------
// Stages 2-5 epilogue of the bit-plane kernels: status / selected node / int64 score for one pod.
// im / ix / ia: first feasible match / first feasible non-match / first feasible node (node index,
// -1 = none). ix is only read by the modes that need it (needs_kx).
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

// decode_pod for the identity-like modes (NONE, DEFAULT: everything that does not need the first
// feasible non-match), as selects on launch-constant flags instead of a branch per mode.
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
  const bool fit = ia < 0;                                                  // FitError (minisched.go:143)
  const bool serr = !fit && (d.err_all || (d.err_nodigit && !pd_valid));  // Score error (nodenumber.go:74-77)
  const bool hit = d.use_im && im >= 0;
  *out_status = fit ? 1 : (serr ? 2 : 0);
  *out_idx = (fit || serr) ? -1 : (int32_t)(hit ? im : ia);
  *out_score = (fit || serr || !hit) ? 0 : d.sm;
}

// Shard keys (int32): GKEY_MAX - global node index, 0 = none.
__device__ __forceinline__ int32_t shard_key(int64_t node_base, uint32_t local_idx) {
  return GKEY_MAX - (int32_t)(node_base + (int64_t)local_idx);
}

constexpr uint32_t NO_GROUP = 0xFFFFFFFFu;

// v_ffbl_b32: the lowest set bit, all-ones for 0 (ctz's 0 is UB)
__device__ __forceinline__ uint32_t lowbit(uint32_t x) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
// The first node among 8 hit words of group g (words ascend in List order, bits within a word):
// each word's lowest set bit (all-ones for an empty word, which ORed with the word's offset 32 c stays
// all-ones); the unsigned minimum over the words is the first hit. The group must hold a hit.
__device__ __forceinline__ uint32_t hits_first(const uint32_t (&h)[PLANE_GW], uint32_t g) {
  uint32_t t[PLANE_GW];
#pragma unroll
  for (int c = 0; c < PLANE_GW; ++c) t[c] = lowbit(h[c]) | (uint32_t)(32 * c);
  const uint32_t m = umin(umin(umin(t[0], t[1]), umin(t[2], t[3])), umin(umin(t[4], t[5]), umin(t[6], t[7])));
  return g * GROUP_NODES + m;
}

// v_bitop3_b32 forms (the builtin, not inline asm: the backend then knows the instruction's hazards;
// after inline asm it inserts an s_nop every other VALU)
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
__device__ __forceinline__ uint32_t bop3_or_xor(uint32_t t, uint32_t d, uint32_t p) {  // t | (d ^ p)
  return __builtin_amdgcn_bitop3_b32(t, d, p, 0xf6);
}
__device__ __forceinline__ uint32_t bop3_andn_of_and(uint32_t k, uint32_t x, uint32_t m) {  // k & ~(x & m)
  return __builtin_amdgcn_bitop3_b32(k, x, m, 0x70);
}
__device__ __forceinline__ uint32_t bop3_or_and(uint32_t k, uint32_t x, uint32_t m) {  // k | (x & m)
  return __builtin_amdgcn_bitop3_b32(k, x, m, 0xf8);
}

typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

}  // namespace msh
