// msh_internal.h — shared between the C-ABI (msh_capi.cpp) and the gfx950 kernels
// (msh_kernels.hip). Not part of the public ABI (include/minisched_hip.h is).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace msh {

// Local node key: KMAX - node_index (> 0 for every valid index), 0 = "no node".
// A larger key is a smaller index, so an unsigned max is the reference's first-max scan
// order (selectHost, minisched.go:304-325, with the deterministic tie-break).
constexpr uint32_t KMAX = 0xFFFFFFu;
constexpr int32_t MAX_NODES = 0xFFFFFE;          // node index must stay < KMAX
constexpr uint32_t DIGIT_NONE = 0xFFu;           // node suffix is not '0'..'9'
constexpr uint32_t POD_DIGIT_NONE = 0xFEu;       // never equals a node digit (0..9 / 0xFF)
constexpr int WAVE = 64;
constexpr int BATCH_THREADS = 256;               // 4 waves per workgroup
constexpr int32_t GKEY_MAX = 0x7FFFFFFF;         // global (sharded) int32 key = GKEY_MAX - global_idx
// Node "cost" for the first-match search: idx if the node is feasible for the pod class,
// NOFIT otherwise. cost + |D - pd| * 2^24 (one v_sad_u32) is < 2^24 exactly for feasible
// nodes whose digit equals the pod's; its unsigned min is the first such node in List order.
constexpr uint32_t NOFIT = 0x80000000u;
constexpr uint32_t MATCH_LIMIT = 1u << 24;

// Per-ctx plugin set as the kernels see it (minisched/initialize.go:80-123 lists).
struct PluginParams {
  int32_t has_nu_filter;  // "NodeUnschedulable" in filter list
  int32_t has_nn_score;   // "NodeNumber" in score list
  int32_t nn_prescore;    // "NodeNumber" in prescore list (state written)
  int32_t mode;           // NodeNumber normalize mode (msh_normalize)
  int64_t weight;         // NodeNumber weight
};

// Whether the argmax needs the "first feasible NON-match" key per pod (reverse / min-max
// normalization); otherwise the first feasible node of the pod's class suffices.
inline bool needs_kx(const PluginParams& pp) {
  return pp.has_nn_score && pp.nn_prescore && (pp.mode == 2 || pp.mode == 3);
}

// Device facts and launch choices, resolved once in msh_create (never on the launch path).
struct DeviceInfo {
  int cus = 256;
  int legacy_batch = 0;  // A/B only (MSH_BATCH_KERNEL=legacy at msh_create): the packed-16 kernels
  int bits_slices = 0;   // A/B only (MSH_BITS_SLICES at msh_create): slice waves per pod block, 0 = auto
};

// ---- launchers (msh_kernels.hip) ----
// Packed-16 first-match words (IDENT batch path): per node i (chunk c = i / 64, lane i % 64),
//   w16 = (code << CODE_SHIFT) | (c mod TILE_CHUNKS),  code = node digit if the node is feasible
//   for pods that do NOT tolerate the unschedulable taint (class 0) and its name ends in
//   '0'..'9', else 15 (never equals a pod code 0..9 or 14).
// With the 4-bit code in bits 10..13 and bits 14..15 zero, w16 ^ (pod code << 10) read as an
// f16 is a subnormal equal to the chunk exactly on a match and a finite normal number (exponent
// 1..15) otherwise, never inf or NaN: its f16 order is its integer order, so the IEEE
// v_pk_minimum3_f16 folds two node words per instruction.
// w0 holds w16 in both 16-bit halves, so one v_xor_b32 serves two pods. Within one lane the
// nodes are ordered by chunk, so the per-lane minimum only needs the chunk number; the lane
// is folded back in (chunk << 6 | lane = node index in the tile) before the cross-lane min.
// A compute tile is TILE_CHUNKS chunks (64,512 nodes: chunk < 1023 keeps chunk<<6|lane in 16
// bits). The only pairs whose feasibility differs for tolerating pods (class 1) are the nodes
// infeasible for class 0 but feasible for class 1 (the unschedulable ones): they are listed
// once in `ulist` as (code1 << 24) | idx, in any order (the search is a min), and scanned for
// tolerating pods only.
constexpr int TILE_CHUNKS = 1008;                 // 16 * 63
constexpr int TILE_NODES = TILE_CHUNKS * 64;
constexpr int STAGE_CHUNKS = TILE_CHUNKS / 3;     // LDS stage: 336 chunks = 86,016 B
constexpr uint32_t CODE_NONE_NODE = 15u;
constexpr int CODE_SHIFT = 10;                    // code bits 10..13 of a w16 half

// Position of node i's word in w0: 4-chunk groups of 256 words, lane-major inside a group
// (lane l's words for chunks 4g..4g+3 are contiguous: one 16-byte load per lane).
__host__ __device__ inline uint32_t word_pos(uint32_t i) {
  return (i & ~255u) | ((i & 63u) << 2) | ((i >> 6) & 3u);
}
constexpr uint32_t CODE_NONE_POD = 14u;

// Bit-sliced node table (the batch kernel's input). Node i is bit (i mod 32) of word i / 32;
// words come in groups of PLANE_GW (256 nodes), and a group holds PLANE_N planes of PLANE_GW
// words each, plane-major, so one scalar load brings one plane of a whole group:
//   planes[(g * PLANE_N + k) * PLANE_GW + j] = plane k of word g * PLANE_GW + j
//   k = 0..3  bit k of the node's NodeNumber code: its suffix digit 0..9, or 15 when the name
//             has no digit suffix or the slot is padding (15 never equals a pod code 0..9 / 14)
//   k = 4     X: NodeUnschedulable rejects the node for pods that do not tolerate the
//             unschedulable taint (Spec.Unschedulable with the filter in the list)
//   k = 5     V: the slot holds a real node (i < n), i.e. it is feasible for tolerating pods
// 0.75 B per node. A (pod, node) pair is a feasible digit match exactly when, in the node's bit,
//   (X & ~tol) | (D0 ^ P0) | (D1 ^ P1) | (D2 ^ P2) | (D3 ^ P3) == 0
// with P_k = all-ones when bit k of the pod's code is set.
constexpr int PLANE_GW = 8;
constexpr int PLANE_N = 6;
constexpr int PLANE_X = 4, PLANE_V = 5;
constexpr int GROUP_NODES = PLANE_GW * 32;
constexpr int GROUP_DWORDS = PLANE_GW * PLANE_N;

hipError_t launch_node_prep(const uint8_t* d_unsched, const int8_t* d_digit, int32_t n,
                            int32_t n_pad, int32_t has_nu, uint32_t* d_c0, uint8_t* d_dig,
                            uint32_t* d_w0, uint32_t* d_ulist, uint32_t* d_ucount,
                            unsigned long long* d_mask, uint32_t* d_ball, uint32_t* d_planes,
                            hipStream_t s, const unsigned long long* d_patch = nullptr,
                            int32_t patch_count = 0);

constexpr int64_t EXPORT_NONE = INT64_MIN;  // msh_export_results: no score recorded
hipError_t launch_export(const uint8_t* d_unsched, const int8_t* d_digit, int32_t n,
                         const int8_t* d_pod_digit, const uint8_t* d_pod_tol, int32_t p,
                         const PluginParams& pp, uint8_t* d_filter, int64_t* d_raw, int64_t* d_fin,
                         hipStream_t s);

// entries[k] = idx | unsched << 32 | (uint8)digit << 40


struct BatchArgs {
  const uint32_t* c0;        // [n_pad] class-0 node cost: idx if feasible for !tolerating pods, else NOFIT
  const uint8_t* dig;        // [n_pad] node digit 0..9 / 0xFF
  const uint32_t* w0;        // [n_pad] packed-16 class-0 word, duplicated in both halves
  const uint32_t* ulist;     // [ucount] (code1 << 24) | idx of class-0-infeasible, class-1-feasible nodes
  const uint32_t* ucount;    // device scalar
  int32_t n_nodes, n_chunks; // n_chunks = n_pad / 64
  const int8_t* pod_digit;
  const uint8_t* pod_tol;
  int32_t n_pods;
  const uint32_t* ball;      // [2] first feasible key per pod class (0: !tol, 1: tol)
  PluginParams pp;
  int32_t* out_idx;
  int64_t* out_score;
  int32_t* out_status;
  int32_t* keys;             // shard mode: [n_pods + slot-1 count] global keys (msh_shard_keys_len)
  int64_t node_base;
  uint32_t* partial;         // [2][n_pods] running keys when the node table spans > 1 LDS tile
  int32_t unit_q, unit_r;    // work-queue kernel: workgroup b owns unit_q (+1 if b < unit_r) units
  int32_t unit_w;            // wave-range kernel: wave count W (pairs = W * unit_q + unit_r)
  const uint32_t* planes;    // bit-sliced node table (PLANE_* layout), n_pad / GROUP_NODES groups
  int32_t n_groups;
  int32_t gps;               // bit-sliced kernel: groups per slice wave
};

// LDS tile geometry of the batched kernel (host needs it to size the partial-key scratch).
int32_t batch_tile_chunks(int32_t n_chunks);
bool batch_needs_partial(int32_t n_chunks);
// does the batch kernel launch_batch picks for these plugins keep running results in `partial`
// (a per-ctx scratch: such launches must not overlap on different streams)
bool batch_uses_partial(const PluginParams& pp, int32_t n_chunks, const DeviceInfo& dev);

hipError_t launch_batch(const BatchArgs& a, bool shard, const DeviceInfo& dev, hipStream_t s,
                        std::string* err);

hipError_t launch_decode_keys(const int8_t* pod_digit, const uint8_t* pod_tol, int32_t p,
                              const int32_t* keys, int32_t slot1_any, PluginParams pp,
                              int32_t* out_idx, int64_t* out_score, int32_t* out_status,
                              hipStream_t s);

struct SeqArgs {
  const uint32_t* c0;
  const uint8_t* dig;
  int32_t n_nodes, n_chunks;
  const int8_t* pod_digit;
  const uint8_t* pod_tol;
  int32_t n_pods;
  PluginParams pp;
  int32_t max_pods;
  int32_t* counts;           // [n_pad] per-node assigned pods (read at start, written back)
  int32_t* out_idx;
  int64_t* out_score;
  int32_t* out_status;
};

hipError_t launch_sequential(const SeqArgs& a, hipStream_t s, std::string* err);

}  // namespace msh
