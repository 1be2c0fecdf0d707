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
constexpr int WAVE = 64;
constexpr int32_t GKEY_MAX = 0x7FFFFFFF;         // global (sharded) int32 key = GKEY_MAX - global_idx
constexpr uint32_t NOFIT = 0x80000000u;          // "no node" as a node index (above every real one)

// Per-ctx plugin set as the kernels see it (minisched/initialize.go:80-123 lists).
struct PluginParams {
  int32_t has_nu_filter;  // "NodeUnschedulable" in filter list
  int32_t has_nn_score;   // "NodeNumber" in score list
  int32_t nn_prescore;    // "NodeNumber" in prescore list (state written)
  int32_t mode;           // NodeNumber normalize mode (msh_normalize)
  int64_t weight;         // NodeNumber weight
};

// Whether the argmax needs the "first feasible NON-match" per pod (reverse / min-max
// normalization); otherwise the first feasible node of the pod's class suffices.
inline bool needs_kx(const PluginParams& pp) {
  return pp.has_nn_score && pp.nn_prescore && (pp.mode == 2 || pp.mode == 3);
}

// Device facts and launch choices, resolved once in msh_create (never on the launch path).
struct DeviceInfo {
  int cus = 256;
  int bits_slices = 0;   // tests / A-B only (MSH_BITS_SLICES at msh_create): slice waves per pod block, 0 = auto
  int seq_waves = 0;     // tests / A-B only (MSH_SEQ_WAVES at msh_create): sequential scanning waves, 0 = auto
  int rows_ppl = 1;      // pods per lane of the digit-row kernel (1 or 2; MSH_ROWS_PPL at msh_create, A/B)
  int kx_bits = 0;       // A/B only (MSH_KX_BITS=1 at msh_create): REVERSE / MINMAX on the code-plane kernel
  // Host-buffer calls (msh_schedule_batch / _sequential): the kernel reads the pod columns from and
  // writes the outputs to page-locked host memory (default). A/B only, MSH_HOST_IO at msh_create:
  // "dma" = columns and outputs DMA'd through device scratch, "zc" = columns DMA'd, outputs zero-copy.
  int host_io_dma = 0;
  int host_io_zc_in = 1;
  int host_sync_poll = 0;  // A/B only (MSH_HOST_SYNC=poll): poll an event instead of hipStreamSynchronize
  int batch_kernel = 0;    // 0 = wg_kernel (default), 1 = the round-2 slice kernel rows_kernel (MSH_BATCH_KERNEL=slices,
                           // A/B), 2 = generic_kernel for every plugin list (MSH_BATCH_KERNEL=generic, A/B)
  int wg_waves = 0;        // A/B only (MSH_WG_WAVES=1|2|4|8): waves per workgroup of wg_kernel, 0 = auto
  int wg_no_persist = 0;   // A/B only (MSH_WG_PERSIST=0): multi-batch launches on the 2-D wg_kernel grid
};

// NodeNumber codes: a node's suffix digit 0..9, or CODE_NONE_NODE when its name has no digit
// suffix (and for padding slots); a pod's digit, or CODE_NONE_POD. The two "none" codes differ
// from each other and from every digit, so they never match.
constexpr uint32_t CODE_NONE_NODE = 15u;
constexpr uint32_t CODE_NONE_POD = 14u;

// Bit-sliced node table (the input of every batch / sequential kernel). Node i is bit (i mod 32)
// of word i / 32; words come in groups of PLANE_GW (256 nodes), and a group holds PLANE_N planes
// of PLANE_GW words each, plane-major, so one scalar load brings one plane of a whole group:
//   planes[(g * PLANE_N + k) * PLANE_GW + j] = plane k of word g * PLANE_GW + j
//   k = 0..3  bit k of the node's NodeNumber code (digit 0..9, or 15: no digit / padding)
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
constexpr int32_t NODE_PAD = 1024;  // tables are padded to whole 1,024-node prep blocks (4 groups)

// Digit rows (a bitmap index on NodeNumber's node digit; the input of the identity-mode batch
// kernel): for every word, ER_ROWS row words, row r = the word's real nodes whose suffix digit is
// r (r = 0..9); row 10 stays zero (the row of pods without a digit suffix). Per group, two chunks
// of 4 consecutive words, each chunk row-major with a row's 4 words contiguous, then the group's 8
// X words (the PLANE_X plane again, so that one copy brings a group's whole input):
//   erows[g * ER_GD + (c * ER_ROWS + r) * 4 + k] = row r of word g * PLANE_GW + 4 c + k
//   erows[g * ER_GD + ER_Q * 4 + j]              = X of word g * PLANE_GW + j
// so a pod's row words of one chunk are one 16-byte read, and the 11 rows of a chunk (44 dwords)
// sit in distinct LDS banks. 1.5 B per node. (The REVERSE / MINMAX modes also read the V plane,
// from the code planes.)
constexpr int ER_ROWS = 11;
constexpr int ER_Q = 2 * ER_ROWS;      // 16-byte row chunks per group
constexpr int ER_GQ = ER_Q + 2;        // 16-byte chunks per group: the rows, then X
constexpr int ER_GD = ER_GQ * 4;       // dwords per group
constexpr int ER_TG = 8;               // groups per LDS tile of the batch kernel (3,072 B per wave)

// Class rows (the input of the persistent batch kernel): the digit rows with the filter folded in per
// pod class, t = 0 (does not tolerate the unschedulable taint) and t = 1 (tolerates), so that a pod's
// hit words are one row read, H[t][r] = the word's nodes that pass NodeUnschedulable for class t AND
// have suffix digit r (row 10 zero); then F[t] = the word's nodes feasible for class t (the REVERSE /
// MINMAX modes' non-matches are F[t] & ~H[t][r]). Per group 48 16-byte entries: H[t][r] of chunk c
// (words 4 c .. 4 c + 3 of the group) is entry hr_entry(c, t, r), F[t] entries HR_F + 2 t (words 0-3)
// and HR_F + 2 t + 1 (words 4-7):
//   hrows[g * HR_GD + hr_entry(c, t, r) * 4 + k] = H[t][r] of word g * PLANE_GW + 4 c + k
//   hrows[g * HR_GD + (HR_F + 2 t) * 4 + j]      = F[t] of word g * PLANE_GW + j
// 3 B per node; a pod reads 32 B per 256-node group (two 16-byte entries), half of the digit rows + X.
// The order is LDS-bank aware: the lanes of one ds_read_b128 are served in groups of 16, each lane's
// 16 B from bank slot (entry mod 16) (MI355X_MICROARCH.md, LDS), so two lanes of a group that read
// different entries of one slot cost an extra LDS cycle. A scan instruction reads chunk 0 (or chunk 1)
// for every lane: the 11 non-tolerating rows of a chunk take 11 slots and the tolerating rows the
// other 5, tolerating rows 0-4 and 5-9 sharing them (a conflict needs two tolerating pods of different
// rows in one 16-lane group); row 10 (pods without a digit suffix) of the tolerating class shares a
// slot with a rare non-tolerating row. Rows [slot]:
//   entries  0-15: chunk 0: t=0 r=0..10 [0..10], t=1 r=0..4 [11..15]
//   entries 16-31: chunk 1: t=1 r=0..4 [0..4], t=0 r=0..10 [5..15]
//   entries 32-47: chunk 1 t=1 r=5..9 [0..4], F[0] F[1] [5..8], chunk 1 t=1 r=10 [9],
//                  chunk 0 t=1 r=10 [10], chunk 0 t=1 r=5..9 [11..15]
// (with conflicting class rows, 16-lane groups holding a tolerating pod made the C3 scan ~10% slower,
// profiles/ab/r3_wgp_ab.jsonl).
// After the 48 row entries, 6 entries (48 uint16) of first-node offsets, written by hr_first_kernel
// after each prep: [cls] = the first node of the group in H[t][r] (cls = 11 t + r), [24 + cls] = the
// first in F[t] & ~H[t][r], as an offset 0..255, HR_NONE when the group has none. The batch kernel
// resolves a pod's exact node from them once its scan has found the first pair of groups with a hit.
// The group stride (54 entries) shifts every entry of a group by the same slot: no new conflicts.
constexpr int HR_ROWQ = 48;            // 16-byte row entries per group
constexpr int HR_FIRST = HR_ROWQ;      // first-node offsets (uint16) at entries 48-53
constexpr int HR_CLS = 24;             // offsets per kind (22 pod classes, padded)
constexpr int HR_GQ = HR_ROWQ + 6;     // 16-byte entries per group
constexpr int HR_GD = HR_GQ * 4;       // dwords per group
constexpr int HR_F = 37;               // F[0] at entries 37-38, F[1] at 39-40
constexpr uint16_t HR_NONE = 0xFFFF;
__host__ __device__ constexpr uint32_t hr_entry(uint32_t c, uint32_t t, uint32_t r) {
  return t == 0 ? (c == 0 ? r : 21 + r)
                : r < 5 ? (c == 0 ? 11 + r : 16 + r) : r < 10 ? (c == 0 ? 38 + r : 27 + r) : (c == 0 ? 42u : 41u);
}
constexpr int ER_PAD = 2 * ER_TG;      // groups of padding: whole-tile copies need no clamp

// ---- launchers (msh_kernels.hip) ----
// Applies `patch_count` pending msh_patch_nodes entries (idx | unsched << 32 | (uint8)digit << 40)
// to the raw columns, then rebuilds the planes and the first feasible node per class (ball).
hipError_t launch_node_prep(const uint8_t* d_unsched, const int8_t* d_digit, int32_t n, int32_t n_pad,
                            int32_t has_nu, uint32_t* d_ball, uint32_t* d_planes, uint32_t* d_erows,
                            uint32_t* d_hrows, hipStream_t s,
                            const unsigned long long* d_patch = nullptr, int32_t patch_count = 0);

constexpr int64_t EXPORT_NONE = INT64_MIN;  // msh_export_results: no score recorded
hipError_t launch_export(const uint8_t* d_unsched, const int8_t* d_digit, int32_t n,
                         const int8_t* d_pod_digit, const uint8_t* d_pod_tol, int32_t p,
                         const PluginParams& pp, uint8_t* d_filter, int64_t* d_raw, int64_t* d_fin,
                         hipStream_t s);

struct BatchArgs {
  const uint32_t* planes;    // bit-sliced node table, n_groups groups
  const uint32_t* erows;     // digit rows (ER_* layout), n_groups groups
  const uint32_t* hrows;     // class rows (HR_* layout), n_groups groups
  int32_t n_groups;          // n_pad / GROUP_NODES
  int32_t gps;               // groups per slice wave (set by the launcher)
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
};

hipError_t launch_batch(const BatchArgs& a, bool shard, const DeviceInfo& dev, hipStream_t s);

// One batch of a multi-batch launch (msh_schedule_batches_device): its own pod columns and
// outputs. The launch grid is 2-D: blockIdx.y = the batch, blockIdx.x = the pod block within it
// (the x extent is the largest batch's; a workgroup past its batch's end exits at once).
struct BatchDesc {
  const int8_t* pod_digit;
  const uint8_t* pod_tol;
  int32_t* out_idx;
  int64_t* out_score;  // may be null
  int32_t* out_status;
  int32_t n_pods;
  int32_t reserved;
};
constexpr int RANK_MAX = 8;     // persistent kernel: workgroups per CU (age slots)
constexpr int MULTI_MAX = 32;  // batches per launch (kernel-argument descriptors, 48 B each: ~1.7 KB)
struct MultiArgs {
  BatchArgs a;  // the node table, plugin set and launch geometry (its pod / output fields unused)
  int32_t nb;
  int32_t bpb;  // pod blocks per batch (the largest batch's), set by the launcher
  // persistent kernel: walk 0 = strided items (g, g + G, ...); walk 1 = workgroup g (age slot
  // r = g / rank_wgs on its CU) owns a share of the item range [rank_lo[r], rank_lo[r + 1]), split
  // evenly over the rank_wgs workgroups of the slot
  int32_t walk;
  int32_t rank_wgs;
  int32_t rank_lo[RANK_MAX + 1];
  BatchDesc d[MULTI_MAX];
};

// nb (1..MULTI_MAX) independent batches of device-resident pods in ONE launch of the workgroup
// kernel. `a` carries the table and plugin set.
hipError_t launch_batches(const BatchArgs& a, const BatchDesc* d, int nb, const DeviceInfo& dev, hipStream_t s);

hipError_t launch_decode_keys(const int8_t* pod_digit, const uint8_t* pod_tol, int32_t p,
                              const int32_t* keys, int32_t slot1_any, PluginParams pp,
                              int32_t* out_idx, int64_t* out_score, int32_t* out_status,
                              hipStream_t s);

// ---- generic score pipeline (any score plugin list; generic_kernel) ----
constexpr int GEN_MAX_SCORE = 5;  // score plugins per list: NodeNumber + up to four score columns
constexpr int GEN_COLS = 4;       // score-column plugins MSH_PLUGIN_SCORE_COLUMN0..3
struct GenericArgs {
  const uint8_t* unsched;  // the uploaded columns, List order
  const int8_t* digit;
  const int64_t* cols;     // GEN_COLS x col_stride int64: column k at cols + k * col_stride
  int64_t col_stride;
  int32_t n_nodes;
  int32_t has_nu;          // NodeUnschedulable in the filter list
  int32_t nn_prescore;     // NodeNumber in the prescore list
  int32_t nn_score;        // NodeNumber in the score list
  int32_t ns;              // score plugins
  int32_t need_ext;        // some plugin normalizes: the extent pass runs
  int32_t kind[GEN_MAX_SCORE];   // 0 = NodeNumber, 1 + k = score column k
  int32_t mode[GEN_MAX_SCORE];   // msh_normalize
  int64_t weight[GEN_MAX_SCORE];
  const int8_t* pod_digit;
  const uint8_t* pod_tol;
  int32_t n_pods;
  int32_t* out_idx;
  int64_t* out_score;      // may be null
  int32_t* out_status;
};
hipError_t launch_generic(const GenericArgs& a, hipStream_t s);

struct SeqArgs {
  const uint32_t* planes;    // bit-sliced node table (PLANE_* layout)
  int32_t n_words;           // n_pad / 32
  const uint32_t* ball;      // [2] first feasible key per pod class (no capacity: constant)
  int32_t n_nodes;
  const int8_t* pod_digit;
  const uint8_t* pod_tol;
  int32_t n_pods;
  PluginParams pp;
  int32_t max_pods;
  int32_t* counts;           // [n_pad] per-node assigned pods (read at start, updated)
  int32_t* out_idx;
  int64_t* out_score;
  int32_t* out_status;
};

hipError_t launch_sequential(const SeqArgs& a, const DeviceInfo& dev, hipStream_t s, std::string* err);

// Launch timing (msh_timing_begin / _end): the next hot-kernel launch on this thread (batch, multi-
// batch, generic, sequential kernels) records `start` / `stop` at the kernel's own start and end.
void set_launch_events(hipEvent_t start, hipEvent_t stop);
bool launch_events_pending();

}  // namespace msh
