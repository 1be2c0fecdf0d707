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
  int bits_slices = 0;   // tests / A-B only (MSH_BITS_SLICES at msh_create): pair_kernel slice waves per pod block
                         // (1, 2, 4), 0 = auto
  int seq_waves = 0;     // tests / A-B only (MSH_SEQ_WAVES at msh_create): sequential scanning waves, 0 = auto
  // Host-buffer calls (msh_schedule_batch / _sequential): the kernel reads the pod columns from and
  // writes the outputs to page-locked host memory (default). A/B only, MSH_HOST_IO at msh_create:
  // "dma" = columns and outputs DMA'd through device scratch, "zc" = columns DMA'd, outputs zero-copy.
  int host_io_dma = 0;
  int host_io_zc_in = 1;
  int host_sync_poll = 0;  // A/B only (MSH_HOST_SYNC=poll): poll an event instead of hipStreamSynchronize
  // Batch kernel (MSH_BATCH_KERNEL at msh_create): 0 = pair_kernel, the per-pair evaluation (default);
  // 1 = the class-row kernel wgp_kernel (opt-in "classrows": a pod's verdicts read from tables indexed
  // by its class, tables up to 8,192 nodes; larger tables and shard keys stay on pair_kernel);
  // 2 = generic_kernel for every plugin list ("generic", A/B)
  int batch_kernel = 0;
  // Where pair_kernel's node planes come from (MSH_PAIR_PLANES at msh_create): 0 = auto (LDS-staged
  // for tables up to PAIR_LDS_MAX_GROUPS groups and launches that fill the chip, scalar loads
  // otherwise), 1 = scalar loads into SGPRs, 2 = LDS-staged (tables that fit)
  int pair_planes = 0;
  int pair_lds_bpw = 2;  // A/B (MSH_PAIR_LDS_BPW): 64-pod blocks per wave of the LDS-staged form, 1-4
  // MSH_PAIR_COMPACT: the LDS-staged form (2 blocks per wave) reorders each workgroup's pods by their
  // tolerates bit first, so that most blocks scan with the filter term folded (1 = on)
  // (-1 = auto: on for REVERSE / MINMAX, where it measured 2% faster, off for the identity-like modes)
  int pair_compact = -1;
  // MSH_PAIR_HYBRID: the LDS-staged form reads a full group's X and D3 planes by scalar loads and
  // D0-D2 from LDS, 6 broadcast reads per group instead of 10 (1: per group, one wait each; 2: both
  // groups of a step under one wait; 0: off; A/B builds with D2 too from SGPRs, or compiler-
  // scheduled loads, measured slower / the same). -1 = auto: 1 for the
  // identity-like modes (81.1 against 86.1 us per 32-batch C3 launch), 2 for REVERSE / MINMAX (87.9
  // against 90.7 with 1), profiles/r4_ab_pair_planes.txt
  int pair_hybrid = -1;
  // MSH_PAIR_NOAX: the LDS-staged form scans group 0 first and drops the non-match / feasible
  // reduction from the scan of the other groups when group 0 has settled it for every lane of the
  // wave (1), or scans group 0 last and never drops it (0). -1 = auto: 1 for REVERSE / MINMAX (78.1
  // against 89.0 us per 32-batch C3 launch), 0 for the identity-like modes (77.3-78.3 against
  // 80.9-81.2), profiles/r4_ab_pair_planes.txt
  int pair_noax = -1;
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

// Row count of the class rows below: rows 0..9 = suffix digits, row 10 = pods without a digit.
constexpr int ER_ROWS = 11;

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

// ---- launchers (msh_kernels.hip) ----
// Applies `patch_count` pending msh_patch_nodes entries (idx | unsched << 32 | (uint8)digit << 40)
// to the raw columns, then rebuilds the planes and the first feasible node per class (ball).
hipError_t launch_node_prep(const uint8_t* d_unsched, const int8_t* d_digit, int32_t n, int32_t n_pad,
                            int32_t has_nu, uint32_t* d_ball, uint32_t* d_planes, uint32_t* d_hrows,
                            uint32_t* d_nrec, hipStream_t s,
                            const unsigned long long* d_patch = nullptr, int32_t patch_count = 0);

constexpr int64_t EXPORT_NONE = INT64_MIN;  // msh_export_results: no score recorded
hipError_t launch_export(const uint8_t* d_unsched, const int8_t* d_digit, int32_t n,
                         const int8_t* d_pod_digit, const uint8_t* d_pod_tol, int32_t p,
                         const PluginParams& pp, uint8_t* d_filter, int64_t* d_raw, int64_t* d_fin,
                         hipStream_t s);

// The class-row kernel's table and plugin set (MSH_BATCH_KERNEL=classrows).
struct BatchArgs {
  const uint32_t* hrows;     // class rows (HR_* layout), n_groups groups
  int32_t n_groups;          // n_pad / GROUP_NODES
  const uint32_t* ball;      // [2] first feasible key per pod class (0: !tol, 1: tol)
  PluginParams pp;
};

// One batch of a (multi-batch) launch: its own pod columns and outputs.
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
constexpr int MULTI_MAX = 32;  // batches per launch (kernel-argument descriptors, 40 B each: ~1.3 KB)
struct MultiArgs {
  BatchArgs a;  // the node table and plugin set
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

// The class-row kernel (opt-in): nb (1..MULTI_MAX) batches in ONE launch; tables up to
// classrows_fit groups.
bool classrows_fit(int32_t n_groups);
hipError_t launch_classrows(const BatchArgs& a, const BatchDesc* d, int nb, const DeviceInfo& dev, hipStream_t s);

// The per-pair kernel (pair_kernel): nb (1..MULTI_MAX) batches in one launch, or (shard) the
// per-pod shard keys of ONE batch, d[0].
struct PairArgs {
  const uint32_t* planes;  // bit-sliced node table (PLANE_* layout), n_groups groups
  int32_t n_groups;
  int32_t g_full;          // groups [0, g_full) hold real nodes only (no padding slot)
  int32_t gps;             // groups per slice wave (set by the launcher)
  int32_t noax;            // pair_lds_kernel: group 0 may settle the non-match reduction (launcher)
  int32_t nb;
  PluginParams pp;
  int64_t node_base;       // shard mode: global index of local node 0
  int32_t* keys;           // shard mode: [2 * d[0].n_pods] keys (first feasible match, non-match)
  BatchDesc d[MULTI_MAX];
};
hipError_t launch_pairs(PairArgs& a, bool shard, const DeviceInfo& dev, hipStream_t s);

hipError_t launch_decode_keys(const int8_t* pod_digit, const uint8_t* pod_tol, int32_t p,
                              const int32_t* keys, int32_t slot1_any, PluginParams pp,
                              int32_t* out_idx, int64_t* out_score, int32_t* out_status,
                              hipStream_t s);

// ---- generic score pipeline (any score plugin list; generic_kernel) ----
constexpr int GEN_MAX_SCORE = 5;  // score plugins per list: NodeNumber + up to four score columns
constexpr int GEN_COLS = 4;       // score-column plugins MSH_PLUGIN_SCORE_COLUMN0..3
constexpr int GEN_CH = 8;         // nodes per scalar-load chunk of generic_kernel
// Node record of generic_kernel (NREC uint32 per node, n_pad records, written by the prep):
// [0] NodeNumber code (suffix digit 0..9, or 15), [1] 0, [2..3] a 64-bit lane mask: all-ones when
// NodeUnschedulable passes the node for every pod, 0 when it is Spec.Unschedulable with the filter listed
// (then only the lanes of pods that tolerate the taint pass: OR with the wave's tolerates ballot).
constexpr int NREC = 4;
struct GenericArgs {
  const uint32_t* nrec;    // node records (NREC per node), List order
  const int64_t* cols;     // GEN_COLS x col_stride raw column values, List order
  const double* cols100;   // GEN_COLS x col_stride: 100 x the column value as a double (exact)
  int64_t col_stride;
  int32_t n_nodes;
  int32_t n_chunks;        // ceil(n / GEN_CH) node chunks scanned (the last may be partial)
  int32_t cps;             // chunks per slice wave (set by the launcher)
  int32_t nn_score;        // NodeNumber in the score list
  int32_t nn_prescore;     // NodeNumber in the prescore list (its PreScore state is written)
  int32_t nn_mode;         // NodeNumber's msh_normalize
  int64_t nn_weight;
  int32_t ncol;            // score-column plugins in the list
  int32_t ccol[GEN_COLS];  // ... their column (0..GEN_COLS-1), msh_normalize and weight, list order
  int32_t cmode[GEN_COLS];
  int64_t cweight[GEN_COLS];
  int32_t need_ext;        // some plugin normalizes: the extent sweep runs
  int32_t nb;              // batches (mode 0: up to MULTI_MAX; sharded modes: 1)
  int64_t node_base;       // sharded modes: global index of local node 0
  int64_t* ext;            // mode 1: out, mode 2: in; [2 (1 + ncol)][p] per-pod extents, mins negated
  int64_t* best_total;     // mode 2 out: per pod, the shard's best total (INT64_MIN: no feasible node)
  int32_t* best_idx;       // mode 2 out: its global node index (INT32_MAX: none)
  BatchDesc d[MULTI_MAX];
};
// mode 0: schedule nb batches; 1: per-pod extents over this shard; 2: per-pod best over this shard.
hipError_t launch_generic(GenericArgs& a, int mode, const DeviceInfo& dev, hipStream_t s);
hipError_t launch_generic_candidates(int32_t p, const int64_t* local_total, const int64_t* merged_total, int32_t* idx,
                                     hipStream_t s);
hipError_t launch_generic_decode(const int8_t* pod_digit, int32_t p, const int64_t* best_total, const int32_t* best_idx,
                                 int32_t nn_score, int32_t nn_prescore, int32_t* out_idx, int64_t* out_score,
                                 int32_t* out_status, hipStream_t s);
// 100 x each valid column as a double, for the normalizing columns (after a column changes)
hipError_t launch_cols100(const int64_t* cols, double* cols100, int64_t stride, int32_t n, int32_t n_pad,
                          uint32_t col_mask, hipStream_t s);

struct SeqArgs {
  const uint32_t* planes;    // bit-sliced node table (PLANE_* layout)
  int32_t n_words;           // n_pad / 32
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
