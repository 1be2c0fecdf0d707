// msh_internal.h — shared between the C-ABI (msh_capi.cpp) and the gfx950 kernels (msh_prep.hip,
// msh_pair.hip, msh_generic.hip, msh_seq.hip). Not part of the public ABI (include/minisched_hip.h is).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace msh {

constexpr int32_t MAX_NODES = 0xFFFFFE;          // nodes per context (2^24 - 2)
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

// Device facts and launch choices, resolved once in msh_create / msh_create_ex (never on the launch
// path). The overrides come only from msh_create_ex's msh_options (tests and A/B measurement); the
// library reads no environment variable.
struct DeviceInfo {
  int cus = 256;
  int bits_slices = 0;   // msh_options.pair_slices: pair_kernel slice waves per pod block (1, 2, 4) and
                         // generic_kernel waves per pod group, 0 = auto
  int seq_waves = 0;     // msh_options.seq_waves: sequential scanning waves, 0 = auto
  // msh_options.batch_kernel: 0 = the per-pair bit-plane kernels for the reference's plugins (default);
  // 1 = generic_kernel for every plugin list (A/B and cross-check)
  int batch_kernel = 0;
  // msh_options.pair_planes, where pair_kernel's node planes come from: 0 = auto (LDS-staged for tables
  // up to PAIR_LDS_BIG_GROUPS groups and launches that fill the chip, scalar loads otherwise), 1 = scalar
  // loads into SGPRs, 2 = LDS-staged (tables that fit)
  int pair_planes = 0;
  // msh_options.pair_noax: the LDS-staged form scans group 0 first and drops the non-match / feasible
  // reduction from the scan of the other groups when group 0 has settled it for every lane of the
  // wave (1), or scans group 0 last and never drops it (0). -1 = auto: 1 for REVERSE / MINMAX (78.1
  // against 89.0 us per 32-batch C3 launch), 0 for the identity-like modes (77.3-78.3 against
  // 80.9-81.2), profiles/r4_ab_pair_planes.txt
  int pair_noax = -1;
  // msh_options.seq_split, without a capacity: the per-pair batch kernel with the commit epilogue (auto,
  // 2), the sequential kernel's 64-pod blocks of consecutive pods, one workgroup each (1), or the whole
  // batch in one workgroup, in order (serial, 0)
  int seq_split = 2;
  int seq_pod_waves = 0;  // msh_options.seq_pod_waves: pod waves per pod-block workgroup (1, 2, 4, 8), 0 = auto
  int gen_f53 = 1;    // msh_options.gen_keys: generic_kernel's double keys for 64-bit totals below 2^53 (1) or uint64_t (0)
  int gen_nnkey = 1;  // msh_options.gen_nnkey: generic_kernel's compare-free NodeNumber key (1) or the select (0)
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

// ---- launchers (msh_prep.hip, msh_pair.hip, msh_generic.hip, msh_seq.hip) ----
// The bit planes of the whole table from the uploaded columns (n nodes, n_pad slots).
hipError_t launch_node_prep(const uint8_t* d_unsched, const int8_t* d_digit, int32_t n, int32_t n_pad,
                            int32_t has_nu, uint32_t* d_planes, hipStream_t s);
// A rewrite's copy of the published table version (the uploaded columns and the planes, n_words 32-node
// words), with up to PATCH_INLINE msh_patch_nodes entries (idx | unsched << 32 | (uint8)digit << 40)
// applied on the way: the patched words' planes are rebuilt, nothing else is (O(N / 32) threads).
constexpr int PATCH_INLINE = 64;
struct TableCopyArgs {
  const uint8_t* src_unsched;
  const int8_t* src_digit;
  const uint32_t* src_planes;
  uint8_t* dst_unsched;
  int8_t* dst_digit;
  uint32_t* dst_planes;
  int32_t n, n_words, has_nu, count;
  unsigned long long inl[PATCH_INLINE];
};
hipError_t launch_table_copy(const TableCopyArgs& a, hipStream_t s);
// A larger patch: its entries scattered into the copied columns (the full prep re-runs after it).
hipError_t launch_patch_scatter(const unsigned long long* d_entries, int32_t count, uint8_t* d_unsched,
                                int8_t* d_digit, hipStream_t s);

constexpr int64_t EXPORT_NONE = INT64_MIN;  // msh_export_results: no score recorded
hipError_t launch_export(const uint8_t* d_unsched, const int8_t* d_digit, int32_t n,
                         const int8_t* d_pod_digit, const uint8_t* d_pod_tol, int32_t p,
                         const PluginParams& pp, uint8_t* d_filter, int64_t* d_raw, int64_t* d_fin,
                         hipStream_t s);

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
constexpr int MULTI_MAX = 32;  // batches per launch (kernel-argument descriptors, 40 B each: ~1.3 KB)

// The per-pair kernel (pair_kernel): nb (1..MULTI_MAX) batches in one launch, or (shard) the
// per-pod shard keys of ONE batch, d[0].
struct PairCommon {
  const uint32_t* planes;  // bit-sliced node table (PLANE_* layout), n_groups groups
  int32_t n_groups;
  int32_t g_full;          // groups [0, g_full) hold real nodes only (no padding slot)
  int32_t gps;             // groups per slice wave (set by the launcher)
  int32_t noax;            // pair_lds_kernel: group 0 may settle the non-match reduction (launcher)
  int32_t nb;
  PluginParams pp;
  int64_t node_base;       // shard mode: global index of local node 0
  int32_t* keys;           // shard mode: [2 * d[0].n_pods] keys (first feasible match, non-match)
  // sequential mode without a capacity (one batch): every placed pod adds 1 to its node's count in
  // replica (64-pod block mod SEQ_COUNT_REPLICAS) of these SEQ_COUNT_REPLICAS arrays; null otherwise
  int32_t* counts;
  int64_t count_stride;
};
// The kernel arguments with room for NB batch descriptors: the host builds PairArgs (MULTI_MAX); a
// one-batch launch passes PairArgsN<1> (136 B of arguments instead of 1,624 B: the argument copy of a
// 1.6 KB block costs ~3-4 us of host time per hipLaunchKernel)
template <int NB>
struct PairArgsN : PairCommon {
  BatchDesc d[NB];
};
using PairArgs = PairArgsN<MULTI_MAX>;
hipError_t launch_pairs(PairArgs& a, bool shard, const DeviceInfo& dev, hipStream_t s);

hipError_t launch_decode_keys(const int8_t* pod_digit, int32_t p, const int32_t* keys, PluginParams pp,
                              int32_t* out_idx, int64_t* out_score, int32_t* out_status, hipStream_t s);

// Device groups (msh_group_*, msh_prep.hip): the merge on the home device over every shard's per-pod
// buffers (peer-mapped pointers, one per shard, List order of the shards).
constexpr int GROUP_MAX = 16;  // MSH_GROUP_MAX_SHARDS
struct GroupPtrs {
  const int32_t* keys[GROUP_MAX];  // shard keys, 2p each (group_keys_decode)
  const int64_t* v[GROUP_MAX];     // extents (group_max_i64) or best totals (group_best_merge)
  const int32_t* idx[GROUP_MAX];   // best global indices (group_best_merge)
  int32_t n;
};
// element-wise MAX of the shards' keys, then decode_pod (msh_decode_keys_device's decode)
hipError_t launch_group_keys_decode(const GroupPtrs& g, const int8_t* pod_digit, int32_t p, PluginParams pp,
                                    int32_t* out_idx, int64_t* out_score, int32_t* out_status, hipStream_t s);
// element-wise MAX of the shards' len int64 (the generic extents: maxima and negated minima)
hipError_t launch_group_max_i64(const GroupPtrs& g, int64_t len, int64_t* out, hipStream_t s);
// per pod: the largest total, then the lowest global index among the shards holding it
hipError_t launch_group_best_merge(const GroupPtrs& g, int32_t p, int64_t* out_total, int32_t* out_idx,
                                   hipStream_t s);

// ---- generic score pipeline (any score plugin list; generic_kernel) ----
constexpr int GEN_MAX_SCORE = 5;  // score plugins per list: NodeNumber + up to four score columns
constexpr int GEN_COLS = 4;       // score-column plugins MSH_PLUGIN_SCORE_COLUMN0..3
struct GenericArgs {
  const uint8_t* unsched;  // the uploaded node columns, List order (n_nodes valid)
  const int8_t* digit;
  const int64_t* cols;     // GEN_COLS x col_stride raw column values, List order
  int64_t col_stride;
  int32_t n_nodes;
  int32_t has_nu;          // NodeUnschedulable in the filter list
  int32_t tile;            // nodes per LDS tile (set by the launcher)
  int32_t slices;          // waves per pod group (set by the launcher)
  int32_t nn_score;        // NodeNumber in the score list
  int32_t nn_prescore;     // NodeNumber in the prescore list (its PreScore state is written)
  int32_t nn_mode;         // NodeNumber's msh_normalize
  int64_t nn_weight;
  int32_t ncol;            // score-column plugins in the list
  // the columns with a normalizer, in list order: column id, list position (among the columns), mode,
  // weight; and the columns without one (their weight x raw is a node-only sum)
  int32_t nnc, ncc[GEN_COLS], npos[GEN_COLS], nmode[GEN_COLS];
  int64_t nw[GEN_COLS];
  int32_t nts, tcc[GEN_COLS];
  int64_t tw[GEN_COLS];
  int32_t need_ext;        // some plugin normalizes: the extent pass runs
  int32_t w64;             // 64-bit totals (the host could not bound every feasible total within 31 bits, or a
                           // normalizing column's weight or normalized score reaches 2^23)
  int32_t f53;             // every feasible |total| below 2^53: 8-byte keys as doubles (exact integers)
  int32_t nn24;            // NodeNumber's two weighted values differ by less than 2^24 (32-bit keys: no compare)
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

struct SeqArgs {
  const uint32_t* planes;    // bit-sliced node table (PLANE_* layout)
  int32_t n_words;           // n_pad / 32
  int32_t n_nodes;
  const int8_t* pod_digit;
  const uint8_t* pod_tol;
  int32_t n_pods;
  PluginParams pp;
  int32_t max_pods;
  // per-node assigned pods, count_replicas arrays of count_stride: a node's count is its sum over the
  // replicas (pod blocks add to replica blockIdx % SEQ_COUNT_REPLICAS); read at start, updated
  int32_t* counts;
  int64_t count_stride;
  int32_t count_replicas;    // 1, or SEQ_COUNT_REPLICAS (pod blocks need them all)
  int32_t fold;              // one workgroup: first fold replicas 1.. into replica 0 (some hold counts)
  int32_t* out_idx;
  int64_t* out_score;
  int32_t* out_status;
  int32_t pods_per_block;    // set by the launcher: pods per workgroup (the whole batch when one workgroup)
};

// No-capacity sequential launches (pair_kernel's commit epilogue, seq_kernel's pod blocks) add their
// commits to one of this many count replicas: a digit's pods all land on its first feasible match, and
// device atomics from every wave onto one address queue. Per C5 launch (pair_kernel<4, .., true>,
// profiles/ab/r6_seq_pair_replicas.txt): 16 replicas 15.5 us, 64 8.5 us, 256 8.5 us (6.99 without the
// epilogue). Tables up to SEQ_SPLIT_MAX_NODES only, so larger ones keep one count array.
constexpr int SEQ_COUNT_REPLICAS = 64;
constexpr int32_t SEQ_SPLIT_MAX_NODES = 4 * 64 * 4 * 32;  // four scanning waves x 64 lanes x 4 words
// Workgroups launch_sequential runs the batch on: 64-pod blocks without a capacity on tables whose
// counts fit LDS (DeviceInfo::seq_split), else 1.
int32_t seq_blocks(const SeqArgs& a, const DeviceInfo& dev);
// counts[i] (replica 0) = the node's sum over the replicas, the others zeroed, for i < n
hipError_t launch_count_fold(int32_t* counts, int64_t stride, int32_t replicas, int32_t n, hipStream_t s);

hipError_t launch_sequential(const SeqArgs& a, const DeviceInfo& dev, hipStream_t s, std::string* err);
// The capacity form (msh_seq_cap.hip): nw scanning waves with rs words per lane, one workgroup.
hipError_t launch_seq_capacity(const SeqArgs& a, int nw, int rs, hipStream_t s);
// Pod waves per pod-block workgroup without a capacity (one scanning wave): each walks 64 / this many pods.
constexpr int SEQ_POD_WAVES = 1;  // measured: 1 / 2 / 4 / 8 waves 11.6 / 14.2 / 13.2 / 18.3 us per C5 launch (profiles/ab/r6_seq_pod_waves.jsonl)
int seq_pod_waves(const DeviceInfo& dev);

// Launch timing (msh_timing_begin / _end): the next hot-kernel launch on this thread (batch, multi-
// batch, generic, sequential kernels) records `start` / `stop` at the kernel's own start and end.
void set_launch_events(hipEvent_t start, hipEvent_t stop);
bool launch_events_pending();

}  // namespace msh
