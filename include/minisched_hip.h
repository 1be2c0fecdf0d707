/*
 * minisched_hip.h — C-ABI of libminisched_hip.so, the MI355X (gfx950) scheduling core.
 *
 * This is the drop-in boundary for the reference's per-pod hot path
 * (shopetan/mini-kube-scheduler, Go, k8s v1.22.0):
 *
 *   minisched/minisched.go:32-87   Scheduler.scheduleOne (selection part)
 *   minisched/minisched.go:115-151 RunFilterPlugins   -> feasibility stage
 *   minisched/minisched.go:153-162 RunPreScorePlugins -> per-pod prescore (pod digit)
 *   minisched/minisched.go:164-199 RunScorePlugins    -> score + normalize + sum stage
 *   minisched/minisched.go:304-325 selectHost         -> argmax stage (first max, see below)
 *   minisched/plugins/score/nodenumber/nodenumber.go:50-100  NodeNumber PreScore/Score
 *   k8s.io/kubernetes@v1.22.0 .../nodeunschedulable Filter (wired minisched/initialize.go:193-202)
 *
 * The reference evaluates ONE pod against a freshly LISTed []v1.Node per cycle.
 * Here a whole batch of pods is evaluated against a device-resident node table.
 * A cgo binding replaces scheduleOne's :40-80 segment for a batch
 * drained from activeQ; Permit/Bind stay per pod on the host.
 *
 * Conventions
 *  - Every function returns an int: MSH_OK (0) or a negative msh_err code.
 *    Per-pod outcomes are NOT errors: they go to out_status (MSH_PLACED /
 *    MSH_FIT_ERROR / MSH_SCORE_ERROR), mirroring minisched.go:50-80 + ErrorFunc :283-298.
 *  - Host pointers are caller-owned; the library copies them in/out and keeps
 *    no pointer past the call. "_device" entry points take device pointers and a
 *    hipStream_t passed as void* (NULL = the null stream) and are asynchronous.
 *  - A ctx is bound to one device and is not thread-safe; every entry point
 *    calls hipSetDevice(ctx->device) first (cgo calls land on arbitrary OS threads).
 *  - Node tables are in the reference's LIST order: byte-wise sorted node names
 *    (etcd key order, minisched.go:40). msh_pack_nodes produces that order.
 *  - Tie-break: the reference's selectHost reservoir-samples ties with math/rand
 *    (minisched.go:316-321). This library's contract is deterministic: the
 *    LOWEST node index among the maximum total score (first max in List order).
 */
#ifndef MINISCHED_HIP_H
#define MINISCHED_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MSH_ABI_VERSION 8

/* ---- error codes (return values) ---- */
typedef enum msh_err {
  MSH_OK = 0,
  MSH_ERR_INVALID = -1,     /* bad argument (null pointer, negative size, bad plugin id, ...) */
  MSH_ERR_NO_DEVICE = -2,   /* no HIP device / bad device ordinal */
  MSH_ERR_HIP = -3,         /* a HIP runtime call failed (message in msh_last_error) */
  MSH_ERR_STATE = -4,       /* call order: e.g. schedule before msh_upload_nodes */
  MSH_ERR_UNSUPPORTED = -5, /* plugin combination / size the device path does not implement */
  MSH_ERR_NOMEM = -6
} msh_err;

/* ---- per-pod outcome (out_status) ---- */
typedef enum msh_status {
  MSH_PLACED = 0,      /* selectHost returned a node (minisched.go:80-87) */
  MSH_FIT_ERROR = 1,   /* no feasible node: *framework.FitError (minisched.go:143-148) */
  MSH_SCORE_ERROR = 2  /* a Score plugin failed (minisched.go:70-75); e.g. NodeNumber with
                          no PreScore state (nodenumber.go:74-77) */
} msh_status;

/* ---- device plugin ids (framework.Plugin.Name() -> id) ---- */
typedef enum msh_plugin_id {
  MSH_PLUGIN_NODE_UNSCHEDULABLE = 1, /* "NodeUnschedulable" (Filter) */
  MSH_PLUGIN_NODE_NUMBER = 2,        /* "NodeNumber" (PreScore, Score) */
  /* Score-column plugins (ABI v5, build extension): a score plugin whose Score(pod, node) is an
   * int64 the host computed per node (msh_upload_score_column), e.g. a node-only scorer evaluated
   * once per snapshot. Score lists with one of these run on the generic pipeline (an explicit
   * int64 score per pair, per-plugin NormalizeScore over the feasible list, weights, first max):
   * the batch entry points and the node-sharded msh_generic_* entry points (shard keys, sequential
   * mode and the export: MSH_ERR_UNSUPPORTED). */
  MSH_PLUGIN_SCORE_COLUMN0 = 16,
  MSH_PLUGIN_SCORE_COLUMN1 = 17,
  MSH_PLUGIN_SCORE_COLUMN2 = 18,
  MSH_PLUGIN_SCORE_COLUMN3 = 19
} msh_plugin_id;

/* ---- per-score-plugin normalize stage ----
 * NONE reproduces the reference (NodeNumber.ScoreExtensions() == nil, nodenumber.go:98-100).
 * The others are build extensions (parity unpinned by the reference), applied once per
 * pod over the feasible list (upstream framework order: Score -> NormalizeScore -> weight):
 *   DEFAULT         upstream helper.DefaultNormalizeScore(MaxNodeScore=100, reverse=false)
 *   DEFAULT_REVERSE upstream helper.DefaultNormalizeScore(MaxNodeScore=100, reverse=true)
 *   MINMAX          100*(s-min)/(max-min) over the feasible list; 0 when max==min           */
typedef enum msh_normalize {
  MSH_NORMALIZE_NONE = 0,
  MSH_NORMALIZE_DEFAULT = 1,
  MSH_NORMALIZE_DEFAULT_REVERSE = 2,
  MSH_NORMALIZE_MINMAX = 3
} msh_normalize;

typedef struct msh_ctx msh_ctx;

/* Library ABI version (MSH_ABI_VERSION). */
int msh_abi_version(void);

/* Number of visible HIP devices (0 on a machine without a GPU). */
int msh_device_count(int* out_count);

/* Page-locked host memory (hipHostMalloc) for the host-buffer entry points' pod columns and
 * outputs. With buffers from here (or registered with HIP) msh_schedule_batch / _sequential copy
 * nothing on the host and issue no DMA: the kernel reads the pod columns from these buffers and
 * writes idx / score / status straight into them over PCIe (zero-copy). Pageable buffers work too;
 * they are staged through a page-locked buffer of the ctx. A cgo caller allocates its batch buffers
 * here once and reuses them. msh_host_free(NULL) is a no-op. */
int msh_host_alloc(size_t bytes, void** out_ptr);
void msh_host_free(void* ptr);

/* Create/destroy a context on `device`. Default plugin set = the reference's
 * (initialize.go:80-123): filter=[NodeUnschedulable], prescore=[NodeNumber],
 * score=[NodeNumber] weight 1, normalize NONE. msh_create picks every kernel automatically; the
 * library reads no environment variable. msh_destroy first waits for the launches this ctx queued
 * with the *_device entry points (they read the ctx's tables), not for the rest of the device. */
int msh_create(int device, msh_ctx** out_ctx);
void msh_destroy(msh_ctx* ctx);

/* Kernel-selection overrides (ABI v8), for parity tests and A/B measurement only: a scheduler calls
 * msh_create. Every field's 0 is the automatic choice, so a zeroed struct (with struct_size set) is
 * msh_create. A value outside a field's set is MSH_ERR_INVALID (message in msh_last_error(NULL)).
 * Results never depend on the options; only which kernel instance computes them does. */
typedef struct msh_options {
  int32_t struct_size;  /* sizeof(msh_options) */
  int32_t batch_kernel; /* 0 auto | 1 generic_kernel (explicit int64 score per pair) for every plugin list */
  int32_t pair_planes;  /* 0 auto | 1 node planes by scalar loads | 2 staged in LDS (tables that fit) */
  int32_t pair_noax;    /* 0 auto | 1 LDS form: group 0 first, settled reductions dropped | 2 group 0 last */
  int32_t pair_slices;  /* 0 auto | 1, 2, 4 slice waves per 64-pod block (and generic_kernel pod group) */
  int32_t seq_waves;    /* 0 auto | 1, 4, 15, 16 scanning waves of the sequential kernel (raised when too few) */
  int32_t seq_split;    /* 0 auto (no capacity: the batch kernel + counts) | 1 one workgroup walks the
                           whole batch | 2 64-pod blocks of consecutive pods, one workgroup each */
  int32_t seq_pod_waves; /* 0 auto | 1, 2, 4, 8 waves sharing a 64-pod block (one scanning wave, no capacity) */
  int32_t gen_keys;     /* 0 auto (64-bit totals below 2^53 as double keys) | 1 uint64 keys */
  int32_t gen_nnkey;    /* 0 auto (compare-free NodeNumber key) | 1 compare + select */
} msh_options;
int msh_create_ex(int device, const msh_options* opts, msh_ctx** out_ctx);

/* Message for the last failing call on this ctx ("" if none). Valid until the next call. With a
 * NULL ctx: the message of the last failed msh_create on the calling thread. */
const char* msh_last_error(const msh_ctx* ctx);

/* Plugin lists (Scheduler.filterPlugins / preScorePlugins / scorePlugins,
 * minisched/initialize.go:25-27). Ids must be unique within a list (the reference keys
 * score maps by plugin Name(), minisched.go:173, so duplicates collapse; rejected here).
 * weights[i] in [1, 2^32]; "TODO: plugin weight" (minisched.go:187): weight 1 == reference.
 * msh_set_plugins: prescore list = the score plugins that implement PreScore. */
int msh_set_plugins(msh_ctx* ctx, const int32_t* filter_ids, int32_t nf,
                    const int32_t* score_ids, const int64_t* weights, int32_t ns);
int msh_set_plugins_ex(msh_ctx* ctx, const int32_t* filter_ids, int32_t nf,
                       const int32_t* prescore_ids, int32_t npre,
                       const int32_t* score_ids, const int64_t* weights,
                       const int32_t* normalize, int32_t ns);

/* Node table in List order (name-sorted). unsched[i] = node.Spec.Unschedulable (0/1);
 * digit[i] = last byte of node.Name as '0'..'9' -> 0..9, else -1 (nodenumber.go:81-87).
 * 0 <= n < 2^24. Replaces the per-cycle Nodes().List (minisched.go:40). */
int msh_upload_nodes(msh_ctx* ctx, int32_t n, const uint8_t* unsched, const int8_t* digit);
int msh_num_nodes(const msh_ctx* ctx, int32_t* out_n);

/* The per-node scores of score-column plugin `plugin_id` (MSH_PLUGIN_SCORE_COLUMN0..3), n = the
 * uploaded node count, List order, each in [-2^31, 2^31]. An msh_upload_nodes drops every column
 * (its nodes are gone); a batch whose score list names a column not uploaded since is
 * MSH_ERR_STATE. Totals are Go int64 arithmetic: weight x normalized score summed with wrap-around. */
int msh_upload_score_column(msh_ctx* ctx, int32_t plugin_id, int32_t n, const int64_t* scores);

/* Per-pair plugin results for a small batch: the matrices the simulator's result store
 * turns into pod annotations (scheduler/plugin/resultstore/store.go:170-234, recorded by the
 * wrapped plugins in scheduler/plugin/plugins.go:278-325). Row j, column i (List order):
 *   out_filter[j*n+i] = 1 if node i passes the filter plugins for pod j ("passed"), else 0;
 *   out_score[j*n+i]  = NodeNumber.Score raw value (AddScoreResult);
 *   out_final[j*n+i]  = NormalizeScore(raw) * weight (AddNormalizedScoreResult ->
 *                       applyWeightOnScore, store.go:231-234);
 * score/final = MSH_EXPORT_NONE (INT64_MIN) where no score is recorded (node filtered out, or
 * the pod never reaches Score). Host buffers; p*n <= 2^28. Debug path, not the hot path. */
#define MSH_EXPORT_NONE ((int64_t)(-9223372036854775807LL - 1))
int msh_export_results(msh_ctx* ctx, int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol,
                       uint8_t* out_filter, int64_t* out_score, int64_t* out_final);

/* In-place update of `count` entries of the uploaded table (an informer Update event that
 * leaves the List order alone, e.g. a cordon flipping Spec.Unschedulable; eventhandler.go:45-50).
 * idx[k] in [0, n) and pairwise distinct; unsched[k] / digit[k] as in msh_upload_nodes.
 * O(count) host->device traffic; the per-node pod counts of sequential mode are kept.
 * Adds and deletes shift List positions: re-upload with msh_upload_nodes. */
int msh_patch_nodes(msh_ctx* ctx, int32_t count, const int32_t* idx, const uint8_t* unsched,
                    const int8_t* digit);

/* Batched hot path: p pods against the uploaded node table.
 * pod_digit[j] = last byte of pod.Name as digit or -1 (nodenumber.go:50-55);
 * pod_tol[j]   = pod tolerates taint {node.kubernetes.io/unschedulable, NoSchedule} (0/1).
 * Outputs per pod: out_idx (node index, -1 unless PLACED), out_score (total int64 score of
 * the selected node, 0 unless PLACED), out_status (msh_status). Synchronous. Host buffers:
 * page-locked ones (msh_host_alloc) take the zero-copy path, pageable ones are staged.
 * out_score may be NULL, here and in every entry point below that takes one (ABI v4): the scores
 * are then not written, 8 of the 16 output bytes per pod (a binding that only places pods, as
 * scheduleOne does after selectHost, needs the node and the status). */
int msh_schedule_batch(msh_ctx* ctx, int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol,
                       int32_t* out_idx, int64_t* out_score, int32_t* out_status);

/* Asynchronous host-buffer batch (ABI v5): msh_schedule_batch for page-locked buffers (msh_host_alloc
 * or registered with HIP; pageable ones are MSH_ERR_INVALID) that returns once the batch is launched.
 * The kernel reads the pod columns and writes the outputs over PCIe as in the synchronous call; they
 * are valid once msh_wait(ctx, ticket) returns MSH_OK. A caller packs batch i + 1 (msh_pack_pods)
 * while batch i runs, the pipeline a cgo caller draining activeQ batch after batch (minisched.go:28-34)
 * runs. Batches of one ctx complete in submission order; at most MSH_ASYNC_DEPTH are in flight (a
 * further submission first waits for the oldest). The caller must not touch a batch's buffers before
 * its msh_wait. Tickets are positive and increase by one per call. */
#define MSH_ASYNC_DEPTH 4
int msh_schedule_batch_async(msh_ctx* ctx, int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol,
                             int32_t* out_idx, int64_t* out_score, int32_t* out_status, uint64_t* out_ticket);
/* Wait for batch `ticket` (and every earlier one) of msh_schedule_batch_async. A ticket the ctx
 * never handed out is MSH_ERR_INVALID; an already completed one returns at once. */
int msh_wait(msh_ctx* ctx, uint64_t ticket);

/* Same, device-resident inputs/outputs, asynchronous on `stream` (hipStream_t).
 * Launches on different streams may overlap (independent batches pipelined): each needs its own
 * pod and output buffers. The node table is double-buffered: an upload, patch, score-column upload or
 * filter-list change rebuilds the version no launch reads, on the ctx's own high-priority stream,
 * and publishes it before the call returns (the rebuild is synchronous; launches made after it read
 * the new version, launches already queued keep reading the old one). The ctx records an event on
 * `stream` after each launch; a rebuild waits on the host only for the launches of two rebuilds ago,
 * which read the version it overwrites, and never for other ctxs' or the caller's other work. */
int msh_schedule_batch_device(msh_ctx* ctx, int32_t p, const int8_t* d_pod_digit,
                              const uint8_t* d_pod_tol, int32_t* d_out_idx,
                              int64_t* d_out_score, int32_t* d_out_status, void* stream);

/* Several independent batches in one submission (ABI v5): what a caller draining a deep activeQ
 * (minisched.go:28-34, one scheduleOne per pod) hands over when it has more than one batch ready,
 * e.g. consecutive next_batch drains. batches[i] describes batch i exactly as the arguments of
 * msh_schedule_batch_device (device pointers, out_score may be NULL); the descriptor array itself
 * is host memory, read during the call. Up to MSH_BATCHES_PER_LAUNCH batches share one kernel
 * launch (a larger nb takes ceil(nb / MSH_BATCHES_PER_LAUNCH) launches, in order, on `stream`),
 * which spreads the launch cost and the kernel's fill and drain over them. Results are identical to
 * nb msh_schedule_batch_device calls. Asynchronous, like msh_schedule_batch_device. */
#define MSH_BATCHES_PER_LAUNCH 32
typedef struct msh_batch {
  int32_t p;
  int32_t reserved; /* 0 */
  const int8_t* pod_digit;
  const uint8_t* pod_tol;
  int32_t* out_idx;
  int64_t* out_score;
  int32_t* out_status;
} msh_batch;
int msh_schedule_batches_device(msh_ctx* ctx, int32_t nb, const msh_batch* batches, void* stream);

/* Sequential-commit mode (one pod at a time, node state committed between placements).
 * The node table stays in the registers of a workgroup: up to 368,640 nodes without a capacity,
 * 262,144 with one (larger tables: MSH_ERR_UNSUPPORTED).
 * The commit increments the selected node's assigned-pod count on the device (the
 * NodeInfo.AddPod analogue). max_pods_per_node > 0 additionally makes a node infeasible
 * once it holds that many pods (build extension): one workgroup walks the whole batch. 0 =
 * reference semantics, where no commit feeds a later decision and the placements equal
 * msh_schedule_batch's: tables up to 32,768 nodes then run on the per-pair batch kernel, whose waves
 * add their placed pods to the counts (a no-capacity shortcut: the pods are not decided in order, exact
 * because the counts are the same in any order). msh_options.seq_split = 2 runs 64-pod blocks of
 * consecutive pods instead, one workgroup each, concurrently, the pods within a block in order; = 1
 * walks the whole batch in one workgroup, in order, as a capacity does.
 * `commit_cb` (may be NULL) is replayed on the host after the device run, in
 * placement order, once per PLACED pod. The counts carry over from call to call; sequential launches
 * of one ctx on different streams are ordered by the library (each waits for the ones in flight). */
typedef void (*msh_commit_cb)(void* user, int32_t pod, int32_t node_idx, int64_t score);
int msh_schedule_sequential(msh_ctx* ctx, int32_t p, const int8_t* pod_digit,
                            const uint8_t* pod_tol, int32_t max_pods_per_node,
                            int32_t* out_idx, int64_t* out_score, int32_t* out_status,
                            msh_commit_cb commit_cb, void* user);
int msh_schedule_sequential_device(msh_ctx* ctx, int32_t p, const int8_t* d_pod_digit,
                                   const uint8_t* d_pod_tol, int32_t max_pods_per_node,
                                   int32_t* d_out_idx, int64_t* d_out_score,
                                   int32_t* d_out_status, void* stream);
/* Per-node assigned-pod counts accumulated by the sequential commits (n entries). */
int msh_node_pod_counts(msh_ctx* ctx, int32_t* out_counts);
int msh_reset_node_pod_counts(msh_ctx* ctx);

/* ---- node-sharded mode (a cluster's node table split over devices) ----
 * Each shard holds a contiguous slice [node_base, node_base + n) of the global List order and
 * produces int32 keys, key = 0x7FFFFFFF - global_idx (0 = none), so that the element-wise MAX
 * over shards (one RCCL allreduce MAX) is the global first node. Layout (ABI v7), msh_shard_keys_len
 * = 2p entries, every entry a property of pod j alone (evaluated per (pod, node) pair of the shard):
 *   keys[j]      first feasible node whose NodeNumber score is 10 for pod j (feasible match)
 *   keys[p + j]  REVERSE / MINMAX normalize: first feasible node whose NodeNumber score is 0 for pod j
 *                (feasible non-match); every other mode: first feasible node for pod j
 * 8 B per pod cross the interconnect (selectHost over the merged keys replaces minisched.go:304-325
 * across shards; the first feasible node is the larger of the two keys in either case). msh_decode_keys_device then
 * produces idx/score/status exactly as msh_schedule_batch over the whole table. Score-column plugin
 * lists use msh_generic_extents_device / msh_generic_best_device / msh_generic_decode_device below. */
int msh_shard_keys_len(const msh_ctx* ctx, int32_t p, int32_t* out_len);
int msh_shard_keys_device(msh_ctx* ctx, int32_t p, const int8_t* d_pod_digit,
                          const uint8_t* d_pod_tol, int64_t node_base, int32_t* d_keys,
                          void* stream);
int msh_decode_keys_device(msh_ctx* ctx, int32_t p, const int8_t* d_pod_digit,
                           const uint8_t* d_pod_tol, const int32_t* d_keys,
                           int32_t* d_out_idx, int64_t* d_out_score, int32_t* d_out_status,
                           void* stream);
/* Kept for ABI compatibility: always 0 since ABI v7 (keys[p + j] is per pod, never per pod class). */
int msh_keys_slot1_is_any(const msh_ctx* ctx, int32_t* out_flag);

/* ---- node-sharded generic pipeline (ABI v7): any plugin list, score-column lists included ----
 * Each shard (a contiguous List-order slice, as above) computes per pod its best (int64 total, global
 * node index) over its nodes; the merge is two all-reduces, MAX over the totals, then MIN over the
 * indices of the shards that hold the maximum (the global first maximum: selectHost,
 * minisched.go:304-325, across shards). A plugin that normalizes needs the pod's extent (max, min of
 * its raw scores) over the feasible nodes of EVERY shard before any total is formed:
 *   1. len = msh_generic_ext_len(ctx, p); when len > 0: msh_generic_extents_device on every shard into
 *      len int64 (the minima stored negated), then one all-reduce MAX of them;
 *   2. msh_generic_best_device(..., d_ext (the merged extents, or NULL when len == 0), node_base,
 *      d_total, d_idx): this shard's best per pod (INT64_MIN / INT32_MAX: no feasible node here);
 *   3. d_merged = copy of d_total, all-reduce MAX over d_merged;
 *   4. msh_generic_candidates_device(p, d_total, d_merged, d_idx): d_idx[j] = INT32_MAX unless this
 *      shard holds pod j's maximum; then all-reduce MIN over d_idx;
 *   5. msh_generic_decode_device(..., d_merged, d_idx, outputs): idx / score / status exactly as
 *      msh_schedule_batch over the whole table (FitError when no shard has a feasible node).
 * Device pointers, asynchronous on `stream` (hipStream_t as void*, NULL = the null stream). */
int msh_generic_ext_len(const msh_ctx* ctx, int32_t p, int64_t* out_len);
int msh_generic_extents_device(msh_ctx* ctx, int32_t p, const int8_t* d_pod_digit, const uint8_t* d_pod_tol,
                               int64_t* d_ext, void* stream);
int msh_generic_best_device(msh_ctx* ctx, int32_t p, const int8_t* d_pod_digit, const uint8_t* d_pod_tol,
                            const int64_t* d_ext, int64_t node_base, int64_t* d_best_total, int32_t* d_best_idx,
                            void* stream);
int msh_generic_candidates_device(msh_ctx* ctx, int32_t p, const int64_t* d_local_total, const int64_t* d_merged_total,
                                  int32_t* d_best_idx, void* stream);
int msh_generic_decode_device(msh_ctx* ctx, int32_t p, const int8_t* d_pod_digit, const int64_t* d_merged_total,
                              const int32_t* d_merged_idx, int32_t* d_out_idx, int64_t* d_out_score,
                              int32_t* d_out_status, void* stream);

/* ---- node-sharded scheduling with the merge inside the library (ABI v8) ----
 * The entry points above leave the cross-shard merge to the caller. These own it, in the two shapes a
 * scheduler process takes; both give exactly msh_schedule_batch over the whole List-order table
 * (selectHost's first maximum, minisched.go:304-325, across shards), for every plugin list.
 *
 * (1) One process per GPU: an RCCL communicator inside the ctx (librccl.so.1, loaded on the first
 *     msh_comm_* call). Rank 0 makes an id with msh_comm_unique_id; the caller ships its
 *     MSH_COMM_ID_BYTES bytes to every rank over any channel (a Go scheduler: its own RPC or a file);
 *     every rank then calls msh_comm_init (collective: it returns once all `world` ranks have joined).
 *     msh_schedule_nodeshard_device runs, on `stream`: the shard kernel over this ctx's slice, the
 *     all-reduce(s) over xGMI (ncclAllReduce on the same stream), and the decode; every rank ends with
 *     every pod's decision. The reference plugins take one all-reduce(MAX) of 8 B per pod; a list with
 *     score columns or a normalizer takes the generic form's three (extents MAX, totals MAX, indices
 *     MIN). All ranks must make the same sequence of calls with the same p. A ctx without a
 *     communicator runs the same path as a world of one. node_base = the global List index of this
 *     ctx's first node. The ctx's merge buffers are shared by its node-sharded launches: a launch on
 *     another stream first waits for the previous one. */
#define MSH_COMM_ID_BYTES 128
int msh_comm_unique_id(uint8_t* out_id); /* out_id: MSH_COMM_ID_BYTES bytes (ncclGetUniqueId) */
int msh_comm_init(msh_ctx* ctx, const uint8_t* id, int32_t world, int32_t rank);
/* world / rank of the ctx's communicator (world 0, rank 0 when msh_comm_init has not been called). */
int msh_comm_info(const msh_ctx* ctx, int32_t* out_world, int32_t* out_rank);
int msh_schedule_nodeshard_device(msh_ctx* ctx, int32_t p, const int8_t* d_pod_digit, const uint8_t* d_pod_tol,
                                  int64_t node_base, int32_t* d_out_idx, int64_t* d_out_score,
                                  int32_t* d_out_status, void* stream);
/* The same from host buffers (the cgo form), synchronous: the pod columns go to the device and the
 * decisions come back as in msh_schedule_batch. */
int msh_schedule_nodeshard(msh_ctx* ctx, int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol,
                           int64_t node_base, int32_t* out_idx, int64_t* out_score, int32_t* out_status);

/* (2) One process driving several devices (the reference's single scheduling loop, minisched.go:28-30,
 *     with its node table split over the node's GPUs): a group of shard ctxs, shards[k] holding the k-th
 *     contiguous slice of the List order (node_base = the node counts of shards[0..k) at call time).
 *     The ctxs stay owned by the caller (destroy the group first) and may sit on any devices, the same
 *     one included; shards on different devices need peer access to shards[0]'s device (xGMI; else
 *     MSH_ERR_UNSUPPORTED at msh_group_create). Every shard must hold the same plugin lists (checked per
 *     call: MSH_ERR_STATE). msh_group_schedule_batch: the pod columns are copied to every shard device,
 *     each shard runs its kernel on its own stream, and the merge runs on shards[0]'s device as one
 *     kernel that reads every shard's per-pod result over xGMI (peer loads) and decodes; a list with
 *     normalizers first merges the per-pod extents the same way and every shard reads them back. Host
 *     buffers, synchronous. Up to MSH_GROUP_MAX_SHARDS shards. */
#define MSH_GROUP_MAX_SHARDS 16
typedef struct msh_group msh_group;
int msh_group_create(msh_ctx* const* shards, int32_t n, msh_group** out_group);
void msh_group_destroy(msh_group* group);
const char* msh_group_last_error(const msh_group* group); /* NULL group: the last failed msh_group_create */
int msh_group_schedule_batch(msh_group* group, int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol,
                             int32_t* out_idx, int64_t* out_score, int32_t* out_status);

/* ---- kernel timing (measurement hook) ----
 * msh_timing_begin arms up to max_launches (1..4096) event pairs: each following hot-kernel launch of
 * this ctx made from this thread (the batch, multi-batch, generic and sequential kernels) records its
 * pair at the kernel's own start and completion (hipExtLaunchKernelGGL), the interval a kernel trace
 * (rocprofv3) reports, without the stream gaps around it. msh_timing_end waits for the recorded
 * launches and returns their count, summed and longest duration (ms), and disarms. Launches past
 * max_launches are not timed. Not needed by a scheduler; used by bench.py's roofline. */
int msh_timing_begin(msh_ctx* ctx, int32_t max_launches);
int msh_timing_end(msh_ctx* ctx, int32_t* out_launches, double* out_total_ms, double* out_max_ms);

/* ---- snapshot packer (host, no device needed) ----
 * Names are given as one byte blob + n+1 offsets (name i = blob[off[i]:off[i+1]]).
 * msh_pack_nodes sorts nodes byte-wise by name (the apiserver LIST order), and writes
 * out_order[k] = input index of the k-th node in List order, plus the SoA columns.
 * Empty names are rejected (the reference would panic on name[len-1:]). Duplicate names
 * are rejected (apiserver names are unique). */
int msh_pack_nodes(int32_t n, const char* names, const int64_t* name_off,
                   const uint8_t* unschedulable, int32_t* out_order, uint8_t* out_unsched,
                   int8_t* out_digit);

/* One toleration of pod.Spec.Tolerations (k8s.io/api core/v1 Toleration). NULL == "". */
typedef struct msh_toleration {
  const char* key;
  const char* op;     /* "", "Equal", "Exists" */
  const char* value;
  const char* effect; /* "", "NoSchedule", "PreferNoSchedule", "NoExecute" */
} msh_toleration;

/* Pods: digit from the name's last byte; tolerates from tolerations
 * [tol_off[j], tol_off[j+1]) of `tols` (upstream v1helper.TolerationsTolerateTaint with the
 * taint {Key: node.kubernetes.io/unschedulable, Effect: NoSchedule}). */
int msh_pack_pods(int32_t p, const char* names, const int64_t* name_off,
                  const msh_toleration* tols, const int64_t* tol_off, int8_t* out_digit,
                  uint8_t* out_tol);

/* Single-toleration predicate (Toleration.ToleratesTaint against the unschedulable taint). */
int msh_toleration_tolerates_unschedulable(const msh_toleration* t);

#ifdef __cplusplus
}
#endif

#endif /* MINISCHED_HIP_H */
