// msh_ctx.h — the msh_ctx behind include/minisched_hip.h and the host helpers its translation units
// share (msh_capi.cpp: single-device entry points; msh_shard.cpp: node-sharded merge, RCCL communicator
// and device groups). Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "../../include/minisched_hip.h"
#include "msh_internal.h"

// One version of the node-side device tables (List order, padded to cap nodes).
struct NodeTable {
  size_t cap = 0;
  uint8_t* d_unsched = nullptr;  // the uploaded columns (read by generic_kernel and the export as they are)
  int8_t* d_digit = nullptr;
  uint32_t* d_planes = nullptr;  // bit-sliced node table (msh_internal.h PLANE_* layout): pair / seq kernels
  // score-column plugins (generic pipeline): GEN_COLS x cap int64, column k valid when col_ok[k], with the
  // range of its values (host side: the generic launch bounds the totals from it)
  int64_t* d_cols = nullptr;
  bool col_ok[msh::GEN_COLS] = {};
  int64_t col_lo[msh::GEN_COLS] = {}, col_hi[msh::GEN_COLS] = {};
  // launches that read this version: one event per caller stream, re-recorded after each launch
  std::vector<std::pair<hipStream_t, hipEvent_t>> readers;
};

// The merge buffers of the node-sharded entry points (msh_schedule_nodeshard_device), per ctx: the
// shard keys (2p int32), or the generic form's extents, totals and indices, grown on demand.
struct ShardScratch {
  size_t pods = 0, ext = 0;   // capacities: pods, extent entries
  int32_t* keys = nullptr;    // 2 x pods
  int64_t* ext_buf = nullptr; // ext
  int64_t* total = nullptr;   // pods: this shard's best totals
  int64_t* merged = nullptr;  // pods: the merged maximum
  int32_t* idx = nullptr;     // pods: best global index (merged by MIN)
  // the last node-sharded launch (its stream and completion event): the next one on another stream waits
  // for it, a reallocation waits for it on the host
  hipStream_t last_stream = nullptr;
  hipEvent_t last_ev = nullptr;
  bool in_flight = false;
};

struct msh_ctx {
  int device = 0;
  std::string err;
  msh::DeviceInfo dev;
  hipStream_t stream = nullptr;  // used by the synchronous host-buffer entry points

  // plugin descriptor
  std::vector<int32_t> filter_ids, prescore_ids, score_ids, normalize;
  std::vector<int64_t> weights;
  msh::PluginParams pp{1, 1, 1, 0, 1};

  // node table: two versions. Launches read tab[cur]; a rewrite (upload, patch, plugin change,
  // score column) builds the other version on prep_stream and then publishes it, so it never waits
  // for launches in flight on the version they read (only for those of two rewrites ago, on the
  // version it overwrites, long done in practice).
  bool have_nodes = false;
  int32_t n_nodes = 0, n_pad = 0;
  NodeTable tab[2];
  int cur = 0;
  // sequential-mode state (not versioned: carried from call to call): pods committed per node, and
  // the sequential launches in flight that update it
  // (counts_replicas arrays of counts_cap: msh::SEQ_COUNT_REPLICAS for tables pod blocks can take, else
  // 1; counts_dirty: replicas 1.. may hold counts, folded into replica 0 by the next one-workgroup
  // launch or count read)
  int32_t* d_counts = nullptr;
  size_t counts_cap = 0;
  int32_t counts_replicas = 1;
  bool counts_dirty = false;
  // per caller stream, the event of its last sequential launch: an alias of a table version's reader
  // event (not owned here; track_launch)
  std::vector<std::pair<hipStream_t, hipEvent_t>> seq_inflight;
  // the rewrites' own stream, created with the device's highest priority: HIP gives each priority
  // its own hardware queues, so a rewrite never queues behind other streams' kernels that happen to
  // share a hardware queue with it (GPU_MAX_HW_QUEUES per priority)
  hipStream_t prep_stream = nullptr;
  bool generic = false;  // the score list names a score-column plugin

  // host-path buffers
  size_t pod_cap = 0;
  int8_t* d_pd = nullptr;         // device scratch for the pod columns
  uint8_t* d_pt = nullptr;
  size_t stage_cap = 0;
  unsigned char* h_stage = nullptr;  // page-locked: digit p | tol p | idx 4p | score 8p | status 4p
  // msh_schedule_batch_async: a ring of MSH_ASYNC_DEPTH events on the ctx's stream; ticket t's event
  // is async_ev[t % MSH_ASYNC_DEPTH]; every ticket <= async_done has completed
  hipEvent_t async_ev[MSH_ASYNC_DEPTH] = {};
  uint64_t async_issued = 0, async_done = 0;
  size_t patch_cap = 0;
  unsigned long long* d_patch = nullptr;  // msh_patch_nodes entries
  std::vector<unsigned long long> h_patch;
  // page-locked staging of node columns / patch entries (uploads copy from it, never from pageable
  // memory: a pageable copy may wait for more than this ctx's stream)
  size_t nstage_cap = 0;
  unsigned char* h_nstage = nullptr;
  // msh_timing_begin / _end: kernel start / stop event pairs for the next hot-kernel launches
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> tev;
  size_t t_next = 0;

  // node-sharded mode (msh_shard.cpp): the RCCL communicator (ncclComm_t; null: a world of one) and
  // the merge buffers
  void* comm = nullptr;
  int32_t comm_world = 0, comm_rank = 0;
  ShardScratch shard;
};

namespace msh::capi {

int fail(msh_ctx* c, int code, const std::string& msg);
int hip_fail(msh_ctx* c, hipError_t e, const char* what);

#define MSH_HIP(ctx, call)                                          \
  do {                                                              \
    hipError_t e_ = (call);                                         \
    if (e_ != hipSuccess) return ::msh::capi::hip_fail(ctx, e_, #call); \
  } while (0)

NodeTable& cur_table(msh_ctx* c);
// Launch-path check: the tables are always published ready (rewrites are synchronous).
int ready(msh_ctx* c);
// After a launch on caller stream s that reads the current table version (seq: and updates the
// sequential-mode counts).
int track_launch(msh_ctx* c, hipStream_t s, bool seq = false);
// pair_kernel's arguments for the current table (the batches are filled in by the caller).
msh::PairArgs pair_args(msh_ctx* c);
// generic_kernel's arguments for the current table and plugin list (MSH_ERR_STATE: a column missing).
int generic_args(msh_ctx* c, msh::GenericArgs& g);
// The generic pipeline runs the batch entry points when the score list names a score column (or for
// every list with msh_options.batch_kernel = 1).
bool use_generic(const msh_ctx* c);

// One hot-kernel launch under msh_timing_begin: arms the next event pair for the launcher on this
// thread; a launcher that launched nothing leaves it unused.
struct TimedLaunch {
  msh_ctx* c;
  bool armed = false;
  explicit TimedLaunch(msh_ctx* ctx);
  ~TimedLaunch();
};

// The ctx's device current for the call, the caller's restored after it (no switch at all in the
// common case of a caller already on that device).
struct DeviceGuard {
  int prev = -1, want;
  explicit DeviceGuard(int d) : want(d) {
    if (hipGetDevice(&prev) != hipSuccess || prev != d) (void)hipSetDevice(d);
  }
  ~DeviceGuard() {
    if (prev >= 0 && prev != want) (void)hipSetDevice(prev);
  }
};

// Host-buffer I/O of one synchronous call: pod columns and outputs in page-locked host memory, read
// and written by the kernel; then, for a pageable caller, outputs copied from the stage into the
// caller's arrays.
struct HostIO {
  int8_t* d_pd = nullptr;
  uint8_t* d_pt = nullptr;
  int32_t* o_idx = nullptr;    // what the kernel writes (device-visible)
  int64_t* o_score = nullptr;
  int32_t* o_status = nullptr;
  int32_t* h_idx = nullptr;    // page-locked destination: the caller's arrays or the stage
  int64_t* h_score = nullptr;
  int32_t* h_status = nullptr;
  bool staged = false;
};
int host_io_begin(msh_ctx* c, int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol, int32_t* out_idx,
                  int64_t* out_score, int32_t* out_status, HostIO& io);
int host_io_end(msh_ctx* c, int32_t p, int32_t* out_idx, int64_t* out_score, int32_t* out_status, const HostIO& io);

// Device-visible address of page-locked host memory (msh_host_alloc'd or registered), or nullptr.
void* pinned_device_ptr(const void* p);

}  // namespace msh::capi

// msh_shard.cpp: releases the ctx's communicator and merge buffers (msh_destroy).
void msh_shard_release(msh_ctx* c);
