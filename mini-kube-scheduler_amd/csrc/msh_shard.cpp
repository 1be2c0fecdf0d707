// msh_shard.cpp — node-sharded scheduling with the cross-shard merge inside the library
// (include/minisched_hip.h, ABI v8: msh_comm_*, msh_schedule_nodeshard*, msh_group_*).
//
// The reference schedules one pod at a time against the whole node list (minisched/minisched.go:28-30,
// :40) and picks the first maximum (selectHost, :304-325). With the List-order table split into
// contiguous slices, each shard finds its own first maximum per pod; because the slices ascend, the
// global first maximum is the best over the shards with ties to the lowest global index. Two shapes:
//
//  * one process per GPU: an RCCL communicator in the ctx. The reference plugins' shard result is two
//    int32 keys per pod (0x7FFFFFFF - global index of the first feasible match / non-match), merged by one
//    ncclAllReduce(MAX) of 8 B per pod on the launch stream; any other list runs the generic form's three
//    all-reduces (per-pod extents MAX, totals MAX, indices MIN). RCCL is opened with dlopen on the first
//    msh_comm_* call (librccl.so.1: the copy already in the process, e.g. PyTorch's, when there is one),
//    so a scheduler that never shards carries no RCCL dependency.
//  * one process driving several devices (msh_group): the shards' results stay in their own HBM and one
//    merge kernel on the home device reads them through peer mappings (xGMI) and decodes.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/minisched_hip.h"
#include "msh_ctx.h"
#include "msh_internal.h"

using namespace msh::capi;

static_assert(MSH_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "the comm id is an ncclUniqueId");
static_assert(MSH_GROUP_MAX_SHARDS == msh::GROUP_MAX, "group size limit");

namespace {

// ---- librccl.so.1, resolved once ----
struct Rccl {
  bool ok = false;
  std::string err;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      r.err = std::string("librccl.so.1 not loadable: ") + (e ? e : "?");
      return;
    }
    auto sym = [&](const char* name, auto& fn) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      if (!fn && r.err.empty()) r.err = std::string("librccl.so.1 lacks ") + name;
    };
    sym("ncclGetUniqueId", r.get_unique_id);
    sym("ncclCommInitRank", r.comm_init_rank);
    sym("ncclCommDestroy", r.comm_destroy);
    sym("ncclAllReduce", r.all_reduce);
    sym("ncclGetErrorString", r.error_string);
    r.ok = r.err.empty();
  });
  return r;
}

int nccl_fail(msh_ctx* c, ncclResult_t e, const char* what) {
  const Rccl& r = rccl();
  return fail(c, MSH_ERR_HIP, std::string(what) + ": " + (r.error_string ? r.error_string(e) : "rccl error"));
}

// In-place all-reduce over the ctx's communicator on stream s (nothing without one: a world of one).
int all_reduce(msh_ctx* c, void* buf, size_t count, ncclDataType_t t, ncclRedOp_t op, hipStream_t s) {
  if (!c->comm || count == 0) return MSH_OK;
  const ncclResult_t e = rccl().all_reduce(buf, buf, count, t, op, static_cast<ncclComm_t>(c->comm), s);
  return e == ncclSuccess ? MSH_OK : nccl_fail(c, e, "ncclAllReduce");
}

// The ctx's merge buffers for p pods and `ext` extent entries (a reallocation first waits, on the host,
// for the node-sharded launch in flight that may still use them).
int ensure_shard_scratch(msh_ctx* c, int32_t p, int64_t ext) {
  ShardScratch& s = c->shard;
  const bool grow_p = (size_t)p > s.pods, grow_e = (size_t)ext > s.ext;
  if (!grow_p && !grow_e) return MSH_OK;
  if (s.in_flight) MSH_HIP(c, hipEventSynchronize(s.last_ev));
  if (grow_p) {
    (void)hipFree(s.keys);
    (void)hipFree(s.total);
    (void)hipFree(s.merged);
    (void)hipFree(s.idx);
    s.keys = nullptr;
    s.total = s.merged = nullptr;
    s.idx = nullptr;
    s.pods = 0;
    const size_t cap = std::max<size_t>((size_t)p, 4096);
    MSH_HIP(c, hipMalloc(&s.keys, 2 * cap * sizeof(int32_t)));
    MSH_HIP(c, hipMalloc(&s.total, cap * sizeof(int64_t)));
    MSH_HIP(c, hipMalloc(&s.merged, cap * sizeof(int64_t)));
    MSH_HIP(c, hipMalloc(&s.idx, cap * sizeof(int32_t)));
    s.pods = cap;
  }
  if (grow_e) {
    (void)hipFree(s.ext_buf);
    s.ext_buf = nullptr;
    s.ext = 0;
    MSH_HIP(c, hipMalloc(&s.ext_buf, (size_t)ext * sizeof(int64_t)));
    s.ext = (size_t)ext;
  }
  return MSH_OK;
}

int generic_launch(msh_ctx* c, int mode, int32_t p, const int8_t* pd, const uint8_t* pt, int64_t* ext,
                   int64_t node_base, int64_t* bt, int32_t* bi, hipStream_t s) {
  msh::GenericArgs g;
  int rc = generic_args(c, g);
  if (rc != MSH_OK) return rc;
  g.nb = 1;
  g.d[0] = msh::BatchDesc{pd, pt, nullptr, nullptr, nullptr, p, 0};
  g.ext = ext;
  g.node_base = node_base;
  g.best_total = bt;
  g.best_idx = bi;
  hipError_t e;
  {
    TimedLaunch tl(c);
    e = msh::launch_generic(g, mode, c->dev, s);
  }
  return e == hipSuccess ? MSH_OK : hip_fail(c, e, "generic_kernel (node-sharded)");
}

int keys_launch(msh_ctx* c, int32_t p, const int8_t* pd, const uint8_t* pt, int64_t node_base, int32_t* keys,
                hipStream_t s) {
  msh::PairArgs a = pair_args(c);
  a.nb = 1;
  a.d[0] = msh::BatchDesc{pd, pt, nullptr, nullptr, nullptr, p, 0};
  a.keys = keys;
  a.node_base = node_base;
  hipError_t e;
  {
    TimedLaunch tl(c);
    e = msh::launch_pairs(a, true, c->dev, s);
  }
  return e == hipSuccess ? MSH_OK : hip_fail(c, e, "pair_kernel (shard keys)");
}

int64_t generic_ext_entries(const msh_ctx* c, int32_t p) {
  int64_t len = 0;
  msh_generic_ext_len(c, p, &len);
  return len;
}

// The node-sharded pipeline on stream s: shard kernel(s), all-reduce(s), decode.
int nodeshard(msh_ctx* c, int32_t p, const int8_t* pd, const uint8_t* pt, int64_t node_base, int32_t* oi,
              int64_t* os, int32_t* ost, hipStream_t s) {
  int rc = ready(c);
  if (rc != MSH_OK) return rc;
  const bool gen = use_generic(c);
  const int64_t lim = gen ? (int64_t)INT32_MAX : (int64_t)msh::GKEY_MAX;
  if (node_base < 0 || node_base + (int64_t)c->n_nodes >= lim)
    return fail(c, MSH_ERR_INVALID, "node_base outside [0, 2^31 - 1 - n)");
  if (p == 0) return MSH_OK;
  const int64_t ext = gen ? generic_ext_entries(c, p) : 0;
  if ((rc = ensure_shard_scratch(c, p, ext)) != MSH_OK) return rc;
  ShardScratch& b = c->shard;
  // one node-sharded launch of a ctx at a time on its merge buffers
  if (b.in_flight && b.last_stream != s) MSH_HIP(c, hipStreamWaitEvent(s, b.last_ev, 0));
  if (!gen) {
    if ((rc = keys_launch(c, p, pd, pt, node_base, b.keys, s)) != MSH_OK) return rc;
    if ((rc = all_reduce(c, b.keys, 2 * (size_t)p, ncclInt32, ncclMax, s)) != MSH_OK) return rc;
    const hipError_t e = msh::launch_decode_keys(pd, p, b.keys, c->pp, oi, os, ost, s);
    if (e != hipSuccess) return hip_fail(c, e, "decode_keys_kernel");
  } else {
    if (ext > 0) {
      if ((rc = generic_launch(c, 1, p, pd, pt, b.ext_buf, 0, nullptr, nullptr, s)) != MSH_OK) return rc;
      if ((rc = all_reduce(c, b.ext_buf, (size_t)ext, ncclInt64, ncclMax, s)) != MSH_OK) return rc;
    }
    if ((rc = generic_launch(c, 2, p, pd, pt, ext > 0 ? b.ext_buf : nullptr, node_base, b.total, b.idx, s)) != MSH_OK)
      return rc;
    MSH_HIP(c, hipMemcpyAsync(b.merged, b.total, (size_t)p * sizeof(int64_t), hipMemcpyDeviceToDevice, s));
    if ((rc = all_reduce(c, b.merged, (size_t)p, ncclInt64, ncclMax, s)) != MSH_OK) return rc;
    hipError_t e = msh::launch_generic_candidates(p, b.total, b.merged, b.idx, s);
    if (e != hipSuccess) return hip_fail(c, e, "generic_candidate_kernel");
    if ((rc = all_reduce(c, b.idx, (size_t)p, ncclInt32, ncclMin, s)) != MSH_OK) return rc;
    int32_t nn_score = 0;
    for (int32_t id : c->score_ids) nn_score |= id == MSH_PLUGIN_NODE_NUMBER ? 1 : 0;
    e = msh::launch_generic_decode(pd, p, b.merged, b.idx, nn_score, c->pp.nn_prescore, oi, os, ost, s);
    if (e != hipSuccess) return hip_fail(c, e, "generic_decode_kernel");
  }
  if (!b.last_ev) MSH_HIP(c, hipEventCreateWithFlags(&b.last_ev, hipEventDisableTiming));
  MSH_HIP(c, hipEventRecord(b.last_ev, s));
  b.last_stream = s;
  b.in_flight = true;
  return track_launch(c, s);
}

}  // namespace

void msh_shard_release(msh_ctx* c) {
  ShardScratch& s = c->shard;
  if (s.in_flight) (void)hipEventSynchronize(s.last_ev);
  if (s.last_ev) (void)hipEventDestroy(s.last_ev);
  (void)hipFree(s.keys);
  (void)hipFree(s.ext_buf);
  (void)hipFree(s.total);
  (void)hipFree(s.merged);
  (void)hipFree(s.idx);
  s = ShardScratch{};
  if (c->comm) (void)rccl().comm_destroy(static_cast<ncclComm_t>(c->comm));
  c->comm = nullptr;
  c->comm_world = c->comm_rank = 0;
}

// ---------------------------------------------------------------------------------------------------
// device groups
// ---------------------------------------------------------------------------------------------------
struct msh_group {
  std::string err;
  std::vector<msh_ctx*> shards;
  // per shard, on its device: the pod columns, its keys / extents / best
  struct Shard {
    int8_t* pd = nullptr;
    uint8_t* pt = nullptr;
    int32_t* keys = nullptr;
    int64_t* ext = nullptr;
    int64_t* total = nullptr;
    int32_t* idx = nullptr;
    hipEvent_t ev = nullptr;
  };
  std::vector<Shard> sh;
  size_t pods = 0, ext = 0;  // capacities
  // on the home device (shards[0]): the merged extents / best and the decisions
  int64_t* m_ext = nullptr;
  int64_t* m_total = nullptr;
  int32_t* m_idx = nullptr;
  int32_t* o_idx = nullptr;
  int64_t* o_score = nullptr;
  int32_t* o_status = nullptr;
  hipEvent_t home_ev = nullptr;
  // page-locked (portable: every device DMAs from / to it): pod columns in, decisions out
  unsigned char* h_stage = nullptr;
  size_t stage_cap = 0;
};

namespace {

thread_local std::string g_group_create_err;

int gfail(msh_group* g, int code, const std::string& msg) {
  g->err = msg;
  return code;
}

#define MSH_GHIP(g, call)                                                                                 \
  do {                                                                                                   \
    hipError_t e_ = (call);                                                                              \
    if (e_ != hipSuccess)                                                                                \
      return gfail(g, MSH_ERR_HIP, std::string(#call) + ": " + hipGetErrorName(e_) + " (" + hipGetErrorString(e_) + ")"); \
  } while (0)

void free_group_buffers(msh_group* g) {
  for (size_t k = 0; k < g->sh.size(); ++k) {
    DeviceGuard dg(g->shards[k]->device);
    msh_group::Shard& s = g->sh[k];
    (void)hipFree(s.pd);
    (void)hipFree(s.pt);
    (void)hipFree(s.keys);
    (void)hipFree(s.ext);
    (void)hipFree(s.total);
    (void)hipFree(s.idx);
    s.pd = nullptr;
    s.pt = nullptr;
    s.keys = nullptr;
    s.ext = s.total = nullptr;
    s.idx = nullptr;
  }
  DeviceGuard dg(g->shards[0]->device);
  (void)hipFree(g->m_ext);
  (void)hipFree(g->m_total);
  (void)hipFree(g->m_idx);
  (void)hipFree(g->o_idx);
  (void)hipFree(g->o_score);
  (void)hipFree(g->o_status);
  g->m_ext = g->m_total = g->o_score = nullptr;
  g->m_idx = g->o_idx = g->o_status = nullptr;
  g->pods = g->ext = 0;
}

int ensure_group_buffers(msh_group* g, int32_t p, int64_t ext) {
  if ((size_t)p <= g->pods && (size_t)ext <= g->ext) return MSH_OK;
  free_group_buffers(g);  // every group call is synchronous: nothing in flight uses them
  const size_t cap = std::max<size_t>((size_t)p, 4096), ecap = (size_t)std::max<int64_t>(ext, 0);
  for (size_t k = 0; k < g->sh.size(); ++k) {
    DeviceGuard dg(g->shards[k]->device);
    msh_group::Shard& s = g->sh[k];
    MSH_GHIP(g, hipMalloc(&s.pd, cap));
    MSH_GHIP(g, hipMalloc(&s.pt, cap));
    MSH_GHIP(g, hipMalloc(&s.keys, 2 * cap * sizeof(int32_t)));
    MSH_GHIP(g, hipMalloc(&s.total, cap * sizeof(int64_t)));
    MSH_GHIP(g, hipMalloc(&s.idx, cap * sizeof(int32_t)));
    if (ecap) MSH_GHIP(g, hipMalloc(&s.ext, ecap * sizeof(int64_t)));
  }
  DeviceGuard dg(g->shards[0]->device);
  if (ecap) MSH_GHIP(g, hipMalloc(&g->m_ext, ecap * sizeof(int64_t)));
  MSH_GHIP(g, hipMalloc(&g->m_total, cap * sizeof(int64_t)));
  MSH_GHIP(g, hipMalloc(&g->m_idx, cap * sizeof(int32_t)));
  MSH_GHIP(g, hipMalloc(&g->o_idx, cap * sizeof(int32_t)));
  MSH_GHIP(g, hipMalloc(&g->o_score, cap * sizeof(int64_t)));
  MSH_GHIP(g, hipMalloc(&g->o_status, cap * sizeof(int32_t)));
  g->pods = cap;
  g->ext = ecap;
  return MSH_OK;
}

// stage layout: digit p | tol p | idx 4p | score 8p | status 4p (16-byte aligned sections)
struct GStage {
  size_t pt, idx, score, status, total;
  explicit GStage(size_t p) {
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    pt = al(p);
    idx = pt + al(p);
    score = idx + al(4 * p);
    status = score + 8 * p;
    total = status + al(4 * p);
  }
};

bool same_plugins(const msh_ctx* a, const msh_ctx* b) {
  return a->filter_ids == b->filter_ids && a->prescore_ids == b->prescore_ids && a->score_ids == b->score_ids &&
         a->weights == b->weights && a->normalize == b->normalize && a->dev.batch_kernel == b->dev.batch_kernel;
}

// A shard ctx's error (its launch failed) surfaced on the group.
int from_shard(msh_group* g, msh_ctx* c, int rc) {
  if (rc != MSH_OK) g->err = "shard on device " + std::to_string(c->device) + ": " + c->err;
  return rc;
}

}  // namespace

extern "C" {

int msh_comm_unique_id(uint8_t* out_id) {
  if (!out_id) return MSH_ERR_INVALID;
  const Rccl& r = rccl();
  if (!r.ok) return MSH_ERR_UNSUPPORTED;
  ncclUniqueId id;
  if (r.get_unique_id(&id) != ncclSuccess) return MSH_ERR_HIP;
  std::memcpy(out_id, id.internal, MSH_COMM_ID_BYTES);
  return MSH_OK;
}

int msh_comm_init(msh_ctx* c, const uint8_t* id, int32_t world, int32_t rank) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (!id || world < 1 || rank < 0 || rank >= world) return fail(c, MSH_ERR_INVALID, "bad id / world / rank");
  if (c->comm) return fail(c, MSH_ERR_STATE, "the ctx already has a communicator");
  const Rccl& r = rccl();
  if (!r.ok) return fail(c, MSH_ERR_UNSUPPORTED, r.err);
  DeviceGuard g(c->device);  // RCCL binds the communicator to the current device
  ncclUniqueId uid;
  std::memcpy(uid.internal, id, MSH_COMM_ID_BYTES);
  ncclComm_t comm = nullptr;
  const ncclResult_t e = r.comm_init_rank(&comm, world, uid, rank);
  if (e != ncclSuccess) return nccl_fail(c, e, "ncclCommInitRank");
  c->comm = comm;
  c->comm_world = world;
  c->comm_rank = rank;
  return MSH_OK;
}

int msh_comm_info(const msh_ctx* c, int32_t* out_world, int32_t* out_rank) {
  if (!c || !out_world || !out_rank) return MSH_ERR_INVALID;
  *out_world = c->comm_world;
  *out_rank = c->comm_rank;
  return MSH_OK;
}

int msh_schedule_nodeshard_device(msh_ctx* c, int32_t p, const int8_t* d_pod_digit, const uint8_t* d_pod_tol,
                                  int64_t node_base, int32_t* d_out_idx, int64_t* d_out_score,
                                  int32_t* d_out_status, void* stream) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (p < 0) return fail(c, MSH_ERR_INVALID, "negative pod count");
  if (p > 0 && (!d_pod_digit || !d_pod_tol || !d_out_idx || !d_out_status))  // d_out_score optional
    return fail(c, MSH_ERR_INVALID, "null device pointer");
  DeviceGuard g(c->device);
  return nodeshard(c, p, d_pod_digit, d_pod_tol, node_base, d_out_idx, d_out_score, d_out_status,
                   reinterpret_cast<hipStream_t>(stream));
}

int msh_schedule_nodeshard(msh_ctx* c, int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol, int64_t node_base,
                           int32_t* out_idx, int64_t* out_score, int32_t* out_status) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (p < 0) return fail(c, MSH_ERR_INVALID, "negative pod count");
  if (p > 0 && (!pod_digit || !pod_tol || !out_idx || !out_status))  // out_score optional
    return fail(c, MSH_ERR_INVALID, "null host pointer");
  if (!c->have_nodes) return fail(c, MSH_ERR_STATE, "msh_upload_nodes has not been called");
  DeviceGuard g(c->device);
  if (p == 0) return nodeshard(c, 0, nullptr, nullptr, node_base, nullptr, nullptr, nullptr, c->stream);
  HostIO io;
  int rc = host_io_begin(c, p, pod_digit, pod_tol, out_idx, out_score, out_status, io);
  if (rc != MSH_OK) return rc;
  if ((rc = nodeshard(c, p, io.d_pd, io.d_pt, node_base, io.o_idx, io.o_score, io.o_status, c->stream)) != MSH_OK)
    return rc;
  return host_io_end(c, p, out_idx, out_score, out_status, io);
}

int msh_group_create(msh_ctx* const* shards, int32_t n, msh_group** out) {
  g_group_create_err.clear();
  if (!out) return MSH_ERR_INVALID;
  *out = nullptr;
  if (!shards || n < 1 || n > MSH_GROUP_MAX_SHARDS) {
    g_group_create_err = "1 to MSH_GROUP_MAX_SHARDS shard ctxs";
    return MSH_ERR_INVALID;
  }
  for (int32_t k = 0; k < n; ++k) {
    if (!shards[k]) {
      g_group_create_err = "null shard ctx";
      return MSH_ERR_INVALID;
    }
    for (int32_t j = 0; j < k; ++j)
      if (shards[j] == shards[k]) {
        g_group_create_err = "a ctx appears twice";
        return MSH_ERR_INVALID;
      }
  }
  // every shard's results are read on the home device, and the home's merged extents on every shard's
  const int home = shards[0]->device;
  for (int32_t k = 1; k < n; ++k) {
    const int d = shards[k]->device;
    if (d == home) continue;
    int a = 0, b = 0;
    if (hipDeviceCanAccessPeer(&a, home, d) != hipSuccess || hipDeviceCanAccessPeer(&b, d, home) != hipSuccess || !a ||
        !b) {
      g_group_create_err = "no peer access between devices " + std::to_string(home) + " and " + std::to_string(d);
      return MSH_ERR_UNSUPPORTED;
    }
    for (auto [from, to] : {std::pair<int, int>{home, d}, std::pair<int, int>{d, home}}) {
      DeviceGuard dg(from);
      const hipError_t e = hipDeviceEnablePeerAccess(to, 0);
      if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
      else if (e != hipSuccess) {
        g_group_create_err = std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorName(e);
        return MSH_ERR_HIP;
      }
    }
  }
  msh_group* g = new (std::nothrow) msh_group();
  if (!g) return MSH_ERR_NOMEM;
  g->shards.assign(shards, shards + n);
  g->sh.resize((size_t)n);
  for (int32_t k = 0; k < n; ++k) {
    DeviceGuard dg(shards[k]->device);
    if (hipEventCreateWithFlags(&g->sh[k].ev, hipEventDisableTiming) != hipSuccess) {
      msh_group_destroy(g);
      g_group_create_err = "hipEventCreateWithFlags";
      return MSH_ERR_HIP;
    }
  }
  {
    DeviceGuard dg(home);
    if (hipEventCreateWithFlags(&g->home_ev, hipEventDisableTiming) != hipSuccess) {
      msh_group_destroy(g);
      g_group_create_err = "hipEventCreateWithFlags";
      return MSH_ERR_HIP;
    }
  }
  *out = g;
  return MSH_OK;
}

void msh_group_destroy(msh_group* g) {
  if (!g) return;
  free_group_buffers(g);
  for (size_t k = 0; k < g->sh.size(); ++k)
    if (g->sh[k].ev) {
      DeviceGuard dg(g->shards[k]->device);
      (void)hipEventDestroy(g->sh[k].ev);
    }
  if (g->home_ev) {
    DeviceGuard dg(g->shards[0]->device);
    (void)hipEventDestroy(g->home_ev);
  }
  (void)hipHostFree(g->h_stage);
  delete g;
}

const char* msh_group_last_error(const msh_group* g) { return g ? g->err.c_str() : g_group_create_err.c_str(); }

int msh_group_schedule_batch(msh_group* g, int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol,
                             int32_t* out_idx, int64_t* out_score, int32_t* out_status) {
  if (!g) return MSH_ERR_INVALID;
  g->err.clear();
  if (p < 0) return gfail(g, MSH_ERR_INVALID, "negative pod count");
  if (p > 0 && (!pod_digit || !pod_tol || !out_idx || !out_status)) return gfail(g, MSH_ERR_INVALID, "null host pointer");
  const size_t n = g->shards.size();
  msh_ctx* home = g->shards[0];
  // the slices' global bases, and one plugin configuration for the whole group
  std::vector<int64_t> base(n);
  int64_t total_nodes = 0;
  for (size_t k = 0; k < n; ++k) {
    msh_ctx* c = g->shards[k];
    if (!c->have_nodes) return gfail(g, MSH_ERR_STATE, "shard " + std::to_string(k) + ": no node table uploaded");
    if (!same_plugins(c, home)) return gfail(g, MSH_ERR_STATE, "shard " + std::to_string(k) + ": other plugin lists");
    base[k] = total_nodes;
    total_nodes += c->n_nodes;
  }
  const bool gen = use_generic(home);
  if (total_nodes >= (gen ? (int64_t)INT32_MAX : (int64_t)msh::GKEY_MAX))
    return gfail(g, MSH_ERR_INVALID, "the group's node count overflows the global index");
  if (p == 0) return MSH_OK;
  const int64_t ext = gen ? generic_ext_entries(home, p) : 0;
  int rc;
  if ((rc = ensure_group_buffers(g, p, ext)) != MSH_OK) return rc;
  const GStage L((size_t)p);
  if (L.total > g->stage_cap) {
    (void)hipHostFree(g->h_stage);
    g->h_stage = nullptr;
    g->stage_cap = 0;
    MSH_GHIP(g, hipHostMalloc(reinterpret_cast<void**>(&g->h_stage), L.total, hipHostMallocPortable));
    g->stage_cap = L.total;
  }
  std::memcpy(g->h_stage, pod_digit, (size_t)p);
  std::memcpy(g->h_stage + L.pt, pod_tol, (size_t)p);
  msh::GroupPtrs gp{};
  gp.n = (int32_t)n;
  // 1. every shard: the pod columns, then its kernel (keys; or the extents of a normalizing list)
  for (size_t k = 0; k < n; ++k) {
    msh_ctx* c = g->shards[k];
    msh_group::Shard& s = g->sh[k];
    DeviceGuard dg(c->device);
    MSH_GHIP(g, hipMemcpyAsync(s.pd, g->h_stage, (size_t)p, hipMemcpyHostToDevice, c->stream));
    MSH_GHIP(g, hipMemcpyAsync(s.pt, g->h_stage + L.pt, (size_t)p, hipMemcpyHostToDevice, c->stream));
    if (!gen) rc = keys_launch(c, p, s.pd, s.pt, base[k], s.keys, c->stream);
    else if (ext > 0) rc = generic_launch(c, 1, p, s.pd, s.pt, s.ext, 0, nullptr, nullptr, c->stream);
    if ((rc = from_shard(g, c, rc)) != MSH_OK) return rc;
    MSH_GHIP(g, hipEventRecord(s.ev, c->stream));
    gp.keys[k] = s.keys;
    gp.v[k] = s.ext;
  }
  DeviceGuard dh(home->device);
  hipStream_t hs = home->stream;
  for (size_t k = 0; k < n; ++k) MSH_GHIP(g, hipStreamWaitEvent(hs, g->sh[k].ev, 0));
  const msh_group::Shard& h0 = g->sh[0];
  if (!gen) {
    // 2. the merge and decode on the home device, reading every shard's keys over the peer mapping
    MSH_GHIP(g, msh::launch_group_keys_decode(gp, h0.pd, p, home->pp, g->o_idx, g->o_score, g->o_status, hs));
  } else {
    if (ext > 0) {  // 2a. the extents' MAX, read back by every shard
      MSH_GHIP(g, msh::launch_group_max_i64(gp, ext, g->m_ext, hs));
      MSH_GHIP(g, hipEventRecord(g->home_ev, hs));
    }
    // 2b. every shard's best (total, global index) per pod
    for (size_t k = 0; k < n; ++k) {
      msh_ctx* c = g->shards[k];
      msh_group::Shard& s = g->sh[k];
      DeviceGuard dg(c->device);
      if (ext > 0) MSH_GHIP(g, hipStreamWaitEvent(c->stream, g->home_ev, 0));
      rc = generic_launch(c, 2, p, s.pd, s.pt, ext > 0 ? g->m_ext : nullptr, base[k], s.total, s.idx, c->stream);
      if ((rc = from_shard(g, c, rc)) != MSH_OK) return rc;
      MSH_GHIP(g, hipEventRecord(s.ev, c->stream));
      gp.v[k] = s.total;
      gp.idx[k] = s.idx;
    }
    for (size_t k = 0; k < n; ++k) MSH_GHIP(g, hipStreamWaitEvent(hs, g->sh[k].ev, 0));
    // 2c. the first maximum across the shards, then the decode
    MSH_GHIP(g, msh::launch_group_best_merge(gp, p, g->m_total, g->m_idx, hs));
    int32_t nn_score = 0;
    for (int32_t id : home->score_ids) nn_score |= id == MSH_PLUGIN_NODE_NUMBER ? 1 : 0;
    MSH_GHIP(g, msh::launch_generic_decode(h0.pd, p, g->m_total, g->m_idx, nn_score, home->pp.nn_prescore, g->o_idx,
                                           g->o_score, g->o_status, hs));
  }
  // 3. the decisions to the host
  MSH_GHIP(g, hipMemcpyAsync(g->h_stage + L.idx, g->o_idx, (size_t)p * 4, hipMemcpyDeviceToHost, hs));
  if (out_score) MSH_GHIP(g, hipMemcpyAsync(g->h_stage + L.score, g->o_score, (size_t)p * 8, hipMemcpyDeviceToHost, hs));
  MSH_GHIP(g, hipMemcpyAsync(g->h_stage + L.status, g->o_status, (size_t)p * 4, hipMemcpyDeviceToHost, hs));
  MSH_GHIP(g, hipStreamSynchronize(hs));
  for (size_t k = 1; k < n; ++k) {  // (every shard's work precedes the home's merge; drained for the caller)
    DeviceGuard dg(g->shards[k]->device);
    MSH_GHIP(g, hipStreamSynchronize(g->shards[k]->stream));
  }
  std::memcpy(out_idx, g->h_stage + L.idx, (size_t)p * 4);
  if (out_score) std::memcpy(out_score, g->h_stage + L.score, (size_t)p * 8);
  std::memcpy(out_status, g->h_stage + L.status, (size_t)p * 4);
  return MSH_OK;
}

}  // extern "C"
