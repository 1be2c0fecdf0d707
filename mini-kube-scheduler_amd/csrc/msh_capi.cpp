// msh_capi.cpp — implementation of include/minisched_hip.h (the drop-in C-ABI).
//
// One msh_ctx per device. The ctx owns the device-resident node table (the replacement for
// the per-cycle Nodes().List at minisched/minisched.go:40), the plugin descriptor
// (minisched/initialize.go:80-123) and the buffers of the host-buffer entry points.
// There is no CPU fallback: every schedule call runs the gfx950 kernels, and a missing
// device is an error (MSH_ERR_NO_DEVICE).
//
// Host-buffer entry points (msh_schedule_batch / msh_schedule_sequential), the path a cgo caller
// takes: the kernel reads the pod columns from and writes idx / score / status into page-locked
// host memory over PCIe (zero-copy: no DMA command and no copy after the kernel; measured at C3,
// 56.6 us per 100k-pod call against 73 us with the columns DMA'd and 97 us with everything DMA'd,
// profiles/ab/r2_e2e_host2.jsonl). When the caller's buffers are page-locked (msh_host_alloc, or
// registered with HIP) they are used as they are; otherwise the ctx stages through its own
// page-locked buffer, and the copies between the caller's memory and the stage are split over a
// small pool of host threads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <initializer_list>
#include <iterator>
#include <mutex>
#include <new>
#include <optional>
#include <string>
#include <thread>
#include <vector>

#include "../../include/minisched_hip.h"
#include "msh_ctx.h"
#include "msh_internal.h"
#include "msh_pool.h"

using msh::HostPool;
using msh::PoolLease;
using msh::PluginParams;

namespace {

struct CopyJob {
  void* dst;
  const void* src;
  size_t bytes;
};

// The copies, each split into pool.parts() contiguous pieces (64-byte aligned cuts), in ONE run of
// the process-wide pool (msh_pool.h); small totals, or no pool to lease, on the calling thread.
void par_copy(const CopyJob* jobs, int n_jobs) {
  size_t total = 0;
  for (int i = 0; i < n_jobs; ++i) total += jobs[i].bytes;
  // small copies stay on the calling thread without touching the pool (no lease, no busy flag: a
  // concurrent large pack keeps every pool thread)
  std::optional<PoolLease> lease;
  if (total >= (256u << 10)) lease.emplace();
  HostPool* pool = lease ? lease->get() : nullptr;
  if (!pool) {
    for (int i = 0; i < n_jobs; ++i) std::memcpy(jobs[i].dst, jobs[i].src, jobs[i].bytes);
    return;
  }
  const int n = pool->parts();
  pool->run([&](int k) {
    for (int i = 0; i < n_jobs; ++i) {
      const size_t b = jobs[i].bytes;
      const size_t lo = (b * k / n) & ~(size_t)63, hi = k + 1 == n ? b : (b * (k + 1) / n) & ~(size_t)63;
      if (hi > lo)
        std::memcpy(static_cast<char*>(jobs[i].dst) + lo, static_cast<const char*>(jobs[i].src) + lo, hi - lo);
    }
  });
}

}  // namespace

namespace msh::capi {

int fail(msh_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

int hip_fail(msh_ctx* c, hipError_t e, const char* what) {
  std::string m = std::string(what) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")";
  return fail(c, MSH_ERR_HIP, m);
}

NodeTable& cur_table(msh_ctx* c) { return c->tab[c->cur]; }

void free_table(NodeTable& t) {
  (void)hipFree(t.d_cols);
  (void)hipFree(t.d_unsched);
  (void)hipFree(t.d_digit);
  (void)hipFree(t.d_planes);
  t.d_cols = nullptr;
  t.d_unsched = nullptr;
  t.d_digit = nullptr;
  t.d_planes = nullptr;
  for (bool& ok : t.col_ok) ok = false;
  t.cap = 0;
}

// Host wait for the launches recorded in `evs` (their events are kept for reuse).
void wait_events(const std::vector<std::pair<hipStream_t, hipEvent_t>>& evs) {
  for (auto& e : evs) (void)hipEventSynchronize(e.second);
}

void destroy_events(std::vector<std::pair<hipStream_t, hipEvent_t>>& evs) {
  for (auto& e : evs) (void)hipEventDestroy(e.second);
  evs.clear();
}

// layout of the page-locked stage for p pods (16-byte aligned sections)
struct StageLayout {
  size_t pd, pt, idx, score, status, total;
  explicit StageLayout(size_t p) {
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    pd = 0;
    pt = al(p);
    idx = pt + al(p);
    score = idx + al(4 * p);
    status = score + 8 * p;
    total = status + al(4 * p);
  }
};

int ensure_stage(msh_ctx* c, int32_t p) {
  const size_t need = StageLayout((size_t)p).total;
  if (need > c->stage_cap) {
    (void)hipHostFree(c->h_stage);
    c->h_stage = nullptr;
    c->stage_cap = 0;
    const size_t cap = StageLayout(std::max<size_t>((size_t)p, 4096)).total;
    MSH_HIP(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_stage), cap, hipHostMallocDefault));
    c->stage_cap = cap;
  }
  return MSH_OK;
}

// Buffers from msh_host_alloc, [start, end) by start: a host-buffer call finds its page-locked
// arrays here without asking HIP (five hipPointerGetAttributes per call otherwise).
std::mutex g_host_mu;
std::vector<std::pair<uintptr_t, uintptr_t>> g_host_allocs;

bool in_host_allocs(const void* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  std::lock_guard<std::mutex> g(g_host_mu);
  auto it = std::upper_bound(g_host_allocs.begin(), g_host_allocs.end(), std::make_pair(a, UINTPTR_MAX));
  return it != g_host_allocs.begin() && a < std::prev(it)->second;
}

// Device-visible address of page-locked host memory (msh_host_alloc'd: the same address, as for
// any hipHostMalloc memory; otherwise hipHostRegister'ed, asked of HIP), or nullptr for pageable
// memory. A failed query is not an error of the call: it is cleared so that the next launch's
// hipGetLastError does not report it.
void* pinned_device_ptr(const void* p) {
  if (in_host_allocs(p)) return const_cast<void*>(p);
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (at.type != hipMemoryTypeHost || !at.devicePointer) return nullptr;
  return at.devicePointer;
}

bool contains(const std::vector<int32_t>& v, int32_t id) {
  return std::find(v.begin(), v.end(), id) != v.end();
}

bool is_column(int32_t id) { return id >= MSH_PLUGIN_SCORE_COLUMN0 && id < MSH_PLUGIN_SCORE_COLUMN0 + msh::GEN_COLS; }

// kind: 0 filter list, 1 prescore list, 2 score list
int check_ids(msh_ctx* c, const int32_t* ids, int32_t n, int kind, const char* what) {
  if (n < 0 || n > 8) return fail(c, MSH_ERR_INVALID, std::string(what) + ": bad list length");
  if (n > 0 && !ids) return fail(c, MSH_ERR_INVALID, std::string(what) + ": null list");
  for (int32_t i = 0; i < n; i++) {
    const int32_t id = ids[i];
    const bool ok = kind == 0 ? id == MSH_PLUGIN_NODE_UNSCHEDULABLE
                              : (id == MSH_PLUGIN_NODE_NUMBER || (kind == 2 && is_column(id)));
    if (!ok)
      return fail(c, MSH_ERR_UNSUPPORTED,
                  std::string(what) + ": plugin id " + std::to_string(id) + " has no device implementation");
    for (int32_t k = 0; k < i; k++)
      if (ids[k] == id) return fail(c, MSH_ERR_INVALID, std::string(what) + ": duplicate plugin id");
  }
  return MSH_OK;
}

// After a *_device launch on caller stream s: (re-)record the ctx's event for s. One event per
// stream the ctx has launched on (a linear search: callers use a handful of streams).
// The events only say that launches finished (a table version or the counts may then be rewritten on
// the device, or freed): no host reads what those launches wrote through them, so they are recorded
// without the system-scope fence (hipEventDisableSystemFence; a kernel's own end-of-kernel release at
// agent scope writes back L2 on gfx950). With the fence each record put ~5 us on the stream: one-batch
// launches back to back 12-14 -> 8-9.5 us each, profiles/ab/r6_event_fence.txt.
int record_on(msh_ctx* c, std::vector<std::pair<hipStream_t, hipEvent_t>>& evs, hipStream_t s,
              hipEvent_t* out = nullptr) {
  for (auto& e : evs)
    if (e.first == s) {
      MSH_HIP(c, hipEventRecord(e.second, s));
      if (out) *out = e.second;
      return MSH_OK;
    }
  hipEvent_t ev = nullptr;
  MSH_HIP(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventDisableSystemFence));
  hipError_t e = hipEventRecord(ev, s);
  if (e != hipSuccess) {
    (void)hipEventDestroy(ev);
    return hip_fail(c, e, "hipEventRecord");
  }
  evs.emplace_back(s, ev);
  if (out) *out = ev;
  return MSH_OK;
}

// After a launch on caller stream s that reads the current table version (seq: and updates the
// sequential-mode counts). One record per launch: a sequential launch's entry in seq_inflight is the
// table version's reader event for s itself (a non-owning alias; the readers' events live until
// msh_destroy, and a later record of the same event on s only marks a later point of the stream).
int track_launch(msh_ctx* c, hipStream_t s, bool seq) {
  hipEvent_t ev = nullptr;
  int rc = record_on(c, cur_table(c).readers, s, &ev);
  if (rc != MSH_OK || !seq) return rc;
  for (auto& e : c->seq_inflight)
    if (e.first == s) {
      e.second = ev;
      return MSH_OK;
    }
  c->seq_inflight.emplace_back(s, ev);
  return MSH_OK;
}

// Order prep_stream after the sequential launches in flight (device-side waits): they update the
// counts that a count read, reset or re-upload touches next.
int after_seq(msh_ctx* c) {
  for (auto& e : c->seq_inflight) MSH_HIP(c, hipStreamWaitEvent(c->prep_stream, e.second, 0));
  return MSH_OK;
}

// The page-locked node staging buffer, at least `bytes` long. Every rewrite finishes its copies
// before returning (it synchronizes prep_stream), so the buffer is free on entry.
int node_stage(msh_ctx* c, size_t bytes) {
  if (bytes <= c->nstage_cap) return MSH_OK;
  (void)hipHostFree(c->h_nstage);
  c->h_nstage = nullptr;
  c->nstage_cap = 0;
  const size_t cap = std::max<size_t>(bytes, 4096);
  MSH_HIP(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_nstage), cap, hipHostMallocDefault));
  c->nstage_cap = cap;
  return MSH_OK;
}

// A node table version with room for n_pad nodes (a reallocation first waits for its readers).
int ensure_table(msh_ctx* c, NodeTable& t, size_t n_pad) {
  if (t.cap >= n_pad && t.d_planes) return MSH_OK;
  wait_events(t.readers);
  free_table(t);
  MSH_HIP(c, hipMalloc(&t.d_unsched, n_pad));
  MSH_HIP(c, hipMalloc(&t.d_digit, n_pad));
  MSH_HIP(c, hipMalloc(&t.d_planes, n_pad / msh::GROUP_NODES * msh::GROUP_DWORDS * sizeof(uint32_t)));
  t.cap = n_pad;
  return MSH_OK;
}

// The zero fill goes on prep_stream, ahead of the column copies queued there: a plain hipMemset runs
// on the null stream, which a non-blocking prep_stream does not order against (the fill landed
// after the first column upload and zeroed it).
int ensure_cols(msh_ctx* c, NodeTable& t) {
  if (!t.d_cols) {
    MSH_HIP(c, hipMalloc(&t.d_cols, (size_t)msh::GEN_COLS * t.cap * sizeof(int64_t)));
    MSH_HIP(c, hipMemsetAsync(t.d_cols, 0, (size_t)msh::GEN_COLS * t.cap * sizeof(int64_t), c->prep_stream));
  }
  return MSH_OK;
}

// What a rewrite changes relative to the published version.
struct Rewrite {
  enum Kind { UPLOAD, PATCH, REPREP, COLUMN } kind;
  int32_t n = 0;                    // UPLOAD: the new node count and columns
  const uint8_t* unsched = nullptr;
  const int8_t* digit = nullptr;
  int32_t patch_count = 0;          // PATCH: entries in c->h_patch
  int col = -1;                     // COLUMN: column k and its n scores
  const int64_t* scores = nullptr;
};

// Build the unpublished table version from the published one (or from the upload) on prep_stream,
// wait for that work alone, and publish it. Launches in flight keep reading the old version.
int rewrite(msh_ctx* c, const Rewrite& w) {
  const int s = 1 - c->cur;
  NodeTable& src = c->tab[c->cur];
  NodeTable& dst = c->tab[s];
  hipStream_t ps = c->prep_stream;
  const bool up = w.kind == Rewrite::UPLOAD;
  const int32_t n = up ? w.n : c->n_nodes;
  // Padded to whole 1,024-node blocks, and never empty: an empty cluster is a table of padding
  // slots (infeasible for every pod), so every pod gets FitError from the kernel.
  const int32_t n_pad = std::max(((n + msh::NODE_PAD - 1) / msh::NODE_PAD) * msh::NODE_PAD, msh::NODE_PAD);
  // the version overwritten here was last read by launches of two rewrites ago
  wait_events(dst.readers);
  int rc = ensure_table(c, dst, (size_t)n_pad);
  if (rc != MSH_OK) return rc;
  hipError_t e = hipSuccess;
  // the uploaded columns and the planes: uploaded and prepped, or copied from the published version (a
  // patch of at most PATCH_INLINE nodes applied on the way, its words' planes rebuilt)
  const bool inline_patch = w.kind == Rewrite::PATCH && w.patch_count <= msh::PATCH_INLINE;
  if (up) {
    if (n > 0) {
      if ((rc = node_stage(c, 2 * (size_t)n)) != MSH_OK) return rc;
      std::memcpy(c->h_nstage, w.unsched, (size_t)n);
      std::memcpy(c->h_nstage + n, w.digit, (size_t)n);
      MSH_HIP(c, hipMemcpyAsync(dst.d_unsched, c->h_nstage, (size_t)n, hipMemcpyHostToDevice, ps));
      MSH_HIP(c, hipMemcpyAsync(dst.d_digit, c->h_nstage + n, (size_t)n, hipMemcpyHostToDevice, ps));
    }
  } else {
    msh::TableCopyArgs t{};
    t.src_unsched = src.d_unsched;
    t.src_digit = src.d_digit;
    t.src_planes = src.d_planes;
    t.dst_unsched = dst.d_unsched;
    t.dst_digit = dst.d_digit;
    t.dst_planes = dst.d_planes;
    t.n = n;
    t.n_words = n_pad / 32;
    t.has_nu = c->pp.has_nu_filter;
    if (inline_patch) {
      t.count = w.patch_count;
      std::copy(c->h_patch.begin(), c->h_patch.begin() + w.patch_count, t.inl);
    }
    if ((e = msh::launch_table_copy(t, ps)) != hipSuccess) return hip_fail(c, e, "table_copy_kernel");
  }
  // score columns: an upload drops them (they belong to the previous table's nodes)
  for (int k = 0; k < msh::GEN_COLS; ++k) {
    dst.col_ok[k] = !up && src.col_ok[k];
    dst.col_lo[k] = src.col_lo[k];
    dst.col_hi[k] = src.col_hi[k];
    if (w.kind == Rewrite::COLUMN && k == w.col) continue;
    if (dst.col_ok[k] && n > 0) {
      if ((rc = ensure_cols(c, dst)) != MSH_OK) return rc;
      MSH_HIP(c, hipMemcpyAsync(dst.d_cols + (size_t)k * dst.cap, src.d_cols + (size_t)k * src.cap,
                                (size_t)n * sizeof(int64_t), hipMemcpyDeviceToDevice, ps));
    }
  }
  if (w.kind == Rewrite::COLUMN) {
    if ((rc = ensure_cols(c, dst)) != MSH_OK) return rc;
    int64_t lo = 0, hi = 0;
    if (n > 0) {
      const size_t bytes = (size_t)n * sizeof(int64_t);
      if ((rc = node_stage(c, bytes)) != MSH_OK) return rc;
      std::memcpy(c->h_nstage, w.scores, bytes);
      MSH_HIP(c, hipMemcpyAsync(dst.d_cols + (size_t)w.col * dst.cap, c->h_nstage, bytes, hipMemcpyHostToDevice, ps));
      const auto mm = std::minmax_element(w.scores, w.scores + n);
      lo = *mm.first;
      hi = *mm.second;
    }
    dst.col_ok[w.col] = true;
    dst.col_lo[w.col] = lo;
    dst.col_hi[w.col] = hi;
  }
  // a larger patch: its entries scattered into the copied columns, then the full prep below
  if (w.kind == Rewrite::PATCH && !inline_patch) {
    const size_t pbytes = (size_t)w.patch_count * sizeof(unsigned long long);
    if ((size_t)w.patch_count > c->patch_cap) {
      (void)hipFree(c->d_patch);  // last read by a rewrite that has completed
      c->d_patch = nullptr;
      c->patch_cap = 0;
      const size_t cap = std::max<size_t>((size_t)w.patch_count, 256);
      MSH_HIP(c, hipMalloc(&c->d_patch, cap * sizeof(unsigned long long)));
      c->patch_cap = cap;
    }
    if ((rc = node_stage(c, pbytes)) != MSH_OK) return rc;
    std::memcpy(c->h_nstage, c->h_patch.data(), pbytes);
    MSH_HIP(c, hipMemcpyAsync(c->d_patch, c->h_nstage, pbytes, hipMemcpyHostToDevice, ps));
    if ((e = msh::launch_patch_scatter(c->d_patch, w.patch_count, dst.d_unsched, dst.d_digit, ps)) != hipSuccess)
      return hip_fail(c, e, "patch_scatter_kernel");
  }
  // the planes: rebuilt whole after an upload, a filter-list change or a large patch; a small patch and a
  // score column leave the copied (patched) planes as they are
  if (up || w.kind == Rewrite::REPREP || (w.kind == Rewrite::PATCH && !inline_patch)) {
    if ((e = msh::launch_node_prep(dst.d_unsched, dst.d_digit, n, n_pad, c->pp.has_nu_filter, dst.d_planes, ps)) !=
        hipSuccess)
      return hip_fail(c, e, "node_prep_kernel");
  }
  // an upload zeroes the sequential-mode counts (after the sequential launches in flight)
  if (up) {
    const int32_t replicas = n_pad <= msh::SEQ_SPLIT_MAX_NODES ? msh::SEQ_COUNT_REPLICAS : 1;
    if ((size_t)n_pad > c->counts_cap || replicas > c->counts_replicas) {
      wait_events(c->seq_inflight);
      (void)hipFree(c->d_counts);
      c->d_counts = nullptr;
      c->counts_cap = 0;
      c->counts_replicas = 1;
      MSH_HIP(c, hipMalloc(&c->d_counts, (size_t)replicas * (size_t)n_pad * sizeof(int32_t)));
      c->counts_cap = (size_t)n_pad;
      c->counts_replicas = replicas;
    }
    if ((rc = after_seq(c)) != MSH_OK) return rc;
    MSH_HIP(c, hipMemsetAsync(c->d_counts, 0, (size_t)c->counts_replicas * c->counts_cap * sizeof(int32_t), ps));
    c->counts_dirty = false;
  }
  MSH_HIP(c, hipStreamSynchronize(ps));
  c->cur = s;
  c->n_nodes = n;
  c->n_pad = n_pad;
  c->have_nodes = true;
  return MSH_OK;
}

TimedLaunch::TimedLaunch(msh_ctx* ctx) : c(ctx) {
  if (c->timing && c->t_next < c->tev.size()) {
    msh::set_launch_events(c->tev[c->t_next].first, c->tev[c->t_next].second);
    armed = true;
  }
}

TimedLaunch::~TimedLaunch() {
  if (!armed) return;
  if (msh::launch_events_pending()) msh::set_launch_events(nullptr, nullptr);
  else ++c->t_next;
}

int ready(msh_ctx* c) {
  if (!c->have_nodes) return fail(c, MSH_ERR_STATE, "msh_upload_nodes has not been called");
  return MSH_OK;
}

msh::PairArgs pair_args(msh_ctx* c) {
  msh::PairArgs a{};
  const NodeTable& t = cur_table(c);
  a.planes = t.d_planes;
  a.n_groups = c->n_pad / msh::GROUP_NODES;
  a.g_full = c->n_nodes / msh::GROUP_NODES;
  a.pp = c->pp;
  return a;
}

// nb batches on the per-pair kernel, MULTI_MAX per launch.
int launch_generic_descs(msh_ctx* c, const msh::BatchDesc* d, int32_t nb, hipStream_t s);
bool use_generic(const msh_ctx* c);

int launch_batch_descs(msh_ctx* c, const msh::BatchDesc* d, int32_t nb, hipStream_t s) {
  if (use_generic(c)) return launch_generic_descs(c, d, nb, s);
  for (int32_t i0 = 0; i0 < nb; i0 += msh::MULTI_MAX) {
    const int n = std::min<int32_t>(msh::MULTI_MAX, nb - i0);
    TimedLaunch tl(c);
    msh::PairArgs a = pair_args(c);
    a.nb = n;
    for (int k = 0; k < n; ++k) a.d[k] = d[i0 + k];
    const hipError_t e = msh::launch_pairs(a, false, c->dev, s);
    if (e != hipSuccess) return hip_fail(c, e, "pair_kernel");
  }
  return MSH_OK;
}

// The generic pipeline runs the batch entry points when the score list names a score column (or
// for every list with MSH_BATCH_KERNEL=generic, an A/B switch).
bool use_generic(const msh_ctx* c) { return c->generic || c->dev.batch_kernel == 1; }

// The largest |NormalizeScore(raw)| one plugin can give a feasible pair: NodeNumber's raw
// scores are 0 / 10; a column's raw scores lie in [lo, hi] (its upload). DefaultNormalizeScore gives
// 100 raw / m with m = the largest feasible raw (raw unchanged when m <= 0); reverse 100 - that;
// min-max [0, 100].
long double score_bound(bool column, int32_t mode, int64_t lo, int64_t hi) {
  const long double alo = lo < 0 ? -(long double)lo : (long double)lo, ahi = hi < 0 ? -(long double)hi : (long double)hi;
  switch (mode) {
    case MSH_NORMALIZE_DEFAULT: return !column || lo >= 0 ? 100.0L : std::max(100.0L, 100.0L * alo);
    case MSH_NORMALIZE_DEFAULT_REVERSE: return !column || lo >= 0 ? 100.0L : 100.0L + 100.0L * alo;
    case MSH_NORMALIZE_MINMAX: return 100.0L;
    default: return column ? std::max(alo, ahi) : 10.0L;
  }
}

int generic_args(msh_ctx* c, msh::GenericArgs& g) {
  g = msh::GenericArgs{};
  const NodeTable& t = cur_table(c);
  g.unsched = t.d_unsched;
  g.digit = t.d_digit;
  g.cols = t.d_cols;
  g.col_stride = (int64_t)t.cap;
  g.n_nodes = c->n_nodes;
  g.has_nu = c->pp.has_nu_filter;
  g.nn_prescore = c->pp.nn_prescore;
  long double bound = 0;  // the largest |total| a feasible pair can reach
  bool c24 = true;        // every normalizing column's weight and normalized score below 2^23 in magnitude
  for (size_t k = 0; k < c->score_ids.size(); ++k) {
    const int32_t id = c->score_ids[k];
    const int32_t mode = c->normalize[k];
    const int64_t w = c->weights[k];
    if (id == MSH_PLUGIN_NODE_NUMBER) {
      g.nn_score = 1;
      g.nn_mode = mode;
      g.nn_weight = w;
      bound += (long double)w * score_bound(false, mode, 0, 10);
    } else {
      const int32_t col = id - MSH_PLUGIN_SCORE_COLUMN0;
      if (!t.col_ok[col])
        return fail(c, MSH_ERR_STATE, "score column " + std::to_string(id) + " not uploaded since the last node upload");
      if (mode != MSH_NORMALIZE_NONE) {
        g.ncc[g.nnc] = col;
        g.npos[g.nnc] = g.ncol;
        g.nmode[g.nnc] = mode;
        g.nw[g.nnc] = w;
        ++g.nnc;
      } else {
        g.tcc[g.nts] = col;
        g.tw[g.nts] = w;
        ++g.nts;
      }
      ++g.ncol;
      const long double sb = score_bound(true, mode, t.col_lo[col], t.col_hi[col]);
      bound += (long double)w * sb;
      // c24 is what keeps col_term<KT = 0>'s __mul24 operands (weight, normalized score) inside the signed
      // 24-bit range (msh_generic.hip); any other term multiplied there must be checked here too
      if (mode != MSH_NORMALIZE_NONE) c24 = c24 && w < (1 << 23) && sb < (long double)(1 << 23);
    }
    g.need_ext = g.need_ext || mode != MSH_NORMALIZE_NONE;
  }
  // 32-bit totals when every feasible pair's total is bounded away from +-2^31 (biased by 2^31, the
  // key of a feasible pair is then never 0, the infeasible key) and each normalizing column's term is a
  // 24-bit signed product; otherwise Go's int64
  g.w64 = bound > (long double)(((int64_t)1 << 31) - 2) || !c24 ? 1 : 0;
  // totals below 2^53 in magnitude: every term and partial sum is an integer a double holds exactly, so
  // the 8-byte keys (64-bit totals, or the general form) are the totals as doubles (MSH_GEN_F53=0: uint64_t)
  g.f53 = c->dev.gen_f53 && bound <= (long double)(((int64_t)1 << 53) - 2) ? 1 : 0;
  // NodeNumber's key without a compare (base + bit * delta on the 24-bit multiplier) when weight*100 fits
  g.nn24 = c->dev.gen_nnkey && (!g.nn_score || (long double)g.nn_weight * 100.0L < (long double)(1 << 24)) ? 1 : 0;
  return MSH_OK;
}

// nb batches on generic_kernel, MULTI_MAX per launch.
int launch_generic_descs(msh_ctx* c, const msh::BatchDesc* d, int32_t nb, hipStream_t s) {
  msh::GenericArgs g;
  int rc = generic_args(c, g);
  if (rc != MSH_OK) return rc;
  for (int32_t i0 = 0; i0 < nb; i0 += msh::MULTI_MAX) {
    g.nb = std::min<int32_t>(msh::MULTI_MAX, nb - i0);
    for (int k = 0; k < g.nb; ++k) g.d[k] = d[i0 + k];
    TimedLaunch tl(c);
    hipError_t e = msh::launch_generic(g, 0, c->dev, s);
    if (e != hipSuccess) return hip_fail(c, e, "generic_kernel");
  }
  return MSH_OK;
}

int host_io_begin(msh_ctx* c, int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol, int32_t* out_idx,
                  int64_t* out_score, int32_t* out_status, HostIO& io) {
  int rc = MSH_OK;
  // out_score is optional (NULL: scores not written, 8 B per pod less over PCIe)
  void* di = pinned_device_ptr(out_idx);
  void* ds = (di && out_score) ? pinned_device_ptr(out_score) : nullptr;
  const bool score_ok = !out_score || ds;
  void* dt = (di && score_ok) ? pinned_device_ptr(out_status) : nullptr;
  const bool in_pinned = pinned_device_ptr(pod_digit) && pinned_device_ptr(pod_tol);
  io.staged = !(di && score_ok && dt);
  if (io.staged || !in_pinned) {
    if ((rc = ensure_stage(c, p)) != MSH_OK) return rc;
  }
  const StageLayout L((size_t)p);
  const int8_t* src_pd = pod_digit;
  const uint8_t* src_pt = pod_tol;
  if (!in_pinned) {  // through the stage
    const CopyJob jobs[2] = {{c->h_stage + L.pd, pod_digit, (size_t)p}, {c->h_stage + L.pt, pod_tol, (size_t)p}};
    par_copy(jobs, 2);
    src_pd = reinterpret_cast<const int8_t*>(c->h_stage + L.pd);
    src_pt = c->h_stage + L.pt;
  }
  // the kernel reads the page-locked columns itself (zero-copy: no DMA command; 56.6 us per C3 call
  // against 73 us with the columns DMA'd, profiles/ab/r2_e2e_host2.jsonl)
  io.d_pd = static_cast<int8_t*>(pinned_device_ptr(src_pd));
  io.d_pt = static_cast<uint8_t*>(pinned_device_ptr(src_pt));
  if (!io.d_pd || !io.d_pt) return fail(c, MSH_ERR_HIP, "page-locked pod columns without a device address");
  if (io.staged) {
    io.h_idx = reinterpret_cast<int32_t*>(c->h_stage + L.idx);
    io.h_score = out_score ? reinterpret_cast<int64_t*>(c->h_stage + L.score) : nullptr;
    io.h_status = reinterpret_cast<int32_t*>(c->h_stage + L.status);
    io.o_idx = io.h_idx;  // hipHostMalloc memory: the host pointer is valid on the device too
    io.o_score = io.h_score;
    io.o_status = io.h_status;
  } else {
    io.h_idx = out_idx;
    io.h_score = out_score;
    io.h_status = out_status;
    io.o_idx = static_cast<int32_t*>(di);
    io.o_score = static_cast<int64_t*>(ds);
    io.o_status = static_cast<int32_t*>(dt);
  }
  return MSH_OK;
}

int host_io_end(msh_ctx* c, int32_t p, int32_t* out_idx, int64_t* out_score, int32_t* out_status,
                const HostIO& io) {
  MSH_HIP(c, hipStreamSynchronize(c->stream));
  c->async_done = c->async_issued;  // the ctx's stream is drained: every async batch is done too
  if (io.staged) {
    const CopyJob jobs[3] = {{out_idx, io.h_idx, (size_t)p * sizeof(int32_t)},
                             {out_status, io.h_status, (size_t)p * sizeof(int32_t)},
                             {out_score, io.h_score, (size_t)p * sizeof(int64_t)}};
    par_copy(jobs, out_score ? 3 : 2);
  }
  return MSH_OK;
}

// The message of the last failed msh_create on this thread (msh_last_error(NULL)).
thread_local std::string g_create_err;

// msh_create_ex's options into the ctx's launch choices: every field's 0 is the automatic choice, a
// value outside a field's set fails with a message (never mapped to another setting).
bool apply_options(const msh_options& o, msh::DeviceInfo& d, std::string* err) {
  auto in = [&](const char* name, int32_t v, std::initializer_list<int32_t> allowed) {
    for (int32_t a : allowed)
      if (v == a) return true;
    *err = std::string("msh_options.") + name + " = " + std::to_string(v) + ": not one of";
    for (int32_t a : allowed) *err += " " + std::to_string(a);
    return false;
  };
  if (!in("batch_kernel", o.batch_kernel, {0, 1}) || !in("pair_planes", o.pair_planes, {0, 1, 2}) ||
      !in("pair_noax", o.pair_noax, {0, 1, 2}) || !in("pair_slices", o.pair_slices, {0, 1, 2, 4}) ||
      !in("seq_waves", o.seq_waves, {0, 1, 4, 15, 16}) || !in("seq_split", o.seq_split, {0, 1, 2}) ||
      !in("seq_pod_waves", o.seq_pod_waves, {0, 1, 2, 4, 8}) ||
      !in("gen_keys", o.gen_keys, {0, 1}) || !in("gen_nnkey", o.gen_nnkey, {0, 1}))
    return false;
  d.batch_kernel = o.batch_kernel;
  d.pair_planes = o.pair_planes;
  d.pair_noax = o.pair_noax == 0 ? -1 : (o.pair_noax == 1 ? 1 : 0);
  d.bits_slices = o.pair_slices;
  d.seq_waves = o.seq_waves;
  d.seq_split = o.seq_split == 0 ? 2 : (o.seq_split == 1 ? 0 : 1);
  d.seq_pod_waves = o.seq_pod_waves;
  d.gen_f53 = o.gen_keys == 0 ? 1 : 0;
  d.gen_nnkey = o.gen_nnkey == 0 ? 1 : 0;
  return true;
}

}  // namespace msh::capi

using namespace msh::capi;

extern "C" {

int msh_abi_version(void) { return MSH_ABI_VERSION; }

int msh_device_count(int* out_count) {
  if (!out_count) return MSH_ERR_INVALID;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  *out_count = (e == hipSuccess) ? n : 0;
  return MSH_OK;
}

int msh_host_alloc(size_t bytes, void** out_ptr) {
  if (!out_ptr) return MSH_ERR_INVALID;
  *out_ptr = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return MSH_ERR_NO_DEVICE;
  const size_t n_bytes = std::max<size_t>(bytes, 1);
  if (hipHostMalloc(out_ptr, n_bytes, hipHostMallocDefault) != hipSuccess) {
    *out_ptr = nullptr;
    return MSH_ERR_NOMEM;
  }
  const uintptr_t a = reinterpret_cast<uintptr_t>(*out_ptr);
  std::lock_guard<std::mutex> g(g_host_mu);
  g_host_allocs.insert(std::upper_bound(g_host_allocs.begin(), g_host_allocs.end(), std::make_pair(a, a)),
                       std::make_pair(a, a + n_bytes));
  return MSH_OK;
}

void msh_host_free(void* ptr) {
  if (!ptr) return;
  {
    const uintptr_t a = reinterpret_cast<uintptr_t>(ptr);
    std::lock_guard<std::mutex> g(g_host_mu);
    auto it = std::lower_bound(g_host_allocs.begin(), g_host_allocs.end(), std::make_pair(a, (uintptr_t)0));
    if (it != g_host_allocs.end() && it->first == a) g_host_allocs.erase(it);
  }
  (void)hipHostFree(ptr);
}

int msh_create(int device, msh_ctx** out_ctx) { return msh_create_ex(device, nullptr, out_ctx); }

int msh_create_ex(int device, const msh_options* opts, msh_ctx** out_ctx) {
  g_create_err.clear();
  if (!out_ctx) return MSH_ERR_INVALID;
  *out_ctx = nullptr;
  msh::DeviceInfo info;
  if (opts) {
    // kernel-selection overrides (tests / A-B), resolved here once, never on a launch path
    if (opts->struct_size != (int32_t)sizeof(msh_options)) {
      g_create_err = "msh_options.struct_size != sizeof(msh_options)";
      return MSH_ERR_INVALID;
    }
    if (!apply_options(*opts, info, &g_create_err)) return MSH_ERR_INVALID;
  }
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return MSH_ERR_NO_DEVICE;
  if (device < 0 || device >= n) return MSH_ERR_NO_DEVICE;
  DeviceGuard g(device);
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess || cur != device) return MSH_ERR_NO_DEVICE;
  msh_ctx* c = new (std::nothrow) msh_ctx();
  if (!c) return MSH_ERR_NOMEM;
  c->device = device;
  c->dev = info;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    c->dev.cus = prop.multiProcessorCount;
  int lo_prio = 0, hi_prio = 0;  // numerically lower = higher priority
  if (hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio) != hipSuccess) hi_prio = 0;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithPriority(&c->prep_stream, hipStreamNonBlocking, hi_prio) != hipSuccess) {
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return MSH_ERR_HIP;
  }
  // Reference plugin set (minisched/initialize.go:80-123).
  c->filter_ids = {MSH_PLUGIN_NODE_UNSCHEDULABLE};
  c->prescore_ids = {MSH_PLUGIN_NODE_NUMBER};
  c->score_ids = {MSH_PLUGIN_NODE_NUMBER};
  c->weights = {1};
  c->normalize = {MSH_NORMALIZE_NONE};
  c->pp = PluginParams{1, 1, 1, MSH_NORMALIZE_NONE, 1};
  *out_ctx = c;
  return MSH_OK;
}

void msh_destroy(msh_ctx* c) {
  if (!c) return;
  DeviceGuard g(c->device);
  // launches this ctx queued on caller streams (the *_device entry points) may still read the tables
  for (NodeTable& t : c->tab) wait_events(t.readers);
  wait_events(c->seq_inflight);
  msh_shard_release(c);  // its node-sharded launch in flight, merge buffers and communicator
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->prep_stream) (void)hipStreamSynchronize(c->prep_stream);
  for (NodeTable& t : c->tab) {
    destroy_events(t.readers);
    free_table(t);
  }
  c->seq_inflight.clear();  // aliases of the readers' events (destroyed above)
  (void)hipFree(c->d_counts);
  for (hipEvent_t e : c->async_ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->tev) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  (void)hipHostFree(c->h_stage);
  (void)hipHostFree(c->h_nstage);
  (void)hipFree(c->d_patch);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->prep_stream) (void)hipStreamDestroy(c->prep_stream);
  delete c;
}

const char* msh_last_error(const msh_ctx* c) { return c ? c->err.c_str() : g_create_err.c_str(); }

int msh_set_plugins_ex(msh_ctx* c, const int32_t* filter_ids, int32_t nf,
                       const int32_t* prescore_ids, int32_t npre, const int32_t* score_ids,
                       const int64_t* weights, const int32_t* normalize, int32_t ns) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  int rc;
  if ((rc = check_ids(c, filter_ids, nf, 0, "filter")) != MSH_OK) return rc;
  if ((rc = check_ids(c, prescore_ids, npre, 1, "prescore")) != MSH_OK) return rc;
  if ((rc = check_ids(c, score_ids, ns, 2, "score")) != MSH_OK) return rc;
  for (int32_t i = 0; i < ns; i++) {
    const int64_t w = weights ? weights[i] : 1;
    if (w < 1 || w > (int64_t(1) << 32)) return fail(c, MSH_ERR_INVALID, "score weight outside [1, 2^32]");
    const int32_t m = normalize ? normalize[i] : MSH_NORMALIZE_NONE;
    if (m < MSH_NORMALIZE_NONE || m > MSH_NORMALIZE_MINMAX) return fail(c, MSH_ERR_INVALID, "bad normalize mode");
  }
  std::vector<int32_t> f_ids(filter_ids, filter_ids + nf), p_ids(prescore_ids, prescore_ids + npre),
      s_ids(score_ids, score_ids + ns), norms;
  std::vector<int64_t> ws;
  for (int32_t i = 0; i < ns; i++) {
    ws.push_back(weights ? weights[i] : 1);
    norms.push_back(normalize ? normalize[i] : MSH_NORMALIZE_NONE);
  }
  PluginParams pp{};
  pp.has_nu_filter = contains(f_ids, MSH_PLUGIN_NODE_UNSCHEDULABLE) ? 1 : 0;
  pp.nn_prescore = contains(p_ids, MSH_PLUGIN_NODE_NUMBER) ? 1 : 0;
  pp.has_nn_score = 0;
  pp.mode = MSH_NORMALIZE_NONE;
  pp.weight = 1;
  bool generic = false;
  for (int32_t i = 0; i < ns; i++) {
    if (s_ids[i] == MSH_PLUGIN_NODE_NUMBER) {
      pp.has_nn_score = 1;
      pp.mode = norms[i];
      pp.weight = ws[i];
    }
    generic = generic || is_column(s_ids[i]);
  }
  // The filter planes depend on the filter list: rebuild the table first, and publish the new plugin
  // set only once the rebuild succeeded (a failed rebuild leaves the old set with its old table).
  if (pp.has_nu_filter != c->pp.has_nu_filter && c->have_nodes) {
    const PluginParams old = c->pp;
    c->pp = pp;  // rewrite() builds the X plane and the node records from c->pp
    DeviceGuard g(c->device);
    Rewrite w{Rewrite::REPREP};
    const int rc2 = rewrite(c, w);
    if (rc2 != MSH_OK) {
      c->pp = old;
      return rc2;
    }
  }
  c->filter_ids = std::move(f_ids);
  c->prescore_ids = std::move(p_ids);
  c->score_ids = std::move(s_ids);
  c->weights = std::move(ws);
  c->normalize = std::move(norms);
  c->pp = pp;
  c->generic = generic;
  return MSH_OK;
}

int msh_set_plugins(msh_ctx* c, const int32_t* filter_ids, int32_t nf, const int32_t* score_ids,
                    const int64_t* weights, int32_t ns) {
  // NodeNumber implements PreScore too (nodenumber.go:50), so it is its own prescore plugin.
  std::vector<int32_t> pre;
  for (int32_t i = 0; i < ns && score_ids; i++)
    if (score_ids[i] == MSH_PLUGIN_NODE_NUMBER) pre.push_back(score_ids[i]);
  return msh_set_plugins_ex(c, filter_ids, nf, pre.data(), (int32_t)pre.size(), score_ids, weights,
                            nullptr, ns);
}

int msh_upload_nodes(msh_ctx* c, int32_t n, const uint8_t* unsched, const int8_t* digit) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (n < 0 || n > msh::MAX_NODES) return fail(c, MSH_ERR_INVALID, "node count outside [0, 2^24-2]");
  if (n > 0 && (!unsched || !digit)) return fail(c, MSH_ERR_INVALID, "null node arrays");
  DeviceGuard g(c->device);
  Rewrite w{Rewrite::UPLOAD};
  w.n = n;
  w.unsched = unsched;
  w.digit = digit;
  return rewrite(c, w);  // synchronous; launches in flight keep the previous version
}

int msh_patch_nodes(msh_ctx* c, int32_t count, const int32_t* idx, const uint8_t* unsched,
                    const int8_t* digit) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (!c->have_nodes) return fail(c, MSH_ERR_STATE, "msh_upload_nodes has not been called");
  if (count < 0) return fail(c, MSH_ERR_INVALID, "negative patch count");
  if (count == 0) return MSH_OK;
  if (!idx || !unsched || !digit) return fail(c, MSH_ERR_INVALID, "null patch arrays");
  std::vector<int32_t> sorted(idx, idx + count);
  std::sort(sorted.begin(), sorted.end());
  if (sorted.front() < 0 || sorted.back() >= c->n_nodes)
    return fail(c, MSH_ERR_INVALID, "patch index outside [0, n)");
  if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end())
    return fail(c, MSH_ERR_INVALID, "duplicate patch index");
  c->h_patch.resize((size_t)count);
  for (int32_t k = 0; k < count; ++k)
    c->h_patch[k] = (unsigned long long)(uint32_t)idx[k] |
                    ((unsigned long long)(unsched[k] ? 1u : 0u) << 32) |
                    ((unsigned long long)(uint8_t)digit[k] << 40);
  DeviceGuard g(c->device);
  Rewrite w{Rewrite::PATCH};
  w.patch_count = count;
  return rewrite(c, w);  // synchronous; launches in flight keep the previous version
}

int msh_export_results(msh_ctx* c, int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol,
                       uint8_t* out_filter, int64_t* out_score, int64_t* out_final) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (!c->have_nodes) return fail(c, MSH_ERR_STATE, "msh_upload_nodes has not been called");
  if (p < 0) return fail(c, MSH_ERR_INVALID, "negative pod count");
  const size_t pairs = (size_t)p * (size_t)c->n_nodes;
  if (pairs > ((size_t)1 << 28)) return fail(c, MSH_ERR_UNSUPPORTED, "export limited to p*n <= 2^28 pairs");
  if (c->generic) return fail(c, MSH_ERR_UNSUPPORTED, "score-column plugins run on the batch entry points only");
  if (pairs == 0) return MSH_OK;
  if (!pod_digit || !pod_tol || !out_filter || !out_score || !out_final)
    return fail(c, MSH_ERR_INVALID, "null pointer");
  DeviceGuard g(c->device);
  int rc = MSH_OK;
  const NodeTable& t = cur_table(c);
  int8_t* d_pd = nullptr;
  uint8_t* d_pt = nullptr;
  uint8_t* d_f = nullptr;
  int64_t* d_r = nullptr;
  int64_t* d_o = nullptr;
  auto step = [&](hipError_t e, const char* what) {
    if (rc == MSH_OK && e != hipSuccess) rc = hip_fail(c, e, what);
  };
  step(hipMalloc(&d_pd, (size_t)p), "hipMalloc");
  step(hipMalloc(&d_pt, (size_t)p), "hipMalloc");
  step(hipMalloc(&d_f, pairs), "hipMalloc");
  step(hipMalloc(&d_r, pairs * sizeof(int64_t)), "hipMalloc");
  step(hipMalloc(&d_o, pairs * sizeof(int64_t)), "hipMalloc");
  if (rc == MSH_OK) {
    step(hipMemcpyAsync(d_pd, pod_digit, (size_t)p, hipMemcpyHostToDevice, c->stream), "hipMemcpyAsync");
    step(hipMemcpyAsync(d_pt, pod_tol, (size_t)p, hipMemcpyHostToDevice, c->stream), "hipMemcpyAsync");
    step(msh::launch_export(t.d_unsched, t.d_digit, c->n_nodes, d_pd, d_pt, p, c->pp, d_f, d_r, d_o,
                            c->stream), "export_kernel");
    step(hipMemcpyAsync(out_filter, d_f, pairs, hipMemcpyDeviceToHost, c->stream), "hipMemcpyAsync");
    step(hipMemcpyAsync(out_score, d_r, pairs * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream),
         "hipMemcpyAsync");
    step(hipMemcpyAsync(out_final, d_o, pairs * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream),
         "hipMemcpyAsync");
    step(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
  }
  (void)hipFree(d_pd); (void)hipFree(d_pt); (void)hipFree(d_f); (void)hipFree(d_r); (void)hipFree(d_o);
  return rc;
}

int msh_upload_score_column(msh_ctx* c, int32_t plugin_id, int32_t n, const int64_t* scores) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (!is_column(plugin_id)) return fail(c, MSH_ERR_INVALID, "not a score-column plugin id");
  if (!c->have_nodes) return fail(c, MSH_ERR_STATE, "msh_upload_nodes has not been called");
  if (n != c->n_nodes) return fail(c, MSH_ERR_INVALID, "a score column has one entry per uploaded node");
  if (n > 0 && !scores) return fail(c, MSH_ERR_INVALID, "null scores");
  for (int32_t i = 0; i < n; ++i)
    if (scores[i] < -(int64_t(1) << 31) || scores[i] > (int64_t(1) << 31))
      return fail(c, MSH_ERR_INVALID, "score column value outside [-2^31, 2^31] at node " + std::to_string(i));
  DeviceGuard g(c->device);
  Rewrite w{Rewrite::COLUMN};
  w.col = plugin_id - MSH_PLUGIN_SCORE_COLUMN0;
  w.scores = scores;
  return rewrite(c, w);  // generic launches in flight keep reading the previous version
}

int msh_num_nodes(const msh_ctx* c, int32_t* out_n) {
  if (!c || !out_n) return MSH_ERR_INVALID;
  *out_n = c->have_nodes ? c->n_nodes : 0;
  return MSH_OK;
}

int msh_schedule_batch_device(msh_ctx* c, int32_t p, const int8_t* d_pod_digit,
                              const uint8_t* d_pod_tol, int32_t* d_out_idx, int64_t* d_out_score,
                              int32_t* d_out_status, void* stream) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (p < 0) return fail(c, MSH_ERR_INVALID, "negative pod count");
  if (p > 0 && (!d_pod_digit || !d_pod_tol || !d_out_idx || !d_out_status))  // d_out_score optional
    return fail(c, MSH_ERR_INVALID, "null device pointer");
  DeviceGuard g(c->device);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int rc = ready(c);
  if (rc != MSH_OK) return rc;
  if (p == 0) return MSH_OK;
  const msh::BatchDesc d{d_pod_digit, d_pod_tol, d_out_idx, d_out_score, d_out_status, p, 0};
  if ((rc = launch_batch_descs(c, &d, 1, s)) != MSH_OK) return rc;
  return track_launch(c, s);
}

int msh_schedule_batches_device(msh_ctx* c, int32_t nb, const msh_batch* batches, void* stream) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (nb < 0) return fail(c, MSH_ERR_INVALID, "negative batch count");
  if (nb > 0 && !batches) return fail(c, MSH_ERR_INVALID, "null batch array");
  for (int32_t i = 0; i < nb; ++i) {
    const msh_batch& b = batches[i];
    if (b.p < 0) return fail(c, MSH_ERR_INVALID, "batch " + std::to_string(i) + ": negative pod count");
    if (b.p > 0 && (!b.pod_digit || !b.pod_tol || !b.out_idx || !b.out_status))  // out_score optional
      return fail(c, MSH_ERR_INVALID, "batch " + std::to_string(i) + ": null device pointer");
  }
  DeviceGuard g(c->device);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int rc = ready(c);
  if (rc != MSH_OK) return rc;
  for (int32_t i0 = 0; i0 < nb; i0 += msh::MULTI_MAX) {  // MULTI_MAX batches per launch
    const int32_t n = std::min<int32_t>(msh::MULTI_MAX, nb - i0);
    msh::BatchDesc d[msh::MULTI_MAX];
    for (int32_t k = 0; k < n; ++k) {
      const msh_batch& b = batches[i0 + k];
      d[k] = msh::BatchDesc{b.pod_digit, b.pod_tol, b.out_idx, b.out_score, b.out_status, b.p, 0};
    }
    if ((rc = launch_batch_descs(c, d, n, s)) != MSH_OK) return rc;
  }
  return nb > 0 ? track_launch(c, s) : MSH_OK;
}

int msh_schedule_batch(msh_ctx* c, int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol,
                       int32_t* out_idx, int64_t* out_score, int32_t* out_status) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (p < 0) return fail(c, MSH_ERR_INVALID, "negative pod count");
  if (p > 0 && (!pod_digit || !pod_tol || !out_idx || !out_status))  // out_score optional
    return fail(c, MSH_ERR_INVALID, "null host pointer");
  if (!c->have_nodes) return fail(c, MSH_ERR_STATE, "msh_upload_nodes has not been called");
  if (p == 0) return MSH_OK;
  DeviceGuard g(c->device);
  int rc = ready(c);
  if (rc != MSH_OK) return rc;
  HostIO io;
  if ((rc = host_io_begin(c, p, pod_digit, pod_tol, out_idx, out_score, out_status, io)) != MSH_OK) return rc;
  rc = msh_schedule_batch_device(c, p, io.d_pd, io.d_pt, io.o_idx, io.o_score, io.o_status, c->stream);
  if (rc != MSH_OK) return rc;
  return host_io_end(c, p, out_idx, out_score, out_status, io);
}

int msh_schedule_batch_async(msh_ctx* c, int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol,
                             int32_t* out_idx, int64_t* out_score, int32_t* out_status, uint64_t* out_ticket) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (!out_ticket) return fail(c, MSH_ERR_INVALID, "null ticket");
  if (p < 0) return fail(c, MSH_ERR_INVALID, "negative pod count");
  if (p > 0 && (!pod_digit || !pod_tol || !out_idx || !out_status))  // out_score optional
    return fail(c, MSH_ERR_INVALID, "null host pointer");
  if (!c->have_nodes) return fail(c, MSH_ERR_STATE, "msh_upload_nodes has not been called");
  DeviceGuard g(c->device);
  void *dpd = nullptr, *dpt = nullptr, *doi = nullptr, *dos = nullptr, *dost = nullptr;
  if (p > 0) {
    dpd = pinned_device_ptr(pod_digit);
    dpt = pinned_device_ptr(pod_tol);
    doi = pinned_device_ptr(out_idx);
    dos = out_score ? pinned_device_ptr(out_score) : nullptr;
    dost = pinned_device_ptr(out_status);
    if (!dpd || !dpt || !doi || !dost || (out_score && !dos))
      return fail(c, MSH_ERR_INVALID, "msh_schedule_batch_async needs page-locked buffers (msh_host_alloc)");
  }
  int rc = ready(c);
  if (rc != MSH_OK) return rc;
  if (c->async_issued - c->async_done >= MSH_ASYNC_DEPTH) {  // the ring is full: wait for the oldest
    const uint64_t t = c->async_done + 1;
    MSH_HIP(c, hipEventSynchronize(c->async_ev[t % MSH_ASYNC_DEPTH]));
    c->async_done = t;
  }
  hipEvent_t& ev = c->async_ev[(c->async_issued + 1) % MSH_ASYNC_DEPTH];
  if (!ev) MSH_HIP(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  if (p > 0) {
    rc = msh_schedule_batch_device(c, p, static_cast<const int8_t*>(dpd), static_cast<const uint8_t*>(dpt),
                                   static_cast<int32_t*>(doi), static_cast<int64_t*>(dos), static_cast<int32_t*>(dost),
                                   c->stream);
    if (rc != MSH_OK) return rc;
  }
  MSH_HIP(c, hipEventRecord(ev, c->stream));
  *out_ticket = ++c->async_issued;
  return MSH_OK;
}

int msh_wait(msh_ctx* c, uint64_t ticket) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (ticket == 0 || ticket > c->async_issued) return fail(c, MSH_ERR_INVALID, "unknown ticket");
  if (ticket <= c->async_done) return MSH_OK;
  DeviceGuard g(c->device);
  MSH_HIP(c, hipEventSynchronize(c->async_ev[ticket % MSH_ASYNC_DEPTH]));
  c->async_done = ticket;  // in-order completion on the ctx's stream
  return MSH_OK;
}

int msh_schedule_sequential_device(msh_ctx* c, int32_t p, const int8_t* d_pod_digit,
                                   const uint8_t* d_pod_tol, int32_t max_pods_per_node,
                                   int32_t* d_out_idx, int64_t* d_out_score,
                                   int32_t* d_out_status, void* stream) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (p < 0 || max_pods_per_node < 0) return fail(c, MSH_ERR_INVALID, "negative argument");
  if (p > 0 && (!d_pod_digit || !d_pod_tol || !d_out_idx || !d_out_status))  // d_out_score optional
    return fail(c, MSH_ERR_INVALID, "null device pointer");
  if (c->generic) return fail(c, MSH_ERR_UNSUPPORTED, "score-column plugins run on the batch entry points only");
  DeviceGuard g(c->device);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int rc = ready(c);
  if (rc != MSH_OK) return rc;
  msh::SeqArgs a{};
  const NodeTable& t = cur_table(c);
  a.planes = t.d_planes;
  a.n_words = c->n_pad / 32;
  a.n_nodes = c->n_nodes;
  a.pod_digit = d_pod_digit;
  a.pod_tol = d_pod_tol;
  a.n_pods = p;
  a.pp = c->pp;
  a.max_pods = max_pods_per_node;
  a.counts = c->d_counts;
  a.count_stride = (int64_t)c->counts_cap;
  a.count_replicas = c->counts_replicas;
  // Without a capacity no commit feeds a later decision (the counts are read by nothing the plugins
  // score): the default runs the per-pair batch kernel with the commit epilogue (pair_kernel<CNT>, every
  // placed pod's count added to a replica), whose placements are msh_schedule_batch's; seq_split = 2 keeps
  // the sequential kernel's 64-pod blocks, = 1 one workgroup walking the batch in order
  const bool pair_form = max_pods_per_node == 0 && c->dev.seq_split == 2 && p > msh::WAVE &&
                         c->counts_replicas == msh::SEQ_COUNT_REPLICAS;
  const bool split = pair_form || msh::seq_blocks(a, c->dev) > 1;
  a.fold = !split && c->counts_dirty ? 1 : 0;
  // one sequential launch of a ctx at a time: each commits into (and a fold rewrites) the same counts,
  // so this stream first waits for the ctx's sequential launches in flight on other streams
  if (p > 0)
    for (auto& ev : c->seq_inflight)
      if (ev.first != s) MSH_HIP(c, hipStreamWaitEvent(s, ev.second, 0));
  a.out_idx = d_out_idx;
  a.out_score = d_out_score;
  a.out_status = d_out_status;
  std::string err;
  hipError_t e;
  if (pair_form) {
    msh::PairArgs pa = pair_args(c);
    pa.nb = 1;
    pa.d[0] = msh::BatchDesc{d_pod_digit, d_pod_tol, d_out_idx, d_out_score, d_out_status, p, 0};
    pa.counts = c->d_counts;
    pa.count_stride = (int64_t)c->counts_cap;
    TimedLaunch tl(c);
    e = msh::launch_pairs(pa, false, c->dev, s);
  } else {
    TimedLaunch tl(c);
    e = msh::launch_sequential(a, c->dev, s, &err);
  }
  if (e != hipSuccess) {
    if (!err.empty()) return fail(c, MSH_ERR_UNSUPPORTED, err);
    return hip_fail(c, e, "seq_kernel");
  }
  if (p > 0) c->counts_dirty = split || (c->counts_dirty && !a.fold);
  return p > 0 ? track_launch(c, s, true) : MSH_OK;
}

int msh_schedule_sequential(msh_ctx* c, int32_t p, const int8_t* pod_digit, const uint8_t* pod_tol,
                            int32_t max_pods_per_node, int32_t* out_idx, int64_t* out_score,
                            int32_t* out_status, msh_commit_cb commit_cb, void* user) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (p < 0) return fail(c, MSH_ERR_INVALID, "negative pod count");
  if (p > 0 && (!pod_digit || !pod_tol || !out_idx || !out_status))  // out_score optional
    return fail(c, MSH_ERR_INVALID, "null host pointer");
  if (!c->have_nodes) return fail(c, MSH_ERR_STATE, "msh_upload_nodes has not been called");
  if (p == 0) return MSH_OK;
  DeviceGuard g(c->device);
  int rc = ready(c);
  if (rc != MSH_OK) return rc;
  HostIO io;
  if ((rc = host_io_begin(c, p, pod_digit, pod_tol, out_idx, out_score, out_status, io)) != MSH_OK) return rc;
  rc = msh_schedule_sequential_device(c, p, io.d_pd, io.d_pt, max_pods_per_node, io.o_idx, io.o_score,
                                      io.o_status, c->stream);
  if (rc != MSH_OK) return rc;
  if ((rc = host_io_end(c, p, out_idx, out_score, out_status, io)) != MSH_OK) return rc;
  if (commit_cb)
    for (int32_t j = 0; j < p; j++)
      if (out_status[j] == MSH_PLACED) commit_cb(user, j, out_idx[j], out_score ? out_score[j] : 0);
  return MSH_OK;
}

int msh_node_pod_counts(msh_ctx* c, int32_t* out_counts) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (!c->have_nodes) return fail(c, MSH_ERR_STATE, "msh_upload_nodes has not been called");
  if (c->n_nodes > 0 && !out_counts) return fail(c, MSH_ERR_INVALID, "null output");
  if (c->n_nodes == 0) return MSH_OK;
  DeviceGuard g(c->device);
  int rc = after_seq(c);  // sequential launches of this ctx in flight update the counts
  if (rc != MSH_OK) return rc;
  if (c->counts_dirty) {
    hipError_t e = msh::launch_count_fold(c->d_counts, (int64_t)c->counts_cap, c->counts_replicas, c->n_nodes,
                                          c->prep_stream);
    if (e != hipSuccess) return hip_fail(c, e, "count_fold_kernel");
    c->counts_dirty = false;
  }
  MSH_HIP(c, hipMemcpyAsync(out_counts, c->d_counts, (size_t)c->n_nodes * sizeof(int32_t), hipMemcpyDeviceToHost,
                            c->prep_stream));
  MSH_HIP(c, hipStreamSynchronize(c->prep_stream));
  return MSH_OK;
}

int msh_reset_node_pod_counts(msh_ctx* c) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (!c->have_nodes) return fail(c, MSH_ERR_STATE, "msh_upload_nodes has not been called");
  DeviceGuard g(c->device);
  int rc = after_seq(c);  // sequential launches of this ctx in flight update the counts
  if (rc != MSH_OK) return rc;
  MSH_HIP(c, hipMemsetAsync(c->d_counts, 0, (size_t)c->counts_replicas * c->counts_cap * sizeof(int32_t),
                            c->prep_stream));
  MSH_HIP(c, hipStreamSynchronize(c->prep_stream));
  c->counts_dirty = false;
  return MSH_OK;
}

int msh_keys_slot1_is_any(const msh_ctx* c, int32_t* out_flag) {
  if (!c || !out_flag) return MSH_ERR_INVALID;
  *out_flag = 0;  // ABI v7: keys[p + j] is always pod j's own first feasible non-match
  return MSH_OK;
}

int msh_shard_keys_len(const msh_ctx* c, int32_t p, int32_t* out_len) {
  if (!c || !out_len || p < 0) return MSH_ERR_INVALID;
  const int64_t len = 2 * (int64_t)p;  // per pod: first feasible match, first feasible non-match
  if (len > INT32_MAX) return MSH_ERR_INVALID;
  *out_len = (int32_t)len;
  return MSH_OK;
}

int msh_shard_keys_device(msh_ctx* c, int32_t p, const int8_t* d_pod_digit,
                          const uint8_t* d_pod_tol, int64_t node_base, int32_t* d_keys,
                          void* stream) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (p < 0 || node_base < 0) return fail(c, MSH_ERR_INVALID, "negative argument");
  if (p > 0 && (!d_pod_digit || !d_pod_tol || !d_keys)) return fail(c, MSH_ERR_INVALID, "null device pointer");
  if (node_base + (int64_t)c->n_nodes >= msh::GKEY_MAX) return fail(c, MSH_ERR_INVALID, "global node index overflows the key");
  if (c->generic)
    return fail(c, MSH_ERR_UNSUPPORTED, "score-column plugin lists shard through msh_generic_extents_device / "
                                        "msh_generic_best_device");
  DeviceGuard g(c->device);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int rc = ready(c);
  if (rc != MSH_OK) return rc;
  if (p == 0) return MSH_OK;
  msh::PairArgs a = pair_args(c);
  a.nb = 1;
  a.d[0] = msh::BatchDesc{d_pod_digit, d_pod_tol, nullptr, nullptr, nullptr, p, 0};
  a.keys = d_keys;
  a.node_base = node_base;
  hipError_t e;
  {
    TimedLaunch tl(c);
    e = msh::launch_pairs(a, true, c->dev, s);
  }
  if (e != hipSuccess) return hip_fail(c, e, "pair_kernel (shard keys)");
  return track_launch(c, s);
}

int msh_decode_keys_device(msh_ctx* c, int32_t p, const int8_t* d_pod_digit,
                           const uint8_t* d_pod_tol, const int32_t* d_keys, int32_t* d_out_idx,
                           int64_t* d_out_score, int32_t* d_out_status, void* stream) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (p < 0) return fail(c, MSH_ERR_INVALID, "negative pod count");
  if (p > 0 && (!d_pod_digit || !d_pod_tol || !d_keys || !d_out_idx || !d_out_status))  // d_out_score optional
    return fail(c, MSH_ERR_INVALID, "null device pointer");
  DeviceGuard g(c->device);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipError_t e = msh::launch_decode_keys(d_pod_digit, p, d_keys, c->pp, d_out_idx, d_out_score, d_out_status, s);
  if (e != hipSuccess) return hip_fail(c, e, "decode_keys_kernel");
  return MSH_OK;
}

int msh_generic_ext_len(const msh_ctx* c, int32_t p, int64_t* out_len) {
  if (!c || !out_len || p < 0) return MSH_ERR_INVALID;
  bool ext = false;
  int32_t ncol = 0;
  for (size_t k = 0; k < c->score_ids.size(); ++k) {
    ext = ext || c->normalize[k] != MSH_NORMALIZE_NONE;
    ncol += is_column(c->score_ids[k]) ? 1 : 0;
  }
  *out_len = ext ? 2 * (int64_t)(1 + ncol) * p : 0;
  return MSH_OK;
}

namespace {
// One sharded generic launch (mode 1: extents, mode 2: best) over this ctx's node slice.
int generic_shard_launch(msh_ctx* c, int mode, int32_t p, const int8_t* pd, const uint8_t* pt, int64_t* ext,
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
  if (e != hipSuccess) return hip_fail(c, e, "generic_kernel (node-sharded)");
  return track_launch(c, s);
}
}  // namespace

int msh_generic_extents_device(msh_ctx* c, int32_t p, const int8_t* d_pod_digit, const uint8_t* d_pod_tol,
                               int64_t* d_ext, void* stream) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (p < 0) return fail(c, MSH_ERR_INVALID, "negative pod count");
  int64_t len = 0;
  msh_generic_ext_len(c, p, &len);
  if (p == 0 || len == 0) return MSH_OK;  // no plugin normalizes: nothing to merge
  if (!d_pod_digit || !d_pod_tol || !d_ext) return fail(c, MSH_ERR_INVALID, "null device pointer");
  DeviceGuard g(c->device);
  int rc = ready(c);
  if (rc != MSH_OK) return rc;
  return generic_shard_launch(c, 1, p, d_pod_digit, d_pod_tol, d_ext, 0, nullptr, nullptr,
                              reinterpret_cast<hipStream_t>(stream));
}

int msh_generic_best_device(msh_ctx* c, int32_t p, const int8_t* d_pod_digit, const uint8_t* d_pod_tol,
                            const int64_t* d_ext, int64_t node_base, int64_t* d_best_total, int32_t* d_best_idx,
                            void* stream) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (p < 0 || node_base < 0) return fail(c, MSH_ERR_INVALID, "negative argument");
  if (node_base + (int64_t)c->n_nodes >= (int64_t)INT32_MAX)
    return fail(c, MSH_ERR_INVALID, "global node index overflows int32");
  int64_t len = 0;
  msh_generic_ext_len(c, p, &len);
  if (p == 0) return MSH_OK;
  if (!d_pod_digit || !d_pod_tol || !d_best_total || !d_best_idx || (len > 0 && !d_ext))
    return fail(c, MSH_ERR_INVALID, "null device pointer");
  DeviceGuard g(c->device);
  int rc = ready(c);
  if (rc != MSH_OK) return rc;
  return generic_shard_launch(c, 2, p, d_pod_digit, d_pod_tol, const_cast<int64_t*>(d_ext), node_base, d_best_total,
                              d_best_idx, reinterpret_cast<hipStream_t>(stream));
}

int msh_generic_candidates_device(msh_ctx* c, int32_t p, const int64_t* d_local_total, const int64_t* d_merged_total,
                                  int32_t* d_best_idx, void* stream) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (p < 0) return fail(c, MSH_ERR_INVALID, "negative pod count");
  if (p > 0 && (!d_local_total || !d_merged_total || !d_best_idx)) return fail(c, MSH_ERR_INVALID, "null device pointer");
  DeviceGuard g(c->device);
  hipError_t e = msh::launch_generic_candidates(p, d_local_total, d_merged_total, d_best_idx,
                                                reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(c, e, "generic_candidate_kernel");
  return MSH_OK;
}

int msh_generic_decode_device(msh_ctx* c, int32_t p, const int8_t* d_pod_digit, const int64_t* d_merged_total,
                              const int32_t* d_merged_idx, int32_t* d_out_idx, int64_t* d_out_score,
                              int32_t* d_out_status, void* stream) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (p < 0) return fail(c, MSH_ERR_INVALID, "negative pod count");
  if (p > 0 && (!d_pod_digit || !d_merged_total || !d_merged_idx || !d_out_idx || !d_out_status))
    return fail(c, MSH_ERR_INVALID, "null device pointer");  // d_out_score optional
  DeviceGuard g(c->device);
  int32_t nn_score = 0;
  for (int32_t id : c->score_ids) nn_score |= id == MSH_PLUGIN_NODE_NUMBER ? 1 : 0;
  hipError_t e = msh::launch_generic_decode(d_pod_digit, p, d_merged_total, d_merged_idx, nn_score, c->pp.nn_prescore,
                                            d_out_idx, d_out_score, d_out_status, reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(c, e, "generic_decode_kernel");
  return MSH_OK;
}

int msh_timing_begin(msh_ctx* c, int32_t max_launches) {
  if (!c) return MSH_ERR_INVALID;
  c->err.clear();
  if (max_launches < 1 || max_launches > 4096) return fail(c, MSH_ERR_INVALID, "max_launches outside [1, 4096]");
  DeviceGuard g(c->device);
  while (c->tev.size() < (size_t)max_launches) {
    hipEvent_t a = nullptr, b = nullptr;
    MSH_HIP(c, hipEventCreate(&a));
    if (hipEventCreate(&b) != hipSuccess) {
      (void)hipEventDestroy(a);
      return fail(c, MSH_ERR_HIP, "hipEventCreate");
    }
    c->tev.emplace_back(a, b);
  }
  c->timing = true;
  c->t_next = 0;
  return MSH_OK;
}

int msh_timing_end(msh_ctx* c, int32_t* out_launches, double* out_total_ms, double* out_max_ms) {
  if (!c || !out_launches || !out_total_ms) return MSH_ERR_INVALID;
  c->err.clear();
  if (!c->timing) return fail(c, MSH_ERR_STATE, "msh_timing_begin has not been called");
  DeviceGuard g(c->device);
  c->timing = false;
  double total = 0, mx = 0;
  for (size_t i = 0; i < c->t_next; ++i) {
    MSH_HIP(c, hipEventSynchronize(c->tev[i].second));
    float ms = 0;
    MSH_HIP(c, hipEventElapsedTime(&ms, c->tev[i].first, c->tev[i].second));
    total += ms;
    mx = std::max(mx, (double)ms);
  }
  *out_launches = (int32_t)c->t_next;
  *out_total_ms = total;
  if (out_max_ms) *out_max_ms = mx;
  c->t_next = 0;
  return MSH_OK;
}

}  // extern "C"
