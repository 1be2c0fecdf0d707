// msh_pack.cpp — host snapshot packer: v1.Node / v1.Pod fields -> SoA columns of the C-ABI.
//
// Replaces, for a batch, the per-cycle decoding the reference does on every pod:
//   - node order: Nodes().List() with no ResourceVersion is served from etcd in key
//     order, i.e. byte-wise by name (minisched/minisched.go:40). Sorted here once.
//   - node/pod digit: strconv.Atoi(name[len(name)-1:]) (nodenumber.go:51-52, :81-83);
//     only '0'..'9' parse (a lone '+'/'-' is a syntax error), anything else -> -1.
//   - pod tolerates the unschedulable taint: upstream v1helper.TolerationsTolerateTaint
//     (k8s.io/kubernetes v1.22.0 pkg/apis/core/v1/helper/helpers.go) over
//     Toleration.ToleratesTaint (k8s.io/api v0.22.0 core/v1/toleration.go) with the taint
//     {Key: "node.kubernetes.io/unschedulable", Effect: NoSchedule}, as built by
//     NodeUnschedulable.Filter (upstream node_unschedulable.go, v1.22.0).
#include <algorithm>
#include <cstring>
#include <numeric>
#include <string_view>
#include <vector>

#include "../../include/minisched_hip.h"
#include "msh_pool.h"

namespace {

constexpr std::string_view kTaintKey = "node.kubernetes.io/unschedulable";
constexpr std::string_view kTaintEffect = "NoSchedule";
constexpr std::string_view kTaintValue = "";
constexpr int32_t kParallelPods = 16384;  // msh_pack_pods splits batches of at least this many

std::string_view sv(const char* s) { return s ? std::string_view(s) : std::string_view(); }

// the digit of the name ending at byte `end` (exclusive) of its blob
int8_t suffix_digit(const char* blob, int64_t end) {
  const unsigned char c = static_cast<unsigned char>(blob[end - 1]);
  return (c >= '0' && c <= '9') ? static_cast<int8_t>(c - '0') : static_cast<int8_t>(-1);
}

bool tolerates(const msh_toleration& t) {
  const std::string_view effect = sv(t.effect), key = sv(t.key), op = sv(t.op), value = sv(t.value);
  if (!effect.empty() && effect != kTaintEffect) return false;
  if (!key.empty() && key != kTaintKey) return false;
  if (op.empty() || op == "Equal") return value == kTaintValue;  // empty operator means Equal
  if (op == "Exists") return true;
  return false;
}

}  // namespace

extern "C" {

int msh_toleration_tolerates_unschedulable(const msh_toleration* t) {
  if (!t) return MSH_ERR_INVALID;
  return tolerates(*t) ? 1 : 0;
}

int msh_pack_nodes(int32_t n, const char* names, const int64_t* name_off,
                   const uint8_t* unschedulable, int32_t* out_order, uint8_t* out_unsched,
                   int8_t* out_digit) try {
  if (n < 0) return MSH_ERR_INVALID;
  if (n == 0) return MSH_OK;
  if (!names || !name_off || !unschedulable || !out_order || !out_unsched || !out_digit)
    return MSH_ERR_INVALID;
  std::vector<std::string_view> nm(static_cast<size_t>(n));
  for (int32_t i = 0; i < n; i++) {
    const int64_t a = name_off[i], b = name_off[i + 1];
    if (a < 0 || b <= a) return MSH_ERR_INVALID;  // empty name: reference would panic
    nm[i] = std::string_view(names + a, static_cast<size_t>(b - a));
  }
  std::vector<int32_t> order(static_cast<size_t>(n));
  std::iota(order.begin(), order.end(), 0);
  // Go string comparison == byte-wise lexicographic (std::string_view::compare uses
  // char_traits<char>::compare -> memcmp semantics, unsigned bytes).
  std::stable_sort(order.begin(), order.end(),
                   [&](int32_t x, int32_t y) { return nm[x].compare(nm[y]) < 0; });
  for (int32_t k = 1; k < n; k++)
    if (nm[order[k]] == nm[order[k - 1]]) return MSH_ERR_INVALID;  // names are unique keys
  for (int32_t k = 0; k < n; k++) {
    const int32_t i = order[k];
    out_order[k] = i;
    out_unsched[k] = unschedulable[i] ? 1 : 0;
    out_digit[k] = suffix_digit(nm[i].data(), static_cast<int64_t>(nm[i].size()));  // name's own end
  }
  return MSH_OK;
} catch (...) {  // std::bad_alloc: nothing throws across the C-ABI
  return MSH_ERR_NOMEM;
}

int msh_pack_pods(int32_t p, const char* names, const int64_t* name_off,
                  const msh_toleration* tols, const int64_t* tol_off, int8_t* out_digit,
                  uint8_t* out_tol) try {
  if (p < 0) return MSH_ERR_INVALID;
  if (p == 0) return MSH_OK;
  if (!names || !name_off || !tol_off || !out_digit || !out_tol) return MSH_ERR_INVALID;
  // Pods [lo, hi): each pod's offsets are checked BEFORE any read they guard (a name must be
  // non-empty and start at a non-negative offset; a toleration range must be non-negative, ordered
  // and backed by `tols`), so malformed offsets return MSH_ERR_INVALID without touching memory
  // outside the ranges they describe. One pass, split over the pool for large batches.
  auto pack_range = [&](int32_t lo, int32_t hi) {
    bool bad = false;
    for (int32_t j = lo; j < hi; j++) {
      const int64_t n0 = name_off[j], n1 = name_off[j + 1], t0 = tol_off[j], t1 = tol_off[j + 1];
      const bool name_ok = n0 >= 0 && n1 > n0;
      const bool tol_ok = t0 >= 0 && t1 >= t0 && (t1 == t0 || tols != nullptr);
      bad |= !(name_ok && tol_ok);
      out_digit[j] = name_ok ? suffix_digit(names, n1) : static_cast<int8_t>(-1);
      uint8_t tol = 0;
      if (tol_ok)
        for (int64_t k = t0; k < t1 && !tol; k++) tol = tolerates(tols[k]) ? 1 : 0;  // any toleration
      out_tol[j] = tol;
    }
    return bad;
  };
  // Large batches are split over the process-wide pool of host threads (msh_pool.h: one caller at a
  // time; a concurrent caller, a forked child or a host without the threads packs on its own thread).
  if (p >= kParallelPods) {
    msh::PoolLease lease;
    if (msh::HostPool* pool = lease.get()) {
      const int n = pool->parts();
      std::vector<char> bad(static_cast<size_t>(n), 0);
      pool->run([&](int k) {
        bad[k] = pack_range((int32_t)((int64_t)p * k / n), (int32_t)((int64_t)p * (k + 1) / n)) ? 1 : 0;
      });
      for (char b : bad)
        if (b) return MSH_ERR_INVALID;
      return MSH_OK;
    }
  }
  return pack_range(0, p) ? MSH_ERR_INVALID : MSH_OK;
} catch (...) {
  return MSH_ERR_NOMEM;
}

}  // extern "C"
