// pack_stress.cpp — host-only stress driver for the snapshot packer (msh_pack.cpp) and the
// process-wide host thread pool (msh_pool.h), built with ASan+UBSan and with TSan by
// tests/sanitize/Makefile (no HIP: these are the C-ABI's host-only parts). Exits non-zero on a
// wrong result; the sanitizers abort on a memory or threading error.
//   1. 200k pods packed on the pool, against a serial restatement of the rules
//   2. four threads packing at once (one gets the pool, the others pack on their own thread)
//   3. malformed offsets: MSH_ERR_INVALID without reading outside the blob / toleration array
//   4. fork() after the pool exists: the child's large pack runs serially and finishes
//   5. msh_pack_nodes on shuffled names: byte order, duplicates rejected
//   6. pool lease contention: many threads leasing / running / releasing
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/minisched_hip.h"
#include "../../mini-kube-scheduler_amd/csrc/msh_pool.h"

namespace {

int g_fail = 0;
#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      g_fail = 1;                                                   \
    }                                                               \
  } while (0)

struct Pods {
  std::string blob;
  std::vector<int64_t> name_off, tol_off;
  std::vector<msh_toleration> tols;
  std::vector<int8_t> want_digit;
  std::vector<uint8_t> want_tol;
};

Pods make_pods(int p, uint64_t seed) {
  std::mt19937_64 rng(seed);
  Pods d;
  d.name_off.push_back(0);
  d.tol_off.push_back(0);
  static const char* keys[] = {"node.kubernetes.io/unschedulable", "", "other"};
  static const char* ops[] = {"Exists", "Equal", "", "Bogus"};
  static const char* vals[] = {"", "x"};
  static const char* effects[] = {"NoSchedule", "", "NoExecute"};
  for (int j = 0; j < p; ++j) {
    std::string name = "pod" + std::to_string(j);
    if (rng() % 100 == 0) name += "-x";
    d.blob += name;
    d.name_off.push_back((int64_t)d.blob.size());
    const char c = name.back();
    d.want_digit.push_back(c >= '0' && c <= '9' ? (int8_t)(c - '0') : (int8_t)-1);
    const int nt = rng() % 10 == 0 ? 1 + (int)(rng() % 3) : 0;
    uint8_t tol = 0;
    for (int k = 0; k < nt; ++k) {
      msh_toleration t{keys[rng() % 3], ops[rng() % 4], vals[rng() % 2], effects[rng() % 3]};
      d.tols.push_back(t);
      tol |= (uint8_t)msh_toleration_tolerates_unschedulable(&t);
    }
    d.tol_off.push_back((int64_t)d.tols.size());
    d.want_tol.push_back(tol);
  }
  return d;
}

bool pack_ok(const Pods& d, int p) {
  std::vector<int8_t> dg((size_t)p);
  std::vector<uint8_t> tl((size_t)p);
  const int rc = msh_pack_pods(p, d.blob.data(), d.name_off.data(), d.tols.empty() ? nullptr : d.tols.data(),
                               d.tol_off.data(), dg.data(), tl.data());
  return rc == MSH_OK && std::equal(dg.begin(), dg.end(), d.want_digit.begin()) &&
         std::equal(tl.begin(), tl.end(), d.want_tol.begin());
}

}  // namespace

int main() {
  // 1. one large batch (split over the pool)
  const int P = 200000;
  Pods d = make_pods(P, 1);
  CHECK(pack_ok(d, P));

  // 2. concurrent packers
  {
    std::vector<std::thread> th;
    std::atomic<int> bad{0};
    for (int t = 0; t < 4; ++t)
      th.emplace_back([&] {
        for (int r = 0; r < 20; ++r)
          if (!pack_ok(d, P)) bad++;
      });
    for (auto& x : th) x.join();
    CHECK(bad.load() == 0);
  }

  // 3. malformed offsets, on exactly-sized heap copies so that any stray read is caught
  {
    const int p = 20000;
    Pods s = make_pods(p, 2);
    std::vector<int8_t> dg(p);
    std::vector<uint8_t> tl(p);
    auto run = [&](std::vector<int64_t> no, std::vector<int64_t> to, bool with_tols) {
      char* blob = (char*)std::malloc(s.blob.size());
      std::memcpy(blob, s.blob.data(), s.blob.size());
      msh_toleration* tols = nullptr;
      if (with_tols && !s.tols.empty()) {
        tols = (msh_toleration*)std::malloc(s.tols.size() * sizeof(msh_toleration));
        std::memcpy(tols, s.tols.data(), s.tols.size() * sizeof(msh_toleration));
      }
      const int rc = msh_pack_pods(p, blob, no.data(), tols, to.data(), dg.data(), tl.data());
      std::free(blob);
      std::free(tols);
      return rc;
    };
    CHECK(run(s.name_off, s.tol_off, true) == MSH_OK);
    auto no = s.name_off;
    no[1] = 0;  // empty first name: would read blob[-1]
    CHECK(run(no, s.tol_off, true) == MSH_ERR_INVALID);
    no = s.name_off;
    no[p / 2] = no[p / 2 + 1];  // an empty name in the middle
    CHECK(run(no, s.tol_off, true) == MSH_ERR_INVALID);
    no = s.name_off;
    no[0] = -5;
    CHECK(run(no, s.tol_off, true) == MSH_ERR_INVALID);
    auto to = s.tol_off;
    to[1] = to[2] + 1;  // non-monotone toleration offsets
    CHECK(run(s.name_off, to, true) == MSH_ERR_INVALID);
    to.assign((size_t)p + 1, 0);
    to[1] = 1;  // [0, 1, 0, ...]: a range with no toleration array
    CHECK(run(s.name_off, to, false) == MSH_ERR_INVALID);
    to = s.tol_off;
    to[p / 3] = -1;
    CHECK(run(s.name_off, to, true) == MSH_ERR_INVALID);
  }

  // 4. fork after the pool exists: the child packs a large batch on its own thread
  {
    const pid_t pid = fork();
    if (pid == 0) {
      alarm(60);  // a child stuck on a pool with no threads would be killed here
      _exit(pack_ok(d, P) ? 0 : 3);
    }
    int st = 0;
    CHECK(pid > 0 && waitpid(pid, &st, 0) == pid && WIFEXITED(st) && WEXITSTATUS(st) == 0);
  }

  // 5. nodes: shuffled names come back in byte order; a duplicate is rejected
  {
    const int n = 50000;
    std::vector<std::string> names;
    for (int i = 0; i < n; ++i) names.push_back("node" + std::to_string(i));
    std::shuffle(names.begin(), names.end(), std::mt19937_64(3));
    std::string blob;
    std::vector<int64_t> off{0};
    for (auto& x : names) {
      blob += x;
      off.push_back((int64_t)blob.size());
    }
    std::vector<uint8_t> un(n, 0), ou(n);
    std::vector<int32_t> order(n);
    std::vector<int8_t> dg(n);
    CHECK(msh_pack_nodes(n, blob.data(), off.data(), un.data(), order.data(), ou.data(), dg.data()) == MSH_OK);
    bool sorted = true;
    for (int k = 1; k < n; ++k) sorted &= names[order[k - 1]] < names[order[k]];
    CHECK(sorted);
    names[7] = names[8];
    blob.clear();
    off.assign(1, 0);
    for (auto& x : names) {
      blob += x;
      off.push_back((int64_t)blob.size());
    }
    CHECK(msh_pack_nodes(n, blob.data(), off.data(), un.data(), order.data(), ou.data(), dg.data()) ==
          MSH_ERR_INVALID);
  }

  // 6. lease contention on the shared pool
  {
    std::atomic<long> sum{0};
    std::vector<std::thread> th;
    for (int t = 0; t < 8; ++t)
      th.emplace_back([&] {
        for (int r = 0; r < 200; ++r) {
          msh::PoolLease lease;
          if (msh::HostPool* pool = lease.get()) {
            std::vector<long> part((size_t)pool->parts(), 0);
            pool->run([&](int k) { part[(size_t)k] = k + 1; });
            long s2 = 0;
            for (long v : part) s2 += v;
            sum += s2 == (long)pool->parts() * (pool->parts() + 1) / 2 ? 0 : 1;
          }
        }
      });
    for (auto& x : th) x.join();
    CHECK(sum.load() == 0);
  }
  std::printf(g_fail ? "pack_stress: FAILED\n" : "pack_stress: ok\n");
  return g_fail;
}
