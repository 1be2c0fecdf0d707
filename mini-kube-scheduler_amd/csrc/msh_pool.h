// msh_pool.h — ONE process-wide pool of persistent host threads, shared by the C-ABI's staged
// copies (msh_capi.cpp) and the snapshot packer (msh_pack.cpp). Host code only.
//
// Use it through PoolLease: a caller that finds the pool busy (another thread's pack or copy), a
// process forked after the pool was created (its copy of the pool has no threads), or a failed
// thread creation gets no pool and runs on its own thread. Nothing here throws across the C-ABI.
#pragma once

#include <sys/types.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

namespace msh {

// Persistent host threads: run(f) calls f(0..n-1), part 0 on the calling thread, the rest on the
// workers, and returns when all are done. A worker spins on the job counter for a while after each
// job before it blocks, so back-to-back batches do not pay a futex wake-up per call (tens of
// microseconds on a busy host).
class HostPool {
 public:
  // nullptr when a worker thread cannot be created (the ones that were are joined).
  static HostPool* create(int workers) noexcept {
    HostPool* p = new (std::nothrow) HostPool();
    if (!p) return nullptr;
    try {
      p->th_.reserve((size_t)workers);
      for (int w = 0; w < workers; ++w) p->th_.emplace_back([p, w] { p->loop(w + 1); });
    } catch (...) {  // std::system_error from std::thread, std::bad_alloc
      delete p;
      return nullptr;
    }
    return p;
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_.store(true);
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int parts() const { return (int)th_.size() + 1; }
  void run(const std::function<void(int)>& f) {
    job_ = &f;
    pending_.store((int)th_.size(), std::memory_order_relaxed);
    gen_.fetch_add(1, std::memory_order_release);
    { std::lock_guard<std::mutex> g(m_); }  // a worker between its check and its wait sees the new job
    cv_.notify_all();
    f(0);
    while (pending_.load(std::memory_order_acquire) != 0) std::this_thread::yield();
    job_ = nullptr;
  }

 private:
  HostPool() = default;
  void loop(int part) {
    uint64_t seen = 0;
    for (;;) {
      uint64_t g = gen_.load(std::memory_order_acquire);
      for (int spin = 0; g == seen && !stop_.load(std::memory_order_relaxed) && spin < (1 << 16); ++spin) {
        std::this_thread::yield();
        g = gen_.load(std::memory_order_acquire);
      }
      if (g == seen) {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_.load() || gen_.load(std::memory_order_acquire) != seen; });
        g = gen_.load(std::memory_order_acquire);
      }
      if (stop_.load()) return;
      seen = g;
      (*job_)(part);
      pending_.fetch_sub(1, std::memory_order_release);
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_;
  const std::function<void(int)>* job_ = nullptr;
  std::atomic<int> pending_{0};
  std::atomic<uint64_t> gen_{0};
  std::atomic<bool> stop_{false};
};

// Workers for the pool on this host: half the hardware threads less one, at most MSH_POOL_MAX - 1
// (the caller runs a part too). A one-GPU job on the MI355X pool gets a 16-CPU share.
#ifndef MSH_POOL_MAX
#define MSH_POOL_MAX 16
#endif
inline int host_pool_workers() {
  const unsigned hw = std::thread::hardware_concurrency();
  return (int)std::min<unsigned>(MSH_POOL_MAX - 1, hw > 2 ? hw / 2 - 1 : 0u);
}

// The process-wide pool's state: atomics only (no mutex a fork could leave locked in the child).
struct SharedPool {
  std::atomic<int> state{0};  // 0 not created, 1 being created, 2 ready, 3 none (no workers / failed)
  std::atomic<int> busy{0};   // one run at a time
  HostPool* pool = nullptr;
  pid_t owner = 0;            // the process whose threads these are
};
inline SharedPool& shared_pool_state() {
  static SharedPool s;
  return s;
}

// RAII lease of the shared pool: get() is the pool, or nullptr (run on the calling thread).
class PoolLease {
 public:
  PoolLease() {
    SharedPool& s = shared_pool_state();
    int st = s.state.load(std::memory_order_acquire);
    if (st == 0) {
      int zero = 0;
      if (!s.state.compare_exchange_strong(zero, 1, std::memory_order_acq_rel)) return;  // another thread creates it
      const int w = host_pool_workers();
      s.pool = w > 0 ? HostPool::create(w) : nullptr;
      s.owner = getpid();
      s.state.store(s.pool ? 2 : 3, std::memory_order_release);
      st = s.pool ? 2 : 3;
    }
    if (st != 2 || s.owner != getpid()) return;  // none, still being created, or a forked child
    int free_ = 0;
    if (!s.busy.compare_exchange_strong(free_, 1, std::memory_order_acquire)) return;
    pool_ = s.pool;
  }
  ~PoolLease() {
    if (pool_) shared_pool_state().busy.store(0, std::memory_order_release);
  }
  PoolLease(const PoolLease&) = delete;
  PoolLease& operator=(const PoolLease&) = delete;
  HostPool* get() const { return pool_; }

 private:
  HostPool* pool_ = nullptr;
};

}  // namespace msh
