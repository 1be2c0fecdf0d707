// msh_pool.h — a small persistent pool of host threads, shared by the C-ABI's staged copies
// (msh_capi.cpp) and the snapshot packer (msh_pack.cpp). Host code only.
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace msh {

// Persistent host threads: run(f) calls f(0..n-1),
// part 0 on the calling thread, the rest on the workers, and returns when all are done. A worker
// spins on the job counter for a while after each job before it blocks, so back-to-back batches
// do not pay a futex wake-up per call (tens of microseconds on a busy host).
class HostPool {
 public:
  explicit HostPool(int workers) {
    for (int w = 0; w < workers; ++w) th_.emplace_back([this, w] { loop(w + 1); });
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

// Workers for a pool on this host: half the hardware threads less one, at most MSH_POOL_MAX - 1
// (the caller runs a part too). A one-GPU job on the MI355X pool gets a 16-CPU share.
#ifndef MSH_POOL_MAX
#define MSH_POOL_MAX 16
#endif
inline int host_pool_workers() {
  const unsigned hw = std::thread::hardware_concurrency();
  return (int)std::min<unsigned>(MSH_POOL_MAX - 1, hw > 2 ? hw / 2 - 1 : 0u);
}

}  // namespace msh
