// workers.h — the engine actor's host thread pool (backend.cpp): the text
// staging and response fill of large go() calls run on a few threads, the
// caller joining in.  Header-only so that tests/sanitize/workers_stress.cpp
// drives it under ThreadSanitizer.
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace fnnue {

// A few host threads for the per-batch loops of large calls (the caller joins
// in): chunks of [0, n) handed out by an atomic counter.  Only as many workers
// as there are chunks besides the caller's take part (a ticket each), so the
// caller of a small loop waits for those alone to check in.
class Workers {
 public:
  void start(int n) {
    for (int i = 1; i < n; ++i) th_.emplace_back([this] { loop(); });
  }
  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
    }
    cv_.notify_all();
    for (std::thread& t : th_) t.join();
    th_.clear();
  }
  // f(lo, hi) over [0, n) in chunks of `grain` items
  void run(size_t n, size_t grain, const std::function<void(size_t, size_t)>& f) {
    if (!n) return;
    if (th_.empty() || n <= grain) {
      f(0, n);
      return;
    }
    const size_t chunks = (n + grain - 1) / grain;
    const size_t want = std::min(th_.size(), chunks - 1);
    {
      std::lock_guard<std::mutex> lk(mu_);
      task_ = &f;
      total_ = n;
      step_ = grain;
      next_ = 0;
      active_ = want;
      tickets_ = want;
      ++gen_;
    }
    // (notify_one per ticket lost wake-ups under glibc's condition variable
    // in a CPU stress test: the workers without a ticket go back to sleep)
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return active_ == 0; });
    task_ = nullptr;
  }

 private:
  void work() {
    for (;;) {
      const size_t lo = next_.fetch_add(step_);
      if (lo >= total_) return;
      (*task_)(lo, std::min(lo + step_, total_));
    }
  }
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return quit_ || (gen_ != seen && tickets_ > 0); });
      if (quit_) return;
      seen = gen_;
      --tickets_;
      lk.unlock();
      work();
      lk.lock();
      if (--active_ == 0) done_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(size_t, size_t)>* task_ = nullptr;
  size_t total_ = 0, step_ = 1, active_ = 0, tickets_ = 0;
  std::atomic<size_t> next_{0};
  uint64_t gen_ = 0;
  bool quit_ = false;
};

}  // namespace fnnue
