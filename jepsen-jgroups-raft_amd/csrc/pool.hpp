// pool.hpp — the host worker pool of liblincheck.so (product code): the encoder (a4/a8) and
// the dense step-stream builder run their per-history work on it. Workers persist for the
// process, so their per-thread scratch (encode.cpp's Scratch) stays allocated and warm from
// one lc_check to the next, and a call pays no thread creation. Items are taken from a shared
// counter (dynamic scheduling: histories differ in length). One job at a time; concurrent
// callers (lc_check shards on several devices) queue on the submit mutex.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace lc {

class Pool {
 public:
  // workers: LC_ENC_THREADS, else the cores this process may use, at most 16 (a GPU box's CPU
  // share per GPU); the calling thread works too
  static Pool& get() {
    static Pool* p = new Pool();  // never destroyed: workers may outlive static destructors
    return *p;
  }
  int threads() const { return (int)th_.size() + 1; }

  // fn(i) for every i in [0, n), on up to max_threads threads (the caller included)
  void run(int n, int max_threads, const std::function<void(int)>& fn) {
    if (n <= 0) return;
    const int nt = std::max(1, std::min({max_threads, threads(), n}));
    if (nt == 1) {
      for (int i = 0; i < n; ++i) fn(i);
      return;
    }
    std::lock_guard<std::mutex> submit(submit_);
    {
      std::lock_guard<std::mutex> lk(m_);
      fn_ = &fn;
      n_ = n;
      next_.store(0, std::memory_order_relaxed);
      want_ = nt - 1;
      busy_ = 0;
      ++gen_;
    }
    cv_.notify_all();
    work();
    // items are all taken: workers that have not woken yet stay out, the busy ones finish
    std::unique_lock<std::mutex> lk(m_);
    want_ = 0;
    done_.wait(lk, [&] { return busy_ == 0; });
    fn_ = nullptr;
  }

 private:
  Pool() {
    const char* e = getenv("LC_ENC_THREADS");
    int n = e && atoi(e) > 0 ? atoi(e) : (int)std::thread::hardware_concurrency();
    n = std::max(1, std::min(n, 16));
    for (int i = 1; i < n; ++i) th_.emplace_back([this] { loop(); });
    for (auto& t : th_) t.detach();
  }
  void work() {
    for (;;) {
      const int i = next_.fetch_add(1, std::memory_order_relaxed);
      if (i >= n_) break;
      (*fn_)(i);
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen && want_ > 0; });
        seen = gen_;
        --want_;
        ++busy_;
      }
      work();
      {
        std::lock_guard<std::mutex> lk(m_);
        --busy_;
      }
      done_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex submit_, m_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_ = 0, want_ = 0, busy_ = 0;
  uint64_t gen_ = 0;
  std::atomic<int> next_{0};
};

}  // namespace lc
