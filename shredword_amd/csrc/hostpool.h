// A small persistent pool of host threads for the staging copies of sw_encode_batch's pipeline
// (pageable caller buffers <-> pinned staging buffers): parallel_for splits [0, n) into one
// contiguous piece per thread and returns when every piece is done.
#pragma once
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace sw {

class HostPool {
 public:
  explicit HostPool(int n) {
    for (int i = 0; i < n; ++i) workers_.emplace_back([this, i] { loop(i); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  int size() const { return (int)workers_.size() + 1; }
  // fn(lo, hi) over size() contiguous pieces of [0, n); the calling thread takes the first
  void parallel_for(int64_t n, const std::function<void(int64_t, int64_t)>& fn) {
    const int parts = size();
    if (n <= 0) return;
    {
      std::lock_guard<std::mutex> g(m_);
      fn_ = &fn;
      n_ = n;
      pending_ = parts - 1;
      ++gen_;
    }
    cv_.notify_all();
    fn(0, piece(n, 0, parts));
    std::unique_lock<std::mutex> g(m_);
    done_cv_.wait(g, [this] { return pending_ == 0; });
    fn_ = nullptr;
  }

 private:
  static int64_t piece(int64_t n, int k, int parts) {  // end of piece k (pieces are 64-byte aligned)
    const int64_t e = ((n * (k + 1) / parts) + 63) & ~(int64_t)63;
    return e < n ? e : n;
  }
  void loop(int i) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int64_t, int64_t)>* fn;
      int64_t n;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        fn = fn_;
        n = n_;
      }
      const int parts = (int)workers_.size() + 1;
      const int64_t lo = piece(n, i, parts), hi = piece(n, i + 1, parts);
      if (fn && lo < hi) (*fn)(lo, hi);
      {
        std::lock_guard<std::mutex> g(m_);
        if (--pending_ == 0) done_cv_.notify_one();
      }
    }
  }
  std::vector<std::thread> workers_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int64_t, int64_t)>* fn_ = nullptr;
  int64_t n_ = 0;
  int pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace sw
