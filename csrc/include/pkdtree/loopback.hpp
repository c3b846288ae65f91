// Host side of the in-process loopback communicator (make_thread_comms, global_builder.hpp):
// `size` ranks are threads of one process that meet at barriers and exchange HOST byte
// buffers. No HIP here -- the device <-> host copies around each collective belong to the
// communicator -- so the hand-offs between the threads are unit-tested under ThreadSanitizer
// (csrc/tests/tsan_loopback.cpp) without a GPU. This is the reference's "ranks as processes on
// one host" test story (Makefile:36, mpirun -np 16 --oversubscribe) with threads.
#pragma once

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <vector>

namespace pkdtree {
namespace loopback {

class Hub {
 public:
  explicit Hub(int size, double barrier_timeout_s = 120.0)
      : size_(size), timeout_s_(barrier_timeout_s), slots_(size_t(size)), sbytes_(size_t(size)), soff_(size_t(size)) {}
  int size() const { return size_; }

  // Every rank arrives before any leaves. A rank that fails stops arriving: the others give up
  // after the deadline (a runtime_error) instead of hanging.
  void barrier() {
    std::unique_lock<std::mutex> lk(mu_);
    const long gen = generation_;
    if (++arrived_ == size_) {
      arrived_ = 0;
      ++generation_;
      cv_.notify_all();
    } else if (!cv_.wait_until(lk, deadline(), [&] { return generation_ != gen; })) {
      throw std::runtime_error("loopback communicator: a rank did not reach the barrier in time");
    }
  }

  // out[r * bytes, (r + 1) * bytes) = rank r's `mine` (every rank passes the same `bytes`).
  void allgather(int rank, const void* mine, size_t bytes, std::vector<char>* out) {
    stage(rank, mine, bytes);
    out->resize(bytes * size_t(size_));
    for (int r = 0; r < size_; ++r)
      if (bytes) std::memcpy(out->data() + size_t(r) * bytes, slots_[size_t(r)].data(), bytes);
    barrier();  // every rank has read every slot before any slot is rewritten
  }

  // out[i] = f over the ranks' mine[i] (in rank order).
  template <class T, class F>
  void reduce(int rank, const T* mine, size_t count, F f, std::vector<T>* out) {
    stage(rank, mine, count * sizeof(T));
    out->resize(count);
    if (count) std::memcpy(out->data(), slots_[0].data(), count * sizeof(T));
    for (int r = 1; r < size_; ++r) {
      const T* v = reinterpret_cast<const T*>(slots_[size_t(r)].data());
      for (size_t i = 0; i < count; ++i) (*out)[i] = f((*out)[i], v[i]);
    }
    barrier();
  }

  // Rank p's bytes [send_off[q], + send_bytes[q]) land in rank q's recv at recv_off[p]; the sizes
  // both sides declare must agree (runtime_error otherwise).
  void alltoallv(int rank, const void* send, const size_t* send_bytes, const size_t* send_off, void* recv,
                 const size_t* recv_bytes, const size_t* recv_off) {
    size_t total = 0;
    for (int p = 0; p < size_; ++p) total = std::max(total, send_off[p] + send_bytes[p]);
    {
      std::lock_guard<std::mutex> lk(mu_);
      sbytes_[size_t(rank)].assign(send_bytes, send_bytes + size_);
      soff_[size_t(rank)].assign(send_off, send_off + size_);
    }
    stage(rank, send, total);
    bool bad = false;
    for (int p = 0; p < size_; ++p) {
      const size_t n = sbytes_[size_t(p)][size_t(rank)];
      if (n != recv_bytes[p]) {
        bad = true;
        continue;
      }
      if (n)
        std::memcpy(static_cast<char*>(recv) + recv_off[p], slots_[size_t(p)].data() + soff_[size_t(p)][size_t(rank)],
                    n);
    }
    barrier();
    if (bad) throw std::runtime_error("loopback alltoallv: size mismatch");
  }

 private:
  // (system_clock: its waits go through pthread_cond_timedwait, which ThreadSanitizer models;
  // the steady-clock wait of this libstdc++ uses pthread_cond_clockwait, which it does not)
  std::chrono::system_clock::time_point deadline() const {
    return std::chrono::system_clock::now() +
           std::chrono::duration_cast<std::chrono::system_clock::duration>(std::chrono::duration<double>(timeout_s_));
  }
  // my bytes -> my slot; every slot is readable after the barrier
  void stage(int rank, const void* host, size_t bytes) {
    auto& v = slots_[size_t(rank)];
    v.resize(bytes);
    if (bytes) std::memcpy(v.data(), host, bytes);
    barrier();
  }

  const int size_;
  const double timeout_s_;
  std::mutex mu_;
  std::condition_variable cv_;
  int arrived_ = 0;
  long generation_ = 0;
  std::vector<std::vector<char>> slots_;            // each rank's staged bytes
  std::vector<std::vector<size_t>> sbytes_, soff_;  // alltoallv: each rank's send layout
};

}  // namespace loopback
}  // namespace pkdtree
