// The global builder's communicator on RCCL (xGMI between the GPUs of a node): allreduce and
// allgather as single collectives, the all-to-all-v as one grouped set of point-to-point
// sends and receives (xGMI links are point-to-point), the self part as a device copy.
// Used by kdtree_dist (both decompositions) and by the Python extension (bench.py at N > 1).
//
// Failure detection: wait() polls the stream and ncclCommGetAsyncError until
// the communicator's deadline; a stuck peer or an asynchronous RCCL error aborts the
// communicator (so this rank's RCCL kernels stop and the process can exit) and throws a
// rank-tagged error.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdexcept>
#include <string>

#include "pkdtree/global_builder.hpp"
#include "pkdtree/hip_check.hpp"

namespace pkdtree {

inline void nccl_check(ncclResult_t r, const char* expr, int rank) {
  if (r != ncclSuccess)
    throw std::runtime_error("rank " + std::to_string(rank) + ": " + expr + " -> " + ncclGetErrorString(r));
}
#define PKD_RCCL(expr) ::pkdtree::nccl_check((expr), #expr, rank_)

class RcclComm final : public Comm {
 public:
  RcclComm(ncclComm_t c, int rank, int size) : c_(c), rank_(rank), size_(size) {}
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  ncclComm_t handle() const { return c_; }
  bool aborted() const { return aborted_; }
  // Stops the communicator's outstanding operations (idempotent); the handle is then dead and
  // must not be destroyed with ncclCommDestroy.
  void abort() {
    if (!aborted_) {
      aborted_ = true;
      (void)ncclCommAbort(c_);
    }
  }

  void wait(hipStream_t s, const char* what) override {
    wait_query([&] { return hipStreamQuery(s); }, what);
  }
  void wait_event(hipEvent_t e, const char* what) override {
    wait_query([&] { return hipEventQuery(e); }, what);
  }
  void wait_query(const std::function<hipError_t()>& query, const char* what) {
    try {
      poll_query(query, what, [&] {
        ncclResult_t async = ncclSuccess;
        PKD_RCCL(ncclCommGetAsyncError(c_, &async));
        if (async != ncclSuccess)
          throw std::runtime_error("rank " + std::to_string(rank_) + ": " + what + ": asynchronous RCCL error " +
                                   ncclGetErrorString(async));
      });
    } catch (...) {
      abort();
      throw;
    }
  }
  void allreduce_sum_u32(u32* buf, size_t count, hipStream_t s) override {
    PKD_RCCL(ncclAllReduce(buf, buf, count, ncclUint32, ncclSum, c_, s));
  }
  void allreduce_min_i64(i64* buf, size_t count, hipStream_t s) override {
    PKD_RCCL(ncclAllReduce(buf, buf, count, ncclInt64, ncclMin, c_, s));
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    PKD_RCCL(ncclAllGather(send, recv, bytes, ncclChar, c_, s));
  }
  void alltoallv(const void* send, const size_t* send_bytes, const size_t* send_off, void* recv,
                 const size_t* recv_bytes, const size_t* recv_off, hipStream_t s) override {
    alltoallv_planes(send, 0, send_bytes, send_off, recv, 0, recv_bytes, recv_off, 1, s);
  }
  void alltoallv_planes(const void* send, size_t send_plane, const size_t* send_bytes, const size_t* send_off,
                        void* recv, size_t recv_plane, const size_t* recv_bytes, const size_t* recv_off, int planes,
                        hipStream_t s) override {
    const char* sp = static_cast<const char*>(send);
    char* rp = static_cast<char*>(recv);
    if (send_bytes[rank_] != recv_bytes[rank_]) throw std::runtime_error("alltoallv: self size mismatch");
    if (send_bytes[rank_]) {  // the self part of every plane: one strided device copy
      PKD_HIP_CHECK(hipMemcpy2DAsync(rp + recv_off[rank_], planes > 1 ? recv_plane : send_bytes[rank_],
                                     sp + send_off[rank_], planes > 1 ? send_plane : send_bytes[rank_],
                                     send_bytes[rank_], size_t(planes), hipMemcpyDeviceToDevice, s));
    }
    PKD_RCCL(ncclGroupStart());
    for (int q = 0; q < planes; ++q)
      for (int p = 0; p < size_; ++p) {
        if (p == rank_) continue;
        if (send_bytes[p])
          PKD_RCCL(ncclSend(sp + size_t(q) * send_plane + send_off[p], send_bytes[p], ncclChar, p, c_, s));
        if (recv_bytes[p])
          PKD_RCCL(ncclRecv(rp + size_t(q) * recv_plane + recv_off[p], recv_bytes[p], ncclChar, p, c_, s));
      }
    PKD_RCCL(ncclGroupEnd());
  }
  void group_begin() override { PKD_RCCL(ncclGroupStart()); }
  void group_end() override { PKD_RCCL(ncclGroupEnd()); }

 private:
  ncclComm_t c_;
  int rank_, size_;
  bool aborted_ = false;
};

#undef PKD_RCCL

}  // namespace pkdtree
