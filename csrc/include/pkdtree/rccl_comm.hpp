// The global builder's communicator on RCCL (xGMI between the GPUs of a node): allreduce and
// allgather as single collectives, the all-to-all-v as one grouped set of point-to-point
// sends and receives (xGMI links are point-to-point), the self part as a device copy.
// Used by kdtree_dist --decomp global and by the Python extension (bench.py at N > 1).
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
    const char* sp = static_cast<const char*>(send);
    char* rp = static_cast<char*>(recv);
    if (send_bytes[rank_] != recv_bytes[rank_]) throw std::runtime_error("alltoallv: self size mismatch");
    if (send_bytes[rank_])
      PKD_HIP_CHECK(hipMemcpyAsync(rp + recv_off[rank_], sp + send_off[rank_], send_bytes[rank_],
                                   hipMemcpyDeviceToDevice, s));
    PKD_RCCL(ncclGroupStart());
    for (int p = 0; p < size_; ++p) {
      if (p == rank_) continue;
      if (send_bytes[p]) PKD_RCCL(ncclSend(sp + send_off[p], send_bytes[p], ncclChar, p, c_, s));
      if (recv_bytes[p]) PKD_RCCL(ncclRecv(rp + recv_off[p], recv_bytes[p], ncclChar, p, c_, s));
    }
    PKD_RCCL(ncclGroupEnd());
  }

 private:
  ncclComm_t c_;
  int rank_, size_;
};

#undef PKD_RCCL

}  // namespace pkdtree
