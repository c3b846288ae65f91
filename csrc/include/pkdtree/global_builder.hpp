// Native global decomposition: ONE exact kd-tree over P ranks (one process or thread per GPU).
//
// The reference only splits its data into independent per-rank trees (kdtree_mpi.cpp:204-253).
// Here the top LL levels (LL = ceil(log2 P) + k) are decided jointly: per level one
// route+histogram pass, an allreduce(SUM) of the histogram, the median bucket per node, one
// compaction pass, a fixed-size all-gather and a radix select of the exact pivot (the device
// ops of dist_ops.hpp). The T = 2^LL top-level leaves are dealt to the ranks in contiguous runs
// (rank r owns leaves [r T / P, (r + 1) T / P): any P, not only powers of two), and every point
// travels to the rank owning its leaf -- coordinates plus one bit per (row, leaf), ids rebuilt
// on the receiver -- in one all-to-all round per leaf of a rank, on a communication stream, so
// round j + 1 is in flight while leaf j builds. For dim <= 8 the coordinates travel as SoA
// planes straight into the leaf builder's input columns (no AoS -> SoA pass on the receiver).
// The result is slot for slot the tree one GPU builds on all points.
//
// Communication goes through the Comm interface: RCCL over xGMI (kdtree_dist and the Python
// extension, one communicator per process) and an in-process loopback (threads) for tests.
#pragma once
#include <hip/hip_runtime.h>

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "pkdtree/common.hpp"
#include "pkdtree/global_plan.hpp"
#include "pkdtree/loopback.hpp"

namespace pkdtree {

// Collectives used by the global builder. Buffers are device memory; every call is enqueued
// on `stream` (the caller orders it after the data's producers) and completes in stream order.
class Comm {
 public:
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  // Blocks until everything enqueued on `stream` (collectives included) has completed. The
  // wait is bounded: after timeout() seconds without completion -- or as soon as the
  // communicator reports an asynchronous error -- it throws a rank-tagged runtime_error, so a
  // stuck or failed peer makes this rank exit non-zero instead of hanging.
  // The base implementation polls the stream; RcclComm also polls ncclCommGetAsyncError and
  // aborts the communicator before throwing.
  virtual void wait(hipStream_t stream, const char* what);
  // The same bound for an event (work enqueued after it on its stream may still be running).
  virtual void wait_event(hipEvent_t event, const char* what);
  void set_timeout(double seconds) { timeout_s_ = seconds; }
  double timeout() const { return timeout_s_; }
  virtual void allreduce_sum_u32(u32* buf, size_t count, hipStream_t stream) = 0;
  virtual void allreduce_min_i64(i64* buf, size_t count, hipStream_t stream) = 0;
  // recv[r * bytes, (r + 1) * bytes) = send of rank r
  virtual void allgather(const void* send, void* recv, size_t bytes, hipStream_t stream) = 0;
  // bytes and offsets per peer (send side: to peer r; receive side: from peer r)
  virtual void alltoallv(const void* send, const size_t* send_bytes, const size_t* send_off, void* recv,
                         const size_t* recv_bytes, const size_t* recv_off, hipStream_t stream) = 0;
  // `planes` all-to-all-v's with the same per-peer layout, plane q at send + q * send_plane /
  // recv + q * recv_plane (SoA columns). RcclComm issues them as one group.
  virtual void alltoallv_planes(const void* send, size_t send_plane, const size_t* send_bytes, const size_t* send_off,
                                void* recv, size_t recv_plane, const size_t* recv_bytes, const size_t* recv_off,
                                int planes, hipStream_t stream);
  // Collectives between group_begin() and group_end() may be fused into one launch (RCCL
  // groups); the loopback communicator ignores them.
  virtual void group_begin() {}
  virtual void group_end() {}

 protected:
  // Polls `stream` until it completes or the deadline passes; `probe` (may be empty) is called
  // between polls and throws on a communicator error. Spins briefly (the plan wait is on the
  // build's critical path), then yields, then sleeps.
  void poll_until_done(hipStream_t stream, const char* what, const std::function<void()>& probe);
  // `query` returns hipSuccess when done, hipErrorNotReady while pending (hipStreamQuery / hipEventQuery)
  void poll_query(const std::function<hipError_t()>& query, const char* what, const std::function<void()>& probe);
  double timeout_s_ = default_timeout();

 private:
  static double default_timeout();  // PKD_COMM_TIMEOUT seconds, default 300
};


// Per-phase times of one profiled build (GlobalBuilder::set_profile): hipEvent milliseconds
// on the build's streams, plan_wait_ms on the host clock.
struct GlobalPhases {
  double top_ms = 0, pack_ms = 0, plan_wait_ms = 0, exchange_ms = 0, exchange_span_ms = 0, ids_ms = 0,
         leaf_ms = 0, total_ms = 0;
  i64 sent_bytes = 0, recv_bytes = 0, max_peer_bytes = 0;  // exchange payload, self excluded
  int rounds = 0, retries = 0;
  std::map<std::string, double> as_map() const;
};

class GpuBuilder;

class GlobalBuilder {
 public:
  GlobalBuilder(Comm& comm, i64 n_total, int dim, int pipeline_k = -1);
  ~GlobalBuilder();
  GlobalBuilder(const GlobalBuilder&) = delete;
  GlobalBuilder& operator=(const GlobalBuilder&) = delete;

  // This rank's points [n_local][dim] (device), ids id_base + row (the reference's global
  // 1-based ids are first_row + 1 + row). Synchronises once (the exchange plan), with the
  // communicator's deadline.
  void build(const float* pts, i64 n_local, u32 id_base, hipStream_t stream);
  // Waits (bounded, see Comm::wait) until the last build has completed on `stream`.
  void wait(hipStream_t stream) { comm_.wait(stream, "global build"); }

  const global_plan::Layout& layout() const { return lay_; }
  // This rank's share of the tree: slots [slot_lo, slot_lo + n_leaf) of the global in-order tree.
  i64 slot_lo() const { return lay_.share_lo[size_t(rank_)]; }
  i64 n_leaf() const { return lay_.share_n[size_t(rank_)]; }
  int top_levels() const { return lay_.LL; }
  // all-gather slot scale of the middle buckets (stays 1: an overflow switches to radix rounds)
  int middle_scale() const { return scale_; }
  // the top levels find their medians by distributed radix rounds (set by a middle-bucket
  // overflow: duplicate-heavy or skewed data; sticky across builds)
  bool radix_mode() const { return radix_; }
  const float* tree_pts() const { return tree_pts_; }
  const u32* tree_ids() const { return tree_ids_; }
  // The T - 1 top-tree rows, heap order: dim + 1 floats (coordinates, id bits) on the device.
  const float* top_rows() const { return top_rows_; }
  // Slots of the boundary top nodes (heap order, -1: empty or inside a share).
  std::vector<i64> top_slots() const;
  // OR of the device error words of the last build (0 = ok). Synchronises `stream`.
  u32 read_error(hipStream_t stream) const;
  // Exact 1-NN of Q queries (device [Q][dim], replicated on every rank) over the whole tree of
  // the last build, packed (d2 << 32 | id) into out[Q] on every rank. Routed (dim <= 16):
  // each query is searched first only in its home block (the leaf its top-tree descent
  // reaches; ~Q / P searches per rank), one MIN all-reduce gives it a radius, then only in the
  // blocks whose cell that radius reaches, and a second MIN all-reduce combines. dim > 16
  // (no pruning to gain): every block, one all-reduce. Every rank must call it (collectives).
  // Returns this rank's (query, block) searches when `count_work` (synchronises), else -1.
  // method: kQueryAuto (routed traversal for dim <= 16, else brute force over every block),
  // kQueryTraverse (routed traversal at any dim), kQueryBrute (brute force over every block).
  enum { kQueryAuto = 0, kQueryTraverse = 1, kQueryBrute = 2 };
  i64 query(const float* queries, i64 Q, u64* out, hipStream_t stream, bool count_work = false,
            int method = kQueryAuto);
  // Per-phase hipEvent timing of the following builds (adds event records, no host syncs).
  void set_profile(bool on);
  GlobalPhases phases(hipStream_t stream) const;  // of the last profiled build; synchronises

 private:
  void* buf(int slot, size_t bytes);
  GpuBuilder& leaf_builder(i64 n, int depth, bool allow_top = true);
  void ensure_leaf_workspace(size_t bytes);
  hipEvent_t ev(int i) const { return events_[size_t(i)]; }

  Comm& comm_;
  i64 n_total_;
  int dim_, P_, rank_;
  global_plan::Layout lay_;
  bool planar_;  // dim <= 8: SoA planes into the leaf builder's columns
  int scale_ = 1;
  bool radix_ = false;
  float* tree_pts_ = nullptr;
  u32* tree_ids_ = nullptr;
  float* top_rows_ = nullptr;
  hipStream_t comm_stream_ = nullptr;
  i64* host_counts_ = nullptr;  // pinned copy of the all-gathered count matrix
  size_t host_counts_n_ = 0;
  std::vector<std::pair<void*, size_t>> bufs_;
  struct Leaf;
  std::vector<std::unique_ptr<Leaf>> leaves_;
  void* leaf_ws_ = nullptr;  // one workspace shared by the leaf builds (they run in stream order)
  size_t leaf_ws_bytes_ = 0;
  std::vector<hipEvent_t> arrived_;  // per round (untimed), created once
  hipEvent_t packed_ = nullptr;
  hipEvent_t counted_ = nullptr;     // the per-leaf counts are written (the pack's first step)
  hipEvent_t plan_ready_ = nullptr;  // the all-gathered counts are in host memory
  bool profile_ = false;
  std::vector<hipEvent_t> events_;  // timed events of a profiled build (see set_profile)
  GlobalPhases last_;               // host-side parts of the last profiled build
};

// In-process loopback communicator: `size` ranks are threads of one process (sharing one GPU
// or not); collectives stage through the host and meet at a barrier. For tests of the P > 1
// orchestration without several GPUs.
std::vector<std::unique_ptr<Comm>> make_thread_comms(int size);

// Emulation of ONE rank of a P-rank global build on one GPU, timed as a whole chain: the P ranks
// first run once as threads over the loopback communicator, with every collective output of
// rank `rank` recorded; then rank `rank` alone builds again (profiled, `reps` times) against a
// replay communicator whose collectives are stream-ordered device copies of those recorded
// outputs. Its kernels, host waits and stream dependencies are the real ones; the exchange
// costs a device copy instead of the xGMI transfer (report it separately). x: the host points
// [N][dim] (rank r holds the reference's MPI slice r). Returns the phases of the last replay
// and whether its share equals the loopback run's share slot for slot.
struct RankEmulation {
  GlobalPhases phases;
  std::vector<double> total_ms;  // per replay
  bool same_tree = false;
  u32 error = 0;
  int collectives = 0;
};
RankEmulation emulate_rank(const float* x_host, i64 N, int dim, int P, int rank, int pipeline_k, int reps);

}  // namespace pkdtree
