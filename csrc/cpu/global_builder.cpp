// Native global decomposition (see pkdtree/global_builder.hpp): the geometry of who owns what,
// the exchange planner, the build schedule and the loopback communicator. The device work is
// the dist_ops kernels plus one GpuBuilder build per top-level leaf.
#include "pkdtree/global_builder.hpp"

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <numeric>
#include <stdexcept>
#include <string>
#include <thread>

#include "pkdtree/dist_ops.hpp"
#include "pkdtree/gpu_build.hpp"
#include "pkdtree/gpu_query.hpp"
#include "pkdtree/hip_check.hpp"

namespace pkdtree {

// ---------------------------------------------------------------------------------------------
// Comm: bounded waits
double Comm::default_timeout() {
  const char* e = std::getenv("PKD_COMM_TIMEOUT");
  return e ? std::max(0.01, std::atof(e)) : 300.0;
}

void Comm::wait(hipStream_t stream, const char* what) { poll_until_done(stream, what, {}); }
void Comm::wait_event(hipEvent_t event, const char* what) {
  poll_query([&] { return hipEventQuery(event); }, what, {});
}

void Comm::poll_until_done(hipStream_t stream, const char* what, const std::function<void()>& probe) {
  poll_query([&] { return hipStreamQuery(stream); }, what, probe);
}

void Comm::poll_query(const std::function<hipError_t()>& query, const char* what, const std::function<void()>& probe) {
  const auto t0 = std::chrono::steady_clock::now();
  for (long it = 0;; ++it) {
    const hipError_t q = query();
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady)
      throw std::runtime_error("rank " + std::to_string(rank()) + ": " + what + ": " + hipGetErrorString(q));
    if (probe && (it & 63) == 0) probe();
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > timeout_s_)
      throw std::runtime_error("rank " + std::to_string(rank()) + ": " + what + ": not complete after " +
                               std::to_string(timeout_s_) + " s (watchdog: a peer rank is stuck or gone)");
    // The plan wait sits on the build's critical path: spin for the first 2 ms (the usual case
    // ends within tens of microseconds), then yield, then sleep.
    if (el < 2e-3) continue;
    if (el < 20e-3) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

void Comm::alltoallv_planes(const void* send, size_t send_plane, const size_t* send_bytes, const size_t* send_off,
                            void* recv, size_t recv_plane, const size_t* recv_bytes, const size_t* recv_off,
                            int planes, hipStream_t stream) {
  for (int q = 0; q < planes; ++q)
    alltoallv(static_cast<const char*>(send) + size_t(q) * send_plane, send_bytes, send_off,
              static_cast<char*>(recv) + size_t(q) * recv_plane, recv_bytes, recv_off, stream);
}

std::map<std::string, double> GlobalPhases::as_map() const {
  return {{"top_ms", top_ms},
          {"pack_ms", pack_ms},
          {"plan_wait_ms", plan_wait_ms},
          {"exchange_ms", exchange_ms},
          {"exchange_span_ms", exchange_span_ms},
          {"ids_ms", ids_ms},
          {"leaf_ms", leaf_ms},
          {"total_ms", total_ms},
          {"sent_bytes", double(sent_bytes)},
          {"recv_bytes", double(recv_bytes)},
          {"max_peer_bytes", double(max_peer_bytes)},
          {"rounds", double(rounds)},
          {"retries", double(retries)}};
}

// ---------------------------------------------------------------------------------------------

// ---------------------------------------------------------------------------------------------
struct GlobalBuilder::Leaf {
  i64 n;
  int depth;
  bool top;
  std::unique_ptr<GpuBuilder> b;
};

namespace {
// timed events of a profiled build: 4 build-wide, then 5 per round
enum { kEvStart = 0, kEvTop = 1, kEvPack = 2, kEvEnd = 3, kEvRound = 4 };
enum { kRxBegin = 0, kRxEnd = 1, kIdsBegin = 2, kIdsEnd = 3, kLeafEnd = 4, kPerRound = 5 };
int round_ev(int j, int which) { return kEvRound + kPerRound * j + which; }
}  // namespace

GlobalBuilder::GlobalBuilder(Comm& comm, i64 n_total, int dim, int pipeline_k)
    : comm_(comm), n_total_(n_total), dim_(dim), P_(comm.size()), rank_(comm.rank()) {
  if (n_total >= (i64(1) << 32)) throw std::invalid_argument("point ids are 32-bit: at most 2^32 - 1 points");
  if (n_total < 0) throw std::invalid_argument("n_total must be >= 0");
  if (dim < 1) throw std::invalid_argument("dim must be >= 1");
  lay_ = global_plan::make_layout(n_total, P_, pipeline_k);
  planar_ = dim <= 8;
  PKD_HIP_CHECK(hipStreamCreateWithFlags(&comm_stream_, hipStreamNonBlocking));
  arrived_.assign(size_t(lay_.R), nullptr);
  for (auto& e : arrived_) PKD_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  PKD_HIP_CHECK(hipEventCreateWithFlags(&packed_, hipEventDisableTiming));
  PKD_HIP_CHECK(hipEventCreateWithFlags(&counted_, hipEventDisableTiming));
  PKD_HIP_CHECK(hipEventCreateWithFlags(&plan_ready_, hipEventDisableTiming));
}

GlobalBuilder::~GlobalBuilder() {
  for (auto& b : bufs_)
    if (b.first) (void)hipFree(b.first);
  if (tree_pts_) (void)hipFree(tree_pts_);
  if (tree_ids_) (void)hipFree(tree_ids_);
  if (leaf_ws_) (void)hipFree(leaf_ws_);
  for (hipEvent_t e : arrived_) (void)hipEventDestroy(e);
  for (hipEvent_t e : events_) (void)hipEventDestroy(e);
  if (packed_) (void)hipEventDestroy(packed_);
  if (counted_) (void)hipEventDestroy(counted_);
  if (plan_ready_) (void)hipEventDestroy(plan_ready_);
  if (comm_stream_) (void)hipStreamDestroy(comm_stream_);
  if (host_counts_) (void)hipHostFree(host_counts_);
}

void* GlobalBuilder::buf(int slot, size_t bytes) {
  if (bufs_.size() <= size_t(slot)) bufs_.resize(size_t(slot) + 1, {nullptr, 0});
  auto& b = bufs_[size_t(slot)];
  bytes = std::max<size_t>(bytes, 256);
  if (b.second < bytes) {
    if (b.first) PKD_HIP_CHECK(hipFree(b.first));
    PKD_HIP_CHECK(hipMalloc(&b.first, bytes));
    b.second = bytes;
  }
  return b.first;
}

GpuBuilder& GlobalBuilder::leaf_builder(i64 n, int depth, bool allow_top) {
  for (auto& l : leaves_)
    if (l->n == n && l->depth == depth && l->top == allow_top) return *l->b;
  auto l = std::make_unique<Leaf>();
  l->n = n;
  l->depth = depth;
  l->top = allow_top;
  // no split build inside a distributed build: its side streams plus the caller's and the
  // communication stream would exceed the 4 hardware queues, and RCCL's kernels would queue
  // behind partition passes
  // sampled top levels from the received columns at >= 10 M points (a band miss reports error
  // bit 0x20; build() then rebuilds that leaf with allow_top = false from the same columns,
  // which a sampled build reads without clobbering)
  l->b = std::make_unique<GpuBuilder>(n, dim_, BuildOptions{0, depth, false, allow_top});
  leaves_.push_back(std::move(l));
  return *leaves_.back()->b;
}

void GlobalBuilder::ensure_leaf_workspace(size_t bytes) {
  bytes = std::max<size_t>(bytes, 256);
  if (leaf_ws_bytes_ >= bytes) return;
  if (leaf_ws_) PKD_HIP_CHECK(hipFree(leaf_ws_));
  PKD_HIP_CHECK(hipMalloc(&leaf_ws_, bytes));
  leaf_ws_bytes_ = bytes;
}

std::vector<i64> GlobalBuilder::top_slots() const {
  std::vector<i64> s(size_t(std::max(lay_.T - 1, 0)), -1);
  for (int h = 0; h + 1 < lay_.T; ++h)
    if (lay_.top_owner[size_t(h)] < 0) s[size_t(h)] = lay_.top_slot[size_t(h)];
  return s;
}

u32 GlobalBuilder::read_error(hipStream_t stream) const {
  comm_.wait(stream, "read error");  // bounded: a stuck peer aborts the communicator instead of hanging here
  if (bufs_.size() <= 5 || !bufs_[5].first) return 0;
  u32 w[4];
  PKD_HIP_CHECK(hipMemcpy(w, bufs_[5].first, 16, hipMemcpyDeviceToHost));
  return (w[0] & 8u) | w[1];  // the compact exchange's bitmap check | the leaf builds' error words
}

i64 GlobalBuilder::query(const float* queries, i64 Q, u64* out, hipStream_t s, bool count_work, int method) {
  if (Q <= 0) return 0;
  const int dim = dim_;
  std::vector<global_plan::Block> all;
  std::vector<i64> between;
  global_plan::share_blocks(lay_, rank_, &all, &between);
  std::vector<global_plan::Block> bl;
  for (const auto& b : all)
    if (b.n > 0) bl.push_back(b);
  const int nb = int(bl.size());
  if (nb > kRqMaxBlocks) throw std::runtime_error("GlobalBuilder::query: more than 64 blocks");
  const bool routed = method == kQueryTraverse || (method == kQueryAuto && dim <= 16);
  auto* counts = static_cast<u32*>(buf(301, size_t(std::max(nb, 1)) * 4));
  nn_init(out, Q, s);
  // the top rows between this rank's blocks, and on rank 0 the boundary top rows: brute force
  auto brute_tops = [&] {
    for (i64 h : between) {
      const i64 off = lay_.top_slot[size_t(h)] - slot_lo();
      nn_brute(tree_pts_ + off * dim, tree_ids_ + off, 0, 1, dim, queries, Q, out, s);
    }
    if (rank_ == 0 && P_ > 1) {
      const std::vector<i64> slots = top_slots();
      std::vector<int> hs;
      for (size_t h = 0; h < slots.size(); ++h)
        if (slots[h] >= 0) hs.push_back(int(h));
      if (!hs.empty()) {
        auto* tp = static_cast<float*>(buf(304, hs.size() * size_t(dim) * 4));
        auto* ti = static_cast<u32*>(buf(305, hs.size() * 4));
        for (size_t k = 0; k < hs.size(); ++k) {
          const float* row = top_rows_ + size_t(hs[k]) * (dim + 1);
          PKD_HIP_CHECK(hipMemcpyAsync(tp + k * dim, row, size_t(dim) * 4, hipMemcpyDeviceToDevice, s));
          PKD_HIP_CHECK(hipMemcpyAsync(ti + k, row + dim, 4, hipMemcpyDeviceToDevice, s));
        }
        nn_brute(tp, ti, 0, i64(hs.size()), dim, queries, Q, out, s);
      }
    }
  };
  if (!routed) {
    for (const auto& b : bl)
      nn_brute(tree_pts_ + b.off * dim, tree_ids_ + b.off, 0, b.n, dim, queries, Q, out, s);
    brute_tops();
    comm_.allreduce_min_i64(reinterpret_cast<i64*>(out), size_t(Q), s);
    return count_work ? i64(nb) * Q : -1;
  }
  RqBlocks rb{};
  rb.nb = nb;
  rb.LL = lay_.LL;
  rb.T = lay_.T;
  rb.depth0 = 0;
  for (int t = 0; t < 64; ++t) rb.leaf_block[t] = -1;
  for (int i = 0; i < nb; ++i) {
    rb.heap[i] = bl[size_t(i)].heap;
    const int sh = lay_.LL - bl[size_t(i)].depth;  // levels between the block root and the leaves
    const i64 first = ((bl[size_t(i)].heap + 1) << sh) - lay_.T;
    for (i64 t = first; t < first + (i64(1) << sh); ++t) rb.leaf_block[t] = i;
  }
  auto* lists = static_cast<u32*>(buf(300, size_t(std::max(nb, 1)) * size_t(Q) * 4));
  auto* home = static_cast<int*>(buf(302, size_t(Q) * 4));
  i64 work = 0;
  auto search = [&] {
    for (int i = 0; i < nb; ++i)
      nn_traverse_sel(tree_pts_ + bl[size_t(i)].off * dim, tree_ids_ + bl[size_t(i)].off, bl[size_t(i)].n, dim,
                      bl[size_t(i)].depth, queries, lists + size_t(i) * Q, counts + i, Q, out, s);
    if (count_work && nb > 0) {
      std::vector<u32> c(static_cast<size_t>(nb));
      PKD_HIP_CHECK(hipMemcpyAsync(c.data(), counts, size_t(nb) * 4, hipMemcpyDeviceToHost, s));
      comm_.wait(s, "query work count");
      for (u32 v : c) work += v;
    }
  };
  // 1. home blocks
  fill_u32(counts, std::max(nb, 1), 0u, s);
  rq_home(queries, Q, dim, top_rows_, rb, lists, counts, home, s);
  search();
  brute_tops();
  comm_.allreduce_min_i64(reinterpret_cast<i64*>(out), size_t(Q), s);
  // 2. blocks the best ball reaches
  fill_u32(counts, std::max(nb, 1), 0u, s);
  rq_reach(queries, Q, dim, top_rows_, rb, out, home, lists, counts, s);
  search();
  comm_.allreduce_min_i64(reinterpret_cast<i64*>(out), size_t(Q), s);
  return count_work ? work : -1;
}

void GlobalBuilder::set_profile(bool on) {
  profile_ = on;
  if (on && events_.empty()) {
    events_.resize(size_t(kEvRound + kPerRound * lay_.R));
    for (auto& e : events_) PKD_HIP_CHECK(hipEventCreate(&e));
  }
}

GlobalPhases GlobalBuilder::phases(hipStream_t stream) const {
  if (events_.empty()) throw std::runtime_error("GlobalBuilder::phases: no profiled build (set_profile(true))");
  comm_.wait(stream, "global build (profile)");
  auto el = [&](int a, int b) {
    float ms = 0;
    PKD_HIP_CHECK(hipEventElapsedTime(&ms, ev(a), ev(b)));
    return double(ms);
  };
  GlobalPhases p = last_;
  p.top_ms = el(kEvStart, kEvTop);
  p.pack_ms = el(kEvTop, kEvPack);
  p.total_ms = el(kEvStart, kEvEnd);
  const int R = lay_.R, mine = lay_.leaf_lo[size_t(rank_) + 1] - lay_.leaf_lo[size_t(rank_)];
  for (int j = 0; j < R; ++j) p.exchange_ms += el(round_ev(j, kRxBegin), round_ev(j, kRxEnd));
  p.exchange_span_ms = el(round_ev(0, kRxBegin), round_ev(R - 1, kRxEnd));
  for (int j = 0; j < mine; ++j) {
    p.ids_ms += el(round_ev(j, kIdsBegin), round_ev(j, kIdsEnd));
    p.leaf_ms += el(round_ev(j, kIdsEnd), round_ev(j, kLeafEnd));
  }
  return p;
}

void GlobalBuilder::build(const float* pts, i64 n_local, u32 id_base, hipStream_t s) {
  const int dim = dim_, P = P_, me = rank_, LL = lay_.LL, T = lay_.T, R = lay_.R;
  const TopPoints tp{pts, nullptr, n_local, dim, id_base};
  global_plan::Plan plan;
  float* top_rows = nullptr;
  GlobalPhases info;
  if (profile_) PKD_HIP_CHECK(hipEventRecord(ev(kEvStart), s));
  // send side: planar (SoA, dim <= 8) or 12-B rows; one bitmap of send_words words per leaf
  const i64 send_stride = planar_ ? std::max<i64>(64, (n_local + 63) / 64 * 64) : 0;
  const i64 send_words = std::max<i64>(1, (n_local + 31) / 32);
  for (;;) {  // until no middle bucket overflows its all-gather slot
    // 1. bounding box: one allreduce(MIN) of the encoded per-rank boxes
    auto* box = static_cast<i64*>(buf(0, size_t(2 * dim) * 8));
    auto* cells = static_cast<float*>(buf(1, size_t(2 * T - 1) * dim * 2 * 4));
    auto* node = static_cast<u32*>(buf(2, size_t(std::max<i64>(n_local, 1)) * 4));
    auto* pivots = static_cast<u64*>(buf(3, size_t(std::max(T - 1, 1)) * 8));
    top_rows = static_cast<float*>(buf(4, size_t(std::max(T - 1, 1)) * (dim + 1) * 4 + 8));  // + 8: 64-bit fill
    auto* err = static_cast<u32*>(buf(5, 16));
    auto* sel = static_cast<u32*>(buf(6, size_t(kTopMaxNodes) * 4 * 4));
    u32* hist[2] = {static_cast<u32*>(buf(7, size_t(kTopBins) * 4)), static_cast<u32*>(buf(17, size_t(kTopBins) * 4))};
    {  // the top phase's initial state, one launch
      FillSegs f;
      f.add(box, 2 * dim, 0xffffffffull);
      f.add(pivots, std::max(T - 1, 1), ~0ull);
      f.add(top_rows, (i64(std::max(T - 1, 1)) * (dim + 1) + 1) / 2, 0ull);
      f.add(err, 2, 0ull);
      if (LL > 0) f.add(hist[0], kTopBins / 2, 0ull);
      fill_u64_multi(f, s);
    }
    top_bbox(tp, box, s);
    comm_.allreduce_min_i64(box, size_t(2 * dim), s);
    top_root_cell(box, dim, cells, s);
    // 2. top levels: level 0's histogram, then per level one fused pass (median-bucket rows
    // staged, every other row routed to its child and counted into the next level's histogram)
    // and, after the pivot, the fix-up of the staged rows
    for (int level = 0; level < LL; ++level) {
      const int nodes = 1 << level, bins = kTopBins / nodes, next_bins = kTopBins / (2 * nodes);
      const int axis = level % dim, next_axis = (level + 1) % dim;
      u32* hcur = hist[level & 1];
      u32* hnext = level + 1 < LL ? hist[(level + 1) & 1] : nullptr;
      TopSizes sizes{};
      for (int j = 0; j < nodes; ++j) {
        i64 lo;
        global_plan::segment(n_total_, nodes - 1 + j, &lo, &sizes.n[j]);
      }
      if (level == 0) top_route_hist(tp, node, 0, pivots, 0, axis, cells, bins, hcur, s);
      comm_.allreduce_sum_u32(hcur, size_t(nodes) * bins, s);
      const i64 cap = global_plan::middle_cap(n_total_, P, level, scale_);
      const size_t words = top_middle_words(dim, cap);
      auto* mid = static_cast<float*>(buf(8, words * 4));
      top_select(hcur, level, bins, sizes, sel, err, hnext, reinterpret_cast<u32*>(mid), s);
      if (radix_) {
        // duplicate-heavy / skewed data (a median bucket outgrew the all-gather slots once):
        // the bucket's rows stay at their node; 8 rounds of a 256-bin digit histogram of the
        // (key, id) composite with one all-reduce each fix the median byte by byte; the one
        // rank holding the median row contributes it to a MIN all-reduce. No P x bucket buffer.
        top_collect_route(tp, node, level, axis, next_axis, cells, bins, next_bins, sel, mid, 0, hnext, s, true);
        auto* rs = static_cast<TopRadix*>(buf(306, size_t(kTopMaxNodes) * sizeof(TopRadix)));
        auto* rh = static_cast<u32*>(buf(307, size_t(kTopMaxNodes) * 256 * 4));
        auto* rowbuf = static_cast<i64*>(buf(308, size_t(kTopMaxNodes) * (dim + 1) * 8));
        top_radix_init(sel, sizes, level, rs, s);
        fill_u32(rh, i64(nodes) * 256, 0u, s);
        for (int pass = 7; pass >= 0; --pass) {
          top_radix_hist(tp, node, level, axis, rs, pass, rh, s);
          comm_.allreduce_sum_u32(rh, size_t(nodes) * 256, s);
          top_radix_sel(rh, level, pass, rs, err, s);  // also re-zeroes rh
        }
        fill_u64(rowbuf, i64(nodes) * (dim + 1), u64(INT64_MAX), s);
        top_radix_row(tp, node, level, axis, rs, rowbuf, s);
        comm_.allreduce_min_i64(rowbuf, size_t(nodes) * (dim + 1), s);
        top_radix_pivot(rowbuf, rs, level, axis, dim, pivots, top_rows, cells, err, s);
        top_radix_fixup(tp, node, level, axis, next_axis, pivots, cells, next_bins, hnext, s);
        continue;
      }
      top_collect_route(tp, node, level, axis, next_axis, cells, bins, next_bins, sel, mid, cap, hnext, s);
      auto* gathered = static_cast<float*>(buf(9, size_t(P) * words * 4));
      comm_.allgather(mid, gathered, words * 4, s);
      top_pivot(gathered, P, cap, level, axis, dim, sizes, sel, pivots, top_rows, cells, err, s);
      top_fixup(mid, cap, dim, level, axis, next_axis, pivots, cells, next_bins, node, hnext, s);
    }
    if (profile_) PKD_HIP_CHECK(hipEventRecord(ev(kEvTop), s));
    // 3. pack by destination leaf: coordinates (planes or rows) + one bit per (row, leaf)
    auto* send = static_cast<float*>(
        buf(10, planar_ ? size_t(dim) * send_stride * 4 : size_t(std::max<i64>(n_local, 1)) * dim * 4));
    auto* counts = static_cast<i64*>(buf(11, size_t(T) * 4 * 8));
    top_counts_init(counts, T, i64(id_base), n_local, s);
    auto* bm = static_cast<u32*>(buf(12, size_t(T) * send_words * 4));
    void* scratch = buf(13, top_pack_scratch_bytes(n_local, T));
    top_pack_count(tp, node, LL, counts, err, scratch, s);
    // 4. the count matrix, all-gathered on the communication stream and read back to the host
    // (the one host read-back of the build, bounded wait) while the pack's scatter runs
    auto* all = static_cast<i64*>(buf(14, size_t(P) * T * 4 * 8));
    const size_t nall = size_t(P) * T * 4;
    if (host_counts_n_ < nall) {
      if (host_counts_) PKD_HIP_CHECK(hipHostFree(host_counts_));
      PKD_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&host_counts_), nall * 8, hipHostMallocDefault));
      host_counts_n_ = nall;
    }
    PKD_HIP_CHECK(hipEventRecord(counted_, s));
    PKD_HIP_CHECK(hipStreamWaitEvent(comm_stream_, counted_, 0));
    comm_.allgather(counts, all, size_t(T) * 4 * 8, comm_stream_);
    PKD_HIP_CHECK(hipMemcpyAsync(host_counts_, all, nall * 8, hipMemcpyDeviceToHost, comm_stream_));
    PKD_HIP_CHECK(hipEventRecord(plan_ready_, comm_stream_));
    top_pack_scatter(tp, node, LL, send, dim, send_stride, bm, send_words, scratch, s);
    if (profile_) PKD_HIP_CHECK(hipEventRecord(ev(kEvPack), s));
    const auto w0 = std::chrono::steady_clock::now();
    comm_.wait_event(plan_ready_, "exchange plan");
    info.plan_wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
    const std::vector<i64> hall(host_counts_, host_counts_ + nall);
    if (global_plan::make_plan(hall, lay_, me, &plan) == 0) break;
    // a median bucket outgrew its all-gather slot: redo the top levels by radix rounds (sticky
    // for the builder; memory stays O(P x the default slot))
    if (radix_) throw std::runtime_error("global top levels: median selection inconsistent in radix mode");
    radix_ = true;
    ++info.retries;
  }
  top_rows_ = top_rows;  // buffer slot 4, exposed through top_rows()

  // 5. everything the rounds need, sized once from the plan: no allocation (and no implicit
  // device synchronisation) once the first exchange is in flight
  const int my_a = lay_.leaf_lo[size_t(me)], mine = lay_.leaf_lo[size_t(me) + 1] - my_a;
  std::vector<i64> src_words(static_cast<size_t>(P)), bm_off(static_cast<size_t>(P));
  i64 bm_total = 0, max_words = 0;
  for (int p = 0; p < P; ++p) {
    src_words[size_t(p)] = std::max<i64>(1, (plan.src_n[size_t(p)] + 31) / 32);
    bm_off[size_t(p)] = bm_total;
    bm_total += src_words[size_t(p)];
    max_words = std::max(max_words, src_words[size_t(p)]);
  }
  const i64 n_share = lay_.share_n[size_t(me)];
  if (!tree_pts_) {
    PKD_HIP_CHECK(hipMalloc(&tree_pts_, size_t(std::max<i64>(n_share, 1)) * dim * 4));
    PKD_HIP_CHECK(hipMalloc(&tree_ids_, size_t(std::max<i64>(n_share, 1)) * 4));
  }
  std::vector<GpuBuilder*> lb(size_t(mine), nullptr);
  std::vector<float*> recv(size_t(R), nullptr);
  std::vector<u32*> recv_bm(size_t(R), nullptr), lids(size_t(R), nullptr);
  std::vector<i64> col_stride(size_t(R), 0);
  size_t ws_need = 0;
  for (int j = 0; j < mine; ++j) {
    // every source sends its bitmap for each of my leaves, empty leaves included
    recv_bm[size_t(j)] = static_cast<u32*>(buf(21 + 3 * j, size_t(bm_total) * 4));
    const i64 n_j = lay_.leaf_n[size_t(my_a + j)];
    if (n_j <= 0) continue;
    GpuBuilder& b = leaf_builder(n_j, LL);
    lb[size_t(j)] = &b;
    ws_need = std::max(ws_need, b.workspace_bytes());
    if (planar_) {
      col_stride[size_t(j)] = b.column_stride();
      recv[size_t(j)] = static_cast<float*>(buf(20 + 3 * j, size_t(dim + 1) * b.column_stride() * 4));
      lids[size_t(j)] = reinterpret_cast<u32*>(recv[size_t(j)] + size_t(dim) * b.column_stride());
    } else {
      recv[size_t(j)] = static_cast<float*>(buf(20 + 3 * j, size_t(n_j) * dim * 4));
      lids[size_t(j)] = static_cast<u32*>(buf(22 + 3 * j, size_t(n_j) * 4));
    }
  }
  ensure_leaf_workspace(ws_need);
  void* ids_scratch = buf(16, ids_from_bitmaps_scratch_bytes(max_words, P));
  auto* send = static_cast<float*>(buf(10, 0));
  auto* bm = static_cast<u32*>(buf(12, 0));
  auto* err = static_cast<u32*>(buf(5, 16));
  auto* leaf_err = static_cast<u32*>(buf(260, size_t(std::max(mine, 1)) * 4));  // each leaf's own error word
  // the top nodes between my leaves are replicated rows: straight into my share
  {
    TopPlacement pl{};
    for (int h = 0; h + 1 < T; ++h)
      if (lay_.top_owner[size_t(h)] == me && lay_.top_slot[size_t(h)] >= 0) {
        pl.heap[pl.count] = h;
        pl.slot[pl.count] = lay_.top_slot[size_t(h)] - lay_.share_lo[size_t(me)];
        ++pl.count;
      }
    top_place_rows(top_rows, dim, pl, tree_pts_, tree_ids_, s);
  }
  // exchange volume (self excluded), for the profile
  {
    std::vector<i64> peer(static_cast<size_t>(P), 0);
    for (int j = 0; j < R; ++j)
      for (int p = 0; p < P; ++p) {
        if (p == me) continue;
        const bool to_leaf = j < lay_.leaf_lo[size_t(p) + 1] - lay_.leaf_lo[size_t(p)];
        const i64 sb = plan.send_rows[size_t(j)][size_t(p)] * dim * 4 + (to_leaf ? send_words * 4 : 0);
        const i64 rb = plan.recv_rows[size_t(j)][size_t(p)] * dim * 4 + (j < mine ? src_words[size_t(p)] * 4 : 0);
        info.sent_bytes += sb;
        info.recv_bytes += rb;
        peer[size_t(p)] += sb;
      }
    info.max_peer_bytes = *std::max_element(peer.begin(), peer.end());
    info.rounds = R;
  }
  PKD_HIP_CHECK(hipEventRecord(packed_, s));
  PKD_HIP_CHECK(hipStreamWaitEvent(comm_stream_, packed_, 0));
  // 6. round j: leaf leaf_lo[q] + j of every rank q that has one, on the communication stream
  auto issue = [&](int j) {
    std::vector<size_t> sb(static_cast<size_t>(P)), so(sb), rb(sb), ro(sb);
    i64 roff = 0;
    for (int p = 0; p < P; ++p) {
      sb[size_t(p)] = size_t(plan.send_rows[size_t(j)][size_t(p)]) * 4 * (planar_ ? 1 : dim);
      so[size_t(p)] = size_t(plan.send_off[size_t(j)][size_t(p)]) * 4 * (planar_ ? 1 : dim);
      rb[size_t(p)] = size_t(plan.recv_rows[size_t(j)][size_t(p)]) * 4 * (planar_ ? 1 : dim);
      ro[size_t(p)] = size_t(roff) * 4 * (planar_ ? 1 : dim);
      roff += plan.recv_rows[size_t(j)][size_t(p)];
    }
    if (profile_) PKD_HIP_CHECK(hipEventRecord(ev(round_ev(j, kRxBegin)), comm_stream_));
    comm_.group_begin();
    if (planar_)
      comm_.alltoallv_planes(send, size_t(send_stride) * 4, sb.data(), so.data(), recv[size_t(j)],
                             size_t(col_stride[size_t(j)]) * 4, rb.data(), ro.data(), dim, comm_stream_);
    else
      comm_.alltoallv(send, sb.data(), so.data(), recv[size_t(j)], rb.data(), ro.data(), comm_stream_);
    // id bitmaps: to every rank with a leaf in this round, from every rank if I have one
    for (int p = 0; p < P; ++p) {
      const int t = lay_.leaf_lo[size_t(p)] + j;
      const bool has = t < lay_.leaf_lo[size_t(p) + 1];
      sb[size_t(p)] = has ? size_t(send_words) * 4 : 0;
      so[size_t(p)] = has ? size_t(t) * send_words * 4 : 0;
      rb[size_t(p)] = j < mine ? size_t(src_words[size_t(p)]) * 4 : 0;
      ro[size_t(p)] = size_t(bm_off[size_t(p)]) * 4;
    }
    comm_.alltoallv(bm, sb.data(), so.data(), recv_bm[size_t(j)], rb.data(), ro.data(), comm_stream_);
    comm_.group_end();
    PKD_HIP_CHECK(hipEventRecord(arrived_[size_t(j)], comm_stream_));
    if (profile_) PKD_HIP_CHECK(hipEventRecord(ev(round_ev(j, kRxEnd)), comm_stream_));
  };
  issue(0);
  for (int j = 0; j < R; ++j) {
    if (j + 1 < R) issue(j + 1);  // in flight while leaf j builds
    if (j >= mine) continue;
    PKD_HIP_CHECK(hipStreamWaitEvent(s, arrived_[size_t(j)], 0));
    if (profile_) PKD_HIP_CHECK(hipEventRecord(ev(round_ev(j, kIdsBegin)), s));
    const int t = my_a + j;
    const i64 n_j = lay_.leaf_n[size_t(t)];
    if (n_j > 0) {
      BmSources src{};
      i64 off = 0;
      for (int p = 0; p < P; ++p) {
        src.off[p] = off;
        src.cnt[p] = plan.recv_rows[size_t(j)][size_t(p)];
        off += src.cnt[p];
        src.bm_off[p] = bm_off[size_t(p)];
        src.words[p] = src_words[size_t(p)];
        src.base[p] = u32(plan.src_base[size_t(p)]);
      }
      ids_from_bitmaps(recv_bm[size_t(j)], P, src, lids[size_t(j)], ids_scratch, err, s);
    }
    if (profile_) PKD_HIP_CHECK(hipEventRecord(ev(round_ev(j, kIdsEnd)), s));
    if (n_j > 0) {
      GpuBuilder& b = *lb[size_t(j)];
      const i64 a = lay_.leaf_slot[size_t(t)] - lay_.share_lo[size_t(me)];
      // the leaf's top-level cell bounds its points: no bounding-box pass over the received columns
      const float* leaf_cell = static_cast<const float*>(bufs_[1].first) + size_t(T - 1 + t) * dim * 2;
      if (planar_) b.build_columns(recv[size_t(j)], tree_pts_ + a * dim, tree_ids_ + a, leaf_ws_, s, leaf_cell);
      else b.build(recv[size_t(j)], lids[size_t(j)], 0, tree_pts_ + a * dim, tree_ids_ + a, leaf_ws_, s);
      or_error_word(b.error_word(leaf_ws_), err + 1, s);  // the leaves share one workspace
      PKD_HIP_CHECK(hipMemcpyAsync(leaf_err + j, b.error_word(leaf_ws_), 4, hipMemcpyDeviceToDevice, s));
    }
    if (profile_) PKD_HIP_CHECK(hipEventRecord(ev(round_ev(j, kLeafEnd)), s));
  }
  // the send buffers are rewritten by the next build: the caller's stream waits for the rounds
  PKD_HIP_CHECK(hipEventRecord(packed_, comm_stream_));
  PKD_HIP_CHECK(hipStreamWaitEvent(s, packed_, 0));
  // A sampled leaf whose band missed its median (error bit 0x20) is rebuilt locally without
  // sampling, from its received columns (intact: the sampled top reads them into the
  // workspace's own, and a leaf with sampled triples only builds on a copy). No collective is involved, so the ranks stay in step. One host wait per
  // build, after everything is enqueued, and only when some leaf sampled its top levels.
  bool any_top = false;
  for (int j = 0; j < mine; ++j) any_top = any_top || (lb[size_t(j)] && lb[size_t(j)]->sampled());
  if (any_top) {
    comm_.wait(s, "leaf band check");
    std::vector<u32> le(size_t(mine), 0u);
    PKD_HIP_CHECK(hipMemcpy(le.data(), leaf_err, size_t(mine) * 4, hipMemcpyDeviceToHost));
    bool redo = false;
    for (int j = 0; j < mine; ++j)
      if (lb[size_t(j)] && lb[size_t(j)]->sampled() && (le[size_t(j)] & top4_band_miss_bit())) redo = true;
    if (redo) {
      PKD_HIP_CHECK(hipMemsetAsync(err + 1, 0, 4, s));
      for (int j = 0; j < mine; ++j) {
        GpuBuilder* b = lb[size_t(j)];
        if (!b) continue;
        if (b->sampled() && (le[size_t(j)] & top4_band_miss_bit())) {
          const int t = my_a + j;
          GpuBuilder& fb = leaf_builder(lay_.leaf_n[size_t(t)], LL, false);
          ensure_leaf_workspace(fb.workspace_bytes());
          const i64 a = lay_.leaf_slot[size_t(t)] - lay_.share_lo[size_t(me)];
          const float* leaf_cell = static_cast<const float*>(bufs_[1].first) + size_t(T - 1 + t) * dim * 2;
          fb.build_columns(recv[size_t(j)], tree_pts_ + a * dim, tree_ids_ + a, leaf_ws_, s, leaf_cell);
          PKD_HIP_CHECK(hipMemcpyAsync(leaf_err + j, fb.error_word(leaf_ws_), 4, hipMemcpyDeviceToDevice, s));
        }
        or_error_word(leaf_err + j, err + 1, s);
      }
    }
  }
  if (profile_) {
    PKD_HIP_CHECK(hipEventRecord(ev(kEvEnd), s));
    last_ = info;
  }
}

// ---------------------------------------------------------------------------------------------
// Loopback communicator: ranks are threads; every collective stages through the host.
namespace {

class ThreadComm final : public Comm {
 public:
  ThreadComm(std::shared_ptr<loopback::Hub> hub, int rank) : hub_(std::move(hub)), rank_(rank) {}
  int rank() const override { return rank_; }
  int size() const override { return hub_->size(); }

  void allreduce_sum_u32(u32* buf, size_t count, hipStream_t s) override {
    reduce<u32>(buf, count, s, [](u32 a, u32 b) { return a + b; });
  }
  void allreduce_min_i64(i64* buf, size_t count, hipStream_t s) override {
    reduce<i64>(buf, count, s, [](i64 a, i64 b) { return std::min(a, b); });
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    const std::vector<char> mine = to_host(send, bytes, s);
    std::vector<char> out;
    hub_->allgather(rank_, mine.data(), bytes, &out);
    if (bytes) PKD_HIP_CHECK(hipMemcpy(recv, out.data(), out.size(), hipMemcpyHostToDevice));
  }
  void alltoallv(const void* send, const size_t* send_bytes, const size_t* send_off, void* recv,
                 const size_t* recv_bytes, const size_t* recv_off, hipStream_t s) override {
    size_t total = 0, rtotal = 0;
    for (int p = 0; p < size(); ++p) {
      total = std::max(total, send_off[p] + send_bytes[p]);
      rtotal = std::max(rtotal, recv_off[p] + recv_bytes[p]);
    }
    const std::vector<char> mine = to_host(send, total, s);
    std::vector<char> in(rtotal);
    hub_->alltoallv(rank_, mine.data(), send_bytes, send_off, in.data(), recv_bytes, recv_off);
    for (int p = 0; p < size(); ++p)  // only the received ranges: the rest of recv is not ours
      if (recv_bytes[p])
        PKD_HIP_CHECK(hipMemcpy(static_cast<char*>(recv) + recv_off[p], in.data() + recv_off[p], recv_bytes[p],
                                hipMemcpyHostToDevice));
  }

 private:
  template <class T, class F>
  void reduce(T* buf, size_t count, hipStream_t s, F f) {
    const std::vector<char> mine = to_host(buf, count * sizeof(T), s);
    std::vector<T> acc;
    hub_->reduce<T>(rank_, reinterpret_cast<const T*>(mine.data()), count, f, &acc);
    if (count) PKD_HIP_CHECK(hipMemcpy(buf, acc.data(), count * sizeof(T), hipMemcpyHostToDevice));
  }
  // the device bytes, after everything enqueued on s before this collective
  static std::vector<char> to_host(const void* dev, size_t bytes, hipStream_t s) {
    PKD_HIP_CHECK(hipStreamSynchronize(s));
    std::vector<char> v(bytes);
    if (bytes) PKD_HIP_CHECK(hipMemcpy(v.data(), dev, bytes, hipMemcpyDeviceToHost));
    return v;
  }
  std::shared_ptr<loopback::Hub> hub_;
  int rank_;
};

}  // namespace

std::vector<std::unique_ptr<Comm>> make_thread_comms(int size) {
  auto hub = std::make_shared<loopback::Hub>(size);
  std::vector<std::unique_ptr<Comm>> out;
  for (int r = 0; r < size; ++r) out.push_back(std::make_unique<ThreadComm>(hub, r));
  return out;
}

// ---------------------------------------------------------------------------------------------
// Rank emulation: record one rank's collective outputs, replay them as device copies.
namespace {

struct Recorded {  // one collective's output: byte chunks at offsets of the destination buffer
  std::vector<std::pair<size_t, std::vector<char>>> chunks;
};

class RecordingComm final : public Comm {
 public:
  RecordingComm(Comm& inner, std::vector<Recorded>* out) : in_(inner), out_(out) { set_timeout(inner.timeout()); }
  int rank() const override { return in_.rank(); }
  int size() const override { return in_.size(); }
  void allreduce_sum_u32(u32* buf, size_t count, hipStream_t s) override {
    in_.allreduce_sum_u32(buf, count, s);
    record1(buf, count * 4, s);
  }
  void allreduce_min_i64(i64* buf, size_t count, hipStream_t s) override {
    in_.allreduce_min_i64(buf, count, s);
    record1(buf, count * 8, s);
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    in_.allgather(send, recv, bytes, s);
    record1(recv, bytes * size_t(size()), s);
  }
  void alltoallv(const void* send, const size_t* send_bytes, const size_t* send_off, void* recv,
                 const size_t* recv_bytes, const size_t* recv_off, hipStream_t s) override {
    in_.alltoallv(send, send_bytes, send_off, recv, recv_bytes, recv_off, s);
    PKD_HIP_CHECK(hipStreamSynchronize(s));
    Recorded r;
    for (int p = 0; p < size(); ++p) {
      if (!recv_bytes[p]) continue;
      std::vector<char> v(recv_bytes[p]);
      PKD_HIP_CHECK(hipMemcpy(v.data(), static_cast<const char*>(recv) + recv_off[p], v.size(), hipMemcpyDeviceToHost));
      r.chunks.emplace_back(recv_off[p], std::move(v));
    }
    out_->push_back(std::move(r));
  }
  void group_begin() override { in_.group_begin(); }
  void group_end() override { in_.group_end(); }

 private:
  void record1(const void* dst, size_t bytes, hipStream_t s) {
    PKD_HIP_CHECK(hipStreamSynchronize(s));
    Recorded r;
    std::vector<char> v(bytes);
    if (bytes) PKD_HIP_CHECK(hipMemcpy(v.data(), dst, bytes, hipMemcpyDeviceToHost));
    r.chunks.emplace_back(0, std::move(v));
    out_->push_back(std::move(r));
  }
  Comm& in_;
  std::vector<Recorded>* out_;
};

class ReplayComm final : public Comm {
 public:
  ReplayComm(int rank, int size, const std::vector<Recorded>& recs) : rank_(rank), size_(size) {
    for (const Recorded& r : recs) {
      std::vector<Chunk> cs;
      for (const auto& c : r.chunks) {
        Chunk d{c.first, c.second.size(), nullptr};
        if (d.bytes) {
          PKD_HIP_CHECK(hipMalloc(&d.dev, d.bytes));
          PKD_HIP_CHECK(hipMemcpy(d.dev, c.second.data(), d.bytes, hipMemcpyHostToDevice));
        }
        cs.push_back(d);
      }
      calls_.push_back(std::move(cs));
    }
  }
  ~ReplayComm() override {
    for (auto& cs : calls_)
      for (auto& c : cs)
        if (c.dev) (void)hipFree(c.dev);
  }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  void rewind() { next_ = 0; }
  int calls() const { return int(calls_.size()); }
  void allreduce_sum_u32(u32* buf, size_t count, hipStream_t s) override { replay1(buf, count * 4, s); }
  void allreduce_min_i64(i64* buf, size_t count, hipStream_t s) override { replay1(buf, count * 8, s); }
  void allgather(const void*, void* recv, size_t bytes, hipStream_t s) override {
    replay1(recv, bytes * size_t(size_), s);
  }
  void alltoallv(const void*, const size_t*, const size_t*, void* recv, const size_t* recv_bytes,
                 const size_t* recv_off, hipStream_t s) override {
    const auto& cs = take();
    size_t k = 0;
    for (int p = 0; p < size_; ++p) {
      if (!recv_bytes[p]) continue;
      if (k >= cs.size() || cs[k].off != recv_off[p] || cs[k].bytes != recv_bytes[p])
        throw std::runtime_error("replay communicator: all-to-all layout differs from the recording");
      PKD_HIP_CHECK(hipMemcpyAsync(static_cast<char*>(recv) + recv_off[p], cs[k].dev, cs[k].bytes,
                                   hipMemcpyDeviceToDevice, s));
      ++k;
    }
  }

 private:
  struct Chunk {
    size_t off, bytes;
    void* dev;
  };
  const std::vector<Chunk>& take() {
    if (next_ >= calls_.size()) throw std::runtime_error("replay communicator: more collectives than recorded");
    return calls_[next_++];
  }
  void replay1(void* dst, size_t bytes, hipStream_t s) {
    const auto& cs = take();
    if (cs.size() != 1 || cs[0].bytes != bytes)
      throw std::runtime_error("replay communicator: collective size differs from the recording");
    if (bytes) PKD_HIP_CHECK(hipMemcpyAsync(dst, cs[0].dev, bytes, hipMemcpyDeviceToDevice, s));
  }
  int rank_, size_;
  std::vector<std::vector<Chunk>> calls_;
  size_t next_ = 0;
};

}  // namespace

RankEmulation emulate_rank(const float* x_host, i64 N, int dim, int P, int rank, int pipeline_k, int reps) {
  if (rank < 0 || rank >= P) throw std::invalid_argument("emulate_rank: rank out of range");
  int dev = 0;
  PKD_HIP_CHECK(hipGetDevice(&dev));
  auto slice = [&](int r, i64* first, i64* local) {
    const i64 base = N / P;
    *first = base * r;
    *local = base + (r == P - 1 ? N % P : 0);
  };
  std::vector<Recorded> recs;
  std::vector<float> ref_pts;
  std::vector<u32> ref_ids;
  {  // 1. the P ranks as threads; rank `rank` records its collective outputs
    auto comms = make_thread_comms(P);
    RecordingComm recorder(*comms[size_t(rank)], &recs);
    std::vector<std::exception_ptr> errs(static_cast<size_t>(P));
    std::vector<std::thread> th;
    for (int r = 0; r < P; ++r)
      th.emplace_back([&, r] {
        float* d = nullptr;
        hipStream_t s = nullptr;
        try {
          PKD_HIP_CHECK(hipSetDevice(dev));
          i64 first = 0, local = 0;
          slice(r, &first, &local);
          PKD_HIP_CHECK(hipStreamCreate(&s));
          PKD_HIP_CHECK(hipMalloc(&d, size_t(std::max<i64>(local, 1)) * dim * 4));
          PKD_HIP_CHECK(hipMemcpy(d, x_host + first * dim, size_t(local) * dim * 4, hipMemcpyHostToDevice));
          Comm& c = r == rank ? static_cast<Comm&>(recorder) : *comms[size_t(r)];
          GlobalBuilder gb(c, N, dim, pipeline_k);
          gb.build(d, local, u32(first + 1), s);
          gb.wait(s);
          if (r == rank) {
            ref_pts.resize(size_t(gb.n_leaf()) * dim);
            ref_ids.resize(size_t(gb.n_leaf()));
            if (gb.n_leaf() > 0) {
              PKD_HIP_CHECK(hipMemcpy(ref_pts.data(), gb.tree_pts(), ref_pts.size() * 4, hipMemcpyDeviceToHost));
              PKD_HIP_CHECK(hipMemcpy(ref_ids.data(), gb.tree_ids(), ref_ids.size() * 4, hipMemcpyDeviceToHost));
            }
          }
        } catch (...) {
          errs[size_t(r)] = std::current_exception();
        }
        if (d) (void)hipFree(d);
        if (s) (void)hipStreamDestroy(s);
      });
    for (auto& t : th) t.join();
    for (auto& e : errs)
      if (e) std::rethrow_exception(e);
  }
  // 2. rank `rank` alone against the recording, profiled
  RankEmulation out;
  out.collectives = int(recs.size());
  ReplayComm replay(rank, P, recs);
  recs.clear();
  i64 first = 0, local = 0;
  slice(rank, &first, &local);
  float* d = nullptr;
  hipStream_t s = nullptr;
  PKD_HIP_CHECK(hipStreamCreate(&s));
  PKD_HIP_CHECK(hipMalloc(&d, size_t(std::max<i64>(local, 1)) * dim * 4));
  PKD_HIP_CHECK(hipMemcpy(d, x_host + first * dim, size_t(local) * dim * 4, hipMemcpyHostToDevice));
  {
    GlobalBuilder gb(replay, N, dim, pipeline_k);
    gb.set_profile(true);
    for (int i = 0; i < std::max(1, reps) + 1; ++i) {  // the first build warms up (allocations)
      replay.rewind();
      gb.build(d, local, u32(first + 1), s);
      gb.wait(s);
      if (i > 0) out.total_ms.push_back(gb.phases(s).total_ms);
    }
    out.phases = gb.phases(s);
    out.error = gb.read_error(s);
    std::vector<float> tp(size_t(gb.n_leaf()) * dim);
    std::vector<u32> ti(size_t(gb.n_leaf()));
    if (gb.n_leaf() > 0) {
      PKD_HIP_CHECK(hipMemcpy(tp.data(), gb.tree_pts(), tp.size() * 4, hipMemcpyDeviceToHost));
      PKD_HIP_CHECK(hipMemcpy(ti.data(), gb.tree_ids(), ti.size() * 4, hipMemcpyDeviceToHost));
    }
    out.same_tree = tp == ref_pts && ti == ref_ids;
  }
  (void)hipFree(d);
  (void)hipStreamDestroy(s);
  return out;
}

}  // namespace pkdtree
