// Bindings of the distributed-decomposition device ops (csrc/gpu/dist_ops.hip).
#include <torch/extension.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include <algorithm>
#include <optional>
#include <vector>

#include "pkdtree/dist_ops.hpp"
#include "pkdtree/global_builder.hpp"
#include "pkdtree/hip_check.hpp"
#include "pkdtree/rccl_comm.hpp"

#include <cstring>
#include <exception>
#include <thread>
#include <tuple>

namespace pkdtree {

namespace {

hipStream_t stream_of(const torch::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check_cuda(const torch::Tensor& t, torch::ScalarType st, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == st && t.is_contiguous(), what, ": contiguous cuda tensor of ",
              c10::toString(st), " expected");
}

TopPoints points_of(const torch::Tensor& pts, const std::optional<torch::Tensor>& ids, int64_t id_base) {
  check_cuda(pts, torch::kFloat32, "points");
  TORCH_CHECK(pts.dim() == 2, "points must be [n, dim]");
  TopPoints p;
  p.pts = pts.data_ptr<float>();
  p.n = pts.size(0);
  p.dim = int(pts.size(1));
  p.id_base = u32(id_base);
  p.ids = nullptr;
  if (ids && ids->defined()) {
    check_cuda(*ids, torch::kInt32, "ids");
    TORCH_CHECK(ids->numel() == p.n, "ids must have one entry per point");
    p.ids = reinterpret_cast<const u32*>(ids->data_ptr<int32_t>());
  }
  return p;
}

TopSizes sizes_of(const std::vector<int64_t>& v) {
  TORCH_CHECK(v.size() <= size_t(kTopMaxNodes), "too many nodes per top level");
  TopSizes s{};
  for (size_t i = 0; i < v.size(); ++i) s.n[i] = v[i];
  return s;
}

u32* u32p(torch::Tensor& t) { return reinterpret_cast<u32*>(t.data_ptr<int32_t>()); }
const u32* cu32p(const torch::Tensor& t) { return reinterpret_cast<const u32*>(t.data_ptr<int32_t>()); }
u64* u64p(torch::Tensor& t) { return reinterpret_cast<u64*>(t.data_ptr<int64_t>()); }
const u64* cu64p(const torch::Tensor& t) { return reinterpret_cast<const u64*>(t.data_ptr<int64_t>()); }

void bbox(const torch::Tensor& pts, torch::Tensor box) {
  const c10::DeviceGuard g(pts.device());
  check_cuda(box, torch::kInt64, "box");
  TopPoints p = points_of(pts, std::nullopt, 0);
  TORCH_CHECK(box.numel() == 2 * p.dim, "box must have 2*dim entries");
  top_bbox(p, box.data_ptr<int64_t>(), stream_of(pts));
}

void root_cell(const torch::Tensor& box, int64_t dim, torch::Tensor cells) {
  const c10::DeviceGuard g(box.device());
  check_cuda(cells, torch::kFloat32, "cells");
  top_root_cell(box.data_ptr<int64_t>(), int(dim), cells.data_ptr<float>(), stream_of(box));
}

void route_hist(const torch::Tensor& pts, const std::optional<torch::Tensor>& ids, int64_t id_base,
                torch::Tensor node, int64_t level, const torch::Tensor& pivots, int64_t prev_axis, int64_t axis,
                const torch::Tensor& cells, int64_t bins, torch::Tensor hist) {
  const c10::DeviceGuard g(pts.device());
  TopPoints p = points_of(pts, ids, id_base);
  TORCH_CHECK(node.numel() >= p.n, "node array too small");
  TORCH_CHECK(hist.numel() >= (int64_t(1) << level) * bins, "hist too small");
  top_route_hist(p, u32p(node), int(level), cu64p(pivots), int(prev_axis), int(axis), cells.data_ptr<float>(),
                 int(bins), u32p(hist), stream_of(pts));
}

void select(const torch::Tensor& hist, int64_t level, int64_t bins, const std::vector<int64_t>& sizes,
            torch::Tensor sel, torch::Tensor err, std::optional<torch::Tensor> zero_hist,
            std::optional<torch::Tensor> zero_hdr) {
  const c10::DeviceGuard g(hist.device());
  TORCH_CHECK(int64_t(sizes.size()) == (int64_t(1) << level), "one size per node");
  u32* zh = nullptr;
  if (zero_hist && zero_hist->defined()) {
    TORCH_CHECK(zero_hist->numel() >= kTopBins, "zero_hist must hold kTopBins words");
    zh = u32p(*zero_hist);
  }
  u32* zd = zero_hdr && zero_hdr->defined() ? reinterpret_cast<u32*>(zero_hdr->data_ptr()) : nullptr;
  top_select(cu32p(hist), int(level), int(bins), sizes_of(sizes), u32p(sel), u32p(err), zh, zd, stream_of(hist));
}

void collect_route(const torch::Tensor& pts, const std::optional<torch::Tensor>& ids, int64_t id_base,
                   torch::Tensor node, int64_t level, int64_t axis, int64_t next_axis, const torch::Tensor& cells,
                   int64_t bins, int64_t next_bins, const torch::Tensor& sel, torch::Tensor buf, int64_t cap,
                   std::optional<torch::Tensor> hist_next) {
  const c10::DeviceGuard g(pts.device());
  TopPoints p = points_of(pts, ids, id_base);
  TORCH_CHECK(size_t(buf.numel()) >= top_middle_words(p.dim, cap), "middle buffer too small");
  TORCH_CHECK(node.numel() >= p.n, "node array too small");
  u32* hn = hist_next && hist_next->defined() ? u32p(*hist_next) : nullptr;
  top_collect_route(p, u32p(node), int(level), int(axis), int(next_axis), cells.data_ptr<float>(), int(bins),
                    int(next_bins), cu32p(sel), buf.data_ptr<float>(), cap, hn, stream_of(pts));
}

void fixup(const torch::Tensor& buf, int64_t cap, int64_t dim, int64_t level, int64_t axis, int64_t next_axis,
           const torch::Tensor& pivots, const torch::Tensor& cells, int64_t next_bins, torch::Tensor node,
           std::optional<torch::Tensor> hist_next) {
  const c10::DeviceGuard g(buf.device());
  u32* hn = hist_next && hist_next->defined() ? u32p(*hist_next) : nullptr;
  top_fixup(buf.data_ptr<float>(), cap, int(dim), int(level), int(axis), int(next_axis), cu64p(pivots),
            cells.data_ptr<float>(), int(next_bins), u32p(node), hn, stream_of(buf));
}

void pivot(const torch::Tensor& gathered, int64_t P, int64_t cap, int64_t level, int64_t axis, int64_t dim,
           const std::vector<int64_t>& sizes, const torch::Tensor& sel, torch::Tensor pivots, torch::Tensor top_rows,
           torch::Tensor cells, torch::Tensor err) {
  const c10::DeviceGuard g(gathered.device());
  TORCH_CHECK(size_t(gathered.numel()) >= size_t(P) * top_middle_words(int(dim), cap), "gathered buffer too small");
  TORCH_CHECK(int64_t(sizes.size()) == (int64_t(1) << level), "one size per node");
  top_pivot(gathered.data_ptr<float>(), int(P), cap, int(level), int(axis), int(dim), sizes_of(sizes), cu32p(sel),
            u64p(pivots), top_rows.data_ptr<float>(), cells.data_ptr<float>(), u32p(err), stream_of(gathered));
}

// out: [>= n, dim + 1] / [>= n, dim] rows, or (col_stride > 0) planes of col_stride floats.
// node: as the top levels left it (leaf heap nodes, kTopDone for pivots).
void pack(const torch::Tensor& pts, const std::optional<torch::Tensor>& ids, int64_t id_base,
          const torch::Tensor& node, int64_t levels, torch::Tensor out, int64_t col_stride,
          std::optional<torch::Tensor> bitmaps, torch::Tensor counts, const torch::Tensor& err, torch::Tensor scratch) {
  const c10::DeviceGuard g(pts.device());
  TopPoints p = points_of(pts, ids, id_base);
  check_cuda(out, torch::kFloat32, "out");
  const int64_t T = int64_t(1) << levels;
  int row_stride = p.dim;
  if (col_stride > 0) {
    TORCH_CHECK(out.numel() >= col_stride * p.dim && col_stride >= p.n, "out must hold dim planes of col_stride >= n");
  } else {
    TORCH_CHECK(out.dim() == 2 && out.size(0) >= p.n && (out.size(1) == p.dim + 1 || out.size(1) == p.dim),
                "out must be [>= n, dim+1] or [>= n, dim]");
    row_stride = int(out.size(1));
  }
  check_cuda(counts, torch::kInt64, "counts");
  TORCH_CHECK(counts.numel() == 4 * T, "counts must have 4 * 2^levels entries");
  TORCH_CHECK(size_t(scratch.numel()) >= top_pack_scratch_bytes(p.n, int(T)), "scratch too small");
  u32* bm = nullptr;
  int64_t words = 0;
  if (bitmaps && bitmaps->defined()) {
    check_cuda(*bitmaps, torch::kInt32, "bitmaps");
    TORCH_CHECK(bitmaps->dim() == 2 && bitmaps->size(0) == T && bitmaps->size(1) * 32 >= p.n,
                "bitmaps must be [2^levels, >= n/32]");
    bm = u32p(*bitmaps);
    words = bitmaps->size(1);
  }
  top_pack(p, cu32p(node), int(levels), out.data_ptr<float>(), row_stride, col_stride, bm, words,
           counts.data_ptr<int64_t>(), cu32p(err), scratch.data_ptr(), stream_of(pts));
}

// bitmaps: all sources' words back to back; per source (row offset, rows, word offset, words, id base)
void ids_from_bm(const torch::Tensor& bitmaps, const std::vector<int64_t>& off, const std::vector<int64_t>& cnt,
                 const std::vector<int64_t>& bm_off, const std::vector<int64_t>& words,
                 const std::vector<int64_t>& base, torch::Tensor ids, torch::Tensor scratch, torch::Tensor err) {
  const c10::DeviceGuard g(bitmaps.device());
  check_cuda(bitmaps, torch::kInt32, "bitmaps");
  check_cuda(ids, torch::kInt32, "ids");
  const size_t P = off.size();
  TORCH_CHECK(P >= 1 && P <= size_t(kBmMaxSources) && cnt.size() == P && bm_off.size() == P && words.size() == P &&
                  base.size() == P,
              "one row offset / count / bitmap offset / word count / id base per source");
  BmSources src{};
  int64_t max_words = 0;
  for (size_t s = 0; s < P; ++s) {
    src.off[s] = off[s];
    src.cnt[s] = cnt[s];
    src.bm_off[s] = bm_off[s];
    src.words[s] = words[s];
    src.base[s] = u32(base[s]);
    TORCH_CHECK(off[s] >= 0 && off[s] + cnt[s] <= ids.numel(), "ids too small");
    TORCH_CHECK(bm_off[s] >= 0 && bm_off[s] + words[s] <= bitmaps.numel(), "bitmap buffer too small");
    max_words = std::max(max_words, words[s]);
  }
  TORCH_CHECK(size_t(scratch.numel()) >= ids_from_bitmaps_scratch_bytes(max_words, int(P)), "scratch too small");
  ids_from_bitmaps(cu32p(bitmaps), int(P), src, u32p(ids), scratch.data_ptr(), u32p(err), stream_of(bitmaps));
}

// ---- geometry and planning (host, CPU-testable) --------------------------------------------
pybind11::dict layout_dict(const global_plan::Layout& lay) {
  pybind11::dict d;
  d["P"] = lay.P;
  d["LL"] = lay.LL;
  d["T"] = lay.T;
  d["R"] = lay.R;
  d["leaf_lo"] = lay.leaf_lo;
  d["leaf_slot"] = std::vector<int64_t>(lay.leaf_slot.begin(), lay.leaf_slot.end());
  d["leaf_n"] = std::vector<int64_t>(lay.leaf_n.begin(), lay.leaf_n.end());
  d["top_slot"] = std::vector<int64_t>(lay.top_slot.begin(), lay.top_slot.end());
  d["top_owner"] = lay.top_owner;
  d["share_lo"] = std::vector<int64_t>(lay.share_lo.begin(), lay.share_lo.end());
  d["share_n"] = std::vector<int64_t>(lay.share_n.begin(), lay.share_n.end());
  pybind11::list blocks, between;
  for (int r = 0; r < lay.P; ++r) {
    std::vector<global_plan::Block> b;
    std::vector<i64> bw;
    global_plan::share_blocks(lay, r, &b, &bw);
    pybind11::list bl;
    for (const auto& x : b) bl.append(pybind11::make_tuple(int64_t(x.off), int64_t(x.n), x.depth, int64_t(x.heap)));
    blocks.append(bl);
    between.append(std::vector<int64_t>(bw.begin(), bw.end()));
  }
  d["blocks"] = blocks;    // per rank: (offset in share, points, root depth, heap node)
  d["between"] = between;  // per rank: heap nodes of the top rows between its blocks
  return d;
}

pybind11::dict layout_py(int64_t n_total, int64_t P, int64_t k) {
  return layout_dict(global_plan::make_layout(n_total, int(P), int(k)));
}

// The native exchange planner: counts [P][T][4] (rows, err, id base, n_local) flattened.
std::tuple<int, std::vector<std::vector<int64_t>>, std::vector<std::vector<int64_t>>,
           std::vector<std::vector<int64_t>>, std::vector<int64_t>>
plan_py(const std::vector<int64_t>& counts, int64_t n_total, int64_t P, int64_t k, int64_t me) {
  const auto lay = global_plan::make_layout(n_total, int(P), int(k));
  std::vector<i64> c(counts.begin(), counts.end());
  global_plan::Plan plan;
  const int rc = global_plan::make_plan(c, lay, int(me), &plan);
  auto cv = [](const std::vector<std::vector<i64>>& v) {
    std::vector<std::vector<int64_t>> o;
    for (const auto& r : v) o.emplace_back(r.begin(), r.end());
    return o;
  };
  return {rc, cv(plan.send_rows), cv(plan.send_off), cv(plan.recv_rows),
          std::vector<int64_t>(plan.leaf_start.begin(), plan.leaf_start.end())};
}

// The native global builder with P ranks as threads of this process sharing the current GPU
// (loopback communicator): rank r holds rows [first_r, first_r + local_r) of `x` (the reference's
// MPI slicing), ids 1..N. Returns the assembled in-order tree (rank shares + boundary top rows)
// on the host, the OR of the ranks' error words and the middle-bucket scale they ended at.
// builds > 1: the same GlobalBuilder builds the input that many times (its leaf builders and their
// shared workspace reused: a leaf whose sampled bands missed in one build is built again by the
// same sampled builder in the next); the error words of all builds are OR-ed, the last tree returned.
std::tuple<torch::Tensor, torch::Tensor, int64_t, int64_t, bool> global_loopback(const torch::Tensor& x, int64_t P,
                                                                                 int64_t k, int64_t builds) {
  TORCH_CHECK(!x.is_cuda() && x.scalar_type() == torch::kFloat32 && x.is_contiguous() && x.dim() == 2,
              "x: contiguous float32 [N, dim] host tensor");
  const int64_t N = x.size(0);
  const int dim = int(x.size(1));
  int dev = 0;
  PKD_HIP_CHECK(hipGetDevice(&dev));
  torch::Tensor tp = torch::zeros({N, dim}, torch::kFloat32);
  torch::Tensor ti = torch::zeros({N}, torch::kInt32);
  auto comms = make_thread_comms(int(P));
  std::vector<std::exception_ptr> errs(static_cast<size_t>(P));
  std::vector<u32> ew(static_cast<size_t>(P), 0u);
  std::vector<int> scales(static_cast<size_t>(P), 0);
  std::vector<char> radix(static_cast<size_t>(P), 0);
  std::vector<std::thread> th;
  for (int r = 0; r < int(P); ++r)
    th.emplace_back([&, r] {
      float* d = nullptr;
      hipStream_t s = nullptr;
      try {
        PKD_HIP_CHECK(hipSetDevice(dev));
        const int64_t base = N / P, first = base * r, local = base + (r == P - 1 ? N % P : 0);
        PKD_HIP_CHECK(hipStreamCreate(&s));
        PKD_HIP_CHECK(hipMalloc(&d, size_t(std::max<int64_t>(local, 1)) * dim * 4));
        PKD_HIP_CHECK(hipMemcpy(d, x.data_ptr<float>() + first * dim, size_t(local) * dim * 4, hipMemcpyHostToDevice));
        GlobalBuilder gb(*comms[size_t(r)], N, dim, int(k));
        for (int64_t it = 0; it < std::max<int64_t>(builds, 1); ++it) {
          gb.build(d, local, u32(first + 1), s);
          gb.wait(s);
          ew[size_t(r)] |= gb.read_error(s);
        }
        scales[size_t(r)] = gb.middle_scale();
        radix[size_t(r)] = gb.radix_mode() ? 1 : 0;
        PKD_HIP_CHECK(hipMemcpy(tp.data_ptr<float>() + gb.slot_lo() * dim, gb.tree_pts(), size_t(gb.n_leaf()) * dim * 4,
                                hipMemcpyDeviceToHost));
        PKD_HIP_CHECK(hipMemcpy(ti.data_ptr<int32_t>() + gb.slot_lo(), gb.tree_ids(), size_t(gb.n_leaf()) * 4,
                                hipMemcpyDeviceToHost));
        if (r == 0) {
          const auto slots = gb.top_slots();
          std::vector<float> rows(slots.size() * size_t(dim + 1));
          if (!rows.empty())
            PKD_HIP_CHECK(hipMemcpy(rows.data(), gb.top_rows(), rows.size() * 4, hipMemcpyDeviceToHost));
          for (size_t h = 0; h < slots.size(); ++h)
            if (slots[h] >= 0) {
              std::memcpy(tp.data_ptr<float>() + slots[h] * dim, &rows[h * size_t(dim + 1)], size_t(dim) * 4);
              std::memcpy(ti.data_ptr<int32_t>() + slots[h], &rows[h * size_t(dim + 1) + dim], 4);
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
  u32 e = 0;
  for (u32 v : ew) e |= v;
  return {tp, ti, int64_t(e), int64_t(*std::max_element(scales.begin(), scales.end())),
          *std::max_element(radix.begin(), radix.end()) != 0};
}

// The native global builder on its own RCCL communicator, one per process (rank). The
// communicator's unique id comes from rank 0 (rccl_unique_id) and reaches the other ranks
// through the Python process group; then no Python runs between the collectives of a build.
class NativeGlobal {
 public:
  NativeGlobal(int64_t n_total, int64_t dim, int64_t rank, int64_t world, const std::string& uid,
               int64_t pipeline_k, int64_t device, double timeout_s)
      : dim_(int(dim)), rank_(int(rank)), world_(int(world)), device_(int(device)) {
    TORCH_CHECK(uid.size() == sizeof(ncclUniqueId), "rccl unique id: ", sizeof(ncclUniqueId), " bytes expected");
    TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "rank out of range");
    PKD_HIP_CHECK(hipSetDevice(device_));
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    nccl_check(ncclCommInitRank(&c_, world_, id, rank_), "ncclCommInitRank", rank_);
    comm_ = std::make_unique<RcclComm>(c_, rank_, world_);
    if (timeout_s > 0) comm_->set_timeout(timeout_s);
    gb_ = std::make_unique<GlobalBuilder>(*comm_, n_total, dim_, int(pipeline_k));
  }
  ~NativeGlobal() {
    gb_.reset();
    const bool dead = comm_ && comm_->aborted();
    comm_.reset();
    if (c_ && !dead) (void)ncclCommDestroy(c_);
  }
  NativeGlobal(const NativeGlobal&) = delete;
  NativeGlobal& operator=(const NativeGlobal&) = delete;

  void build(const torch::Tensor& x, int64_t id_base) {
    check_cuda(x, torch::kFloat32, "points");
    TORCH_CHECK(x.dim() == 2 && x.size(1) == dim_, "points must be [n, dim]");
    TORCH_CHECK(x.device().index() == device_, "points must live on the builder's device");
    const c10::DeviceGuard g(x.device());
    const hipStream_t s = stream_of(x);
    const float* p = x.data_ptr<float>();
    const int64_t n = x.size(0);
    pybind11::gil_scoped_release nogil;  // the exchange plan blocks on the other ranks
    gb_->build(p, n, u32(id_base), s);
  }
  // bounded wait for the last build on the current stream (raises on a stuck / failed peer)
  void sync() {
    const c10::DeviceGuard g(torch::Device(torch::kCUDA, device_));
    const hipStream_t s = c10::hip::getCurrentHIPStream(device_).stream();
    pybind11::gil_scoped_release nogil;
    gb_->wait(s);
  }
  // views of the builder's buffers (valid until the next build / the builder's end)
  torch::Tensor tree_pts() const {
    return torch::from_blob(const_cast<float*>(gb_->tree_pts()), {gb_->n_leaf(), dim_}, opts(torch::kFloat32));
  }
  torch::Tensor tree_ids() const {
    return torch::from_blob(const_cast<u32*>(gb_->tree_ids()), {gb_->n_leaf()}, opts(torch::kInt32));
  }
  torch::Tensor top_rows() const {
    const int64_t t = std::max(gb_->layout().T - 1, 0);
    if (t == 0) return torch::empty({0, dim_ + 1}, opts(torch::kFloat32));
    return torch::from_blob(const_cast<float*>(gb_->top_rows()), {t, dim_ + 1}, opts(torch::kFloat32));
  }
  std::vector<int64_t> top_slots() const {
    const auto v = gb_->top_slots();
    return std::vector<int64_t>(v.begin(), v.end());
  }
  pybind11::dict layout() const { return layout_dict(gb_->layout()); }
  int64_t slot_lo() const { return gb_->slot_lo(); }
  int64_t n_leaf() const { return gb_->n_leaf(); }
  int64_t top_levels() const { return gb_->top_levels(); }
  int64_t middle_scale() const { return gb_->middle_scale(); }
  int64_t read_error() const {
    const c10::DeviceGuard g(torch::Device(torch::kCUDA, device_));
    return int64_t(gb_->read_error(c10::hip::getCurrentHIPStream(device_).stream()));
  }
  void set_profile(bool on) { gb_->set_profile(on); }
  // routed exact 1-NN over the whole tree (collective: every rank calls it with the same queries)
  std::tuple<torch::Tensor, int64_t> query(const torch::Tensor& q, bool count_work) {
    check_cuda(q, torch::kFloat32, "queries");
    TORCH_CHECK(q.dim() == 2 && q.size(1) == dim_ && q.is_contiguous(), "queries must be contiguous [Q, dim]");
    TORCH_CHECK(q.device().index() == device_, "queries must live on the builder's device");
    const c10::DeviceGuard g(q.device());
    torch::Tensor out = torch::empty({q.size(0)}, opts(torch::kInt64));
    const hipStream_t s = stream_of(q);
    const float* qp = q.data_ptr<float>();
    u64* op = reinterpret_cast<u64*>(out.data_ptr<int64_t>());
    const int64_t Q = q.size(0);
    int64_t work = 0;
    {
      pybind11::gil_scoped_release nogil;
      work = gb_->query(qp, Q, op, s, count_work);
    }
    return {out, work};
  }
  std::map<std::string, double> phases() const {
    const c10::DeviceGuard g(torch::Device(torch::kCUDA, device_));
    return gb_->phases(c10::hip::getCurrentHIPStream(device_).stream()).as_map();
  }

 private:
  torch::TensorOptions opts(torch::ScalarType t) const {
    return torch::TensorOptions().dtype(t).device(torch::kCUDA, device_);
  }
  int dim_, rank_, world_, device_;
  ncclComm_t c_ = nullptr;
  std::unique_ptr<RcclComm> comm_;
  std::unique_ptr<GlobalBuilder> gb_;
};

pybind11::bytes rccl_unique_id() {
  ncclUniqueId id;
  nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId", 0);
  return pybind11::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
}

}  // namespace

void bind_dist_ops(pybind11::module& m) {
  m.def("rccl_unique_id", &rccl_unique_id);
  pybind11::class_<NativeGlobal>(m, "NativeGlobal")
      .def(pybind11::init<int64_t, int64_t, int64_t, int64_t, const std::string&, int64_t, int64_t, double>(),
           pybind11::arg("n_total"), pybind11::arg("dim"), pybind11::arg("rank"), pybind11::arg("world"),
           pybind11::arg("uid"), pybind11::arg("pipeline_k") = -1, pybind11::arg("device") = 0,
           pybind11::arg("timeout_s") = 0.0, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("build", &NativeGlobal::build, pybind11::arg("x"), pybind11::arg("id_base"))
      .def("sync", &NativeGlobal::sync)
      .def("tree_pts", &NativeGlobal::tree_pts)
      .def("tree_ids", &NativeGlobal::tree_ids)
      .def("top_rows", &NativeGlobal::top_rows)
      .def("top_slots", &NativeGlobal::top_slots)
      .def("layout", &NativeGlobal::layout)
      .def("slot_lo", &NativeGlobal::slot_lo)
      .def("n_leaf", &NativeGlobal::n_leaf)
      .def("top_levels", &NativeGlobal::top_levels)
      .def("middle_scale", &NativeGlobal::middle_scale)
      .def("read_error", &NativeGlobal::read_error)
      .def("set_profile", &NativeGlobal::set_profile)
      .def("query", &NativeGlobal::query, pybind11::arg("queries"), pybind11::arg("count_work") = false)
      .def("phases", &NativeGlobal::phases);
  m.def(
      "global_emulate_rank",
      [](const torch::Tensor& x, int64_t P, int64_t rank, int64_t k, int64_t reps) {
        TORCH_CHECK(!x.is_cuda() && x.scalar_type() == torch::kFloat32 && x.is_contiguous() && x.dim() == 2,
                    "x: contiguous float32 [N, dim] host tensor");
        pybind11::gil_scoped_release nogil;
        const RankEmulation e =
            emulate_rank(x.data_ptr<float>(), x.size(0), int(x.size(1)), int(P), int(rank), int(k), int(reps));
        pybind11::gil_scoped_acquire gil;
        pybind11::dict d;
        for (const auto& kv : e.phases.as_map()) d[pybind11::str(kv.first)] = kv.second;
        d["total_ms_reps"] = e.total_ms;
        d["same_tree"] = e.same_tree;
        d["error"] = int64_t(e.error);
        d["collectives"] = e.collectives;
        return d;
      },
      pybind11::arg("x"), pybind11::arg("P"), pybind11::arg("rank") = 0, pybind11::arg("k") = -1,
      pybind11::arg("reps") = 5);
  m.def("global_layout", &layout_py, pybind11::arg("n_total"), pybind11::arg("P"), pybind11::arg("k") = -1);
  m.def("global_plan", &plan_py, pybind11::arg("counts"), pybind11::arg("n_total"), pybind11::arg("P"),
        pybind11::arg("k"), pybind11::arg("me"));
  m.def("global_loopback", &global_loopback, pybind11::arg("x"), pybind11::arg("P"), pybind11::arg("k") = -1,
        pybind11::arg("builds") = 1,
        pybind11::call_guard<pybind11::gil_scoped_release>());
  m.def("top_bbox", &bbox);
  m.def("fill_u64_multi", [](const std::vector<std::tuple<torch::Tensor, int64_t, uint64_t>>& segs) {
    FillSegs f;
    hipStream_t s = nullptr;
    for (const auto& [t, words, value] : segs) {
      TORCH_CHECK(t.is_cuda() && t.element_size() * t.numel() >= words * 8, "fill_u64_multi: segment too small");
      s = stream_of(t);
      f.add(t.data_ptr(), words, value);
    }
    fill_u64_multi(f, s);
  });
  m.def("top_root_cell", &root_cell);
  m.def("top_route_hist", &route_hist);
  m.def("top_select", &select, pybind11::arg("hist"), pybind11::arg("level"), pybind11::arg("bins"),
        pybind11::arg("sizes"), pybind11::arg("sel"), pybind11::arg("err"), pybind11::arg("zero_hist") = std::nullopt,
        pybind11::arg("zero_hdr") = std::nullopt);
  m.def("top_collect_route", &collect_route);
  m.def("top_fixup", &fixup);
  m.def("top_pivot", &pivot);
  m.def("top_pack", &pack, pybind11::arg("pts"), pybind11::arg("ids"), pybind11::arg("id_base"), pybind11::arg("node"),
        pybind11::arg("levels"), pybind11::arg("out"), pybind11::arg("col_stride"), pybind11::arg("bitmaps"),
        pybind11::arg("counts"), pybind11::arg("err"), pybind11::arg("scratch"));
  m.def("top_middle_words", [](int64_t dim, int64_t cap) { return int64_t(top_middle_words(int(dim), cap)); });
  m.def("top_pack_scratch_bytes", [](int64_t n, int64_t T) { return int64_t(top_pack_scratch_bytes(n, int(T))); });
  m.def("ids_from_bitmaps", &ids_from_bm);
  m.def("ids_from_bitmaps_scratch_bytes",
        [](int64_t words, int64_t P) { return int64_t(ids_from_bitmaps_scratch_bytes(words, int(P))); });
}

}  // namespace pkdtree
