// PyTorch-ROCm binding of the native kd-tree core (module parallel_kd_tree_amd._C).
// Device work runs on the caller's current HIP stream; workspaces come from the torch
// caching allocator, so repeated builds allocate nothing from HIP.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include <algorithm>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "pkdtree/common.hpp"
#include "pkdtree/cpu_tree.hpp"
#include "pkdtree/generator.hpp"
#include "pkdtree/gpu_build.hpp"
#include "pkdtree/gpu_generator.hpp"
#include "pkdtree/gpu_query.hpp"
#include "pkdtree/gpu_reference.hpp"
#include "pkdtree/trace.hpp"

namespace pkdtree {
std::string subtree_stamp_report();
std::string tail_stamp_report();
}

namespace pk = pkdtree;
using pk::u32;

namespace pkdtree {
void bind_dist_ops(pybind11::module& m);  // dist_bindings.cpp
}

namespace {

hipStream_t cur_stream(const torch::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void check_points(const torch::Tensor& pts, bool cuda) {
  TORCH_CHECK(pts.dim() == 2, "points must be [n, dim]");
  TORCH_CHECK(pts.scalar_type() == torch::kFloat32, "points must be float32");
  TORCH_CHECK(pts.is_contiguous(), "points must be contiguous");
  TORCH_CHECK(pts.is_cuda() == cuda, cuda ? "points must be on a GPU" : "points must be on the CPU");
}

const pk::u32* opt_ids(const c10::optional<torch::Tensor>& ids, int64_t n, const torch::Device& dev) {
  if (!ids.has_value() || !ids->defined()) return nullptr;
  TORCH_CHECK(ids->scalar_type() == torch::kInt32, "ids must be int32 (bits are used as uint32)");
  TORCH_CHECK(ids->is_contiguous() && ids->numel() == n, "ids must be contiguous [n]");
  TORCH_CHECK(ids->device() == dev, "ids must be on the points' device (", dev, "), got ", ids->device());
  return reinterpret_cast<const pk::u32*>(ids->data_ptr<int32_t>());
}

// Reusable builder bound to (n, dim, options) with a torch-allocated workspace.
struct Builder {
  pk::GpuBuilder b;
  torch::Tensor ws;
  Builder(int64_t n, int64_t dim, int64_t depth0, int64_t subtree_max, bool allow_top)
      : b(n, int(dim), pk::BuildOptions{int(subtree_max), int(depth0), true, allow_top}) {}

  void ensure_ws(const torch::Device& dev) {
    if (!ws.defined() || ws.device() != dev)
      ws = torch::empty({int64_t(b.workspace_bytes())}, torch::TensorOptions().dtype(torch::kUInt8).device(dev));
  }

  std::vector<torch::Tensor> build(const torch::Tensor& pts, const c10::optional<torch::Tensor>& ids,
                                   int64_t id_base, c10::optional<torch::Tensor> out_pts,
                                   c10::optional<torch::Tensor> out_ids) {
    check_points(pts, true);
    TORCH_CHECK(pts.size(0) == b.n() && pts.size(1) == b.dim(), "points shape does not match the builder");
    const c10::DeviceGuard guard(pts.device());
    ensure_ws(pts.device());
    torch::Tensor op = out_pts.has_value() ? *out_pts : torch::empty_like(pts);
    torch::Tensor oi = out_ids.has_value() ? *out_ids
                                           : torch::empty({b.n()}, pts.options().dtype(torch::kInt32));
    TORCH_CHECK(op.sizes() == pts.sizes() && op.is_contiguous() && op.scalar_type() == torch::kFloat32,
                "out_pts must be a contiguous float32 tensor shaped like points");
    TORCH_CHECK(oi.numel() == b.n() && oi.scalar_type() == torch::kInt32 && oi.is_contiguous(),
                "out_ids must be contiguous int32 [n]");
    TORCH_CHECK(op.device() == pts.device() && oi.device() == pts.device(),
                "out_pts / out_ids must be on the points' device");
    b.build(pts.data_ptr<float>(), opt_ids(ids, b.n(), pts.device()), pk::u32(id_base), op.data_ptr<float>(),
            reinterpret_cast<pk::u32*>(oi.data_ptr<int32_t>()), ws.data_ptr(), cur_stream(pts));
    return {op, oi};
  }

  // Rows [n, dim+1] (coordinates, id bits): the all-to-all exchange format.
  std::vector<torch::Tensor> build_rows(const torch::Tensor& rows) {
    TORCH_CHECK(rows.is_cuda() && rows.scalar_type() == torch::kFloat32 && rows.is_contiguous(), "rows: cuda f32");
    TORCH_CHECK(rows.dim() == 2 && rows.size(0) == b.n() && rows.size(1) == b.dim() + 1, "rows must be [n, dim+1]");
    const c10::DeviceGuard guard(rows.device());
    ensure_ws(rows.device());
    torch::Tensor op = torch::empty({b.n(), b.dim()}, rows.options());
    torch::Tensor oi = torch::empty({b.n()}, rows.options().dtype(torch::kInt32));
    b.build_rows(rows.data_ptr<float>(), op.data_ptr<float>(), reinterpret_cast<pk::u32*>(oi.data_ptr<int32_t>()),
                 ws.data_ptr(), cur_stream(rows));
    return {op, oi};
  }

  // SoA input view inside the workspace: [(dim+1), n] float32 (row dim holds id bits).
  torch::Tensor soa_input(const torch::Device& dev) {
    ensure_ws(dev);
    return torch::from_blob(b.soa_input(ws.data_ptr()), {b.dim() + 1, b.n()}, {b.column_stride(), 1},
                            torch::TensorOptions().dtype(torch::kFloat32).device(dev));
  }

  // Columns [(dim+1), column_stride()] float32 (row dim holds id bits), 256-B aligned, NOT the
  // workspace's own SoA view: the distributed leaves' input format (GpuBuilder::build_columns).
  std::vector<torch::Tensor> build_columns(const torch::Tensor& cols) {
    TORCH_CHECK(cols.is_cuda() && cols.scalar_type() == torch::kFloat32 && cols.is_contiguous(), "cols: cuda f32");
    TORCH_CHECK(cols.dim() == 2 && cols.size(0) == b.dim() + 1 && cols.size(1) == b.column_stride(),
                "cols must be [dim+1, column_stride]");
    const c10::DeviceGuard guard(cols.device());
    ensure_ws(cols.device());
    torch::Tensor op = torch::empty({b.n(), b.dim()}, cols.options());
    torch::Tensor oi = torch::empty({b.n()}, cols.options().dtype(torch::kInt32));
    b.build_columns(cols.data_ptr<float>(), op.data_ptr<float>(), reinterpret_cast<pk::u32*>(oi.data_ptr<int32_t>()),
                    ws.data_ptr(), cur_stream(cols));
    return {op, oi};
  }

  std::vector<torch::Tensor> build_from_soa(const torch::Device& dev) {
    const c10::DeviceGuard guard(dev);
    ensure_ws(dev);
    auto opts = torch::TensorOptions().device(dev);
    torch::Tensor op = torch::empty({b.n(), b.dim()}, opts.dtype(torch::kFloat32));
    torch::Tensor oi = torch::empty({b.n()}, opts.dtype(torch::kInt32));
    b.build_from_soa(op.data_ptr<float>(), reinterpret_cast<pk::u32*>(oi.data_ptr<int32_t>()), ws.data_ptr(),
                     c10::hip::getCurrentHIPStream(dev.index()).stream());
    return {op, oi};
  }
};

// Reference-mode GPU builder (build_reference.hip) with a torch-allocated workspace.
struct RefBuilder {
  pk::ReferenceBuilder b;
  int64_t n, dim;
  torch::Tensor ws;
  RefBuilder(int64_t n_, int64_t dim_, int64_t depth0) : b(n_, int(dim_), int(depth0)), n(n_), dim(dim_) {}
  std::vector<torch::Tensor> build(const torch::Tensor& pts, const c10::optional<torch::Tensor>& ids, int64_t id_base) {
    check_points(pts, true);
    TORCH_CHECK(pts.size(0) == n && pts.size(1) == dim, "points shape does not match the builder");
    const c10::DeviceGuard guard(pts.device());
    if (!ws.defined() || ws.device() != pts.device())
      ws = torch::empty({int64_t(b.workspace_bytes())}, pts.options().dtype(torch::kUInt8));
    torch::Tensor op = torch::empty_like(pts);
    torch::Tensor oi = torch::empty({n}, pts.options().dtype(torch::kInt32));
    b.build(pts.data_ptr<float>(), opt_ids(ids, n, pts.device()), pk::u32(id_base), op.data_ptr<float>(),
            reinterpret_cast<pk::u32*>(oi.data_ptr<int32_t>()), ws.data_ptr(), cur_stream(pts));
    return {op, oi};
  }
};

// Hybrid reference mode (cpu_tree.hpp reference_repair): points [n, dim] (host), the GPU tree's
// slot -> input row map [n] (int32, host), the tied segments' median slots. Returns (perm int32 [n]:
// slot -> row of the reference tree, decided slots int64 [k]: the slots the host decided).
std::vector<torch::Tensor> reference_repair(const torch::Tensor& pts, const torch::Tensor& gpu_rows,
                                            const std::vector<int64_t>& tied, int64_t depth0, int64_t threads) {
  check_points(pts, false);
  const int64_t n = pts.size(0);
  TORCH_CHECK(gpu_rows.scalar_type() == torch::kInt32 && !gpu_rows.is_cuda() && gpu_rows.is_contiguous() &&
                  gpu_rows.numel() == n, "gpu_rows: int32 [n] host tensor");
  std::vector<pk::u32> ts(tied.begin(), tied.end());
  torch::Tensor perm = torch::empty({n}, torch::kInt32);
  const auto ranges = pk::reference_repair(pts.data_ptr<float>(), n, int(pts.size(1)), int(depth0),
                                           reinterpret_cast<const pk::u32*>(gpu_rows.data_ptr<int32_t>()), ts.data(),
                                           ts.size(), reinterpret_cast<pk::u32*>(perm.data_ptr<int32_t>()),
                                           int(threads));
  int64_t k = 0;
  for (const auto& r : ranges) k += r.second;
  torch::Tensor slots = torch::empty({k}, torch::kInt64);
  int64_t* sp = slots.data_ptr<int64_t>();
  for (const auto& r : ranges)
    for (int64_t j = 0; j < r.second; ++j) *sp++ = r.first + j;
  return {perm, slots};
}

// The reference's std::sort of row indices by keys: libstdc++ itself (replica = false) or the
// parallel replica (cpu_tree.hpp std_sort_replica) -- the test that they agree bit for bit.
torch::Tensor sort_indices(const torch::Tensor& keys, bool replica, int64_t threads) {
  TORCH_CHECK(keys.scalar_type() == torch::kFloat32 && !keys.is_cuda() && keys.is_contiguous() && keys.dim() == 1,
              "keys: float32 host vector");
  const int64_t n = keys.numel();
  torch::Tensor idx = torch::arange(n, torch::kInt32);
  auto* ip = reinterpret_cast<pk::u32*>(idx.data_ptr<int32_t>());
  const float* k = keys.data_ptr<float>();
  if (replica) pk::std_sort_replica(k, ip, n, int(threads));
  else std::sort(ip, ip + n, [k](pk::u32 a, pk::u32 b) { return k[a] < k[b]; });
  return idx;
}

torch::Tensor generate(int64_t seed, int64_t dim, int64_t rows, int64_t first, int64_t threads) {
  TORCH_CHECK(dim > 0 && rows >= 0 && first >= 0, "bad generator arguments");
  torch::Tensor x = torch::empty({rows, dim}, torch::kFloat32);
  pk::generate_rows(int(seed), int(dim), first, rows, x.data_ptr<float>(), int(threads));
  return x;
}

// Rows [first, first + rows) of the reference stream generated on `out`'s GPU.
torch::Tensor generate_gpu(int64_t seed, int64_t first, torch::Tensor out) {
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == torch::kFloat32 && out.is_contiguous() && out.dim() == 2,
              "out must be a contiguous float32 [rows, dim] GPU tensor");
  TORCH_CHECK(first >= 0, "first must be >= 0");
  const c10::DeviceGuard guard(out.device());
  const pk::DevGenPlan p = pk::devgen_plan(uint64_t(out.size(0)) * uint64_t(out.size(1)));
  torch::Tensor ws = torch::empty({int64_t(pk::devgen_workspace_bytes(p)) + 1},
                                  out.options().dtype(torch::kUInt8));
  pk::generate_rows_device(uint32_t(seed), int(out.size(1)), first, out.size(0), out.data_ptr<float>(),
                           ws.data_ptr(), cur_stream(out));
  return out;
}

// The device algorithm on the host (CPU oracle for the kernels' arithmetic).
torch::Tensor generate_emulated(int64_t seed, int64_t dim, int64_t rows, int64_t first) {
  TORCH_CHECK(dim > 0 && rows >= 0 && first >= 0, "bad generator arguments");
  torch::Tensor x = torch::empty({rows, dim}, torch::kFloat32);
  pk::devgen_emulate(uint32_t(seed), uint64_t(first) * uint64_t(dim), uint64_t(rows) * uint64_t(dim),
                     x.data_ptr<float>());
  return x;
}

std::vector<torch::Tensor> build_cpu(const torch::Tensor& pts, const c10::optional<torch::Tensor>& ids,
                                     const std::string& mode, int64_t depth0, int64_t threads) {
  check_points(pts, false);
  const int64_t n = pts.size(0);
  const int dim = int(pts.size(1));
  std::vector<pk::u32> perm(size_t(std::max<int64_t>(n, 1)));
  const pk::u32* idp = opt_ids(ids, n, pts.device());
  if (mode == "exact") {
    pk::build_exact_cpu(pts.data_ptr<float>(), idp, n, dim, int(depth0), perm.data(), int(threads));
  } else if (mode == "reference") {
    pk::build_reference_cpu(pts.data_ptr<float>(), n, dim, perm.data(), int(threads), int(depth0));
  } else {
    TORCH_CHECK(false, "mode must be 'exact' or 'reference'");
  }
  torch::Tensor tp = torch::empty_like(pts);
  torch::Tensor ti = torch::empty({n}, torch::kInt32);
  pk::gather_rows(pts.data_ptr<float>(), idp, perm.data(), n, dim, tp.data_ptr<float>(),
                  reinterpret_cast<pk::u32*>(ti.data_ptr<int32_t>()));
  return {tp, ti};
}

// CPU search with the reference's procedure: returns (slot, d2) per query.
std::vector<torch::Tensor> search_cpu(const torch::Tensor& tree_pts, const torch::Tensor& queries, int64_t depth0,
                                      bool brute) {
  check_points(tree_pts, false);
  check_points(queries, false);
  TORCH_CHECK(queries.size(1) == tree_pts.size(1), "dimension mismatch");
  const int64_t nq = queries.size(0);
  const int dim = int(tree_pts.size(1));
  torch::Tensor slots = torch::empty({nq}, torch::kInt64);
  torch::Tensor d2 = torch::empty({nq}, torch::kFloat32);
  for (int64_t i = 0; i < nq; ++i) {
    const float* q = queries.data_ptr<float>() + i * dim;
    const pk::NNResult r = brute ? pk::nn_brute_cpu(tree_pts.data_ptr<float>(), tree_pts.size(0), dim, q)
                                 : pk::nn_search_cpu(tree_pts.data_ptr<float>(), tree_pts.size(0), dim, int(depth0), q);
    slots.data_ptr<int64_t>()[i] = r.slot;
    d2.data_ptr<float>()[i] = r.d2;
  }
  return {slots, d2};
}

// Reference tree dumps (Utility.cpp:21-63) of a CPU implicit tree, as a string.
std::string tree_dump(const torch::Tensor& tree_pts, const torch::Tensor& tree_ids, const std::string& what) {
  check_points(tree_pts, false);
  TORCH_CHECK(tree_ids.scalar_type() == torch::kInt32 && tree_ids.is_contiguous() &&
                  tree_ids.numel() == tree_pts.size(0) && !tree_ids.is_cuda(),
              "tree_ids must be int32 [n] on the CPU");
  std::ostringstream os;
  const auto* ids = reinterpret_cast<const pk::u32*>(tree_ids.data_ptr<int32_t>());
  if (what == "tree") pk::print_tree(os, tree_pts.data_ptr<float>(), ids, tree_pts.size(0), int(tree_pts.size(1)));
  else if (what == "head_and_leaves")
    pk::print_head_and_leaves(os, tree_pts.data_ptr<float>(), ids, tree_pts.size(0), int(tree_pts.size(1)));
  else TORCH_CHECK(false, "what must be tree or head_and_leaves");
  return os.str();
}

std::string point_str(int64_t id, const torch::Tensor& coords) {
  TORCH_CHECK(coords.scalar_type() == torch::kFloat32 && coords.is_contiguous() && !coords.is_cuda() &&
                  coords.dim() == 1, "coords must be a float32 CPU vector");
  std::ostringstream os;
  pk::print_point(os, id, coords.data_ptr<float>(), int(coords.numel()));
  return os.str();
}

int64_t invariant_violations(const torch::Tensor& tree_pts, const torch::Tensor& tree_ids, int64_t depth0) {
  TORCH_CHECK(tree_ids.scalar_type() == torch::kInt32 && tree_ids.is_contiguous() &&
                  tree_ids.numel() == tree_pts.size(0) && tree_ids.device() == tree_pts.device(),
              "tree_ids must be int32 [n] on the points' device");
  if (tree_pts.is_cuda()) {  // the device checker (query.hip)
    check_points(tree_pts, true);
    const c10::DeviceGuard guard(tree_pts.device());
    torch::Tensor cnt = torch::zeros({1}, tree_pts.options().dtype(torch::kInt64));
    pk::check_tree(tree_pts.data_ptr<float>(), reinterpret_cast<const pk::u32*>(tree_ids.data_ptr<int32_t>()),
                   tree_pts.size(0), int(tree_pts.size(1)), int(depth0),
                   reinterpret_cast<unsigned long long*>(cnt.data_ptr<int64_t>()), cur_stream(tree_pts));
    return cnt.item<int64_t>();
  }
  check_points(tree_pts, false);
  return pk::count_invariant_violations(tree_pts.data_ptr<float>(),
                                        reinterpret_cast<const pk::u32*>(tree_ids.data_ptr<int32_t>()),
                                        tree_pts.size(0), int(tree_pts.size(1)), int(depth0));
}

// Packed (d2, id) results as int64 (bit pattern of the u64 packing).
torch::Tensor nn_gpu(const torch::Tensor& pts, const c10::optional<torch::Tensor>& ids, int64_t id_base,
                     const torch::Tensor& queries, const std::string& method, int64_t depth0,
                     c10::optional<torch::Tensor> into) {
  check_points(pts, true);
  check_points(queries, true);
  TORCH_CHECK(queries.size(1) == pts.size(1), "dimension mismatch");
  TORCH_CHECK(queries.device() == pts.device(), "queries must be on the tree's device");
  const c10::DeviceGuard guard(pts.device());
  const int64_t nq = queries.size(0);
  hipStream_t s = cur_stream(pts);
  torch::Tensor out;
  if (into.has_value()) {
    out = *into;
    TORCH_CHECK(out.scalar_type() == torch::kInt64 && out.numel() == nq && out.is_contiguous() &&
                    out.device() == pts.device(), "`into` must be a contiguous int64 [nq] tensor on the tree's device");
  } else {
    out = torch::empty({nq}, queries.options().dtype(torch::kInt64));
    pk::nn_init(reinterpret_cast<pk::u64*>(out.data_ptr<int64_t>()), nq, s);
  }
  auto* o = reinterpret_cast<pk::u64*>(out.data_ptr<int64_t>());
  const pk::u32* idp = opt_ids(ids, pts.size(0), pts.device());
  if (method == "brute") {
    pk::nn_brute(pts.data_ptr<float>(), idp, pk::u32(id_base), pts.size(0), int(pts.size(1)),
                 queries.data_ptr<float>(), nq, o, s);
  } else if (method == "traverse") {
    TORCH_CHECK(idp != nullptr, "traverse needs the tree ids");
    pk::nn_traverse(pts.data_ptr<float>(), idp, pts.size(0), int(pts.size(1)), int(depth0), queries.data_ptr<float>(),
                    nq, o, s);
  } else if (method == "reference") {  // the reference's search procedure (reference-mode trees)
    TORCH_CHECK(idp != nullptr, "the reference search needs the tree ids");
    pk::nn_traverse_reference(pts.data_ptr<float>(), idp, pts.size(0), int(pts.size(1)), int(depth0),
                              queries.data_ptr<float>(), nq, o, s);
  } else {
    TORCH_CHECK(false, "method must be 'brute', 'traverse' or 'reference'");
  }
  return out;
}

std::vector<torch::Tensor> nn_finalize(const torch::Tensor& packed) {
  TORCH_CHECK(packed.is_cuda() && packed.scalar_type() == torch::kInt64 && packed.is_contiguous(), "bad packed");
  const c10::DeviceGuard guard(packed.device());
  torch::Tensor d = torch::empty({packed.numel()}, packed.options().dtype(torch::kFloat32));
  torch::Tensor i = torch::empty({packed.numel()}, packed.options().dtype(torch::kInt64));
  pk::nn_finalize(reinterpret_cast<const pk::u64*>(packed.data_ptr<int64_t>()), packed.numel(), d.data_ptr<float>(),
                  i.data_ptr<int64_t>(), cur_stream(packed));
  return {d, i};
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X-native kd-tree core (HIP/CDNA4 kernels + C++ runtime)";
  py::class_<Builder>(m, "GpuBuilder")
      .def(py::init<int64_t, int64_t, int64_t, int64_t, bool>(), py::arg("n"), py::arg("dim"), py::arg("depth0") = 0,
           py::arg("subtree_max") = 0, py::arg("allow_top") = true)
      .def("build", &Builder::build, py::arg("points"), py::arg("ids") = c10::nullopt, py::arg("id_base") = 0,
           py::arg("out_pts") = c10::nullopt, py::arg("out_ids") = c10::nullopt)
      .def("build_rows", &Builder::build_rows, py::arg("rows"))
      .def("soa_input", &Builder::soa_input)
      .def("build_columns", &Builder::build_columns)
      .def("build_from_soa", &Builder::build_from_soa)
      .def_property_readonly("workspace_bytes", [](const Builder& b) { return int64_t(b.b.workspace_bytes()); })
      .def_property_readonly("global_levels", [](const Builder& b) { return b.b.global_levels(); })
      .def_property_readonly("subtree_max", [](const Builder& b) { return b.b.subtree_max(); })
      .def_property_readonly("split_parts", [](const Builder& b) { return b.b.split_parts(); })
      .def_property_readonly("split_level", [](const Builder& b) { return b.b.split_level(); })
      .def_property_readonly("split_streams", [](const Builder& b) { return b.b.split_streams(); })
      .def("describe", [](const Builder& b) { return b.b.describe(); })
      .def_property_readonly("sampled_top", [](const Builder& b) { return b.b.sampled_top(); })
      .def_property_readonly("sampled", [](const Builder& b) { return b.b.sampled(); })
      .def_property_readonly("column_stride", [](const Builder& b) { return int64_t(b.b.column_stride()); })
      .def("top_band_report", [](Builder& b) {  // per top node: band rows, rank in the median's bin, staged rows
        TORCH_CHECK(b.ws.defined(), "no build yet");
        const auto v = b.b.top_band_report(b.ws.data_ptr(), c10::hip::getCurrentHIPStream(b.ws.device().index()).stream());
        return std::vector<int64_t>(v.begin(), v.end());
      })
      .def("g3_report", [](Builder& b) {  // last sampled triple: level, then 25 words per segment
        TORCH_CHECK(b.ws.defined(), "no build yet");
        const auto v = b.b.g3_report(b.ws.data_ptr(), c10::hip::getCurrentHIPStream(b.ws.device().index()).stream());
        return std::vector<int64_t>(v.begin(), v.end());
      })
      .def("error_words", [](Builder& b) {  // view of the workspace's 4 error words (int32)
        TORCH_CHECK(b.ws.defined(), "no build yet");
        return torch::from_blob(const_cast<pk::u32*>(b.b.error_word(b.ws.data_ptr())), {4},
                                b.ws.options().dtype(torch::kInt32));
      })
      .def("accumulate_error", [](Builder& b, torch::Tensor acc) {  // acc: int32 [>= 3] on the build's device
        TORCH_CHECK(b.ws.defined(), "no build yet");
        TORCH_CHECK(acc.is_cuda() && acc.scalar_type() == torch::kInt32 && acc.numel() >= 3 && acc.is_contiguous() &&
                        acc.device() == b.ws.device(), "acc must be a contiguous int32 [>= 3] tensor on the build's device");
        b.b.accumulate_error(b.ws.data_ptr(), reinterpret_cast<pk::u32*>(acc.data_ptr<int32_t>()),
                             c10::hip::getCurrentHIPStream(b.ws.device().index()).stream());
      })
      .def("read_error", [](Builder& b) {
        u32 d[3];
        const u32 e = b.b.read_error(b.ws.data_ptr(), c10::hip::getCurrentHIPStream(b.ws.device().index()).stream(), d);
        return std::vector<int64_t>{int64_t(e), int64_t(d[0]), int64_t(d[1]), int64_t(d[2])};
      });
  py::class_<RefBuilder>(m, "ReferenceBuilder")
      .def(py::init<int64_t, int64_t, int64_t>(), py::arg("n"), py::arg("dim"), py::arg("depth0") = 0)
      .def("build", &RefBuilder::build, py::arg("points"), py::arg("ids") = c10::nullopt, py::arg("id_base") = 0)
      .def("read_ties", [](RefBuilder& b) {
        TORCH_CHECK(b.ws.defined(), "read_ties: no build yet");
        return int64_t(b.b.read_ties(b.ws.data_ptr(), c10::hip::getCurrentHIPStream(b.ws.device().index()).stream()));
      })
      .def("read_tie_slots", [](RefBuilder& b) {
        TORCH_CHECK(b.ws.defined(), "read_tie_slots: no build yet");
        const auto v = b.b.read_tie_slots(b.ws.data_ptr(), c10::hip::getCurrentHIPStream(b.ws.device().index()).stream());
        return std::vector<int64_t>(v.begin(), v.end());
      })
      .def_property_readonly_static("tie_slots_cap", [](py::object) { return int64_t(pk::ReferenceBuilder::kTieSlots); })
      .def_property_readonly("sorted_levels", [](const RefBuilder& b) { return b.b.sorted_levels(); })
      .def_property_readonly("global_levels", [](const RefBuilder& b) { return b.b.global_levels(); })
      .def_property_readonly("workspace_bytes", [](const RefBuilder& b) { return int64_t(b.b.workspace_bytes()); });
  m.def("generate", &generate, py::arg("seed"), py::arg("dim"), py::arg("rows"), py::arg("first") = 0,
        py::arg("threads") = 0);
  m.def("generate_gpu", &generate_gpu, py::arg("seed"), py::arg("first"), py::arg("out"));
  m.def("generate_emulated", &generate_emulated, py::arg("seed"), py::arg("dim"), py::arg("rows"),
        py::arg("first") = 0);
  m.def("devgen_plan", [](int64_t total) {
    const pk::DevGenPlan p = pk::devgen_plan(uint64_t(total));
    return std::vector<int64_t>{int64_t(p.S), int64_t(p.C), int64_t(p.R)};
  });
  m.def("reference_repair", &reference_repair, py::arg("points"), py::arg("gpu_rows"), py::arg("tied"),
        py::arg("depth0") = 0, py::arg("threads") = 1, py::call_guard<py::gil_scoped_release>());
  m.def("sort_indices", &sort_indices, py::arg("keys"), py::arg("replica"), py::arg("threads") = 1,
        py::call_guard<py::gil_scoped_release>());
  m.def("build_cpu", &build_cpu, py::arg("points"), py::arg("ids") = c10::nullopt, py::arg("mode") = "exact",
        py::arg("depth0") = 0, py::arg("threads") = 1);
  m.def("search_cpu", &search_cpu, py::arg("tree_pts"), py::arg("queries"), py::arg("depth0") = 0,
        py::arg("brute") = false);
  m.def("trace_push", [](const std::string& name) { pk::trace_push(name.c_str()); }, py::arg("name"));
  m.def("trace_pop", &pk::trace_pop);
  m.def("ab_knob", [](const std::string& name) -> py::object {
    const char* v = pk::ab_knob(name.c_str());
    return v ? py::object(py::str(v)) : py::object(py::none());
  }, py::arg("name"), "Value of an A/B tuning knob: honoured only under PKD_AB=1, else None.");
  m.def("tree_dump", &tree_dump, py::arg("tree_pts"), py::arg("tree_ids"), py::arg("what") = "tree");
  m.def("point_str", &point_str, py::arg("id"), py::arg("coords"));
  m.def("invariant_violations", &invariant_violations, py::arg("tree_pts"), py::arg("tree_ids"),
        py::arg("depth0") = 0);
  m.def("nn", &nn_gpu, py::arg("points"), py::arg("ids"), py::arg("id_base"), py::arg("queries"),
        py::arg("method") = "brute", py::arg("depth0") = 0, py::arg("into") = c10::nullopt);
  m.def("nn_finalize", &nn_finalize, py::arg("packed"));
  m.def("subtree_capacity", &pk::default_subtree_max);
  m.def("subtree_stamp_report", &pk::subtree_stamp_report);
  m.def("tail_stamp_report", &pk::tail_stamp_report);
  pkdtree::bind_dist_ops(m);
}
