// Bindings of the distributed-decomposition device ops (csrc/gpu/dist_ops.hip).
#include <torch/extension.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include "pkdtree/dist_ops.hpp"

namespace pkdtree {

namespace {

hipStream_t stream_of(const torch::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check_rows(const torch::Tensor& rows, int64_t dim) {
  TORCH_CHECK(rows.is_cuda() && rows.scalar_type() == torch::kFloat32 && rows.is_contiguous(), "rows: cuda f32");
  TORCH_CHECK(rows.dim() == 2 && rows.size(1) == dim + 1, "rows must be [n, dim+1]");
}

u32* u32p(torch::Tensor& t) { return reinterpret_cast<u32*>(t.data_ptr<int32_t>()); }
const u64* u64p(const torch::Tensor& t) { return reinterpret_cast<const u64*>(t.data_ptr<int64_t>()); }

void route_hist(const torch::Tensor& rows, int64_t dim, torch::Tensor node, int64_t level, const torch::Tensor& pivots,
                int64_t prev_axis, int64_t axis, const torch::Tensor& params, int64_t bins, torch::Tensor hist) {
  check_rows(rows, dim);
  const c10::DeviceGuard g(rows.device());
  top_route_hist(rows.data_ptr<float>(), rows.size(0), int(dim), u32p(node), int(level), u64p(pivots),
                 int(prev_axis), int(axis), params.data_ptr<float>(), int(bins), u32p(hist), stream_of(rows));
}

int64_t collect_middle(const torch::Tensor& rows, int64_t dim, const torch::Tensor& node, int64_t level,
                       int64_t axis, const torch::Tensor& params, int64_t bins, const torch::Tensor& bstar,
                       torch::Tensor out, torch::Tensor count) {
  check_rows(rows, dim);
  const c10::DeviceGuard g(rows.device());
  top_collect_middle(rows.data_ptr<float>(), rows.size(0), int(dim),
                     reinterpret_cast<const u32*>(node.data_ptr<int32_t>()), int(level), int(axis),
                     params.data_ptr<float>(), int(bins), reinterpret_cast<const u32*>(bstar.data_ptr<int32_t>()),
                     out.data_ptr<float>(), out.size(0), reinterpret_cast<unsigned long long*>(count.data_ptr<int64_t>()),
                     stream_of(rows));
  return 0;
}

void pack(const torch::Tensor& rows, int64_t dim, torch::Tensor node, int64_t levels, const torch::Tensor& pivots,
          int64_t last_axis, int64_t P, torch::Tensor out, torch::Tensor counts, torch::Tensor scratch) {
  check_rows(rows, dim);
  const c10::DeviceGuard g(rows.device());
  TORCH_CHECK(size_t(scratch.numel()) >= top_pack_scratch_bytes(rows.size(0), int(P)), "scratch too small");
  top_pack(rows.data_ptr<float>(), rows.size(0), int(dim), u32p(node), int(levels), u64p(pivots), int(last_axis),
           int(P), out.data_ptr<float>(), u32p(counts), scratch.data_ptr(), stream_of(rows));
}

}  // namespace

void bind_dist_ops(pybind11::module& m) {
  m.def("top_route_hist", &route_hist);
  m.def("top_collect_middle", &collect_middle);
  m.def("top_pack", &pack);
  m.def("top_pack_scratch_bytes", [](int64_t n, int64_t P) { return int64_t(top_pack_scratch_bytes(n, int(P))); });
}

}  // namespace pkdtree
