// Bindings of the distributed-decomposition device ops (filled in with the global mode).
#include <torch/extension.h>

namespace pkdtree {
void bind_dist_ops(pybind11::module& m) { (void)m; }
}  // namespace pkdtree
