// Tree files from device memory (see pkdtree/tree_io.hpp): the GPU executables' --save.
#include <algorithm>
#include <vector>

#include "pkdtree/hip_check.hpp"
#include "pkdtree/tree_io.hpp"

namespace pkdtree {

void tree_file_write_device(const std::string& path, i64 n_total, int dim, i64 slot0, i64 count, const float* pts,
                            const u32* ids, hipStream_t stream) {
  if (count <= 0) return;
  const i64 rows = i64(16) << 20;  // 16 Mi slots per chunk: <= 64 MiB of ids, 64 MiB * dim of rows
  std::vector<u32> hi;
  std::vector<float> hp;
  for (i64 s0 = 0; s0 < count; s0 += rows) {
    const i64 c = std::min(rows, count - s0);
    hi.resize(size_t(c));
    hp.resize(size_t(c) * dim);
    PKD_HIP_CHECK(hipMemcpyAsync(hi.data(), ids + s0, size_t(c) * 4, hipMemcpyDeviceToHost, stream));
    PKD_HIP_CHECK(hipMemcpyAsync(hp.data(), pts + s0 * dim, size_t(c) * dim * 4, hipMemcpyDeviceToHost, stream));
    PKD_HIP_CHECK(hipStreamSynchronize(stream));
    tree_file_write(path, n_total, dim, slot0 + s0, c, hp.data(), hi.data());
  }
}

}  // namespace pkdtree
