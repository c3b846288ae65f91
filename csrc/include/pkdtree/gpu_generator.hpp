// Device generator of the reference data stream (std::mt19937(seed) +
// uniform_real_distribution<float>(-100, 100), Utility.cpp:6-18 / kdtree_mpi.cpp:19-41),
// bit-identical to the host generator, for any slice [first_row, first_row + rows).
//
// The stream is cut into C chunks (DevGenPlan, generator.hpp). Chunk 0's MT state comes from
// the host (O(log n) jump-ahead); the other C-1 states are produced on the device by log2(C)
// doubling rounds (extension + GF(2) correlation kernels), then one workgroup per chunk
// twists its state in LDS and writes tempered, mapped floats. Nothing here walks the stream
// serially: the reference's discard() over the whole prefix is gone.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pkdtree/generator.hpp"

namespace pkdtree {

// Device workspace bytes for a plan (states, extensions, polynomials).
size_t devgen_workspace_bytes(const DevGenPlan& p);
// Writes rows * dim floats (row-major, the reference layout) to out. The host part (jump
// polynomials, start window) is computed before the enqueue; the copy of those inputs to the
// workspace is a synchronous hipMemcpy. Kernels run on `stream`.
void generate_rows_device(uint32_t seed, int dim, int64_t first_row, int64_t rows, float* out, void* workspace,
                          hipStream_t stream);

}  // namespace pkdtree
