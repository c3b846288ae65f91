// GPU reference mode, repaired on the host where the reference's std::sort order decides.
//
// The reference sorts with std::sort, which is unstable: where equal keys meet at a segment's
// deciding ranks (m-2..m+1), its tree is whatever its library's introsort produced, and that
// depends on the segment's exact input order -- i.e. on every ancestor's sort. ReferenceBuilder
// counts those segments and lists their median slots (read_tie_slots); reference_repair then
// replays, on the host and with the reference's own algorithm (a bit-exact parallel replica of
// std::sort), only the ancestors' sorts and the tied segments' subtrees, and keeps every other
// subtree of the GPU tree (no deciding tie at or below it: exact there). The host-decided slots
// are patched into the device tree (reference_patch). Above ReferenceBuilder::kTieSlots tied
// segments the whole tree is rebuilt by the threaded host builder (build_reference_cpu).
// kdtree_sequential.cpp:30-66 is the reference.
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>
#include <iostream>
#include <memory>
#include <vector>

#include "pkdtree/cpu_tree.hpp"
#include "pkdtree/gpu_reference.hpp"
#include "pkdtree/hip_check.hpp"

namespace pkdtree {
namespace cli {

// Builds the reference tree of the device points d_pts [n][dim] (ids id_base + row) into
// d_tree / d_ids on the GPU; returns the tie count of the GPU build (non-zero: the host repaired
// the tree). `who` prefixes the stderr note. Synchronises `s`.
inline u32 build_reference_checked(const ReferenceBuilder& rb, const float* d_pts, i64 n, int dim, u32 id_base,
                                   float* d_tree, u32* d_ids, void* ws, hipStream_t s, const char* who) {
  if (n <= 0) return 0;
  rb.build(d_pts, nullptr, id_base, d_tree, d_ids, ws, s);
  const u32 ties = rb.read_ties(ws, s);
  if (ties == 0) return 0;
  const auto t0 = std::chrono::steady_clock::now();
  // the host sorts read one key per row and level: with more columns than levels, only the
  // levels' keys travel (500 k x 128D: 19 columns, 38 MB instead of 256 MB)
  int levels = 0;
  while ((i64(1) << levels) <= n) ++levels;
  const bool narrow = levels < dim;
  const int hdim = narrow ? levels : dim;
  std::unique_ptr<float[]> h(new float[size_t(n) * size_t(hdim)]);
  if (narrow) {
    float* d_keys = nullptr;
    PKD_HIP_CHECK(hipMallocAsync(reinterpret_cast<void**>(&d_keys), size_t(n) * size_t(hdim) * 4, s));
    reference_level_keys(d_pts, n, dim, 0, levels, d_keys, s);
    PKD_HIP_CHECK(hipMemcpyAsync(h.get(), d_keys, size_t(n) * size_t(hdim) * 4, hipMemcpyDeviceToHost, s));
    PKD_HIP_CHECK(hipFreeAsync(d_keys, s));
  } else {
    PKD_HIP_CHECK(hipMemcpyAsync(h.get(), d_pts, size_t(n) * size_t(dim) * 4, hipMemcpyDeviceToHost, s));
  }
  std::vector<u32> perm(static_cast<size_t>(n));
  i64 patched = n;
  if (ties <= ReferenceBuilder::kTieSlots) {
    const std::vector<u32> slots = rb.read_tie_slots(ws, s);
    std::vector<u32> gpu(static_cast<size_t>(n));
    PKD_HIP_CHECK(hipMemcpyAsync(gpu.data(), d_ids, size_t(n) * 4, hipMemcpyDeviceToHost, s));
    PKD_HIP_CHECK(hipStreamSynchronize(s));
    for (auto& g : gpu) g -= id_base;  // slot -> input row
    const auto ranges = reference_repair(h.get(), n, hdim, 0, gpu.data(), slots.data(), slots.size(), perm.data(),
                                         default_cpu_threads());
    std::vector<u32> sl, rw;
    for (const auto& r : ranges)
      for (i64 k = r.first; k < r.first + r.second; ++k) {
        sl.push_back(u32(k));
        rw.push_back(perm[size_t(k)]);
      }
    patched = i64(sl.size());
    u32* d_patch = nullptr;
    PKD_HIP_CHECK(hipMalloc(&d_patch, std::max<size_t>(1, sl.size()) * 8));
    PKD_HIP_CHECK(hipMemcpyAsync(d_patch, sl.data(), sl.size() * 4, hipMemcpyHostToDevice, s));
    PKD_HIP_CHECK(hipMemcpyAsync(d_patch + sl.size(), rw.data(), rw.size() * 4, hipMemcpyHostToDevice, s));
    reference_patch(d_pts, nullptr, id_base, dim, d_patch, d_patch + sl.size(), patched, d_tree, d_ids, s);
    PKD_HIP_CHECK(hipStreamSynchronize(s));
    PKD_HIP_CHECK(hipFree(d_patch));
  } else {  // too many tied segments to list: the whole tree on the host, rows placed on the device
    PKD_HIP_CHECK(hipStreamSynchronize(s));
    build_reference_cpu(h.get(), n, hdim, perm.data(), default_cpu_threads());
    std::vector<u32> sl(static_cast<size_t>(n));
    for (i64 k = 0; k < n; ++k) sl[size_t(k)] = u32(k);
    u32* d_patch = nullptr;
    PKD_HIP_CHECK(hipMalloc(&d_patch, size_t(n) * 8));
    PKD_HIP_CHECK(hipMemcpyAsync(d_patch, sl.data(), size_t(n) * 4, hipMemcpyHostToDevice, s));
    PKD_HIP_CHECK(hipMemcpyAsync(d_patch + n, perm.data(), size_t(n) * 4, hipMemcpyHostToDevice, s));
    reference_patch(d_pts, nullptr, id_base, dim, d_patch, d_patch + n, n, d_tree, d_ids, s);
    PKD_HIP_CHECK(hipStreamSynchronize(s));
    PKD_HIP_CHECK(hipFree(d_patch));
  }
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  std::cerr << who << ": reference mode: " << ties
            << " segment(s) decided by equal keys (the reference's std::sort is unstable there); "
            << (ties <= ReferenceBuilder::kTieSlots ? "replayed their sorts on the host and patched "
                                                    : "rebuilt the tree on the host: ")
            << patched << " of " << n << " slots (" << ms << " ms)" << std::endl;
  return ties;
}

}  // namespace cli
}  // namespace pkdtree
