// kdtree_gpu — single-MI355X executable with the reference's protocol
// (kdtree_sequential.cpp:140-208): the reference data generated on the GPU
// (csrc/gpu/generator.hip, bit-identical to the host stream; --host-gen: on the host), the
// level-synchronous HIP build and exact GPU queries; --mode reference builds the reference's
// own tree on the GPU (build_reference.hip) and answers with its search procedure.
// --metrics-json prints per-phase times (hipEvents) on stderr; --save PATH writes the tree
// (tree_io.hpp); --leaf-threshold N caps the LDS subtree kernel's segments.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <algorithm>
#include <cstdio>
#include <iostream>
#include <vector>

#include "cli_common.hpp"
#include "ref_fallback.hpp"
#include "pkdtree/generator.hpp"
#include "pkdtree/gpu_build.hpp"
#include "pkdtree/gpu_generator.hpp"
#include "pkdtree/gpu_query.hpp"
#include "pkdtree/gpu_reference.hpp"
#include "pkdtree/hip_check.hpp"
#include "pkdtree/tree_io.hpp"

using namespace pkdtree;

int main(int argc, char** argv) {
  cli::Options o = cli::parse(argc, argv);
  const bool ref = o.mode == "reference";
  const auto tick = std::chrono::high_resolution_clock::now();
  const Problem p = cli::specify(o);
  const int Q = o.num_queries;
  const i64 N = p.num_points;
  const int dim = p.dim;
  try {
    PKD_HIP_CHECK(hipSetDevice(o.device));
    hipStream_t s;
    PKD_HIP_CHECK(hipStreamCreate(&s));
    const size_t total = size_t(N + Q) * size_t(dim);
    const auto g0 = std::chrono::high_resolution_clock::now();
    std::vector<float> x;
    float* d_x = nullptr;
    PKD_HIP_CHECK(hipMalloc(&d_x, total * 4));
    if (o.host_gen) {
      x = generate_problem(p.seed, dim, N + Q);
    } else {
      const DevGenPlan gp = devgen_plan(total);
      void* gws = nullptr;
      PKD_HIP_CHECK(hipMalloc(&gws, std::max<size_t>(1, devgen_workspace_bytes(gp))));
      generate_rows_device(uint32_t(p.seed), dim, 0, N + Q, d_x, gws, s);
      PKD_HIP_CHECK(hipStreamSynchronize(s));
      PKD_HIP_CHECK(hipFree(gws));
    }
    const auto g1 = std::chrono::high_resolution_clock::now();
    GpuBuilder b(N, dim, BuildOptions{o.leaf_threshold, 0});
    ReferenceBuilder rb(ref ? N : 0, dim);
    float* d_tree = nullptr;
    u32* d_ids = nullptr;
    u64* d_res = nullptr;
    void* ws = nullptr;
    PKD_HIP_CHECK(hipMalloc(&d_tree, size_t(N) * dim * 4));
    PKD_HIP_CHECK(hipMalloc(&d_ids, size_t(N) * 4));
    PKD_HIP_CHECK(hipMalloc(&d_res, size_t(Q) * 8));
    size_t ws_bytes = std::max(ref ? rb.workspace_bytes() : b.workspace_bytes(), size_t(256));
    PKD_HIP_CHECK(hipMalloc(&ws, ws_bytes));
    hipEvent_t e0, e1, e2, e3;
    for (hipEvent_t* e : {&e0, &e1, &e2, &e3}) PKD_HIP_CHECK(hipEventCreate(e));
    PKD_HIP_CHECK(hipEventRecord(e0, s));
    if (o.host_gen) PKD_HIP_CHECK(hipMemcpyAsync(d_x, x.data(), total * 4, hipMemcpyHostToDevice, s));
    PKD_HIP_CHECK(hipEventRecord(e1, s));
    if (ref) cli::build_reference_checked(rb, d_x, N, dim, 1u, d_tree, d_ids, ws, s, "kdtree_gpu");  // IDs 1..N
    else b.build(d_x, nullptr, 1u, d_tree, d_ids, ws, s);
    PKD_HIP_CHECK(hipEventRecord(e2, s));
    const float* d_q = d_x + size_t(N) * dim;
    nn_init(d_res, Q, s);
    const bool traverse = o.query == "traverse" || (o.query == "auto" && dim <= 16);
    auto query = [&] {
      if (ref) nn_traverse_reference(d_tree, d_ids, N, dim, 0, d_q, Q, d_res, s);  // the reference's search
      else if (traverse) nn_traverse(d_tree, d_ids, N, dim, 0, d_q, Q, d_res, s);
      else nn_brute(d_tree, d_ids, 0, N, dim, d_q, Q, d_res, s);
    };
    query();
    PKD_HIP_CHECK(hipEventRecord(e3, s));
    std::vector<u64> res(static_cast<size_t>(Q));
    PKD_HIP_CHECK(hipMemcpyAsync(res.data(), d_res, size_t(Q) * 8, hipMemcpyDeviceToHost, s));
    PKD_HIP_CHECK(hipStreamSynchronize(s));
    u32 detail[3] = {0, 0, 0};
    u32 err0 = ref ? 0u : b.read_error(ws, s, detail);
    if ((err0 & top4_band_miss_bit()) && b.sampled()) {
      // a sampled top band missed its median (reported, never silent): rebuild unsampled
      // (its plan differs, e.g. a split build's per-stream histogram sets: the workspace is
      // grown to its size before the rebuild, never written past)
      GpuBuilder fb(N, dim, BuildOptions{o.leaf_threshold, 0, true, false});
      if (fb.workspace_bytes() > ws_bytes) {
        PKD_HIP_CHECK(hipFree(ws));
        ws_bytes = fb.workspace_bytes();
        PKD_HIP_CHECK(hipMalloc(&ws, ws_bytes));
      }
      fb.build(d_x, nullptr, 1u, d_tree, d_ids, ws, s);
      nn_init(d_res, Q, s);
      query();
      PKD_HIP_CHECK(hipMemcpyAsync(res.data(), d_res, size_t(Q) * 8, hipMemcpyDeviceToHost, s));
      err0 = fb.read_error(ws, s, detail);
    }
    if (const u32 err = err0) {  // after the queries: no extra sync in the build
      std::cerr << "kdtree_gpu: device build error word 0x" << std::hex << err << std::dec << " (code " << detail[0]
                << ", level " << detail[1] << ", value " << detail[2] << "); no results printed" << std::endl;
      return 3;
    }
    if (!o.save.empty()) {
      tree_file_create(o.save, N, dim, 0, ref ? kTreeModeReference : kTreeModeExact);
      tree_file_write_device(o.save, N, dim, 0, N, d_tree, d_ids, s);
    }
    for (int q = 0; q < Q; ++q) print_result_line(N + q, std::sqrt(packed_dist(res[size_t(q)])));
    if (o.debug) {
      const auto tock = std::chrono::high_resolution_clock::now();
      print_elapsed(std::chrono::duration<double>(tock - tick).count());
    }
    print_done();
    if (o.metrics) {
      float h2d = 0, bld = 0, qry = 0;
      PKD_HIP_CHECK(hipEventElapsedTime(&h2d, e0, e1));
      PKD_HIP_CHECK(hipEventElapsedTime(&bld, e1, e2));
      PKD_HIP_CHECK(hipEventElapsedTime(&qry, e2, e3));
      const double gen = std::chrono::duration<double, std::milli>(g1 - g0).count();
      std::fprintf(stderr,
                   "{\"gen_ms\": %.3f, \"h2d_ms\": %.3f, \"build_ms\": %.3f, \"query_ms\": %.3f, "
                   "\"build_mpts_per_s\": %.2f, \"mode\": \"%s\", \"global_levels\": %d, \"subtree_max\": %d}\n",
                   gen, h2d, bld, qry, double(N) / 1e3 / bld, o.mode.c_str(), ref ? 0 : b.global_levels(),
                   ref ? 0 : b.subtree_max());
    }
    (void)hipFree(d_x); (void)hipFree(d_tree); (void)hipFree(d_ids); (void)hipFree(d_res); (void)hipFree(ws);
    (void)hipStreamDestroy(s);
  } catch (const std::exception& ex) {
    std::cerr << "kdtree_gpu: " << ex.what() << std::endl;
    return 2;
  }
  return 0;
}
