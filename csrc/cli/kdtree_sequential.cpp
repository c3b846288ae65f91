// kdtree_sequential — CPU executable with the reference's protocol
// (kdtree_sequential.cpp:140-208). Options: --mode exact|reference, --threads T
// (threaded exact build: the reference's missing OMP variant, Makefile:23-27), --save PATH
// (the tree in the tree_io.hpp format; ids are the reference's 1-based point ids).
#include <chrono>
#include <cmath>
#include <cstdio>
#include <vector>

#include "cli_common.hpp"
#include "pkdtree/cpu_tree.hpp"
#include "pkdtree/generator.hpp"
#include "pkdtree/tree_io.hpp"

using namespace pkdtree;

int main(int argc, char** argv) {
  cli::Options o = cli::parse(argc, argv);
  const auto tick = std::chrono::high_resolution_clock::now();
  const Problem p = cli::specify(o);
  const int Q = o.num_queries;
  const i64 N = p.num_points;
  std::vector<float> x = generate_problem(p.seed, p.dim, N + Q);
  std::vector<u32> perm(static_cast<size_t>(N));
  if (o.mode == "reference") {
    build_reference_cpu(x.data(), N, p.dim, perm.data(), o.threads > 0 ? o.threads : 1);
  } else {
    build_exact_cpu(x.data(), nullptr, N, p.dim, 0, perm.data(), o.threads > 0 ? o.threads : 1);
  }
  std::vector<float> tree(static_cast<size_t>(N) * static_cast<size_t>(p.dim));
  gather_rows(x.data(), nullptr, perm.data(), N, p.dim, tree.data(), nullptr);
  if (!o.save.empty()) {
    std::vector<u32> ids(static_cast<size_t>(N));
    for (i64 i = 0; i < N; ++i) ids[size_t(i)] = perm[size_t(i)] + 1;  // reference ids 1..N
    tree_file_create(o.save, N, p.dim, 0, o.mode == "reference" ? kTreeModeReference : kTreeModeExact);
    tree_file_write(o.save, N, p.dim, 0, N, tree.data(), ids.data());
  }
  for (int q = 0; q < Q; ++q) {
    const float* qp = x.data() + size_t(N + q) * size_t(p.dim);
    const NNResult r = nn_search_cpu(tree.data(), N, p.dim, 0, qp);
    const float d = std::sqrt(sq_dist(qp, tree.data() + size_t(r.slot) * size_t(p.dim), p.dim));
    print_result_line(N + q, d);
  }
  if (o.debug) {
    const auto tock = std::chrono::high_resolution_clock::now();
    print_elapsed(std::chrono::duration<double>(tock - tick).count());
  }
  print_done();
  return 0;
}
