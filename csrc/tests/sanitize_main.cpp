// Host sanitizer harness: the CPU paths compiled with AddressSanitizer +
// UndefinedBehaviorSanitizer (tests/test_sanitizers.py) and exercised end to end: generator
// slices (jump-ahead vs sequential), threaded exact build, reference-mode build, both NN
// searches and the invariant checker, over sizes that hit every recursion edge case.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "pkdtree/cpu_tree.hpp"
#include "pkdtree/generator.hpp"

using namespace pkdtree;

static int fail(const char* what, long long a, long long b) {
  std::fprintf(stderr, "FAIL %s: %lld vs %lld\n", what, a, b);
  return 1;
}

int main() {
  const int sizes[] = {1, 2, 3, 7, 64, 1000, 4097};
  for (int dim : {1, 3, 8}) {
    for (int n : sizes) {
      const std::vector<float> all = generate_problem(11, dim, n + 4);
      std::vector<float> part(size_t(n) * dim);
      generate_rows(11, dim, 0, n, part.data(), 3);  // threaded jump-ahead slices
      for (size_t i = 0; i < part.size(); ++i)
        if (part[i] != all[i]) return fail("generate_rows", long(i), 0);
      std::vector<u32> ids(n), perm(n);
      for (int i = 0; i < n; ++i) ids[i] = u32(3 * i + 1);
      for (int threads : {1, 4}) {
        build_exact_cpu(all.data(), ids.data(), n, dim, 0, perm.data(), threads);
        std::vector<float> tp(size_t(n) * dim);
        std::vector<u32> ti(n);
        gather_rows(all.data(), ids.data(), perm.data(), n, dim, tp.data(), ti.data());
        const i64 bad = count_invariant_violations(tp.data(), ti.data(), n, dim, 0);
        if (bad) return fail("invariant", bad, 0);
        for (int q = 0; q < 4; ++q) {
          const float* qp = all.data() + size_t(n + q) * dim;
          const NNResult a = nn_search_cpu(tp.data(), n, dim, 0, qp);
          const NNResult b = nn_brute_cpu(tp.data(), n, dim, qp);
          if (a.d2 != b.d2) return fail("nn", a.slot, b.slot);
        }
      }
      build_reference_cpu(all.data(), n, dim, perm.data());
      std::vector<int> seen(n, 0);
      for (int i = 0; i < n; ++i) seen[perm[i]]++;
      for (int i = 0; i < n; ++i)
        if (seen[i] != 1) return fail("reference permutation", i, seen[i]);
    }
  }
  std::printf("sanitize ok\n");
  return 0;
}
