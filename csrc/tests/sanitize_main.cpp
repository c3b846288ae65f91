// Host sanitizer harness: the CPU paths compiled with AddressSanitizer +
// UndefinedBehaviorSanitizer (tests/test_sanitizers.py) and exercised end to end: generator
// slices (jump-ahead vs sequential), threaded exact build, reference-mode build, both NN
// searches and the invariant checker, over sizes that hit every recursion edge case; and the
// global decomposition's planner (global_plan.cpp: segment, make_layout, share_blocks,
// make_plan) swept over P = 1..64, k = -1..6 and n from 0 to 2^32 - 1 with its invariants
// checked -- the code that replaces the reference's N < P-crashing slice arithmetic
// (kdtree_mpi.cpp:208-216).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <stdexcept>
#include <utility>
#include <vector>

#include "pkdtree/cpu_tree.hpp"
#include "pkdtree/generator.hpp"
#include "pkdtree/global_plan.hpp"

using namespace pkdtree;

static int fail(const char* what, long long a, long long b) {
  std::fprintf(stderr, "FAIL %s: %lld vs %lld\n", what, a, b);
  return 1;
}

// Every invariant of one layout; returns 0 or the fail() code.
static int check_layout(i64 n, int P, int k, std::mt19937_64& rng) {
  using namespace global_plan;
  const Layout lay = make_layout(n, P, k);
  const int T = lay.T, LL = lay.LL;
  if (T != (1 << LL) || LL != top_levels_for(P, k) || LL > 6) return fail("layout LL", LL, T);
  if (int(lay.leaf_lo.size()) != P + 1 || lay.leaf_lo[0] != 0 || lay.leaf_lo[size_t(P)] != T) return fail("leaf_lo", P, T);
  // heap geometry: children split the parent as build_tree_rec does (kdtree_sequential.cpp:51-62)
  for (i64 h = 0; h + 1 < 2 * i64(T); ++h) {
    i64 lo, m, l1, n1, l2, n2;
    segment(n, h, &lo, &m);
    if (lo < 0 || m < 0 || (m > 0 && lo + m > n)) return fail("segment range", h, lo);  // empty: lo is moot
    if (2 * h + 2 < 2 * i64(T) - 1) {
      segment(n, 2 * h + 1, &l1, &n1);
      segment(n, 2 * h + 2, &l2, &n2);
      if (n1 != m / 2 || (m > 0 && (l1 != lo || l2 != lo + m / 2 + 1 || n2 != m - m / 2 - 1)))
        return fail("segment children", h, m);
    }
  }
  // every slot exactly once: the leaves' ranges and the non-empty top slots tile [0, n)
  std::vector<std::pair<i64, i64>> iv;
  for (int t = 0; t < T; ++t) {
    i64 lo, m;
    segment(n, T - 1 + t, &lo, &m);
    if (m != lay.leaf_n[size_t(t)] || (m > 0 && lo != lay.leaf_slot[size_t(t)])) return fail("leaf geometry", t, m);
    if (m > 0) iv.push_back({lay.leaf_slot[size_t(t)], m});
  }
  for (int h = 0; h + 1 < T; ++h)
    if (lay.top_slot[size_t(h)] >= 0) iv.push_back({lay.top_slot[size_t(h)], 1});
  std::sort(iv.begin(), iv.end());
  i64 pos = 0;
  for (const auto& e : iv) {
    if (e.first != pos) return fail("slot tiling", e.first, pos);
    pos += e.second;
  }
  if (pos != n) return fail("slot cover", pos, n);
  // shares: contiguous, in rank order, disjoint; the boundary top rows fill the gaps
  i64 covered = 0, boundary = 0;
  for (int h = 0; h + 1 < T; ++h)
    if (lay.top_slot[size_t(h)] >= 0 && lay.top_owner[size_t(h)] < 0) ++boundary;
  for (int r = 0; r < P; ++r) {
    covered += lay.share_n[size_t(r)];
    if (r > 0 && lay.share_lo[size_t(r)] < lay.share_lo[size_t(r - 1)] + lay.share_n[size_t(r - 1)])
      return fail("share overlap", r, lay.share_lo[size_t(r)]);
    for (int h = 0; h + 1 < T; ++h) {  // an owned top node lies inside its owner's share
      if (lay.top_owner[size_t(h)] != r || lay.top_slot[size_t(h)] < 0) continue;
      const i64 s0 = lay.top_slot[size_t(h)];
      if (s0 < lay.share_lo[size_t(r)] || s0 >= lay.share_lo[size_t(r)] + lay.share_n[size_t(r)])
        return fail("top owner", h, s0);
    }
    // blocks: complete subtrees tiling the share with the top rows between them
    std::vector<Block> bl;
    std::vector<i64> between;
    share_blocks(lay, r, &bl, &between);
    i64 at = 0;
    size_t bi = 0;
    for (const Block& b : bl) {
      i64 lo, m;
      segment(n, b.heap, &lo, &m);
      if (m != b.n || (m > 0 && lo != lay.share_lo[size_t(r)] + b.off)) return fail("block geometry", b.heap, b.n);
      if (b.n > 0 && b.off != at) return fail("block tiling", b.off, at);
      at = b.n > 0 ? b.off + b.n : at;
      if (bi < between.size() && b.n >= 0) {
        const i64 ts = lay.top_slot[size_t(between[bi])] - lay.share_lo[size_t(r)];
        if (ts == at) {
          ++at;
          ++bi;
        }
      }
    }
    if (bi != between.size() || at != lay.share_n[size_t(r)]) return fail("share tiling", at, lay.share_n[size_t(r)]);
  }
  if (covered + boundary != n) return fail("shares + boundary", covered + boundary, n);
  // exchange plan from random per-leaf counts: each leaf's rows spread over the P sources
  std::vector<i64> counts(size_t(P) * T * 4, 0);
  std::vector<i64> local(size_t(P), 0);
  for (int t = 0; t < T; ++t) {
    i64 left = lay.leaf_n[size_t(t)];
    for (int p = 0; p < P; ++p) {
      const i64 c = p + 1 == P ? left : (left > 0 ? i64(rng() % u64(left + 1)) : 0);
      counts[(size_t(p) * T + t) * 4] = c;
      left -= c;
      local[size_t(p)] += c;
    }
  }
  i64 base = 0;
  for (int p = 0; p < P; ++p) {
    for (int t = 0; t < T; ++t) {
      counts[(size_t(p) * T + t) * 4 + 2] = base;
      counts[(size_t(p) * T + t) * 4 + 3] = local[size_t(p)];
    }
    base += local[size_t(p)];
  }
  for (int me = 0; me < P; ++me) {
    Plan pl;
    if (make_plan(counts, lay, me, &pl) != 0) return fail("make_plan", me, 1);
    if (pl.leaf_start[size_t(T)] != local[size_t(me)]) return fail("pack extent", pl.leaf_start[size_t(T)], local[size_t(me)]);
    const int my_a = lay.leaf_lo[size_t(me)], mine = lay.leaf_lo[size_t(me) + 1] - my_a;
    for (int j = 0; j < lay.R; ++j) {
      i64 got = 0;
      for (int q = 0; q < P; ++q) {
        const i64 o = pl.send_off[size_t(j)][size_t(q)], c = pl.send_rows[size_t(j)][size_t(q)];
        if (o < 0 || c < 0 || o + c > pl.leaf_start[size_t(T)]) return fail("send range", o, c);
        got += pl.recv_rows[size_t(j)][size_t(q)];
      }
      const i64 want = j < mine ? lay.leaf_n[size_t(my_a + j)] : 0;
      if (got != want) return fail("recv rows", got, want);
    }
  }
  // a count matrix that over-fills a leaf raises on every rank, it never plans
  int t = 0;
  while (t < T && lay.leaf_n[size_t(t)] == 0) ++t;  // (n < T: every point may sit in the top nodes)
  if (t < T) {
    counts[size_t(t) * 4] += 1;
    bool threw = false;
    try {
      Plan pl;
      make_plan(counts, lay, 0, &pl);
    } catch (const std::runtime_error&) {
      threw = true;
    }
    if (!threw) return fail("overfilled leaf accepted", t, 0);
  }
  return 0;
}

static int planner_sweep() {
  std::mt19937_64 rng(20260517);
  int layouts = 0;
  for (int P = 1; P <= 64; ++P)
    for (int k = -1; k <= 6; ++k) {
      const i64 ns[] = {0, 1, i64(P) - 1, i64(P), (i64(1) << 20) + 3, (i64(1) << 32) - 1, i64(rng() % 100000)};
      for (i64 n : ns) {
        if (n < 0) continue;
        if (const int r = check_layout(n, P, k, rng)) return r;
        ++layouts;
      }
    }
  std::printf("planner sweep: %d layouts ok\n", layouts);
  return 0;
}

int main() {
  if (const int r = planner_sweep()) return r;
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
