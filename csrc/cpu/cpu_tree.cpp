// CPU kd-tree builders and searches on the implicit in-order layout (see cpu_tree.hpp).
#include "pkdtree/cpu_tree.hpp"

#include <algorithm>
#include <thread>
#include <unordered_set>
#include <vector>

namespace pkdtree {

// ---------------------------------------------------------------------------------------------
// A parallel replica of libstdc++'s std::sort (introsort: __introsort_loop with median-of-three
// pivots and __unguarded_partition, a heapsort fallback at depth 2 floor(log2 n), ranges of at
// most 16 left for __final_insertion_sort). The reference's tree IS std::sort's output order --
// an unstable sort, so equal keys land wherever this exact algorithm puts them -- and the
// permutation depends only on the comparisons it makes, so the replica reproduces it bit for
// bit (tests/test_cpu_tree.py checks it against std::sort on duplicate-heavy inputs):
//   * after a partition, [first, cut) <= pivot <= [cut, last): the two sides are independent, so
//     they may run on two threads;
//   * the final insertion pass can never move an element across such a boundary (it only moves
//     an element left past STRICTLY greater ones), so it equals a stable insertion sort of each
//     leaf range, done as soon as the leaf exists.
// The critical path of one sort drops from n log n to ~2n comparisons (the top partitions).
namespace refsort {

constexpr std::ptrdiff_t kThreshold = 16;      // libstdc++ _S_threshold
constexpr std::ptrdiff_t kSpawnMin = 1 << 15;  // smallest side worth its own thread

template <class C>
inline void move_median_to_first(u32* r, u32* a, u32* b, u32* c, const C& comp) {
  if (comp(*a, *b)) {
    if (comp(*b, *c)) std::iter_swap(r, b);
    else if (comp(*a, *c)) std::iter_swap(r, c);
    else std::iter_swap(r, a);
  } else if (comp(*a, *c)) {
    std::iter_swap(r, a);
  } else if (comp(*b, *c)) {
    std::iter_swap(r, c);
  } else {
    std::iter_swap(r, b);
  }
}

template <class C>
inline u32* unguarded_partition(u32* first, u32* last, u32* pivot, const C& comp) {
  while (true) {
    while (comp(*first, *pivot)) ++first;
    --last;
    while (comp(*pivot, *last)) --last;
    if (!(first < last)) return first;
    std::iter_swap(first, last);
    ++first;
  }
}

template <class C>
inline void insertion(u32* first, u32* last, const C& comp) {  // stable: = the final pass on this leaf
  for (u32* i = first + (first != last ? 1 : 0); i < last; ++i) {
    const u32 v = *i;
    u32* j = i;
    while (j > first && comp(v, *(j - 1))) {
      *j = *(j - 1);
      --j;
    }
    *j = v;
  }
}

template <class C>
void loop(u32* first, u32* last, long depth, const C& comp, int spawn) {
  while (last - first > kThreshold) {
    if (depth == 0) {  // libstdc++: __partial_sort(first, last, last) -- heap select + sort_heap
      std::partial_sort(first, last, last, comp);
      return;
    }
    --depth;
    u32* mid = first + (last - first) / 2;
    move_median_to_first(first, first + 1, mid, last - 1, comp);
    u32* cut = unguarded_partition(first + 1, last, first, comp);
    if (spawn > 0 && last - cut >= kSpawnMin && cut - first >= kSpawnMin) {
      std::thread t([=, &comp] { loop(cut, last, depth, comp, spawn - 1); });
      loop(first, cut, depth, comp, spawn - 1);
      t.join();
      return;
    }
    loop(cut, last, depth, comp, 0);
    last = cut;
  }
  insertion(first, last, comp);
}

template <class C>
void sort(u32* first, u32* last, const C& comp, int spawn) {
  if (last - first < 2) return;
  const long n = long(last - first);
  loop(first, last, 2L * long(63 - __builtin_clzl(static_cast<unsigned long>(n))), comp, spawn);
}

}  // namespace refsort

void std_sort_replica(const float* keys, u32* idx, i64 n, int threads) {
  int spawn = 0;
  while ((1 << spawn) < threads && spawn < 8) ++spawn;
  refsort::sort(idx, idx + n, [keys](u32 a, u32 b) { return keys[a] < keys[b]; }, spawn);
}

namespace {

struct ExactCtx {
  const float* pts;
  const u32* ids;
  int dim;
  int depth0;
  u32* perm;
};

inline u64 ckey(const ExactCtx& c, u32 row, int axis) {
  const u32 id = c.ids ? c.ids[row] : row;
  return composite_key(c.pts[size_t(row) * size_t(c.dim) + size_t(axis)], id);
}

void exact_rec(const ExactCtx& c, i64 lo, i64 n, int depth, int spawn_levels) {
  while (n > 1) {
    const int axis = (c.depth0 + depth) % c.dim;
    u32* b = c.perm + lo;
    std::nth_element(b, b + n / 2, b + n, [&](u32 x, u32 y) { return ckey(c, x, axis) < ckey(c, y, axis); });
    const i64 nl = left_n(n), nr = right_n(n);
    if (spawn_levels > 0) {
      std::thread t([&c, lo, nl, depth, spawn_levels] { exact_rec(c, lo, nl, depth + 1, spawn_levels - 1); });
      exact_rec(c, lo + nl + 1, nr, depth + 1, spawn_levels - 1);
      t.join();
      return;
    }
    exact_rec(c, lo, nl, depth + 1, 0);
    lo = lo + nl + 1;
    n = nr;
    ++depth;
  }
}

void reference_rec(const float* pts, int dim, int depth0, u32* perm, i64 lo, i64 n, int depth, int spawn_levels) {
  // Mirrors build_tree_rec (kdtree_sequential.cpp:30-66) on an index array: the sort
  // range deliberately excludes the last element of the segment. After a segment's sort its two
  // children are disjoint ranges of perm, so they may run on two threads: std::sort is
  // deterministic for a given input order, so the tree is the same for any thread count (the
  // critical path drops from the whole O(N log^2 N) build to ~2 N log N: one sort per level).
  while (n > 1) {
    const int axis = (depth0 + depth) % dim;
    // (the replica of std::sort: the same permutation; with threads to spare, the sort of a large
    // segment splits its own partitions over threads too)
    refsort::sort(perm + lo, perm + lo + (n - 1), [&](u32 a, u32 b) {
      return pts[size_t(a) * size_t(dim) + size_t(axis)] < pts[size_t(b) * size_t(dim) + size_t(axis)];
    }, spawn_levels);
    const i64 nl = left_n(n), nr = right_n(n);
    if (spawn_levels > 0 && n >= 4096) {
      std::thread t([=] { reference_rec(pts, dim, depth0, perm, lo, nl, depth + 1, spawn_levels - 1); });
      reference_rec(pts, dim, depth0, perm, lo + nl + 1, nr, depth + 1, spawn_levels - 1);
      t.join();
      return;
    }
    reference_rec(pts, dim, depth0, perm, lo, nl, depth + 1, 0);
    lo = lo + nl + 1;
    n = nr;
    ++depth;
  }
}

struct SearchCtx {
  const float* P;
  int dim;
  int depth0;
  const float* q;
};

inline float d2_at(const SearchCtx& s, i64 slot) { return sq_dist(s.P + size_t(slot) * size_t(s.dim), s.q, s.dim); }

// Returns the best slot of this subtree given the incoming best (never -1 unless n <= 0).
i64 nearest_rec(const SearchCtx& s, i64 lo, i64 n, int depth, i64 best, float best_dist) {
  if (n <= 0) return -1;
  const int axis = (s.depth0 + depth) % s.dim;
  const i64 m = median_pos(lo, n);
  const float* p = s.P + size_t(m) * size_t(s.dim);
  i64 best_local = best;
  float bdl = best_dist;
  const float d_e = sq_dist(p, s.q, s.dim);
  const float d_axis = s.q[axis] - p[axis];
  const float d_axis2 = d_axis * d_axis;
  if (d_e < bdl) { best_local = m; bdl = d_e; }
  const i64 l_lo = lo, l_n = left_n(n), r_lo = m + 1, r_n = right_n(n);
  const bool go_left = d_axis < 0;
  i64 further = go_left ? nearest_rec(s, l_lo, l_n, depth + 1, best_local, bdl)
                        : nearest_rec(s, r_lo, r_n, depth + 1, best_local, bdl);
  if (further >= 0) {
    const float df = d2_at(s, further);
    if (df < bdl) { bdl = df; best_local = further; }
  }
  if (d_axis2 < bdl) {
    further = go_left ? nearest_rec(s, r_lo, r_n, depth + 1, best_local, bdl)
                      : nearest_rec(s, l_lo, l_n, depth + 1, best_local, bdl);
    if (further >= 0) {
      const float df = d2_at(s, further);
      if (df < bdl) best_local = further;
    }
  }
  return best_local;
}

struct MinMax {
  u64 mn, mx;
};

// Returns per-axis (min, max) composite keys of the subtree; counts violations.
void check_rec(const float* P, const u32* ids, int dim, int depth0, i64 lo, i64 n, int depth,
               MinMax* out, std::vector<std::vector<MinMax>>& scratch, i64& bad) {
  for (int a = 0; a < dim; ++a) out[a] = {~u64(0), 0};
  if (n <= 0) return;
  if (scratch.size() < size_t(2 * (depth + 1))) scratch.resize(size_t(2 * (depth + 1)));
  auto& L = scratch[size_t(2 * depth)];
  auto& R = scratch[size_t(2 * depth + 1)];
  L.assign(size_t(dim), {~u64(0), 0});
  R.assign(size_t(dim), {~u64(0), 0});
  const i64 m = median_pos(lo, n);
  check_rec(P, ids, dim, depth0, lo, left_n(n), depth + 1, L.data(), scratch, bad);
  check_rec(P, ids, dim, depth0, m + 1, right_n(n), depth + 1, R.data(), scratch, bad);
  // scratch may have been resized by the recursion: re-fetch
  auto& L2 = scratch[size_t(2 * depth)];
  auto& R2 = scratch[size_t(2 * depth + 1)];
  const int axis = (depth0 + depth) % dim;
  const u64 km = composite_key(P[size_t(m) * size_t(dim) + size_t(axis)], ids[m]);
  if (left_n(n) > 0 && !(L2[size_t(axis)].mx < km)) ++bad;
  if (right_n(n) > 0 && !(R2[size_t(axis)].mn > km)) ++bad;
  for (int a = 0; a < dim; ++a) {
    const u64 k = composite_key(P[size_t(m) * size_t(dim) + size_t(a)], ids[m]);
    out[a].mn = std::min({L2[size_t(a)].mn, R2[size_t(a)].mn, k});
    out[a].mx = std::max({L2[size_t(a)].mx, R2[size_t(a)].mx, k});
  }
}

}  // namespace

void build_exact_cpu(const float* pts, const u32* ids, i64 n, int dim, int depth0, u32* perm, int threads) {
  for (i64 i = 0; i < n; ++i) perm[i] = u32(i);
  int spawn = 0;
  while ((1 << spawn) < threads && spawn < 6) ++spawn;
  ExactCtx c{pts, ids, dim, depth0, perm};
  exact_rec(c, 0, n, 0, spawn);
}

void build_reference_cpu(const float* pts, i64 n, int dim, u32* perm, int threads, int depth0) {
  for (i64 i = 0; i < n; ++i) perm[i] = u32(i);
  int spawn = 0;
  while ((1 << spawn) < threads && spawn < 8) ++spawn;
  reference_rec(pts, dim, depth0, perm, 0, n, 0, spawn);
}

namespace {

// Segment key of the implicit tree: (depth, start slot).
inline u64 seg_key(int depth, i64 lo) { return (u64(u32(depth)) << 40) | u64(lo); }

struct RepairCtx {
  const float* pts;
  int dim, depth0;
  const u32* gpu;  // the GPU tree's slot -> row
  u32* order;      // working input order of every CPU segment (the reference's array)
  u32* out;        // result: slot -> row
  const std::unordered_set<u64>* closure;
  const std::unordered_set<u64>* tied;
  std::vector<std::vector<std::pair<i64, i64>>>* cpu_ranges;  // per spawned task: slot ranges it decided
};

void repair_rec(const RepairCtx& c, i64 lo, i64 n, int depth, int spawn, int task) {
  while (n > 0) {
    const u64 key = seg_key(depth, lo);
    const bool is_tied = c.tied->count(key) != 0;
    if (!is_tied && c.closure->count(key) == 0) {  // no deciding tie at or below: the GPU's slots stand
      std::copy(c.gpu + lo, c.gpu + lo + n, c.out + lo);
      return;
    }
    if (is_tied) {  // std::sort decides here: the whole subtree from this segment's exact input order
      reference_rec(c.pts, c.dim, c.depth0, c.order, lo, n, depth, spawn);
      std::copy(c.order + lo, c.order + lo + n, c.out + lo);
      (*c.cpu_ranges)[size_t(task)].push_back({lo, n});
      return;
    }
    // an ancestor of a tied segment: its sort fixes the exact order its children start from
    const int axis = (c.depth0 + depth) % c.dim;
    refsort::sort(c.order + lo, c.order + lo + (n - 1), [&](u32 a, u32 b) {
      return c.pts[size_t(a) * size_t(c.dim) + size_t(axis)] < c.pts[size_t(b) * size_t(c.dim) + size_t(axis)];
    }, spawn);
    const i64 nl = left_n(n), nr = right_n(n);
    c.out[lo + nl] = c.order[lo + nl];
    (*c.cpu_ranges)[size_t(task)].push_back({lo + nl, 1});
    if (spawn > 0 && nl >= 4096) {
      const int t2 = task + (1 << (spawn - 1));
      std::thread t([&c, lo, nl, depth, spawn, t2] { repair_rec(c, lo, nl, depth + 1, spawn - 1, t2); });
      repair_rec(c, lo + nl + 1, nr, depth + 1, spawn - 1, task);
      t.join();
      return;
    }
    repair_rec(c, lo, nl, depth + 1, 0, task);
    lo = lo + nl + 1;
    n = nr;
    ++depth;
  }
}

}  // namespace

std::vector<std::pair<i64, i64>> reference_repair(const float* pts, i64 n, int dim, int depth0, const u32* gpu_perm,
                                                  const u32* tied_slots, size_t ntied, u32* perm, int threads) {
  std::unordered_set<u64> closure, tied;
  for (size_t k = 0; k < ntied; ++k) {  // the path from the root to each tied segment (by its median slot)
    const i64 s = i64(tied_slots[k]);
    i64 lo = 0, m = n;
    for (int d = 0; m > 0; ++d) {
      const i64 nl = left_n(m);
      if (s == lo + nl) {
        tied.insert(seg_key(d, lo));
        break;
      }
      closure.insert(seg_key(d, lo));
      if (s < lo + nl) {
        m = nl;
      } else {
        lo = lo + nl + 1;
        m = right_n(m);
      }
    }
  }
  std::vector<u32> order(static_cast<size_t>(std::max<i64>(n, 1)));
  for (i64 i = 0; i < n; ++i) order[size_t(i)] = u32(i);
  int spawn = 0;
  while ((1 << spawn) < threads && spawn < 8) ++spawn;
  std::vector<std::vector<std::pair<i64, i64>>> ranges(size_t(1) << spawn);
  RepairCtx c{pts, dim, depth0, gpu_perm, order.data(), perm, &closure, &tied, &ranges};
  repair_rec(c, 0, n, 0, spawn, 0);
  std::vector<std::pair<i64, i64>> all;
  for (auto& r : ranges) all.insert(all.end(), r.begin(), r.end());
  std::sort(all.begin(), all.end());
  return all;
}

int default_cpu_threads() {
  const unsigned hw = std::thread::hardware_concurrency();
  return int(std::max(1u, std::min(hw, 64u)));
}

void gather_rows(const float* pts, const u32* ids, const u32* perm, i64 n, int dim, float* tree_pts, u32* tree_ids) {
  for (i64 k = 0; k < n; ++k) {
    const u32 r = perm[k];
    std::copy(pts + size_t(r) * size_t(dim), pts + size_t(r + 1) * size_t(dim), tree_pts + size_t(k) * size_t(dim));
    if (tree_ids) tree_ids[k] = ids ? ids[r] : r;
  }
}

NNResult nn_search_cpu(const float* tree_pts, i64 n, int dim, int depth0, const float* q) {
  if (n <= 0) return {-1, 0.0f};
  SearchCtx s{tree_pts, dim, depth0, q};
  const i64 root = median_pos(0, n);
  const i64 best = nearest_rec(s, 0, n, 0, root, d2_at(s, root));
  return {best, d2_at(s, best)};
}

NNResult nn_brute_cpu(const float* pts, i64 n, int dim, const float* q) {
  NNResult r{-1, 0.0f};
  for (i64 i = 0; i < n; ++i) {
    const float d = sq_dist(pts + size_t(i) * size_t(dim), q, dim);
    if (r.slot < 0 || d < r.d2) r = {i, d};
  }
  return r;
}

i64 count_invariant_violations(const float* tree_pts, const u32* tree_ids, i64 n, int dim, int depth0) {
  std::vector<MinMax> root(static_cast<size_t>(dim));
  std::vector<std::vector<MinMax>> scratch(size_t(2 * (tree_height(n) + 2)));
  i64 bad = 0;
  check_rec(tree_pts, tree_ids, dim, depth0, 0, n, 0, root.data(), scratch, bad);
  return bad;
}

// ---- tree utilities ----------------------------------------------------------------------
void print_point(std::ostream& os, i64 id, const float* coords, int dim) {
  constexpr int kMaxPrintDimension = 5;  // Node.hpp:5
  os << "Point(ID=" << id << ", dimension=" << dim << ", coordinates=[";
  for (int d = 0; d < dim - 1; ++d) {
    os << coords[d] << ", ";
    if (d >= kMaxPrintDimension - 1) {
      os << ", ..., ";
      break;
    }
  }
  if (dim > 0) os << coords[dim - 1];
  os << "])";
}

namespace {
void print_tree_rec(std::ostream& os, const float* tree_pts, const u32* tree_ids, int dim, i64 lo, i64 n, int depth) {
  if (n <= 0) return;
  const i64 m = lo + n / 2;
  for (int d = 0; d < depth; ++d) os << "\t";
  os << "NODE(@depth=" << depth << "): ";
  print_point(os, i64(tree_ids[m]), tree_pts + size_t(m) * size_t(dim), dim);
  os << "\n";
  print_tree_rec(os, tree_pts, tree_ids, dim, lo, n / 2, depth + 1);
  print_tree_rec(os, tree_pts, tree_ids, dim, m + 1, n - n / 2 - 1, depth + 1);
}
}  // namespace

void print_tree(std::ostream& os, const float* tree_pts, const u32* tree_ids, i64 n, int dim) {
  print_tree_rec(os, tree_pts, tree_ids, dim, 0, n, 0);
}

void print_head_and_leaves(std::ostream& os, const float* tree_pts, const u32* tree_ids, i64 n, int dim) {
  if (n <= 0) return;
  auto pt = [&](i64 k) { print_point(os, i64(tree_ids[k]), tree_pts + size_t(k) * size_t(dim), dim); };
  const i64 head = n / 2;
  i64 lo = 0, m = n;  // left-most leaf: keep the left child while it exists
  while (m / 2 > 0) m = m / 2;
  const i64 left = lo + m / 2;
  lo = 0;
  m = n;  // right-most leaf: keep the right child while it exists
  while (m - m / 2 - 1 > 0) {
    lo = lo + m / 2 + 1;
    m = m - m / 2 - 1;
  }
  const i64 right = lo + m / 2;
  os << "\nHead: ";
  pt(head);
  os << "\nLeft Leaf: ";
  pt(left);
  os << "\nRight Leaf: ";
  pt(right);
  os << "\n\n";
}

}  // namespace pkdtree
