// Geometry and exchange planning of the global decomposition (pkdtree/global_plan.hpp): host
// C++ only, shared by GlobalBuilder and the Python bindings, and sanitizer-tested on its own.
#include "pkdtree/global_plan.hpp"

#include <algorithm>
#include <stdexcept>
#include <string>

namespace pkdtree {

namespace global_plan {

void segment(i64 n_total, i64 h, i64* lo_out, i64* n_out) {
  int l = 0;
  while ((i64(1) << (l + 1)) - 1 <= h) ++l;  // level of heap node h
  const i64 j = h + 1 - (i64(1) << l);
  i64 lo = 0, m = n_total;
  for (int b = l - 1; b >= 0; --b) {
    if ((j >> b) & 1) {
      lo = lo + m / 2 + 1;
      m = std::max<i64>(0, m - m / 2 - 1);
    } else {
      m = m / 2;
    }
  }
  *lo_out = lo;
  *n_out = m;
}

i64 middle_cap(i64 n_total, int P, int level, int scale) {
  const i64 expect = n_total * (i64(1) << level) / (i64(kTopBins) * P) + 1;
  return std::min<i64>(std::max<i64>(2048, 3 * expect) * scale, std::max<i64>(n_total, 1));
}

int top_levels_for(int P, int pipeline_k) {
  if (P < 1 || P > 64) throw std::invalid_argument("global decomposition: 1 <= P <= 64 ranks");
  int L = 0;
  while ((1 << L) < P) ++L;
  const bool pow2 = (P & (P - 1)) == 0;
  // P not a power of two: T = 2^LL leaves split over P ranks as floor / ceil(T / P); 8x more
  // leaves than the next power of two keeps the busiest rank within ~3-9 % of the mean (P = 3:
  // 22 / 21 of 64 instead of 6 / 5 of 16), as far as the 6-level cap allows
  const int extra = pipeline_k >= 0 ? pipeline_k : (P == 2 ? 1 : (pow2 ? 0 : 3));
  return std::min(6, L + extra);
}

namespace {
// heap node between leaves a and a + 1 of the T leaves at the bottom of the top tree: their
// lowest common ancestor
i64 gap_node(int T, int a) {
  i64 x = T - 1 + a, y = T + a;
  while (x != y) {
    x = (x - 1) / 2;
    y = (y - 1) / 2;
  }
  return x;
}
}  // namespace

Layout make_layout(i64 n_total, int P, int pipeline_k) {
  Layout lay;
  lay.P = P;
  lay.LL = top_levels_for(P, pipeline_k);
  lay.T = 1 << lay.LL;
  const int T = lay.T;
  lay.leaf_lo.resize(size_t(P) + 1);
  lay.R = 0;
  for (int r = 0; r <= P; ++r) lay.leaf_lo[size_t(r)] = int(i64(r) * T / P);
  for (int r = 0; r < P; ++r) lay.R = std::max(lay.R, lay.leaf_lo[size_t(r) + 1] - lay.leaf_lo[size_t(r)]);
  lay.leaf_slot.assign(size_t(T), 0);
  lay.leaf_n.assign(size_t(T), 0);
  lay.top_slot.assign(size_t(T - 1), -1);
  lay.top_owner.assign(size_t(T - 1), -1);
  // in-order walk of the top tree's fringe: leaf 0, gap 0, leaf 1, ..., leaf T - 1
  i64 pos = 0;
  for (int t = 0; t < T; ++t) {
    i64 lo, n;
    segment(n_total, T - 1 + t, &lo, &n);
    if (n > 0 && lo != pos) throw std::logic_error("global layout: leaf slot mismatch");
    lay.leaf_slot[size_t(t)] = pos;
    lay.leaf_n[size_t(t)] = n;
    pos += n;
    if (t + 1 < T) {
      const i64 h = gap_node(T, t);
      segment(n_total, h, &lo, &n);
      if (n > 0) {
        if (lo + n / 2 != pos) throw std::logic_error("global layout: top slot mismatch");
        lay.top_slot[size_t(h)] = pos++;
      }
    }
  }
  if (pos != n_total) throw std::logic_error("global layout: slots do not cover the tree");
  lay.share_lo.assign(size_t(P), 0);
  lay.share_n.assign(size_t(P), 0);
  for (int r = 0; r < P; ++r) {
    const int a = lay.leaf_lo[size_t(r)], b = lay.leaf_lo[size_t(r) + 1];
    for (int t = a; t + 1 < b; ++t) lay.top_owner[size_t(gap_node(T, t))] = r;
    lay.share_lo[size_t(r)] = lay.leaf_slot[size_t(a)];
    lay.share_n[size_t(r)] = lay.leaf_slot[size_t(b - 1)] + lay.leaf_n[size_t(b - 1)] - lay.leaf_slot[size_t(a)];
  }
  return lay;
}

void share_blocks(const Layout& lay, int r, std::vector<Block>* blocks, std::vector<i64>* between_heap) {
  blocks->clear();
  between_heap->clear();
  const int a = lay.leaf_lo[size_t(r)], b = lay.leaf_lo[size_t(r) + 1];
  const i64 base = lay.share_lo[size_t(r)];
  for (int t = a; t < b;) {
    int s = 0;  // largest aligned power-of-two run of leaves starting at t inside [t, b)
    while (s < lay.LL && (t % (1 << (s + 1))) == 0 && t + (1 << (s + 1)) <= b) ++s;
    const int e = t + (1 << s);  // leaves [t, e)
    const i64 lo = lay.leaf_slot[size_t(t)];
    const i64 hi = lay.leaf_slot[size_t(e - 1)] + lay.leaf_n[size_t(e - 1)];
    blocks->push_back(Block{lo - base, hi - lo, lay.LL - s, ((i64(lay.T) + t) >> s) - 1});
    if (e < b) {
      const i64 h = gap_node(lay.T, e - 1);
      if (lay.top_slot[size_t(h)] >= 0) between_heap->push_back(h);
    }
    t = e;
  }
}

int make_plan(const std::vector<i64>& counts, const Layout& lay, int me, Plan* plan) {
  const int P = lay.P, T = lay.T, R = lay.R;
  if (counts.size() != size_t(P) * T * 4) throw std::invalid_argument("make_plan: counts must be [P][T][4]");
  auto at = [&](int src, int leaf, int f) { return counts[(size_t(src) * T + leaf) * 4 + f]; };
  i64 errs = 0;
  for (int src = 0; src < P; ++src)
    for (int t = 0; t < T; ++t) errs |= at(src, t, 1);
  if (errs & 1) return 1;  // a middle bucket overflowed its all-gather slot: retry larger
  if (errs & 2) throw std::runtime_error("global top levels: histogram totals disagree with the tree geometry");
  // every rank checks every leaf's total: a failure raises on all ranks together
  for (int t = 0; t < T; ++t) {
    i64 got = 0;
    for (int src = 0; src < P; ++src) got += at(src, t, 0);
    if (got != lay.leaf_n[size_t(t)])
      throw std::runtime_error("global exchange: top-level leaf " + std::to_string(t) + " would receive " +
                               std::to_string(got) + " points for a subtree of " +
                               std::to_string(lay.leaf_n[size_t(t)]));
  }
  plan->leaf_start.assign(size_t(T) + 1, 0);
  for (int t = 0; t < T; ++t) plan->leaf_start[size_t(t) + 1] = plan->leaf_start[size_t(t)] + at(me, t, 0);
  plan->send_rows.assign(size_t(R), std::vector<i64>(size_t(P), 0));
  plan->send_off.assign(size_t(R), std::vector<i64>(size_t(P), 0));
  plan->recv_rows.assign(size_t(R), std::vector<i64>(size_t(P), 0));
  const int my_a = lay.leaf_lo[size_t(me)], my_cnt = lay.leaf_lo[size_t(me) + 1] - my_a;
  for (int j = 0; j < R; ++j) {
    for (int q = 0; q < P; ++q) {
      const int t = lay.leaf_lo[size_t(q)] + j;
      if (t < lay.leaf_lo[size_t(q) + 1]) {
        plan->send_rows[size_t(j)][size_t(q)] = at(me, t, 0);
        plan->send_off[size_t(j)][size_t(q)] = plan->leaf_start[size_t(t)];
      }
    }
    if (j < my_cnt)
      for (int p = 0; p < P; ++p) plan->recv_rows[size_t(j)][size_t(p)] = at(p, my_a + j, 0);
  }
  plan->src_base.resize(size_t(P));
  plan->src_n.resize(size_t(P));
  for (int p = 0; p < P; ++p) {
    plan->src_base[size_t(p)] = at(p, 0, 2);
    plan->src_n[size_t(p)] = at(p, 0, 3);
  }
  return 0;
}

}  // namespace global_plan

}  // namespace pkdtree
