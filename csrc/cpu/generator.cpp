// Reference-compatible problem generator with O(log n) jump-ahead.
//
// The reference (kdtree_mpi.cpp:24,32) reaches a rank's slice with mt19937::discard,
// which walks the whole stream on every rank. Here the slice start is reached by
// evaluating x^J mod phi(x) at the one-step transition (phi = characteristic polynomial
// of MT19937, recovered once by Berlekamp-Massey from 2*19937 output bits), and long
// slices are split over threads with the same jump.
#include "pkdtree/generator.hpp"

#include <algorithm>
#include <mutex>
#include <thread>
#include <vector>

namespace pkdtree {

void MT19937::seed(uint32_t s) {
  mt[0] = s;
  for (int i = 1; i < N; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + uint32_t(i);
  idx = N;
}

void MT19937::twist() {
  for (int i = 0; i < N; ++i) {
    uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % N] & 0x7fffffffu);
    mt[i] = mt[(i + M) % N] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }
  idx = 0;
}

void MT19937::discard(uint64_t n) {
  while (n > 0) {
    if (idx >= N) twist();
    uint64_t step = std::min<uint64_t>(n, uint64_t(N - idx));
    idx += int(step);
    n -= step;
  }
}

namespace {

// ---- GF(2) polynomials, bit i = coefficient of x^i --------------------------------
using Poly = std::vector<uint64_t>;

inline bool pbit(const Poly& p, size_t i) { return (i / 64 < p.size()) && ((p[i / 64] >> (i % 64)) & 1u); }
inline void pset(Poly& p, size_t i) {
  if (i / 64 >= p.size()) p.resize(i / 64 + 1, 0);
  p[i / 64] ^= (uint64_t(1) << (i % 64));
}
int pdeg(const Poly& p) {
  for (size_t w = p.size(); w-- > 0;)
    if (p[w]) return int(w * 64 + 63 - __builtin_clzll(p[w]));
  return -1;
}
// dst ^= src << shift
void pxor_shift(Poly& dst, const Poly& src, size_t shift) {
  size_t ws = shift / 64, bs = shift % 64;
  size_t need = src.size() + ws + 1;
  if (dst.size() < need) dst.resize(need, 0);
  for (size_t i = 0; i < src.size(); ++i) {
    uint64_t v = src[i];
    if (!v) continue;
    dst[i + ws] ^= v << bs;
    if (bs) dst[i + ws + 1] ^= v >> (64 - bs);
  }
}
void pmod(Poly& a, const Poly& m, int dm) {
  for (int d = pdeg(a); d >= dm; d = pdeg(a)) {
    // clear the top bit, and every lower set bit down to dm, one shift each
    pxor_shift(a, m, size_t(d - dm));
  }
  a.resize(size_t(dm) / 64 + 1);
}
Poly psquare(const Poly& a) {
  Poly r(a.size() * 2 + 1, 0);
  for (size_t i = 0; i < a.size(); ++i) {
    uint64_t v = a[i];
    uint64_t lo = 0, hi = 0;
    for (int b = 0; b < 32; ++b) {
      lo |= ((v >> b) & 1u) << (2 * b);
      hi |= ((v >> (b + 32)) & 1u) << (2 * b);
    }
    r[2 * i] = lo;
    r[2 * i + 1] = hi;
  }
  return r;
}

// Berlekamp-Massey on the LSB sequence of MT19937(5489) -> characteristic polynomial.
// The discrepancy is evaluated 64 coefficients at a time against a bit-reversed copy of
// the sequence, so the whole run is O(n^2 / 64).
Poly compute_charpoly() {
  const int L_expected = 19937;
  const size_t n = size_t(2) * L_expected + 64;
  const size_t nw = n / 64 + 2;
  std::vector<uint64_t> rev(nw + 8, 0);  // rev bit t = s[n-1-t]
  std::vector<uint8_t> s(n);
  MT19937 g(5489u);
  for (size_t i = 0; i < n; ++i) {
    s[i] = uint8_t(g.next() & 1u);
    const size_t t = n - 1 - i;
    if (s[i]) rev[t / 64] |= uint64_t(1) << (t % 64);
  }
  auto rev64 = [&](size_t off) -> uint64_t {  // 64 bits of rev starting at bit off
    const size_t w = off / 64, b = off % 64;
    uint64_t lo = rev[w] >> b;
    if (b) lo |= rev[w + 1] << (64 - b);
    return lo;
  };
  Poly C(1, 1), B(1, 1);
  int L = 0;
  size_t m = 1;
  for (size_t i = 0; i < n; ++i) {
    // d = sum_{j=0..L} C_j s[i-j]; s[i-j] = rev[n-1-i+j]
    const size_t base = n - 1 - i;
    const size_t words = size_t(L) / 64 + 1;
    uint64_t acc = 0;
    for (size_t w = 0; w < words && w < C.size(); ++w) {
      uint64_t c = C[w];
      if (w == words - 1 && (L % 64) != 63) c &= (uint64_t(2) << (L % 64)) - 1;
      acc ^= c & rev64(base + 64 * w);
    }
    const uint64_t d = uint64_t(__builtin_parityll(acc));
    if (!d) { ++m; continue; }
    if (2 * size_t(L) <= i) {
      Poly T = C;
      pxor_shift(C, B, m);
      L = int(i + 1) - L;
      B = T;
      m = 1;
    } else {
      pxor_shift(C, B, m);
      ++m;
    }
  }
  // phi(x) = x^L C(1/x)
  Poly phi;
  for (int j = 0; j <= L; ++j)
    if (pbit(C, size_t(j))) pset(phi, size_t(L - j));
  return phi;
}

const Poly& charpoly() {
  static Poly phi;
  static std::once_flag once;
  std::call_once(once, [] { phi = compute_charpoly(); });
  return phi;
}

// x^J mod phi
Poly x_pow_mod(uint64_t J, const Poly& phi) {
  const int dm = pdeg(phi);
  Poly r(1, 1);
  int top = 63;
  while (top >= 0 && !((J >> top) & 1u)) --top;
  for (int b = top; b >= 0; --b) {
    r = psquare(r);
    pmod(r, phi, dm);
    if ((J >> b) & 1u) {
      Poly t;
      pxor_shift(t, r, 1);
      r.swap(t);
      pmod(r, phi, dm);
    }
  }
  return r;
}

// Circular-buffer state: logical word k = st[(i + k) % 624]; one step writes one word.
struct Lin {
  uint32_t st[MT19937::N];
  int i;
  void step() {
    const int N = MT19937::N, M = MT19937::M;
    uint32_t y = (st[i] & 0x80000000u) | (st[(i + 1) % N] & 0x7fffffffu);
    st[i] = st[(i + M) % N] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    i = (i + 1) % N;
  }
  void add(const Lin& o) {
    const int N = MT19937::N;
    for (int k = 0; k < N; ++k) st[(i + k) % N] ^= o.st[(o.i + k) % N];
  }
};

}  // namespace

void MT19937::jump(uint64_t n) {
  if (n < 4 * uint64_t(N)) { discard(n); return; }
  if (idx < N) {  // finish the current block: then mt[] is exactly the Lin state at i=0
    const uint64_t head = uint64_t(N - idx);
    discard(head);
    n -= head;
  }
  Lin s;
  std::copy(mt, mt + N, s.st);
  s.i = 0;
  const Poly& phi = charpoly();
  const Poly q = x_pow_mod(n, phi);
  Lin acc;
  std::fill(acc.st, acc.st + N, 0u);
  acc.i = 0;
  for (int k = pdeg(q); k >= 0; --k) {  // Horner: acc = q(f) s = f^n s on every output
    acc.step();
    if (pbit(q, size_t(k))) acc.add(s);
  }
  // idx == N means: the next twist rewrites logical word 0 from words 0, 1 and M.
  for (int k = 0; k < N; ++k) mt[k] = acc.st[(acc.i + k) % N];
  idx = N;
}

// ---- device generator host side -------------------------------------------------------
DevGenPlan devgen_plan(uint64_t total) {
  DevGenPlan p;
  p.total = total;
  if (total == 0) return p;
  // >= 64 twists per chunk so the jump rounds stay small next to generation; at most
  // 2048 chunks (8 workgroups per CU on 256 CUs).
  const uint64_t min_chunk = uint64_t(kMtWords) * 64;
  uint64_t C = std::min<uint64_t>(2048, std::max<uint64_t>(1, total / min_chunk));
  p.S = (total + C - 1) / C;
  p.C = int((total + p.S - 1) / p.S);
  while ((1 << p.R) < p.C) ++p.R;
  return p;
}

void mt_window_after(uint32_t seed, uint64_t n, uint32_t* out) {
  MT19937 g(seed);  // idx == N: mt is the window after 0 draws
  if (n >= 4 * uint64_t(MT19937::N)) {
    g.jump(n);  // a fresh generator takes the Horner path: mt = window after n, idx == N
    std::copy(g.mt, g.mt + MT19937::N, out);
    return;
  }
  Lin s;
  std::copy(g.mt, g.mt + MT19937::N, s.st);
  s.i = 0;
  for (uint64_t k = 0; k < n; ++k) s.step();
  for (int k = 0; k < MT19937::N; ++k) out[k] = s.st[(s.i + k) % MT19937::N];
}

std::vector<uint32_t> mt_jump_polys(uint64_t S, int R) {
  static std::mutex mu;
  static std::vector<std::pair<std::pair<uint64_t, int>, std::vector<uint32_t>>> cache;
  std::lock_guard<std::mutex> lock(mu);
  for (auto& e : cache)
    if (e.first.first == S && e.first.second == R) return e.second;
  const Poly& phi = charpoly();
  const int dm = pdeg(phi);
  std::vector<uint32_t> out(size_t(R) * kMtWords, 0u);
  Poly q = x_pow_mod(S, phi);
  for (int r = 0; r < R; ++r) {
    if (r > 0) {
      q = psquare(q);
      pmod(q, phi, dm);
    }
    for (int k = 0; k <= pdeg(q); ++k)
      if (pbit(q, size_t(k))) out[size_t(r) * kMtWords + size_t(k / 32)] |= 1u << (k % 32);
  }
  if (cache.size() > 8) cache.erase(cache.begin());
  cache.push_back({{S, R}, out});
  return out;
}

namespace {
// In-place twist of a 624-word block: the next 624 untempered words.
void twist_block(uint32_t* mt) {
  MT19937 g;
  std::copy(mt, mt + MT19937::N, g.mt);
  g.twist();
  std::copy(g.mt, g.mt + MT19937::N, mt);
}
}  // namespace

void devgen_emulate(uint32_t seed, uint64_t first_draw, uint64_t total, float* out) {
  const DevGenPlan p = devgen_plan(total);
  if (p.C == 0) return;
  const int N = MT19937::N;
  std::vector<uint32_t> states(size_t(p.C) * N);
  mt_window_after(seed, first_draw, states.data());
  const std::vector<uint32_t> polys = mt_jump_polys(p.S, p.R);
  std::vector<uint32_t> ext(kMtExtWords);
  for (int r = 0; r < p.R; ++r) {
    const int src = 1 << r;
    for (int i = 0; i < src && src + i < p.C; ++i) {
      // extension of state i: the window, then 32 twisted blocks
      std::copy(&states[size_t(i) * N], &states[size_t(i) * N] + N, ext.begin());
      for (int b = 1; b < kMtExtWords / N; ++b) {
        std::copy(ext.begin() + (b - 1) * N, ext.begin() + b * N, ext.begin() + b * N);
        twist_block(&ext[size_t(b) * N]);
      }
      uint32_t* dst = &states[size_t(src + i) * N];
      std::fill(dst, dst + N, 0u);
      const uint32_t* q = &polys[size_t(r) * kMtWords];
      for (int wi = 0; wi < kMtWords; ++wi)
        for (uint32_t word = q[wi]; word; word &= word - 1) {
          const int k = wi * 32 + __builtin_ctz(word);
          for (int m = 0; m < N; ++m) dst[m] ^= ext[size_t(k + m)];
        }
    }
  }
  for (int c = 0; c < p.C; ++c) {
    uint32_t mt[624];
    std::copy(&states[size_t(c) * N], &states[size_t(c) * N] + N, mt);
    const uint64_t b = uint64_t(c) * p.S, e = std::min(p.total, b + p.S);
    for (uint64_t pos = b; pos < e; pos += N) {
      twist_block(mt);
      for (int j = 0; j < N && pos + uint64_t(j) < e; ++j) {
        uint32_t y = mt[j];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        out[pos + uint64_t(j)] = u32_to_uniform(y);
      }
    }
  }
}

std::vector<float> generate_problem(int seed, int dim, int64_t rows) {
  std::vector<float> x(size_t(rows) * size_t(dim));
  generate_rows(seed, dim, 0, rows, x.data(), 0);
  return x;
}

void generate_rows(int seed, int dim, int64_t first, int64_t rows, float* out, int threads) {
  const uint64_t per_row = uint64_t(dim);
  const uint64_t total = uint64_t(rows) * per_row;
  if (threads <= 0) threads = int(std::min<unsigned>(8u, std::max(1u, std::thread::hardware_concurrency())));
  // Threads only pay off on long slices (each jump costs a few ms).
  if (total < (uint64_t(1) << 24)) threads = 1;
  MT19937 base{static_cast<uint32_t>(seed)};
  base.jump(uint64_t(first) * per_row);
  if (threads == 1) {
    for (uint64_t k = 0; k < total; ++k) out[k] = u32_to_uniform(base.next());
    return;
  }
  const uint64_t chunk = (total + uint64_t(threads) - 1) / uint64_t(threads);
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) {
    const uint64_t b = uint64_t(t) * chunk;
    const uint64_t e = std::min(total, b + chunk);
    if (b >= e) break;
    pool.emplace_back([&base, out, b, e] {
      MT19937 g = base;
      g.jump(b);
      for (uint64_t k = b; k < e; ++k) out[k] = u32_to_uniform(g.next());
    });
  }
  for (auto& th : pool) th.join();
}

}  // namespace pkdtree
