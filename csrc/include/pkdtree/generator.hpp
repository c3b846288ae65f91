// Problem generator bit-compatible with the reference data contract:
//   std::mt19937(seed) + std::uniform_real_distribution<float>(-100, 100), row-major
//   (N+Q) x dim, last Q rows are the queries  (Utility.cpp:6-18, kdtree_sequential.cpp:157).
// The per-rank slice generator reproduces kdtree_mpi.cpp:19-41 (rows [first, first+n) of the
// same stream) but uses an O(log) GF(2) jump-ahead instead of discard().
#pragma once
#include <cstdint>
#include <vector>

namespace pkdtree {

// Own MT19937 (same recurrence and tempering as std::mt19937) so the state can be
// jumped and shipped to the GPU generator.
struct MT19937 {
  static constexpr int N = 624;
  static constexpr int M = 397;
  uint32_t mt[N];
  int idx;

  explicit MT19937(uint32_t seed = 5489u) { this->seed(seed); }
  void seed(uint32_t s);
  void twist();
  uint32_t next() {
    if (idx >= N) twist();
    uint32_t y = mt[idx++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  // Advance by n raw draws, like std::mt19937::discard (O(n) twisting).
  void discard(uint64_t n);
  // Advance by n raw draws in O(19937^2/64 * log n) via the characteristic polynomial.
  void jump(uint64_t n);
};

// libstdc++ generate_canonical<float,24> + uniform_real_distribution<float>(a, b):
//   u = float(x) / 2^32 (clamped below 1), result = u * (b - a) + a, no FMA.
inline float u32_to_uniform(uint32_t x, float a = -100.0f, float b = 100.0f) {
  float u = float(x) / 4294967296.0f;
  if (u >= 1.0f) u = 0.99999994f;  // std::nextafter(1.0f, 0.0f)
  volatile float span = b - a;      // keep mul and add separately rounded
  float t = u * span;
  return t + a;
}

// ---- device generator support (csrc/gpu/generator.hip) ---------------------------------
// The stream [first_draw, first_draw + total) is cut into C chunks of S draws. Chunk c
// starts from the MT state after first_draw + c*S draws. Chunk 0's state is computed on the
// host; the others come from log2(C) doubling rounds on the device: in round r, chunk
// 2^r + i is chunk i advanced by S*2^r draws, i.e. q_r(f) applied to chunk i's state with
// q_r = x^(S*2^r) mod phi. Applying q(f) to a state s is a GF(2) correlation with the
// state's own extension w (the untempered word sequence starting at s):
//   (q(f) s)[m] = XOR over k with q_k = 1 of w[k + m],   m = 0..623.
struct DevGenPlan {
  uint64_t total = 0;  // draws
  uint64_t S = 0;      // draws per chunk
  int C = 0;           // chunks
  int R = 0;           // doubling rounds (2^R >= C)
};
constexpr int kMtWords = 624;
constexpr int kMtExtWords = 624 * 33;  // >= 19937 + 623: extension window per source state
DevGenPlan devgen_plan(uint64_t total);
// Untempered window after n draws from seed (624 words, logical order; next twist outputs
// draw n). O(log n) via jump-ahead.
void mt_window_after(uint32_t seed, uint64_t n, uint32_t* out);
// R jump polynomials x^(S * 2^r) mod phi, r = 0..R-1, 624 little-endian u32 words each
// (bit k = coefficient of x^k). Cached per (S, R).
std::vector<uint32_t> mt_jump_polys(uint64_t S, int R);
// The device algorithm run on the host (same plan, rounds and chunk generation): a CPU
// oracle for the GPU kernels' arithmetic. Writes total draws as floats.
void devgen_emulate(uint32_t seed, uint64_t first_draw, uint64_t total, float* out);

// Rows [0, rows) of the reference stream.
std::vector<float> generate_problem(int seed, int dim, int64_t rows);
// Rows [first, first+rows) of the reference stream (jump-ahead; any first).
void generate_rows(int seed, int dim, int64_t first, int64_t rows, float* out, int threads = 0);

}  // namespace pkdtree
