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

// Rows [0, rows) of the reference stream.
std::vector<float> generate_problem(int seed, int dim, int64_t rows);
// Rows [first, first+rows) of the reference stream (jump-ahead; any first).
void generate_rows(int seed, int dim, int64_t first, int64_t rows, float* out, int threads = 0);

}  // namespace pkdtree
