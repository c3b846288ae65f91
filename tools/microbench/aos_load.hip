// Read ceiling of the 3-D AoS input (100 M rows of 12 B) for two load shapes:
//   quad    a lane reads 4 whole rows with three 16-B loads at 48-B lane stride (the sampled
//           top scatter's and the prep's shape: each load instruction spans 3 KiB of lines);
//   linear  a lane reads 16-B element tid of each 1 KiB wave chunk (each instruction spans
//           1 KiB; rows straddle lanes, so a kernel would reassemble them through LDS).
// U = 16-B loads in flight per lane. Build: hipcc --offload-arch=gfx950 -O3 -o aos_load aos_load.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kB = 256;

// quads: nq groups of 4 rows (48 B); Q quads per lane per round
template <int Q>
__global__ __launch_bounds__(kB) void k_quad(const f4* __restrict__ a, long nq, float* __restrict__ sink) {
  const long stride = long(gridDim.x) * kB;
  f4 acc = {0, 0, 0, 0};
  for (long q0 = blockIdx.x * long(kB) + threadIdx.x; q0 < nq; q0 += stride * Q) {
    f4 v[Q][3];
#pragma unroll
    for (int u = 0; u < Q; ++u) {
      const long q = q0 + u * stride;
      const long qq = q < nq ? q : 0;
#pragma unroll
      for (int c = 0; c < 3; ++c) v[u][c] = a[qq * 3 + c];
    }
#pragma unroll
    for (int u = 0; u < Q; ++u)
#pragma unroll
      for (int c = 0; c < 3; ++c) acc += v[u][c];
  }
  if (acc.x + acc.y + acc.z + acc.w == 1234.5f) sink[threadIdx.x] = acc.x;
}

// linear: n4 16-B elements; a block's round covers 3 * Q * kB consecutive elements (the same
// 4 * Q rows per lane as k_quad), lane tid reading elements tid, tid + kB, ...
template <int Q>
__global__ __launch_bounds__(kB) void k_linear(const f4* __restrict__ a, long n4, float* __restrict__ sink) {
  constexpr int E = 3 * Q;
  f4 acc = {0, 0, 0, 0};
  for (long b0 = long(blockIdx.x) * E * kB; b0 < n4; b0 += long(gridDim.x) * E * kB) {
    f4 v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const long i = b0 + e * kB + threadIdx.x;
      v[e] = a[i < n4 ? i : 0];
    }
#pragma unroll
    for (int e = 0; e < E; ++e) acc += v[e];
  }
  if (acc.x + acc.y + acc.z + acc.w == 1234.5f) sink[threadIdx.x] = acc.x;
}

template <class F>
float best_ms(F launch) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  launch();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 10; ++r) {
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  return best;
}

int main() {
  const long rows = 100000000;
  const long nq = rows / 4, n4 = rows * 3 / 4;
  const double bytes = double(rows) * 12;
  f4* a = nullptr;
  float* sink = nullptr;
  CK(hipMalloc(&a, size_t(n4) * 16));
  CK(hipMalloc(&sink, kB * 4));
  CK(hipMemset(a, 0, size_t(n4) * 16));
  for (int grid : {1024, 2048, 4096, 8192}) {
    auto rep = [&](const char* name, int q, float ms) {
      std::printf("{\"shape\": \"%s\", \"Q\": %d, \"grid\": %d, \"ms\": %.4f, \"TBps\": %.3f}\n", name, q, grid, ms,
                  bytes / (ms * 1e-3) / 1e12);
    };
    rep("quad", 1, best_ms([&] { k_quad<1><<<grid, kB>>>(a, nq, sink); }));
    rep("quad", 2, best_ms([&] { k_quad<2><<<grid, kB>>>(a, nq, sink); }));
    rep("quad", 4, best_ms([&] { k_quad<4><<<grid, kB>>>(a, nq, sink); }));
    rep("linear", 1, best_ms([&] { k_linear<1><<<grid, kB>>>(a, n4, sink); }));
    rep("linear", 2, best_ms([&] { k_linear<2><<<grid, kB>>>(a, n4, sink); }));
    rep("linear", 4, best_ms([&] { k_linear<4><<<grid, kB>>>(a, n4, sink); }));
  }
  CK(hipGetLastError());
  return 0;
}
