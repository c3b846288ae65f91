// HBM roofline of one MI355X: read-only, write-only and copy streams of 16-B elements, each
// swept over grid size, unroll depth (16-B accesses in flight per lane) and cache policy
// (default vs nontemporal). The best row of each class is the ceiling the builder's passes
// are judged against (profiles/r2_hbm_roofline.txt).
// Build: hipcc --offload-arch=gfx950 -O3 -o hbm_roofline hbm_roofline.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kB = 256;

template <int U, bool NT>
__global__ __launch_bounds__(kB) void k_read(const f4* __restrict__ a, long n, float* __restrict__ sink) {
  const long stride = long(gridDim.x) * kB;
  f4 acc = {0, 0, 0, 0};
  for (long i0 = blockIdx.x * long(kB) + threadIdx.x; i0 < n; i0 += stride * U) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * stride;
      v[u] = i < n ? (NT ? __builtin_nontemporal_load(a + i) : a[i]) : f4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc.x + acc.y + acc.z + acc.w == 1234.5f) sink[threadIdx.x] = acc.x;  // keeps the loads alive
}

template <int U, bool NT>
__global__ __launch_bounds__(kB) void k_write(f4* __restrict__ b, long n) {
  const long stride = long(gridDim.x) * kB;
  for (long i0 = blockIdx.x * long(kB) + threadIdx.x; i0 < n; i0 += stride * U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * stride;
      const f4 v = {float(i), 1.0f, 2.0f, 3.0f};
      if (i < n) {
        if (NT) __builtin_nontemporal_store(v, b + i);
        else b[i] = v;
      }
    }
  }
}

template <int U, bool NT>
__global__ __launch_bounds__(kB) void k_copy(const f4* __restrict__ a, f4* __restrict__ b, long n) {
  const long stride = long(gridDim.x) * kB;
  for (long i0 = blockIdx.x * long(kB) + threadIdx.x; i0 < n; i0 += stride * U) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * stride;
      if (i < n) v[u] = NT ? __builtin_nontemporal_load(a + i) : a[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * stride;
      if (i < n) {
        if (NT) __builtin_nontemporal_store(v[u], b + i);
        else b[i] = v[u];
      }
    }
  }
}

// Contiguous chunk per block (the partition kernels' shape: each block owns a run of rows).
template <int U, bool NT>
__global__ __launch_bounds__(kB) void k_copy_chunk(const f4* __restrict__ a, f4* __restrict__ b, long n) {
  const long per = (n + gridDim.x - 1) / gridDim.x;
  const long lo = long(blockIdx.x) * per, hi = std::min(n, lo + per);
  for (long i0 = lo + threadIdx.x; i0 < hi; i0 += long(kB) * U) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * kB;
      if (i < hi) v[u] = NT ? __builtin_nontemporal_load(a + i) : a[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * kB;
      if (i < hi) {
        if (NT) __builtin_nontemporal_store(v[u], b + i);
        else b[i] = v[u];
      }
    }
  }
}

template <typename F>
float best_ms(F&& launch, int reps = 7) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  launch();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms);
  }
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return best;
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? std::atol(argv[1]) : 100000000L;  // 16-B elements (1.6 GB per buffer)
  f4 *a = nullptr, *b = nullptr;
  float* sink = nullptr;
  CK(hipMalloc(&a, n * 16));
  CK(hipMalloc(&b, n * 16));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(a, 0, n * 16));
  CK(hipMemset(b, 0, n * 16));
  const double gb = double(n) * 16 / 1e9;
  std::printf("n=%ld elements of 16 B (%.2f GB per buffer); TB/s counts every byte read or written\n", n, gb);
  const int grids[] = {256, 512, 1024, 2048, 4096, 8192};
#define ROW(name, bytes_factor, U, NT, call)                                                              \
  for (int g : grids) {                                                                                   \
    const float ms = best_ms([&] { call; });                                                              \
    std::printf("%-12s U=%-2d nt=%d grid=%-5d %8.1f us  %5.2f TB/s\n", name, U, int(NT), g, ms * 1e3,      \
                bytes_factor * gb / ms);                                                 \
  }
  ROW("read", 1.0, 4, false, (k_read<4, false><<<g, kB>>>(a, n, sink)))
  ROW("read", 1.0, 8, false, (k_read<8, false><<<g, kB>>>(a, n, sink)))
  ROW("read", 1.0, 8, true, (k_read<8, true><<<g, kB>>>(a, n, sink)))
  ROW("write", 1.0, 4, false, (k_write<4, false><<<g, kB>>>(b, n)))
  ROW("write", 1.0, 8, true, (k_write<8, true><<<g, kB>>>(b, n)))
  ROW("copy", 2.0, 2, false, (k_copy<2, false><<<g, kB>>>(a, b, n)))
  ROW("copy", 2.0, 4, false, (k_copy<4, false><<<g, kB>>>(a, b, n)))
  ROW("copy", 2.0, 8, false, (k_copy<8, false><<<g, kB>>>(a, b, n)))
  ROW("copy", 2.0, 4, true, (k_copy<4, true><<<g, kB>>>(a, b, n)))
  ROW("copy", 2.0, 8, true, (k_copy<8, true><<<g, kB>>>(a, b, n)))
  ROW("copy_chunk", 2.0, 4, false, (k_copy_chunk<4, false><<<g, kB>>>(a, b, n)))
  ROW("copy_chunk", 2.0, 8, false, (k_copy_chunk<8, false><<<g, kB>>>(a, b, n)))
  ROW("copy_chunk", 2.0, 8, true, (k_copy_chunk<8, true><<<g, kB>>>(a, b, n)))
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(sink));
  return 0;
}
