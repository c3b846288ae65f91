// Microbenchmark: HBM ceilings of the partition pass shapes on one MI355X.
//   copy4        float4 copy (read + write n rows of 16 B)
//   soa_scatter  4 SoA columns, 4-way zone scatter, per-lane stores (the k_partition2 shape)
//   aos_scatter  16-B rows (x, y, z, id), 4-way zone scatter, one dwordx4 store per row
//   aos_lds      16-B rows staged zone-sorted in LDS, written out as contiguous runs
// Zones come from the row's first coordinate (uniform), cursors are global atomics per
// zone per chunk, exactly as in the partition kernels. Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

typedef unsigned int u32;
typedef unsigned long long u64;
constexpr int kB = 256;
constexpr int kZ = 4;

__global__ void k_init(float4* rows, float* cols, long n) {
  for (long i = blockIdx.x * long(kB) + threadIdx.x; i < n; i += long(gridDim.x) * kB) {
    u32 h = u32(i) * 2654435761u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    const float x = float(h & 0xffffff) / 16777216.0f;
    rows[i] = make_float4(x, x * 0.5f, x * 0.25f, __uint_as_float(u32(i)));
    cols[i] = x;
    cols[n + i] = x * 0.5f;
    cols[2 * n + i] = x * 0.25f;
    cols[3 * n + i] = __uint_as_float(u32(i));
  }
}

__global__ __launch_bounds__(kB) void k_copy4(const float4* __restrict__ a, float4* __restrict__ b, long n) {
  constexpr int U = 4;
  const long stride = long(gridDim.x) * kB;
  for (long i0 = blockIdx.x * long(kB) + threadIdx.x; i0 < n; i0 += stride * U) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * stride;
      if (i < n) v[u] = a[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * stride;
      if (i < n) b[i] = v[u];
    }
  }
}

typedef float f4v __attribute__((ext_vector_type(4)));
template <int U>
__global__ __launch_bounds__(kB) void k_copy_nt(const f4v* __restrict__ a, f4v* __restrict__ b, long n) {
  const long stride = long(gridDim.x) * kB;
  for (long i0 = blockIdx.x * long(kB) + threadIdx.x; i0 < n; i0 += stride * U) {
    f4v v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * stride;
      if (i < n) v[u] = __builtin_nontemporal_load(a + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * stride;
      if (i < n) __builtin_nontemporal_store(v[u], b + i);
    }
  }
}

__device__ __forceinline__ u32 zone_of(float x) { return min(u32(x * kZ), u32(kZ - 1)); }
__device__ __forceinline__ u32 mbcnt(u64 m) {
  return __builtin_amdgcn_mbcnt_hi(u32(m >> 32), __builtin_amdgcn_mbcnt_lo(u32(m), 0u));
}

// Per chunk of kB*KI rows: ballot ranks per (item, wave) and zone, one scan per zone, one
// global atomic per zone per chunk, then the stores.
template <int KI, bool AOS>
__global__ __launch_bounds__(kB) void k_scatter(const float* __restrict__ src, float* __restrict__ dst, long n,
                                                long per, u32* __restrict__ cur0, long zcap0, int bps) {
  const int seg = blockIdx.x / bps;
  u32* cur = cur0 + seg * kZ;
  const long zcap = zcap0;
  const long zoff = long(seg) * kZ * zcap0;
  __shared__ u32 gcnt[kZ][KI * 4];
  const long ncs = long(gridDim.x / bps) * kZ * zcap0;  // column stride of the SoA output
  const long b0 = min(n, blockIdx.x * per), b1 = min(n, b0 + per);
  const int w = threadIdx.x / 64, ln = threadIdx.x % 64;
  for (long c0 = b0; c0 < b1; c0 += kB * KI) {
    float4 row[KI];
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      const long e = c0 + i * kB + threadIdx.x;
      const long p = e < b1 ? e : b0;
      if (AOS) {
        row[i] = reinterpret_cast<const float4*>(src)[p];
      } else {
        row[i].x = src[p];
        row[i].y = src[n + p];
        row[i].z = src[2 * n + p];
        row[i].w = src[3 * n + p];
      }
    }
    u32 zp[KI];
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      const long e = c0 + i * kB + threadIdx.x;
      const u32 q = e < b1 ? zone_of(row[i].x) : 7u;
      u32 my = 0;
#pragma unroll
      for (int z = 0; z < kZ; ++z) {
        const u64 m = __ballot(q == u32(z));
        if (ln == 0) gcnt[z][i * 4 + w] = __popcll(m);
        if (q == u32(z)) my = mbcnt(m);
      }
      zp[i] = (q << 16) | my;
    }
    __syncthreads();
    if (w < kZ) {
      const u32 v = ln < KI * 4 ? gcnt[w][ln] : 0u;
      u32 incl = v;
      for (int o = 1; o < 64; o <<= 1) {
        const u32 t = __shfl_up(incl, o, 64);
        if (ln >= o) incl += t;
      }
      const u32 tot = __shfl(incl, 63, 64);
      u32 base = 0;
      if (ln == 0 && tot) base = atomicAdd(&cur[w], tot);
      base = __shfl(base, 0, 64);
      if (ln < KI * 4) gcnt[w][ln] = base + incl - v;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      const u32 q = zp[i] >> 16;
      if (q < kZ) {
        const long d = zoff + long(q) * zcap + gcnt[q][i * 4 + w] + (zp[i] & 0xffffu);
        if (AOS) {
          reinterpret_cast<float4*>(dst)[d] = row[i];
        } else {
          dst[d] = row[i].x;
          dst[ncs + d] = row[i].y;
          dst[2 * ncs + d] = row[i].z;
          dst[3 * ncs + d] = row[i].w;
        }
      }
    }
    __syncthreads();
  }
}

// AoS rows staged zone-sorted in LDS; each zone's run of the chunk is written with
// consecutive lanes on consecutive rows (contiguous 16-B stores).
template <int KI>
__global__ __launch_bounds__(kB) void k_scatter_lds(const float4* __restrict__ src, float4* __restrict__ dst0, long n,
                                                    long per, u32* __restrict__ cur0, long zcap, int bps) {
  const int seg = blockIdx.x / bps;
  u32* cur = cur0 + seg * kZ;
  float4* dst = dst0 + long(seg) * kZ * zcap;
  __shared__ u32 gcnt[kZ][KI * 4];
  __shared__ u32 zst[kZ + 1], zbase[kZ];
  __shared__ float4 stage[kB * KI];
  const long b0 = min(n, blockIdx.x * per), b1 = min(n, b0 + per);
  const int w = threadIdx.x / 64, ln = threadIdx.x % 64;
  for (long c0 = b0; c0 < b1; c0 += kB * KI) {
    float4 row[KI];
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      const long e = c0 + i * kB + threadIdx.x;
      row[i] = src[e < b1 ? e : b0];
    }
    u32 zp[KI];
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      const long e = c0 + i * kB + threadIdx.x;
      const u32 q = e < b1 ? zone_of(row[i].x) : 7u;
      u32 my = 0;
#pragma unroll
      for (int z = 0; z < kZ; ++z) {
        const u64 m = __ballot(q == u32(z));
        if (ln == 0) gcnt[z][i * 4 + w] = __popcll(m);
        if (q == u32(z)) my = mbcnt(m);
      }
      zp[i] = (q << 16) | my;
    }
    __syncthreads();
    if (w < kZ) {
      const u32 v = ln < KI * 4 ? gcnt[w][ln] : 0u;
      u32 incl = v;
      for (int o = 1; o < 64; o <<= 1) {
        const u32 t = __shfl_up(incl, o, 64);
        if (ln >= o) incl += t;
      }
      const u32 tot = __shfl(incl, 63, 64);
      if (ln < KI * 4) gcnt[w][ln] = incl - v;
      if (ln == 0) {
        zst[w] = tot;
        zbase[w] = tot ? atomicAdd(&cur[w], tot) : 0u;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      u32 s = 0;
      for (int z = 0; z < kZ; ++z) {
        const u32 t = zst[z];
        zst[z] = s;
        s += t;
      }
      zst[kZ] = s;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      const u32 q = zp[i] >> 16;
      if (q < kZ) stage[zst[q] + gcnt[q][i * 4 + w] + (zp[i] & 0xffffu)] = row[i];
    }
    __syncthreads();
    const u32 tot = zst[kZ];
    for (u32 k = threadIdx.x; k < tot; k += kB) {
      int z = 0;
#pragma unroll
      for (int t = 1; t < kZ; ++t) z += k >= zst[t] ? 1 : 0;
      dst[long(z) * zcap + zbase[z] + (k - zst[z])] = stage[k];
    }
    __syncthreads();
  }
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 100000000L;
  const int blocks = argc > 2 ? atoi(argv[2]) : 2048;
  const int bps = argc > 3 ? atoi(argv[3]) : 32;  // blocks per segment (cursor sharing)
  const int nseg = blocks / bps;
  const long per = (n + blocks - 1) / blocks;
  const long zcap = (per * bps) / kZ + (per * bps) / 8 + 4096;  // per segment and zone
  float *a, *b, *cols;
  u32* cur;
  CK(hipMalloc(&a, size_t(n) * 16));
  CK(hipMalloc(&cols, size_t(n) * 16));
  CK(hipMalloc(&b, size_t(nseg) * kZ * zcap * 16));
  CK(hipMalloc(&cur, size_t(nseg) * kZ * 4));
  k_init<<<4096, kB>>>(reinterpret_cast<float4*>(a), cols, n);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("n=%ld blocks=%d blocks/segment=%d\n", n, blocks, bps);
  auto timeit = [&](const char* name, auto&& f) {
    for (int r = 0; r < 2; ++r) {
      CK(hipMemset(cur, 0, size_t(nseg) * kZ * 4));
      f();
    }
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CK(hipMemset(cur, 0, size_t(nseg) * kZ * 4));
      CK(hipEventRecord(e0));
      f();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    std::printf("%-22s %8.1f us  %5.2f TB/s (read + write of 16 B rows)\n", name, best * 1e3,
                2.0 * n * 16 / (best * 1e-3) / 1e12);
  };
  timeit("copy4 2x", [&] { k_copy4<<<blocks * 2, kB>>>((const float4*)a, (float4*)b, n); });
  timeit("copy4 8x", [&] { k_copy4<<<blocks * 8, kB>>>((const float4*)a, (float4*)b, n); });
  timeit("copy_nt U4 2x", [&] { k_copy_nt<4><<<blocks * 2, kB>>>((const f4v*)a, (f4v*)b, n); });
  timeit("copy_nt U8 1x", [&] { k_copy_nt<8><<<blocks, kB>>>((const f4v*)a, (f4v*)b, n); });
  timeit("soa_scatter KI=8", [&] { k_scatter<8, false><<<blocks, kB>>>(cols, b, n, per, cur, zcap, bps); });
  timeit("aos_scatter KI=8", [&] { k_scatter<8, true><<<blocks, kB>>>(a, b, n, per, cur, zcap, bps); });
  timeit("aos_scatter KI=4", [&] { k_scatter<4, true><<<blocks, kB>>>(a, b, n, per, cur, zcap, bps); });
  timeit("aos_lds KI=8", [&] { k_scatter_lds<8><<<blocks, kB>>>((const float4*)a, (float4*)b, n, per, cur, zcap, bps); });
  timeit("aos_lds KI=4", [&] { k_scatter_lds<4><<<blocks, kB>>>((const float4*)a, (float4*)b, n, per, cur, zcap, bps); });
  return 0;
}
