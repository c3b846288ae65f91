// Device generator of the reference stream: see pkdtree/gpu_generator.hpp.
//
// Kernels (256 threads = 4 waves per workgroup, MT state in LDS):
//   k_mt_extend   one workgroup per source state: the 624-word window followed by 32 twisted
//                 blocks (the state's untempered extension, 20592 words) -> workspace;
//   k_mt_apply    one workgroup per target state: (q(f) s)[m] = XOR_{k: q_k = 1} w[k + m],
//                 with w staged in LDS (82 KB) and q scanned word by word on the scalar unit;
//   k_mt_generate one workgroup per chunk: twist in LDS (4 dependency phases of the MT
//                 recurrence), temper, libstdc++ float map, coalesced stores.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "pkdtree/common.hpp"
#include "pkdtree/gpu_generator.hpp"
#include "pkdtree/hip_check.hpp"
#include "pkdtree/trace.hpp"

namespace pkdtree {
namespace {

constexpr int kGenBlock = 256;
constexpr int kN = 624, kM = 397;
constexpr u32 kUpper = 0x80000000u, kLower = 0x7fffffffu, kMatrix = 0x9908b0dfu;

__device__ __forceinline__ u32 mt_rec(u32 a, u32 b, u32 c) {
  const u32 y = (a & kUpper) | (b & kLower);
  return c ^ (y >> 1) ^ ((y & 1u) ? kMatrix : 0u);
}

// In-place twist of mt[624] in LDS, the same result as the serial loop
//   for i in 0..623: mt[i] = rec(mt[i], mt[(i+1)%N], mt[(i+M)%N]).
// Word i reads mt[i+M] (old for i < 227, new mt[i-227] after) and mt[i+1] (new mt[0] for
// i = 623), so the loop splits into phases [0,227), [227,454), [454,623), {623}; each phase
// computes into registers, then writes after a barrier.
__device__ __forceinline__ void twist_lds(u32* mt) {
  const int t = threadIdx.x;
  constexpr int kA = kN - kM;  // 227
  u32 v = 0;
  if (t < kA) v = mt_rec(mt[t], mt[t + 1], mt[t + kM]);
  __syncthreads();
  if (t < kA) mt[t] = v;
  __syncthreads();
  if (t < kA) v = mt_rec(mt[kA + t], mt[kA + t + 1], mt[t]);
  __syncthreads();
  if (t < kA) mt[kA + t] = v;
  __syncthreads();
  if (t < kN - 1 - 2 * kA) v = mt_rec(mt[2 * kA + t], mt[2 * kA + t + 1], mt[kA + t]);
  __syncthreads();
  if (t < kN - 1 - 2 * kA) mt[2 * kA + t] = v;
  __syncthreads();
  if (t == 0) mt[kN - 1] = mt_rec(mt[kN - 1], mt[0], mt[kM - 1]);
  __syncthreads();
}

__device__ __forceinline__ float mt_float(u32 y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  // generate_canonical<float, 24>: float(y) / 2^32, clamped below 1; then u * 200 + (-100)
  // with separately rounded multiply and add (this TU is built with -ffp-contract=off).
  float u = __fmul_rn(float(y), 2.3283064365386963e-10f);
  if (u >= 1.0f) u = 0.99999994f;
  return __fadd_rn(__fmul_rn(u, 200.0f), -100.0f);
}

__global__ __launch_bounds__(kGenBlock) void k_mt_extend(const u32* __restrict__ states, u32* __restrict__ ext) {
  __shared__ u32 mt[kN];
  const u32* s = states + size_t(blockIdx.x) * kN;
  u32* w = ext + size_t(blockIdx.x) * kMtExtWords;
  for (int i = threadIdx.x; i < kN; i += kGenBlock) {
    const u32 v = s[i];
    mt[i] = v;
    w[i] = v;
  }
  __syncthreads();
  for (int b = 1; b < kMtExtWords / kN; ++b) {
    twist_lds(mt);
    for (int i = threadIdx.x; i < kN; i += kGenBlock) w[b * kN + i] = mt[i];
  }
}

// Target state dst0 + blockIdx.x from source state blockIdx.x with polynomial q. Wave v
// takes q's words [v*39, (v+1)*39); lane l accumulates m = l + 64j (j < 10) so every set bit
// issues 10 independent LDS reads; the 16 partial states are XOR-reduced through LDS.
constexpr int kApplyBlock = 1024;
constexpr int kApplyWaves = kApplyBlock / 64;
constexpr int kApplyLds = (kMtExtWords + kApplyWaves * kN) * 4;
__global__ __launch_bounds__(kApplyBlock) void k_mt_apply(const u32* __restrict__ ext, const u32* __restrict__ q,
                                                          u32* __restrict__ states, int dst0) {
  extern __shared__ u32 w[];  // [kMtExtWords] extension, then [kApplyWaves][kN] partials
  u32* red = w + kMtExtWords;
  const u32* src = ext + size_t(blockIdx.x) * kMtExtWords;
  for (int i = threadIdx.x; i < kMtExtWords; i += kApplyBlock) w[i] = src[i];
  __syncthreads();
  const int l = threadIdx.x & 63, v = threadIdx.x >> 6;
  constexpr int kJ = (kN + 63) / 64;  // 10
  constexpr int kWordsPerWave = (kMtWords + kApplyWaves - 1) / kApplyWaves;
  u32 a[kJ];
#pragma unroll
  for (int j = 0; j < kJ; ++j) a[j] = 0;
  const int w0 = v * kWordsPerWave, w1 = min(kMtWords, w0 + kWordsPerWave);
  for (int wi = w0; wi < w1; ++wi) {
    u32 word = __builtin_amdgcn_readfirstlane(q[wi]);
    while (word) {
      const int k = wi * 32 + __builtin_ctz(word);
      word &= word - 1;
      // lanes with m >= 624 read inside the extension (k + m < 19937 + 640) and are dropped
#pragma unroll
      for (int j = 0; j < kJ; ++j) a[j] ^= w[k + l + 64 * j];
    }
  }
#pragma unroll
  for (int j = 0; j < kJ; ++j)
    if (l + 64 * j < kN) red[v * kN + l + 64 * j] = a[j];
  __syncthreads();
  u32* d = states + size_t(dst0 + blockIdx.x) * kN;
  for (int m = threadIdx.x; m < kN; m += kApplyBlock) {
    u32 x = 0;
#pragma unroll
    for (int u = 0; u < kApplyWaves; ++u) x ^= red[u * kN + m];
    d[m] = x;
  }
}

__global__ __launch_bounds__(kGenBlock) void k_mt_generate(const u32* __restrict__ states, u64 S, u64 total,
                                                           float* __restrict__ out) {
  __shared__ u32 mt[kN];
  const u32* s = states + size_t(blockIdx.x) * kN;
  for (int i = threadIdx.x; i < kN; i += kGenBlock) mt[i] = s[i];
  __syncthreads();
  const u64 b = u64(blockIdx.x) * S;
  const u64 e = b + S < total ? b + S : total;
  for (u64 pos = b; pos < e; pos += kN) {
    twist_lds(mt);
    for (int j = threadIdx.x; j < kN; j += kGenBlock)
      if (pos + u64(j) < e) out[pos + u64(j)] = mt_float(mt[j]);
    // the next twist's first barrier orders these reads before its writes
  }
}

struct WsLayout {
  size_t states, ext, polys, bytes;
};

WsLayout layout(const DevGenPlan& p) {
  WsLayout l{};
  auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
  const size_t src_max = p.R > 0 ? size_t(1) << (p.R - 1) : 0;
  l.states = 0;
  l.ext = al(size_t(p.C) * kN * 4);
  l.polys = l.ext + al(src_max * kMtExtWords * 4);
  l.bytes = l.polys + al(size_t(p.R) * kMtWords * 4 + kN * 4);
  return l;
}

}  // namespace

size_t devgen_workspace_bytes(const DevGenPlan& p) { return p.C ? layout(p).bytes : 0; }

void generate_rows_device(uint32_t seed, int dim, int64_t first_row, int64_t rows, float* out, void* workspace,
                          hipStream_t stream) {
  const u64 total = u64(rows) * u64(dim);
  const DevGenPlan p = devgen_plan(total);
  if (p.C == 0) return;
  TraceRange tr("pkd.generate");
  const WsLayout l = layout(p);
  char* ws = static_cast<char*>(workspace);
  u32* states = reinterpret_cast<u32*>(ws + l.states);
  u32* ext = reinterpret_cast<u32*>(ws + l.ext);
  u32* polys = reinterpret_cast<u32*>(ws + l.polys);
  // host inputs: the R jump polynomials, then chunk 0's start window
  std::vector<u32> host = mt_jump_polys(p.S, p.R);
  host.resize(size_t(p.R) * kMtWords + kN);
  mt_window_after(seed, u64(first_row) * u64(dim), host.data() + size_t(p.R) * kMtWords);
  PKD_HIP_CHECK(hipStreamSynchronize(stream));  // the workspace may still be in use by earlier work
  PKD_HIP_CHECK(hipMemcpy(polys, host.data(), host.size() * 4, hipMemcpyHostToDevice));
  PKD_HIP_CHECK(hipMemcpyAsync(states, polys + size_t(p.R) * kMtWords, kN * 4, hipMemcpyDeviceToDevice, stream));
  ensure_dynamic_lds(reinterpret_cast<const void*>(&k_mt_apply), kApplyLds);
  for (int r = 0; r < p.R; ++r) {
    const int src = 1 << r;
    const int n = std::min(src, p.C - src);
    if (n <= 0) break;
    k_mt_extend<<<n, kGenBlock, 0, stream>>>(states, ext);
    k_mt_apply<<<n, kApplyBlock, kApplyLds, stream>>>(ext, polys + size_t(r) * kMtWords, states, src);
  }
  k_mt_generate<<<p.C, kGenBlock, 0, stream>>>(states, p.S, p.total, out);
  PKD_HIP_CHECK(hipGetLastError());
}

}  // namespace pkdtree
