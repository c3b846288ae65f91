// LDS subtree kernel: one workgroup builds a whole segment (<= NMAX points) in LDS.
//
// The segment's rows are loaded once into LDS (SoA, fixed) and only a 32-bit slot word
// per point moves: slot = local row index | (sub-segment id << 16). Every level:
//   * sub-segments larger than kSmall: per-sub-segment key range (LDS min/max), linear
//     bucket histogram, bucket of the median, stable 3-zone scatter computed with wave
//     ballots + one 64-entry scan per zone, then exact (key,id) ranking of the few points
//     of the median bucket;
//   * sub-segments of at most kSmall points: each point counts the smaller (key,id) in its
//     sub-segment, which sorts it on the level's axis (median and partition at once).
// Points whose slot is final are marked done and never move again, so after the last level
// the slot array is the in-order tree; it is written out AoS with coalesced stores.
// This collapses the bottom ~12 levels of build_tree_rec (kdtree_sequential.cpp:30-66),
// where the reference spends millions of tiny sorts and `new Node`s.
#include <algorithm>
#include <stdexcept>

#include "device_utils.hpp"
#include "pkdtree/hip_check.hpp"
#include "subtree.hpp"

namespace pkdtree {

using dev::BucketParams;
using dev::bucket_of;
using dev::make_params;
using dev::mbcnt;

namespace {

constexpr int kBlock = 256;
constexpr int kSmall = 16;
constexpr u32 kDone = 0xffffu;
constexpr u32 kMid = 0x8000u;
constexpr size_t kLdsBudget = 160 * 1024 - 2048;  // leave room for static LDS

size_t subtree_lds_bytes(int dim, int nmax) {
  // rows (dim+1) + slot + keyv + sub + hist (nmax/2) + stats (nmax/2), all 32-bit words
  return size_t(dim + 1) * size_t(nmax) * 4 + size_t(nmax) * 4 * 3 + size_t(nmax) * 4;
}

struct SubArgs {
  const float* cols;
  i64 ncol;
  int dim;
  const i64* seg_lo;
  const i64* seg_n;
  i64 heap0;
  int depth_base;
  int nmax;
  float* out_pts;
  u32* out_ids;
};

__device__ __forceinline__ int pow2_floor_dev(int v) { return v <= 1 ? 1 : 1 << (31 - __clz(v)); }

template <int ITEMS>
__global__ __launch_bounds__(kBlock) void k_subtree(SubArgs a) {
  extern __shared__ __align__(16) u32 smem[];
  __shared__ u32 gcnt[3][64];
  const int dim = a.dim;
  const int NM = a.nmax;
  const i64 h = a.heap0 + blockIdx.x;
  const int n = int(a.seg_n[h]);
  if (n <= 0) return;
  const i64 glo = a.seg_lo[h];
  float* rows = reinterpret_cast<float*>(smem);          // [(dim+1) * NM]
  u32* slot = smem + size_t(dim + 1) * NM;               // [NM]
  u32* keyv = slot + NM;                                 // [NM]
  u32* sub = keyv + NM;                                  // [NM]   (lo << 16) | n
  u32* hist = sub + NM;                                  // [NM/2]
  u32* stats = hist + NM / 2;                            // [NM/2]
  const int tid = threadIdx.x;
  const int w = tid / 64;
  const int ln = dev::lane();

  for (int c = 0; c <= dim; ++c) {
    const float* col = a.cols + i64(c) * a.ncol + glo;
    for (int k = tid; k < n; k += kBlock) rows[c * NM + k] = col[k];
  }
  for (int k = tid; k < n; k += kBlock) slot[k] = u32(k);
  if (tid == 0) sub[0] = u32(n);
  const u32* idrow = reinterpret_cast<const u32*>(rows + dim * NM);
  __syncthreads();

  for (int l = 0;; ++l) {
    const int ml = n >> l;
    if (ml == 0) break;
    const int S = 1 << l;
    const int axis = (a.depth_base + l) % dim;
    const float* kcol = rows + axis * NM;
    u32 sl[ITEMS], ok[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const int p = tid + i * kBlock;
      sl[i] = p < n ? slot[p] : (kDone << 16);
      ok[i] = 0;
      if ((sl[i] >> 16) != kDone) {
        ok[i] = orderable(kcol[sl[i] & 0xffffu]);
        keyv[p] = ok[i];
      }
    }
    if (ml > kSmall) {
      // ---------------- bucket path ----------------
      const int B = min(1024, max(8, pow2_floor_dev(ml / 4)));
      u32* mn = stats;
      u32* mx = stats + S;
      u32* bst = stats + 2 * S;
      u32* cle = stats + 3 * S;
      u32* cmi = stats + 4 * S;
      u32* bas = stats + 5 * S;  // [3][S]
      for (int j = tid; j < S; j += kBlock) {
        mn[j] = 0xffffffffu;
        mx[j] = 0u;
      }
      for (int b = tid; b < S * B; b += kBlock) hist[b] = 0;
      __syncthreads();
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const u32 sid = sl[i] >> 16;
        const bool act = sid != kDone;
        // waves mostly sit inside one sub-segment: reduce first when they do
        const u32 s0 = __builtin_amdgcn_readfirstlane(act ? sid : 0xffffffffu);
        if (__all(!act || sid == s0)) {
          const u32 vmin = dev::wave_min_u32(act ? ok[i] : 0xffffffffu);
          const u32 vmax = dev::wave_max_u32(act ? ok[i] : 0u);
          if (ln == 0 && s0 != 0xffffffffu) {
            atomicMin(&mn[s0], vmin);
            atomicMax(&mx[s0], vmax);
          }
        } else if (act) {
          atomicMin(&mn[sid], ok[i]);
          atomicMax(&mx[sid], ok[i]);
        }
      }
      __syncthreads();
      // The bucket goes through LDS (keyv) rather than a register array: carrying it in
      // registers across the select phase crashes ROCm 7.2's gfx950 instruction selector.
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const u32 sid = sl[i] >> 16;
        if (sid != kDone) {
          const BucketParams prm = make_params(from_orderable(mn[sid]), from_orderable(mx[sid]), B);
          const u32 b = bucket_of(from_orderable(ok[i]), prm, B);
          keyv[tid + i * kBlock] = b;
          atomicAdd(&hist[sid * B + b], 1u);
        }
      }
      __syncthreads();
      // select: G lanes per sub-segment
      {
        const int G = min(64, max(1, kBlock / S));
        const int groups = kBlock / G;
        const int gl = tid & (G - 1);
        const int per = (B + G - 1) / G;
        for (int j = tid / G; j < S; j += groups) {
          const u32 e = sub[j];
          const u32 r = (e & 0xffffu) / 2;
          const u32* hs = hist + j * B;
          const int b0 = min(B, gl * per), b1 = min(B, b0 + per);
          u32 sum = 0;
          for (int b = b0; b < b1; ++b) sum += hs[b];
          u32 incl = sum;
          for (int o = 1; o < G; o <<= 1) {
            const u32 t = __shfl_up(incl, o, G);
            if (gl >= o) incl += t;
          }
          const u32 excl = incl - sum;
          if ((e & 0xffffu) > 0 && r >= excl && r < incl) {
            u32 c = excl;
            for (int b = b0; b < b1; ++b) {
              const u32 v = hs[b];
              if (r < c + v) {
                bst[j] = u32(b);
                cle[j] = c;
                cmi[j] = v;
                break;
              }
              c += v;
            }
          }
        }
      }
      __syncthreads();
      u32 zz[ITEMS];
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const u32 sid = sl[i] >> 16;
        u32 z = 3;
        if (sid != kDone) {
          const u32 bs = bst[sid];
          const u32 b = keyv[tid + i * kBlock];
          z = b < bs ? 0u : (b == bs ? 1u : 2u);
        }
        zz[i] = z;
        const u64 m0 = __ballot(z == 0), m1 = __ballot(z == 1), m2 = __ballot(z == 2);
        if (ln == 0) {
          gcnt[0][i * 4 + w] = __popcll(m0);
          gcnt[1][i * 4 + w] = __popcll(m1);
          gcnt[2][i * 4 + w] = __popcll(m2);
        }
      }
      for (int i = ITEMS; i < 16; ++i) {
        if (ln == 0) gcnt[0][i * 4 + w] = gcnt[1][i * 4 + w] = gcnt[2][i * 4 + w] = 0;
      }
      __syncthreads();
      if (w < 3) {
        const u32 v = gcnt[w][ln];
        gcnt[w][ln] = dev::wave_incl_scan(v) - v;
      }
      __syncthreads();
      // zone prefix of every point; first point of each sub-segment publishes the bases
      u32 pz[ITEMS];
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const int p = tid + i * kBlock;
        const u32 z = zz[i];
        const u64 m0 = __ballot(z == 0), m1 = __ballot(z == 1), m2 = __ballot(z == 2);
        const u32 p0 = gcnt[0][i * 4 + w] + mbcnt(m0);
        const u32 p1 = gcnt[1][i * 4 + w] + mbcnt(m1);
        const u32 p2 = gcnt[2][i * 4 + w] + mbcnt(m2);
        pz[i] = z == 0 ? p0 : (z == 1 ? p1 : p2);
        if (z < 3) {
          const u32 sid = sl[i] >> 16;
          if (u32(p) == (sub[sid] >> 16)) {
            bas[sid] = p0;
            bas[S + sid] = p1;
            bas[2 * S + sid] = p2;
          }
        }
      }
      __syncthreads();
      u32 np[ITEMS], ns[ITEMS];
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const u32 z = zz[i];
        np[i] = 0xffffffffu;
        if (z < 3) {
          const u32 sid = sl[i] >> 16;
          const u32 jlo = sub[sid] >> 16;
          const u32 start = z == 0 ? 0u : (z == 1 ? cle[sid] : cle[sid] + cmi[sid]);
          np[i] = jlo + start + pz[i] - bas[z * S + sid];
          const u32 nsid = z == 0 ? 2 * sid : (z == 2 ? 2 * sid + 1 : (kMid | sid));
          ns[i] = (sl[i] & 0xffffu) | (nsid << 16);
        }
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < ITEMS; ++i)
        if (np[i] != 0xffffffffu) slot[np[i]] = ns[i];
      __syncthreads();
      // exact ranking inside the median bucket
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const int p = tid + i * kBlock;
        np[i] = 0xffffffffu;
        if (p < n) {
          const u32 s = slot[p];
          const u32 tag = s >> 16;
          if (tag != kDone && (tag & kMid)) {
            const u32 sid = tag & 0x7fffu;
            const u32 idx = s & 0xffffu;
            const u32 e = sub[sid];
            const u32 jlo = e >> 16, jn = e & 0xffffu;
            const u32 zlo = jlo + cle[sid], zc = cmi[sid];
            const u32 mk = orderable(kcol[idx]);
            const u32 mid = idrow[idx];
            u32 rank = 0;
            for (u32 q = zlo; q < zlo + zc; ++q) {
              const u32 oi = slot[q] & 0xffffu;
              const u32 qk = orderable(kcol[oi]);
              rank += (qk < mk || (qk == mk && idrow[oi] < mid)) ? 1u : 0u;
            }
            const u32 t = jn / 2 - cle[sid];
            const u32 nsid = rank < t ? 2 * sid : (rank > t ? 2 * sid + 1 : kDone);
            np[i] = zlo + rank;
            ns[i] = idx | (nsid << 16);
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < ITEMS; ++i)
        if (np[i] != 0xffffffffu) slot[np[i]] = ns[i];
      __syncthreads();
    } else {
      // ---------------- counting path (sub-segments of <= kSmall points) ----------------
      __syncthreads();  // keyv complete
      u32 np[ITEMS], ns[ITEMS];
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        np[i] = 0xffffffffu;
        const u32 sid = sl[i] >> 16;
        if (sid != kDone) {
          const u32 idx = sl[i] & 0xffffu;
          const u32 e = sub[sid];
          const u32 jlo = e >> 16, jn = e & 0xffffu;
          const u32 mk = ok[i];
          const u32 mid = idrow[idx];
          u32 rank = 0;
          for (u32 q = jlo; q < jlo + jn; ++q) {
            const u32 qk = keyv[q];
            rank += (qk < mk || (qk == mk && idrow[slot[q] & 0xffffu] < mid)) ? 1u : 0u;
          }
          const u32 half = jn / 2;
          const u32 nsid = rank < half ? 2 * sid : (rank > half ? 2 * sid + 1 : kDone);
          np[i] = jlo + rank;
          ns[i] = idx | (nsid << 16);
        }
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < ITEMS; ++i)
        if (np[i] != 0xffffffffu) slot[np[i]] = ns[i];
      __syncthreads();
    }
    // sub-segment table of the next level
    if ((n >> (l + 1)) > 0) {
      u32 ev[ITEMS];
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const int j = tid + i * kBlock;
        ev[i] = j < S ? sub[j] : 0u;
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const int j = tid + i * kBlock;
        if (j < S) {
          const u32 lo = ev[i] >> 16, m = ev[i] & 0xffffu;
          const u32 mr = m >= 1 ? m - m / 2 - 1 : 0u;
          sub[2 * j] = (lo << 16) | (m / 2);
          sub[2 * j + 1] = ((lo + m / 2 + 1) << 16) | mr;
        }
      }
      __syncthreads();
    }
  }
  // in-order rows out, AoS, coalesced
  const i64 total = i64(n) * dim;
  float* outp = a.out_pts + glo * dim;
  for (i64 f = tid; f < total; f += kBlock) {
    const int k = int(f / dim);
    const int c = int(f - i64(k) * dim);
    outp[f] = rows[c * NM + (slot[k] & 0xffffu)];
  }
  for (int k = tid; k < n; k += kBlock) a.out_ids[glo + k] = idrow[slot[k] & 0xffffu];
}

template <int ITEMS>
void launch_items(const SubArgs& a, i64 segs, size_t lds, hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    PKD_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_subtree<ITEMS>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, int(kLdsBudget)));
    attr_set = true;
  }
  k_subtree<ITEMS><<<dim3(unsigned(segs)), kBlock, lds, stream>>>(a);
  PKD_LAUNCH_CHECK();
}

}  // namespace

int subtree_capacity(int dim) {
  for (int nm = 4096; nm >= 32; nm /= 2)
    if (subtree_lds_bytes(dim, nm) <= kLdsBudget) return nm;
  throw std::invalid_argument("pkdtree: dimension too large for the LDS subtree kernel");
}

void launch_subtree(const float* cols, i64 ncol, int dim, const i64* seg_lo, const i64* seg_n, i64 heap0, i64 segs,
                    int depth_base, int nmax, float* out_pts, u32* out_ids, hipStream_t stream) {
  if (segs <= 0) return;
  SubArgs a{cols, ncol, dim, seg_lo, seg_n, heap0, depth_base, nmax, out_pts, out_ids};
  const size_t lds = subtree_lds_bytes(dim, nmax);
  if (nmax > 2048) launch_items<16>(a, segs, lds, stream);
  else if (nmax > 1024) launch_items<8>(a, segs, lds, stream);
  else if (nmax > 512) launch_items<4>(a, segs, lds, stream);
  else if (nmax > 256) launch_items<2>(a, segs, lds, stream);
  else launch_items<1>(a, segs, lds, stream);
}

}  // namespace pkdtree
