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

constexpr int kSmall = 16;
constexpr u32 kDone = 0xffffu;
constexpr u32 kMid = 0x8000u;
constexpr size_t kLdsMax = 160 * 1024 - 1024;  // minus static LDS

// 32-bit words of dynamic LDS for capacity nm:
//   rows (dim+1)*nm | slot nm | keyv nm | sub nm | hist nm/2 | st 8*(nm/16) | cells 2*(nm/8)*dim*2
size_t subtree_lds_words(int dim, int nm) {
  return size_t(dim + 1) * nm + 3 * size_t(nm) + nm / 2 + 8 * size_t(nm / 16) + 2 * size_t(nm / 8) * dim * 2;
}
size_t subtree_lds_bytes(int dim, int nm) { return 4 * subtree_lds_words(dim, nm); }

struct SubArgs {
  const float* cols;
  i64 ncol;
  int dim;
  const i64* seg_lo;
  const i64* seg_n;
  const float* cells;  // heap-indexed [h][dim][2] cell of every segment root
  i64 heap0;
  int depth_base;
  float* out_pts;
  u32* out_ids;
  u32* err;
};

__device__ __forceinline__ int pow2_floor_dev(int v) { return v <= 1 ? 1 : 1 << (31 - __clz(v)); }

// Wave-aggregated LDS reservation: lanes with equal `key` get consecutive slots from
// cursor[key]; returns this lane's slot. One LDS atomic per distinct key per wave; the
// atomics are issued back to back (group leaders are found with scalar readlanes) and
// their results are gathered with a single permute at the end.
__device__ __forceinline__ u32 reserve(u32 key, bool active, u32* cursor) {
  u64 pending = __ballot(active);
  u32 lead_res = 0, my_leader = 0, my_rank = 0;
  const int ln = dev::lane();
  while (pending) {
    const int leader = __ffsll((long long)pending) - 1;
    const u32 lk = __builtin_amdgcn_readlane(key, leader);
    const u64 m = __ballot(active && key == lk) & pending;
    if (ln == leader) lead_res = atomicAdd(&cursor[lk], u32(__popcll(m)));
    if (active && key == lk) {
      my_leader = u32(leader);
      my_rank = mbcnt(m);
    }
    pending &= ~m;
  }
  return __shfl(lead_res, int(my_leader), 64) + my_rank;
}

template <int ITEMS, int THREADS>
__global__ __launch_bounds__(THREADS) void k_subtree(SubArgs a) {
  extern __shared__ __align__(16) u32 smem[];
  constexpr int NM = ITEMS * THREADS;
  const int dim = a.dim;
  const i64 h = a.heap0 + blockIdx.x;
  const int n = int(a.seg_n[h]);
  if (n <= 0) return;
  const i64 glo = a.seg_lo[h];
  float* rows = reinterpret_cast<float*>(smem);  // [(dim+1)][NM]
  u32* slot = smem + size_t(dim + 1) * NM;       // idx | sid << 16
  u32* keyv = slot + NM;                         // orderable key by slot (counting levels)
  u32* sub = keyv + NM;                          // (lo << 16) | n per sub-segment
  u32* hist = sub + NM;                          // [NM/2]
  u32* st = hist + NM / 2;                       // [8][NM/16]: bstar, cless, cmid, -, cursors[4]
  float* cellA = reinterpret_cast<float*>(st + 8 * (NM / 16));  // [NM/8][dim][2]
  float* cellB = cellA + (NM / 8) * dim * 2;
  constexpr int SB = NM / 16;
  u32* bst = st;
  u32* cle = st + SB;
  u32* cmi = st + 2 * SB;
  u32* cur = st + 4 * SB;  // [SB][4]
  const int tid = threadIdx.x;
  const u32* idrow = reinterpret_cast<const u32*>(rows + dim * NM);

  for (int c = 0; c <= dim; ++c) {
    const float* col = a.cols + i64(c) * a.ncol + glo;
    float v[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const int k = tid + i * THREADS;
      v[i] = k < n ? col[k] : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const int k = tid + i * THREADS;
      if (k < n) rows[c * NM + k] = v[i];
    }
  }
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int k = tid + i * THREADS;
    if (k < n) slot[k] = u32(k);
  }
  for (int b = tid; b < NM / 2; b += THREADS) hist[b] = 0;
  if (tid == 0) sub[0] = u32(n);
  for (int c = tid; c < 2 * dim; c += THREADS) cellA[c] = a.cells[h * 2 * dim + c];
  __syncthreads();
  float* cc = cellA;  // cells of the current level
  float* nc = cellB;  // cells of the next level

  for (int l = 0;; ++l) {
    const int ml = n >> l;
    if (ml == 0) break;
    const int S = 1 << l;
    const int axis = (a.depth_base + l) % dim;
    const float* kcol = rows + axis * NM;
    const bool more = (n >> (l + 1)) > 0;
    u32 sl[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const int p = tid + i * THREADS;
      sl[i] = p < n ? slot[p] : (kDone << 16);
    }
    float kf[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) kf[i] = ((sl[i] >> 16) != kDone) ? kcol[sl[i] & 0xffffu] : 0.0f;
    u32 ev[ITEMS];  // sub-segment table entries this thread rewrites for the next level
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const int j = tid + i * THREADS;
      ev[i] = (more && j < S) ? sub[j] : 0u;
    }
    u32 np[ITEMS], ns[ITEMS];
    if (ml > kSmall) {
      // ---------------- bucket path ----------------
      const int B = min(1024, max(8, pow2_floor_dev(ml / 2)));
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const u32 sid = sl[i] >> 16;
        if (sid != kDone) {
          const float* cl = cc + (sid * dim + axis) * 2;
          const BucketParams prm = make_params(cl[0], cl[1], B);
          atomicAdd(&hist[sid * B + bucket_of(kf[i], prm, B)], 1u);
        }
      }
      __syncthreads();
      {  // select: G lanes per sub-segment
        const int G = min(64, max(1, THREADS / S));
        const int groups = THREADS / G;
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
          if (r >= excl && r < incl) {
            u32 c = excl;
            for (int b = b0; b < b1; ++b) {
              const u32 v = hs[b];
              if (r < c + v) {
                bst[j] = u32(b);
                cle[j] = c;
                cmi[j] = v;
                cur[4 * j + 0] = 0;
                cur[4 * j + 1] = c;
                cur[4 * j + 2] = c + v;
                break;
              }
              c += v;
            }
          }
        }
      }
      __syncthreads();
      // zones -> reserved slots (LDS cursors), in place: all reads of `slot` are done
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const u32 sid = sl[i] >> 16;
        const bool act = sid != kDone;
        u32 z = 0;
        if (act) {
          const float* cl = cc + (sid * dim + axis) * 2;
          const BucketParams prm = make_params(cl[0], cl[1], B);
          const u32 b = bucket_of(kf[i], prm, B);
          const u32 bs = bst[sid];
          z = b < bs ? 0u : (b == bs ? 1u : 2u);
        }
        const u32 d = reserve(sid * 4 + z, act, cur);
        np[i] = 0xffffffffu;
        if (act) {
          np[i] = (sub[sid] >> 16) + d;
          const u32 nsid = z == 0 ? 2 * sid : (z == 2 ? 2 * sid + 1 : (kMid | sid));
          ns[i] = (sl[i] & 0xffffu) | (nsid << 16);
        }
      }
#pragma unroll
      for (int i = 0; i < ITEMS; ++i)
        if (np[i] != 0xffffffffu) slot[np[i]] = ns[i];
      for (int b = tid; b < NM / 2; b += THREADS) hist[b] = 0;  // for the next level
      __syncthreads();
      // exact (key, id) ranking inside each median bucket; the median fixes the cells
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const int p = tid + i * THREADS;
        np[i] = 0xffffffffu;
        const u32 s = p < n ? slot[p] : (kDone << 16);
        const u32 tag = s >> 16;
        if (tag != kDone && (tag & kMid)) {
          const u32 sid = tag & 0x7fffu;
          const u32 idx = s & 0xffffu;
          const u32 e = sub[sid];
          const u32 jn = e & 0xffffu;
          const u32 zlo = (e >> 16) + cle[sid], zc = cmi[sid];
          const float mkf = kcol[idx];
          const u32 mk = orderable(mkf);
          const u32 mid = idrow[idx];
          // the zone holds ~2 points on average: gather up to 8 with independent loads
          constexpr int kZ = 8;
          u32 oi[kZ];
#pragma unroll
          for (int k = 0; k < kZ; ++k) oi[k] = u32(k) < zc ? (slot[zlo + k] & 0xffffu) : idx;
          u32 rank = 0;
#pragma unroll
          for (int k = 0; k < kZ; ++k) {
            const u32 qk = orderable(kcol[oi[k]]);
            const u32 qi = idrow[oi[k]];
            rank += (qk < mk || (qk == mk && qi < mid)) ? 1u : 0u;
          }
          for (u32 q = zlo + kZ; q < zlo + zc; ++q) {
            const u32 o = slot[q] & 0xffffu;
            const u32 qk = orderable(kcol[o]);
            rank += (qk < mk || (qk == mk && idrow[o] < mid)) ? 1u : 0u;
          }
          const u32 t = jn / 2 - cle[sid];
          const u32 nsid = rank < t ? 2 * sid : (rank > t ? 2 * sid + 1 : kDone);
          np[i] = zlo + rank;
          ns[i] = idx | (nsid << 16);
          if (rank == t && more) {
            const float* pc = cc + sid * dim * 2;
            float* lc = nc + (2 * sid) * dim * 2;
            float* rc = nc + (2 * sid + 1) * dim * 2;
            for (int c = 0; c < dim; ++c) {
              const float clo = pc[2 * c], chi = pc[2 * c + 1];
              lc[2 * c] = clo;
              lc[2 * c + 1] = c == axis ? mkf : chi;
              rc[2 * c] = c == axis ? mkf : clo;
              rc[2 * c + 1] = chi;
            }
          }
        }
      }
      __syncthreads();
      float* t = cc;
      cc = nc;
      nc = t;
    } else {
      // ---------------- counting path (sub-segments of <= kSmall points) ----------------
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const int p = tid + i * THREADS;
        if ((sl[i] >> 16) != kDone) keyv[p] = orderable(kf[i]);
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        np[i] = 0xffffffffu;
        const u32 sid = sl[i] >> 16;
        if (sid != kDone) {
          const u32 idx = sl[i] & 0xffffu;
          const u32 e = sub[sid];
          const u32 jlo = e >> 16, jn = e & 0xffffu;
          const u32 mk = orderable(kf[i]);
          u32 qk[kSmall];
#pragma unroll
          for (int k = 0; k < kSmall; ++k) qk[k] = k < int(jn) ? keyv[jlo + k] : 0xffffffffu;
          u32 rank = 0, ties = 0;
#pragma unroll
          for (int k = 0; k < kSmall; ++k) {
            rank += qk[k] < mk ? 1u : 0u;
            ties |= (k < int(jn) && qk[k] == mk && jlo + k != u32(tid + i * THREADS)) ? (1u << k) : 0u;
          }
          if (ties) {  // equal coordinates: order by id
            const u32 mid = idrow[idx];
            for (int k = 0; k < kSmall; ++k)
              if ((ties >> k) & 1u) rank += idrow[slot[jlo + k] & 0xffffu] < mid ? 1u : 0u;
          }
          const u32 half = jn / 2;
          const u32 nsid = rank < half ? 2 * sid : (rank > half ? 2 * sid + 1 : kDone);
          np[i] = jlo + rank;
          ns[i] = idx | (nsid << 16);
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < ITEMS; ++i)
      if (np[i] != 0xffffffffu) slot[np[i]] = ns[i];
    if (more) {
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const int j = tid + i * THREADS;
        if (j < S) {
          const u32 lo = ev[i] >> 16, m = ev[i] & 0xffffu;
          const u32 mr = m >= 1 ? m - m / 2 - 1 : 0u;
          sub[2 * j] = (lo << 16) | (m / 2);
          sub[2 * j + 1] = ((lo + m / 2 + 1) << 16) | mr;
        }
      }
    }
    __syncthreads();
  }
  // in-order rows out, AoS, coalesced
  const i64 total = i64(n) * dim;
  float* outp = a.out_pts + glo * dim;
  for (i64 f = tid; f < total; f += THREADS) {
    const int k = int(f / dim);
    const int c = int(f - i64(k) * dim);
    outp[f] = rows[c * NM + (slot[k] & 0xffffu)];
  }
  for (int k = tid; k < n; k += THREADS) a.out_ids[glo + k] = idrow[slot[k] & 0xffffu];
}

template <int ITEMS, int THREADS>
void launch_cfg(const SubArgs& a, i64 segs, hipStream_t stream) {
  static bool attr_set = false;
  const size_t lds = subtree_lds_bytes(a.dim, ITEMS * THREADS);
  if (!attr_set) {
    PKD_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_subtree<ITEMS, THREADS>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, int(kLdsMax)));
    attr_set = true;
  }
  k_subtree<ITEMS, THREADS><<<dim3(unsigned(segs)), THREADS, lds, stream>>>(a);
  PKD_LAUNCH_CHECK();
}

}  // namespace

int subtree_capacity(int dim) {
  // Prefer two workgroups per CU (LDS <= ~78 KiB) so one block's barriers hide behind the
  // other's work; fall back to smaller capacities for high dimensions.
  for (int nm = 2048; nm >= 64; nm /= 2)
    if (subtree_lds_bytes(dim, nm) <= kLdsMax / 2) return nm;
  for (int nm = 64; nm >= 32; nm /= 2)
    if (subtree_lds_bytes(dim, nm) <= kLdsMax) return nm;
  throw std::invalid_argument("pkdtree: dimension too large for the LDS subtree kernel");
}

int subtree_capacity_max(int dim) {
  for (int nm = 4096; nm >= 32; nm /= 2)
    if (subtree_lds_bytes(dim, nm) <= kLdsMax) return nm;
  throw std::invalid_argument("pkdtree: dimension too large for the LDS subtree kernel");
}

void launch_subtree(const float* cols, i64 ncol, int dim, const i64* seg_lo, const i64* seg_n, const float* cells,
                    i64 heap0, i64 segs, int depth_base, int nmax, float* out_pts, u32* out_ids, u32* err,
                    hipStream_t stream) {
  if (segs <= 0) return;
  SubArgs a{cols, ncol, dim, seg_lo, seg_n, cells, heap0, depth_base, out_pts, out_ids, err};
  if (nmax > 2048) launch_cfg<4, 1024>(a, segs, stream);
  else if (nmax > 1024) launch_cfg<4, 512>(a, segs, stream);
  else if (nmax > 512) launch_cfg<4, 256>(a, segs, stream);
  else if (nmax > 256) launch_cfg<2, 256>(a, segs, stream);
  else if (nmax > 128) launch_cfg<1, 256>(a, segs, stream);
  else if (nmax > 64) launch_cfg<1, 128>(a, segs, stream);
  else launch_cfg<1, 64>(a, segs, stream);
}

}  // namespace pkdtree
