// Rank subtree kernel ("wave" kernel): one workgroup finishes a segment of at most NM points
// (all levels below the global ones), for compile-time dims 1..8.
//
//   1. init    : one bucket-counting sort per axis over the whole segment gives every point its
//                root rank under the (orderable(key), id) order on every axis -- the only key
//                comparisons of the kernel. Ranks are never updated afterwards.
//   2. block levels (sub-segments larger than a wave): a sub-segment's members set their bits
//                in one bitmap over the root-rank space of the level's axis; one wave per
//                sub-segment scans its bitmap's word popcounts; a point's rank inside its
//                sub-segment is then one prefix read plus a popcount. Rank == n/2 is the
//                median (its slot lo + n/2 is final), smaller goes left. Two barriers a level.
//   3. wave levels (every sub-segment at most 64 points): each wave takes whole sub-segments,
//                one point per lane, turns root ranks into ranks inside the sub-segment once
//                (a 64-word bitmap and a wave scan per axis), then every level is one 64-bit
//                ds_or, one read and a popcount per point -- no workgroup barrier at all.
// The slot -> point table is streamed out at the end with coalesced stores. The reference
// spends these levels in std::sort calls and `new Node`s (kdtree_sequential.cpp:30-66).
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "device_utils.hpp"
#include "pkdtree/hip_check.hpp"
#include "subtree.hpp"
#include "subtree_common.hpp"

namespace pkdtree {
namespace {
using namespace subtree_detail;
using dev::BucketParams;
using dev::bucket_of;
using dev::make_params;
using dev::mbcnt;

using u8 = unsigned char;
constexpr int kWaveSeg = 64;  // sub-segments of at most this many points are finished by one wave

__host__ __device__ constexpr int cmax(int a, int b) { return a > b ? a : b; }

// LDS layout in 32-bit words. Persistent: rows (D keys + id bits) and the slot -> point table;
// one scratch region reused by the init, block-level and wave-level phases.
template <int D, int ITEMS, int THREADS>
struct WL {
  static constexpr int NM = ITEMS * THREADS;
  static constexpr int W = THREADS / 64;
  static constexpr int NA = D <= 3 ? D : 2;  // axes ranked per init pass
  static constexpr int kFin = (D + 1) * NM;            // u16 [NM]
  static constexpr int kScr = kFin + NM / 2;
  // init
  static constexpr int kHist = kScr;                   // u32 [NA * NM + 1], then the scan's wave sums
  static constexpr int kHistW = kHist + NA * NM + 2;   // u32 [W]
  static constexpr int kList = kHistW + W;             // u16 [NA * NM]
  static constexpr int kInitEnd = kList + NA * NM / 2;
  // block levels: bitmaps over the root-rank space, one per sub-segment (double-buffered by
  // level parity), and their word prefix counts
  static constexpr int NG = NM / 128 > 0 ? NM / 128 : 1;  // most sub-segments of a block level
  static constexpr int NW = NM / 32;                      // bitmap words
  static constexpr int kBm = kScr;                        // u32 [2][NG][NW]
  static constexpr int kPre = kBm + 2 * NG * NW;          // u32 [NG][NW]
  static constexpr int kBlockEnd = kPre + NG * NW;
  // transition (overlaps the block levels' scratch): points staged by sub-segment
  static constexpr int kStK = kScr;                       // u16 [NM] point index
  static constexpr int kStR = kStK + NM / 2;              // u16 [D][NM] root ranks
  static constexpr int kStEnd = kStR + D * NM / 2;
  // region B: per-sub-segment staging counters, later the waves' 64-bit masks
  static constexpr int kB0 = cmax(kBlockEnd, kStEnd);
  static constexpr int kB = kB0 + (kB0 & 1);
  static constexpr int kGcnt = kB;                        // u32 [NM / 64]
  static constexpr int kMask = kB;                        // u64 [W * ITEMS][64]
  static constexpr int kWaveEnd = kMask + W * ITEMS * 128;
  static constexpr int kWords = cmax(kInitEnd, cmax(kBlockEnd, kWaveEnd));
  static_assert(kMask % 2 == 0, "64-bit masks need 8-byte alignment");
};

// Exclusive scan of v[0, m) in place by the whole block (m = CPT * THREADS); v[m] = total.
template <int THREADS, int CPT>
__device__ __forceinline__ void block_scan(u32* v, u32* wsum) {
  constexpr int W = THREADS / 64;
  const int tid = threadIdx.x, w = tid / 64, ln = dev::lane();
  u32 x[CPT], s = 0;
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    x[j] = v[tid * CPT + j];
    s += x[j];
  }
  const u32 incl = dev::wave_incl_scan(s);
  if (ln == 63) wsum[w] = incl;
  __syncthreads();
  const u32 pin = dev::wave_incl_scan(ln < W ? wsum[ln < W ? ln : 0] : 0u);
  u32 run = (w > 0 ? u32(__builtin_amdgcn_readlane(int(pin), w - 1)) : 0u) + incl - s;
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    v[tid * CPT + j] = run;
    run += x[j];
  }
  if (tid == THREADS - 1) v[CPT * THREADS] = run;
}

template <int D, int ITEMS, int THREADS>
__device__ __forceinline__ void subtree_wave_body(const SubArgs& a) {
  using L = WL<D, ITEMS, THREADS>;
  constexpr int NM = L::NM, W = L::W, NA = L::NA;
  extern __shared__ __align__(16) u32 smem[];
  const i64 h = a.heap0 + blockIdx.x;
  const int n = int(a.seg_n[h]);
  if (n <= 0) return;
  const i64 glo = a.seg_lo[h];
  const int tid = threadIdx.x, w = tid / 64, ln = dev::lane();
  float* rows = reinterpret_cast<float*>(smem);
  const u32* idrow = reinterpret_cast<const u32*>(rows + D * NM);
  u16* fin = reinterpret_cast<u16*>(smem + L::kFin);
  // item i of a thread is point / slot position kid(i): each wave owns 64 * ITEMS consecutive ones
  const int kbase = w * 64 * ITEMS + ln;
  auto kid = [&](int i) { return kbase + i * 64; };
  const int db = a.depth_base;
  int lsub = 0;  // levels of the implicit subtree of n points
  for (u32 v = u32(n); v; v >>= 1) ++lsub;
  int T = 0;  // block levels: sub-segments larger than a wave
  while ((n >> T) > kWaveSeg) ++T;
  stamp(a, 0);

  // ---- rows -> LDS (every load of a thread issued before its LDS stores) ----
  {
    float v[D + 1][ITEMS];
#pragma unroll
    for (int c = 0; c <= D; ++c)
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const int k = tid + i * THREADS;
        v[c][i] = k < n ? a.cols[i64(c) * a.ncol + glo + k] : 0.0f;
      }
#pragma unroll
    for (int c = 0; c <= D; ++c)
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const int k = tid + i * THREADS;
        if (k < n) rows[c * NM + k] = v[c][i];
      }
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) fin[tid + i * THREADS] = 0xffffu;
  }
  __syncthreads();
  stamp(a, 1);

  // ---- 1. init: every point's rank on every axis over the whole segment ----
  // A register vector per point: an index the compiler cannot resolve becomes an indirect
  // register move (s_set_gpr_idx), never a scratch array.
  typedef u32 rvec __attribute__((ext_vector_type(D <= 4 ? 4 : 8)));
  rvec r[ITEMS];
  {
    u32* hist = smem + L::kHist;
    u32* hw = smem + L::kHistW;
    u16* list = reinterpret_cast<u16*>(smem + L::kList);
    const float* cells = a.cells + h * D * 2;
#pragma unroll
    for (int b0 = 0; b0 < D; b0 += NA) {
      constexpr int CPT = NA * ITEMS;  // scan entries per thread (NA * NM = CPT * THREADS)
#pragma unroll
      for (int j = 0; j < CPT; ++j) hist[tid * CPT + j] = 0u;
      __syncthreads();
      stamp(a, 24);
      u32 hb[NA][ITEMS], cb[NA][ITEMS];
#pragma unroll
      for (int b = 0; b < NA; ++b) {
        const int ax = b0 + b;
        if (ax >= D) continue;
        const BucketParams pr = make_params(cells[2 * ax], cells[2 * ax + 1], NM);
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
          const int k = kid(i);
          if (k < n) {
            hb[b][i] = u32(b * NM) + bucket_of(rows[ax * NM + k], pr, NM);
            cb[b][i] = atomicAdd(&hist[hb[b][i]], 1u);
          }
        }
      }
      __syncthreads();
      stamp(a, 25);
      block_scan<THREADS, CPT>(hist, hw);
      __syncthreads();
      // bucket ranges and positions into registers; the histogram's storage then takes the
      // orderable keys in bucket order, so a comparison is one LDS read (ids only on equal keys)
      // bucket start << 12 | bucket size (< 2^13 positions, <= 2048 points), and the position
      u32 sc[NA][ITEMS], pos[NA][ITEMS];
#pragma unroll
      for (int b = 0; b < NA; ++b) {
        if (b0 + b >= D) continue;
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
          const bool in = kid(i) < n;
          const u32 st = in ? hist[hb[b][i]] : 0u;
          sc[b][i] = (st << 12) | (in ? hist[hb[b][i] + 1] - st : 0u);
          pos[b][i] = st + (in ? cb[b][i] : 0u);
        }
      }
      __syncthreads();
      stamp(a, 26);
      u32* tk = hist;
#pragma unroll
      for (int b = 0; b < NA; ++b) {
        const int ax = b0 + b;
        if (ax >= D) continue;
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
          if (kid(i) < n) {
            tk[pos[b][i]] = orderable(rows[ax * NM + kid(i)]);
            list[pos[b][i]] = u16(kid(i));
          }
      }
      __syncthreads();
      stamp(a, 27);
      u32 id[ITEMS];
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) id[i] = kid(i) < n ? idrow[kid(i)] : 0u;
#pragma unroll
      for (int b = 0; b < NA; ++b) {
        const int ax = b0 + b;
        if (ax >= D) continue;
        u32 less[ITEMS], mx = 0, st[ITEMS], cn[ITEMS], ok[ITEMS];
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
          less[i] = 0;
          st[i] = sc[b][i] >> 12;
          cn[i] = sc[b][i] & 0xfffu;
          ok[i] = kid(i) < n ? orderable(rows[ax * NM + kid(i)]) : 0u;
          mx = max(mx, cn[i]);
        }
        mx = dev::wave_max_u32(mx);  // wave-uniform trip count: the wave's largest bucket
        u32 eq[ITEMS];
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) eq[i] = 0;
        for (u32 j = 0; j < mx; ++j) {
#pragma unroll
          for (int i = 0; i < ITEMS; ++i) {
            const u32 v = tk[j < cn[i] ? st[i] + j : pos[b][i]];  // own key past the bucket end
            less[i] += v < ok[i] ? 1u : 0u;
            eq[i] += v == ok[i] ? 1u : 0u;
          }
        }
        // equal keys (rare): the id decides. Without ties a point counts its own key once as a
        // member and once per iteration past its bucket's end: eq = mx - cn + 1.
        bool tie[ITEMS], anyt = false;
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
          tie[i] = cn[i] > 0 && eq[i] > mx - cn[i] + 1;
          anyt |= tie[i];
        }
        if (__ballot(anyt)) {
#pragma unroll
          for (int i = 0; i < ITEMS; ++i) {
            if (!tie[i]) continue;
            for (u32 j = 0; j < cn[i]; ++j) {
              const u32 e = st[i] + j;
              if (e != pos[b][i] && tk[e] == ok[i]) less[i] += idrow[list[e]] < id[i] ? 1u : 0u;
            }
          }
        }
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
          const u32 v = st[i] - u32(b * n) + less[i];
#pragma unroll
          for (int c = 0; c < D; ++c)
            if (c == ax) r[i][c] = v;
        }
      }
      __syncthreads();  // hist / list are reused by the next pass or the block levels
    }
  }
  stamp(a, 20);

  // per-item sub-segment state: slot range [lo, lo + nn) (nn = 0: finished), index g in its level
  u32 lo[ITEMS], nn[ITEMS], g[ITEMS];
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    lo[i] = 0;
    nn[i] = kid(i) < n ? u32(n) : 0u;
    g[i] = 0;
  }
  const int nw = (n + 31) >> 5;  // bitmap words over the root-rank space (<= 64)
  u32* gcnt = smem + L::kGcnt;

  // ---- 2. block levels ----
  {
    u32* bm = smem + L::kBm;
    u32* pre = smem + L::kPre;
    if (T > 0) {
      for (int j = tid; j < nw; j += THREADS) bm[j] = 0u;  // level 0's bitmap (parity 0)
    } else if (tid < 64) {
      gcnt[tid] = 0u;
    }
    __syncthreads();
    for (int t = 0; t < T; ++t) {
      const int ax = (db + t) % D;
      const int G = 1 << t;
      u32* bmt = bm + (t & 1) * L::NG * L::NW;
      // bits of the sub-segments' members
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        if (nn[i] == 0) continue;
        const u32 ra = r[i][ax];
        atomicOr(&bmt[g[i] * L::NW + (ra >> 5)], 1u << (ra & 31));
      }
      __syncthreads();
      // wave w scans the word popcounts of sub-segment w; the next level's bitmaps (the other
      // parity, last read before this level's first barrier) or the staging counters are reset
      if (w < G) {
        const u32 v = ln < nw ? u32(__popc(bmt[w * L::NW + ln])) : 0u;
        const u32 inc = dev::wave_incl_scan(v);
        if (ln < nw) pre[w * L::NW + ln] = inc - v;
      }
      if (t + 1 < T) {
        u32* bmn = bm + ((t + 1) & 1) * L::NG * L::NW;
        for (int j = tid; j < 2 * G * L::NW; j += THREADS) bmn[j] = 0u;
      } else if (tid < 2 * G) {
        gcnt[tid] = 0u;
      }
      __syncthreads();
      // rank inside the sub-segment: median, left or right
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        if (nn[i] == 0) continue;
        const u32 ra = r[i][ax], q = g[i] * L::NW + (ra >> 5);
        const u32 rank = pre[q] + u32(__popc(bmt[q] & ((1u << (ra & 31)) - 1u)));
        const u32 mid = nn[i] >> 1;
        if (rank == mid) {
          fin[lo[i] + mid] = u16(kid(i));
          nn[i] = 0;
        } else if (rank < mid) {
          nn[i] = mid;
          g[i] = 2 * g[i];
        } else {
          lo[i] += mid + 1;
          nn[i] -= mid + 1;
          g[i] = 2 * g[i] + 1;
        }
      }
      stamp(a, 2 + t);
    }
  }
  __syncthreads();  // the block levels' bitmaps become the staging area

  // ---- 3. wave levels: whole sub-segments per wave, one point per lane ----
  {
    u16* stk = reinterpret_cast<u16*>(smem + L::kStK);
    u16* str = reinterpret_cast<u16*>(smem + L::kStR);
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      if (nn[i] == 0) continue;
      const u32 p = lo[i] + atomicAdd(&gcnt[g[i]], 1u);  // a slot of the sub-segment
      stk[p] = u16(kid(i));
#pragma unroll
      for (int b = 0; b < D; ++b) str[b * NM + p] = u16(r[i][b]);
    }
    __syncthreads();
    stamp(a, 21);
    u64* masks = reinterpret_cast<u64*>(smem + L::kMask) + w * ITEMS * 64;
    u32 glo_[ITEMS], k_[ITEMS];
    bool in[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      // sub-segment gi of level T: heap node 2^T - 1 + gi of the segment's implicit tree
      const int gi = w * ITEMS + i;
      u32 slo = 0, sn = 0;
      if (gi < (1 << T)) {
        sn = u32(n);
        for (int bit = T - 1; bit >= 0; --bit) {
          if ((gi >> bit) & 1) {
            slo += (sn >> 1) + 1;
            sn = sn - (sn >> 1) - 1;
          } else {
            sn >>= 1;
          }
        }
      }
      glo_[i] = slo;
      in[i] = u32(ln) < sn;
      lo[i] = slo;
      nn[i] = in[i] ? sn : 0u;
      k_[i] = in[i] ? stk[slo + ln] : 0u;
#pragma unroll
      for (int b = 0; b < D; ++b) r[i][b] = in[i] ? u32(str[b * NM + slo + ln]) : 0u;
    }
    // root ranks -> ranks inside the sub-segment (< 64): a 64-word bitmap per item and axis
    u32* wb = reinterpret_cast<u32*>(masks);
#pragma unroll
    for (int b = 0; b < D; ++b) {
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) wb[i * 128 + ln] = 0u;
      wave_sync();
#pragma unroll
      for (int i = 0; i < ITEMS; ++i)
        if (in[i]) atomicOr(&wb[i * 128 + (r[i][b] >> 5)], 1u << (r[i][b] & 31));
      wave_sync();
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const u32 word = wb[i * 128 + ln];
        const u32 c = u32(__popc(word));
        const u32 ex = dev::wave_incl_scan(c) - c;
        const int q = int(r[i][b] >> 5);
        const u32 pq = u32(__shfl(int(ex), q, 64)), wq = u32(__shfl(int(word), q, 64));
        r[i][b] = pq + u32(__popc(wq & ((1u << (r[i][b] & 31)) - 1u)));
      }
      wave_sync();
    }
    stamp(a, 22);
    // Every level, per item: the point of rank p on the level's axis hands its sub-segment tag
    // (index inside the wave's range + 1) to lane p (ds_permute); lanes holding equal tags are
    // found with one ballot per tag bit; a point's rank inside its sub-segment is the count of
    // equal tags below its rank's lane (ds_bpermute back). No LDS memory, no barrier.
    u32 sub[ITEMS];  // sub-segment index inside the wave's range at the current level
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) sub[i] = 0;
    for (int t = T; t < lsub; ++t) {
      bool any = false;
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) any |= nn[i] != 0;
      if (!__ballot(any)) break;
      const int ax = (db + t) % D;
      const int bits = t - T + 1;  // tags are 1 .. 2^(t - T)
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const u32 ra = r[i][ax];
        const int addr = in[i] ? int(ra) : ln;  // lanes outside the range park on their own (unused) lane
        const u32 tag = u32(__builtin_amdgcn_ds_permute(addr * 4, nn[i] != 0 ? int(sub[i] + 1) : 0));
        u64 eqm = ~0ull;
        for (int bt = 0; bt < bits; ++bt) {
          const bool on = (tag >> bt) & 1u;
          const u64 bm = __ballot(on);
          eqm &= on ? bm : ~bm;
        }
        const u32 below = mbcnt(eqm);  // equal tags in lanes (= ranks) below this lane
        const u32 rank = u32(__builtin_amdgcn_ds_bpermute(addr * 4, int(below)));
        if (nn[i] == 0) continue;
        const u32 mid = nn[i] >> 1;
        if (rank == mid) {
          fin[lo[i] + mid] = u16(k_[i]);
          nn[i] = 0;
        } else if (rank < mid) {
          nn[i] = mid;
          sub[i] = 2 * sub[i];
        } else {
          lo[i] += mid + 1;
          nn[i] -= mid + 1;
          sub[i] = 2 * sub[i] + 1;
        }
      }
    }
  }
  stamp(a, 23);
  __syncthreads();
  stamp(a, 30);

  // ---- in-order rows out (consecutive threads cover consecutive 4*D-byte runs) ----
  float* outp = a.out_pts + glo * D;
  for (int k = tid; k < n; k += THREADS) {
    u32 p = fin[k];
    if (p >= u32(n)) {
      report(a.err, 0x1000u, u32(k), p);
      p = 0;
    }
#pragma unroll
    for (int c = 0; c < D; ++c) outp[i64(k) * D + c] = rows[c * NM + p];
    a.out_ids[glo + k] = idrow[p];
  }
  stamp(a, 31);
}

template <int D, int ITEMS, int THREADS>
__global__ __launch_bounds__(THREADS) void k_subtree_wave(SubArgs a) {
  subtree_wave_body<D, ITEMS, THREADS>(a);
}

// Same kernel held to 64 VGPRs (8 waves per SIMD: two 1024-thread workgroups per CU) for the
// dims whose rank vectors would otherwise take a 65th register.
template <int D, int ITEMS, int THREADS>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(8))) void k_subtree_wave8(SubArgs a) {
  subtree_wave_body<D, ITEMS, THREADS>(a);
}

template <int D, int ITEMS, int THREADS>
void launch_wave(const SubArgs& a, i64 segs, hipStream_t stream) {
  const size_t lds = size_t(WL<D, ITEMS, THREADS>::kWords) * 4;
  constexpr bool tight = D >= 4;
  const void* fn = tight ? reinterpret_cast<const void*>(&k_subtree_wave8<D, ITEMS, THREADS>)
                         : reinterpret_cast<const void*>(&k_subtree_wave<D, ITEMS, THREADS>);
  ensure_dynamic_lds(fn, int(lds));
  if constexpr (tight) k_subtree_wave8<D, ITEMS, THREADS><<<dim3(unsigned(segs)), THREADS, lds, stream>>>(a);
  else k_subtree_wave<D, ITEMS, THREADS><<<dim3(unsigned(segs)), THREADS, lds, stream>>>(a);
  PKD_LAUNCH_CHECK();
}

template <int D>
bool launch_dim(const SubArgs& a, i64 segs, int nmax, hipStream_t stream) {
  if (nmax > 2048) return false;
  if (nmax > 1024) {
    if constexpr (size_t(WL<D, 2, 1024>::kWords) * 4 <= 80 * 1024) {
      launch_wave<D, 2, 1024>(a, segs, stream);
      return true;
    }
    return false;
  }
  if (nmax > 512) launch_wave<D, 1, 1024>(a, segs, stream);
  else if (nmax > 256) launch_wave<D, 1, 512>(a, segs, stream);
  else if (nmax > 128) launch_wave<D, 1, 256>(a, segs, stream);
  else if (nmax > 64) launch_wave<D, 1, 128>(a, segs, stream);
  else launch_wave<D, 1, 64>(a, segs, stream);
  return true;
}

}  // namespace

// Opt-in (PKD_SUBTREE_IMPL=wave): same-box A/B at 100M x 3D / 8D puts it within 1-2% of the
// per-level ranking kernel (profiles/r2_subtree_wave_ab.txt), so the older kernel stays default.
bool subtree_wave_enabled() {
  const char* e = std::getenv("PKD_SUBTREE_IMPL");  // read per launch: tests switch it in-process
  return e && std::string(e) == "wave";
}

bool launch_subtree_wave(const SubArgs& a, i64 segs, int nmax, hipStream_t stream) {
  switch (a.dim) {
    case 1: return launch_dim<1>(a, segs, nmax, stream);
    case 2: return launch_dim<2>(a, segs, nmax, stream);
    case 3: return launch_dim<3>(a, segs, nmax, stream);
    case 4: return launch_dim<4>(a, segs, nmax, stream);
    case 5: return launch_dim<5>(a, segs, nmax, stream);
    case 6: return launch_dim<6>(a, segs, nmax, stream);
    case 7: return launch_dim<7>(a, segs, nmax, stream);
    case 8: return launch_dim<8>(a, segs, nmax, stream);
    default: return false;
  }
}

}  // namespace pkdtree
