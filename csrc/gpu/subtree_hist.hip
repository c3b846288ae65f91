// Cross-check subtree kernel (PKD_SUBTREE_IMPL=hist): the older histogram-partition LDS
// kernel, kept out of the shipping translation unit (build_subtree.hip). Same contract as
// k_subtree_rank -- one workgroup builds a segment's whole subtree in LDS -- so the two give
// slot-for-slot identical trees (tests/test_gpu_build.py runs both).
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
#include "device_utils.hpp"
#include "pkdtree/hip_check.hpp"
#include "subtree.hpp"
#include "subtree_common.hpp"

namespace pkdtree {

using dev::BucketParams;
using dev::bucket_of;
using dev::make_params;
using dev::mbcnt;

namespace {
using namespace subtree_detail;

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

constexpr int kWaveMax = 256;   // sub-segments of at most this many points are finished by one wave
constexpr int kWI = kWaveMax / 64;

// LDS views shared by the block phase and the wave phase.
struct Lds {
  float* rows;   // [(dim+1)][NM] fixed rows (column dim = id bits)
  u32* slot;     // [NM] idx | sid << 16 (sid = kDone once final)
  u32* keyv;     // [NM] orderable keys by slot (counting levels)
  u32* sub;      // [NM] (lo << 16) | n per sub-segment
  u32* hist;     // [NM/2]
  u32* st;       // [NM/2]
  float* cellA;  // [NM/8][dim][2]
  float* cellB;  // [NM/8][dim][2]
};

// One wave builds the whole subtree of the sub-segment [lo0, lo0+n0) (n0 <= kWaveMax) whose
// root sits at absolute depth `depth0`, with no workgroup barrier: every LDS region it
// touches is private to the wave and LDS operations of one wave execute in order.
//   wsub  : local sub-segment table (rel_lo << 16 | n), n0 entries (aliases sub + lo0)
//   whist : 128 bins; wst: 128 words of per-sub-segment state; wcA/wcB: 2 x [16][dim][2]
__device__ void wave_build(const Lds& L, int NM, int dim, int lo0, int n0, int depth0, u32* wsub, u32* whist,
                           u32* wst, float* wcA, float* wcB, u32* err) {
  const int ln = dev::lane();
  const u32* idrow = reinterpret_cast<const u32*>(L.rows + dim * NM);
  u32* bst = wst;
  u32* cle = wst + 16;
  u32* cmi = wst + 32;
  u32* bas = wst + 48;  // [3][16]
  float* plo = reinterpret_cast<float*>(wst + 96);
  float* psc = reinterpret_cast<float*>(wst + 112);
  if (ln == 0) wsub[0] = u32(n0);
  // the block phase left its own sub-segment ids in the slots: restart at local id 0
  for (int q = ln; q < n0; q += 64) {
    const u32 sv = L.slot[lo0 + q];
    if ((sv >> 16) != kDone) L.slot[lo0 + q] = sv & 0xffffu;
  }
  const int rows_used = (n0 + 63) / 64;  // wave-uniform: rows of 64 slots that exist
  for (int t = 0;; ++t) {
    const int m = n0 >> t;
    if (m == 0) break;
    const int S = 1 << t;
    const int axis = (depth0 + t) % dim;
    const float* kcol = L.rows + axis * NM;
    const bool more = (n0 >> (t + 1)) > 0;
    u32 sl[kWI];
    float kf[kWI];
#pragma unroll
    for (int k = 0; k < kWI; ++k) {
      const int q = ln + 64 * k;
      sl[k] = (k < rows_used && q < n0) ? L.slot[lo0 + q] : (kDone << 16);
    }
#pragma unroll
    for (int k = 0; k < kWI; ++k) kf[k] = ((sl[k] >> 16) != kDone) ? kcol[sl[k] & 0xffffu] : 0.0f;
    u32 ev[kWI];
#pragma unroll
    for (int k = 0; k < kWI; ++k) {
      const int j = ln + 64 * k;
      ev[k] = (more && j < S) ? wsub[j] : 0u;
    }
    u32 np[kWI], ns[kWI];
    if (m > kSmall) {
      const int B = min(64, max(2, pow2_floor_dev(m / 2)));  // S * B <= n0 / 2 <= 128
      if (ln < S) {
        cmi[ln] = 0;
        cle[ln] = 0xffffffffu;
        const float* c = wcA + (ln * dim + axis) * 2;
        const BucketParams pr = make_params(c[0], c[1], B);
        plo[ln] = pr.lo;
        psc[ln] = pr.scale;
      }
      for (int b = ln; b < S * B; b += 64) whist[b] = 0;
      u32 bk[kWI];
#pragma unroll
      for (int k = 0; k < kWI; ++k) {
        const u32 sid = sl[k] >> 16;
        bk[k] = 0;
        if (sid != kDone) {
          BucketParams pr;
          pr.lo = plo[sid];
          pr.scale = psc[sid];
          bk[k] = bucket_of(kf[k], pr, B);
          atomicAdd(&whist[sid * B + bk[k]], 1u);
        }
      }
      {  // select: lane l owns bins [2l, 2l+2); sub-segment j owns lanes [j*B/2, (j+1)*B/2)
        const int nb = S * B;
        const int b0 = 2 * ln;
        const u32 sum = b0 < nb ? whist[b0] + whist[b0 + 1] : 0u;
        const u32 incl = dev::wave_incl_scan(sum);
        const u32 ex = incl - sum;
        const int js = b0 / B;
        const u32 segbase = __shfl(ex, min(63, js * (B / 2)), 64);
        if (b0 < nb) {
          const u32 r = (wsub[js] & 0xffffu) / 2;
          const u32 rel = ex - segbase;
          if (r >= rel && r < rel + sum) {
            const u32 v0 = whist[b0];
            const bool first = r < rel + v0;
            bst[js] = (first ? u32(b0) : u32(b0 + 1)) - u32(js * B);  // bucket index within js
            cle[js] = first ? rel : rel + v0;
            cmi[js] = first ? v0 : whist[b0 + 1];
          }
        }
      }
      if (ln < S) {  // every sub-segment must have found its median bucket
        const u32 r = (wsub[ln] & 0xffffu) / 2;
        if (cle[ln] == 0xffffffffu || r < cle[ln] || r >= cle[ln] + cmi[ln]) report(err, 0x100u | u32(ln), u32(t), wsub[ln]);
      }
      // zone prefixes over the wave's slots (rows of 64 in slot order) with ballots
      u32 zk[kWI], pz[kWI];
      u32 run0 = 0, run1 = 0, run2 = 0;
#pragma unroll
      for (int k = 0; k < kWI; ++k) {
        const u32 sid = sl[k] >> 16;
        u32 z = 3;
        if (sid != kDone) {
          const u32 bs = bst[sid];
          z = bk[k] < bs ? 0u : (bk[k] == bs ? 1u : 2u);
        }
        zk[k] = z;
        const u64 m0 = __ballot(z == 0), m1 = __ballot(z == 1), m2 = __ballot(z == 2);
        const u32 p0 = run0 + mbcnt(m0), p1 = run1 + mbcnt(m1), p2 = run2 + mbcnt(m2);
        pz[k] = z == 0 ? p0 : (z == 1 ? p1 : p2);
        if (z < 3 && u32(ln + 64 * k) == (wsub[sid] >> 16)) {  // first slot of its sub-segment
          bas[sid] = p0;
          bas[16 + sid] = p1;
          bas[32 + sid] = p2;
        }
        run0 += __popcll(m0);
        run1 += __popcll(m1);
        run2 += __popcll(m2);
      }
#pragma unroll
      for (int k = 0; k < kWI; ++k) {
        np[k] = 0xffffffffu;
        const u32 z = zk[k];
        if (z < 3) {
          const u32 sid = sl[k] >> 16;
          const u32 start = z == 0 ? 0u : (z == 1 ? cle[sid] : cle[sid] + cmi[sid]);
          np[k] = (wsub[sid] >> 16) + start + pz[k] - bas[16 * z + sid];
          if (np[k] - (wsub[sid] >> 16) >= (wsub[sid] & 0xffffu)) {
            report(err, 0x200u | z, u32(t), np[k]);
            np[k] = 0xffffffffu;
          }
          const u32 nsid = z == 0 ? 2 * sid : (z == 2 ? 2 * sid + 1 : (kMid | sid));
          ns[k] = (sl[k] & 0xffffu) | (nsid << 16);
        }
      }
#pragma unroll
      for (int k = 0; k < kWI; ++k)
        if (np[k] != 0xffffffffu) L.slot[lo0 + np[k]] = ns[k];
      // exact ranking inside each median bucket
#pragma unroll
      for (int k = 0; k < kWI; ++k) {
        const int q = ln + 64 * k;
        np[k] = 0xffffffffu;
        const u32 s = q < n0 ? L.slot[lo0 + q] : (kDone << 16);
        const u32 tag = s >> 16;
        if (tag != kDone && (tag & kMid)) {
          const u32 sid = tag & 0x7fffu;
          const u32 idx = s & 0xffffu;
          const u32 e = wsub[sid];
          const u32 jn = e & 0xffffu;
          const u32 zlo = (e >> 16) + cle[sid], zc = cmi[sid];
          const float mkf = kcol[idx];
          const u32 mk = orderable(mkf);
          const u32 mid = idrow[idx];
          u32 rank = 0;
#pragma unroll 4
          for (u32 r = 0; r < zc && r < 4096u; ++r) {
            const u32 o = L.slot[lo0 + zlo + r] & 0xffffu;
            const u32 qk = orderable(kcol[o]);
            rank += (qk < mk || (qk == mk && idrow[o] < mid)) ? 1u : 0u;
          }
          const u32 tt = jn / 2 - cle[sid];
          const u32 nsid = rank < tt ? 2 * sid : (rank > tt ? 2 * sid + 1 : kDone);
          np[k] = zlo + rank;
          ns[k] = idx | (nsid << 16);
          if (rank == tt && more) {
            const float* pc = wcA + sid * dim * 2;
            float* lc = wcB + (2 * sid) * dim * 2;
            float* rc = wcB + (2 * sid + 1) * dim * 2;
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
      float* tmp = wcA;
      wcA = wcB;
      wcB = tmp;
    } else {
      // counting: each point counts the smaller (key, id) of its sub-segment (<= kSmall)
#pragma unroll
      for (int k = 0; k < kWI; ++k)
        if ((sl[k] >> 16) != kDone) L.keyv[lo0 + ln + 64 * k] = orderable(kf[k]);
#pragma unroll
      for (int k = 0; k < kWI; ++k) {
        np[k] = 0xffffffffu;
        const u32 sid = sl[k] >> 16;
        if (sid != kDone) {
          const u32 idx = sl[k] & 0xffffu;
          const u32 e = wsub[sid];
          const u32 jlo = e >> 16, jn = e & 0xffffu;
          const u32 mk = orderable(kf[k]);
          u32 rank = 0;
          const u32 self = u32(ln + 64 * k) - jlo;
#pragma unroll 8
          for (u32 r = 0; r < jn; ++r) {
            const u32 qk = L.keyv[lo0 + jlo + r];
            rank += (qk < mk || (qk == mk && r != self && idrow[L.slot[lo0 + jlo + r] & 0xffffu] < idrow[idx])) ? 1u : 0u;
          }
          const u32 half = jn / 2;
          const u32 nsid = rank < half ? 2 * sid : (rank > half ? 2 * sid + 1 : kDone);
          np[k] = jlo + rank;
          ns[k] = idx | (nsid << 16);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kWI; ++k)
      if (np[k] != 0xffffffffu) L.slot[lo0 + np[k]] = ns[k];
    if (more) {
#pragma unroll
      for (int k = 0; k < kWI; ++k) {
        const int j = ln + 64 * k;
        if (j < S) {
          const u32 lo = ev[k] >> 16, mm = ev[k] & 0xffffu;
          const u32 mr = mm >= 1 ? mm - mm / 2 - 1 : 0u;
          wsub[2 * j] = (lo << 16) | (mm / 2);
          wsub[2 * j + 1] = ((lo + mm / 2 + 1) << 16) | mr;
        }
      }
    }
  }
}

template <int ITEMS, int THREADS>
__global__ __launch_bounds__(THREADS) void k_subtree(SubArgs a) {
  extern __shared__ __align__(16) u32 smem[];
  constexpr int NM = ITEMS * THREADS;
  constexpr int W = THREADS / 64;
  const int dim = a.dim;
  const i64 h = a.heap0 + blockIdx.x;
  const int n = int(a.seg_n[h]);
  if (n <= 0) return;
  const i64 glo = a.seg_lo[h];
  Lds L;
  L.rows = reinterpret_cast<float*>(smem);
  L.slot = smem + size_t(dim + 1) * NM;
  L.keyv = L.slot + NM;
  L.sub = L.keyv + NM;
  L.hist = L.sub + NM;
  L.st = L.hist + NM / 2;
  L.cellA = reinterpret_cast<float*>(L.st + NM / 2);
  L.cellB = L.cellA + (NM / 8) * dim * 2;
  float* rows = L.rows;
  u32* slot = L.slot;
  u32* sub = L.sub;
  u32* hist = L.hist;
  constexpr int SB = NM / 16;
  u32* bst = L.st;
  u32* cle = L.st + SB;
  u32* cmi = L.st + 2 * SB;
  u32* cur = L.st + 4 * SB;  // [SB][4]
  const int tid = threadIdx.x;
  const int w = tid / 64;
  const u32* idrow = reinterpret_cast<const u32*>(rows + dim * NM);
  stamp(a, 0);

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
  for (int c = tid; c < 2 * dim; c += THREADS) L.cellA[c] = a.cells[h * 2 * dim + c];
  __syncthreads();
  stamp(a, 1);
  float* cc = L.cellA;  // cells of the current level
  float* nc = L.cellB;  // cells of the next level

  // ---------------- block phase: sub-segments larger than one wave's share ----------------
  int l = 0;
  for (;; ++l) {
    const int ml = n >> l;
    if (ml <= kWaveMax) break;
    const int S = 1 << l;
    const int axis = (a.depth_base + l) % dim;
    const float* kcol = rows + axis * NM;
    u32 sl[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const int p = tid + i * THREADS;
      sl[i] = p < n ? slot[p] : (kDone << 16);
    }
    float kf[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) kf[i] = ((sl[i] >> 16) != kDone) ? kcol[sl[i] & 0xffffu] : 0.0f;
    u32 ev[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const int j = tid + i * THREADS;
      ev[i] = j < S ? sub[j] : 0u;
    }
    u32 np[ITEMS], ns[ITEMS];
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
    for (int b = tid; b < NM / 2; b += THREADS) hist[b] = 0;
    __syncthreads();
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
        constexpr int kZ = 8;
        u32 oi[kZ];
#pragma unroll
        for (int k = 0; k < kZ; ++k) oi[k] = u32(k) < zc ? (slot[zlo + k] & 0xffffu) : idx;
        u32 rank = 0;
#pragma unroll
        for (int k = 0; k < kZ; ++k) {
          const u32 qk = orderable(kcol[oi[k]]);
          rank += (qk < mk || (qk == mk && idrow[oi[k]] < mid)) ? 1u : 0u;
        }
        for (u32 q = zlo + kZ; q < zlo + zc && q < zlo + 4096u; ++q) {
          const u32 o = slot[q] & 0xffffu;
          const u32 qk = orderable(kcol[o]);
          rank += (qk < mk || (qk == mk && idrow[o] < mid)) ? 1u : 0u;
        }
        const u32 t = jn / 2 - cle[sid];
        const u32 nsid = rank < t ? 2 * sid : (rank > t ? 2 * sid + 1 : kDone);
        np[i] = zlo + rank;
        ns[i] = idx | (nsid << 16);
        if (rank == t) {
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
#pragma unroll
    for (int i = 0; i < ITEMS; ++i)
      if (np[i] != 0xffffffffu) slot[np[i]] = ns[i];
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
    float* t = cc;
    cc = nc;
    nc = t;
    __syncthreads();
  }

  stamp(a, 2);
  // ---------------- wave phase: every sub-segment (<= kWaveMax) to one wave ----------------
  {
    const int S0 = 1 << l;  // <= W by construction (NM <= W * kWaveMax)
    const u32 e = w < S0 ? sub[w] : 0u;
    __syncthreads();  // the wave-private tables below alias the block table
    if (w < S0 && (e & 0xffffu) > 0) {
      const int lo0 = int(e >> 16), n0 = int(e & 0xffffu);
      float* wcA = nc + w * 64 * dim;  // the non-current cell buffer is free now
      float* wcB = wcA + 32 * dim;
      for (int c = dev::lane(); c < 2 * dim; c += 64) wcA[c] = cc[w * 2 * dim + c];
      wave_build(L, NM, dim, lo0, n0, a.depth_base + l, sub + lo0, hist + w * 128, L.st + w * 128, wcA, wcB, a.err);
    }
  }
  __syncthreads();
  stamp(a, 30);
  // in-order rows out, AoS, coalesced
  const i64 total = i64(n) * dim;
  float* outp = a.out_pts + glo * dim;
  for (i64 f = tid; f < total; f += THREADS) {
    const int k = int(f / dim);
    const int c = int(f - i64(k) * dim);
    outp[f] = rows[c * NM + (slot[k] & 0xffffu)];
  }
  for (int k = tid; k < n; k += THREADS) a.out_ids[glo + k] = idrow[slot[k] & 0xffffu];
  __syncthreads();
  stamp(a, 31);
  (void)W;
}

template <int ITEMS, int THREADS>
void launch_cfg(const SubArgs& a, i64 segs, hipStream_t stream) {
  const size_t lds = subtree_lds_bytes(a.dim, ITEMS * THREADS);
  ensure_dynamic_lds(reinterpret_cast<const void*>(&k_subtree<ITEMS, THREADS>), int(kLdsMax));
  k_subtree<ITEMS, THREADS><<<dim3(unsigned(segs)), THREADS, lds, stream>>>(a);
  PKD_LAUNCH_CHECK();
}

}  // namespace

size_t subtree_hist_lds_bytes(int dim, int nm) { return subtree_lds_bytes(dim, nm); }

void launch_subtree_hist(const SubArgs& a, i64 segs, int nmax, hipStream_t stream) {
  if (nmax > 2048) launch_cfg<4, 1024>(a, segs, stream);
  else if (nmax > 1024) launch_cfg<4, 512>(a, segs, stream);
  else if (nmax > 512) launch_cfg<4, 256>(a, segs, stream);
  else if (nmax > 256) launch_cfg<2, 256>(a, segs, stream);
  else if (nmax > 128) launch_cfg<1, 256>(a, segs, stream);
  else if (nmax > 64) launch_cfg<1, 128>(a, segs, stream);
  else launch_cfg<1, 64>(a, segs, stream);
}

}  // namespace pkdtree
