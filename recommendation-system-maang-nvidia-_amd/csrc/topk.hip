// topk.hip — exact brute-force inner-product top-K over an item table (row-sharded capable).
//
// Reference: ProductionTrainer._evaluate (src/trainer.py:204-212: sims = np.dot(user_embs,
// item_embs.T); np.argpartition(-sim, k)[:k]) and the FAISS IndexFlatIP search of
// _build_faiss / RecommendationService (src/trainer.py:240-243,
// app/recommendation_service.py:71-72). Output order is the build contract of SURVEY A.8:
// (-score, index) ascending, so the result is a deterministic function of the scores.
//
// Stage 1 (scan) is a GEMM S = items . Q^T with a selecting epilogue. A 4-wave workgroup owns
// WQ query tiles of QT queries (register-resident, one tile per wave) and a contiguous slice of
// items. The slice streams through one LDS tile of IT = (4/WQ) x QT rows, loaded with fully
// coalesced 16-B pieces (one 512-B row per 32 lanes) and prefetched into registers a tile ahead;
// wave w scores item sub-tile w / WQ against query tile w % WQ with v_mfma_f32_32x32x2_f32
// (QT = 32, > 64 queries) or v_mfma_f32_16x16x4_f32 (QT = 16), reading the A operand with one
// conflict-free ds_read_b128 per 4 MFMAs (k-permuted like the queries). Scores are exact fp32:
// on dyadic-grid data every score is exact, so indices are bit-exact vs the CPU oracle.
// Few queries: the 4 waves split the items (HBM-bound scan, every byte read once); many
// queries: they split the queries and share every item row staged in LDS (MFMA-bound).
//
// Selection is threshold filtering. Each (query, wave sub-slice) keeps a sorted top-k list in
// the per-slice output (global memory) and carries the (score, index) of its k-th entry in
// registers; the rare item that beats it is appended to the wave's LDS candidate buffer. When
// a buffer could overflow on the next tile the wave compacts that query: the buffer is
// bitonic-sorted across the wave's lanes (register shuffles) and merged by rank with the list.
// A full list's k-th score is also a bound for the whole query (at least k items reach it), so
// compaction publishes it with an atomic max and takes back the best bound any slice has
// published; items below it are not appended. Stage 2 merges the per-slice lists.
#include "common.hpp"
#include "split.hpp"

#include <cmath>

namespace rs {

constexpr int TK_KMAX = 128;
constexpr int TK_MERGE = 4096;  // entries sorted per merge workgroup
#ifndef TK_WGS
#define TK_WGS 512              // scan workgroups per launch (2 resident per CU)
#endif

__device__ __forceinline__ bool tk_better(float s, int64_t i, float ts, int64_t ti) {
  return s > ts || (s == ts && i < ti);
}

__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// order-preserving int32 key of a float (for atomicMax) and its inverse
__device__ __forceinline__ int32_t tk_key(float f) {
  const int32_t u = __float_as_int(f);
  return u ^ ((u >> 31) & 0x7fffffff);
}
__device__ __forceinline__ float tk_unkey(int32_t kk) { return __int_as_float(kk ^ ((kk >> 31) & 0x7fffffff)); }


template <int QT>
struct TkAcc;
template <>
struct TkAcc<32> {
  using T = f32x16;
  static constexpr int N = 16;
  __device__ static int row(int r, int slot) { return acc_row(r, slot); }
  __device__ static T mma(float a, float b, T c) { return mfma32x32x2(a, b, c); }
};
template <>
struct TkAcc<16> {
  using T = f32x4;
  static constexpr int N = 4;
  __device__ static int row(int r, int slot) { return 4 * slot + r; }
  __device__ static T mma(float a, float b, T c) { return mfma16x16x4(a, b, c); }
};

template <int D, int QT, int WQ, int IPW, int NP = 0>
struct TkGeo {
  static constexpr int NS = 64 / QT;                      // MFMA k slots = lanes per query
  static constexpr int TI = QT;                           // items per wave sub-tile
  static constexpr int IS = 4 / WQ;                       // waves sharing a query tile
  static constexpr int IT = IS * IPW * TI;                // items per LDS tile (IPW sub-tiles per wave)
  static constexpr int KP = D + 4;                        // LDS row stride (floats)
  static constexpr int NG = D / (4 * NS);                 // b128 operand reads per lane per sub-tile
  // candidate buffer entries per query (40 with split operands: their 24-KB tile image must
  // leave room for 2 workgroups per CU)
  static constexpr int CB = QT == 32 ? (NP ? 40 : 48) : 64;
  static constexpr int CBS = CB + 1;
  static constexpr int NF4 = IT * D / 4;                  // float4 pieces per LDS tile
  static constexpr int NLD = (NF4 + 255) / 256;           // per thread
};

constexpr int TK_POOLJ = 4;     // a list publishes its 4th-best score to the query's pool
constexpr int TK_POOLN = 256;   // lists (sub-slices) per query that publish

#ifdef RS_TOPK_EXP_STATS
__device__ unsigned long long tk_stats[8];  // compactions, compaction cycles, appends, scan cycles, waves
#endif

struct TkNew {
  float ts;   // new k-th entry (valid when nl == k)
  int32_t ti;
  int nl;     // valid list entries
  float tg;   // query-wide bound
};

// Merge one query's candidate buffer (cq <= 64 entries, unsorted) into its sorted list (lq <= k
// entries, global memory; positions p = lane, lane + 64 are always read and written by the same
// lane) and refresh the query-wide bound. Wave-cooperative, out of line (the scan loop's
// registers are not shaped by this rare path), and free of memory fences: the wave's LDS
// accesses execute in order, so only the compiler needs fencing, and the global stores and the
// bound's atomic are left in flight.
//
// Ranks instead of a sort: a buffer entry's rank is the number of buffer entries better than it
// (broadcast LDS reads) plus its insertion point in the sorted list (binary search); a list
// entry's rank is its position plus the number of better buffer entries. Entries are distinct
// items, so the ranks of real entries are distinct; sentinels only collide with sentinels.
//
// Bound: every list of the query publishes its 4th-best score to pool_q (lists cover disjoint
// items). If r = ceil(k / 4) lists each hold 4 items scoring >= x then at least k items do, so
// the r-th largest published score bounds the query's k-th score from below: items below it are
// never appended. This tracks the best ~k items of ALL lists together (a list's own k-th only
// tracks its own slice), which cuts appends ~10x; it is also published to tau for lists that
// rarely compact (they refresh from it periodically).
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void lds_order() { __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __noinline__ TkNew topk_compact(const float* bufs, const int32_t* bufi, int cq, int lq, int k,
                                           float* Ls, int32_t* Li, float* scs, int32_t* sci, int32_t* tau,
                                           int32_t* pool_q, int pool_n, int my_pool) {
  const int lane = threadIdx.x & 63;
  // the LDS arguments arrive as generic pointers (out-of-line call): re-qualify them so the
  // accesses are ds_read/ds_write, not flat operations that also wait on the vector memory count
  using lf = __attribute__((address_space(3))) float;
  using li = __attribute__((address_space(3))) int32_t;
  lf* ls_ = (lf*)scs;
  lf* ns_ = (lf*)scs + TK_KMAX;
  lf* bs_ = (lf*)scs + 2 * TK_KMAX;
  li* li_ = (li*)sci;
  li* ni_ = (li*)sci + TK_KMAX;
  li* bi_ = (li*)sci + 2 * TK_KMAX;
  const lf* bufs_l = (const lf*)bufs;
  const li* bufi_l = (const li*)bufi;
  using gf = __attribute__((address_space(1))) float;
  using gi = __attribute__((address_space(1))) int32_t;
  gf* Lsg = (gf*)Ls;
  gi* Lig = (gi*)Li;
  gi* poolg = (gi*)pool_q;
  // global reads first: the list and the pool
  float lv[TK_KMAX / 64];
  int32_t lvi[TK_KMAX / 64];
#pragma unroll
  for (int m = 0; m < TK_KMAX / 64; ++m) {
    const int p = lane + 64 * m;
    lv[m] = -INFINITY;
    lvi[m] = 0x7fffffff;
    if (p < lq) {
      lv[m] = Lsg[p];
      lvi[m] = Lig[p];
    }
  }
  int32_t pk[TK_POOLN / 64];
#pragma unroll
  for (int m = 0; m < TK_POOLN / 64; ++m) {
    const int p = lane + 64 * m;
    pk[m] = p < pool_n ? __hip_atomic_load(poolg + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : (int32_t)0x807fffff;
  }
  float xs = -INFINITY;
  int32_t xi = 0x7fffffff;
  if (lane < cq) {
    xs = bufs_l[lane];
    xi = bufi_l[lane];
  }
  bs_[lane] = xs;
  bi_[lane] = xi;
#pragma unroll
  for (int m = 0; m < TK_KMAX / 64; ++m) {
    ls_[lane + 64 * m] = lv[m];
    li_[lane + 64 * m] = lvi[m];
    const int p = lane + 64 * m;
    if (p >= lq + cq && p < k) {  // positions no entry will fill
      ns_[p] = -INFINITY;
      ni_[p] = 0x7fffffff;
    }
  }
  lds_order();
  // rank of my buffer entry
  if (lane < cq) {
    int r = 0;
#pragma unroll 4
    for (int j = 0; j < 64; j += 4) {
      const f32x4 s4 = *reinterpret_cast<const __attribute__((address_space(3))) f32x4*>(bs_ + j);
      const i32x4 i4 = *reinterpret_cast<const __attribute__((address_space(3))) i32x4*>(bi_ + j);
      r += tk_better(s4[0], i4[0], xs, xi) + tk_better(s4[1], i4[1], xs, xi) + tk_better(s4[2], i4[2], xs, xi) +
           tk_better(s4[3], i4[3], xs, xi);
    }
    int lo = 0, hi = lq;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (tk_better(ls_[mid], li_[mid], xs, xi)) lo = mid + 1; else hi = mid;
    }
    r += lo;
    if (r < k) {
      ns_[r] = xs;
      ni_[r] = xi;
    }
  }
  // ranks of my list entries
#pragma unroll
  for (int m = 0; m < TK_KMAX / 64; ++m) {
    const int p = lane + 64 * m;
    if (p < lq) {
      int r = p;
#pragma unroll 4
      for (int j = 0; j < 64; j += 4) {
        const f32x4 s4 = *reinterpret_cast<const __attribute__((address_space(3))) f32x4*>(bs_ + j);
        const i32x4 i4 = *reinterpret_cast<const __attribute__((address_space(3))) i32x4*>(bi_ + j);
        r += tk_better(s4[0], i4[0], lv[m], lvi[m]) + tk_better(s4[1], i4[1], lv[m], lvi[m]) +
             tk_better(s4[2], i4[2], lv[m], lvi[m]) + tk_better(s4[3], i4[3], lv[m], lvi[m]);
      }
      if (r < k) {
        ns_[r] = lv[m];
        ni_[r] = lvi[m];
      }
    }
  }
  lds_order();
#pragma unroll
  for (int m = 0; m < TK_KMAX / 64; ++m) {
    const int p = lane + 64 * m;
    if (p < k) {
      Lsg[p] = ns_[p];
      Lig[p] = ni_[p];
    }
  }
  TkNew out;
  out.nl = lq + cq < k ? lq + cq : k;
  out.ts = ns_[k - 1];
  out.ti = ni_[k - 1];
  // publish my 4th-best; fold it into the snapshot (the read above may predate it)
  if (my_pool >= 0 && out.nl >= TK_POOLJ) {
    const int32_t mine = tk_key(ns_[TK_POOLJ - 1]);
    if (lane == 0) poolg[my_pool] = mine;
#pragma unroll
    for (int m = 0; m < TK_POOLN / 64; ++m)
      if (lane + 64 * m == my_pool && mine > pk[m]) pk[m] = mine;
  }
  int32_t bkey = out.nl == k ? tk_key(out.ts) : (int32_t)0x807fffff;
  const int need = (k + TK_POOLJ - 1) / TK_POOLJ;
  if (pool_n >= need) {
    // r-th largest published key: greedy bit construction over the order-preserving unsigned keys
    uint32_t u[TK_POOLN / 64];
#pragma unroll
    for (int m = 0; m < TK_POOLN / 64; ++m) u[m] = (uint32_t)pk[m] ^ 0x80000000u;
    uint32_t ans = 0;
    for (int bit = 31; bit >= 0; --bit) {
      const uint32_t cand = ans | (1u << bit);
      int c = 0;
#pragma unroll
      for (int m = 0; m < TK_POOLN / 64; ++m) c += __popcll(__ballot(u[m] >= cand));
      if (c >= need) ans = cand;
    }
    const int32_t pkey = (int32_t)(ans ^ 0x80000000u);
    if (pkey > bkey) bkey = pkey;
  }
  if (lane == 0 && bkey != (int32_t)0x807fffff) atomicMax(tau, bkey);
  out.tg = tk_unkey(bkey);
  lds_order();
  return out;
}

// NP > 0 (precision 6 / 9, D = 128, QT = 32, one 32-item sub-tile per LDS tile): the item tile is
// split at staging into the three bf16 plane images of split.hpp and the queries' planes sit in
// registers; the scores come from v_mfma_f32_32x32x16_bf16 with NP products per fp32 product
// (same accumulator layout, so the selection below is unchanged).
template <int D, int QT, int WQ, int IPW, int NP>
__global__ __launch_bounds__(256) void topk_scan_kernel(const float* __restrict__ Q, int64_t nq,
                                                        const float* __restrict__ items, int64_t N,
                                                        int k, int64_t per_split, int64_t nsplit,
                                                        int64_t nqb, float* __restrict__ cand_s,
                                                        int32_t* __restrict__ cand_i,
                                                        int32_t* __restrict__ tau_key,
                                                        int32_t* __restrict__ pool, int pool_n) {
  using G = TkGeo<D, QT, WQ, IPW, NP>;
  using Acc = TkAcc<QT>;
  static_assert(NP == 0 || (D == IBX_D && QT == 32 && G::IT == 32), "split top-k: D = 128, 32-item tiles");
  __shared__ __attribute__((aligned(16))) float tile[NP ? IBX_BUF / 4 : G::IT * G::KP];
  __shared__ float cs[4][QT * G::CBS];
  __shared__ int32_t ci[4][QT * G::CBS];
  __shared__ float scs[4][2 * TK_KMAX + 64];
  __shared__ int32_t sci[4][2 * TK_KMAX + 64];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wq = w % WQ, wi = w / WQ;
  const int qs = lane & (QT - 1);  // my query (B column) and my item row (A row) in a sub-tile
  const int slot = lane / QT;      // my MFMA k slot
  int64_t qb, split;
  const int64_t b = blockIdx.x;
  if ((nsplit & 7) == 0) {  // XCD-aware: the query blocks of one slice share an XCD (and its L2)
    const int64_t loc = b >> 3;
    qb = loc % nqb;
    split = (loc / nqb) * 8 + (b & 7);
  } else {
    qb = b % nqb;
    split = b / nqb;
  }
  const int64_t qtile = qb * WQ + wq;
  const int64_t q = qtile * QT + qs;
  const bool qvalid = q < nq;
  const int64_t i0 = split * per_split;
  const int64_t i1 = (i0 + per_split < N) ? i0 + per_split : N;
  const int e1 = (int)i1;  // item indices fit in int32 (N < 2^31 per call)
  const int64_t nvs = nsplit * G::IS, vs = split * G::IS + wi;

  // queries: qf[4g + t] = Q[q][4 NS g + 4 slot + t] (the same k permutation as the tile reads)
  float qf[NP ? 1 : D / G::NS];
  u32x4 qp[NP ? D / 16 : 1][3];  // split: chunk c = Q[q][16c + 8 slot + j], j < 8
  if constexpr (NP == 0) {
#pragma unroll
    for (int g = 0; g < G::NG; ++g) {
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (qvalid) v = *reinterpret_cast<const f32x4*>(Q + q * D + 4 * G::NS * g + 4 * slot);
#pragma unroll
      for (int t = 0; t < 4; ++t) qf[4 * g + t] = v[t];
    }
  } else {
#pragma unroll
    for (int c = 0; c < D / 16; ++c) {
      f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = v0;
      if (qvalid) {
        v0 = *reinterpret_cast<const f32x4*>(Q + q * D + 16 * c + 8 * slot);
        v1 = *reinterpret_cast<const f32x4*>(Q + q * D + 16 * c + 8 * slot + 4);
      }
      const IbSplit x0 = ib_split2(v0[0], v0[1]), x1 = ib_split2(v0[2], v0[3]), x2 = ib_split2(v1[0], v1[1]),
                    x3 = ib_split2(v1[2], v1[3]);
      qp[c][0] = u32x4{x0.h, x1.h, x2.h, x3.h};
      qp[c][1] = u32x4{x0.m, x1.m, x2.m, x3.m};
      qp[c][2] = u32x4{x0.l, x1.l, x2.l, x3.l};
    }
  }

  float ts = -INFINITY;  // k-th entry of my (query, sub-slice) list; sentinel while it is short
  int32_t ti = 0x7fffffff;
  float tg = -INFINITY;  // query-wide bound
  int cnt = 0, ln = 0;   // buffered candidates / valid list entries

  f32x4 ld[G::NLD];
  auto gload = [&](int base) {
#pragma unroll
    for (int j = 0; j < G::NLD; ++j) {
      const int f = tid + 256 * j;
      if (G::NF4 % 256 == 0 || f < G::NF4) {
        int row = base + f / (D / 4);
        if (row >= e1) row = e1 - 1;  // clamped rows are never selected
        ld[j] = __builtin_nontemporal_load(
            reinterpret_cast<const f32x4*>(items + (int64_t)row * D + 4 * (f % (D / 4))));
      }
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int j = 0; j < G::NLD; ++j) {
      const int f = tid + 256 * j;
      if (G::NF4 % 256 == 0 || f < G::NF4) {
        if constexpr (NP == 0)
          *reinterpret_cast<f32x4*>(tile + (f / (D / 4)) * G::KP + 4 * (f % (D / 4))) = ld[j];
        else
          ibx_put4(reinterpret_cast<char*>(tile), f / (D / 4), f % (D / 4), ld[j]);
      }
    }
  };

  auto compact = [&](int qq) {
#ifdef RS_TOPK_EXP_STATS
    const long long c0 = clock64();
#endif
    const int cq = __shfl(cnt, qq);
    const int lq = __shfl(ln, qq);
    const int64_t qg = qtile * QT + qq;
    const TkNew r = topk_compact(&cs[w][qq * G::CBS], &ci[w][qq * G::CBS], cq, lq, k,
                                 cand_s + (qg * nvs + vs) * k, cand_i + (qg * nvs + vs) * k, scs[w], sci[w],
                                 tau_key + qg, pool + qg * pool_n, pool_n, vs < pool_n ? (int)vs : -1);
    if (qs == qq) {
      cnt = 0;
      ln = r.nl;
      if (r.tg > tg) tg = r.tg;
      if (r.nl == k) {
        ts = r.ts;
        ti = r.ti;
      }
    }
#ifdef RS_TOPK_EXP_STATS
    if (lane == 0) {
      atomicAdd(&tk_stats[0], 1ull);
      atomicAdd(&tk_stats[1], (unsigned long long)(clock64() - c0));
      atomicAdd(&tk_stats[2], (unsigned long long)cq);
    }
#endif
  };

  // every 16 tiles each lane refreshes its query's bound from tau (loaded with the next tile's
  // items, so the wait for it is the wait the LDS store makes anyway)
  const int32_t* tq = tau_key + (qvalid ? q : 0);
  int32_t tnext = (int32_t)0x807fffff;
  int tile_no = 0;
#ifdef RS_TOPK_EXP_STATS
  const long long k0 = clock64();
#endif
  int base = (int)i0;
  gload(base);
  lstore();
  __syncthreads();
  for (;;) {
    const int nb = base + G::IT;
    const bool more = nb < e1;
    if ((tile_no & 15) == 15) {
      const float t2 = tk_unkey(tnext);
      if (t2 > tg) tg = t2;
    }
    if ((tile_no & 15) == 14) tnext = __hip_atomic_load(tq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ++tile_no;
    if (more) gload(nb);
#pragma unroll 1
    for (int p = 0; p < IPW; ++p) {
      typename Acc::T acc;
#pragma unroll
      for (int r = 0; r < Acc::N; ++r) acc[r] = 0.f;
      if constexpr (NP == 0) {
        const float* trow = tile + ((wi * IPW + p) * G::TI + qs) * G::KP + 4 * slot;
        // all operand reads of the sub-tile are issued before the MFMAs (distinct registers), so
        // the LDS latency is paid once per tile rather than once per 4 MFMAs
        f32x4 a[G::NG];
#pragma unroll
        for (int g = 0; g < G::NG; ++g) a[g] = *reinterpret_cast<const f32x4*>(trow + 4 * G::NS * g);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < G::NG; ++g)
#pragma unroll
          for (int t = 0; t < 4; ++t) acc = Acc::mma(a[g][t], qf[4 * g + t], acc);
      } else {
        const char* img = reinterpret_cast<const char*>(tile);
        const int rb0 = 2048 * (qs >> 3) + 64 * (qs & 7) + 16 * (slot ^ ((qs >> 2) & 3));
        const int rb1 = 2048 * (qs >> 3) + 64 * (qs & 7) + 16 * ((2 + slot) ^ ((qs >> 2) & 3));
#pragma unroll
        for (int c = 0; c < D / 16; ++c) {
          u32x4 a[3];
#pragma unroll
          for (int pl = 0; pl < 3; ++pl)
            a[pl] = *reinterpret_cast<const u32x4*>(img + pl * IBX_PLANE + ((c & 1) ? rb1 : rb0) + 512 * (c >> 1));
          acc = mfma_split<NP>(a, qp[c], acc);
        }
      }
      // fast filter: an entry is selected only if it reaches both bounds, so a wave whose lanes'
      // largest scores of the sub-tile all stay below max(ts, tg) skips the per-entry test (one
      // max tree and one compare per lane per tile; -3 % at Q = 1024 on the split scan)
      float mx = acc[0];
#pragma unroll
      for (int r = 1; r < Acc::N; ++r) mx = fmaxf(mx, acc[r]);
      if (!__any(mx >= fmaxf(ts, tg))) continue;
      const int sb = base + (wi * IPW + p) * G::TI;
      int n = 0;
      unsigned mask = 0;
#pragma unroll
      for (int r = 0; r < Acc::N; ++r) {
        const int item = sb + Acc::row(r, slot);
        const float v = acc[r];
#ifdef RS_TOPK_EXP_NOSEL  // experiment build: scan cost without selection
        const bool c = qvalid & (item < e1) & (v > 3.0e38f);
#else
        const bool c = qvalid & (item < e1) & ((v > ts) | ((v == ts) & (item < ti))) & (v >= tg);
#endif
        mask |= (unsigned)c << r;
        n += c;
      }
      if (__any(n)) {  // rare after warm-up
        int before = 0, total = 0;
#pragma unroll
        for (int m = 0; m < G::NS; ++m) {
          const int nm = __shfl(n, qs + QT * m);
          total += nm;
          if (m < slot) before += nm;
        }
        int pos = cnt + before;
#pragma unroll
        for (int r = 0; r < Acc::N; ++r) {
          if ((mask >> r) & 1u) {
            cs[w][qs * G::CBS + pos] = acc[r];
            ci[w][qs * G::CBS + pos] = sb + Acc::row(r, slot);
            ++pos;
          }
        }
        cnt += total;
        lds_order();
        uint64_t need = __ballot(slot == 0 && cnt > G::CB - G::TI);
        while (need) {
          const int qq = __ffsll((unsigned long long)need) - 1;
          need &= need - 1;
          compact(qq);
        }
      }
    }
    if (!more) break;
    __syncthreads();
    lstore();
    __syncthreads();
    base = nb;
  }
  // lists start as sentinels (memset by the host), so only buffered candidates need a final merge
  uint64_t need = __ballot(slot == 0 && qvalid && cnt > 0);
  while (need) {
    const int qq = __ffsll((unsigned long long)need) - 1;
    need &= need - 1;
    compact(qq);
  }
#ifdef RS_TOPK_EXP_STATS
  if (lane == 0) {
    atomicAdd(&tk_stats[3], (unsigned long long)(clock64() - k0));
    atomicAdd(&tk_stats[4], 1ull);
  }
#endif
}

// Merge `group` sorted lists of k entries per query into one (bitonic sort of <= 4096 entries).
// With a query bound (the scan's final tau: at least k items reach it), entries below it are
// dropped while loading, so a workgroup sorts only the survivors (typically a few hundred of
// its 4096 entries).
template <typename IdxT>
__device__ __forceinline__ IdxT tk_sentinel() { return (IdxT)(sizeof(IdxT) == 4 ? 0x7fffffffLL : 0x7fffffffffffffffLL); }

template <typename IdxT>
__global__ __launch_bounds__(256) void topk_merge_kernel(const float* __restrict__ in_s,
                                                         const IdxT* __restrict__ in_i,
                                                         int64_t nlists, int k, int group,
                                                         int64_t nout, float* __restrict__ out_s,
                                                         IdxT* __restrict__ out_i,
                                                         float* __restrict__ fin_s,
                                                         int64_t* __restrict__ fin_i,
                                                         int64_t index_base,
                                                         const int32_t* __restrict__ bound) {
  __shared__ float ss[TK_MERGE];
  __shared__ IdxT si[TK_MERGE];
  __shared__ int nsurv;
  const int64_t q = blockIdx.y, o = blockIdx.x;
  const int64_t l0 = o * group;
  int64_t l1 = l0 + group;
  if (l1 > nlists) l1 = nlists;
  const int m = (int)((l1 - l0) * k);
  const IdxT SENT = tk_sentinel<IdxT>();
  int msurv = m;
  if (bound) {
    const float b = tk_unkey(bound[q]);
    if (threadIdx.x == 0) nsurv = 0;
    __syncthreads();
    for (int e = threadIdx.x; e < m; e += 256) {
      const float v = in_s[(q * nlists + l0) * k + e];
      const IdxT vi = in_i[(q * nlists + l0) * k + e];
      if (v >= b && vi != SENT) {
        const int slot = atomicAdd(&nsurv, 1);
        ss[slot] = v;
        si[slot] = vi;
      }
    }
    __syncthreads();
    msurv = nsurv;
  } else {
    for (int e = threadIdx.x; e < m; e += 256) {
      ss[e] = in_s[(q * nlists + l0) * k + e];
      si[e] = in_i[(q * nlists + l0) * k + e];
    }
  }
  int P = 1;
  while (P < msurv || P < k) P <<= 1;
  for (int e = msurv + threadIdx.x; e < P; e += 256) {
    ss[e] = -INFINITY;
    si[e] = SENT;
  }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int e = threadIdx.x; e < P / 2; e += 256) {
        const int lo = 2 * stride * (e / stride) + (e % stride), hi = lo + stride;
        const bool desc = (lo & size) == 0;  // blocks alternate direction; final pass: best first
        const bool hb = tk_better(ss[hi], (int64_t)si[hi], ss[lo], (int64_t)si[lo]);
        if (hb == desc) {
          const float ts = ss[lo];
          const IdxT ti = si[lo];
          ss[lo] = ss[hi];
          si[lo] = si[hi];
          ss[hi] = ts;
          si[hi] = ti;
        }
      }
      __syncthreads();
    }
  }
  for (int j = threadIdx.x; j < k; j += 256) {
    if (fin_s) {
      fin_s[q * k + j] = ss[j];
      fin_i[q * k + j] = si[j] == SENT ? (int64_t)-1 : (int64_t)si[j] + index_base;
    } else {
      out_s[(q * nout + o) * k + j] = ss[j];
      out_i[(q * nout + o) * k + j] = si[j];
    }
  }
}

template <typename IdxT>
static int merge_rounds(float* s0, IdxT* i0, float* s1, IdxT* i1, int64_t nq, int64_t nl, int k,
                        int64_t index_base, float* out_s, int64_t* out_i, const int32_t* bound,
                        hipStream_t st) {
  const int group = TK_MERGE / k;
  while (true) {
    const int64_t nout = ceil_div(nl, group);
    const bool last = nout == 1;
    hipLaunchKernelGGL((topk_merge_kernel<IdxT>), dim3((unsigned)nout, (unsigned)nq), dim3(256), 0, st, s0,
                       i0, nl, k, group, nout, s1, i1, last ? out_s : nullptr,
                       last ? out_i : nullptr, index_base, bound);
    int rc = check_launch("topk_merge");
    if (rc || last) return rc;
    float* ts = s0; s0 = s1; s1 = ts;
    IdxT* ti = i0; i0 = i1; i1 = ti;
    nl = nout;
  }
}

// ---- threshold scan (the bound-first top-K below) -------------------------------------------
// The scan of topk_scan_kernel<D = 128, QT = 32, WQ = 4, IPW = 1, NP> with its selection replaced by a
// fixed per-query bound: no lists and no merge scratch, so the item tile is double-buffered in LDS
// (one barrier per tile: tile t + 1 is split into the other buffer, from registers loaded during
// tile t - 1, while tile t is scored). A wave whose 32 x 32 sub-tile maxima all stay below the bounds
// skips the per-entry test. The rare entries that reach the bound go to the wave's flat LDS buffer
// (score, item, query) by ballot + mbcnt; a full buffer is copied to the queries' candidate slots
// in global memory (one slot reservation per entry: app_n[q] counts, cap slots per query), so the
// global stores and their atomics stay rare and the tile loads' counted waits seldom cover them.
constexpr int TT_CAPB = 128;   // flat candidate buffer entries per wave

// NTL: non-temporal item loads (timing experiment only: the 8 query blocks of a slice share an
// XCD, and plain loads let them share each item line in its L2 — 7.4 vs 34.9 GB of HBM-side
// traffic and -6 % time at Q = 1024 on a 12.5M-row shard)
// NW: waves per workgroup (each its own 32 queries, all sharing the item tile): 4, or 8 so that one
// tile load + split feeds twice the MFMA work. SUB: 32-row sub-tiles per tile (one barrier per tile;
// a wave scores its sub-tiles with independent accumulator chains, interleaved)
// The bound-first scan's permuted block order (bs > 0): the table is cut into n blocks of bs rows and
// logical block b is physical block (a b + c) mod n (a coprime to n); range j of the scan is a run
// of logical blocks, one slice per block, so every range is a sample of blocks from the whole table
// and an item order correlated with the scores (rows sorted by norm or popularity) does not make
// every later range beat the earlier ranges' k-th score. bs = 0: slices of one contiguous range.
constexpr int TK_BLOCK_ROWS = 2048;  // rows per block of the permuted order (= the first range)
struct TkBlocks {
  int64_t bs, lo, hi, n, a, c, bpw, spb;  // block rows; the range's logical blocks [lo, hi); blocks in
                                          // the table; the permutation (a, c); blocks per workgroup;
                                          // workgroups per block (> 1: a block split in equal parts)
};

template <int NP, bool NTL = false, int NW = 4, int SUB = 1>
__global__ __launch_bounds__(64 * NW) void topk_thr_kernel(const float* __restrict__ Q, int64_t nq,
                                                       const float* __restrict__ items, int64_t N,
                                                       int64_t per_split, int64_t nsplit, int64_t nqb,
                                                       const float* __restrict__ thr, int64_t thr_ld,
                                                       int32_t* __restrict__ app_n, float* __restrict__ app_s,
                                                       int32_t* __restrict__ app_i, int cap, TkBlocks bk) {
  constexpr int D = IBX_D, QT = 32, TI = 32 * SUB;
  constexpr int NT = 64 * NW;
  constexpr int NLD = TI * D / 4 / NT;  // float4 pieces per thread per tile
  __shared__ __attribute__((aligned(16))) char tile[2][SUB][IBX_BUF];
  __shared__ float bs[NW][TT_CAPB];
  __shared__ int32_t bi[NW][TT_CAPB];
  __shared__ int32_t bq[NW][TT_CAPB];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int qs = lane & (QT - 1), slot = lane / QT;
  int64_t qb, split;
  const int64_t b = blockIdx.x;
  if ((nsplit & 7) == 0) {  // XCD-aware: the query blocks of one slice share an XCD (and its L2)
    const int64_t loc = b >> 3;
    qb = loc % nqb;
    split = (loc / nqb) * 8 + (b & 7);
  } else {
    qb = b % nqb;
    split = b / nqb;
  }
  const int64_t qtile = qb * NW + w;
  const int64_t q = qtile * QT + qs;
  const bool qvalid = q < nq;
  const int64_t i0 = split * per_split;
  const int64_t i1 = (i0 + per_split < N) ? i0 + per_split : N;
  // the workgroup's tiles: slice [i0, i1) of a contiguous range, or (permuted block order) the
  // tiles of its logical blocks [lb0, lb1), each block's physical rows; rows >= e1 are masked
  // the workgroup's tiles: slice [i0, i1) of a contiguous range, or (permuted block order) bpw
  // whole logical blocks from lo + split bpw, or (spb > 1) the sub-th of spb equal parts of block
  // lo + split / spb; rows >= e1 are masked. Tile rows come from an incremental walk of the
  // permutation (one 64-bit modulo per workgroup; per tile an add and a compare)
  constexpr int TPB = TK_BLOCK_ROWS / TI;  // tiles per block
  int64_t ntile = (i1 - i0 + TI - 1) / TI;
  int seg = 1 << 30, tile0 = 0, ld_pb = (int)i0, pbn = 0;  // tiles per block segment, first tile, row
  if (bk.bs > 0) {
    int64_t lb0, nblk;
    if (bk.spb > 1) {
      lb0 = bk.lo + split / bk.spb;
      nblk = lb0 < bk.hi ? 1 : 0;
      seg = TPB / (int)bk.spb;
      tile0 = (int)(split % bk.spb) * seg;
    } else {
      lb0 = bk.lo + split * bk.bpw;
      const int64_t lb1 = lb0 + bk.bpw < bk.hi ? lb0 + bk.bpw : bk.hi;
      nblk = lb1 > lb0 ? lb1 - lb0 : 0;
      seg = TPB;
    }
    ntile = nblk * seg;
    pbn = (int)((bk.a * lb0 + bk.c) % bk.n);
    ld_pb = pbn * (int)bk.bs;
  }
  const int e1 = bk.bs > 0 ? (int)N : (int)i1;
  int ld_in = 0;
  auto next_row = [&]() -> int {  // the row of the next tile to load
    const int row = ld_pb + (tile0 + ld_in) * TI;
    if (++ld_in == seg) {
      ld_in = 0;
      pbn += (int)bk.a;
      if (pbn >= (int)bk.n) pbn -= (int)bk.n;
      ld_pb = pbn * (int)bk.bs;
    }
    return row;
  };

  u32x4 qp[D / 16][3];  // chunk c = Q[q][16c + 8 slot + j], j < 8, as three bf16 planes
#pragma unroll
  for (int c = 0; c < D / 16; ++c) {
    f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = v0;
    if (qvalid) {
      v0 = *reinterpret_cast<const f32x4*>(Q + q * D + 16 * c + 8 * slot);
      v1 = *reinterpret_cast<const f32x4*>(Q + q * D + 16 * c + 8 * slot + 4);
    }
    const IbSplit x0 = ib_split2(v0[0], v0[1]), x1 = ib_split2(v0[2], v0[3]), x2 = ib_split2(v1[0], v1[1]),
                  x3 = ib_split2(v1[2], v1[3]);
    qp[c][0] = u32x4{x0.h, x1.h, x2.h, x3.h};
    qp[c][1] = u32x4{x0.m, x1.m, x2.m, x3.m};
    qp[c][2] = u32x4{x0.l, x1.l, x2.l, x3.l};
  }
  const float tq = qvalid ? thr[q * thr_ld] : INFINITY;

  f32x4 ld[NLD];
  auto gload = [&](int base) {
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const int f = tid + NT * j;
      int row = base + f / (D / 4);
      if (row >= e1) row = e1 - 1;  // clamped rows are never selected
      const f32x4* src = reinterpret_cast<const f32x4*>(items + (int64_t)row * D + 4 * (f % (D / 4)));
      ld[j] = NTL ? __builtin_nontemporal_load(src) : *src;
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const int f = tid + NT * j;
      const int row = f / (D / 4);
      ibx_put4(tile[buf][row >> 5], row & 31, f % (D / 4), ld[j]);
    }
  };
  int bufn = 0;  // entries in my wave's buffer (wave-uniform)
  auto flush = [&]() {
    lds_order();
    for (int e = lane; e < bufn; e += 64) {
      const int64_t qg = qtile * QT + bq[w][e];
      const int pos = atomicAdd(app_n + qg, 1);
      if (pos < cap) {
        app_s[qg * cap + pos] = bs[w][e];
        app_i[qg * cap + pos] = bi[w][e];
      }
    }
    lds_order();
    bufn = 0;
  };

  if (ntile <= 0) return;  // (no barrier reached by any wave of this workgroup)
  int64_t t = 0;
  int base = next_row(), row1 = 0;
  gload(base);
  lstore(0);
  if (ntile > 1) {
    row1 = next_row();
    gload(row1);
  }
  __syncthreads();
  int cur = 0;
  const int rb0 = 2048 * (qs >> 3) + 64 * (qs & 7) + 16 * (slot ^ ((qs >> 2) & 3));
  const int rb1 = 2048 * (qs >> 3) + 64 * (qs & 7) + 16 * ((2 + slot) ^ ((qs >> 2) & 3));
  for (;;) {
    f32x16 accs[SUB];
#pragma unroll
    for (int h = 0; h < SUB; ++h)
#pragma unroll
      for (int r = 0; r < 16; ++r) accs[h][r] = 0.f;
#pragma unroll
    for (int c = 0; c < D / 16; ++c) {
#pragma unroll
      for (int h = 0; h < SUB; ++h) {
        const char* img = tile[cur][h];
        u32x4 a[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          a[pl] = *reinterpret_cast<const u32x4*>(img + pl * IBX_PLANE + ((c & 1) ? rb1 : rb0) + 512 * (c >> 1));
        accs[h] = mfma_split<NP>(a, qp[c], accs[h]);
      }
    }
#pragma unroll
    for (int h = 0; h < SUB; ++h) {
    const f32x16& acc = accs[h];
    const int hb = base + 32 * h;
    float mx = acc[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, acc[r]);
    if (__any(mx >= tq)) {
      unsigned mask = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        mask |= (unsigned)(qvalid & (hb + acc_row(r, slot) < e1) & (acc[r] >= tq)) << r;
      int total = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) total += __popcll(__ballot((mask >> r) & 1u));
      if (bufn + total > TT_CAPB) flush();
      if (total > TT_CAPB) {  // more than a buffer in one tile (the first range): straight to the slots
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if ((mask >> r) & 1u) {
            const int pos = atomicAdd(app_n + q, 1);
            if (pos < cap) {
              app_s[q * cap + pos] = acc[r];
              app_i[q * cap + pos] = hb + acc_row(r, slot);
            }
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint64_t bl = __ballot((mask >> r) & 1u);
          if (bl) {
            if ((mask >> r) & 1u) {
              const int pos = bufn + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bl >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)bl, 0u));
              bs[w][pos] = acc[r];
              bi[w][pos] = hb + acc_row(r, slot);
              bq[w][pos] = qs;
            }
            bufn += __popcll(bl);
          }
        }
      }
    }
    }
    if (t + 1 >= ntile) break;
    lstore(cur ^ 1);  // tile t + 1, loaded during tile t
    int row2 = 0;
    if (t + 2 < ntile) {
      row2 = next_row();
      gload(row2);
    }
    __syncthreads();
    cur ^= 1;
    ++t;
    base = row1;
    row1 = row2;
  }
  if (bufn > 0) flush();
}

// Scan configuration by query count: (QT, WQ, IPW) = (16, 1, 1) for <= 16 queries,
// (16, 2, 2) <= 32, (16, 4, 4) <= 64, else (32, 4, 1): 64-row LDS tiles below 64 queries.
static void topk_cfg(int64_t nq, int* qt, int* wq, int* ipw) {
  if (nq <= 16) { *qt = 16; *wq = 1; *ipw = 1; }
  else if (nq <= 32) { *qt = 16; *wq = 2; *ipw = 2; }
  else if (nq <= 64) { *qt = 16; *wq = 4; *ipw = 4; }
  else { *qt = 32; *wq = 4; *ipw = 1; }
}

// Slices: ~TK_WGS workgroups in all (2 resident per CU), each wave sub-slice at least
// max(32 k, 1024) items, a multiple of 8 when possible (XCD-aware mapping).
// th: a threshold scan (no lists to fill, so slices only need a few tiles: 256 items)
static void topk_geometry(int64_t nq, int64_t N, int k, int64_t* per, int64_t* nse, int64_t* nvs,
                          bool th = false) {
  int qt, wq, ipw;
  topk_cfg(nq, &qt, &wq, &ipw);
  const int64_t nqb = ceil_div(ceil_div(nq, qt), wq);
  const int is = 4 / wq;
  int64_t s = ceil_div(TK_WGS, nqb);
  int64_t minper = 32 * (int64_t)k;
  if (minper < 1024) minper = 1024;
  if (th) minper = 256;
  const int64_t maxs = N / (minper * is);
  if (s > maxs) s = maxs;
  if (s >= 8) s = s / 8 * 8;
  if (s < 1) s = 1;
  const int64_t it = (int64_t)is * ipw * qt;
  *per = ceil_div(ceil_div(N, s), it) * it;
  *nse = ceil_div(N, *per);
  *nvs = *nse * is;
}

template <int D, int QT, int WQ, int IPW, int NP = 0>
static void topk_launch(const float* Q, int64_t nq, const float* items, int64_t N, int k, int64_t per,
                        int64_t nse, float* s0, int32_t* i0, int32_t* tau, int32_t* pool, int pool_n,
                        hipStream_t st) {
  const int64_t nqb = ceil_div(ceil_div(nq, QT), WQ);
  hipLaunchKernelGGL((topk_scan_kernel<D, QT, WQ, IPW, NP>), dim3((unsigned)(nqb * nse)), dim3(256), 0, st, Q, nq,
                     items, N, k, per, nse, nqb, s0, i0, tau, pool, pool_n);
}

// Single-pass scan: per-(query, sub-slice) lists + merge rounds (every configuration).
template <int D>
static int topk_impl_lists(const float* Q, int64_t nq, const float* items, int64_t N, int k,
                           int64_t index_base, float* out_s, int64_t* out_i, void* ws, size_t wsb,
                           hipStream_t st, int prec = 0) {
  int64_t per, nse, nvs;
  topk_geometry(nq, N, k, &per, &nse, &nvs);
  Carve c(ws, wsb);
  const int pool_n = (int)(nvs < TK_POOLN ? nvs : TK_POOLN);
  int32_t* tau = c.take<int32_t>(nq + nq * pool_n);  // [nq] bounds, then [nq][pool_n] published keys
  int32_t* pool = tau + nq;
  RS_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(tau), (int)0x807fffff, (size_t)(nq + nq * pool_n),
                           st));  // key(-inf)
  float* s0 = c.take<float>(nq * nvs * k);
  int32_t* i0 = c.take<int32_t>(nq * nvs * k);
  RS_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(s0), (int)0xff800000, (size_t)(nq * nvs * k), st));
  RS_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(i0), 0x7fffffff, (size_t)(nq * nvs * k), st));
  float* s1 = c.take<float>(nq * nvs * k);
  int32_t* i1 = c.take<int32_t>(nq * nvs * k);
  int qt, wq, ipw;
  topk_cfg(nq, &qt, &wq, &ipw);
  if (qt == 16 && wq == 1) topk_launch<D, 16, 1, 1>(Q, nq, items, N, k, per, nse, s0, i0, tau, pool, pool_n, st);
  else if (qt == 16 && wq == 2) topk_launch<D, 16, 2, 2>(Q, nq, items, N, k, per, nse, s0, i0, tau, pool, pool_n, st);
  else if (qt == 16) topk_launch<D, 16, 4, 4>(Q, nq, items, N, k, per, nse, s0, i0, tau, pool, pool_n, st);
  else if (D == IBX_D && prec == 6)
    topk_launch<D, 32, 4, 1, (D == IBX_D ? 6 : 0)>(Q, nq, items, N, k, per, nse, s0, i0, tau, pool, pool_n, st);
  else if (D == IBX_D && prec == 9)
    topk_launch<D, 32, 4, 1, (D == IBX_D ? 9 : 0)>(Q, nq, items, N, k, per, nse, s0, i0, tau, pool, pool_n, st);
  else topk_launch<D, 32, 4, 1>(Q, nq, items, N, k, per, nse, s0, i0, tau, pool, pool_n, st);
  int rc = check_launch("topk_scan");
  if (rc) return rc;
  return merge_rounds<int32_t>(s0, i0, s1, i1, nq, nvs, k, index_base, out_s, out_i, tau, st);
}

static size_t topk_lists_workspace_bytes(int64_t nq, int64_t N, int k) {
  int64_t per, nse, nvs;
  topk_geometry(nq > 0 ? nq : 1, N > 0 ? N : 1, k > 0 ? k : 1, &per, &nse, &nvs);
  const size_t e = (size_t)(nq > 0 ? nq : 1) * nvs * (k > 0 ? k : 1);
  const size_t pn = (size_t)(nvs < TK_POOLN ? nvs : TK_POOLN);
  return align_up((size_t)(nq > 0 ? nq : 1) * (1 + pn) * 4, 256) + 2 * (align_up(e * 4, 256) + align_up(e * 4, 256)) +
         1024;
}

// ---- bound-first scan (many queries, large shards) ----------------------------------------
// The list scan above spends about a quarter of its time keeping 64 sub-slice lists per query
// sorted (compactions), because a list's own k-th entry only becomes a useful bound after its
// slice has produced k survivors. Here the bound comes first. The items are cut into ranges of
// 2048-row blocks taken in a fixed permuted block order (TkBlocks): 1 block, then 3, 12, 48, ...
// blocks (ratio 4), the last range ending with the table; range j is scanned by
// topk_scan_kernel<..., TH> against a fixed per-query bound T_j (no lists, no merge scratch: an
// item reaching T_j is buffered in LDS and copied to its (query, wave sub-slice) candidate slots),
// and the select kernel sorts the previous range's exact list with the candidates under
// (-score, index): the exact top-k of [0, r_{j+1}), whose k-th score is T_{j+1}. T_0 = -inf (every
// item of the first range is a candidate). A subset's k-th best cannot beat the whole set's, so
// T_j bounds the k-th score over [0, r_{j+1}) from below: every item of that exact top-k is in the
// previous list or reaches T_j, and the result is exactly the list scan's (the same kernel
// arithmetic scores every item). On exchangeable data a range yields ~k (r_{j+1} - r_j) / r_j
// candidates per query, and the block permutation makes a table sorted by norm or popularity as
// good as exchangeable (tools/microbench_topk.py ORDER=norm: 528 ms through the list-scan rerun in
// contiguous ranges). A query whose candidates overflow their slots (mass ties at a bound, an order
// built against the permutation) sets a flag and the call reruns as the list scan (one 4-byte read
// back; graph capture keeps the list scan).
constexpr int TK_SEL = 4096;                // entries a select workgroup sorts (a power of two)
constexpr int TK_CAPQ = TK_SEL - TK_KMAX;   // candidate slots per query
constexpr int64_t TK_TP_MIN_N = 1 << 20;    // shards below this keep the list scan
constexpr int TK_R0 = 2048;                 // first range (all candidates)
constexpr int TK_RMAX = 12;                 // ranges at most

static int64_t topk_range_ratio() {
  const char* e = exp_env("RS_TOPK_RANGE_RATIO");  // experiment switch (default 4)
  const int64_t v = e ? atoi(e) : 4;
  return v < 2 ? 2 : v;
}


static bool topk_two_phase_ok(int64_t nq, int64_t N, int k, int prec) {
  int qt, wq, ipw;
  topk_cfg(nq, &qt, &wq, &ipw);
  // the permuted-block walk forms tile rows in 32 bits up to n_blocks * 2048 (the last block's
  // padding past N included): N must leave that room below 2^31 (larger shards take the list scan)
  return qt == 32 && (prec == 6 || prec == 9) && N >= TK_TP_MIN_N && k <= TK_KMAX &&
         N <= ((int64_t)1 << 31) - 1 - 2 * TK_BLOCK_ROWS;
}

static size_t topk_two_phase_extra_bytes(int64_t nq, int k) {
  return 2 * (align_up((size_t)nq * k * 4, 256) + align_up((size_t)nq * k * 8, 256)) +
         align_up((size_t)nq * 4 + 8, 256) + 2 * align_up((size_t)nq * TK_CAPQ * 4, 256) + 1024;
}

// Per query: the previous range's exact list (kp entries, or none) and the range's candidates
// (app_n[q] of them, cap slots) sorted under (-score, index); the first k kept. Resets app_n[q]
// for the next range. Too many candidates: the overflow flag (the caller reruns the list scan).
__global__ __launch_bounds__(512) void topk_select_kernel(const float* __restrict__ a_s,
                                                          const int64_t* __restrict__ a_i, int kp, int k,
                                                          int32_t* __restrict__ app_n,
                                                          const float* __restrict__ app_s,
                                                          const int32_t* __restrict__ app_i, int cap,
                                                          int64_t app_off, int64_t index_base,
                                                          float* __restrict__ out_s,
                                                          int64_t* __restrict__ out_i,
                                                          int32_t* __restrict__ overflow) {
  __shared__ float ss[TK_SEL];
  __shared__ int32_t si[TK_SEL];
  const int64_t q = blockIdx.x;
  const int SENT = 0x7fffffff;
  const int cn = app_n[q];
  __syncthreads();
  if (threadIdx.x == 0) app_n[q] = 0;
  if (cn > cap || kp + cn > TK_SEL) {
    if (threadIdx.x == 0) atomicOr(overflow, 1);
    return;
  }
  const int m = kp + cn;
  for (int e = threadIdx.x; e < kp; e += 512) {
    const int64_t ix = a_i[q * kp + e];
    ss[e] = a_s[q * kp + e];
    si[e] = ix < 0 ? SENT : (int32_t)ix;
  }
  for (int e = threadIdx.x; e < cn; e += 512) {
    ss[kp + e] = app_s[q * cap + e];
    si[kp + e] = (int32_t)(app_i[q * cap + e] + app_off);
  }
  int P = 1;
  while (P < m || P < k) P <<= 1;  // <= TK_SEL
  for (int e = m + threadIdx.x; e < P; e += 512) {
    ss[e] = -INFINITY;
    si[e] = SENT;
  }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int e = threadIdx.x; e < P / 2; e += 512) {
        const int lo = 2 * stride * (e / stride) + (e % stride), hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const bool hb = tk_better(ss[hi], (int64_t)si[hi], ss[lo], (int64_t)si[lo]);
        if (hb == desc) {
          const float ts = ss[lo];
          const int32_t ti = si[lo];
          ss[lo] = ss[hi];
          si[lo] = si[hi];
          ss[hi] = ts;
          si[hi] = ti;
        }
      }
      __syncthreads();
    }
  }
  for (int j = threadIdx.x; j < k; j += 512) {
    out_s[q * k + j] = ss[j];
    out_i[q * k + j] = si[j] == SENT ? (int64_t)-1 : (int64_t)si[j] + index_base;
  }
}

template <int D>
static int topk_impl(const float* Q, int64_t nq, const float* items, int64_t N, int k,
                     int64_t index_base, float* out_s, int64_t* out_i, void* ws, size_t wsb,
                     hipStream_t st, int prec = 0, bool list_scan = false) {
  hipStreamCaptureStatus cap_st = hipStreamCaptureStatusNone;
  RS_HIP(hipStreamIsCapturing(st, &cap_st));
  if (D != IBX_D || list_scan || !topk_two_phase_ok(nq, N, k, prec) || cap_st != hipStreamCaptureStatusNone)
    return topk_impl_lists<D>(Q, nq, items, N, k, index_base, out_s, out_i, ws, wsb, st, prec);
  const size_t lb = align_up(topk_lists_workspace_bytes(nq, N, k), 256);
  Carve c(static_cast<char*>(ws) + lb, wsb - lb);
  // ranges of whole TK_R0-row blocks in the permuted block order (TkBlocks): r[] in blocks
  static_assert(TK_R0 == TK_BLOCK_ROWS, "the first range is one block");
  TkBlocks bk{TK_R0, 0, 0, ceil_div(N, TK_R0), 1, 0, 1, 1};
  {
    int64_t a = (bk.n * 5) / 8 | 1;  // an odd multiplier near 0.62 n, coprime to n
    auto gcd = [](int64_t x, int64_t y) { while (y) { const int64_t t = x % y; x = y; y = t; } return x; };
    while (a > 1 && gcd(a, bk.n) != 1) a -= 2;
    bk.a = a < 1 ? 1 : a;
    bk.c = bk.n / 3;
#ifdef TK_PERM_IDENTITY  // (A/B: the block machinery in table order)
    bk.a = 1;
    bk.c = 0;
#endif
  }
  int64_t r[TK_RMAX + 1];
  int nr = 0;
  {
    const int64_t ratio = topk_range_ratio();
    r[0] = 0;
    int64_t b = 1;
    while (b < bk.n && nr < TK_RMAX - 1) {
      r[++nr] = b;
      b *= ratio;
    }
    r[++nr] = bk.n;
  }
  float* l_s[2] = {c.take<float>(nq * k), c.take<float>(nq * k)};
  int64_t* l_i[2] = {c.take<int64_t>(nq * k), c.take<int64_t>(nq * k)};
  int32_t* app_n = c.take<int32_t>(nq + 2);
  int32_t* overflow = app_n + nq;
  float* ninf = reinterpret_cast<float*>(overflow + 1);
  float* app_s = c.take<float>(nq * TK_CAPQ);
  int32_t* app_i = c.take<int32_t>(nq * TK_CAPQ);
  RS_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(app_n), 0, (size_t)nq + 1, st));
  // the bound of the first range: -inf (every item a candidate). The timing-only experiment switch
  // RS_TOPK_EXP_TH_INF (+inf for every range: no candidates, wrong lists) exists only in builds
  // made with -DRS_EXPERIMENTS; release builds cannot be switched into it.
#ifdef RS_EXPERIMENTS
  const bool exp_inf = exp_env("RS_TOPK_EXP_TH_INF") != nullptr;
#else
  constexpr bool exp_inf = false;
#endif
  RS_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(ninf), exp_inf ? 0x7f800000 : (int)0xff800000, 1, st));
  int qt, wq, ipw;
  topk_cfg(nq, &qt, &wq, &ipw);
  const int64_t nqb = ceil_div(ceil_div(nq, qt), wq);
  for (int j = 0; j < nr; ++j) {
    // scan [r[j], r[j + 1]) against the k-th score of the list of [0, r[j]), then select
    const bool first = j == 0, last = j == nr - 1;
    const float* prev_s = first ? nullptr : l_s[(j - 1) & 1];
    const int64_t* prev_i = first ? nullptr : l_i[(j - 1) & 1];
    // the range's blocks dealt to about as many workgroups as the contiguous scan's geometry uses
    bk.lo = r[j];
    bk.hi = r[j + 1];
    // (a range of fewer blocks than wanted slices splits each block in up to 8 parts of >= 256 rows)
    int64_t per, nse, nvs;
    const int64_t L = bk.hi - bk.lo;
    topk_geometry(nq, L * TK_R0, k, &per, &nse, &nvs, true);
    if (nse > L) {
      bk.spb = 1;
      while (bk.spb < 8 && L * bk.spb * 2 <= nse) bk.spb *= 2;
      bk.bpw = 1;
      nse = L * bk.spb;
    } else {
      bk.spb = 1;
      bk.bpw = ceil_div(L, nse);
      nse = ceil_div(L, bk.bpw);
    }
    // slices padded to a multiple of 8 (empty ones return at once): the XCD-aware workgroup order
    // then keeps the query blocks of a slice on one XCD, sharing its item lines in that L2
    nse = ceil_div(nse, 8) * 8;
    const float* thr = (first || exp_inf) ? ninf : prev_s + (k - 1);
    const int64_t thr_ld = (first || exp_inf) ? 0 : k;
    static const bool nt_loads = exp_env("RS_TOPK_NT_LOADS") != nullptr;  // experiment switch
    // default: 8-wave workgroups (two 4-wave query blocks, nqb8 of them per slice) over 64-row tiles;
    // RS_TOPK_THR_W4 keeps the 4-wave 32-row-tile kernel (A/B switch, timing)
    static const bool w4 = exp_env("RS_TOPK_THR_W4") != nullptr;
    const int64_t nqb8 = ceil_div(nqb, 2);
    if (prec == 6 && nt_loads)
      hipLaunchKernelGGL((topk_thr_kernel<6, true>), dim3((unsigned)(nqb * nse)), dim3(256), 0, st, Q, nq,
                         items, N, per, nse, nqb, thr, thr_ld, app_n, app_s, app_i, TK_CAPQ, bk);
    else if (prec == 6 && w4)
      hipLaunchKernelGGL(topk_thr_kernel<6>, dim3((unsigned)(nqb * nse)), dim3(256), 0, st, Q, nq, items, N,
                         per, nse, nqb, thr, thr_ld, app_n, app_s, app_i, TK_CAPQ, bk);
    else if (prec == 6)
      hipLaunchKernelGGL((topk_thr_kernel<6, false, 8, 2>), dim3((unsigned)(nqb8 * nse)), dim3(512), 0, st, Q, nq,
                         items, N, per, nse, nqb8, thr, thr_ld, app_n, app_s, app_i, TK_CAPQ, bk);
    else
      hipLaunchKernelGGL((topk_thr_kernel<9, false, 8, 2>), dim3((unsigned)(nqb8 * nse)), dim3(512), 0, st, Q, nq,
                         items, N, per, nse, nqb8, thr, thr_ld, app_n, app_s, app_i, TK_CAPQ, bk);
    int rc = check_launch("topk_thr");
    if (rc) return rc;
    hipLaunchKernelGGL(topk_select_kernel, dim3((unsigned)nq), dim3(512), 0, st, prev_s, prev_i, first ? 0 : k, k,
                       app_n, app_s, app_i, TK_CAPQ, 0, last ? index_base : 0, last ? out_s : l_s[j & 1],
                       last ? out_i : l_i[j & 1], overflow);
    rc = check_launch("topk_select");
    if (rc) return rc;
  }
  int32_t ovf = 0;
  RS_HIP(hipMemcpyAsync(&ovf, overflow, 4, hipMemcpyDeviceToHost, st));
  RS_HIP(hipStreamSynchronize(st));
  if (ovf) return topk_impl_lists<D>(Q, nq, items, N, k, index_base, out_s, out_i, ws, lb, st, prec);
  return RS_OK;
}

}  // namespace rs

using namespace rs;

extern "C" {

#ifdef RS_TOPK_EXP_STATS
int rs_topk_debug_stats(unsigned long long* out, int reset) {
  RS_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(tk_stats), sizeof(unsigned long long) * 8));
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    RS_HIP(hipMemcpyToSymbol(HIP_SYMBOL(tk_stats), z, sizeof(z)));
  }
  return 0;
}
#endif

size_t rs_topk_ip_workspace_bytes(int64_t nq, int64_t N, int64_t D, int k) {
  (void)D;
  const size_t lb = align_up(topk_lists_workspace_bytes(nq, N, k), 256);
  // the two-phase scan's sample lists, bounds and candidate arrays follow the list scan's part
  // (sized whenever the shape could take it: the precision is not an argument here)
  if (nq > 0 && k > 0 && topk_two_phase_ok(nq, N, k, 6)) return lb + topk_two_phase_extra_bytes(nq, k);
  return lb;
}

int rs_topk_ip_prec_f32(const float* queries, int64_t nq, const float* items, int64_t N, int64_t D,
                        int k, int64_t index_base, float* out_scores, int64_t* out_index, int precision,
                        void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(nq >= 0 && N > 0 && k > 0, "rs_topk_ip_f32: bad sizes");
  RS_REQUIRE(k <= TK_KMAX, "rs_topk_ip_f32: k must be <= %d", TK_KMAX);
  RS_REQUIRE(k <= N, "rs_topk_ip_f32: k must be <= N");
  RS_REQUIRE(N < ((int64_t)1 << 31) - 1, "rs_topk_ip_f32: N must be < 2^31 per call (shard it)");
  RS_REQUIRE(queries && items && out_scores && out_index, "rs_topk_ip_f32: null");
  RS_REQUIRE(aligned16(queries) && aligned16(items), "rs_topk_ip_f32: 16-byte alignment");
  const bool list_scan = (precision & RS_TOPK_LIST_SCAN) != 0;
  precision &= ~RS_TOPK_LIST_SCAN;
  RS_REQUIRE(precision == RS_PREC_F32 || precision == RS_PREC_F32_SPLIT6 || precision == RS_PREC_F32_SPLIT9,
             "rs_topk_ip_f32: precision must be 0, 6 or 9 (| RS_TOPK_LIST_SCAN)");
  if (nq == 0) return RS_OK;
  if (!workspace || workspace_bytes < rs_topk_ip_workspace_bytes(nq, N, D, k)) {
    set_error("rs_topk_ip_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  switch (D) {
    case 32: return topk_impl<32>(queries, nq, items, N, k, index_base, out_scores, out_index, workspace, workspace_bytes, st);
    case 64: return topk_impl<64>(queries, nq, items, N, k, index_base, out_scores, out_index, workspace, workspace_bytes, st);
    case 128:
      return topk_impl<128>(queries, nq, items, N, k, index_base, out_scores, out_index, workspace, workspace_bytes, st,
                            precision, list_scan);
    default:
      set_error("rs_topk_ip_f32: D=%lld not compiled (32, 64, 128)", (long long)D);
      return RS_ERR_UNSUPPORTED;
  }
}

int rs_topk_ip_f32(const float* queries, int64_t nq, const float* items, int64_t N, int64_t D,
                   int k, int64_t index_base, float* out_scores, int64_t* out_index,
                   void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  return rs_topk_ip_prec_f32(queries, nq, items, N, D, k, index_base, out_scores, out_index, RS_PREC_F32, workspace,
                             workspace_bytes, stream);
}

size_t rs_topk_merge_workspace_bytes(int64_t nq, int64_t nlists, int k) {
  const size_t e = (size_t)(nq > 0 ? nq : 1) * (nlists > 0 ? nlists : 1) * (k > 0 ? k : 1);
  return 2 * (align_up(e * 4, 256) + align_up(e * 8, 256)) + 1024;
}

int rs_topk_merge_f32(const float* in_scores, const int64_t* in_index, int64_t nq, int64_t nlists,
                      int k, float* out_scores, int64_t* out_index, void* workspace,
                      size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(nq >= 0 && nlists > 0 && k > 0 && k <= TK_KMAX, "rs_topk_merge_f32: bad sizes");
  RS_REQUIRE(in_scores && in_index && out_scores && out_index, "rs_topk_merge_f32: null");
  if (nq == 0) return RS_OK;
  if (!workspace || workspace_bytes < rs_topk_merge_workspace_bytes(nq, nlists, k)) {
    set_error("rs_topk_merge_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  const size_t e = (size_t)nq * nlists * k;
  Carve c(workspace, workspace_bytes);
  float* s0 = c.take<float>(e);
  int64_t* i0 = c.take<int64_t>(e);
  float* s1 = c.take<float>(e);
  int64_t* i1 = c.take<int64_t>(e);
  RS_HIP(hipMemcpyAsync(s0, in_scores, e * sizeof(float), hipMemcpyDeviceToDevice, st));
  RS_HIP(hipMemcpyAsync(i0, in_index, e * sizeof(int64_t), hipMemcpyDeviceToDevice, st));
  return merge_rounds<int64_t>(s0, i0, s1, i1, nq, nlists, k, 0, out_scores, out_index, nullptr, st);
}

}  // extern "C"
