// inbatch.hip — tfrs.tasks.Retrieval() in-batch softmax cross-entropy, fwd + bwd, fp32 MFMA.
//
// Reference: src/models.py:116,137 — scores = U C^T (B x B), labels = I, CategoricalCrossentropy
// (from_logits=True, reduction=SUM) [TFRS semantics, SURVEY Appendix A.6]:
//   L = sum_i ( logsumexp_j S_ij - S_ii ),  dL/dU = (P - I) C,  dL/dC = (P - I)^T U.
// At B = 65536 the logits are 17 GB, so nothing B x B is ever stored (flash-attention style):
//
//   row pass  (owned = users, streamed = items):  online max/sum over j, O_i = sum_j P_ij C_j
//             -> lse_i, row loss, and dU_i = w (O_i / l_i - C_i) in the SAME pass (P C is the
//                attention-forward product with V = C, so the forward yields dU for free);
//   col pass  (owned = items, streamed = users):  P_ij = exp(S_ij - lse_i) (no online max),
//             O'_j = sum_i P_ij U_i -> dC_j = w (O'_j - U_j).
// 4 B^2 D FLOP-pairs per training step instead of the 5 a recompute-per-gradient scheme needs.
//
// MFMA mapping (v_mfma_f32_32x32x2_f32, exact fp32): S^T tile = K_tile Q^T so each lane owns
// one q (column) and 16 streamed rows in its accumulator registers; the row max/sum is in
// registers + one cross-half shuffle. The accumulator then feeds the P.V product directly as
// the MFMA B operand (its row index = the streamed index = the contraction index), so P never
// leaves registers. Streamed tiles (64 rows x D) are staged in LDS, double-buffered, stride D+4
// floats (conflict-free ds_read_b128 for the S operand, ds_read_b32 rows for the PV operand).
// The streamed range is split over workgroups when B is small so the grid fills 256 CUs; the
// partial (m, l, O) are merged in a fixed order by the finalize pass (bitwise reproducible).
#include "common.hpp"
#include "split.hpp"
#include <cstdlib>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>
#include <rocprim/block/block_radix_sort.hpp>

#include <cmath>
#include <type_traits>

namespace rs {

// log2(e) in fp32: the base of every exponential here (v_exp_f32 computes 2^x; __expf(x) is
// 2^(x IB_LOG2E)), so the passes exponentiate in base e' = 2^IB_LOG2E, not e
constexpr float IB_LOG2E = 1.4426950408889634f;
#ifndef IB_COL_COPY_FIRST
#define IB_COL_COPY_FIRST 1  // col pass: U tile copy at the step's head, the scores of t + 2 not waited for at its end
#endif
#ifndef IB_COL_MAKE_P_DT
#define IB_COL_MAKE_P_DT 3  // the d-tile after whose MFMAs the next P is formed
#endif
#ifndef IB_ROW_DMA_FIRST
#define IB_ROW_DMA_FIRST 1  // row pass: next tile's DMA before the score stores, which the step end does not wait for
#endif
#ifndef IB_FRESH_TILE_ACC
#define IB_FRESH_TILE_ACC 1
#endif
#ifndef IB_FRESH_WK
#define IB_FRESH_WK 0
#endif
#ifndef IB_PRIO_HALF
#define IB_PRIO_HALF 0  // row / col passes: s_setprio 1 for the second half of the waves (timing switch)
#endif
#ifndef IB_ROW_STAGGER
#define IB_ROW_STAGGER 0  // deduplicated row pass: the second half of the waves one phase late
#endif
// The next d-tile's transposed operand read ahead of this d-tile's MFMAs (12 VGPRs; same products,
// bitwise). Row pass P.K: -26..-34 us per C3 step in three A/Bs, both orders; col pass: neutral
// (profiles/r06n_read_ahead_ab.txt).
// Row pass S phase with the next chunk's K rows read ahead (IB_ROW_S_PREFETCH): row -9 us, col
// +5 us per C3 step, neutral (profiles/r06s_read_ahead_fin_ab.txt); on the final tree four A/Bs gave
// row -1.6 / +4.9 / -12.4 / +6.0 us, bitwise (profiles/r06ag_row_s_prefetch_ab.txt): off.
#ifndef IB_ROW_S_PREFETCH
#define IB_ROW_S_PREFETCH 0
#endif
#ifndef IB_COL_PREFETCH_A
#define IB_COL_PREFETCH_A 1
#endif
#ifndef IB_ROW_PREFETCH_A
#define IB_ROW_PREFETCH_A 1
#endif
#ifndef IB_ROW_SPLIT_UB
#define IB_ROW_SPLIT_UB 0  // deduplicated row pass per owned subtile (step_ub): bitwise, +89..+114 us per C3 step, off
#endif
#ifndef IB_COL_PROBE
#define IB_COL_PROBE 0  // col pass timing probes (A/B builds only; 1-3 compute wrong results)
#endif
#ifndef IB_COL_CHAIN
#define IB_COL_CHAIN 1  // col pass: per-accumulator product chains, the fresh-tile adds six MFMAs late
#endif
#ifndef IB_COL_TIMG
// deduplicated col pass: U^T from the transposed image (3 ds_read_b128 per d-tile instead of 6
// transposed reads). Measured slower at C3 (col pass +2.4 %, plus the image pass, 21 us;
// profiles/r06g_col_timg_ab.txt): kept as a switch, off
#define IB_COL_TIMG 0
#endif

constexpr int IB_QW = 32;   // owned rows per wave
constexpr int IB_QB = 128;  // owned rows per workgroup (4 waves)
constexpr int IB_KT = 64;   // streamed rows per LDS tile
#ifndef IBX_NW
#define IBX_NW 8  // waves per workgroup of the split kernels (one workgroup per CU, 2 waves per SIMD)
#endif
constexpr int64_t IB_SKB = IB_QW * IBX_NW;  // owned rows per stream-K block (one split-kernel workgroup)

struct InbatchParams {
  const float* Q;  // owned rows [B][D]
  const float* K;  // streamed rows [B][D]
  int64_t B;
  int64_t k_per_split;
  const float* lse_k;  // MODE 2: lse of the streamed rows
  float* part_m;       // [nsplit][B]
  float* part_l;       // [nsplit][B]
  float* part_o;       // [nsplit][B][D]
  float* S;            // MODE 1 (nullable): score tiles written for the stored col pass
  // split kernels only (the deduplicated pair): B owned rows against Bs streamed rows, each
  // streamed row standing for kw[r] bitwise-identical rows of the batch (the row pass's key
  // weights); the col pass reads streamed user r's exponent bias at lse_k[r] (ib_lz_kernel: the lse
  // of its first row and its count folded together)
  int64_t Bs = 0;
  const float* kw = nullptr;
  const int32_t* krow = nullptr;
  // split kernels, stream-K order (sk_wg > 0, grid = sk_wg workgroups): the ceil(B / rows per
  // workgroup) x sk_ntk (owned block, 32-key tile) units cut into sk_wg equal shares (IbSeg)
  int64_t sk_wg = 0;
  int64_t sk_ntk = 0;
  // device-count form (graph-capturable deduplicated pair): when dinfo is set, B = dinfo[d_own]
  // and Bs = dinfo[d_str] are read on the device (the distinct-row search's counts, never copied
  // to the host), and sk_ntk / sk_wg are derived from them (ib_resolve); the grid is sized for the
  // worst case and workgroups past the stream-K share count exit
  const int64_t* dinfo = nullptr;
  int d_own = 0, d_str = 0;
};

// Stream-K bookkeeping shared by the split kernels and the finalizes. The key tiles are cut into R
// ranges (ib_sk_ranges) and workgroup w serves range r = w % R as its j = w / R-th of the Wr
// workgroups there: it owns units [floor(j Tr / Wr), floor((j + 1) Tr / Wr)) of the range's
// Tr = blocks x (the range's tiles) block-major units; unit u of the range lies in its workgroup
// ceil((u + 1) Wr / Tr) - 1. A workgroup's share is cut at block ends into segments; block b's
// partial slots are its ranges' slots in range order, and within a range the slot of workgroup j's
// segment is j - (the range's workgroup of b's first unit): slots stay in ascending key order.
// With R = 1 (the default) this is plain stream-K over the blocks x ntk units.
__host__ __device__ inline int64_t ib_sk_wg_of(int64_t u, int64_t T, int64_t W) { return ((u + 1) * W + T - 1) / T - 1; }
// IB_SK_RANGES (timing switch): 8 ranges, one per XCD (blocks are dealt round-robin over the 8 XCDs,
// MI355X_MICROARCH.md; speed only, nothing depends on it), so all the workgroups of a range share
// one L2 and stream the same 1/8 of the key images (2.5 MB at C3, resident). It cut the dedup col
// pass's HBM fetch to the kept scores alone (3.89 -> 2.27 GB at C3) and still ran slower — col
// +1.9 %, row +2.9 %, the finalizes +82 us over 4x the partial slots (profiles/r06i_sk_ranges_ab.txt):
// the col pass is not bound by its fetch. Off (1).
#ifndef IB_SK_RANGES
#define IB_SK_RANGES 1
#endif
__host__ __device__ inline int ib_sk_ranges(int64_t xg, int64_t ntk, int64_t W) {
  constexpr int64_t R = IB_SK_RANGES;
  if (R == 1 || ntk < R || W < R) return 1;
  // every workgroup needs a unit: the smallest range's units >= the largest range's workgroups
  return xg * (ntk / R) >= (W + R - 1) / R ? (int)R : 1;
}
// slots of block blk in range r of R (I: 32-bit arithmetic when (T + 1) W fits, else int64_t)
template <typename I>
__host__ __device__ inline I ib_sk_range_slots(I blk, I xg, I ntk, I W, I R, I r) {
  const I Wr = (W - r + R - 1) / R, klo = r * ntk / R, nr = (r + 1) * ntk / R - klo, Tr = xg * nr;
  auto wg_of = [&](I u) { return ((u + 1) * Wr + Tr - 1) / Tr - 1; };
  return wg_of((blk + 1) * nr - 1) - wg_of(blk * nr) + 1;
}
template <typename I>
__host__ __device__ inline int ib_sk_slots_t(I blk, I ntk, I T, I W) {
  const I xg = T / ntk, R = (I)ib_sk_ranges((int64_t)xg, (int64_t)ntk, (int64_t)W);
  I s = 0;
  for (I r = 0; r < R; ++r) s += ib_sk_range_slots<I>(blk, xg, ntk, W, R, r);
  return (int)s;
}
__host__ __device__ inline int ib_sk_slots(int64_t blk, int64_t ntk, int64_t T, int64_t W) {
  if ((T + 1) * W <= 0xffffffffLL && blk <= 0xffffffffLL)
    return ib_sk_slots_t<uint32_t>((uint32_t)blk, (uint32_t)ntk, (uint32_t)T, (uint32_t)W);
  return ib_sk_slots_t<int64_t>(blk, ntk, T, W);
}

// stream-K workgroup count for B owned rows (blocks of 256) against ntk key tiles on at most
// `grid` workgroups: every block's units spread over at most 64 partial slots (W <= (64 - 2 R)
// blocks: a block has at most W / blocks + 2 R slots)
__host__ __device__ inline int64_t ib_sk_workgroups(int64_t B, int64_t ntk, int64_t grid) {
  const int64_t xg = (B + IB_SKB - 1) / IB_SKB;
  const int64_t T = xg * ntk;
  int64_t W = T < grid ? T : grid;
  if (W > (64 - 2 * IB_SK_RANGES) * xg) W = (64 - 2 * IB_SK_RANGES) * xg;
  return W > 0 ? W : 1;
}

// the device-count form: the counts from dinfo, the stream-K shape from them (same rule as the host)
__device__ inline void ib_resolve(InbatchParams& p) {
  if (!p.dinfo) return;
  p.B = p.dinfo[p.d_own];
  p.Bs = p.dinfo[p.d_str];
  p.sk_ntk = (p.Bs + 31) / 32;
  p.sk_wg = ib_sk_workgroups(p.B, p.sk_ntk, gridDim.x);
}

// The segments of one workgroup: the grid split (blockIdx.x, key range blockIdx.y, slot
// blockIdx.y; SK = false, one trip), or its stream-K share (SK = true)
template <bool SK>
struct IbSeg {
  int64_t cur, end, ntk, W, w, kps, Bs, klo, nr, Tr, Wr, j;
  int R, r;
  __device__ IbSeg(const InbatchParams& p, int64_t rows_per_wg) {
    Bs = p.Bs;
    kps = p.k_per_split;
    w = blockIdx.x;
    cur = 0;
    end = 1;
    if constexpr (SK) {
      W = p.sk_wg;
      ntk = p.sk_ntk;
      const int64_t xg = (p.B + rows_per_wg - 1) / rows_per_wg;
      R = ib_sk_ranges(xg, ntk, W);
      r = (int)(w % R);
      j = w / R;
      Wr = (W - r + R - 1) / R;
      klo = r * ntk / R;
      nr = (r + 1) * ntk / R - klo;
      Tr = xg * nr;
      cur = j * Tr / Wr;
      end = (j + 1) * Tr / Wr;
      if (w >= W) cur = end = 0;  // device-count form: a workgroup past the share count
    }
  }
  __device__ bool next(int64_t& blk, int64_t& kb0, int64_t& ke, int64_t& slot) {
    if (cur >= end) return false;
    if constexpr (!SK) {
      cur = 1;
      blk = blockIdx.x;
      kb0 = (int64_t)blockIdx.y * kps;
      ke = kb0 + kps < Bs ? kb0 + kps : Bs;
      slot = blockIdx.y;
      return true;
    }
    blk = cur / nr;
    const int64_t bend = end < (blk + 1) * nr ? end : (blk + 1) * nr;
    kb0 = (klo + cur - blk * nr) * 32;
    ke = (klo + bend - blk * nr) * 32;
    if (ke > Bs) ke = Bs;
    // the block's slots in the ranges before this one, then this workgroup's place in the range
    int64_t base = 0;
    const int64_t xg = Tr / nr;
    for (int q = 0; q < r; ++q) base += ib_sk_range_slots<int64_t>(blk, xg, ntk, W, R, q);
    slot = base + j - ib_sk_wg_of(blk * nr, Tr, Wr);
    cur = bend;
    return true;
  }
};

// Score-tile layout shared by the row pass (writer) and the stored col pass (reader): the B x B
// scores in 32 x 32 tiles, tile (item tile it, user tile ut) at (it * NT + ut) * 1024 floats.
// Inside a tile, S(user 32 ut + u, item 32 it + i) sits at float 512 (u / 16) + 16 i + ib_slot(u),
// ib_slot(u) = u % 16 with bits 2 and 3 swapped: two 16-user halves, each item's 16 users one
// 64-B run. The row passes store straight from their accumulators (one dword per register:
// every store instruction fills 64-B runs, no register transpose); the col passes load 4
// consecutive slots (their B operand's k order follows the slot order) and each load
// instruction of the 16x16 col pass reads 1 KB contiguous.
__host__ __device__ inline int64_t ib_ntiles(int64_t B) { return (B + 31) / 32; }
__host__ __device__ inline int ib_slot(int u) { return (u & 3) | ((u >> 1) & 4) | ((u << 1) & 8); }

// value of `v` in another lane of the same quad (quad_perm DPP)
template <int CTRL>
__device__ __forceinline__ float dpp_quad(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

// max(v, v of lane ^ 16) and max(v, v of lane ^ 32) on the VALU (v_permlane16/32_swap exchange
// the two 16-lane rows of each pair / the two 32-lane halves) instead of ds_bpermute round trips
__device__ __forceinline__ float ib_max_x16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float ib_max_x32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float ib_sum_x16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float ib_sum_x32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// MODE 0: row pass, lse only. MODE 1: row pass + P.K. MODE 2: col pass (fixed bias) + P.K.
template <int D, int MODE>
__global__ __launch_bounds__(256, 2) void inbatch_pass_kernel(InbatchParams p) {
  constexpr int KPAD = D + 4;
  constexpr int NDT = D / 32;                      // d tiles of the output
  constexpr int NSTG = IB_KT * D / 4 / 256;        // float4 per thread per tile
  constexpr int TILE = IB_KT * KPAD;
  constexpr int OT_ELEMS = 4 * IB_QW * (D + 1);
  constexpr int SMEM = (2 * TILE > OT_ELEMS) ? 2 * TILE : OT_ELEMS;
  static_assert(NSTG >= 1, "D too small");
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  __shared__ float lse_s[2][IB_KT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  const int64_t B = p.B;
  const int64_t q = (int64_t)blockIdx.x * IB_QB + wave * IB_QW + l32;
  const int64_t kb = (int64_t)blockIdx.y * p.k_per_split;
  const int64_t ke = (kb + p.k_per_split < B) ? kb + p.k_per_split : B;
  const int ntiles = ke > kb ? (int)((ke - kb + IB_KT - 1) / IB_KT) : 0;

  // owned-row fragments: MFMA step (g, t) uses k = 8g + 4*half + t in both operands
  float qf[D / 2];
#pragma unroll
  for (int g = 0; g < D / 8; ++g) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (q < B) v = *reinterpret_cast<const f32x4*>(p.Q + q * D + 8 * g + 4 * half);
#pragma unroll
    for (int t = 0; t < 4; ++t) qf[4 * g + t] = v[t];
  }

  f32x16 O[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) O[dt][r] = 0.f;
  float m = -INFINITY, l = 0.f;

  f32x4 stg[NSTG];
  float lse_reg = 0.f;
  auto load_tile = [&](int t) {
    const int64_t base = kb + (int64_t)t * IB_KT;
#pragma unroll
    for (int i = 0; i < NSTG; ++i) {
      const int f = tid + 256 * i;
      const int row = f / (D / 4), c4 = f % (D / 4);
      // rows past the range are clamped to a real row (no load branch, so the waits before the
      // MFMAs can count this prefetch); their scores are masked out
      const int64_t gr = base + row < ke ? base + row : ke - 1;
      stg[i] = *reinterpret_cast<const f32x4*>(p.K + gr * D + 4 * c4);
    }
    if (MODE == 2 && tid < IB_KT) {
      const int64_t gr = base + tid;
      lse_reg = p.lse_k[gr < ke ? gr : ke - 1];
    }
  };
  auto store_tile = [&](int buf) {
    float* Ks = smem + buf * TILE;
#pragma unroll
    for (int i = 0; i < NSTG; ++i) {
      const int f = tid + 256 * i;
      const int row = f / (D / 4), c4 = f % (D / 4);
      *reinterpret_cast<f32x4*>(Ks + row * KPAD + 4 * c4) = stg[i];
    }
    if (MODE == 2 && tid < IB_KT) lse_s[buf][tid] = lse_reg;
  };

  if (ntiles > 0) {
    load_tile(0);
    store_tile(0);
    __syncthreads();
  }
  for (int t = 0; t < ntiles; ++t) {
    if (t + 1 < ntiles) load_tile(t + 1);
    const float* Ks = smem + (t & 1) * TILE;
#pragma unroll
    for (int st = 0; st < IB_KT / 32; ++st) {
      const int64_t kbase = kb + (int64_t)t * IB_KT + st * 32;
      if (kbase >= ke) break;
      const int rem = (int)((ke - kbase) < 32 ? (ke - kbase) : 32);  // valid streamed rows in this step
      // ---- S^T tile: acc[r] = S(q, kbase + acc_row(r, half)) ----
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      const float* krow = Ks + (st * 32 + l32) * KPAD + 4 * half;
#pragma unroll
      for (int g = 0; g < D / 8; ++g) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(krow + 8 * g);
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) acc = mfma32x32x2(a[tt], qf[4 * g + tt], acc);
      }
      if (MODE == 1 && p.S && (int64_t)blockIdx.x * IB_QB + wave * IB_QW < B) {
        // lane l32 holds user l32 of the tile at items acc_row(r, half): one dword store per
        // register, each store two 64-B runs (the halves' users 0-15 / 16-31 of one item)
        const int64_t NT = ib_ntiles(B);
        float* tb = p.S + ((kbase / 32) * NT + (int64_t)((blockIdx.x * IB_QB + wave * IB_QW) / 32)) * 1024 +
                    512 * (l32 >> 4) + ib_slot(l32 & 15) + 16 * 4 * half;
#pragma unroll
        for (int r = 0; r < 16; ++r) tb[16 * ((r & 3) + 8 * (r >> 2))] = acc[r];
      }
      // ---- softmax weights ----
      float pr[16];
      if (MODE == 2) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kr = st * 32 + acc_row(r, half);
          const float e = __expf(acc[r] - lse_s[t & 1][kr]);
          pr[r] = acc_row(r, half) < rem ? e : 0.f;
        }
      } else {
        float mx = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          acc[r] = acc_row(r, half) < rem ? acc[r] : -INFINITY;
          mx = fmaxf(mx, acc[r]);
        }
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float m_new = fmaxf(m, mx);
        const float alpha = __expf(m - m_new);
        float ps = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          pr[r] = __expf(acc[r] - m_new);
          ps += pr[r];
        }
        l = l * alpha + ps;
        // O only needs rescaling when some lane's running max grew (alpha == 1 exactly
        // otherwise); after the first tiles that is rare, so the 64-register pass is skipped.
        if (MODE == 1 && __any(m_new > m)) {
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
            for (int r = 0; r < 16; ++r) O[dt][r] *= alpha;
        }
        m = m_new;
      }
      // ---- O^T[d][q] += sum_k K[k][d] P[q][k] (accumulator feeds the B operand) ----
      // d is permuted across the output tiles: lane l32 of tile dt holds d = NDT*l32 + dt, so
      // one ds_read_b128 (D=128) feeds all NDT tiles' A operands for a key row.
      if (MODE != 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float* krow_pv = Ks + (st * 32 + acc_row(r, half)) * KPAD + NDT * l32;
          float a[NDT];
          if constexpr (NDT == 4) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(krow_pv);
            a[0] = v[0]; a[1] = v[1]; a[2] = v[2]; a[3] = v[3];
          } else if constexpr (NDT == 2) {
            const float2 v = *reinterpret_cast<const float2*>(krow_pv);
            a[0] = v.x; a[1] = v.y;
          } else {
            a[0] = krow_pv[0];
          }
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) O[dt] = mfma32x32x2(a[dt], pr[r], O[dt]);
        }
      }
    }
    if (t + 1 < ntiles) store_tile((t + 1) & 1);
    __syncthreads();
  }

  // ---- partials: m, l (row pass), O (unnormalised) ----
  const int64_t split = blockIdx.y;
  if (MODE != 2) {
    const float lt = l + __shfl_xor(l, 32, 64);
    if (half == 0 && q < B) {
      p.part_m[split * B + q] = m;
      p.part_l[split * B + q] = lt;
    }
  }
  if (MODE != 0) {
    // transpose O^T (d in registers, q on lanes) through LDS -> coalesced row stores
    float* Ow = smem + wave * IB_QW * (D + 1);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) Ow[l32 * (D + 1) + NDT * acc_row(r, half) + dt] = O[dt][r];
    __syncthreads();
    const int64_t qw0 = (int64_t)blockIdx.x * IB_QB + wave * IB_QW;
    for (int idx = lane; idx < IB_QW * D; idx += 64) {
      const int qq = idx / D, d = idx % D;
      if (qw0 + qq < B) p.part_o[(split * B + qw0 + qq) * D + d] = Ow[qq * (D + 1) + d];
    }
  }
}

// Col pass from the stored scores: owned = items, streamed = users (their rows staged in LDS for
// the P.U product, their lse for P); the S^T tile of each 32-user step is read from the row
// pass's score tiles (4 x 1 KB per wave, one step ahead) instead of being recomputed, so the
// pass is half the MFMA work of MODE 2. Bitwise equal to MODE 2: the stored scores are the same
// fp32 MFMA sums (same products, same k order).
template <int D>
__global__ __launch_bounds__(256, 2) void inbatch_col_stored_kernel(InbatchParams p, const float* __restrict__ S) {
  constexpr int KPAD = D + 4;
  constexpr int NDT = D / 32;
  constexpr int NSTG = IB_KT * D / 4 / 256;
  constexpr int TILE = IB_KT * KPAD;
  constexpr int OT_ELEMS = 4 * IB_QW * (D + 1);
  constexpr int SMEM = (2 * TILE > OT_ELEMS) ? 2 * TILE : OT_ELEMS;
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  __shared__ float lse_s[2][IB_KT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  const int64_t B = p.B;
  const int64_t kb = (int64_t)blockIdx.y * p.k_per_split;
  const int64_t ke = (kb + p.k_per_split < B) ? kb + p.k_per_split : B;
  const int ntiles = ke > kb ? (int)((ke - kb + IB_KT - 1) / IB_KT) : 0;
  const int64_t NT = ib_ntiles(B);
  // a wave whose items are all past B reads the last real tile (its results are never written)
  int64_t itile = (int64_t)(blockIdx.x * IB_QB + wave * IB_QW) / 32;
  if (itile >= NT) itile = NT - 1;
  // lane l32 = item: register group c holds users 8 c + 4 half + 0..3 = slots 4 (c & 1) + 8 half
  // + 0..3 of half c / 2
  const float* Sbase = S + itile * NT * 1024 + 16 * l32 + 8 * half;

  f32x16 O[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) O[dt][r] = 0.f;

  f32x4 stg[NSTG];
  float lse_reg = 0.f;
  auto load_tile = [&](int t) {
    const int64_t base = kb + (int64_t)t * IB_KT;
#pragma unroll
    for (int i = 0; i < NSTG; ++i) {
      const int f = tid + 256 * i;
      const int row = f / (D / 4), c4 = f % (D / 4);
      // rows past the range are clamped to a real row (no load branch, so the waits before the
      // MFMAs can count this prefetch); their scores are masked out
      const int64_t gr = base + row < ke ? base + row : ke - 1;
      stg[i] = *reinterpret_cast<const f32x4*>(p.K + gr * D + 4 * c4);
    }
    if (tid < IB_KT) {
      const int64_t gr = base + tid;
      lse_reg = p.lse_k[gr < ke ? gr : ke - 1];
    }
  };
  auto store_tile = [&](int buf) {
    float* Ks = smem + buf * TILE;
#pragma unroll
    for (int i = 0; i < NSTG; ++i) {
      const int f = tid + 256 * i;
      const int row = f / (D / 4), c4 = f % (D / 4);
      *reinterpret_cast<f32x4*>(Ks + row * KPAD + 4 * c4) = stg[i];
    }
    if (tid < IB_KT) lse_s[buf][tid] = lse_reg;
  };
  // score tile of the 32-user step starting at user kbase
  auto load_scores = [&](int64_t kbase, f32x4* dst) {
    const float* src = Sbase + (kbase / 32) * 1024;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      dst[c] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + 512 * (c >> 1) + 4 * (c & 1)));
  };

  // score tiles ride two 32-user steps ahead: slot st holds step (t, st); once its exponentials
  // are taken the slot is refilled with step (t + 1, st)
  f32x4 sb[IB_KT / 32][4];
  if (ntiles > 0) {
    load_tile(0);
#pragma unroll
    for (int st = 0; st < IB_KT / 32; ++st) {
      const int64_t k0 = kb + st * 32;
      load_scores(k0 < ke ? k0 : kb, sb[st]);
    }
    store_tile(0);
    __syncthreads();
  }
  for (int t = 0; t < ntiles; ++t) {
#ifndef RS_IB_EXP_NOULOAD
    if (t + 1 < ntiles) load_tile(t + 1);
#endif
    const float* Ks = smem + (t & 1) * TILE;
#pragma unroll
    for (int st = 0; st < IB_KT / 32; ++st) {
      const int64_t kbase = kb + (int64_t)t * IB_KT + st * 32;
      if (kbase >= ke) break;
      const int rem = (int)((ke - kbase) < 32 ? (ke - kbase) : 32);  // valid users in this step
      float pr[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kr = st * 32 + acc_row(r, half);
        const float e = __expf(sb[st][r >> 2][r & 3] - lse_s[t & 1][kr]);
        pr[r] = acc_row(r, half) < rem ? e : 0.f;
      }
      {
        const int64_t kn = kbase + IB_KT;
        load_scores(kn < ke ? kn : kbase, sb[st]);  // unconditional (clamped) prefetch
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float* krow_pv = Ks + (st * 32 + acc_row(r, half)) * KPAD + NDT * l32;
        float a[NDT];
        if constexpr (NDT == 4) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(krow_pv);
          a[0] = v[0]; a[1] = v[1]; a[2] = v[2]; a[3] = v[3];
        } else if constexpr (NDT == 2) {
          const float2 v = *reinterpret_cast<const float2*>(krow_pv);
          a[0] = v.x; a[1] = v.y;
        } else {
          a[0] = krow_pv[0];
        }
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) O[dt] = mfma32x32x2(a[dt], pr[r], O[dt]);
      }
    }
    if (t + 1 < ntiles) store_tile((t + 1) & 1);
    __syncthreads();
  }

  const int64_t split = blockIdx.y;
  float* Ow = smem + wave * IB_QW * (D + 1);
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) Ow[l32 * (D + 1) + NDT * acc_row(r, half) + dt] = O[dt][r];
  __syncthreads();
  const int64_t qw0 = (int64_t)blockIdx.x * IB_QB + wave * IB_QW;
  for (int idx = lane; idx < IB_QW * D; idx += 64) {
    const int qq = idx / D, d = idx % D;
    if (qw0 + qq < B) p.part_o[(split * B + qw0 + qq) * D + d] = Ow[qq * (D + 1) + d];
  }
}

// The last workgroup of a grid to finish sums the grid's fp64 partials in final_sum_kernel's
// order (bitwise its result). Thread 0 of each workgroup has published its partial
// (ticket_publish) and arrives; the last one reads the partials agent-coherently (common.hpp).
__device__ void ib_last_block_total(unsigned int* done, const double* part, int64_t np, float* out_f, double* out_d) {
  __shared__ double red[256];
  if (!ticket_last(done, blockIdx.x, np)) return;
  double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int64_t i0 = threadIdx.x; i0 < np; i0 += 256 * 8) {
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = i0 + 256 * j < np ? ticket_collect(part + i0 + 256 * j) : 0.0;
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += v[j];
  }
  red[threadIdx.x] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (out_f) out_f[0] = (float)red[0];
    if (out_d) out_d[0] = red[0];
  }
}

// Row finalize: merge splits, lse, row loss, optional dU; IB_FIN_RPW rows per wave (a row on all 64
// lanes; the rows' partial indices and slot counts lane-parallel, then every row's loads before
// any row's max / exp / log chain, so that the chains of a wave overlap), 4 waves per workgroup; per-workgroup fp64 loss partials (the rows' losses in
// row order) for the ordered total. Per row the arithmetic is that of one row per wave, so lse,
// row_loss and dU do not depend on IB_FIN_RPW.
// (C3 step, rocprof: 1 row per wave 74.5 us, 2 rows 65.0 us, 4 rows 73.3 us; profiles/r06s_read_ahead_fin_ab.txt)
#ifndef IB_FIN_RPW
#define IB_FIN_RPW 2
#endif
constexpr int IB_FIN_ROWS = 4 * IB_FIN_RPW;  // rows per workgroup
#ifndef IB_FIN_PRE
// O partials per row loaded up front (the rest inside the dU loop): 2 / 3 / 6 / 8 measured +13 / +7 /
// +6 / +12 us per C3 step against 4 (profiles/r06ah_fin_prefetch_ab.txt)
#define IB_FIN_PRE 4
#endif
template <int D>
__global__ __launch_bounds__(256) void inbatch_row_finalize_kernel(
    const float* __restrict__ U, const float* __restrict__ C, int64_t B, int nsplit_,
    const float* __restrict__ part_m, const float* __restrict__ part_l,
    const float* __restrict__ part_o, float weight, float* __restrict__ row_loss,
    float* __restrict__ lse, float* __restrict__ dU, double* __restrict__ loss_part,
    const int32_t* __restrict__ inv = nullptr, int64_t Bp = 0, int64_t sk_ntk = 0, int64_t sk_T = 0,
    int64_t sk_W = 0, const int64_t* __restrict__ dinfo = nullptr, int d_own = 0, int d_str = 0, int64_t sk_grid = 0,
    unsigned int* __restrict__ done = nullptr, float* __restrict__ loss_sum = nullptr,
    double* __restrict__ loss_sum64 = nullptr) {
  constexpr int R = IB_FIN_RPW;
  // partials of row i at pi = inv[i] of Bp owned rows (the deduplicated pair) or at i of B
  if (dinfo) {  // device-count form: the row pass's shape from the counts (ib_resolve's rule)
    Bp = dinfo[d_own];
    sk_ntk = (dinfo[d_str] + 31) / 32;
    sk_T = ((Bp + IB_SKB - 1) / IB_SKB) * sk_ntk;
    sk_W = ib_sk_workgroups(Bp, sk_ntk, sk_grid);
  }
  __shared__ double wl[4];
  __shared__ float sc_s[4][R][64], pl_s[4][R][64];
  __shared__ double tl_s[4][R][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t i0 = ((int64_t)blockIdx.x * 4 + wave) * R;
  const int64_t P = inv ? Bp : B;
  // the wave's rows' partial indices and slot counts lane-parallel (lane r < R: row i0 + r), so
  // the R rows share one inv load and one slot computation instead of R dependent chains
  int64_t pil = 0;
  int nsl = nsplit_;
  {
    const int64_t il = i0 + (lane < R ? lane : 0) < B ? i0 + (lane < R ? lane : 0) : B - 1;
    pil = inv ? (int64_t)inv[il] : il;
    // stream-K partials: the slot count of the row's 256-row block
    if (sk_W) nsl = ib_sk_slots(pil / IB_SKB, sk_ntk, sk_T, sk_W);
  }
  // the rows' U, C and first four splits' O partials are loaded up front (indices clamped), so
  // their latency overlaps the max / exp / log chains below
  constexpr int NDL = (D + 63) / 64, PRE = IB_FIN_PRE;
  float ur[R][NDL], cr[R][NDL], por[R][PRE][NDL], msr[R], lsr[R];
  int64_t pir[R];
  int nsr[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t i = i0 + r < B ? i0 + r : B - 1;
    const int64_t pi = __shfl(pil, r, 64);
    const int nsplit = __builtin_amdgcn_readfirstlane(__shfl(nsl, r, 64));
    pir[r] = pi;
    nsr[r] = nsplit;
#pragma unroll
    for (int k = 0; k < NDL; ++k) {
      const int d = lane + 64 * k < D ? lane + 64 * k : D - 1;
      ur[r][k] = U[i * D + d];
      cr[r][k] = C[i * D + d];
#pragma unroll
      for (int s = 0; s < PRE; ++s)
        por[r][s][k] = part_o[((int64_t)(s < nsplit ? s : nsplit - 1) * P + pi) * D + d];
    }
    // split partials loaded by one lane each (nsplit <= 64: see inbatch_nsplit)
    msr[r] = lane < nsplit ? part_m[(int64_t)lane * P + pi] : -INFINITY;
    lsr[r] = lane < nsplit ? part_l[(int64_t)lane * P + pi] : 0.f;
  }
  float Mr[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    // the max across the wave, the scale factors once per split; L and O then sum the splits in
    // order with the same fused operations as a sequential loop (bitwise the same result)
    float M = msr[r];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) M = fmaxf(M, __shfl_xor(M, o, 64));
    Mr[r] = M;
    // accurate exp / log here (once per row and split): the backward normalises P_ij =
    // exp(S_ij - lse_i) with this lse, so an error common to every row (an approximation bias of
    // a fast log at the nearly equal L of a batch) would not average out in dC's sums over rows;
    // lse is formed in fp64 and rounded once (an unbiased per-row rounding)
    sc_s[wave][r][lane] = lane < nsr[r] ? expf(msr[r] - M) : 0.f;
    pl_s[wave][r][lane] = lsr[r];
    // lse in the base the passes exponentiate in: the row's exponentials sum to
    // L' = sum_s l_s 2^((m_s - M) IB_LOG2E), and the col pass's P_ij = 2^((s_ij - lse) IB_LOG2E)
    // sums to 1 over j exactly when lse = M + log2(L') / IB_LOG2E. (With the natural log the P of
    // every row would sum to 1 - 8.4 * 1.3e-8, log2(e) rounded to fp32 — a bias common to all rows
    // that the batch sums of dC (the item tower's bias and weight gradients) amplify ~100x.)
    const double l2e = (double)IB_LOG2E;
    tl_s[wave][r][lane] = lane < nsr[r] ? (double)lsr[r] * exp2(((double)msr[r] - (double)M) * l2e) : 0.0;
  }
  __builtin_amdgcn_wave_barrier();
  double my_loss = 0.0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t i = i0 + r;
    if (i >= B) break;  // (wave-uniform)
    const int nsplit = nsr[r];
    float L = 0.f;
    for (int s = 0; s < nsplit; ++s) L = fmaf(pl_s[wave][r][s], sc_s[wave][r][s], L);
    double Ld = 0.0;
    for (int s = 0; s < nsplit; ++s) Ld += tl_s[wave][r][s];
    const double l2e = (double)IB_LOG2E;
    const double lse_d = (double)Mr[r] + log2(Ld) / l2e;
    const float lse_i = (float)lse_d;
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < NDL; ++k)
      if (lane + 64 * k < D) dot += ur[r][k] * cr[r][k];
    dot = wave_sum(dot);
    const double li_d = lse_d - (double)dot;
    const float li = (float)li_d;
    if (lane == 0) {
      lse[i] = lse_i;
      row_loss[i] = li;
    }
    my_loss += li_d;
    if (dU) {
      const float invL = 1.f / L;
      const int64_t pi = pir[r];
#pragma unroll
      for (int k = 0; k < NDL; ++k) {
        const int d = lane + 64 * k;
        if (d >= D) break;
        float o = 0.f;
#pragma unroll
        for (int s = 0; s < PRE; ++s)
          if (s < nsplit) o = fmaf(por[r][s][k], sc_s[wave][r][s], o);
        for (int s = PRE; s < nsplit; ++s) o = fmaf(part_o[((int64_t)s * P + pi) * D + d], sc_s[wave][r][s], o);
        dU[i * D + d] = weight * (o * invL - cr[r][k]);
      }
    }
  }
  if (lane == 0) wl[wave] = my_loss;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double v = ((wl[0] + wl[1]) + wl[2]) + wl[3];
    if (done) ticket_publish(loss_part + blockIdx.x, v);
    else loss_part[blockIdx.x] = v;
  }
  // the ordered total over the workgroups' partials (final_sum_kernel's sums) by the last
  // workgroup to finish instead of another launch; `done` was zeroed by this sequence's image pass
  if (done) ib_last_block_total(done, loss_part, (int64_t)gridDim.x, loss_sum, loss_sum64);
}

// Col finalize: dC_j = g w (sum_s O'_s[j] - U_j); dU_out = g * dU_unit (both nullable).
template <int D>
__global__ __launch_bounds__(256) void inbatch_col_finalize_kernel(
    const float* __restrict__ U, int64_t B, int nsplit, const float* __restrict__ part_o,
    float weight, const float* __restrict__ gscale, const float* __restrict__ dU_unit,
    float* __restrict__ dU_out, float* __restrict__ dC) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= B * D) return;
  const float g = gscale ? gscale[0] : 1.f;
  float o = 0.f;
  for (int s = 0; s < nsplit; ++s) o += part_o[(int64_t)s * B * D + idx];
  dC[idx] = g * (weight * (o - U[idx]));
  if (dU_unit && dU_out) dU_out[idx] = g * dU_unit[idx];
}

// The same on float4 lanes (every operand 16-B aligned, B D a multiple of 4): one float4 of each
// stream per thread, the partials of all splits loaded before they are summed (same order, so
// bitwise the scalar kernel's result).
template <int NS>
__global__ __launch_bounds__(256) void inbatch_col_finalize4_kernel(
    const f32x4* __restrict__ U, int64_t n4, int nsplit_, const f32x4* __restrict__ part_o, float weight,
    const float* __restrict__ gscale, const f32x4* __restrict__ dU_unit, f32x4* __restrict__ dU_out,
    f32x4* __restrict__ dC, const int32_t* __restrict__ inv = nullptr, int64_t n4p = 0, int dq = 1,
    int64_t sk_ntk = 0, int64_t sk_T = 0, int64_t sk_W = 0, const int64_t* __restrict__ dinfo = nullptr,
    int d_own = 0, int d_str = 0, int64_t sk_grid = 0) {
  // row j's partials at row inv[j] of n4p / dq owned rows (the deduplicated pair), else at j
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= n4) return;
  if (dinfo) {  // device-count form: the col pass's shape from the counts (ib_resolve's rule)
    const int64_t Bo = dinfo[d_own];
    n4p = Bo * dq;
    sk_ntk = (dinfo[d_str] + 31) / 32;
    sk_T = ((Bo + IB_SKB - 1) / IB_SKB) * sk_ntk;
    sk_W = ib_sk_workgroups(Bo, sk_ntk, sk_grid);
  }
  const float g = gscale ? gscale[0] : 1.f;
  // the row / block / slot arithmetic in 32 bits when it fits (it does for every batch the library
  // sizes: B D / 4 < 2^31, (T + 1) W < 2^32): 64-bit divisions were ~4 per thread
  const bool narrow = n4 <= 0x7fffffffLL && n4p <= 0x7fffffffLL && (sk_T + 1) * sk_W <= 0xffffffffLL;
  int64_t pidx = idx, pst = n4;
  if (inv) {
    const int64_t j = narrow ? (int64_t)((uint32_t)idx / (uint32_t)dq) : idx / dq;
    pidx = (int64_t)inv[j] * dq + (idx - j * dq);
    pst = n4p;
  }
  // stream-K partials: the slot count of the owned row's 256-row block
  int nsplit = nsplit_;
  if (sk_W) {
    if (narrow)
      nsplit = ib_sk_slots_t<uint32_t>(((uint32_t)pidx / (uint32_t)dq) / (uint32_t)IB_SKB, (uint32_t)sk_ntk, (uint32_t)sk_T,
                                       (uint32_t)sk_W);
    else
      nsplit = ib_sk_slots(pidx / dq / IB_SKB, sk_ntk, sk_T, sk_W);
  }
  f32x4 po[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) po[s] = s < nsplit ? part_o[(int64_t)s * pst + pidx] : f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 u = U[idx];
  const bool du = dU_unit && dU_out;
  const f32x4 dun = du ? dU_unit[idx] : f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (s < nsplit) o += po[s];
  for (int s = NS; s < nsplit; ++s) o += part_o[(int64_t)s * pst + pidx];
  f32x4 r;
#pragma unroll
  for (int t = 0; t < 4; ++t) r[t] = g * (weight * (o[t] - u[t]));
  dC[idx] = r;
  if (du) {
    f32x4 v;
#pragma unroll
    for (int t = 0; t < 4; ++t) v[t] = g * dun[t];
    dU_out[idx] = v;
  }
}

// ---- fp32 operands on the bf16 matrix cores (precision 6 / 9) -----------------------------------
// Every fp32 operand x is split exactly into three bf16 terms, x = h + m + l (h = bf16(x),
// m = bf16(x - h), l = x - h - m; each difference is exact in fp32 and the last term fits bf16's
// 8-bit significand), and a product x.y becomes the sum of the cross products of the terms, each
// exact in the fp32 accumulator of v_mfma_f32_16x16x32_bf16. precision 9 sums all nine: the
// fp32 products exactly, fp32 accumulation (only the order of the additions differs from the
// f32 MFMA). precision 6 drops m.l, l.m and l.l, whose sum is below 2^-23 of |x.y|: an error at
// the level of one fp32 rounding of each product. The bf16 MFMA does 16x the f32 MFMA's work per
// cycle, so 6 products run the contraction at 2.7x and 9 at 1.8x the f32 MFMA peak.
//
// Kernels (D = 128): both operands are split once into three bf16 plane images per 32-row tile
// (ibx_split_image_kernel; 8-row x 32-column subtiles with XOR-swizzled 16-B chunks, so that
// both the row reads of the S product and the ds_read_b64_tr_b16 column reads of the P.X product
// are conflict-free); the owned rows' planes stay in registers (96 VGPRs); P is split in
// registers and used as the B operand straight from the S accumulator (its k order is the
// accumulator's key order, and the column reads of the other operand follow that order).


// ---- split plane images in HBM ---------------------------------------------------------------
// ibx_split_image_kernel writes X [B][128] fp32 as ceil(B/32) tiles of 24 KB: the three plane
// images of 32 rows, byte for byte the LDS image the kernels read (rows past B are zero). The
// row pass then stages each streamed tile with six 16-B LDS-DMA copies per thread (no VGPRs,
// no VALU) and reads its owned rows' planes straight from the image; the stored col pass
// stages its U tiles the same way, issued after its score-tile waits.
__device__ __forceinline__ void ibx_split_image_block(const float* __restrict__ X, int64_t B, int64_t ntiles,
                                                      char* __restrict__ img, const int32_t* __restrict__ rowmap,
                                                      const int64_t* __restrict__ dcount, int64_t blk) {
  if (dcount) {  // device-count form: B rows from the device, the grid sized for the worst case
    B = dcount[0];
    ntiles = (B + 31) / 32;
  }
  const int64_t f = blk * 256 + threadIdx.x;  // one float4 of X
  if (f >= ntiles * 32 * 32) return;
  const int64_t row = f >> 5;
  const int c4 = (int)(f & 31);
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  // image row `row` = X row rowmap[row] (the deduplicated pair's distinct rows) or X row `row`
  if (row < B) v = *reinterpret_cast<const f32x4*>(X + (rowmap ? (int64_t)rowmap[row] : row) * IBX_D + 4 * c4);
  const IbSplit s0 = ib_split2(v[0], v[1]), s1 = ib_split2(v[2], v[3]);
  char* t = img + (row >> 5) * IBX_BUF + ibx_off((int)(row & 31), c4 >> 1) + 8 * (c4 & 1);
  *reinterpret_cast<u32x2*>(t) = u32x2{s0.h, s1.h};
  *reinterpret_cast<u32x2*>(t + IBX_PLANE) = u32x2{s0.m, s1.m};
  *reinterpret_cast<u32x2*>(t + 2 * IBX_PLANE) = u32x2{s0.l, s1.l};
}

__global__ __launch_bounds__(256) void ibx_split_image_kernel(const float* __restrict__ X, int64_t B,
                                                             int64_t ntiles, char* __restrict__ img,
                                                             const int32_t* __restrict__ rowmap = nullptr,
                                                             const int64_t* __restrict__ dcount = nullptr,
                                                             unsigned int* __restrict__ zero = nullptr) {
  if (zero && blockIdx.x == 0) ticket_zero(zero, threadIdx.x, 256);  // a later pass's ticket counters
  ibx_split_image_block(X, B, ntiles, img, rowmap, dcount, blockIdx.x);
}

// both operands' images in one launch: workgroups [0, na) image side a, the rest side b
struct IbxImg {
  const float* X;
  int64_t B, ntiles;
  char* img;
  const int32_t* rowmap;
  const int64_t* dcount;
};
__global__ __launch_bounds__(256) void ibx_split_image2_kernel(IbxImg a, IbxImg b, int64_t na,
                                                              unsigned int* __restrict__ zero) {
  if (zero && blockIdx.x == 0) ticket_zero(zero, threadIdx.x, 256);  // a later pass's ticket counters
  const int64_t blk = blockIdx.x;
  if (blk < na) ibx_split_image_block(a.X, a.B, a.ntiles, a.img, a.rowmap, a.dcount, blk);
  else ibx_split_image_block(b.X, b.B, b.ntiles, b.img, b.rowmap, b.dcount, blk - na);
}

// Transposed plane image of a 32-row tile (the col pass's U^T operand): per plane 128 d-rows of
// 64 B, row d holding the tile's 32 values of column d in the col pass's k order — 16-B chunk g
// = users ku + 0..3, 16 + ku + 0..3 with ku = 8 (g & 1) + 4 (g >> 1), which is lane (i16, g)'s
// A operand for d = 16 dt + i16, one ds_read_b128 per plane. The chunk of row d sits at slot
// g ^ ((d >> 2) & 2): within each of ds_read_b128's four 16-lane groups the 16 chunks then fall
// in 16 distinct 16-B bank groups (conflict-free). Same bytes per tile (24 KB) and same bf16 words
// as the row image, so the products and their order are unchanged (bitwise the same pass).
__device__ __forceinline__ int ibx_toff(int d, int g) { return 64 * d + 16 * (g ^ ((d >> 2) & 2)); }

__global__ __launch_bounds__(256) void ibx_split_timage_kernel(const float* __restrict__ X, int64_t B,
                                                              int64_t ntiles, char* __restrict__ img,
                                                              const int32_t* __restrict__ rowmap,
                                                              const int64_t* __restrict__ dcount) {
  if (dcount) {  // device-count form: the grid sized for the worst case
    B = dcount[0];
    ntiles = (B + 31) / 32;
  }
  const int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (tile, g, d): a wave = 64 d of one g
  if (f >= ntiles * 512) return;
  const int64_t tile = f >> 9;
  const int d = (int)(f & 127), g = (int)((f >> 7) & 3);
  const int ku = 8 * (g & 1) + 4 * (g >> 1);
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t row = tile * 32 + (j < 4 ? ku + j : 16 + ku + j - 4);
    v[j] = row < B ? X[(rowmap ? (int64_t)rowmap[row] : row) * IBX_D + d] : 0.f;
  }
  IbSplit s[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) s[w] = ib_split2(v[2 * w], v[2 * w + 1]);
  char* t = img + tile * IBX_BUF + ibx_toff(d, g);
  *reinterpret_cast<u32x4*>(t) = u32x4{s[0].h, s[1].h, s[2].h, s[3].h};
  *reinterpret_cast<u32x4*>(t + IBX_PLANE) = u32x4{s[0].m, s[1].m, s[2].m, s[3].m};
  *reinterpret_cast<u32x4*>(t + 2 * IBX_PLANE) = u32x4{s[0].l, s[1].l, s[2].l, s[3].l};
}

// one 24-KB tile image -> LDS by LDS-DMA: thread t copies bytes t*16 + 4096 i, i < 6. Issued in
// inline asm so that the compiler, which cannot tell the two LDS buffers apart, does not drain
// the copies (vmcnt(0)) before the reads of the other buffer; the caller waits vmcnt(0) itself
// before the barrier that publishes the buffer.
// (The saddr form — a uniform SGPR base + one 32-bit offset VGPR for all six copies — measured
// slower: col pass +2.3 %, profiles/r06j_dma_saddr_stagger_ab.txt.)
template <int NW>
__device__ __forceinline__ void ibx_glds_tile(const char* __restrict__ src, char* dst, int tid) {
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)dst);
#pragma unroll
  for (int i = 0; i < IBX_BUF / (NW * 1024); ++i) {
    const char* g = src + i * NW * 1024 + tid * 16;
    const uint32_t m0v = __builtin_amdgcn_readfirstlane(lds0 + i * NW * 1024 + wave * 1024);
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(g), "s"(m0v)
        : "memory");
  }
}


// one dword per lane -> LDS by LDS-DMA (lane l's word lands at dst + 4 l; issued in inline asm like
// ibx_glds_tile, so only the caller's explicit vmcnt waits for it)
__device__ __forceinline__ void ibx_glds_dword(const float* src, float* dst) {
  const uint32_t m0v =
      __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)dst));
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(m0v)
               : "memory");
}

// ---- row pass on v_mfma_f32_16x16x32_bf16 (default for D = 128) --------------------------------
// Row pass of the split kernels on the 16x16x32 shape: under this bf16 load the chip holds a
// higher clock on it than on 32x32x16 (MI355X_MICROARCH.md 'DVFS give-back' item 7; measured
// here: 1.63 -> 1.73 GHz, the row pass 10.45 -> 9.73 ms at B = 65536 at equal MFMA cycles). Per wave: 32 owned users (two 16-column B
// subtiles ub, their planes in registers) against each 32-key tile (two 16-row A subtiles kb).
// Key map: A subtile kb row i = 4 g + r reads tile row r + 4 kb + 8 g, so accumulator acc[kb][ub]
// (lane group g = lane / 16, register r) holds key 8 g + 4 kb + r and user 16 ub + lane % 16.
// The P.K product (O^T = K^T P, m = d, n = user, k = key) then takes [acc[0][ub], acc[1][ub]]
// split into planes as its B operand in natural key order (k = 8 g + j), and its K^T operand is
// two ds_read_b64_tr_b16 per plane (rows 8 g + 4 h + q, h = 0, 1). On the plane image both the
// row reads and the transposed reads are conflict-free with this map (the natural one is 2-way).
// WK (the deduplicated pair): key r of the streamed tiles stands for p.kw[r] identical columns,
// so its exponential enters l and P.K multiplied by that count (kw is padded with zeros to whole
// tiles); the counts of the two buffered tiles sit in LDS beside their images.
template <int NP, int NW, int UB, bool WK = false, bool SK = false>
__global__ __launch_bounds__(64 * NW, 8 / NW) void inbatch_row_m16_kernel(InbatchParams p, const char* __restrict__ Qimg,
                                                                    const char* __restrict__ Kimg) {
  constexpr int D = IBX_D;
  constexpr int NDT = D / 16;
  constexpr bool FRESH = IB_FRESH_TILE_ACC && (!WK || IB_FRESH_WK);  // see the P.K product below
  constexpr bool DF = IB_ROW_DMA_FIRST && WK;  // (the full pair's kernel spills with it)
  constexpr bool STG = IB_ROW_STAGGER && WK;     // see the tile phases below
  constexpr int NB = STG ? 3 : 2;                // LDS tile buffers
  __shared__ __attribute__((aligned(16))) char smem[NB * IBX_BUF];
  __shared__ __attribute__((aligned(16))) float kw_s[NB][32];
  // STG: a late wave's S tile across the barrier (in LDS, not in 16 VGPRs live around the loop)
  __shared__ __attribute__((aligned(16))) f32x4 acc_s[STG ? NW / 2 : 1][2 * UB][64];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  ib_resolve(p);
  if (IB_PRIO_HALF && __builtin_amdgcn_readfirstlane(wave) >= NW / 2) __builtin_amdgcn_s_setprio(1);
  const int64_t B = p.B;              // owned users
  const int64_t NT = ib_ntiles(B);    // owned tiles (the score tiles' user stride)
  const int64_t Bs = p.Bs;            // streamed keys
  const int64_t NTs = ib_ntiles(Bs);
  constexpr int QW = 16 * UB;  // owned users per wave
  IbSeg<SK> sg(p, QW * NW);  // the workgroup's (owned block, key range, partial slot) segments
  int64_t blk, kb0, ke, split;
  while (sg.next(blk, kb0, ke, split)) {
    const int64_t q0 = blk * (QW * NW) + wave * QW;  // the wave's first user
    const int ntiles = ke > kb0 ? (int)((ke - kb0 + 31) / 32) : 0;
    const int64_t kt0 = kb0 / 32;

    if (ntiles > 0) {
      ibx_glds_tile<NW>(Kimg + kt0 * IBX_BUF, smem, tid);
      if constexpr (WK)
        if (tid < 32) kw_s[0][tid] = p.kw[kt0 * 32 + tid];
    }

    // owned users' planes (B operand of S^T = K Q^T): tile q0 / 32 + ub / 2, row 16 (ub & 1) + i16,
    // chunk 4 c + g (waves past the last tile read the last tile; never stored)
    u32x4 qp[UB][D / 32][3];
  #pragma unroll
    for (int ub = 0; ub < UB; ++ub) {
      int64_t qt = q0 / 32 + ub / 2;
      if (qt >= NT) qt = NT - 1;
      const char* qi = Qimg + qt * IBX_BUF;
  #pragma unroll
      for (int c = 0; c < D / 32; ++c)
  #pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          qp[ub][c][pl] =
              *reinterpret_cast<const u32x4*>(qi + pl * IBX_PLANE + ibx_off(16 * (ub & 1) + i16, 4 * c + g));
    }
    // row-read bases (A operand of S^T: subtile kb row i16 -> tile row rho, chunk 4 c + g = base + 512 c)
    int rb[2];
  #pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const int rho = (i16 & 3) + 4 * kb + 8 * ((i16 >> 2) & 1) + 16 * (i16 >> 3);
      rb[kb] = ibx_off(rho, g);
    }
    // transposed-read bases: lane 4 q + pp of group g reads row 8 g + 4 h + q, columns 16 dt + 4 pp
    // .. + 3 (chunk 2 dt + pp / 2, byte 8 (pp & 1)) = tb[h][dt & 1] + 512 (dt >> 1)
    int tb[2][2];
    {
      const int q = i16 >> 2, pp = i16 & 3;
  #pragma unroll
      for (int h = 0; h < 2; ++h)
  #pragma unroll
        for (int o = 0; o < 2; ++o) tb[h][o] = ibx_off(8 * g + 4 * h + q, 2 * o + (pp >> 1)) + 8 * (pp & 1);
    }

    f32x4 Ot[NDT][UB];  // O^T: d = 16 dt + 4 g + r, user 16 ub + i16
  #pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
  #pragma unroll
      for (int ub = 0; ub < UB; ++ub) Ot[dt][ub] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m[UB], l[UB];
  #pragma unroll
    for (int ub = 0; ub < UB; ++ub) {
      m[ub] = -INFINITY;
      l[ub] = 0.f;
    }
    const bool store_s = p.S && q0 < B;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // One key tile is three phases: S (the scores' MFMAs, the next tile's copy, the score stores),
    // P (softmax, P split, the P.K MFMAs) and the block end (waits, barrier). STG (IB_ROW_STAGGER):
    // the second half of the waves runs each tile's P phase one block late, ahead of the next
    // tile's S phase, so that one half's softmax VALU sits beside the other half's MFMAs instead of
    // both halves leaving the matrix pipe idle together; the tiles then rotate through three LDS
    // buffers (a late wave reads tile t - 1 while tile t + 1 lands). Each wave's arithmetic and its
    // order are unchanged (bitwise the unstaggered pass).
    // PARTIAL: the split may end inside a tile (B % 32 != 0 on the last split); otherwise the
    // per-key masking is compiled out
    f32x4 acc[2][UB];
    float wn = 0.f;
    // the next tile by LDS-DMA into buffer nbuf (read by nobody since the last barrier)
    auto next_tile = [&](int t, int nbuf) __attribute__((always_inline)) {
      int64_t nt = kt0 + t + 1;
      if (nt >= NTs) nt = NTs - 1;
      ibx_glds_tile<NW>(Kimg + nt * IBX_BUF, smem + nbuf * IBX_BUF, tid);
      if constexpr (WK) {
        if constexpr (DF) {  // the counts by LDS-DMA too: no register the compiler would wait for
          if (tid < 32) ibx_glds_dword(p.kw + nt * 32 + tid, &kw_s[nbuf][0]);
        } else {
          if (tid < 32) wn = p.kw[nt * 32 + tid];
        }
      }
    };
    // dma: the next tile's copy is issued here (else the caller issued it at the block's start)
    auto phase_s = [&](int t, int buf, int nbuf, auto partial, bool dma = true) __attribute__((always_inline)) {
      const char* img = smem + buf * IBX_BUF;
      const int64_t kbase = kb0 + 32 * (int64_t)t;
      const int rem = (int)((ke - kbase) < 32 ? (ke - kbase) : 32);
  #pragma unroll
      for (int kb = 0; kb < 2; ++kb)
  #pragma unroll
        for (int ub = 0; ub < UB; ++ub) acc[kb][ub] = f32x4{0.f, 0.f, 0.f, 0.f};
      // IB_ROW_S_PREFETCH (timing switch): chunk c + 1's K rows read ahead of chunk c's MFMAs
      constexpr bool SPF = IB_ROW_S_PREFETCH != 0;
      auto read_k = [&](int c, u32x4 (&a)[2][3]) __attribute__((always_inline)) {
  #pragma unroll
        for (int kb = 0; kb < 2; ++kb)
  #pragma unroll
          for (int pl = 0; pl < 3; ++pl)
            a[kb][pl] = *reinterpret_cast<const u32x4*>(img + pl * IBX_PLANE + rb[kb] + 512 * c);
      };
      u32x4 k_pf[2][2][3];
      if constexpr (SPF) read_k(0, k_pf[0]);
  #pragma unroll
      for (int c = 0; c < D / 32; ++c) {
        u32x4 a[2][3];
        if constexpr (SPF) {
          if (c + 1 < D / 32) read_k(c + 1, k_pf[(c + 1) & 1]);
  #pragma unroll
          for (int kb = 0; kb < 2; ++kb)
  #pragma unroll
            for (int pl = 0; pl < 3; ++pl) a[kb][pl] = k_pf[c & 1][kb][pl];
        } else {
          read_k(c, a);
        }
        const u32x4* aa[2 * UB];
        const u32x4* bb[2 * UB];
        f32x4* cc[2 * UB];
  #pragma unroll
        for (int kb = 0; kb < 2; ++kb)
  #pragma unroll
          for (int ub = 0; ub < UB; ++ub) {
            aa[kb * UB + ub] = a[kb];
            bb[kb * UB + ub] = qp[ub][c];
            cc[kb * UB + ub] = &acc[kb][ub];
          }
        mfma16_split_n<NP, 2 * UB>(aa, bb, cc);
      }
      // DF: the next tile's copy before the score stores, so that the end-of-step wait leaves the
      // stores in flight
      if constexpr (DF)
        if (dma) next_tile(t, nbuf);
      if (store_s) {
        // straight from the accumulators: register r of acc[kb][ub] is S(user 16 ub + i16,
        // item 8 g + 4 kb + r), one dword store each (the offsets past the lane's base are
        // instruction immediates; each store fills four 64-B runs)
        float* tbp = p.S + ((kbase / 32) * NT + q0 / 32) * 1024 + 128 * g + ib_slot(i16);
  #pragma unroll
        for (int kb = 0; kb < 2; ++kb)
  #pragma unroll
          for (int ub = 0; ub < UB; ++ub)
  #pragma unroll
            for (int r = 0; r < 4; ++r)
              tbp[1024 * (ub / 2) + 512 * (ub & 1) + 16 * (4 * kb + r)] = acc[kb][ub][r];
      }
      if constexpr (!DF)
        if (dma) next_tile(t, nbuf);
      if constexpr (decltype(partial)::value) {
        if (rem < 32) {
  #pragma unroll
          for (int kb = 0; kb < 2; ++kb)
  #pragma unroll
            for (int ub = 0; ub < UB; ++ub)
  #pragma unroll
              for (int r = 0; r < 4; ++r)
                if (8 * g + 4 * kb + r >= rem) acc[kb][ub][r] = -INFINITY;
        }
      }
    };
    auto phase_p = [&](int buf) __attribute__((always_inline)) {
      const char* img = smem + buf * IBX_BUF;
      float alpha[UB];
      bool grow = false;
      f32x4 wk[2];  // WK: counts of keys 8 g + 4 kb + r
      if constexpr (WK) {
        wk[0] = *reinterpret_cast<const f32x4*>(&kw_s[buf][8 * g]);
        wk[1] = *reinterpret_cast<const f32x4*>(&kw_s[buf][8 * g + 4]);
      }
  #pragma unroll
      for (int ub = 0; ub < UB; ++ub) {
        float mx = fmaxf(fmaxf(fmaxf(acc[0][ub][0], acc[0][ub][1]), fmaxf(acc[0][ub][2], acc[0][ub][3])),
                         fmaxf(fmaxf(acc[1][ub][0], acc[1][ub][1]), fmaxf(acc[1][ub][2], acc[1][ub][3])));
        mx = ib_max_x32(ib_max_x16(mx));
        const float m_new = fmaxf(m[ub], mx);
        alpha[ub] = __expf(m[ub] - m_new);
        grow |= m_new > m[ub];
        float ps = 0.f;
        const float mz = m_new * IB_LOG2E;  // exp(s - m) = 2^(s log2 e - m log2 e): one fma + v_exp
  #pragma unroll
        for (int kb = 0; kb < 2; ++kb)
  #pragma unroll
          for (int r = 0; r < 4; r += 2) {  // packed fma per pair
            const f32x2 y = f32x2{acc[kb][ub][r], acc[kb][ub][r + 1]} * IB_LOG2E - mz;
            f32x2 e = f32x2{__builtin_amdgcn_exp2f(y[0]), __builtin_amdgcn_exp2f(y[1])};
            if constexpr (WK) e = e * f32x2{wk[kb][r], wk[kb][r + 1]};
            acc[kb][ub][r] = e[0];
            acc[kb][ub][r + 1] = e[1];
            ps += e[0] + e[1];
          }
        l[ub] = l[ub] * alpha[ub] + ps;
        m[ub] = m_new;
      }
      if (!FRESH && __any(grow)) {
  #pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
  #pragma unroll
          for (int ub = 0; ub < UB; ++ub) Ot[dt][ub] *= alpha[ub];
      }
      // P (key 8 g + j, user) split into planes: the B operand of O^T += K^T P
      u32x4 pb[UB][3];
  #pragma unroll
      for (int ub = 0; ub < UB; ++ub)
  #pragma unroll
        for (int w = 0; w < 4; ++w) {
          const IbSplit x = ib_split2v(f32x2{acc[w >> 1][ub][2 * (w & 1)], acc[w >> 1][ub][2 * (w & 1) + 1]});
          pb[ub][0][w] = x.h;
          pb[ub][1][w] = x.m;
          pb[ub][2][w] = x.l;
        }
      // K^T of d-tile dt (three planes) from the LDS tile; IB_ROW_PREFETCH_A: d-tile dt + 1's is read
      // before d-tile dt's MFMAs, so its LDS latency hides behind them
      auto read_a = [&](int dt, u32x4 (&a)[3]) __attribute__((always_inline)) {
  #pragma unroll
        for (int h = 0; h < 2; ++h)
  #pragma unroll
          for (int pl = 0; pl < 3; ++pl) {
            const ib_s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) ib_s16x4*)(img + tb[h][dt & 1] + pl * IBX_PLANE + 512 * (dt >> 1)));
            const u32x2 w2 = __builtin_bit_cast(u32x2, v);
            a[pl][2 * h] = w2[0];
            a[pl][2 * h + 1] = w2[1];
          }
      };
      constexpr bool PFA = IB_ROW_PREFETCH_A != 0;
      u32x4 a_pf[2][3];
      if constexpr (PFA) read_a(0, a_pf[0]);
  #pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        u32x4 a[3];
        if constexpr (PFA) {
          if (dt + 1 < NDT) read_a(dt + 1, a_pf[(dt + 1) & 1]);
  #pragma unroll
          for (int pl = 0; pl < 3; ++pl) a[pl] = a_pf[dt & 1][pl];
        } else {
          read_a(dt, a);
        }
        // the tile's products into a fresh accumulator, then one fp32 fma into O (with the
        // rescale: alpha = 1 exactly unless the running max grew): the bf16 MFMA's accumulation
        // loses the low bits of products far below its accumulator, a bias common to every output
        // when the products share a sign (a tower output's bias column: -1.7 * 2^-24 |sum| over
        // 4096 keys on one running accumulator, -0.08 this way; tools/probes/split_dot_bias.hip)
        const u32x4* aa[UB];
        const u32x4* bb[UB];
        f32x4 tile_o[UB];
        f32x4* cc[UB];
  #pragma unroll
        for (int ub = 0; ub < UB; ++ub) {
          aa[ub] = a;
          bb[ub] = pb[ub];
          tile_o[ub] = f32x4{0.f, 0.f, 0.f, 0.f};
          cc[ub] = FRESH ? &tile_o[ub] : &Ot[dt][ub];
        }
        mfma16_split_n<NP, UB>(aa, bb, cc);
        if constexpr (FRESH) {
  #pragma unroll
          for (int ub = 0; ub < UB; ++ub)
  #pragma unroll
            for (int r = 0; r < 4; ++r) Ot[dt][ub][r] = fmaf(Ot[dt][ub][r], alpha[ub], tile_o[ub][r]);
          __builtin_amdgcn_sched_barrier(0);  // one dt's tile accumulators live at a time
        }
      }
    };
    auto block_end = [&](int nbuf) __attribute__((always_inline)) {
      if constexpr (DF) {
        // the next tile's copies have landed; this tile's 8 UB score stores, issued after them, may
        // still be in flight: vmcnt(8 UB) (CDNA counts loads, stores and LDS-DMA in issue order in
        // vmcnt). The count assumes the score stores are the only vector-memory operations between
        // the copies and this wait (the loop body issues nothing else there: the stores come from the
        // accumulators, every other operand is in LDS or registers); the assembler encodes the field
        static_assert(UB == 2, "the end-of-step wait counts the 16 score stores of UB = 2");
        if (store_s) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next tile's copies have landed
      }
      if constexpr (WK && !DF)
        if (tid < 32) kw_s[nbuf][tid] = wn;
      __syncthreads();
    };
    // IB_ROW_SPLIT_UB (the deduplicated row pass): a tile's work per owned subtile ub instead of per
    // phase — S of ub 0; S of ub 1 with ub 0's softmax and P split beside its MFMAs; ub 0's P.K with
    // ub 1's softmax and split beside it; ub 1's P.K — so the softmax VALU sits beside the wave's own
    // MFMAs instead of between its two MFMA phases (where both waves of a SIMD, released by the same
    // barrier, left the matrix pipe idle together). Each accumulator's products, each subtile's
    // softmax and the score stores are those of phase_s / phase_p, in the same order per register
    // (a subtile whose max did not grow has alpha = 1 exactly, so its O rescale is skipped per
    // subtile instead of per wave): bitwise the phase form. The K rows and K^T fragments are read
    // from LDS once per subtile (twice per tile). Measured (profiles/r06aa_row_split_ub_ab.txt): bitwise
    // the phase form (output digests equal), row pass +114 / +89 us per C3 step in the two orders —
    // hipcc still clusters the softmax after the MFMAs (its max / permlane chain gates the rest) and
    // the doubled LDS reads and their waits cost more than the overlap gains. Off.
    auto step_ub = [&](int t, int buf, int nbuf, auto partial) __attribute__((always_inline)) {
      const char* img = smem + buf * IBX_BUF;
      const int64_t kbase = kb0 + 32 * (int64_t)t;
      const int rem = (int)((ke - kbase) < 32 ? (ke - kbase) : 32);
      constexpr int ia[9] = {2, 2, 1, 1, 2, 0, 1, 0, 0}, ibp[9] = {2, 1, 2, 1, 0, 2, 0, 1, 0};
      auto s_ub = [&](int ub) __attribute__((always_inline)) {
        acc[0][ub] = f32x4{0.f, 0.f, 0.f, 0.f};
        acc[1][ub] = f32x4{0.f, 0.f, 0.f, 0.f};
  #pragma unroll
        for (int c = 0; c < D / 32; ++c) {
          u32x4 a[2][3];
  #pragma unroll
          for (int kb = 0; kb < 2; ++kb)
  #pragma unroll
            for (int pl = 0; pl < 3; ++pl)
              a[kb][pl] = *reinterpret_cast<const u32x4*>(img + pl * IBX_PLANE + rb[kb] + 512 * c);
  #pragma unroll
          for (int k = 9 - NP; k < 9; ++k)
  #pragma unroll
            for (int kb = 0; kb < 2; ++kb) acc[kb][ub] = mfma16_bf16(a[kb][ia[k]], qp[ub][c][ibp[k]], acc[kb][ub]);
        }
      };
      auto store_mask_ub = [&](int ub) __attribute__((always_inline)) {
        if (store_s) {
          float* tbp = p.S + ((kbase / 32) * NT + q0 / 32) * 1024 + 128 * g + ib_slot(i16);
  #pragma unroll
          for (int kb = 0; kb < 2; ++kb)
  #pragma unroll
            for (int r = 0; r < 4; ++r) tbp[1024 * (ub / 2) + 512 * (ub & 1) + 16 * (4 * kb + r)] = acc[kb][ub][r];
        }
        if constexpr (decltype(partial)::value) {
          if (rem < 32) {
  #pragma unroll
            for (int kb = 0; kb < 2; ++kb)
  #pragma unroll
              for (int r = 0; r < 4; ++r)
                if (8 * g + 4 * kb + r >= rem) acc[kb][ub][r] = -INFINITY;
          }
        }
      };
      const f32x4 wk[2] = {*reinterpret_cast<const f32x4*>(&kw_s[buf][8 * g]),
                           *reinterpret_cast<const f32x4*>(&kw_s[buf][8 * g + 4])};
      float alpha[UB];
      bool grow[UB];
      u32x4 pb[UB][3];
      auto softmax_ub = [&](int ub) __attribute__((always_inline)) {
        float mx = fmaxf(fmaxf(fmaxf(acc[0][ub][0], acc[0][ub][1]), fmaxf(acc[0][ub][2], acc[0][ub][3])),
                         fmaxf(fmaxf(acc[1][ub][0], acc[1][ub][1]), fmaxf(acc[1][ub][2], acc[1][ub][3])));
        mx = ib_max_x32(ib_max_x16(mx));
        const float m_new = fmaxf(m[ub], mx);
        alpha[ub] = __expf(m[ub] - m_new);
        grow[ub] = m_new > m[ub];
        float ps = 0.f;
        const float mz = m_new * IB_LOG2E;
  #pragma unroll
        for (int kb = 0; kb < 2; ++kb)
  #pragma unroll
          for (int r = 0; r < 4; r += 2) {
            const f32x2 y = f32x2{acc[kb][ub][r], acc[kb][ub][r + 1]} * IB_LOG2E - mz;
            f32x2 e = f32x2{__builtin_amdgcn_exp2f(y[0]), __builtin_amdgcn_exp2f(y[1])};
            e = e * f32x2{wk[kb][r], wk[kb][r + 1]};
            acc[kb][ub][r] = e[0];
            acc[kb][ub][r + 1] = e[1];
            ps += e[0] + e[1];
          }
        l[ub] = l[ub] * alpha[ub] + ps;
        m[ub] = m_new;
  #pragma unroll
        for (int w = 0; w < 4; ++w) {
          const IbSplit x = ib_split2v(f32x2{acc[w >> 1][ub][2 * (w & 1)], acc[w >> 1][ub][2 * (w & 1) + 1]});
          pb[ub][0][w] = x.h;
          pb[ub][1][w] = x.m;
          pb[ub][2][w] = x.l;
        }
      };
      auto read_a = [&](int dt, u32x4 (&a)[3]) __attribute__((always_inline)) {
  #pragma unroll
        for (int h = 0; h < 2; ++h)
  #pragma unroll
          for (int pl = 0; pl < 3; ++pl) {
            const ib_s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) ib_s16x4*)(img + tb[h][dt & 1] + pl * IBX_PLANE + 512 * (dt >> 1)));
            const u32x2 w2 = __builtin_bit_cast(u32x2, v);
            a[pl][2 * h] = w2[0];
            a[pl][2 * h + 1] = w2[1];
          }
      };
      auto pk_ub = [&](int ub) __attribute__((always_inline)) {
        if (__any(grow[ub])) {
  #pragma unroll
          for (int dt = 0; dt < NDT; ++dt) Ot[dt][ub] *= alpha[ub];
        }
        u32x4 a_pf[2][3];
        read_a(0, a_pf[0]);
  #pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          if (dt + 1 < NDT) read_a(dt + 1, a_pf[(dt + 1) & 1]);
  #pragma unroll
          for (int k = 9 - NP; k < 9; ++k) Ot[dt][ub] = mfma16_bf16(a_pf[dt & 1][ia[k]], pb[ub][ibp[k]], Ot[dt][ub]);
        }
      };
      s_ub(0);
      next_tile(t, nbuf);  // (DF: before the score stores, which the block end leaves in flight)
      store_mask_ub(0);
      __builtin_amdgcn_sched_barrier(0);
      // interleave: per S chunk its 6 K-row reads, then each MFMA followed by up to 2 VALU of the
      // other subtile's softmax / split (hipcc otherwise clusters the VALU after the MFMAs)
      auto interleave = [&](auto groups, auto mfmas) __attribute__((always_inline)) {
  #pragma unroll
        for (int i = 0; i < decltype(groups)::value; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
  #pragma unroll
          for (int j = 0; j < decltype(mfmas)::value; ++j) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
          }
        }
      };
      s_ub(1);
      softmax_ub(0);
      interleave(std::integral_constant<int, D / 32>{}, std::integral_constant<int, 2 * NP>{});
      __builtin_amdgcn_sched_barrier(0);
      store_mask_ub(1);
      __builtin_amdgcn_sched_barrier(0);
      pk_ub(0);
      softmax_ub(1);
      interleave(std::integral_constant<int, NDT>{}, std::integral_constant<int, NP>{});
      __builtin_amdgcn_sched_barrier(0);
      pk_ub(1);
    };
    constexpr bool SPLITUB = IB_ROW_SPLIT_UB && WK && DF && !FRESH && !STG && UB == 2;
    if constexpr (STG) {
      const bool late = __builtin_amdgcn_readfirstlane(wave) >= NW / 2;
      auto run = [&](auto partial) __attribute__((always_inline)) {
        f32x4(&as)[2 * UB][64] = acc_s[late ? wave - NW / 2 : 0];
        auto park = [&]() __attribute__((always_inline)) {
  #pragma unroll
          for (int kb = 0; kb < 2; ++kb)
  #pragma unroll
            for (int ub = 0; ub < UB; ++ub) as[kb * UB + ub][lane] = acc[kb][ub];
        };
        auto unpark = [&]() __attribute__((always_inline)) {
  #pragma unroll
          for (int kb = 0; kb < 2; ++kb)
  #pragma unroll
            for (int ub = 0; ub < UB; ++ub) acc[kb][ub] = as[kb * UB + ub][lane];
        };
        int buf = 0, pbuf = NB - 1;  // tile t's buffer t % 3, tile t - 1's
        if (late) {
          for (int t = 0; t < ntiles; ++t) {
            const int nbuf = buf == NB - 1 ? 0 : buf + 1;
            // the next tile's copy first (its buffer was last read before the last barrier), so its
            // latency is not exposed at this block's end, right after the late S phase
            next_tile(t, nbuf);
            if (t > 0) {
              unpark();
              phase_p(pbuf);
            }
            phase_s(t, buf, nbuf, partial, false);
            park();
            block_end(nbuf);
            pbuf = buf;
            buf = nbuf;
          }
          if (ntiles > 0) {
            unpark();
            phase_p(pbuf);
          }
        } else {
          for (int t = 0; t < ntiles; ++t) {
            const int nbuf = buf == NB - 1 ? 0 : buf + 1;
            phase_s(t, buf, nbuf, partial);
            phase_p(buf);
            block_end(nbuf);
            buf = nbuf;
          }
        }
        __syncthreads();  // the late waves' last reads before the next segment's first copy
      };
      if ((ke - kb0) % 32 == 0) run(std::false_type{});
      else run(std::true_type{});
    } else {
      auto step = [&](int t, int buf, auto partial) __attribute__((always_inline)) {
        if (t >= ntiles) return;
        if constexpr (SPLITUB) {
          step_ub(t, buf, buf ^ 1, partial);
        } else {
          phase_s(t, buf, buf ^ 1, partial);
          phase_p(buf);
        }
        block_end(buf ^ 1);
      };
      if ((ke - kb0) % 32 == 0) {
        for (int t = 0; t < ntiles; t += 2) {
          step(t, 0, std::false_type{});
          step(t + 1, 1, std::false_type{});
        }
      } else {
        for (int t = 0; t < ntiles; t += 2) {
          step(t, 0, std::true_type{});
          step(t + 1, 1, std::true_type{});
        }
      }
    }

  #pragma unroll
    for (int ub = 0; ub < UB; ++ub) {
      const float lt = ib_sum_x32(ib_sum_x16(l[ub]));
      const int64_t q = q0 + 16 * ub + i16;
      if (g == 0 && q < B) {
        p.part_m[split * B + q] = m[ub];
        p.part_l[split * B + q] = lt;
      }
      if (q < B) {
        float* po = p.part_o + (split * B + q) * D + 4 * g;
  #pragma unroll
        for (int dt = 0; dt < NDT; ++dt) *reinterpret_cast<f32x4*>(po + 16 * dt) = Ot[dt][ub];
      }
    }
  }  // segments
}

// Stored col pass on the 16x16x32 shape (owned = items, 32 per wave as two 16-column subtiles
// ib; streamed = 32-user tiles): O'^T = U^T P with P = exp(S - lse_user) from the kept scores.
// Lane (g, i16) loads, for subtile ib, slots 4 g + 0..3 of both 16-user halves h at item
// 16 ib + i16 (one 1-KB run per load instruction), which are the B operand's k = 8 g + 4 h + q;
// k = (g, h, q) is user ib_user(g, h, q) = 16 h + 8 (g & 1) + 4 (g / 2) + q (the slot order), and
// the U^T operand is two ds_read_b64_tr_b16 per plane of those user rows (conflict-free on the
// plane image: within each 32-lane half the rows differ in bits 0-1 and the chunk swizzle).
// Software-pipelined by one step: the exp / split of tile t+1's P (VALU) is issued beside tile
// t's MFMAs (P(t) was built during step t-1) instead of ahead of them. Scores are loaded two
// steps ahead, the users' lse one step ahead of their use into a 3-slot LDS ring, the U tile one
// step ahead by LDS-DMA into the other buffer (issued after the wait for the next P's scores, so
// the compiler's counted waits never drain it; one vmcnt(0) before the end-of-step barrier).
// Bitwise equal to the unpipelined pass (same sums, same order).
// WK (the deduplicated pair): streamed user r stands for count_r identical rows; the count enters P
// as 2^(s log2 e - (lse log2 e - log2 count)), whose bias lse_k[r] ib_lz_kernel formed ahead (no
// extra VALU or registers in the loop).
// TIMG: Kimg is the transposed image (ibx_split_timage_kernel): U^T is 3 ds_read_b128 per d-tile
// instead of 6 ds_read_b64_tr_b16, the same words in the same k order.
template <int NP, int NW, bool WK = false, bool SK = false, bool TIMG = false>
__global__ __launch_bounds__(64 * NW, 8 / NW) void inbatch_col_m16_kernel(InbatchParams p, const float* __restrict__ S,
                                                                    const char* __restrict__ Kimg) {
  constexpr int D = IBX_D;
  constexpr int NDT = D / 16;
  constexpr bool FRESH = IB_FRESH_TILE_ACC;  // see the U^T P product below
  __shared__ __attribute__((aligned(16))) char smem[2 * IBX_BUF];
  __shared__ __attribute__((aligned(16))) float lse_s[3][32];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  ib_resolve(p);
  if (IB_PRIO_HALF && __builtin_amdgcn_readfirstlane(wave) >= NW / 2) __builtin_amdgcn_s_setprio(1);
  const int64_t B = p.B;    // owned items
  const int64_t Bs = p.Bs;  // streamed users
  const int64_t NT = ib_ntiles(B);
  const int64_t NTs = ib_ntiles(Bs);  // user tiles: the score tiles' stride
  IbSeg<SK> sg(p, IB_QW * NW);  // the workgroup's (owned block, key range, partial slot) segments
  int64_t blk, kb, ke, split;
  while (sg.next(blk, kb, ke, split)) {
    const int ntiles = ke > kb ? (int)((ke - kb + 31) / 32) : 0;
    const int64_t kt0 = kb / 32;
    const int64_t q0 = blk * (IB_QW * NW) + wave * IB_QW;  // the wave's first item
    int64_t itile = q0 / 32;
    if (itile >= NT) itile = NT - 1;
    const float* Sbase = S + itile * NTs * 1024 + 16 * i16 + 4 * g;

    f32x4 Ot[NDT][2];  // O'^T: d = 16 dt + 4 g + r, item 16 ib + i16
  #pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
  #pragma unroll
      for (int ib = 0; ib < 2; ++ib) Ot[dt][ib] = f32x4{0.f, 0.f, 0.f, 0.f};

    int tb[2][2];
    {
      const int q = i16 >> 2, pp = i16 & 3;
  #pragma unroll
      for (int h = 0; h < 2; ++h)
  #pragma unroll
        for (int o = 0; o < 2; ++o)
          tb[h][o] = ibx_off(16 * h + 8 * (g & 1) + 4 * (g >> 1) + q, 2 * o + (pp >> 1)) + 8 * (pp & 1);
    }
    const int ku = 8 * (g & 1) + 4 * (g >> 1);  // the lane's first user in each half (k = 8 g + 4 h)
    const int tT = ibx_toff(i16, g);             // (TIMG) row d = 16 dt + i16: + 1024 dt
    float lse_reg = 0.f;
    // U tile kt0 + t (clamped) -> LDS buffer buf by LDS-DMA (no VGPR staging, no ds_write pass)
    auto copy_tile = [&](int t, int buf) __attribute__((always_inline)) {
      int64_t kt = kt0 + t;
      if (kt >= NTs) kt = NTs - 1;
      ibx_glds_tile<NW>(Kimg + kt * IBX_BUF, smem + buf * IBX_BUF, tid);
    };
    auto load_lse = [&](int t) __attribute__((always_inline)) {  // user 32 t + tid % 32 (clamped)
      const int64_t gr = kb + 32 * (int64_t)t + (tid & 31);
      const int64_t gi = gr < ke ? gr : ke - 1;
      if constexpr (WK) {
        lse_reg = p.lse_k[gi];   // (ib_lz_kernel's bias, already in the exponent's base)
      } else {
        lse_reg = p.lse_k[gi];
      }
    };
    auto store_lse = [&](int t) __attribute__((always_inline)) {  // lse log2(e) (every thread: equal values)
      if constexpr (WK) lse_s[t % 3][tid & 31] = lse_reg;
      else lse_s[t % 3][tid & 31] = lse_reg * IB_LOG2E;
    };
    // scores of user tile t: [2 ib + h] = users 16 h + ku + 0..3 at item 16 ib + i16 (clamped)
    auto load_scores = [&](int t, f32x4 (&dst)[4]) __attribute__((always_inline)) {
      int64_t kbase = kb + 32 * (int64_t)t;
      if (kbase >= ke) kbase = kb + 32 * (int64_t)(ntiles - 1);
      const float* src = Sbase + (kbase / 32) * 1024;
  #pragma unroll
      for (int i = 0; i < 4; ++i)
        dst[i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src + 256 * (i >> 1) + 512 * (i & 1)));
    };
    // P of tile t split into planes: the B operand of O'^T += U^T P. P = 2^(s log2 e - lse log2 e)
    // as one packed fma per user pair + v_exp (the row pass's form); users past the split are
    // masked to 0 only on a split that ends inside a tile (PARTIAL)
    auto make_p = [&](int t, const f32x4 (&sb)[4], u32x4 (&pb)[2][3], auto partial) __attribute__((always_inline)) {
      const f32x4 z0 = *reinterpret_cast<const f32x4*>(&lse_s[t % 3][ku]);
      const f32x4 z1 = *reinterpret_cast<const f32x4*>(&lse_s[t % 3][16 + ku]);
      const f32x2 lz[4] = {f32x2{z0[0], z0[1]}, f32x2{z0[2], z0[3]}, f32x2{z1[0], z1[1]}, f32x2{z1[2], z1[3]}};
      int rem = 32;
      if constexpr (decltype(partial)::value) {
        const int64_t kbase = kb + 32 * (int64_t)t;
        rem = (int)((ke - kbase) < 32 ? (ke - kbase) : 32);
      }
  #pragma unroll
      for (int ib = 0; ib < 2; ++ib)
  #pragma unroll
        for (int w = 0; w < 4; ++w) {
          const f32x4 v = sb[2 * ib + (w >> 1)];
          const f32x2 s2 = (w & 1) ? f32x2{v[2], v[3]} : f32x2{v[0], v[1]};
          const f32x2 y = s2 * IB_LOG2E - lz[w];
          f32x2 e = f32x2{__builtin_amdgcn_exp2f(y[0]), __builtin_amdgcn_exp2f(y[1])};
          if constexpr (decltype(partial)::value) {
            const int u = 16 * (w >> 1) + ku + 2 * (w & 1);  // the pair's first user
            if (u >= rem) e[0] = 0.f;
            if (u + 1 >= rem) e[1] = 0.f;
          }
          const IbSplit x = ib_split2v(e);
          pb[ib][0][w] = x.h;
          pb[ib][1][w] = x.m;
          pb[ib][2][w] = x.l;
        }
    };
    // one (ib, w) pair slice of make_p, its two lse values lz = read_lz(t, w) (IB_COL_CHAIN: the
    // eight slices spread over the step's eight d-tiles; the same values as make_p)
    [[maybe_unused]] auto read_lz = [&](int t, int w) __attribute__((always_inline)) {
      return *reinterpret_cast<const f32x2*>(&lse_s[t % 3][16 * (w >> 1) + ku + 2 * (w & 1)]);
    };
    [[maybe_unused]] auto make_p_part = [&](int t, const f32x4 (&sb)[4], u32x4 (&pb)[2][3], auto partial, int ib, int w, f32x2 lz)
                           __attribute__((always_inline)) {
      const f32x4 v = sb[2 * ib + (w >> 1)];
      const f32x2 s2 = (w & 1) ? f32x2{v[2], v[3]} : f32x2{v[0], v[1]};
      const f32x2 y = s2 * IB_LOG2E - lz;
#if IB_COL_PROBE == 1  // timing probe only (wrong results): no exponentials
      f32x2 e = y;
#else
      f32x2 e = f32x2{__builtin_amdgcn_exp2f(y[0]), __builtin_amdgcn_exp2f(y[1])};
#endif
      if constexpr (decltype(partial)::value) {
        const int64_t kbase = kb + 32 * (int64_t)t;
        const int rem = (int)((ke - kbase) < 32 ? (ke - kbase) : 32);
        const int u = 16 * (w >> 1) + ku + 2 * (w & 1);  // the pair's first user
        if (u >= rem) e[0] = 0.f;
        if (u + 1 >= rem) e[1] = 0.f;
      }
      const IbSplit x = ib_split2v(e);
      pb[ib][0][w] = x.h;
      pb[ib][1][w] = x.m;
      pb[ib][2][w] = x.l;
    };
    f32x4 sbA[4], sbB[4];
    u32x4 pbA[2][3], pbB[2][3];
    if (ntiles > 0) {
      copy_tile(0, 0);
      load_scores(0, sbA);
      load_scores(1, sbB);
      load_lse(0);
      store_lse(0);
      load_lse(1);
      store_lse(1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile 0 has landed
      __syncthreads();
      if ((ke - kb) % 32 == 0) make_p(0, sbA, pbA, std::false_type{});
      else make_p(0, sbA, pbA, std::true_type{});
    }
    // step t: P(t) in pb_t, scores(t+1) in sb_t1; sb_t (consumed) is refilled with scores(t+2)
    auto step = [&](int t, int buf, f32x4 (&sb_t)[4], const f32x4 (&sb_t1)[4], const u32x4 (&pb_t)[2][3],
                    u32x4 (&pb_t1)[2][3], auto partial) __attribute__((always_inline)) {
      const char* img = smem + buf * IBX_BUF;
#if IB_COL_COPY_FIRST
      // the next U tile into buffer buf ^ 1 (last read in step t - 1, before its barrier) first, then
      // the lse and scores of t + 2: make_p's counted wait for the scores of t + 1 then also covers
      // the copy, and the end of the step waits for neither the scores of t + 2 nor anything later
      copy_tile(t + 1, buf ^ 1);
#endif
      load_lse(t + 2);
      load_scores(t + 2, sb_t);
      // U^T of d-tile dt (three planes) from the LDS tile
      auto read_a = [&](int dt, u32x4 (&a)[3]) __attribute__((always_inline)) {
        if constexpr (TIMG) {
  #pragma unroll
          for (int pl = 0; pl < 3; ++pl)
            a[pl] = *reinterpret_cast<const u32x4*>(img + tT + pl * IBX_PLANE + 1024 * dt);
        } else {
  #pragma unroll
          for (int h = 0; h < 2; ++h)
  #pragma unroll
            for (int pl = 0; pl < 3; ++pl) {
              const ib_s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                  (__attribute__((address_space(3))) ib_s16x4*)(img + tb[h][dt & 1] + pl * IBX_PLANE + 512 * (dt >> 1)));
              const u32x2 w2 = __builtin_bit_cast(u32x2, v);
              a[pl][2 * h] = w2[0];
              a[pl][2 * h + 1] = w2[1];
            }
        }
      };
      // IB_COL_PREFETCH_A: d-tile dt + 1's operand is read before d-tile dt's MFMAs (12 VGPRs), so
      // its LDS latency hides behind them instead of heading every d-tile
      constexpr bool PFA = IB_COL_PREFETCH_A != 0;
      u32x4 a_pf[2][3];
      if constexpr (PFA) read_a(0, a_pf[0]);
#if IB_COL_CHAIN && IB_COL_COPY_FIRST
      if constexpr (FRESH) {
        // Per d-tile: ib 0's product chain into T0; the add of the previous d-tile's ib 1 tile (its
        // chain ended six MFMAs earlier, so the add waits on no MFMA result); ib 1's chain into T1
        // with one slice of the next step's P beside it; then T0's add (likewise six MFMAs after its
        // chain). Each chain keeps mfma16_split_n's product order: bitwise the interleaved form,
        // without its two result waits (s_nop 7) per d-tile.
        constexpr int ia[9] = {2, 2, 1, 1, 2, 0, 1, 0, 0}, ibp[9] = {2, 1, 2, 1, 0, 2, 0, 1, 0};
        f32x4 T0, T1;
  #pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          u32x4 a[3];
          const f32x2 lz = read_lz(t + 1, dt & 3);  // (ahead of the operand reads: its wait is not theirs)
          if constexpr (PFA) {
            if (dt + 1 < NDT) read_a(dt + 1, a_pf[(dt + 1) & 1]);
  #pragma unroll
            for (int pl = 0; pl < 3; ++pl) a[pl] = a_pf[dt & 1][pl];
          } else {
            read_a(dt, a);
          }
          T0 = f32x4{0.f, 0.f, 0.f, 0.f};
  #pragma unroll
          for (int k = 9 - NP; k < 9; ++k) T0 = mfma16_bf16(a[ia[k]], pb_t[0][ibp[k]], T0);
          __builtin_amdgcn_sched_barrier(0);
#if IB_COL_PROBE == 3
          if (dt == NDT - 1) Ot[0][1] += T1;
#else
          if (dt > 0) Ot[dt - 1][1] += T1;
#endif
          __builtin_amdgcn_sched_barrier(0);
          T1 = f32x4{0.f, 0.f, 0.f, 0.f};
  #pragma unroll
          for (int k = 9 - NP; k < 9; ++k) T1 = mfma16_bf16(a[ia[k]], pb_t[1][ibp[k]], T1);
#if IB_COL_PROBE == 2  // (timing probe 2, wrong results: P formed in the first step only, reused after)
          if (t == 0) make_p_part(t + 1, sb_t1, pb_t1, partial, dt >> 2, dt & 3, lz);
#else
          make_p_part(t + 1, sb_t1, pb_t1, partial, dt >> 2, dt & 3, lz);
#endif
          __builtin_amdgcn_sched_barrier(0);
#if IB_COL_PROBE == 3  // (timing probe 3, wrong results: the tile adds folded into one)
          if (dt == NDT - 1) Ot[0][0] += T0;
#else
          Ot[dt][0] += T0;
#endif
          __builtin_amdgcn_sched_barrier(0);
        }
        Ot[NDT - 1][1] += T1;
        store_lse(t + 2);  // (hipcc waits for the lse load: the copy, issued before it, has landed too)
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // the copy and the lse; the 4 score loads of t + 2 may fly
        __syncthreads();
        return;
      }
#endif
  #pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        u32x4 a[3];
        if constexpr (PFA) {
          if (dt + 1 < NDT) read_a(dt + 1, a_pf[(dt + 1) & 1]);
  #pragma unroll
          for (int pl = 0; pl < 3; ++pl) a[pl] = a_pf[dt & 1][pl];
        } else {
          read_a(dt, a);
        }
        // the tile's products into a fresh accumulator, then one fp32 add into O' (the row pass's
        // reason: no accumulation bias common to the outputs)
        const u32x4* const aa[2] = {a, a};
        const u32x4* const bb[2] = {pb_t[0], pb_t[1]};
        f32x4 tile_o[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
        f32x4* const cc[2] = {FRESH ? &tile_o[0] : &Ot[dt][0], FRESH ? &tile_o[1] : &Ot[dt][1]};
        mfma16_split_n<NP, 2>(aa, bb, cc);
        if constexpr (FRESH) {
          Ot[dt][0] += tile_o[0];
          Ot[dt][1] += tile_o[1];
          __builtin_amdgcn_sched_barrier(0);
        }
#if IB_COL_COPY_FIRST
        if (dt == IB_COL_MAKE_P_DT) make_p(t + 1, sb_t1, pb_t1, partial);  // next step's P beside this step's MFMAs
      }
      store_lse(t + 2);  // (hipcc waits for the lse load: the copy, issued before it, has landed too)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // the copy and the lse; the 4 score loads of t + 2 may fly
#else
        if (dt == 1) {
          make_p(t + 1, sb_t1, pb_t1, partial);  // next step's P beside this step's MFMAs
          // the next U tile into buffer buf ^ 1 (last read in step t - 1, before its barrier),
          // issued after make_p's wait for the scores of t + 1 so that hipcc's counted wait there
          // (which does not see these inline-asm copies) is not stretched over them
          copy_tile(t + 1, buf ^ 1);
        }
      }
      store_lse(t + 2);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tile copies (and the scores of t + 2)
#endif
      __syncthreads();
    };
    // branch-free pairs (a guard inside a step lets the compiler sink the next step's P
    // computation past the barrier, back to the head of the step that uses it)
    auto run = [&](auto partial) __attribute__((always_inline)) {
      int t = 0;
      for (; t + 1 < ntiles; t += 2) {
        step(t, 0, sbA, sbB, pbA, pbB, partial);
        step(t + 1, 1, sbB, sbA, pbB, pbA, partial);
      }
      if (t < ntiles) step(t, 0, sbA, sbB, pbA, pbB, partial);
    };
    if ((ke - kb) % 32 == 0) run(std::false_type{});
    else run(std::true_type{});

  #pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      const int64_t q = q0 + 16 * ib + i16;
      if (q < B) {
        float* po = p.part_o + (split * B + q) * D + 4 * g;
  #pragma unroll
        for (int dt = 0; dt < NDT; ++dt) *reinterpret_cast<f32x4*>(po + 16 * dt) = Ot[dt][ib];
      }
    }
  }  // segments
}

static int64_t inbatch_nsplit(int64_t B) {
  const int64_t qblocks = ceil_div(B, IB_QB);
  const int64_t ktiles = ceil_div(B, IB_KT);
  // RS_IB_SPLIT_TARGET (timing switch; the split count changes the merge order of the partials):
  // the (owned block x key range) count the split aims at, default 512
  static const int64_t target = [] {
    const char* e = exp_env("RS_IB_SPLIT_TARGET");
    return e && atoi(e) > 0 ? (int64_t)atoi(e) : (int64_t)512;
  }();
  int64_t s = ceil_div(target, qblocks);
  if (s > ktiles) s = ktiles;
  if (s < 1) s = 1;
  return s;
}

struct InbatchWs {
  float *pm, *pl, *po;
  double* lossp;
  unsigned int* done;  // the row finalize's ticket (zeroed by the sequence's first image pass)
  int64_t nsplit, kps;
  char *img_q, *img_k;  // split plane images (D = 128)
};

static size_t inbatch_ws(int64_t B, int64_t D, void* base, size_t bytes, InbatchWs* w) {
  const int64_t ns = inbatch_nsplit(B);
  Carve c(base, bytes);
  InbatchWs r;
  r.pm = c.take<float>(ns * B);
  r.pl = c.take<float>(ns * B);
  r.po = c.take<float>(ns * B * D);
  r.lossp = c.take<double>(ceil_div(B, 4) + 1);
  r.done = c.take<unsigned int>(TICKET_WORDS);
  r.img_q = r.img_k = nullptr;
  if (D == IBX_D) {
    r.img_q = c.take<char>((size_t)ib_ntiles(B) * IBX_BUF);
    r.img_k = c.take<char>((size_t)ib_ntiles(B) * IBX_BUF);
  }
  r.nsplit = ns;
  r.kps = ceil_div(ceil_div(B, ns), IB_KT) * IB_KT;
  if (w) *w = r;
  return c.off + 256;
}

// reuse (mode 3): the workspace is the storing forward's, whose image of U (its Q) is the col
// pass's streamed operand: no split launch
template <int D>
static int run_pass(int mode, const float* Q, const float* K, int64_t B, const float* lse_k,
                    const InbatchWs& w, hipStream_t st, float* S = nullptr, int prec = 0, bool reuse = false) {
  InbatchParams p{Q, K, B, w.kps, lse_k, w.pm, w.pl, w.po, S};
  p.Bs = B;
  const int64_t Seff = ceil_div(B, w.kps);
  dim3 grid((unsigned)ceil_div(B, IB_QB), (unsigned)Seff);
  if constexpr (D == IBX_D) {
    // split-operand kernels for the stored pair (row pass with P.K, stored col pass)
    if ((prec == 6 || prec == 9) && (mode == 1 || mode == 3)) {
      const int64_t NT = ib_ntiles(B);
      const dim3 sgrid((unsigned)ceil_div(NT * 32 * 32, 256));
      if (mode == 1) {  // both operands' images in one launch (and the row finalize's ticket zeroed)
        hipLaunchKernelGGL(ibx_split_image2_kernel, dim3(2 * sgrid.x), dim3(256), 0, st,
                           IbxImg{K, B, NT, w.img_k, nullptr, nullptr}, IbxImg{Q, B, NT, w.img_q, nullptr, nullptr},
                           (int64_t)sgrid.x, w.done);
      } else if (!reuse) {
        hipLaunchKernelGGL(ibx_split_image_kernel, sgrid, dim3(256), 0, st, K, B, NT, w.img_k);
      }
      constexpr int NW = IBX_NW;
      const dim3 xgrid((unsigned)ceil_div(B, IB_QW * NW), (unsigned)Seff);
      if (mode == 1) {
        // two 16-user subtiles per wave (UB = 4 at one wave per SIMD halves the LDS reads per MFMA
        // but does not fit 512 registers without spills)
        if (prec == 6)
          hipLaunchKernelGGL((inbatch_row_m16_kernel<6, NW, 2>), xgrid, dim3(64 * NW), 0, st, p, w.img_q, w.img_k);
        else
          hipLaunchKernelGGL((inbatch_row_m16_kernel<9, NW, 2>), xgrid, dim3(64 * NW), 0, st, p, w.img_q, w.img_k);
        return check_launch("inbatch_row_m16");
      }
      const char* kimg = reuse ? w.img_q : w.img_k;
      if (prec == 6)
        hipLaunchKernelGGL((inbatch_col_m16_kernel<6, NW>), xgrid, dim3(64 * NW), 0, st, p, (const float*)S, kimg);
      else
        hipLaunchKernelGGL((inbatch_col_m16_kernel<9, NW>), xgrid, dim3(64 * NW), 0, st, p, (const float*)S, kimg);
      return check_launch("inbatch_col_m16");

    }
  }
  if (mode == 0) hipLaunchKernelGGL((inbatch_pass_kernel<D, 0>), grid, dim3(256), 0, st, p);
  else if (mode == 1) hipLaunchKernelGGL((inbatch_pass_kernel<D, 1>), grid, dim3(256), 0, st, p);
  else if (mode == 2) hipLaunchKernelGGL((inbatch_pass_kernel<D, 2>), grid, dim3(256), 0, st, p);
  else hipLaunchKernelGGL((inbatch_col_stored_kernel<D>), grid, dim3(256), 0, st, p, (const float*)S);
  return check_launch("inbatch_pass");
}

template <int D>
static int fwd_impl(const float* U, const float* C, int64_t B, float weight, float* row_loss,
                    float* lse, float* loss_sum, double* loss_sum64, float* dU,
                    const InbatchWs& w, hipStream_t st, float* S = nullptr, int prec = 0) {
  const int mode = (dU || S) ? 1 : 0;
  int rc = run_pass<D>(mode, U, C, B, nullptr, w, st, S, prec);
  if (rc) return rc;
  const int64_t Seff = ceil_div(B, w.kps);
  RS_REQUIRE(Seff <= 64, "inbatch: %lld key splits exceed the finalize's 64 lanes", (long long)Seff);
  const int64_t nb = ceil_div(B, IB_FIN_ROWS);
  // the split kernels' image pass zeroed the ticket: the finalize's last workgroup forms the total
  const bool ticket = D == IBX_D && (prec == 6 || prec == 9) && mode == 1;
  hipLaunchKernelGGL((inbatch_row_finalize_kernel<D>), dim3((unsigned)nb), dim3(256), 0, st, U, C, B,
                     (int)Seff, w.pm, w.pl, w.po, weight, row_loss, lse, dU, w.lossp, nullptr, 0, 0, 0, 0, nullptr, 0, 0,
                     0, ticket ? w.done : nullptr, loss_sum, loss_sum64);
  rc = check_launch("inbatch_row_finalize");
  if (rc || ticket) return rc;
  return launch_final_sum(w.lossp, nb, 1.0, loss_sum, loss_sum64, st);
}

template <int D>
static int bwd_impl(const float* U, const float* C, int64_t B, float weight, const float* lse,
                    const float* gscale, const float* dU_unit, float* dU_out, float* dC,
                    const InbatchWs& w, hipStream_t st, const float* S = nullptr, int prec = 0, bool reuse = false) {
  // owned = items (C), streamed = users (U) with their lse
  int rc = S ? run_pass<D>(3, C, U, B, lse, w, st, const_cast<float*>(S), prec, reuse)
             : run_pass<D>(2, C, U, B, lse, w, st);
  if (rc) return rc;
  const int64_t Seff = ceil_div(B, w.kps);
  if ((B * D) % 4 == 0 && aligned16(U) && aligned16(w.po) && aligned16(dC) && (!dU_unit || aligned16(dU_unit)) &&
      (!dU_out || aligned16(dU_out))) {
    const int64_t n4 = B * D / 4;
    hipLaunchKernelGGL((inbatch_col_finalize4_kernel<4>), dim3((unsigned)ceil_div(n4, 256)), dim3(256), 0, st,
                       reinterpret_cast<const f32x4*>(U), n4, (int)Seff, reinterpret_cast<const f32x4*>(w.po),
                       weight, gscale, reinterpret_cast<const f32x4*>(dU_unit), reinterpret_cast<f32x4*>(dU_out),
                       reinterpret_cast<f32x4*>(dC));
  } else {
    hipLaunchKernelGGL((inbatch_col_finalize_kernel<D>), dim3((unsigned)ceil_div(B * D, 256)), dim3(256),
                       0, st, U, B, (int)Seff, w.po, weight, gscale, dU_unit, dU_out, dC);
  }
  return check_launch("inbatch_col_finalize");
}

// ---- the deduplicated pair ---------------------------------------------------------------------
// A batch drawn from skewed id distributions repeats rows: a column C_b that occurs n_b times
// contributes n_b exp(S_ib) to every row's sum, and a user row that occurs m_u times contributes
// m_u P_ub U_u to every item's col-pass sum. The pair below runs the two passes over the DISTINCT
// rows only (bitwise-identical rows, found by content, never by id), with the counts as weights:
//   row pass  owned = distinct users, streamed = distinct items weighted n_b
//             -> lse, O per distinct user; each batch row i reads its user's partials (u_inv);
//   col pass  owned = distinct items, streamed = distinct users weighted m_u, lse of their rows
//             -> O' per distinct item; dC_j = w (O'_{c_inv[j]} - U_j).
// Every batch row gets exactly the loss, lse, dU and dC of the full B x B pair (up to the order of
// the fp32 sums); the work is Bu x Bc instead of B x B.

__device__ __forceinline__ uint64_t ib_mix64(uint64_t x) {  // splitmix64 finaliser
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}

// The distinct-row search runs over one matrix or over the user and item matrices together
// (IbSides: side 1 = rows B .. 2B - 1 of the sort, X1): one hash / sort / scan / scatter / count /
// verify sequence for both sides of the pair. The sort key's top bit is the side, so every side-0
// row sorts before every side-1 row and side 1's distinct indices start at side 0's count.
struct IbSides {
  const float* X[2];
  int32_t *rep[2], *inv[2];
  float* count[2];
  int64_t B;   // rows per side
  int nsides;  // 1 or 2
  int32_t* order[2] = {nullptr, nullptr};  // nullable: the side's rows in key order (stable)
  // nullable (id plans): each distinct slot's id, in ascending-id order; the reserved group of
  // out-of-range ids gets nrows (a zero row for the gather), slots past the count -1
  int64_t* did[2] = {nullptr, nullptr};
  const int64_t* ids[2] = {nullptr, nullptr};
  int64_t nrows[2] = {0, 0};
  int32_t* start[2] = {nullptr, nullptr};  // nullable: each slot's first position in the side's key order
  // nullable (with did): vinfo[s] = side s's distinct count without the group of out-of-range ids
  // (the count a deduplication of the side's ids keeps)
  int64_t* vinfo = nullptr;
};

// 63-bit content hash of each row (D % 4 == 0) + the side bit: sum of mix(position, bits) over the
// row, 32 lanes per row, 8 rows per workgroup; vals = the row's index in the sort (side B + row)
__global__ __launch_bounds__(256) void ib_row_hash_kernel(IbSides sd, int D, uint64_t* __restrict__ keys,
                                                          int32_t* __restrict__ vals) {
  const int64_t r = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
  const int c = threadIdx.x & 31;
  const int64_t n = sd.B * sd.nsides;
  const int side = r >= sd.B ? 1 : 0;
  const int64_t row = r - side * sd.B;
  const float* X = sd.X[side];
  uint64_t h = 0;
  if (r < n) {
    for (int c4 = c; c4 < D / 4; c4 += 32) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(X + row * D + 4 * c4);
#pragma unroll
      for (int t = 0; t < 4; ++t) h += ib_mix64(((uint64_t)(4 * c4 + t + 1) << 32) | v[t]);
    }
  }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)h, o, 32);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(h >> 32), o, 32);
    h += ((uint64_t)hi << 32) | lo;
  }
  if (r < n && c == 0) {
    keys[r] = (ib_mix64(h) >> 1) | ((uint64_t)side << 63);
    vals[r] = (int32_t)r;
  }
}

// flag i of the sorted keys: key i starts a run (the scan input of plan_heads_scan, and the scatter's test)
__host__ __device__ inline bool ib_is_head(const uint64_t* ks, int64_t i) { return i == 0 || ks[i] != ks[i - 1]; }

// distinct index u = (inclusive run-head count) - 1 in key order (side 1's less side 0's count);
// its representative is the first row of the run (the smallest row index: the sort is stable on
// row-ordered input). info[2 side] = the side's distinct count.
__global__ __launch_bounds__(256) void ib_unique_scatter_kernel(IbSides sd, const uint64_t* __restrict__ keys_s,
                                                                const int32_t* __restrict__ incl,
                                                                const int32_t* __restrict__ vals_s,
                                                                int32_t* __restrict__ pos, int64_t* __restrict__ info) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n = sd.B * sd.nsides;
  if (i >= n) return;
  const int32_t nu0 = sd.nsides == 2 ? incl[sd.B - 1] : 0;
  const int32_t r = vals_s[i];
  const int side = r >= sd.B ? 1 : 0;
  const int32_t u = incl[i] - 1 - (side ? nu0 : 0), row = r - (side ? (int32_t)sd.B : 0);
  sd.inv[side][row] = u;
  if (sd.order[side]) sd.order[side][i - side * sd.B] = row;  // side 1's keys sort after all of side 0's
  if (ib_is_head(keys_s, i)) {
    sd.rep[side][u] = row;
    pos[incl[i] - 1] = (int32_t)i;
    if (sd.did[side]) {
      const int64_t id = sd.ids[side][row];
      sd.did[side][u] = (id < 0 || id >= sd.nrows[side]) ? sd.nrows[side] : id;
    }
    if (sd.start[side]) sd.start[side][u] = (int32_t)(i - side * sd.B);
  }
  if (i == n - 1) {
    if (sd.nsides == 2) {
      info[0] = nu0;
      info[2] = incl[i] - nu0;
    } else {
      info[0] = incl[i];
    }
  }
}

__global__ __launch_bounds__(256) void ib_unique_count_kernel(IbSides sd, const int32_t* __restrict__ pos,
                                                              const int32_t* __restrict__ incl) {
  const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n = sd.B * sd.nsides;
  const int64_t nu = incl[n - 1];
  if (u == 0 && sd.vinfo) {  // (did was written by the scatter pass, the launch before)
    const int64_t n0 = sd.nsides == 2 ? incl[sd.B - 1] : nu;
    for (int k = 0; k < sd.nsides; ++k) {
      const int64_t nk = k ? nu - n0 : n0;
      sd.vinfo[k] = nk - (nk > 0 && sd.did[k][nk - 1] >= sd.nrows[k] ? 1 : 0);
    }
  }
  if (u >= nu) return;
  const int64_t nu0 = sd.nsides == 2 ? incl[sd.B - 1] : nu;
  const int side = u >= nu0 ? 1 : 0;
  sd.count[side][u - side * nu0] = (float)((u + 1 < nu ? (int64_t)pos[u + 1] : n) - pos[u]);
}

// rows whose bits differ from their representative's (a hash collision) -> info[2 side + 1]
__global__ __launch_bounds__(256) void ib_unique_verify_kernel(IbSides sd, int D,
                                                               unsigned long long* __restrict__ info) {
  const int64_t r = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
  const int c = threadIdx.x & 31;
  if (r >= sd.B * sd.nsides) return;
  const int side = r >= sd.B ? 1 : 0;
  const int64_t row = r - side * sd.B;
  const float* X = sd.X[side];
  const int64_t r0 = sd.rep[side][sd.inv[side][row]];
  if (r0 == row) return;
  bool diff = false;
  for (int c4 = c; c4 < D / 4; c4 += 32) {
    const u32x4 a = *reinterpret_cast<const u32x4*>(X + row * D + 4 * c4);
    const u32x4 b = *reinterpret_cast<const u32x4*>(X + r0 * D + 4 * c4);
    diff |= a[0] != b[0] || a[1] != b[1] || a[2] != b[2] || a[3] != b[3];
  }
  if (diff) atomicAdd(info + 2 * side + 1, 1ULL);
}

// id keys for the pair's distinct-row search when the rows are a function of an integer id (the
// reference's towers: Embedding -> Dense stack of the id alone, src/models.py:85-90): equal ids
// give bitwise-equal rows, so rows are grouped by id without hashing or verifying content. The
// side bit sits above `bits` id bits; ids outside [0, rows) share the reserved key 2^bits - 1
// (the gather writes them as zero rows, rs_embedding_gather_tables_f32).
__global__ __launch_bounds__(256) void ib_id_key_kernel(const int64_t* __restrict__ u_ids,
                                                        const int64_t* __restrict__ c_ids, int64_t B,
                                                        int64_t u_rows, int64_t c_rows, int bits,
                                                        uint64_t* __restrict__ keys, int32_t* __restrict__ vals,
                                                        float* __restrict__ u_count, float* __restrict__ c_count,
                                                        int64_t* __restrict__ info, int64_t* __restrict__ u_did,
                                                        int64_t* __restrict__ c_did) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  // the plan's accumulators zeroed here (no memset launches): both sides' counts, padded to whole
  // 32-row tiles (the grid covers 2 * 32 * ceil(B / 32) >= 2 B threads), and the four counts
  const int64_t nc = ib_ntiles(B) * 32;
  if (r < 2 * nc) (r < nc ? u_count : c_count)[r < nc ? r : r - nc] = 0.f;
  if (r < 4) info[r] = 0;
  if (r >= 2 * B) return;
  const int side = r >= B ? 1 : 0;
  const int64_t row = r - side * B;
  int64_t* const did = side ? c_did : u_did;
  if (did) did[row] = -1;  // every slot past the distinct count (the scatter writes the rest)
  const int64_t id = side ? c_ids[row] : u_ids[row];
  const int64_t nrows = side ? c_rows : u_rows;
  const uint64_t k = (id < 0 || id >= nrows) ? ((1ull << bits) - 1) : (uint64_t)id;
  keys[r] = k | ((uint64_t)side << bits);
  vals[r] = (int32_t)r;
}

// ---- the id plan's key sort (round 6): a bucket sort ---------------------------------------------
// The id keys are at most 26 bits (side bit above the id bits) with the batch position as the value,
// so their stable order is the order of (key, position). rocprim's merge path took 9 launches
// (~60 us per C3 step, 131,072 keys); this takes four:
//   ps_hist:    per 2048-key block, the counts of the keys' top PS_BB bits (LDS atomics);
//   ps_scatter: each block forms every bucket's start and its own offset in each bucket from all the
//               blocks' counts (block order inside a bucket), ranks its keys by bucket in LDS (block
//               radix sort of (bucket, local index): unique keys, so position order inside a bucket),
//               and writes them to their buckets: every bucket holds its keys in position order;
//   ps_small:   one workgroup per bucket of at most 256 keys sorts it by the remaining key bits with
//               the position as the tie-break (a rank count in LDS);
//   ps_big:     a bucket of more keys (a hot id is one key) takes stable LSD passes over 4-bit digits
//               of the remaining bits in one workgroup, in LDS up to 8192 keys of <= 16 bits, else in
//               global memory.
// The result is the stable sort: the order rocprim's radix sort produces (the plan tests check it
// against numpy's unique / stable argsort, incl. one-bucket batches).
constexpr int PS_BB = 10, PS_NB = 1 << PS_BB, PS_IPT = 8, PS_EPB = 256 * PS_IPT, PS_SMALL = 256, PS_LDSN = 8192;
constexpr int64_t PS_MAXN = (int64_t)1 << 21;  // (larger plans: rocprim's sort; every scatter block reads all counts)
// Measured (profiles/r06ac_ids_sort_trace.txt, C3 graph step): hist 5.0 + scatter 33.4 + small 9.9 + big
// 59.2 = 107.5 us against rocprim's merge path at ~62 us — every scatter block reads all the blocks'
// counts (256 KB) and the Zipf-hot buckets' LSD passes serialise on the 16-thread digit prefix. Correct
// (the plan tests, numpy-checked, incl. one-bucket batches, pass on it) and slower: off.
#ifndef IB_IDS_SORT
#define IB_IDS_SORT 0  // the id plan's bucket sort (0: rocprim's merge path for every size)
#endif

__global__ __launch_bounds__(256) void ps_hist_kernel(const uint64_t* __restrict__ keys, int64_t n, int shift,
                                                      int32_t* __restrict__ hist) {
  __shared__ int h[PS_NB];
  const int tid = threadIdx.x;
  for (int b = tid; b < PS_NB; b += 256) h[b] = 0;
  __syncthreads();
  const int64_t e0 = (int64_t)blockIdx.x * PS_EPB;
#pragma unroll
  for (int j = 0; j < PS_IPT; ++j) {
    const int64_t e = e0 + j * 256 + tid;
    if (e < n) atomicAdd(&h[(int)(keys[e] >> shift)], 1);
  }
  __syncthreads();
  for (int b = tid; b < PS_NB; b += 256) hist[(int64_t)blockIdx.x * PS_NB + b] = h[b];
}

__global__ __launch_bounds__(256) void ps_scatter_kernel(const uint64_t* __restrict__ keys,
                                                         const int32_t* __restrict__ vals, int64_t n, int shift,
                                                         const int32_t* __restrict__ hist, int32_t* __restrict__ bstart,
                                                         uint64_t* __restrict__ tk, int32_t* __restrict__ tv) {
  using BRS = rocprim::block_radix_sort<uint32_t, 256, PS_IPT>;
  __shared__ typename BRS::storage_type st;
  __shared__ uint16_t sb[PS_EPB];
  __shared__ int first[PS_NB];
  __shared__ int off[PS_NB];
  __shared__ int part[256];
  const int tid = threadIdx.x;
  const int G = (int)gridDim.x, me = (int)blockIdx.x;
  // bucket totals and this block's offset inside each bucket (thread t: buckets 4 t .. 4 t + 3)
  int tot[4] = {0, 0, 0, 0}, bef[4] = {0, 0, 0, 0};
  for (int g2 = 0; g2 < G; ++g2) {
    const int4 v = *reinterpret_cast<const int4*>(hist + (int64_t)g2 * PS_NB + 4 * tid);
    tot[0] += v.x; tot[1] += v.y; tot[2] += v.z; tot[3] += v.w;
    if (g2 < me) { bef[0] += v.x; bef[1] += v.y; bef[2] += v.z; bef[3] += v.w; }
  }
  const int mine = tot[0] + tot[1] + tot[2] + tot[3];
  part[tid] = mine;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {  // inclusive scan of the 256 partials
    const int v = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  int run = part[tid] - mine;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    off[4 * tid + q] = run + bef[q];
    if (me == 0) bstart[4 * tid + q] = run;
    run += tot[q];
  }
  if (me == 0 && tid == 255) bstart[PS_NB] = run;
  const int64_t e0 = (int64_t)me * PS_EPB;
  uint32_t k[PS_IPT];
#pragma unroll
  for (int j = 0; j < PS_IPT; ++j) {  // (bucket, local index): unique; past n the bucket PS_NB (last)
    const int li = tid * PS_IPT + j;
    const int64_t e = e0 + li;
    const uint32_t bk = e < n ? (uint32_t)(keys[e] >> shift) : (uint32_t)PS_NB;
    k[j] = (bk << 11) | (uint32_t)li;
  }
  BRS().sort(k, st, 0, PS_BB + 1 + 11);
#pragma unroll
  for (int j = 0; j < PS_IPT; ++j) sb[tid * PS_IPT + j] = (uint16_t)(k[j] >> 11);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PS_IPT; ++j) {
    const int p = tid * PS_IPT + j;
    const int bk = sb[p];
    if (bk < PS_NB && (p == 0 || sb[p - 1] != bk)) first[bk] = p;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PS_IPT; ++j) {
    const int p = tid * PS_IPT + j;
    const int bk = (int)(k[j] >> 11);
    if (bk >= PS_NB) continue;
    const int64_t e = e0 + (int64_t)(k[j] & 2047u);
    const int64_t pos = (int64_t)off[bk] + (p - first[bk]);
    tk[pos] = keys[e];
    tv[pos] = vals[e];
  }
}

// a bucket of at most PS_SMALL keys: rank = keys below + equal keys earlier in the bucket
__global__ __launch_bounds__(256) void ps_small_kernel(int shift, const int32_t* __restrict__ bstart,
                                                       const uint64_t* __restrict__ tk, const int32_t* __restrict__ tv,
                                                       uint64_t* __restrict__ keys_s, int32_t* __restrict__ vals_s) {
  __shared__ uint64_t kl[PS_SMALL];
  const int tid = threadIdx.x;
  const int64_t lo = bstart[blockIdx.x];
  const int m = bstart[blockIdx.x + 1] - bstart[blockIdx.x];
  if (m <= 0 || m > PS_SMALL) return;
  const uint64_t lowmask = shift > 0 ? ((1ull << shift) - 1) : 0ull;
  uint64_t key = 0, mykl = 0;
  int32_t val = 0;
  if (tid < m) {
    key = tk[lo + tid];
    val = tv[lo + tid];
    mykl = key & lowmask;
    kl[tid] = mykl;
  }
  __syncthreads();
  if (tid < m) {
    int r = 0;
    for (int j = 0; j < m; ++j) {
      const uint64_t o = kl[j];
      r += (o < mykl || (o == mykl && j < tid)) ? 1 : 0;
    }
    keys_s[lo + r] = key;
    vals_s[lo + r] = val;
  }
}

// a bucket of more than PS_SMALL keys: stable LSD passes over 4-bit digits of the low bits, one
// workgroup; thread t owns a contiguous chunk and places its keys after the earlier threads' keys of
// the same digit. In LDS (16-bit low keys and 16-bit bucket positions) when it fits, else in global
// memory ping-ponging between (tk, tv) and (keys_s, vals_s)
__global__ __launch_bounds__(256) void ps_big_kernel(int shift, const int32_t* __restrict__ bstart, uint64_t* tk,
                                                     int32_t* tv, uint64_t* __restrict__ keys_s,
                                                     int32_t* __restrict__ vals_s) {
  __shared__ int cnt[256][17];  // (17: the per-thread rows fall on different banks)
  __shared__ int dbase[16];
  __shared__ uint16_t lk[2][PS_LDSN], li[2][PS_LDSN];
  const int tid = threadIdx.x;
  const int64_t lo = bstart[blockIdx.x];
  const int64_t m = bstart[blockIdx.x + 1] - lo;
  if (m <= PS_SMALL) return;
  const int64_t chunk = (m + 255) / 256;
  const int64_t c0 = tid * chunk < m ? tid * chunk : m, c1 = (tid + 1) * chunk < m ? (tid + 1) * chunk : m;
  const int passes = (shift + 3) / 4;
  // one stable counting pass: digit of element i = dig(i); place(i, slot) writes it
  auto pass = [&](auto dig, auto place) __attribute__((always_inline)) {
    for (int d = 0; d < 16; ++d) cnt[tid][d] = 0;
    for (int64_t i = c0; i < c1; ++i) ++cnt[tid][dig(i)];
    __syncthreads();
    if (tid < 16) {  // digit tid: exclusive prefix over the threads, then its total
      int a = 0;
      for (int t = 0; t < 256; ++t) {
        const int c = cnt[t][tid];
        cnt[t][tid] = a;
        a += c;
      }
      dbase[tid] = a;
    }
    __syncthreads();
    if (tid == 0) {
      int a = 0;
      for (int d = 0; d < 16; ++d) {
        const int c = dbase[d];
        dbase[d] = a;
        a += c;
      }
    }
    __syncthreads();
    for (int d = 0; d < 16; ++d) cnt[tid][d] += dbase[d];
    for (int64_t i = c0; i < c1; ++i) place(i, cnt[tid][dig(i)]++);
    __syncthreads();
  };
  if (m <= PS_LDSN && shift <= 16) {
    const uint64_t lowmask = shift > 0 ? ((1ull << shift) - 1) : 0ull;
    for (int64_t i = tid; i < m; i += 256) {
      lk[0][i] = (uint16_t)(tk[lo + i] & lowmask);
      li[0][i] = (uint16_t)i;
    }
    __syncthreads();
    int cur = 0;
    for (int ps = 0; ps < passes; ++ps) {
      const int sh = 4 * ps;
      const int c = cur;
      pass([&](int64_t i) { return (int)((lk[c][i] >> sh) & 15); },
           [&](int64_t i, int o) {
             lk[c ^ 1][o] = lk[c][i];
             li[c ^ 1][o] = li[c][i];
           });
      cur ^= 1;
    }
    for (int64_t i = tid; i < m; i += 256) {
      const int64_t src = lo + li[cur][i];
      keys_s[lo + i] = tk[src];
      vals_s[lo + i] = tv[src];
    }
    return;
  }
  uint64_t *sk = tk + lo, *dk = keys_s + lo;
  int32_t *sv = tv + lo, *dv = vals_s + lo;
  for (int ps = 0; ps < passes; ++ps) {
    const int sh = 4 * ps;
    pass([&](int64_t i) { return (int)((sk[i] >> sh) & 15); },
         [&](int64_t i, int o) {
           dk[o] = sk[i];
           dv[o] = sv[i];
         });
    uint64_t* k2 = sk;
    sk = dk;
    dk = k2;
    int32_t* v2 = sv;
    sv = dv;
    dv = v2;
  }
  if (sk != keys_s + lo) {  // an even pass count (or none) left the result in (tk, tv)
    for (int64_t i = tid; i < m; i += 256) {
      keys_s[lo + i] = sk[i];
      vals_s[lo + i] = sv[i];
    }
  }
}

struct UniqueWs {
  uint64_t *keys, *keys_s;
  int32_t *vals, *vals_s, *incl, *pos;
  char *sort_temp, *scan_temp;
  size_t sort_bytes, scan_bytes;
  // the id keys' bucket sort (ids_sort): per-block bucket counts, bucket starts, the bucket-ordered
  // keys / values
  int32_t *ps_hist, *ps_bstart, *ps_tv;
  uint64_t* ps_tk;
};

// The plans' key sort (content hashes: 64 bits; id keys: the side bit above the id bits). The
// temp-size query (temp == nullptr) and the sort itself go through this one function with the same
// config, bit range and stream, so the carve always holds what the sort writes. rocprim's default
// path (merge sort below 2^20 keys: 7 launches, ~47 us per C3 step), NOT onesweep: with query and
// call unified here, onesweep (MergeSortLimit 0) still faulted a profiled hipGraph replay of the C3
// step (round 6, profiles/r06_idplan_sort_onesweep_cause.txt), so the round-5 fault was not a
// temp-size mismatch. Onesweep is the only path that adds hipMemsetAsync nodes to the captured
// graph (its look-back states and, on gfx950, its atomic block-id counter); a reset that does not
// land before its kernel leaves block ids past the grid and stale look-back prefixes, which index
// past the key arrays. The merge path resets nothing by memset and runs clean under the profiler.
#ifndef RS_PLAN_SORT_MERGE_LIMIT   // (an A/B variant build may set another limit; 0 = onesweep)
#define RS_PLAN_SORT_MERGE_LIMIT (1 << 20)
#endif
// The merge path's block sort size (RS_PLAN_SORT_BS threads x RS_PLAN_SORT_IPT items; IPT 0 = rocprim's
// default, 1,024 items per block): each doubling of the sorted block removes one odd-even merge
// launch of the 131,072-key C3 plan. 8,192 items: rocprim launches 13.6 -> 7.9 per C3 step, their time
// 86.6 -> 82.4 us in one A/B (4,096: 89.0 -> 88.0; profiles/r06y_plan_sort_block_ab.txt), but the
// kernel trace puts the 8,192-item block sort at 33.8 us against the default's 9.5 (r06ab_plan_sequence.txt):
// the larger block sort takes back what the merges save — neutral within the boxes' noise. Same stable
// order: the plan is bitwise unchanged.
#ifndef RS_PLAN_SORT_IPT
#define RS_PLAN_SORT_IPT 16
#endif
#ifndef RS_PLAN_SORT_BS
#define RS_PLAN_SORT_BS 512
#endif
using PlanMergeConfig = std::conditional_t<RS_PLAN_SORT_IPT == 0, rocprim::default_config,
                                           rocprim::merge_sort_config<512, RS_PLAN_SORT_BS,
                                                                      (RS_PLAN_SORT_IPT > 0 ? RS_PLAN_SORT_IPT : 1)>>;
using PlanSortConfig = rocprim::radix_sort_config<rocprim::default_config, PlanMergeConfig,
                                                  rocprim::default_config, RS_PLAN_SORT_MERGE_LIMIT>;
static hipError_t plan_sort(void* temp, size_t& bytes, const uint64_t* kin, uint64_t* kout, const int32_t* vin,
                            int32_t* vout, int64_t n, int end_bit, hipStream_t st) {
  return rocprim::radix_sort_pairs<PlanSortConfig>(temp, bytes, kin, kout, vin, vout, (unsigned)n, 0u,
                                                   (unsigned)end_bit, st);
}

// Run heads of the sorted keys as the scan's input (flag i = key i starts a run): computed where the
// scan loads them, so no flag array is written and read and no launch computes it (round 6: one
// launch and 0.5 MB fewer per C3 step). The temp-size query and the scan go through this one function
// with the same iterator type. The scatter pass recomputes the flag from the keys the same way.
struct IbRunHead {
  const uint64_t* ks;
  __host__ __device__ int32_t operator()(int64_t i) const { return ib_is_head(ks, i) ? 1 : 0; }
};
static hipError_t plan_heads_scan(void* temp, size_t& bytes, const uint64_t* ks, int32_t* incl, size_t n,
                                  hipStream_t st) {
  auto heads = rocprim::make_transform_iterator(rocprim::counting_iterator<int64_t>(0), IbRunHead{ks});
  return rocprim::inclusive_scan(temp, bytes, heads, incl, n, rocprim::plus<int32_t>(), st);
}

// end_bit / st: those of the sort the carve is for (the host-only size query passes 64 and the
// null stream: onesweep's temp grows with the bit range, so 64 bounds every call's)
static int unique_ws(int64_t B, int end_bit, hipStream_t st, void* base, size_t bytes, UniqueWs* w, size_t* need) {
  const size_t n = (size_t)(B > 0 ? B : 1);
  UniqueWs r{};
  if (plan_sort(nullptr, r.sort_bytes, nullptr, nullptr, nullptr, nullptr, (int64_t)n, end_bit, st) != hipSuccess)
    return RS_ERR_HIP;
  if (plan_heads_scan(nullptr, r.scan_bytes, nullptr, nullptr, n, (hipStream_t)0) != hipSuccess) return RS_ERR_HIP;
  Carve c(base, bytes);
  r.keys = c.take<uint64_t>(n);
  r.keys_s = c.take<uint64_t>(n);
  r.vals = c.take<int32_t>(n);
  r.vals_s = c.take<int32_t>(n);
  r.incl = c.take<int32_t>(n);
  r.pos = c.take<int32_t>(n);
  r.sort_temp = c.take<char>(r.sort_bytes);
  r.scan_temp = c.take<char>(r.scan_bytes);
  if (IB_IDS_SORT) {
    const int64_t G = ceil_div((int64_t)n, PS_EPB);
    r.ps_hist = c.take<int32_t>(G * PS_NB);
    r.ps_bstart = c.take<int32_t>(PS_NB + 1);
    r.ps_tv = c.take<int32_t>(n);
    r.ps_tk = c.take<uint64_t>(n);
  }
  if (w) *w = r;
  *need = c.off + 256;
  return RS_OK;
}

// the id keys' bucket sort: four launches
static int ids_sort(const UniqueWs& w, int64_t n, int kbits, hipStream_t st) {
  const int shift = kbits > PS_BB ? kbits - PS_BB : 0;
  const unsigned G = (unsigned)ceil_div(n, PS_EPB);
  hipLaunchKernelGGL(ps_hist_kernel, dim3(G), dim3(256), 0, st, w.keys, n, shift, w.ps_hist);
  int rc = check_launch("ps_hist");
  if (rc) return rc;
  hipLaunchKernelGGL(ps_scatter_kernel, dim3(G), dim3(256), 0, st, w.keys, w.vals, n, shift, w.ps_hist, w.ps_bstart,
                     w.ps_tk, w.ps_tv);
  rc = check_launch("ps_scatter");
  if (rc) return rc;
  hipLaunchKernelGGL(ps_small_kernel, dim3(PS_NB), dim3(256), 0, st, shift, w.ps_bstart, w.ps_tk, w.ps_tv, w.keys_s,
                     w.vals_s);
  rc = check_launch("ps_small");
  if (rc) return rc;
  hipLaunchKernelGGL(ps_big_kernel, dim3(PS_NB), dim3(256), 0, st, shift, w.ps_bstart, w.ps_tk, w.ps_tv, w.keys_s,
                     w.vals_s);
  return check_launch("ps_big");
}


struct DedupWs {
  float *pm, *pl, *po;
  double* lossp;
  unsigned int* done;  // the row finalize's ticket (zeroed by the user image pass)
  char *img_q, *img_k;
  char* img_t;   // the col pass's transposed user image (IB_COL_TIMG)
  int64_t prow;  // partial rows available (ns x owned rows <= prow)
  float* lz;     // the col pass's per-user exponent bias (ib_lz_kernel)
};

static size_t dedup_ws(int64_t B, void* base, size_t bytes, DedupWs* w) {
  Carve c(base, bytes);
  DedupWs r;
  // >= (W / blocks + 2 R) x owned rows of any stream-K plan (W <= 256, blocks of 256 rows, R ranges)
  r.prow = (2 * IB_SK_RANGES + 1) * B + 65536;
  r.pm = c.take<float>(r.prow);
  r.pl = c.take<float>(r.prow);
  r.po = c.take<float>(r.prow * IBX_D);
  r.lossp = c.take<double>(ceil_div(B, 4) + 1);
  r.lz = c.take<float>(B);
  r.done = c.take<unsigned int>(TICKET_WORDS);
  r.img_q = c.take<char>((size_t)ib_ntiles(B) * IBX_BUF);
  r.img_k = c.take<char>((size_t)ib_ntiles(B) * IBX_BUF);
  r.img_t = IB_COL_TIMG ? c.take<char>((size_t)ib_ntiles(B) * IBX_BUF) : nullptr;
  if (w) *w = r;
  return c.off + 256;
}

// Stream-K plan for Bo owned rows (256 per workgroup) against Bs streamed rows: the
// ceil(Bo / 256) x ceil(Bs / 32) (block, key tile) units in W equal shares, one workgroup per CU
// (W = 256), so a rectangular problem of any shape keeps every CU busy to the end. maxslots = the
// most partial slots of a block (<= 64 for the finalize's lanes).
struct SkPlan {
  int64_t W, ntk, T;
  int maxslots;
};
constexpr int64_t IB_SK_GRID = 256 * (8 / IBX_NW);  // stream-K workgroups: 8 waves per CU
static SkPlan dedup_plan(int64_t Bo, int64_t Bs) {
  SkPlan k;
  const int64_t xg = ceil_div(Bo, IB_SKB);
  k.ntk = ib_ntiles(Bs);
  k.T = xg * k.ntk;
  k.W = ib_sk_workgroups(Bo, k.ntk, IB_SK_GRID);
  k.maxslots = 1;
  for (int64_t b = 0; b < xg; ++b) {
    const int ns = ib_sk_slots(b, k.ntk, k.T, k.W);
    if (ns > k.maxslots) k.maxslots = ns;
  }
  return k;
}

static int fwd_dedup(const float* U, const float* C, int64_t B, float weight, const int32_t* u_rep,
                     const int32_t* u_inv, int64_t Bu, const int32_t* c_rep, const float* c_count, int64_t Bc,
                     float* row_loss, float* lse, float* loss_sum, double* loss_sum64, float* dU, float* S, int prec,
                     const DedupWs& w, hipStream_t st, const int64_t* dinfo = nullptr) {
  // dinfo (device-count form): Bu = dinfo[0], Bc = dinfo[2] on the device; the host sizes every
  // grid for Bu = Bc = B (the caller passes B for both) and the stream-K grid is IB_SK_GRID
  const int64_t NTu = ib_ntiles(Bu), NTc = ib_ntiles(Bc);
  const int64_t nbu = ceil_div(NTu * 1024, 256), nbc = ceil_div(NTc * 1024, 256);
  hipLaunchKernelGGL(ibx_split_image2_kernel, dim3((unsigned)(nbu + nbc)), dim3(256), 0, st,
                     IbxImg{U, Bu, NTu, w.img_q, u_rep, dinfo}, IbxImg{C, Bc, NTc, w.img_k, c_rep, dinfo ? dinfo + 2 : nullptr},
                     nbu, w.done);
  SkPlan k = dedup_plan(Bu, Bc);
  if (dinfo) k.W = IB_SK_GRID;  // the device resolves the share count (ib_resolve)
  RS_REQUIRE(k.maxslots <= 64 && (int64_t)k.maxslots * Bu <= w.prow, "inbatch dedup: %d partial slots", k.maxslots);
  InbatchParams p{nullptr, nullptr, Bu, 0, nullptr, w.pm, w.pl, w.po, S};
  p.Bs = Bc;
  p.kw = c_count;
  p.sk_wg = k.W;
  p.sk_ntk = k.ntk;
  p.dinfo = dinfo;
  p.d_own = 0;
  p.d_str = 2;
  constexpr int NW = IBX_NW;
  static_assert(IB_QW * NW == IB_SKB, "stream-K blocks are one workgroup's owned rows");
  const dim3 grid((unsigned)k.W);
  if (c_count) {
    if (prec == 6) hipLaunchKernelGGL((inbatch_row_m16_kernel<6, NW, 2, true, true>), grid, dim3(64 * NW), 0, st, p, w.img_q, w.img_k);
    else hipLaunchKernelGGL((inbatch_row_m16_kernel<9, NW, 2, true, true>), grid, dim3(64 * NW), 0, st, p, w.img_q, w.img_k);
  } else {
    if (prec == 6) hipLaunchKernelGGL((inbatch_row_m16_kernel<6, NW, 2, false, true>), grid, dim3(64 * NW), 0, st, p, w.img_q, w.img_k);
    else hipLaunchKernelGGL((inbatch_row_m16_kernel<9, NW, 2, false, true>), grid, dim3(64 * NW), 0, st, p, w.img_q, w.img_k);
  }
  int rc = check_launch("inbatch_row_m16 (dedup)");
  if (rc) return rc;
  const int64_t nb = ceil_div(B, IB_FIN_ROWS);
  hipLaunchKernelGGL((inbatch_row_finalize_kernel<IBX_D>), dim3((unsigned)nb), dim3(256), 0, st, U, C, B, k.maxslots,
                     w.pm, w.pl, w.po, weight, row_loss, lse, dU, w.lossp, u_inv, Bu, k.ntk, k.T, k.W, dinfo, 0, 2,
                     IB_SK_GRID, w.done, loss_sum, loss_sum64);
  return check_launch("inbatch_row_finalize (dedup)");
}

// The col pass's exponent bias of each distinct user r (the deduplicated pair, WK):
// P = 2^(s log2 e - lz_r) with lz_r = lse(r's first row) log2 e - log2(count_r), formed in fp64 and
// rounded once, so the col loop reads one value per streamed user (no row map, count or log in
// the loop: 8-10 fewer VGPRs, which is what lets it keep fresh per-tile accumulators).
__global__ __launch_bounds__(256) void ib_lz_kernel(const float* __restrict__ lse, const int32_t* __restrict__ rep,
                                                    const float* __restrict__ cnt, int64_t Bu,
                                                    const int64_t* __restrict__ dinfo, float* __restrict__ lz) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n = dinfo ? dinfo[0] : Bu;
  if (r >= n) return;
  lz[r] = (float)((double)lse[rep[r]] * (double)IB_LOG2E - log2((double)cnt[r]));
}

static int bwd_dedup(const float* U, int64_t B, float weight, const float* lse, const float* S, const float* gscale,
                     const float* dU_unit, float* dU_out, float* dC, const int32_t* u_rep, const float* u_count,
                     int64_t Bu, const int32_t* c_inv, int64_t Bc, int prec, const DedupWs& w, hipStream_t st,
                     const int64_t* dinfo = nullptr, bool reuse = false) {
  const int64_t NTu = ib_ntiles(Bu);
  constexpr bool TI = IB_COL_TIMG != 0;
  if (TI)  // the users' transposed image (the forward's row image is not the col pass's layout)
    hipLaunchKernelGGL(ibx_split_timage_kernel, dim3((unsigned)ceil_div(NTu * 512, 256)), dim3(256), 0, st, U, Bu,
                       NTu, w.img_t, u_rep, dinfo);
  else if (!reuse)  // (reuse: the workspace is the forward's, whose img_q is this image already)
    hipLaunchKernelGGL(ibx_split_image_kernel, dim3((unsigned)ceil_div(NTu * 1024, 256)), dim3(256), 0, st, U, Bu,
                       NTu, w.img_q, u_rep, dinfo);
  const char* uimg = TI ? w.img_t : w.img_q;
  SkPlan k = dedup_plan(Bc, Bu);
  if (dinfo) k.W = IB_SK_GRID;
  RS_REQUIRE(k.maxslots <= 64 && (int64_t)k.maxslots * Bc <= w.prow, "inbatch dedup: %d partial slots", k.maxslots);
  InbatchParams p{nullptr, nullptr, Bc, 0, lse, w.pm, w.pl, w.po, nullptr};
  p.Bs = Bu;
  if (u_count) {   // WK: the streamed users' exponent biases (lse_k then holds them, indexed by user)
    hipLaunchKernelGGL(ib_lz_kernel, dim3((unsigned)ceil_div(Bu, 256)), dim3(256), 0, st, lse, u_rep, u_count, Bu,
                       dinfo, w.lz);
    p.lse_k = w.lz;
  }
  p.sk_wg = k.W;
  p.sk_ntk = k.ntk;
  p.dinfo = dinfo;
  p.d_own = 2;
  p.d_str = 0;
  constexpr int NW = IBX_NW;
  const dim3 grid((unsigned)k.W);
  if (u_count) {
    if (prec == 6) hipLaunchKernelGGL((inbatch_col_m16_kernel<6, NW, true, true, TI>), grid, dim3(64 * NW), 0, st, p, S, uimg);
    else hipLaunchKernelGGL((inbatch_col_m16_kernel<9, NW, true, true, TI>), grid, dim3(64 * NW), 0, st, p, S, uimg);
  } else {
    if (prec == 6) hipLaunchKernelGGL((inbatch_col_m16_kernel<6, NW, false, true, TI>), grid, dim3(64 * NW), 0, st, p, S, uimg);
    else hipLaunchKernelGGL((inbatch_col_m16_kernel<9, NW, false, true, TI>), grid, dim3(64 * NW), 0, st, p, S, uimg);
  }
  int rc = check_launch("inbatch_col_m16 (dedup)");
  if (rc) return rc;
  const int64_t n4 = B * IBX_D / 4;
  hipLaunchKernelGGL((inbatch_col_finalize4_kernel<4>), dim3((unsigned)ceil_div(n4, 256)), dim3(256), 0, st,
                     reinterpret_cast<const f32x4*>(U), n4, k.maxslots, reinterpret_cast<const f32x4*>(w.po), weight,
                     gscale, reinterpret_cast<const f32x4*>(dU_unit), reinterpret_cast<f32x4*>(dU_out),
                     reinterpret_cast<f32x4*>(dC), c_inv, Bc * IBX_D / 4, IBX_D / 4, k.ntk, k.T, k.W, dinfo, 2, 0,
                     IB_SK_GRID);
  return check_launch("inbatch_col_finalize (dedup)");
}

}  // namespace rs

using namespace rs;

extern "C" {

size_t rs_inbatch_softmax_workspace_bytes(int64_t B, int64_t D) {
  return inbatch_ws(B > 0 ? B : 1, D, nullptr, 0, nullptr);
}

int rs_inbatch_softmax_xent_fwd_f32(const float* U, const float* C, int64_t B, int64_t D,
                                    float weight, float* row_loss, float* lse,
                                    float* loss_sum, double* loss_sum64, float* dU,
                                    void* workspace, size_t workspace_bytes,
                                    rs_stream_t stream) {
  RS_REQUIRE(B > 0 && U && C && row_loss && lse && loss_sum,
             "rs_inbatch_softmax_xent_fwd_f32: bad args");
  RS_REQUIRE(aligned16(U) && aligned16(C), "rs_inbatch_softmax_xent_fwd_f32: alignment");
  RS_REQUIRE(B <= ((int64_t)1 << 26), "rs_inbatch_softmax_xent_fwd_f32: B too large");
  if (!workspace || workspace_bytes < rs_inbatch_softmax_workspace_bytes(B, D)) {
    set_error("rs_inbatch_softmax_xent_fwd_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  InbatchWs w;
  inbatch_ws(B, D, workspace, workspace_bytes, &w);
  hipStream_t st = as_stream(stream);
  switch (D) {
    case 32: return fwd_impl<32>(U, C, B, weight, row_loss, lse, loss_sum, loss_sum64, dU, w, st);
    case 64: return fwd_impl<64>(U, C, B, weight, row_loss, lse, loss_sum, loss_sum64, dU, w, st);
    case 128: return fwd_impl<128>(U, C, B, weight, row_loss, lse, loss_sum, loss_sum64, dU, w, st);
    default:
      set_error("rs_inbatch_softmax_xent_fwd_f32: D=%lld not compiled (32, 64, 128)", (long long)D);
      return RS_ERR_UNSUPPORTED;
  }
}

size_t rs_inbatch_scores_bytes(int64_t B) {
  const int64_t nt = ib_ntiles(B > 0 ? B : 1);
  return (size_t)nt * nt * 1024 * sizeof(float);
}

int rs_inbatch_softmax_xent_fwd_store_prec_f32(const float* U, const float* C, int64_t B, int64_t D, float weight,
                                               float* row_loss, float* lse, float* loss_sum, double* loss_sum64,
                                               float* dU, float* scores, int precision, void* workspace,
                                               size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(B > 0 && U && C && row_loss && lse && loss_sum && scores,
             "rs_inbatch_softmax_xent_fwd_store_f32: bad args");
  RS_REQUIRE(aligned16(U) && aligned16(C) && aligned16(scores), "rs_inbatch_softmax_xent_fwd_store_f32: alignment");
  RS_REQUIRE(B <= ((int64_t)1 << 26), "rs_inbatch_softmax_xent_fwd_store_f32: B too large");
  RS_REQUIRE(precision == RS_PREC_F32 || precision == RS_PREC_F32_SPLIT6 || precision == RS_PREC_F32_SPLIT9,
             "rs_inbatch_softmax_xent_fwd_store_f32: precision must be 0, 6 or 9");
  if (!workspace || workspace_bytes < rs_inbatch_softmax_workspace_bytes(B, D)) {
    set_error("rs_inbatch_softmax_xent_fwd_store_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  InbatchWs w;
  inbatch_ws(B, D, workspace, workspace_bytes, &w);
  hipStream_t st = as_stream(stream);
  switch (D) {
    case 32: return fwd_impl<32>(U, C, B, weight, row_loss, lse, loss_sum, loss_sum64, dU, w, st, scores);
    case 64: return fwd_impl<64>(U, C, B, weight, row_loss, lse, loss_sum, loss_sum64, dU, w, st, scores);
    case 128:
      return fwd_impl<128>(U, C, B, weight, row_loss, lse, loss_sum, loss_sum64, dU, w, st, scores, precision);
    default:
      set_error("rs_inbatch_softmax_xent_fwd_store_f32: D=%lld not compiled (32, 64, 128)", (long long)D);
      return RS_ERR_UNSUPPORTED;
  }
}

int rs_inbatch_softmax_xent_fwd_store_f32(const float* U, const float* C, int64_t B, int64_t D, float weight,
                                          float* row_loss, float* lse, float* loss_sum, double* loss_sum64,
                                          float* dU, float* scores, void* workspace, size_t workspace_bytes,
                                          rs_stream_t stream) {
  return rs_inbatch_softmax_xent_fwd_store_prec_f32(U, C, B, D, weight, row_loss, lse, loss_sum, loss_sum64, dU,
                                                    scores, RS_PREC_F32, workspace, workspace_bytes, stream);
}

int rs_inbatch_softmax_xent_bwd_stored_prec_f32(const float* U, const float* C, int64_t B, int64_t D, float weight,
                                                const float* lse, const float* scores, const float* gscale,
                                                const float* dU_unit, float* dU_out, float* dC, int precision,
                                                void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  const bool reuse = (precision & RS_INBATCH_FWD_WS) != 0;
  precision &= ~RS_INBATCH_FWD_WS;
  RS_REQUIRE(B > 0 && U && C && lse && dC && scores, "rs_inbatch_softmax_xent_bwd_stored_f32: bad args");
  RS_REQUIRE(aligned16(U) && aligned16(C) && aligned16(scores), "rs_inbatch_softmax_xent_bwd_stored_f32: alignment");
  RS_REQUIRE(precision == RS_PREC_F32 || precision == RS_PREC_F32_SPLIT6 || precision == RS_PREC_F32_SPLIT9,
             "rs_inbatch_softmax_xent_bwd_stored_f32: precision must be 0, 6 or 9");
  if (!workspace || workspace_bytes < rs_inbatch_softmax_workspace_bytes(B, D)) {
    set_error("rs_inbatch_softmax_xent_bwd_stored_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  InbatchWs w;
  inbatch_ws(B, D, workspace, workspace_bytes, &w);
  hipStream_t st = as_stream(stream);
  switch (D) {
    case 32: return bwd_impl<32>(U, C, B, weight, lse, gscale, dU_unit, dU_out, dC, w, st, scores);
    case 64: return bwd_impl<64>(U, C, B, weight, lse, gscale, dU_unit, dU_out, dC, w, st, scores);
    case 128: return bwd_impl<128>(U, C, B, weight, lse, gscale, dU_unit, dU_out, dC, w, st, scores, precision, reuse);
    default:
      set_error("rs_inbatch_softmax_xent_bwd_stored_f32: D=%lld not compiled (32, 64, 128)", (long long)D);
      return RS_ERR_UNSUPPORTED;
  }
}

int rs_inbatch_softmax_xent_bwd_stored_f32(const float* U, const float* C, int64_t B, int64_t D, float weight,
                                           const float* lse, const float* scores, const float* gscale,
                                           const float* dU_unit, float* dU_out, float* dC, void* workspace,
                                           size_t workspace_bytes, rs_stream_t stream) {
  return rs_inbatch_softmax_xent_bwd_stored_prec_f32(U, C, B, D, weight, lse, scores, gscale, dU_unit, dU_out, dC,
                                                     RS_PREC_F32, workspace, workspace_bytes, stream);
}

int rs_inbatch_softmax_xent_bwd_f32(const float* U, const float* C, int64_t B, int64_t D,
                                    float weight, const float* lse, const float* gscale,
                                    const float* dU_unit, float* dU_out, float* dC,
                                    void* workspace, size_t workspace_bytes,
                                    rs_stream_t stream) {
  RS_REQUIRE(B > 0 && U && C && lse && dC, "rs_inbatch_softmax_xent_bwd_f32: bad args");
  RS_REQUIRE(aligned16(U) && aligned16(C), "rs_inbatch_softmax_xent_bwd_f32: alignment");
  if (!workspace || workspace_bytes < rs_inbatch_softmax_workspace_bytes(B, D)) {
    set_error("rs_inbatch_softmax_xent_bwd_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  InbatchWs w;
  inbatch_ws(B, D, workspace, workspace_bytes, &w);
  hipStream_t st = as_stream(stream);
  switch (D) {
    case 32: return bwd_impl<32>(U, C, B, weight, lse, gscale, dU_unit, dU_out, dC, w, st);
    case 64: return bwd_impl<64>(U, C, B, weight, lse, gscale, dU_unit, dU_out, dC, w, st);
    case 128: return bwd_impl<128>(U, C, B, weight, lse, gscale, dU_unit, dU_out, dC, w, st);
    default:
      set_error("rs_inbatch_softmax_xent_bwd_f32: D=%lld not compiled (32, 64, 128)", (long long)D);
      return RS_ERR_UNSUPPORTED;
  }
}

size_t rs_inbatch_unique_rows_workspace_bytes(int64_t B) {
  size_t need = 0;
  return unique_ws(B, 64, (hipStream_t)0, nullptr, 0, nullptr, &need) == RS_OK ? need : 0;
}

static int unique_run(const char* fn, IbSides sd, int64_t D, int64_t* info, void* workspace,
                      size_t workspace_bytes, hipStream_t st) {
  const int64_t n = sd.B * sd.nsides;
  UniqueWs w;
  size_t need = 0;
  if (unique_ws(n, 64, st, workspace, workspace_bytes, &w, &need) != RS_OK) {
    set_error("%s: rocprim temp query failed", fn);
    return RS_ERR_HIP;
  }
  if (!workspace || workspace_bytes < need) {
    set_error("%s: workspace too small (%zu < %zu)", fn, workspace_bytes, need);
    return RS_ERR_WORKSPACE;
  }
  RS_HIP(hipMemsetAsync(info, 0, 2 * sd.nsides * sizeof(int64_t), st));
  for (int k = 0; k < sd.nsides; ++k)
    RS_HIP(hipMemsetAsync(sd.count[k], 0, (size_t)ib_ntiles(sd.B) * 32 * sizeof(float), st));
  const unsigned g8 = (unsigned)ceil_div(n, 8), g = (unsigned)ceil_div(n, 256);
  hipLaunchKernelGGL(ib_row_hash_kernel, dim3(g8), dim3(256), 0, st, sd, (int)D, w.keys, w.vals);
  int rc = check_launch("ib_row_hash");
  if (rc) return rc;
  hipError_t e = plan_sort(w.sort_temp, w.sort_bytes, w.keys, w.keys_s, w.vals, w.vals_s, n, 64, st);
  if (e != hipSuccess) {
    set_error("%s: radix sort failed: %s", fn, hipGetErrorString(e));
    return RS_ERR_HIP;
  }
  e = plan_heads_scan(w.scan_temp, w.scan_bytes, w.keys_s, w.incl, (size_t)n, st);
  if (e != hipSuccess) {
    set_error("%s: scan failed: %s", fn, hipGetErrorString(e));
    return RS_ERR_HIP;
  }
  hipLaunchKernelGGL(ib_unique_scatter_kernel, dim3(g), dim3(256), 0, st, sd, w.keys_s, w.incl, w.vals_s, w.pos, info);
  rc = check_launch("ib_unique_scatter");
  if (rc) return rc;
  hipLaunchKernelGGL(ib_unique_count_kernel, dim3(g), dim3(256), 0, st, sd, w.pos, w.incl);
  rc = check_launch("ib_unique_count");
  if (rc) return rc;
  hipLaunchKernelGGL(ib_unique_verify_kernel, dim3(g8), dim3(256), 0, st, sd, (int)D,
                     reinterpret_cast<unsigned long long*>(info));
  return check_launch("ib_unique_verify");
}

static int unique_ids_pair(const int64_t* user_ids, const int64_t* item_ids, int64_t B, int64_t user_rows,
                                   int64_t item_rows, int32_t* u_rep, float* u_count, int32_t* u_inv, int32_t* c_rep,
                                   float* c_count, int32_t* c_inv, int64_t* info, void* workspace,
                                   size_t workspace_bytes, rs_stream_t stream, int32_t* u_order = nullptr,
                                   int32_t* c_order = nullptr, int64_t* u_did = nullptr, int64_t* c_did = nullptr,
                                   int32_t* u_start = nullptr, int32_t* c_start = nullptr, int64_t* vinfo = nullptr) {
  RS_REQUIRE(B > 0 && B < ((int64_t)1 << 29) && user_rows > 0 && item_rows > 0 &&
                 user_rows < ((int64_t)1 << 62) && item_rows < ((int64_t)1 << 62),
             "rs_inbatch_unique_ids_pair_i64: bad sizes");
  RS_REQUIRE(user_ids && item_ids && u_rep && u_count && u_inv && c_rep && c_count && c_inv && info,
             "rs_inbatch_unique_ids_pair_i64: bad args");
  const char* fn = "rs_inbatch_unique_ids_pair_i64";
  IbSides sd{{nullptr, nullptr}, {u_rep, c_rep}, {u_inv, c_inv}, {u_count, c_count}, B, 2, {u_order, c_order},
             {u_did, c_did}, {user_ids, item_ids}, {user_rows, item_rows}, {u_start, c_start}, vinfo};
  const int64_t n = 2 * B;
  const int64_t mr = user_rows > item_rows ? user_rows : item_rows;
  int bits = 1;
  while (((int64_t)1 << bits) <= mr) ++bits;  // 2^bits - 1 >= rows: the reserved key is no row
  hipStream_t st = as_stream(stream);
  UniqueWs w;
  size_t need = 0;
  if (unique_ws(n, bits + 1, st, workspace, workspace_bytes, &w, &need) != RS_OK) {
    set_error("%s: rocprim temp query failed", fn);
    return RS_ERR_HIP;
  }
  if (!workspace || workspace_bytes < need) {
    set_error("%s: workspace too small (%zu < %zu)", fn, workspace_bytes, need);
    return RS_ERR_WORKSPACE;
  }
  const unsigned g = (unsigned)ceil_div(n, 256);
  hipLaunchKernelGGL(ib_id_key_kernel, dim3((unsigned)ceil_div(2 * ib_ntiles(B) * 32, 256)), dim3(256), 0, st,
                     user_ids, item_ids, B, user_rows, item_rows, bits, w.keys, w.vals, u_count, c_count, info,
                     u_did, c_did);
  int rc = check_launch("ib_id_key");
  if (rc) return rc;
  hipError_t e = hipSuccess;
  if (IB_IDS_SORT && n <= PS_MAXN) {
    rc = ids_sort(w, n, bits + 1, st);
    if (rc) return rc;
  } else {
    e = plan_sort(w.sort_temp, w.sort_bytes, w.keys, w.keys_s, w.vals, w.vals_s, n, bits + 1, st);
  }
  if (e != hipSuccess) {
    set_error("%s: radix sort failed: %s", fn, hipGetErrorString(e));
    return RS_ERR_HIP;
  }
  e = plan_heads_scan(w.scan_temp, w.scan_bytes, w.keys_s, w.incl, (size_t)n, st);
  if (e != hipSuccess) {
    set_error("%s: scan failed: %s", fn, hipGetErrorString(e));
    return RS_ERR_HIP;
  }
  hipLaunchKernelGGL(ib_unique_scatter_kernel, dim3(g), dim3(256), 0, st, sd, w.keys_s, w.incl, w.vals_s, w.pos, info);
  rc = check_launch("ib_unique_scatter");
  if (rc) return rc;
  hipLaunchKernelGGL(ib_unique_count_kernel, dim3(g), dim3(256), 0, st, sd, w.pos, w.incl);
  return check_launch("ib_unique_count");
}

int rs_inbatch_unique_ids_pair_i64(const int64_t* user_ids, const int64_t* item_ids, int64_t B, int64_t user_rows,
                                   int64_t item_rows, int32_t* u_rep, float* u_count, int32_t* u_inv, int32_t* c_rep,
                                   float* c_count, int32_t* c_inv, int64_t* info, void* workspace,
                                   size_t workspace_bytes, rs_stream_t stream) {
  return unique_ids_pair(user_ids, item_ids, B, user_rows, item_rows, u_rep, u_count, u_inv, c_rep, c_count, c_inv,
                         info, workspace, workspace_bytes, stream);
}

int rs_inbatch_unique_ids_pair_order_i64(const int64_t* user_ids, const int64_t* item_ids, int64_t B,
                                         int64_t user_rows, int64_t item_rows, int32_t* u_rep, float* u_count,
                                         int32_t* u_inv, int32_t* u_order, int32_t* c_rep, float* c_count,
                                         int32_t* c_inv, int32_t* c_order, int64_t* info, void* workspace,
                                         size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(u_order && c_order, "rs_inbatch_unique_ids_pair_order_i64: null order");
  return unique_ids_pair(user_ids, item_ids, B, user_rows, item_rows, u_rep, u_count, u_inv, c_rep, c_count, c_inv,
                         info, workspace, workspace_bytes, stream, u_order, c_order);
}

int rs_inbatch_unique_ids_plan_i64(const int64_t* user_ids, const int64_t* item_ids, int64_t B, int64_t user_rows,
                                   int64_t item_rows, int32_t* u_rep, float* u_count, int32_t* u_inv,
                                   int32_t* u_order, int64_t* u_did, int32_t* u_start, int32_t* c_rep,
                                   float* c_count, int32_t* c_inv, int32_t* c_order, int64_t* c_did,
                                   int32_t* c_start, int64_t* info, void* workspace, size_t workspace_bytes,
                                   rs_stream_t stream) {
  RS_REQUIRE(!u_order == !c_order && !u_did == !c_did && !u_start == !c_start,
             "rs_inbatch_unique_ids_plan_i64: orders / dids / starts in pairs");
  return unique_ids_pair(user_ids, item_ids, B, user_rows, item_rows, u_rep, u_count, u_inv, c_rep, c_count, c_inv,
                         info, workspace, workspace_bytes, stream, u_order, c_order, u_did, c_did, u_start, c_start,
                         u_did ? info + 4 : nullptr);
}

int rs_inbatch_unique_rows_f32(const float* X, int64_t B, int64_t D, int32_t* rep, float* count, int32_t* inv,
                               int64_t* info, void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(B > 0 && B < ((int64_t)1 << 30) && D > 0 && D % 4 == 0, "rs_inbatch_unique_rows_f32: bad sizes");
  RS_REQUIRE(X && rep && count && inv && info && aligned16(X), "rs_inbatch_unique_rows_f32: bad args");
  IbSides sd{{X, X}, {rep, rep}, {inv, inv}, {count, count}, B, 1};
  return unique_run("rs_inbatch_unique_rows_f32", sd, D, info, workspace, workspace_bytes, as_stream(stream));
}

size_t rs_inbatch_unique_pair_workspace_bytes(int64_t B) { return rs_inbatch_unique_rows_workspace_bytes(2 * B); }

int rs_inbatch_unique_pair_f32(const float* U, const float* C, int64_t B, int64_t D, int32_t* u_rep,
                               float* u_count, int32_t* u_inv, int32_t* c_rep, float* c_count, int32_t* c_inv,
                               int64_t* info, void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(B > 0 && B < ((int64_t)1 << 29) && D > 0 && D % 4 == 0, "rs_inbatch_unique_pair_f32: bad sizes");
  RS_REQUIRE(U && C && u_rep && u_count && u_inv && c_rep && c_count && c_inv && info && aligned16(U) &&
                 aligned16(C),
             "rs_inbatch_unique_pair_f32: bad args");
  IbSides sd{{U, C}, {u_rep, c_rep}, {u_inv, c_inv}, {u_count, c_count}, B, 2};
  return unique_run("rs_inbatch_unique_pair_f32", sd, D, info, workspace, workspace_bytes, as_stream(stream));
}

size_t rs_inbatch_dedup_workspace_bytes(int64_t B, int64_t D) {
  (void)D;
  return dedup_ws(B > 0 ? B : 1, nullptr, 0, nullptr);
}

static int dedup_check(const char* fn, int64_t B, int64_t D, int precision, const int32_t* rep, const void* other,
                       int64_t Bx, const void* workspace, size_t workspace_bytes) {
  RS_REQUIRE(D == IBX_D, "%s: D must be %d", fn, IBX_D);
  RS_REQUIRE(precision == RS_PREC_F32_SPLIT6 || precision == RS_PREC_F32_SPLIT9, "%s: precision must be 6 or 9", fn);
  RS_REQUIRE(B > 0 && B <= ((int64_t)1 << 26) && Bx >= 1 && Bx <= B, "%s: bad sizes", fn);
  RS_REQUIRE((rep == nullptr) == (other == nullptr) && (rep != nullptr || Bx == B),
             "%s: a side is either deduplicated (rep and its map given, Bx <= B) or not (both NULL, Bx = B)", fn);
  if (!workspace || workspace_bytes < rs_inbatch_dedup_workspace_bytes(B, D)) {
    set_error("%s: workspace too small", fn);
    return RS_ERR_WORKSPACE;
  }
  return RS_OK;
}

int rs_inbatch_softmax_xent_fwd_dedup_f32(const float* U, const float* C, int64_t B, int64_t D, float weight,
                                          const int32_t* u_rep, const int32_t* u_inv, int64_t Bu,
                                          const int32_t* c_rep, const float* c_count, int64_t Bc, float* row_loss,
                                          float* lse, float* loss_sum, double* loss_sum64, float* dU, float* scores,
                                          int precision, void* workspace, size_t workspace_bytes,
                                          rs_stream_t stream) {
  const char* fn = "rs_inbatch_softmax_xent_fwd_dedup_f32";
  RS_REQUIRE(U && C && row_loss && lse && loss_sum && dU && scores, "%s: bad args", fn);
  RS_REQUIRE(aligned16(U) && aligned16(C) && aligned16(scores) && aligned16(dU), "%s: alignment", fn);
  int rc = dedup_check(fn, B, D, precision, u_rep, u_inv, Bu, workspace, workspace_bytes);
  if (rc) return rc;
  rc = dedup_check(fn, B, D, precision, c_rep, c_count, Bc, workspace, workspace_bytes);
  if (rc) return rc;
  DedupWs w;
  dedup_ws(B, workspace, workspace_bytes, &w);
  return fwd_dedup(U, C, B, weight, u_rep, u_inv, Bu, c_rep, c_count, Bc, row_loss, lse, loss_sum, loss_sum64, dU,
                   scores, precision, w, as_stream(stream));
}

int rs_inbatch_softmax_xent_bwd_dedup_f32(const float* U, int64_t B, int64_t D, float weight, const float* lse,
                                          const float* scores, const float* gscale, const float* dU_unit,
                                          float* dU_out, float* dC, const int32_t* u_rep, const float* u_count,
                                          int64_t Bu, const int32_t* c_inv, int64_t Bc, int precision,
                                          void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  const char* fn = "rs_inbatch_softmax_xent_bwd_dedup_f32";
  const bool reuse = (precision & RS_INBATCH_FWD_WS) != 0;
  precision &= ~RS_INBATCH_FWD_WS;
  RS_REQUIRE(U && lse && scores && dC, "%s: bad args", fn);
  RS_REQUIRE(aligned16(U) && aligned16(scores) && aligned16(dC) && (!dU_unit || aligned16(dU_unit)) &&
                 (!dU_out || aligned16(dU_out)),
             "%s: alignment", fn);
  int rc = dedup_check(fn, B, D, precision, u_rep, u_count, Bu, workspace, workspace_bytes);
  if (rc) return rc;
  RS_REQUIRE(Bc >= 1 && Bc <= B && (c_inv != nullptr || Bc == B), "%s: c_inv is required when Bc < B", fn);
  DedupWs w;
  dedup_ws(B, workspace, workspace_bytes, &w);
  return bwd_dedup(U, B, weight, lse, scores, gscale, dU_unit, dU_out, dC, u_rep, u_count, Bu, c_inv, Bc, precision,
                   w, as_stream(stream), nullptr, reuse);
}

int rs_inbatch_softmax_xent_fwd_dedup_dev_f32(const float* U, const float* C, int64_t B, int64_t D, float weight,
                                              const int32_t* u_rep, const int32_t* u_inv, const int32_t* c_rep,
                                              const float* c_count, const int64_t* info, float* row_loss, float* lse,
                                              float* loss_sum, double* loss_sum64, float* dU, float* scores,
                                              int precision, void* workspace, size_t workspace_bytes,
                                              rs_stream_t stream) {
  const char* fn = "rs_inbatch_softmax_xent_fwd_dedup_dev_f32";
  RS_REQUIRE(U && C && row_loss && lse && loss_sum && dU && scores && info, "%s: bad args", fn);
  RS_REQUIRE(aligned16(U) && aligned16(C) && aligned16(scores) && aligned16(dU), "%s: alignment", fn);
  int rc = dedup_check(fn, B, D, precision, u_rep, u_inv, B, workspace, workspace_bytes);
  if (rc) return rc;
  rc = dedup_check(fn, B, D, precision, c_rep, c_count, B, workspace, workspace_bytes);
  if (rc) return rc;
  RS_REQUIRE(u_rep && c_rep, "%s: both sides' maps are required", fn);
  DedupWs w;
  dedup_ws(B, workspace, workspace_bytes, &w);
  return fwd_dedup(U, C, B, weight, u_rep, u_inv, B, c_rep, c_count, B, row_loss, lse, loss_sum, loss_sum64, dU,
                   scores, precision, w, as_stream(stream), info);
}

int rs_inbatch_softmax_xent_bwd_dedup_dev_f32(const float* U, int64_t B, int64_t D, float weight, const float* lse,
                                              const float* scores, const float* gscale, const float* dU_unit,
                                              float* dU_out, float* dC, const int32_t* u_rep, const float* u_count,
                                              const int32_t* c_inv, const int64_t* info, int precision,
                                              void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  const char* fn = "rs_inbatch_softmax_xent_bwd_dedup_dev_f32";
  const bool reuse = (precision & RS_INBATCH_FWD_WS) != 0;
  precision &= ~RS_INBATCH_FWD_WS;
  RS_REQUIRE(U && lse && scores && dC && info && u_rep && u_count && c_inv, "%s: bad args", fn);
  RS_REQUIRE(aligned16(U) && aligned16(scores) && aligned16(dC) && (!dU_unit || aligned16(dU_unit)) &&
                 (!dU_out || aligned16(dU_out)),
             "%s: alignment", fn);
  int rc = dedup_check(fn, B, D, precision, u_rep, u_count, B, workspace, workspace_bytes);
  if (rc) return rc;
  DedupWs w;
  dedup_ws(B, workspace, workspace_bytes, &w);
  return bwd_dedup(U, B, weight, lse, scores, gscale, dU_unit, dU_out, dC, u_rep, u_count, B, c_inv, B, precision,
                   w, as_stream(stream), info, reuse);
}

}  // extern "C"
