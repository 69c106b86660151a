// gemm_ws.hip — weight-stationary split GEMM for the Dense layers at large batch (its own
// translation unit). Dispatched from gemm.hip ahead of the skinny kernel.
//
// C[M, N] = epi(A[M, K] op(B)) for the towers' and the deep net's forward (op(B) = W [K, N], bias +
// ReLU epilogue) and dX (op(B) = W^T given as B [N][K], ReLU-mask epilogue) at M in the tens of
// thousands and K, N in {64, 128, 256}. At those shapes a layer is ~20 us of MFMA and ~25 us of HBM
// traffic, and per-block staging of W with a barrier per k-chunk (gemm_skinny_kernel) leaves each
// CU two or three serial load -> MFMA -> store phases: 2-3.6 TB/s and 0.2-0.3 MFMA busy (profiles/
// r04_pmc_towers.txt). Here one 512-thread workgroup per CU splits its column slice of W into bf16
// planes ONCE, into LDS (K x NW x 3 planes, <= 96 KB), and its 8 waves then stream 32-row blocks
// with no barrier: each wave prefetches its next block's A rows into registers (two register
// chunks of <= 128 k) while it runs the current block's MFMAs, and its epilogue stores drain while
// the next block computes. Products: v_mfma_f32_32x32x16_bf16 on the transposed problem C^T = op(B)^T
// A^T (W fragments as the row operand from LDS, the A rows as the column operand straight from
// registers), so a lane ends with 4 consecutive columns of one output row per register quad: f32x4
// epilogue loads and stores without a transpose. Same exact 3-term splits and NP cross products as
// the other split GEMMs (split.hpp), fp32 accumulation over K (<= 16 k-steps).
//
// Workgroup -> work: (problem of a grouped launch, column slice) combos are dealt within an XCD
// (workgroup b runs on XCD b % 8), and the row range is partitioned so the workgroups of one XCD
// that own different column slices of the same rows run over the same A rows together (the second
// slice's A reads hit that XCD's L2).
//
// Also here: wgrad_ws_kernel, the large-batch weight gradients (dW = X^T G + db, the contraction
// over the batch rows; see its comment below), dispatched from gemm.hip's wgrad entry points.
#include "common.hpp"
#include "split.hpp"
#include "gemm.hpp"

namespace rs {

constexpr int WS_THREADS = 512;
#ifndef WS_OCC
#define WS_OCC 1  // workgroups per CU (2: 64-column slices, 32-k register chunks, 128 VGPRs)
#endif
#ifndef WS_READ_AHEAD
// the next W fragment read ahead of this one's MFMAs: the six gemm_ws launches of a C3 step
// 583.4 -> 577.1 us (profiles/r06s_read_ahead_fin_ab.txt); same products, bitwise
#define WS_READ_AHEAD 1
#endif
template <int K, int NW, bool TB, int NP, bool MASKED>
__global__ __launch_bounds__(WS_THREADS, 2 * WS_OCC) void gemm_ws_kernel(GemmParams p, int nslice) {
  constexpr int NTT = NW / 32;           // 32-column MFMA tiles of the slice
  // A rows in register chunks of KC k, an even number per block, so chunk c of every block sits in
  // ring slot c % 2 (compile-time register names)
  constexpr int KC = WS_OCC > 1 ? 32 : (K <= 128 ? K / 2 : 64);
  constexpr int NCH = K / KC;            // chunks per row block (2 or 4)
  constexpr int SPC = KC / 16;           // 16-k steps per chunk
  constexpr int IMGB = K * NW * 6;       // the slice image: 3 bf16 planes
  static_assert(IMGB <= 96 * 1024, "slice image must fit LDS");
  __shared__ __attribute__((aligned(16))) char smem[IMGB + NW * 4];
  float* sbias = reinterpret_cast<float*>(smem + IMGB);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int G = p.ngroup > 1 ? p.ngroup : 1;
  const int ncombo = G * nslice;
  const int b = (int)blockIdx.x, xcd = b & 7, i = b >> 3, ni = (int)(gridDim.x >> 3);
  const int combo = i % ncombo;
  const int prt = (i / ncombo) * 8 + xcd, nprt = (ni / ncombo) * 8;
  const int pg = combo / nslice, sl = combo % nslice;
#pragma unroll
  for (int q = 1; q < GEMM_GMAX; ++q)
    if (pg == q) {  // problem of a grouped launch (constant-index selection)
      p.A = p.gA[q];
      p.B = p.gB[q];
      p.C = p.gC[q];
      p.bias = p.gbias[q];
      p.mask = p.gmask[q];
      p.mrow = p.gmrow[q];
      p.mdev = p.gmdev[q];
      p.arow = p.garow[q];
    }
  const int64_t n0 = (int64_t)sl * NW;
  if (p.mdev) {  // the row count from device memory (the grid is sized for p.M)
    const int64_t md = *p.mdev;
    p.M = md < p.M ? (md > 0 ? md : 0) : p.M;
  }

  // the slice image: fragment (s, t) = the row operand of k-step s, column tile t; lane l holds
  // op(B)[16 s + 8 (l >> 5) + j][n0 + 32 t + (l & 31)], j < 8, as three 16-B planes 1 KB apart
  constexpr int NU = (K / 16) * NTT * 64;
  for (int u = tid; u < NU; u += WS_THREADS) {
    const int l = u & 63, st = u >> 6;
    const int t = st % NTT, s = st / NTT;
    const int64_t n = n0 + 32 * t + (l & 31), k = 16 * s + 8 * (l >> 5);
    f32x4 v0, v1;
    if constexpr (TB) {  // B [N][K]: 8 consecutive k of row n
      const float* src = p.B + n * p.ldb + k;
      v0 = *reinterpret_cast<const f32x4*>(src);
      v1 = *reinterpret_cast<const f32x4*>(src + 4);
    } else {  // B [K][N]: column n, rows k .. k + 7
      const float* src = p.B + k * p.ldb + n;
      v0 = f32x4{src[0], src[p.ldb], src[2 * p.ldb], src[3 * p.ldb]};
      v1 = f32x4{src[4 * p.ldb], src[5 * p.ldb], src[6 * p.ldb], src[7 * p.ldb]};
    }
    const IbSplit x0 = ib_split2(v0[0], v0[1]), x1 = ib_split2(v0[2], v0[3]), x2 = ib_split2(v1[0], v1[1]),
                  x3 = ib_split2(v1[2], v1[3]);
    char* dst = smem + st * 3072 + 16 * l;
    *reinterpret_cast<u32x4*>(dst) = u32x4{x0.h, x1.h, x2.h, x3.h};
    *reinterpret_cast<u32x4*>(dst + 1024) = u32x4{x0.m, x1.m, x2.m, x3.m};
    *reinterpret_cast<u32x4*>(dst + 2048) = u32x4{x0.l, x1.l, x2.l, x3.l};
  }
  for (int c = tid; c < NW; c += WS_THREADS) sbias[c] = p.bias ? p.bias[n0 + c] : 0.f;
  __syncthreads();

  // this workgroup's 32-row blocks [jb, je); the wave takes jb + wave, jb + wave + 8, ...
  const int64_t nbt = (p.M + 31) / 32;
  const int64_t jb = nbt * prt / nprt, je = nbt * (prt + 1) / nprt;
  const int64_t nbw = je - jb > wave ? (je - jb - wave + 7) / 8 : 0;
  const int64_t Mlast = p.M - 1;
  if (nbw == 0) return;  // (no barrier follows; M = 0 leaves nbw = 0)

  f32x4 ab[SPC][2];  // the A chunk: lane (r, h) holds row m, k = KC c + 16 s + 8 h .. + 7
  f32x16 acc[NTT];
  f32x4 mreg[MASKED ? NTT : 1][4];
#pragma unroll
  for (int t = 0; t < NTT; ++t) acc[t] = f32x16{};

  // every load is unconditional (rows past M read row M - 1; the chunk after the wave's last one
  // re-reads that one): with no branch around a load, the compiler's vmcnt waits count exactly the
  // loads older than the awaited ones
  auto aload = [&](int64_t j, int c) {
    int64_t m = (jb + wave + 8 * j) * 32 + r;
    if (m > Mlast) m = Mlast;
    if (p.arow) m = p.arow[m];  // the stored A row of output row m (a layer over distinct rows' inputs)
    const float* src = p.A + m * p.lda + c * KC + 8 * h;
#pragma unroll
    for (int s = 0; s < SPC; ++s) {
      ab[s][0] = *reinterpret_cast<const f32x4*>(src + 16 * s);
      ab[s][1] = *reinterpret_cast<const f32x4*>(src + 16 * s + 4);
    }
  };
  // the chunk's A rows split into bf16 planes (this frees the fp32 registers for the next chunk's
  // loads, which then fly during this chunk's MFMAs)
  auto split = [&](u32x4 (&ap)[SPC][3]) {
#pragma unroll
    for (int s = 0; s < SPC; ++s) {
      const IbSplit x0 = ib_split2(ab[s][0][0], ab[s][0][1]), x1 = ib_split2(ab[s][0][2], ab[s][0][3]),
                    x2 = ib_split2(ab[s][1][0], ab[s][1][1]), x3 = ib_split2(ab[s][1][2], ab[s][1][3]);
      ap[s][0] = u32x4{x0.h, x1.h, x2.h, x3.h};
      ap[s][1] = u32x4{x0.m, x1.m, x2.m, x3.m};
      ap[s][2] = u32x4{x0.l, x1.l, x2.l, x3.l};
    }
  };
  auto compute = [&](const u32x4 (&ap)[SPC][3], int c) {
    if constexpr (WS_READ_AHEAD) {
      // fragment q = (k-step s, tile t) = (q / NTT, q % NTT); fragment q + 1's three planes are read
      // before fragment q's MFMAs (12 VGPRs), so their LDS latency hides behind them
      auto rd = [&](int q, u32x4 (&wp)[3]) __attribute__((always_inline)) {
        const char* base = smem + (int64_t)((c * SPC + q / NTT) * NTT + q % NTT) * 3072 + 16 * lane;
        wp[0] = *reinterpret_cast<const u32x4*>(base);
        wp[1] = *reinterpret_cast<const u32x4*>(base + 1024);
        wp[2] = *reinterpret_cast<const u32x4*>(base + 2048);
      };
      u32x4 wpf[2][3];
      rd(0, wpf[0]);
#pragma unroll
      for (int q = 0; q < SPC * NTT; ++q) {
        if (q + 1 < SPC * NTT) rd(q + 1, wpf[(q + 1) & 1]);
        const u32x4 wp[3] = {wpf[q & 1][0], wpf[q & 1][1], wpf[q & 1][2]};
        acc[q % NTT] = mfma_split<NP>(wp, ap[q / NTT], acc[q % NTT]);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < SPC; ++s) {
        const char* base = smem + (int64_t)((c * SPC + s) * NTT) * 3072 + 16 * lane;
#pragma unroll
        for (int t = 0; t < NTT; ++t) {
          const u32x4 wp[3] = {*reinterpret_cast<const u32x4*>(base + t * 3072),
                               *reinterpret_cast<const u32x4*>(base + t * 3072 + 1024),
                               *reinterpret_cast<const u32x4*>(base + t * 3072 + 2048)};
#ifndef WS_PROBE_NOMFMA  // (timing probe: one product instead of NP; wrong results)
          acc[t] = mfma_split<NP>(wp, ap[s], acc[t]);
#else
          acc[t] = mfma_bf16(wp[0], ap[s][0], acc[t]);
#endif
        }
        // one k-step's fragment reads at a time (hoisting them all ahead spills)
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  auto mload = [&](int64_t j) {
    if constexpr (MASKED) {
      int64_t m = (jb + wave + 8 * j) * 32 + r;
      if (m > Mlast) m = Mlast;
      if (p.mrow) m = p.mrow[m];  // the mask row of output row m (distinct-row layers)
      const float* src = p.mask + m * p.ldm + n0 + 4 * h;
#pragma unroll
      for (int t = 0; t < NTT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) mreg[t][q] = *reinterpret_cast<const f32x4*>(src + 32 * t + 8 * q);
    }
  };
  // acc[t] register 4 q + e = C[m][n0 + 32 t + 8 q + 4 h + e], m = 32 (jb + wave + 8 j) + r
  // Rows past M store to row M - 1 the values they computed from row M - 1's A and mask rows: the
  // same bits the live lane of that row stores, so every store is unconditional (a store under a
  // branch makes the compiler assume it may not have been issued and wait for the prefetch early)
  auto epilogue = [&](int64_t j) {
    int64_t m = (jb + wave + 8 * j) * 32 + r;
    if (m > Mlast) m = Mlast;
    float* dst = p.C + m * p.ldc + n0 + 4 * h;
    const bool relu = p.act == RS_ACT_RELU;
#pragma unroll
    for (int t = 0; t < NTT; ++t) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int col = 32 * t + 8 * q + 4 * h;
        f32x4 v = f32x4{acc[t][4 * q], acc[t][4 * q + 1], acc[t][4 * q + 2], acc[t][4 * q + 3]} +
                  *reinterpret_cast<const f32x4*>(sbias + col);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float y = v[e];
          if (relu) y = fmaxf(y, 0.f);
          if constexpr (MASKED) {
            if (!(mreg[t][q][e] > 0.f)) y = 0.f;
          }
          v[e] = y;
        }
#ifndef WS_PROBE_NOSTORE  // (timing probe: no output stores; wrong results)
        *reinterpret_cast<f32x4*>(dst + 32 * t + 8 * q) = v;
#else
        if (v[0] == 12345.f) *reinterpret_cast<f32x4*>(dst + 32 * t + 8 * q) = v;
#endif
      }
      acc[t] = f32x16{};
    }
  };
  // per chunk: the next chunk's loads go out first (they fly during this chunk's MFMAs and this
  // block's stores), then the block's mask (first chunk), the MFMAs, the epilogue (last chunk)
  auto block = [&](int64_t j) {
    [[maybe_unused]] const int64_t jn = j + 1 < nbw ? j + 1 : j;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      u32x4 ap[SPC][3];
      split(ap);
#ifndef WS_PROBE_NOLOAD  // (timing probe: A read once per wave; wrong results)
      if (c + 1 < NCH) aload(j, c + 1);
      else aload(jn, 0);
#endif
      if (c == 0) mload(j);
      __builtin_amdgcn_sched_barrier(0);
      compute(ap, c);
      if (c == NCH - 1) epilogue(j);
    }
  };
  // the first block peeled: the loop is then entered with the memory operations outstanding that
  // its back edge carries (a prefetch behind a block's stores), so its waits match on both paths
#ifdef WS_PRIO  // (A/B: static priority for the second-dispatched half of the waves)
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
#endif
  aload(0, 0);
  block(0);
  for (int64_t j = 1; j < nbw; ++j) block(j);
}

// the envelope: split precision, no trans_a, forward / dX epilogues only (bias, ReLU, mask), K and
// N in {64, 128, 256}, a large batch (the rows of all problems >= WS_MIN_ROWS), 16-B aligned rows
constexpr int64_t WS_MIN_ROWS = 32768;

// column slice width: the slice image K x NW x 6 B must fit 96 KB, and a masked epilogue keeps the
// block's mask in registers (NW / 2 VGPRs) beside the A chunk ring
#ifndef WS_MASKED_K128_NW
// masked K = 128 slice width: 128 (the block's mask in 64 VGPRs, no spills) runs the C3 towers'
// masked dX 12-15 us per step faster than 64 (profiles/r06af_ws_masked_nw_ab.txt); same sums
#define WS_MASKED_K128_NW 128
#endif
static int ws_slice(int64_t K, int64_t N, bool masked) {
  int nw = K <= 64 ? 128 : (K == 128 ? 128 : 64);
  if ((masked && K >= 128) || WS_OCC > 1) nw = 64;
  if (masked && K == 128 && WS_OCC == 1) nw = WS_MASKED_K128_NW;
  if (WS_OCC > 1 && K == 256) nw = 32;  // two 48 KB images per CU
  while (nw > N) nw >>= 1;
  return nw;
}

bool ws_ok(int ta, int tb, const GemmParams& p) {
  if (ta || p.epi != 0 || !(p.prec == 6 || p.prec == 9) || p.ones_row1 || p.addend || p.beta != 0.f) return false;
  if (!(p.K == 64 || p.K == 128 || p.K == 256) || !(p.N == 64 || p.N == 128 || p.N == 256)) return false;
  const int G = p.ngroup > 1 ? p.ngroup : 1;
  if (p.M * G < WS_MIN_ROWS) return false;
  if (p.lda % 4 || p.ldb % 4 || p.ldc % 4 || (p.mask && p.ldm % 4)) return false;
  for (int i = 0; i < G; ++i) {
    const float* A = G > 1 ? p.gA[i] : p.A;
    const float* B = G > 1 ? p.gB[i] : p.B;
    const float* C = G > 1 ? p.gC[i] : p.C;
    const float* mk = G > 1 ? p.gmask[i] : p.mask;
    if (!aligned16(A) || !aligned16(B) || !aligned16(C) || (mk && !aligned16(mk))) return false;
    if (!mk != !p.mask) return false;  // a mask for every problem or for none
    if (G > 1 && (!p.gmrow[i] != !p.mrow || !p.gmdev[i] != !p.mdev || !p.garow[i] != !p.arow))
      return false;  // likewise the row maps
  }
  return true;
}

template <int K, int NW, bool TB, int NP, bool MASKED>
static void ws_launch(const GemmParams& p, hipStream_t st) {
  const int G = p.ngroup > 1 ? p.ngroup : 1;
  const int nslice = (int)(p.N / NW), nc = G * nslice;
  const int per = (nc >= 32 ? 1 : 32 / nc) * WS_OCC;  // workgroups per combo and XCD
  hipLaunchKernelGGL((gemm_ws_kernel<K, NW, TB, NP, MASKED>), dim3((unsigned)(8 * nc * per)), dim3(WS_THREADS), 0, st,
                     p, nslice);
}

template <int K, bool TB, int NP, bool MASKED>
static void ws_launch_nw(const GemmParams& p, hipStream_t st) {
  switch (ws_slice(p.K, p.N, MASKED)) {
    case 128: if constexpr (K <= 128) ws_launch<K, 128, TB, NP, MASKED>(p, st); break;
    case 64: ws_launch<K, 64, TB, NP, MASKED>(p, st); break;
#if WS_OCC > 1
    case 32: ws_launch<K, 32, TB, NP, MASKED>(p, st); break;
#endif
    default: break;
  }
}

template <bool TB, int NP, bool MASKED>
static void ws_launch_k(const GemmParams& p, hipStream_t st) {
  switch (p.K) {
    case 64: ws_launch_nw<64, TB, NP, MASKED>(p, st); break;
    case 128: ws_launch_nw<128, TB, NP, MASKED>(p, st); break;
    case 256: ws_launch_nw<256, TB, NP, MASKED>(p, st); break;
    default: break;
  }
}

template <bool TB, int NP>
static void ws_launch_m(const GemmParams& p, hipStream_t st) {
  GemmParams q = p;
  if (p.ngroup > 1) {  // slot 0 of the group arrays is the kernel's default problem
    q.A = p.gA[0];
    q.B = p.gB[0];
    q.C = p.gC[0];
    q.bias = p.gbias[0];
    q.mask = p.gmask[0];
    q.mrow = p.gmrow[0];
    q.mdev = p.gmdev[0];
    q.arow = p.garow[0];
  }
  if (q.mask) ws_launch_k<TB, NP, true>(q, st);
  else ws_launch_k<TB, NP, false>(q, st);
}

void ws_dispatch(int tb, const GemmParams& p, hipStream_t st) {
  if (tb) { if (p.prec == 6) ws_launch_m<true, 6>(p, st); else ws_launch_m<true, 9>(p, st); }
  else { if (p.prec == 6) ws_launch_m<false, 6>(p, st); else ws_launch_m<false, 9>(p, st); }
}

}  // namespace rs

namespace rs {

// ---- weight gradients: dW = X^T G (+ db = column sums of G) at large batch -----------------------
// The contraction runs over the batch rows, which are the row index of both stored operands, so
// every MFMA operand is a transpose of what HBM holds. A 512-thread workgroup owns one BM x BN tile
// of dW for one K slice (split-K, slabs reduced by launch_slab_reduce_strided as before): per 64-row
// chunk each loader thread reads 8 consecutive batch rows of 4 columns of X or of G (16-B loads; a
// wave instruction reads 2 rows of the tile's columns), splits them into bf16 planes and writes
// per column one 16-B k-run per plane into LDS images X^T [BM][64] and G^T [BN][64] (16-B chunks
// XOR-swizzled, wg_swz: conflict-free fragment reads and writes); the next chunk's
// loads fly during this chunk's MFMAs (v_mfma_f32_32x32x16_bf16, X^T fragments as the row operand,
// G^T as the column operand). 64 contraction rows per barrier pair against gemm_x3_kernel's 16.
// The tiles of one (problem, slice) run on one XCD (block order), so its L2 serves the shared rows.
// Row-mapped X (p.arow, the distinct-row towers): the stored rows of the next chunk are loaded a
// chunk ahead. Tile m == 0 workgroups also sum G's columns (slab row colsum_row).
#ifndef WGWS_KC
#define WGWS_KC 64  // contraction rows per chunk (one 96-KB workgroup per CU; 32 with WGWS_OCC 2: two 48-KB ones, no faster)
#endif
#ifndef WGWS_OCC
#define WGWS_OCC 1  // workgroups per CU (2 needs KC = 32: 48 KB of LDS, <= 128 VGPRs each)
#endif

// 16-B chunk swizzle of an image row of KC bf16 (KC / 8 chunks): KC = 64, (row ^ row >> 2) & 7, a
// bijection on any 8 consecutive rows and on the rows 4 q + e of 8 consecutive column quads q; KC =
// 32, (row >> 2) & 3, distinct (row & 3, chunk) pairs over 8 consecutive rows. Fragment reads are
// conflict-free either way.
template <int KC>
__device__ __forceinline__ int wg_swz(int row) {
  return KC == 64 ? (row ^ (row >> 2)) & 7 : (row >> 2) & 3;
}

template <int BM, int BN, int NP, int KC, int OCC>
__global__ __launch_bounds__(512, 2 * OCC) void wgrad_ws_kernel(GemmParams p, int ntm, int ntn) {
  constexpr int RPT = KC / 8;                               // rows per loader thread (8 k-groups per chunk)
  constexpr int RS = KC * 2;                                // bytes per image row and plane
  constexpr int TT = (BM / 32) * (BN / 32), TPW = TT / 8;  // 32x32 tiles; per wave
  constexpr int XPL = BM * RS, GPL = BN * RS;               // bytes per bf16 plane
  static_assert(TPW >= 1 && 2 * (BM + BN) <= 512 && (KC == 32 || KC == 64), "tile shape");
  __shared__ __attribute__((aligned(16))) char smem[3 * (XPL + GPL)];
  char* const xs = smem;
  char* const gs = smem + 3 * XPL;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int G = p.ngroup > 1 ? p.ngroup : 1;
  // XCD-aware order: blocks b and b + 8 share an XCD (and its L2), so the ntm x ntn tiles of one
  // (problem, slice) unit are blocks 8 j + (unit % 8): they read the same X and G rows together
  const int64_t units = (int64_t)G * p.zper;
  const int64_t hi = blockIdx.x >> 3;
  const int t = (int)(hi % (ntm * ntn));
  const int64_t u = (hi / (ntm * ntn)) * 8 + (blockIdx.x & 7);
  if (u >= units) return;  // the padding of the last 8-unit group
  const int tn = t % ntn, tm = t / ntn;
  const int pg = (int)(u % G);
  const int64_t z = u / G;
  float* slab = p.slab;
#pragma unroll
  for (int q = 1; q < GEMM_GMAX; ++q)
    if (pg == q) {
      p.A = p.gA[q];
      p.B = p.gB[q];
      slab = p.gslab[q];
      p.arow = p.garow[q];
    }
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = z * p.k_per_split;
  const int64_t kend = kbeg + p.k_per_split < p.K ? kbeg + p.k_per_split : p.K;
  const int nch = kend > kbeg ? (int)((kend - kbeg + KC - 1) / KC) : 0;
  const bool do_cs = p.colsum_row > 0 && tm == 0;

  // loaders: threads [0, 2 BM) read X (column quad q, RPT-row group kg of 8), [2 BM, 2 BM + 2 BN)
  // read G; each 16-B load covers 4 columns of one row. Threads past 2 (BM + BN) repeat G loads
  // they do not use: every load is unconditional, so hipcc's s_waitcnt bookkeeping waits for
  // exactly the chunk being stored.
  const bool isx = tid < 2 * BM, act = tid < 2 * (BM + BN);
  const int lt = isx ? tid : (tid - 2 * BM) % (2 * BN), W = isx ? BM : BN;
  const int q4 = lt % (W / 4), kg = lt / (W / 4);
  const float* const src = isx ? p.A + m0 + 4 * q4 : p.B + n0 + 4 * q4;
  const int64_t ld = isx ? p.lda : p.ldb;
  const bool mapped = isx && p.arow;
  // the row indices of row-mapped X (other threads and unmapped launches read G's bits, unused)
  const int32_t* const ip = p.arow ? p.arow : reinterpret_cast<const int32_t*>(p.B);
  char* const img = (isx ? xs : gs);
  const int pl = isx ? XPL : GPL;
  const bool isg = !isx && act;
  float4 va[RPT];
  int32_t xa[RPT], xb[RPT];  // row indices: chunks c even / odd
  float csum[4] = {0.f, 0.f, 0.f, 0.f};
  auto idx_load = [&](int c, int32_t (&xr)[RPT]) {  // the stored X rows of chunk c (c clamped: no branch)
    const int64_t k0 = kbeg + (int64_t)(c < nch ? c : nch - 1) * KC + RPT * kg;
#pragma unroll
    for (int j = 0; j < RPT; ++j) xr[j] = ip[k0 + j < kend ? k0 + j : kend - 1];
  };
  auto load = [&](int c, const int32_t (&xr)[RPT]) {  // rows past the slice: its last row (then 0)
#ifdef WGWS_PROBE_NOLOAD
    if (c >= 2) return;
#endif
    const int64_t k0 = kbeg + (int64_t)(c < nch ? c : nch - 1) * KC + RPT * kg;
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int64_t row = mapped ? (int64_t)xr[j] : (k0 + j < kend ? k0 + j : kend - 1);
      va[j] = *reinterpret_cast<const float4*>(src + row * ld);
    }
  };
  // zero the rows past the slice, split, one RPT-value run per plane (threads past 2 (BM + BN)
  // write the bits their G twin writes); no branch, so the waits stay exact
  const float csf = isg && do_cs ? 1.f : 0.f;
  auto store = [&](int c) {
    const int64_t k0 = kbeg + (int64_t)c * KC + RPT * kg;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float w[RPT];
#pragma unroll
      for (int j = 0; j < RPT; ++j) w[j] = k0 + j < kend ? va[j][e] : 0.f;
#pragma unroll
      for (int j = 0; j < RPT; ++j) csum[e] += w[j] * csf;
      const int col = 4 * q4 + e;
      IbSplit sp[RPT / 2];
#pragma unroll
      for (int j = 0; j < RPT / 2; ++j) sp[j] = ib_split2(w[2 * j], w[2 * j + 1]);
      if constexpr (RPT == 8) {
        char* dst = img + col * RS + 16 * (kg ^ wg_swz<KC>(col));
        *reinterpret_cast<u32x4*>(dst) = u32x4{sp[0].h, sp[1].h, sp[2].h, sp[3].h};
        *reinterpret_cast<u32x4*>(dst + pl) = u32x4{sp[0].m, sp[1].m, sp[2].m, sp[3].m};
        *reinterpret_cast<u32x4*>(dst + 2 * pl) = u32x4{sp[0].l, sp[1].l, sp[2].l, sp[3].l};
      } else {
        char* dst = img + col * RS + 16 * ((kg >> 1) ^ wg_swz<KC>(col)) + 8 * (kg & 1);
        *reinterpret_cast<u32x2*>(dst) = u32x2{sp[0].h, sp[1].h};
        *reinterpret_cast<u32x2*>(dst + pl) = u32x2{sp[0].m, sp[1].m};
        *reinterpret_cast<u32x2*>(dst + 2 * pl) = u32x2{sp[0].l, sp[1].l};
      }
    }
  };

  f32x16 acc[TPW];
#pragma unroll
  for (int t2 = 0; t2 < TPW; ++t2) acc[t2] = f32x16{};
  auto mfmas = [&]() {
#ifndef WGWS_PROBE_NOMFMA
#pragma unroll
    for (int t2 = 0; t2 < TPW; ++t2) {
      const int tt = wave + 8 * t2;
      const int mrow = (tt / (BN / 32)) * 32 + r, nrow = (tt % (BN / 32)) * 32 + r;
#pragma unroll
      for (int ks = 0; ks < KC / 16; ++ks) {
        const int ci = 2 * ks + h;
        const char* pa = xs + mrow * RS + 16 * (ci ^ wg_swz<KC>(mrow));
        const char* pb = gs + nrow * RS + 16 * (ci ^ wg_swz<KC>(nrow));
        const u32x4 a[3] = {*reinterpret_cast<const u32x4*>(pa), *reinterpret_cast<const u32x4*>(pa + XPL),
                            *reinterpret_cast<const u32x4*>(pa + 2 * XPL)};
        const u32x4 bb[3] = {*reinterpret_cast<const u32x4*>(pb), *reinterpret_cast<const u32x4*>(pb + GPL),
                             *reinterpret_cast<const u32x4*>(pb + 2 * GPL)};
        acc[t2] = mfma_split<NP>(a, bb, acc[t2]);
      }
    }
#endif
  };
  // step c: chunk c's registers into the images, then (their registers free) chunk c + 1's loads,
  // which fly during chunk c's MFMAs (and, at two workgroups per CU, the other one's). Issue order
  // idx(c + 2), load(c + 1): load(c + 1) waits for its indices (issued a step earlier) without
  // draining anything later; every load unconditional (past the last chunk: the last chunk again,
  // unused) and the loop body two steps without a branch (an odd chunk count gets a chunk of rows
  // past the slice: zeros)
  auto step = [&](int c, const int32_t (&xc)[RPT], int32_t (&xn)[RPT]) {
    if (c > 0) __syncthreads();  // every wave done with chunk c - 1's images
    store(c);
    __syncthreads();
    idx_load(c + 2, xn);
    load(c + 1, xc);
    mfmas();
  };
  if (nch > 0) {
    idx_load(0, xa);
    load(0, xa);
    idx_load(1, xb);
  }
  for (int c = 0; c < nch; c += 2) {
    step(c, xb, xa);
    step(c + 1, xa, xb);
  }
  // the slab of this slice: acc[t] register i = dW[m0 + 32 (tt / (BN / 32)) + (i & 3) + 8 (i >> 2) + 4 h]
  //                                               [n0 + 32 (tt % (BN / 32)) + r]
  float* sl = slab + z * (p.slab_stride ? p.slab_stride : p.M * p.N);
#pragma unroll
  for (int t2 = 0; t2 < TPW; ++t2) {
    const int tt = wave + 8 * t2;
    const int64_t mb = m0 + (tt / (BN / 32)) * 32 + 4 * h, nb = n0 + (tt % (BN / 32)) * 32 + r;
#pragma unroll
    for (int i = 0; i < 16; ++i) sl[(mb + (i & 3) + 8 * (i >> 2)) * p.N + nb] = acc[t2][i];
  }
  if (do_cs) {  // the 8 row groups' partial sums of each column, in group order
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
    if (isg) {
#pragma unroll
      for (int e = 0; e < 4; ++e) red[kg * BN + 4 * q4 + e] = csum[e];
    }
    __syncthreads();
    if (tid < BN) {
      float s = red[tid];
      for (int q = 1; q < 8; ++q) s += red[q * BN + tid];
      sl[p.colsum_row * p.N + n0 + tid] = s;
    }
  }
}

// ---- weight gradients with the raw operands prefetched by LDS-DMA (round 6, A/B build only) -----
// Tried because wgrad_ws_kernel's loads land in registers one chunk ahead and a probe without its
// MFMAs still took 68 % of its time (loads + split + LDS stores). Measured slower (WGRAD_DMA=1,
// profiles/r06c_dw_dma_ab.txt: towers dW+db 240.5 -> 258.8 us, C3 step +0.03 ms): with the loads
// fully prefetched the 32-row chunks' two barriers and their split / MFMA phases, not the load
// latency, set the time. Kept behind WGRAD_DMA for A/B builds. The raw fp32 chunks of X and G
// (KC = 32 rows) are copied HBM -> LDS by
// global_load_lds_dwordx4 into a ring of WDM_NS staging buffers, WDM_NS chunks ahead, with no
// registers and no compiler-counted waits involved (one explicit vmcnt per chunk); each chunk is
// then split from LDS into the same bf16-plane images as wgrad_ws_kernel's 32-row form and fed to
// the same MFMAs in the same k order, so dW is bitwise wgrad_ws_kernel's (the column sums group
// their rows differently). Row-mapped X (the distinct-row towers): the slice's row indices are
// copied into LDS once before the loop. LDS (128 x 128 tile): 3 x 32 KB ring + 48 KB images.
constexpr int WDM_KC = 32, WDM_NS = 3;
constexpr int WDM_IDX_MAX = 4096;  // row-mapped slices up to this many rows (16 KB of indices)

template <int BM, int BN>
struct WdmShape {
  static constexpr int XST = WDM_KC * BM * 4, GST = WDM_KC * BN * 4;  // staged bytes per chunk
  static constexpr int STG = XST + GST;
  static constexpr int RS = WDM_KC * 2;                               // image row bytes per plane
  static constexpr int XPL = BM * RS, GPL = BN * RS;
  static constexpr int NXI = XST / 8192, NGI = GST / 8192;           // DMA instructions per wave per chunk
  static constexpr int ND = NXI + NGI;
  static constexpr int LDS = WDM_NS * STG + 3 * (XPL + GPL);
};

// 16 B per lane HBM -> LDS at dst + 16 lane (dst wave-uniform), counted in vmcnt only
__device__ __forceinline__ void wdm_dma16(const float* src, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
               : "memory");
}
__device__ __forceinline__ void wdm_dma4(const int32_t* src, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
               : "memory");
}
template <int N>
__device__ __forceinline__ void wdm_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt field");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else static_assert(N == 0, "add the vmcnt immediate");
}

template <int BM, int BN, int NP>
__global__ __launch_bounds__(512, 1) void wgrad_dma_kernel(GemmParams p, int ntm, int ntn) {
  using S = WdmShape<BM, BN>;
  constexpr int KC = WDM_KC, NS = WDM_NS, RPT = KC / 8, RS = S::RS;
  constexpr int TT = (BM / 32) * (BN / 32), TPW = TT / 8;
  constexpr int XPL = S::XPL, GPL = S::GPL;
  static_assert(TPW >= 1 && 2 * (BM + BN) <= 512 && S::NXI >= 1 && S::NGI >= 1, "tile shape");
  static_assert(S::LDS + 4 * WDM_IDX_MAX <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[S::LDS];
  __shared__ __attribute__((aligned(16))) int32_t idx_s[WDM_IDX_MAX];
  char* const stg = smem;                        // NS x [X: KC x BM fp32 | G: KC x BN fp32]
  char* const xs = smem + NS * S::STG;           // 3 planes of X^T [BM][KC]
  char* const gs = xs + 3 * XPL;                 // 3 planes of G^T [BN][KC]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int G = p.ngroup > 1 ? p.ngroup : 1;
  const int64_t units = (int64_t)G * p.zper;
  const int64_t hi = blockIdx.x >> 3;
  const int t = (int)(hi % (ntm * ntn));
  const int64_t u = (hi / (ntm * ntn)) * 8 + (blockIdx.x & 7);
  if (u >= units) return;
  const int tn = t % ntn, tm = t / ntn;
  const int pg = (int)(u % G);
  const int64_t z = u / G;
  float* slab = p.slab;
#pragma unroll
  for (int q = 1; q < GEMM_GMAX; ++q)
    if (pg == q) {
      p.A = p.gA[q];
      p.B = p.gB[q];
      slab = p.gslab[q];
      p.arow = p.garow[q];
    }
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = z * p.k_per_split;
  const int64_t kend = kbeg + p.k_per_split < p.K ? kbeg + p.k_per_split : p.K;
  const int nch = kend > kbeg ? (int)((kend - kbeg + KC - 1) / KC) : 0;
  const bool do_cs = p.colsum_row > 0 && tm == 0;
  const uint32_t lds_stg = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)stg);
  const bool mapped = p.arow != nullptr;

  // the slice's row indices (row-mapped X) into LDS once, then every wave waits and syncs
  if (mapped && nch > 0) {
    const uint32_t lds_idx = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) int32_t*)idx_s);
    const int nrow = (int)(kend - kbeg);
    for (int i0 = wave * 64; i0 < nrow; i0 += 8 * 64) {
      const int i = i0 + lane < nrow ? i0 + lane : nrow - 1;
      wdm_dma4(p.arow + kbeg + i, __builtin_amdgcn_readfirstlane(lds_idx + 4 * i0));
    }
    wdm_wait_vm<0>();
    __syncthreads();
  }
  // chunk cc (clamped to the last: unconsumed copies keep the count per chunk fixed) into stage s.
  // X instruction i of the chunk = rows i RPI .. of BM columns (RPI = 1024 / (4 BM) rows per 1 KB),
  // G the same with BN; wave w issues X instructions w NXI .. and G instructions w NGI ..
  auto dma_chunk = [&](int cc, int s) {
    const int64_t k0 = kbeg + (int64_t)(cc < nch ? cc : nch - 1) * KC;
    const uint32_t dst0 = lds_stg + (uint32_t)(s * S::STG);
#pragma unroll
    for (int q = 0; q < S::NXI; ++q) {
      const int i = wave * S::NXI + q;
      constexpr int LPR = BM / 4;  // lanes per row
      const int64_t k = k0 + i * (1024 / (4 * BM)) + lane / LPR;
      const int64_t kc = k < kend ? k : kend - 1;
      const int64_t row = mapped ? (int64_t)idx_s[kc - kbeg] : kc;
      wdm_dma16(p.A + row * p.lda + m0 + 4 * (lane % LPR), dst0 + (uint32_t)(i * 1024));
    }
#pragma unroll
    for (int q = 0; q < S::NGI; ++q) {
      const int i = wave * S::NGI + q;
      constexpr int LPR = BN / 4;
      const int64_t k = k0 + i * (1024 / (4 * BN)) + lane / LPR;
      const int64_t kc = k < kend ? k : kend - 1;
      wdm_dma16(p.B + kc * p.ldb + n0 + 4 * (lane % LPR), dst0 + (uint32_t)(S::XST + i * 1024));
    }
  };

  // split threads: [0, 2 BM) X (column quad q4, row group kg of RPT rows), [2 BM, 2 (BM + BN)) G
  const bool isx = tid < 2 * BM, act = tid < 2 * (BM + BN);
  const int lt = isx ? tid : (tid - 2 * BM) % (2 * BN), W = isx ? BM : BN;
  const int q4 = lt % (W / 4), kg = lt / (W / 4);
  char* const img = isx ? xs : gs;
  const int pl = isx ? XPL : GPL;
  const bool isg = !isx && act;
  const float csf = isg && do_cs ? 1.f : 0.f;
  float csum[4] = {0.f, 0.f, 0.f, 0.f};
  auto split = [&](int c) {
    if (!act) return;
    const int64_t k0 = kbeg + (int64_t)c * KC + RPT * kg;
    const char* src = stg + (c % NS) * S::STG + (isx ? 0 : S::XST) + (RPT * kg) * W * 4 + 16 * q4;
    f32x4 va[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) va[j] = *reinterpret_cast<const f32x4*>(src + j * W * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float w[RPT];
#pragma unroll
      for (int j = 0; j < RPT; ++j) w[j] = k0 + j < kend ? va[j][e] : 0.f;
#pragma unroll
      for (int j = 0; j < RPT; ++j) csum[e] += w[j] * csf;
      const int col = 4 * q4 + e;
      IbSplit sp[RPT / 2];
#pragma unroll
      for (int j = 0; j < RPT / 2; ++j) sp[j] = ib_split2(w[2 * j], w[2 * j + 1]);
      char* dst = img + col * RS + 16 * ((kg >> 1) ^ wg_swz<KC>(col)) + 8 * (kg & 1);
      *reinterpret_cast<u32x2*>(dst) = u32x2{sp[0].h, sp[1].h};
      *reinterpret_cast<u32x2*>(dst + pl) = u32x2{sp[0].m, sp[1].m};
      *reinterpret_cast<u32x2*>(dst + 2 * pl) = u32x2{sp[0].l, sp[1].l};
    }
  };

  f32x16 acc[TPW];
#pragma unroll
  for (int t2 = 0; t2 < TPW; ++t2) acc[t2] = f32x16{};
  auto mfmas = [&]() {
#pragma unroll
    for (int t2 = 0; t2 < TPW; ++t2) {
      const int tt = wave + 8 * t2;
      const int mrow = (tt / (BN / 32)) * 32 + r, nrow = (tt % (BN / 32)) * 32 + r;
#pragma unroll
      for (int ks = 0; ks < KC / 16; ++ks) {
        const int ci = 2 * ks + h;
        const char* pa = xs + mrow * RS + 16 * (ci ^ wg_swz<KC>(mrow));
        const char* pb = gs + nrow * RS + 16 * (ci ^ wg_swz<KC>(nrow));
        const u32x4 a[3] = {*reinterpret_cast<const u32x4*>(pa), *reinterpret_cast<const u32x4*>(pa + XPL),
                            *reinterpret_cast<const u32x4*>(pa + 2 * XPL)};
        const u32x4 bb[3] = {*reinterpret_cast<const u32x4*>(pb), *reinterpret_cast<const u32x4*>(pb + GPL),
                             *reinterpret_cast<const u32x4*>(pb + 2 * GPL)};
        acc[t2] = mfma_split<NP>(a, bb, acc[t2]);
      }
    }
  };

  if (nch > 0) {
#pragma unroll
    for (int s = 0; s < NS; ++s) dma_chunk(s, s);
    for (int c = 0; c < nch; ++c) {
      // this wave's copies of chunk c have landed (those of chunks c + 1 .. c + NS - 1 may fly),
      // then everyone's have, and every wave is done with the images of chunk c - 1
      wdm_wait_vm<(NS - 1) * S::ND>();
      __syncthreads();
      split(c);
      __syncthreads();           // the images of chunk c are complete; stage c % NS is free
      dma_chunk(c + NS, c % NS);  // (past the last chunk: the last again, never consumed)
      mfmas();
    }
    wdm_wait_vm<0>();  // the trailing copies land before the workgroup's LDS is released
  }
  // the slab of this slice: acc[t] register i = dW[m0 + 32 (tt / (BN / 32)) + (i & 3) + 8 (i >> 2) + 4 h]
  //                                               [n0 + 32 (tt % (BN / 32)) + r]
  float* sl = slab + z * (p.slab_stride ? p.slab_stride : p.M * p.N);
#pragma unroll
  for (int t2 = 0; t2 < TPW; ++t2) {
    const int tt = wave + 8 * t2;
    const int64_t mb = m0 + (tt / (BN / 32)) * 32 + 4 * h, nb = n0 + (tt % (BN / 32)) * 32 + r;
#pragma unroll
    for (int i = 0; i < 16; ++i) sl[(mb + (i & 3) + 8 * (i >> 2)) * p.N + nb] = acc[t2][i];
  }
  if (do_cs) {  // the 8 row groups' partial sums of each column, in group order
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
    if (isg) {
#pragma unroll
      for (int e = 0; e < 4; ++e) red[kg * BN + 4 * q4 + e] = csum[e];
    }
    __syncthreads();
    if (tid < BN) {
      float s2 = red[tid];
      for (int q = 1; q < 8; ++q) s2 += red[q * BN + tid];
      sl[p.colsum_row * p.N + n0 + tid] = s2;
    }
  }
}

bool wgrad_ws_ok(const GemmParams& p) {
  if (!(p.prec == 6 || p.prec == 9) || p.colsum_row != p.M || p.M <= 0 || p.K < 8192) return false;
  if (p.M % 64 || p.N % 64 || (p.M % 128 && p.N % 128)) return false;  // 128 x 128, 128 x 64 or 64 x 128 tiles
  if (p.lda % 4 || p.ldb % 4) return false;                               // 16-B row loads
  const int G = p.ngroup > 1 ? p.ngroup : 1;
  for (int g = 0; g < G; ++g) {
    const float* a = p.ngroup > 1 ? p.gA[g] : p.A;
    const float* b = p.ngroup > 1 ? p.gB[g] : p.B;
    if (reinterpret_cast<uintptr_t>(a) % 16 || reinterpret_cast<uintptr_t>(b) % 16) return false;
  }
  return p.M <= (1 << 16) && p.N <= (1 << 16);
}

#ifndef WGRAD_DMA
#define WGRAD_DMA 0  // 1: the LDS-DMA weight-gradient kernel (an A/B build; measured slower, see its comment)
#endif
#ifndef WGWS_WGS
#define WGWS_WGS 256  // workgroups per problem the slice count aims at
#endif
#ifndef WGWS_MINK
#define WGWS_MINK 512  // fewest rows per slice (256: small layers +5 us)
#endif
// Rows per K slice: a multiple of 128 (an even chunk count) giving ~WGWS_WGS workgroups per problem
// with >= WGWS_MINK rows each, never fewer rows than kps_min (the slab workspace's slice count). A
// function of one problem's shape only, so a grouped launch sums each problem exactly as its own.
int64_t wgrad_ws_kps(const GemmParams& p, int64_t kps_min) {
  const int64_t tiles = (p.M / (p.M % 128 == 0 ? 128 : 64)) * (p.N / (p.N % 128 == 0 ? 128 : 64));
  int64_t s = (WGWS_WGS + tiles / 2) / tiles;
  const int64_t smax = (p.K + WGWS_MINK - 1) / WGWS_MINK;
  if (s > smax) s = smax;
  if (s < 1) s = 1;
  int64_t kps = ((p.K + s - 1) / s + 127) / 128 * 128;
  const int64_t lo = (kps_min + 127) / 128 * 128;
  return kps > lo ? kps : lo;
}

// p: the split-mode wgrad parameters (slab, slab_stride, k_per_split a multiple of 64, colsum_row)
void wgrad_ws_dispatch(const GemmParams& p, int64_t slices, hipStream_t st) {
  const int G = p.ngroup > 1 ? p.ngroup : 1;
  GemmParams q = p;
  if (p.ngroup > 1) {
    q.A = p.gA[0];
    q.B = p.gB[0];
    q.slab = p.gslab[0];
    q.arow = p.garow[0];
  }
  const int bm = p.M % 128 == 0 ? 128 : 64, bn = p.N % 128 == 0 ? 128 : 64;
  const int ntm = (int)(p.M / bm), ntn = (int)(p.N / bn);
  q.zper = slices;
  const dim3 grid((unsigned)((G * slices + 7) / 8 * 8 * ntm * ntn));
  // the LDS-DMA kernel by default: 16-B aligned rows and columns (every tile's rows are 16-B runs),
  // row-mapped slices whose indices fit its LDS table
  bool dma = WGRAD_DMA && p.lda % 4 == 0 && p.ldb % 4 == 0 && (!p.arow || p.k_per_split <= WDM_IDX_MAX);
  for (int g = 0; g < G && dma; ++g) {
    const float* a = p.ngroup > 1 ? p.gA[g] : p.A;
    const float* b = p.ngroup > 1 ? p.gB[g] : p.B;
    dma = reinterpret_cast<uintptr_t>(a) % 16 == 0 && reinterpret_cast<uintptr_t>(b) % 16 == 0;
  }
  if (dma) {
#define RS_WDM(BM_, BN_)                                                                                \
  if (p.prec == 6) hipLaunchKernelGGL((wgrad_dma_kernel<BM_, BN_, 6>), grid, dim3(512), 0, st, q, ntm, ntn); \
  else hipLaunchKernelGGL((wgrad_dma_kernel<BM_, BN_, 9>), grid, dim3(512), 0, st, q, ntm, ntn);
    if (bm == 128 && bn == 128) { RS_WDM(128, 128) }
    else if (bm == 128) { RS_WDM(128, 64) }
    else { RS_WDM(64, 128) }
#undef RS_WDM
    return;
  }
#define RS_WGWS(BM_, BN_)                                                                              \
  if (p.prec == 6)                                                                                     \
    hipLaunchKernelGGL((wgrad_ws_kernel<BM_, BN_, 6, WGWS_KC, WGWS_OCC>), grid, dim3(512), 0, st, q, ntm, ntn); \
  else hipLaunchKernelGGL((wgrad_ws_kernel<BM_, BN_, 9, WGWS_KC, WGWS_OCC>), grid, dim3(512), 0, st, q, ntm, ntn);
  if (bm == 128 && bn == 128) { RS_WGWS(128, 128) }
  else if (bm == 128) { RS_WGWS(128, 64) }
  else { RS_WGWS(64, 128) }
#undef RS_WGWS
}

}  // namespace rs
