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
#include "common.hpp"
#include "split.hpp"
#include "gemm.hpp"

namespace rs {

constexpr int WS_THREADS = 512;
#ifndef WS_OCC
#define WS_OCC 1  // workgroups per CU (2: 64-column slices, 32-k register chunks, 128 VGPRs)
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
static int ws_slice(int64_t K, int64_t N, bool masked) {
  int nw = K <= 64 ? 128 : (K == 128 ? 128 : 64);
  if ((masked && K >= 128) || WS_OCC > 1) nw = 64;
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
