// gemm_skinny.hip — skinny split GEMM for the Dense layers (its own translation unit: the
// 40 template instances compile in parallel with gemm.hip). Dispatched from gemm.hip.
#include "common.hpp"
#include "split.hpp"
#include "gemm.hpp"

#include <cstdlib>

namespace rs {

// ---- skinny GEMM for the Dense layers (precision 6 / 9) ---------------------------------------
// C[M, N] = epi(A[M, K] op(B)) with A row-major (the activations / the output gradient), N <= 256 and
// K <= 256 multiples of 16 / 32, M large: the towers' and the deep net's forward (op(B) = W [K, N])
// and dX (op(B) = W^T, W [N', K'] given as B [N][K] with trans_b). gemm_x3_kernel's 64 x 64 tiles
// spend a barrier and an LDS staging pass per 16-k chunk on 6 x 32 cycles of MFMA; here a 256-thread
// workgroup (two per CU, at different phases) owns 128 rows x ALL N columns: each wave 32 rows (two 16-row A tiles read straight from
// HBM as the 16x16x32 A operand, split into bf16 planes in registers, the next 32-k chunk prefetched)
// against the weight chunk [32 k x N] staged once per workgroup into LDS as split planes in
// fragment order (conflict-free ds_read_b128; one buffer, two barriers per chunk). Per chunk a
// wave issues 2 N / 16 x NP MFMAs between barriers (192 for N = 256 at precision 6). The epilogue
// quad-transposes each 16 x 16 accumulator so a lane stores 4 consecutive columns of one row
// (f32x4 loads of bias / mask / addend / C, f32x4 stores). Same split products as gemm_x3_kernel
// (the k order inside an MFMA differs), fp32 accumulation.
template <int CTRL>
__device__ __forceinline__ float gx_dpp_quad(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
constexpr int SK_KC = 32;      // k per chunk

// NW = 4: 128 rows per workgroup, one weight buffer, two workgroups per CU at different phases;
// NW = 8 (the 256-column forward, whose 4-wave staging registers would spill): 256 rows, a double
// buffer, one workgroup per CU
// EK: the epilogue's operands (skinny_ek): 1 = bias / activation only (the forward), 2 = the ReLU
// mask only (dX), 0 = any combination
// IMG: the weight chunks come pre-split from p.bimg (three 16-B loads per fragment slot, stored to
// LDS as they are) instead of eight fp32 loads and four splits per slot in every workgroup
template <int NT, bool TB, int NP, int NW, int EK, bool IMG>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void gemm_skinny_kernel(GemmParams p) {
  constexpr int NTH = 64 * NW, NBUF = NW == 8 ? 2 : 1, BUFB = 3 * NT * 1024;
  __shared__ __attribute__((aligned(16))) char smem[NBUF * BUFB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i16 = lane & 15, g = lane >> 4;
  const int pg = (int)blockIdx.y;  // problem of a grouped launch (constant-index selection)
#pragma unroll
  for (int i = 1; i < GEMM_GMAX; ++i)
    if (pg == i) {
      p.A = p.gA[i];
      p.B = p.gB[i];
      p.C = p.gC[i];
      p.bias = p.gbias[i];
      p.mask = p.gmask[i];
      p.bimg = p.gbimg[i];
    }
  const int nch = (int)(p.K / SK_KC);
  // row blocks of 32 NW rows, dealt round-robin: the workgroup's next block's first A and weight
  // chunk are loaded before this block's epilogue, so its stores overlap those loads (a launch of
  // one block per workgroup runs its workgroups in lockstep: load, compute and store phases of the
  // whole chip aligned)
  const int64_t nblk = (p.M + 32 * NW - 1) / (32 * NW);
  int64_t m0 = (int64_t)blockIdx.x * (32 * NW) + 32 * wave;  // the wave's first row

  // weight chunk c -> registers: fragment slot s = t 64 + L (L = 16 g' + n') of tile t needs
  // op(B)[k0 + 8 g' + j][16 t + n'], j < 8
  constexpr int NSLOT = NT * 64;
  constexpr int SPT = (NSLOT + NTH - 1) / NTH;  // slots per thread
  f32x4 wr[IMG ? 1 : SPT][2];
  u32x4 wi[IMG ? SPT : 1][3];
  auto wload = [&](int c) {
    const int64_t k0 = (int64_t)c * SK_KC;
    if constexpr (IMG) {
#pragma unroll
      for (int u = 0; u < SPT; ++u) {
        const int s = tid + NTH * u;
        if (s < NSLOT) {
          const u32x4* src = reinterpret_cast<const u32x4*>(p.bimg + ((int64_t)c * NT + (s >> 6)) * 3072) + (s & 63);
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) wi[u][pl] = src[64 * pl];
        }
      }
      return;
    }
#pragma unroll
    for (int u = 0; u < SPT; ++u) {
      const int s = tid + NTH * u;
      const int t = s >> 6, L = s & 63, gg = L >> 4, nn = L & 15;
      const int64_t n = 16 * t + nn, kb = k0 + 8 * gg;
      if (s < NSLOT) {
        if (TB) {  // B [N][K]: 8 consecutive k of row n
          const float* src = p.B + n * p.ldb + kb;
          wr[u][0] = *reinterpret_cast<const f32x4*>(src);
          wr[u][1] = *reinterpret_cast<const f32x4*>(src + 4);
        } else {  // B [K][N]: column n, rows kb .. kb + 7
          const float* src = p.B + kb * p.ldb + n;
#pragma unroll
          for (int j = 0; j < 8; ++j) wr[u][j >> 2][j & 3] = src[j * p.ldb];
        }
      }
    }
  };
  auto wstore = [&](int buf) {
    char* base = smem + buf * BUFB;
    if constexpr (IMG) {
#pragma unroll
      for (int u = 0; u < SPT; ++u) {
        const int s = tid + NTH * u;
        if (s < NSLOT) {
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<u32x4*>(base + pl * NT * 1024 + 16 * s) = wi[u][pl];
        }
      }
      return;
    }
#pragma unroll
    for (int u = 0; u < SPT; ++u) {
      const int s = tid + NTH * u;
      if (s < NSLOT) {
        const IbSplit x0 = ib_split2(wr[u][0][0], wr[u][0][1]), x1 = ib_split2(wr[u][0][2], wr[u][0][3]),
                      x2 = ib_split2(wr[u][1][0], wr[u][1][1]), x3 = ib_split2(wr[u][1][2], wr[u][1][3]);
        *reinterpret_cast<u32x4*>(base + 16 * s) = u32x4{x0.h, x1.h, x2.h, x3.h};
        *reinterpret_cast<u32x4*>(base + NT * 1024 + 16 * s) = u32x4{x0.m, x1.m, x2.m, x3.m};
        *reinterpret_cast<u32x4*>(base + 2 * NT * 1024 + 16 * s) = u32x4{x0.l, x1.l, x2.l, x3.l};
      }
    }
  };
  // A rows of the wave: tile rt, lane (i16, g) -> row m0 + 16 rt + i16, k0 + 8 g .. + 7 (rows past M
  // read row M - 1; never stored)
  f32x4 ar[2][2];
  auto aload = [&](int c, int64_t mb) {
    const int64_t k0 = (int64_t)c * SK_KC + 8 * g;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      int64_t row = mb + 16 * rt + i16;
      if (row >= p.M) row = p.M - 1;
      const float* src = p.A + row * p.lda + k0;
      ar[rt][0] = *reinterpret_cast<const f32x4*>(src);
      ar[rt][1] = *reinterpret_cast<const f32x4*>(src + 4);
    }
  };

  f32x4 acc[2][NT];
  wload(0);
  aload(0, m0);
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
  m0 = blk * (32 * NW) + 32 * wave;
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (blk != (int64_t)blockIdx.x) __syncthreads();  // every wave done with the last block's weight chunks
  if (NBUF == 2) {
    wstore(0);
    __syncthreads();
  }
  for (int c = 0; c < nch; ++c) {
    if (NBUF == 1) {
      // one weight buffer: wait until every wave has read chunk c - 1, store chunk c (loaded during
      // chunk c - 1's MFMAs), publish it
      if (c > 0) __syncthreads();
      wstore(0);
      __syncthreads();
    }
    u32x4 ap[2][3];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const IbSplit x0 = ib_split2(ar[rt][0][0], ar[rt][0][1]), x1 = ib_split2(ar[rt][0][2], ar[rt][0][3]),
                    x2 = ib_split2(ar[rt][1][0], ar[rt][1][1]), x3 = ib_split2(ar[rt][1][2], ar[rt][1][3]);
      ap[rt][0] = u32x4{x0.h, x1.h, x2.h, x3.h};
      ap[rt][1] = u32x4{x0.m, x1.m, x2.m, x3.m};
      ap[rt][2] = u32x4{x0.l, x1.l, x2.l, x3.l};
    }
    const bool more = c + 1 < nch;
    if (more) {
      wload(c + 1);
      aload(c + 1, m0);
    }
    const char* base = smem + (NBUF == 2 ? (c & 1) : 0) * BUFB;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      u32x4 bp[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) bp[pl] = *reinterpret_cast<const u32x4*>(base + pl * NT * 1024 + 1024 * t + 16 * lane);
      const u32x4* const aa[2] = {ap[0], ap[1]};
      const u32x4* const bb[2] = {bp, bp};
      f32x4* const cc[2] = {&acc[0][t], &acc[1][t]};
      mfma16_split_n<NP, 2>(aa, bb, cc);
    }
    if (NBUF == 2) {
      if (more) wstore((c + 1) & 1);
      __syncthreads();
    }
  }
  if (blk + gridDim.x < nblk) {  // the next block's first chunk, in flight during the epilogue
    wload(0);
    aload(0, (blk + gridDim.x) * (32 * NW) + 32 * wave);
  }

  // epilogue: quad transpose (lane & 3 <-> register): lane a of quad q then holds row 4 g + a of the
  // tile, columns 16 t + 4 q .. + 3. The epilogue operands of a group of tiles are loaded before any
  // of them is used (EK 1: the bias of all NT tiles once; EK 2: the mask of a row tile's NT tiles;
  // EK 0: every operand, 4 tiles at a time), so a wave waits on memory once per group instead of
  // once per tile (a round trip per tile left the forward ~2x its MFMA time).
  const int a4 = i16 & 3, q4 = i16 >> 2;
  constexpr int EG = EK == 0 ? (NT < 4 ? NT : 4) : NT;  // tiles per load group (divides NT)
  static_assert(NT % EG == 0, "load groups must tile NT");
  f32x4 bv[EK == 1 ? NT : 1];
  if constexpr (EK == 1) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
      bv[t] = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + 16 * t + 4 * q4) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    const int64_t row = m0 + 16 * rt + 4 * g + a4;
    const bool live = row < p.M;
    const int64_t rowc = live ? row : p.M - 1;
#pragma unroll
    for (int t0 = 0; t0 < NT; t0 += EG) {
      f32x4 mv[EG], av[EG], cv[EG], bg[EG];
      if constexpr (EK == 2) {
#pragma unroll
        for (int j = 0; j < EG; ++j) mv[j] = *reinterpret_cast<const f32x4*>(p.mask + rowc * p.ldm + 16 * (t0 + j) + 4 * q4);
      }
      if constexpr (EK == 0) {
#pragma unroll
        for (int j = 0; j < EG; ++j) {
          const int64_t col = 16 * (t0 + j) + 4 * q4;
          bg[j] = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + col) : f32x4{0.f, 0.f, 0.f, 0.f};
          mv[j] = p.mask ? *reinterpret_cast<const f32x4*>(p.mask + rowc * p.ldm + col) : f32x4{1.f, 1.f, 1.f, 1.f};
          av[j] = p.addend ? *reinterpret_cast<const f32x4*>(p.addend + rowc * p.ldadd + col) : f32x4{0.f, 0.f, 0.f, 0.f};
          cv[j] = p.beta != 0.f ? *reinterpret_cast<const f32x4*>(p.C + rowc * p.ldc + col) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
#pragma unroll
      for (int j = 0; j < EG; ++j) {
        const int t = t0 + j;
        float x0 = acc[rt][t][0], x1 = acc[rt][t][1], x2 = acc[rt][t][2], x3 = acc[rt][t][3];
        const float t0v = gx_dpp_quad<0x4E>(x0), t1v = gx_dpp_quad<0x4E>(x1), t2v = gx_dpp_quad<0x4E>(x2),
                    t3v = gx_dpp_quad<0x4E>(x3);
        if (a4 & 2) { x0 = t2v; x1 = t3v; } else { x2 = t0v; x3 = t1v; }
        const float u0 = gx_dpp_quad<0xB1>(x0), u1 = gx_dpp_quad<0xB1>(x1), u2 = gx_dpp_quad<0xB1>(x2),
                    u3 = gx_dpp_quad<0xB1>(x3);
        if (a4 & 1) { x0 = u1; x2 = u3; } else { x1 = u0; x3 = u2; }
        const int64_t col = 16 * t + 4 * q4;
        f32x4 v = {x0, x1, x2, x3};
        if constexpr (EK == 1) v += bv[t];
        if constexpr (EK == 0) v += bg[j];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float y = v[e];
          if constexpr (EK != 2) {
            if (p.act == RS_ACT_RELU) y = fmaxf(y, 0.f);
          }
          if constexpr (EK == 2) {
            if (!(mv[j][e] > 0.f)) y = 0.f;
          }
          if constexpr (EK == 0) {
            if (p.mask && !(mv[j][e] > 0.f)) y = 0.f;
            if (p.addend) y += av[j][e];
            if (p.beta != 0.f) y += p.beta * cv[j][e];
          }
          v[e] = y;
        }
        if (live) {
          // SKINNY_NT_STORE (build-time experiment switch): non-temporal output stores
#ifdef SKINNY_NT_STORE
          __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p.C + row * p.ldc + col));
#else
          *reinterpret_cast<f32x4*>(p.C + row * p.ldc + col) = v;
#endif
        }
      }
    }
  }
  }  // row blocks
}

// the skinny kernel's envelope: split precision, no trans_a, no split-K / cross epilogue, N one of the
// compiled widths, K a multiple of 32 up to 256, every row pointer and leading dim 16-B aligned
bool skinny_ok(int ta, int tb, const GemmParams& p) {
  if (ta || p.epi != 0 || !(p.prec == 6 || p.prec == 9) || p.ones_row1) return false;
  const int nt = (int)(p.N / 16);   // the compiled widths: 32, 64, 128, 192, 256 columns
  if (p.N % 16 || !(nt == 2 || nt == 4 || nt == 8 || nt == 12 || nt == 16)) return false;
  if (p.K % SK_KC || p.K == 0 || p.K > 256) return false;
  // at least ~one workgroup per CU (128 rows each, 256 for the 256-column forward): a small batch
  // (C2's 4096 rows: 16-32 workgroups) runs faster on the 64 x 64 tiles (skinny 44 vs 12 us)
  const int64_t G = p.ngroup > 1 ? p.ngroup : 1;
  const int64_t rows_wg = (nt == 16 && !tb) ? 256 : 128;
  if (ceil_div(p.M, rows_wg) * G < 256) return false;
  // a wide masked output (the dX of a 256-wide ReLU layer) reads its mask in 64-B row pieces per
  // 16-column tile: measured slower than the 64 x 64 tiles there (C3 256 -> 128 dX 122 -> 140 us)
  static const bool wide_mask = exp_env("RS_SKINNY_WIDE_MASK") != nullptr;   // experiment switch
  if (p.mask && p.N > 128 && !wide_mask) return false;
  if (p.lda % 4 || p.ldb % 4 || p.ldc % 4 || (p.mask && p.ldm % 4) || (p.addend && p.ldadd % 4)) return false;
  for (int i = 0; i < G; ++i) {
    const float* A = G > 1 ? p.gA[i] : p.A;
    const float* C = G > 1 ? p.gC[i] : p.C;
    const float* bi = G > 1 ? p.gbias[i] : p.bias;
    const float* mk = G > 1 ? p.gmask[i] : p.mask;
    if (!aligned16(A) || !aligned16(C) || (bi && !aligned16(bi)) || (mk && !aligned16(mk))) return false;
  }
  return !p.addend || aligned16(p.addend);
}

// the epilogue variant of a launch (every problem of a grouped launch has the same operand set)
static int skinny_ek(const GemmParams& q) {
  if (!q.mask && !q.addend && q.beta == 0.f) return 1;
  if (q.mask && !q.bias && !q.addend && q.beta == 0.f && q.act != RS_ACT_RELU) return 2;
  return 0;
}

// RS_SKINNY_BLOCKS (A/B switch): row blocks per workgroup (default 1: one block each)
static int64_t skinny_grid(int64_t nblk, int G) {
  static const int64_t per = [] {
    const char* e = exp_env("RS_SKINNY_BLOCKS");
    return e && atoi(e) > 0 ? (int64_t)atoi(e) : (int64_t)1;
  }();
  int64_t gx = ceil_div(nblk, per);
  return gx > 0 ? gx : 1;
}

template <int NT, bool TB, int NP, int EK, bool IMG = false>
static void skinny_launch_ek(const GemmParams& q, int G, hipStream_t st) {
  if constexpr (NT == 16 && !TB)
    hipLaunchKernelGGL((gemm_skinny_kernel<NT, TB, NP, 8, EK, IMG>),
                       dim3((unsigned)skinny_grid(ceil_div(q.M, 256), G), (unsigned)G), dim3(512), 0, st, q);
  else
    hipLaunchKernelGGL((gemm_skinny_kernel<NT, TB, NP, 4, EK, IMG>),
                       dim3((unsigned)skinny_grid(ceil_div(q.M, 128), G), (unsigned)G), dim3(256), 0, st, q);
}

template <int NT, bool TB, int NP>
static void skinny_launch_nt(const GemmParams& q, int G, hipStream_t st) {
  static const bool generic = exp_env("RS_SKINNY_EPI_GENERIC") != nullptr;   // A/B switch (timing)
  const int ek = generic ? 0 : skinny_ek(q);
  // the forward (no trans_b) runs EK 1, dX (trans_b) EK 2; anything else the general epilogue;
  // weight images (precision 6) on those two
  if constexpr (!TB) {
    if (ek == 1) {
      if constexpr (NP == 6)
        if (q.bimg) return skinny_launch_ek<NT, TB, NP, 1, true>(q, G, st);
      return skinny_launch_ek<NT, TB, NP, 1>(q, G, st);
    }
  } else {
    if (ek == 2) {
      if constexpr (NP == 6)
        if (q.bimg) return skinny_launch_ek<NT, TB, NP, 2, true>(q, G, st);
      return skinny_launch_ek<NT, TB, NP, 2>(q, G, st);
    }
  }
  skinny_launch_ek<NT, TB, NP, 0>(q, G, st);
}

template <bool TB, int NP>
static void skinny_launch(const GemmParams& p, hipStream_t st) {
  const int G = p.ngroup > 1 ? p.ngroup : 1;
  GemmParams q = p;
  if (G > 1) {  // slot 0 of the group arrays is the kernel's default problem
    q.A = p.gA[0];
    q.B = p.gB[0];
    q.C = p.gC[0];
    q.bias = p.gbias[0];
    q.mask = p.gmask[0];
    q.bimg = p.gbimg[0];
  }
  switch (p.N / 16) {
    case 2: skinny_launch_nt<2, TB, NP>(q, G, st); break;
    case 4: skinny_launch_nt<4, TB, NP>(q, G, st); break;
    case 8: skinny_launch_nt<8, TB, NP>(q, G, st); break;
    case 12: skinny_launch_nt<12, TB, NP>(q, G, st); break;
    case 16: skinny_launch_nt<16, TB, NP>(q, G, st); break;
    default: break;
  }
}

void skinny_dispatch(int tb, const GemmParams& p, hipStream_t st) {
  if (tb) { if (p.prec == 6) skinny_launch<true, 6>(p, st); else skinny_launch<true, 9>(p, st); }
  else { if (p.prec == 6) skinny_launch<false, 6>(p, st); else skinny_launch<false, 9>(p, st); }
}

}  // namespace rs
