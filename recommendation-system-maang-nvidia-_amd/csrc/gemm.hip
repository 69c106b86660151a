// gemm.hip — fp32 MFMA GEMM for the tower / deep-net Dense layers (fwd, dX, dW).
//
// Replaces keras.layers.Dense MatMul+BiasAdd+ReLU (src/models.py:26-29,76-77) and its two
// gradient GEMMs. gfx950 has no xf32/TF32: v_mfma_f32_32x32x2_f32 is exact fp32 (a k-ordered
// fmaf chain) at the fp32 vector rate (157.3 TF/s spec), so these GEMMs are MFMA-bound for
// every shape on the path (K <= 256, N <= 256, M = batch up to 65536+).
//
// Tile: BM x BN per 256-thread workgroup (4 waves, WM x WN), BK = 32 reduction chunk staged
// through LDS, double-buffered with register prefetch (one barrier per chunk). Both operands
// are stored "k-contiguous" when their global layout allows it (read with ds_read_b128, row
// stride BK+4 floats = conflict-free for the b128 lane groups) and "m/n-contiguous" otherwise
// (read with 4 x ds_read_b32, consecutive lanes on consecutive banks). The MFMA's two k slots
// (lane halves) take k = kk+t and kk+4+t, t = 0..3: the same permutation on A and B, so each
// lane reads 4 consecutive k with one b128.
#include "common.hpp"
#include "split.hpp"
#include "gemm.hpp"

#include <algorithm>
#include <cstdlib>

namespace rs {



// XCD-aware tile order. Workgroups are dealt round-robin over the 8 XCDs (linear block id L on
// XCD L % 8; MI355X_MICROARCH.md 'Workgroup dispatch'), and each XCD has its own L2. The map
// gives every XCD a contiguous range of tile indices (a bijection for any grid size) and walks a
// range in groups of GX_GM row tiles, all column tiles of a group before the next: the ~64
// workgroups an XCD holds at once then cover ~8 A row tiles and ~8 B column tiles, which they
// share through the XCD's L2, instead of ~37 A tiles spread over all 8 L2s.
constexpr int GX_GM = 8;
struct GxTile {
  int64_t m, n, z;  // row tile, column tile, K slice
};
// tile t of the grouped order over an nby x nbx tile grid: groups of GX_GM row tiles, all column
// tiles of a group before the next
__device__ __forceinline__ GxTile gx_map(int64_t t, int64_t nbx, int64_t nby) {
  GxTile g;
  g.z = 0;
  const int64_t grp = t / (GX_GM * nbx);
  const int64_t mf = grp * GX_GM;
  const int64_t gsz = (nby - mf) < GX_GM ? (nby - mf) : GX_GM;
  const int64_t w = t - grp * GX_GM * nbx;
  g.m = mf + w % gsz;
  g.n = w / gsz;
  return g;
}
// linear block id -> an index contiguous per XCD (a bijection on [0, T))
__device__ __forceinline__ int64_t gx_xcd(int64_t L, int64_t T) {
  const int64_t q = T >> 3, r = T & 7, xcd = L & 7;
  return xcd * q + (xcd < r ? xcd : r) + (L >> 3);
}
__device__ __forceinline__ GxTile gx_tile() {
  const int64_t nbx = gridDim.x, nby = gridDim.y;
#ifdef RS_GEMM_NO_XCD_MAP
  return GxTile{(int64_t)blockIdx.y, (int64_t)blockIdx.x, (int64_t)blockIdx.z};
#endif
  const int64_t T = nbx * nby * gridDim.z;
  const int64_t L = ((int64_t)blockIdx.z * nby + blockIdx.y) * nbx + blockIdx.x;
  const int64_t t = gx_xcd(L, T);
  const int64_t per = nbx * nby;
  const int64_t z = t / per;
  GxTile g = gx_map(t - z * per, nbx, nby);
  g.z = z;
  return g;
}

// the tile of this workgroup; for a grouped launch also switches p to its problem (constant
// indices only, so the copy of p stays in registers)
__device__ __forceinline__ GxTile gemm_tile(GemmParams& p) {
  GxTile t = gx_tile();
  if (p.ngroup > 1) {
    const int g = (int)(t.z / p.zper);
    t.z -= (int64_t)g * p.zper;
#pragma unroll
    for (int i = 1; i < GEMM_GMAX; ++i)
      if (g == i) {
        p.A = p.gA[i];
        p.B = p.gB[i];
        p.C = p.gC[i];
        p.bias = p.gbias[i];
        p.mask = p.gmask[i];
        p.slab = p.gslab[i];
        p.arow = p.garow[i];
      }
  }
  return t;
}

// Epilogue shared by the f32 and the split kernels (same accumulator layout): bias, DCN-v2
// cross update, ReLU, mask, addend, beta * C; split mode writes the K-slice slab instead.
template <int TM, int TN, bool SPLIT>
__device__ __forceinline__ void gemm_epilogue(const GemmParams& p, f32x16 (&acc)[TM][TN], int64_t mw0, int64_t nw0,
                                              int half, int l32, int64_t zs) {
#pragma clang loop unroll(full)
  for (int i = 0; i < TM; ++i) {
#pragma clang loop unroll(full)
    for (int j = 0; j < TN; ++j) {
      const int64_t col = nw0 + j * 32 + l32;
      if (col >= p.N) continue;
      float bv = 0.f;
      if (!SPLIT && p.bias) bv = p.bias[col];
      if constexpr (!SPLIT && TM * TN <= 4) {
        if (p.epi != 1) {
          // small tiles, no cross update: each operand of the 16 values (mask, addend, C for beta)
          // is loaded for all of them before any is used (rows clamped into [0, M); a
          // branch-guarded load per value made hipcc wait on each one); same arithmetic
          // (two batches of 8 values: half the registers of one batch of 16)
#pragma clang loop unroll(full)
          for (int hb = 0; hb < 16; hb += 8) {
            float mv[8], av[8], cv[8];
            if (p.mask) {
#pragma clang loop unroll(full)
              for (int r = 0; r < 8; ++r) {
                const int64_t row = mw0 + i * 32 + acc_row(hb + r, half);
                mv[r] = p.mask[(row < p.M ? row : p.M - 1) * p.ldm + col];
              }
            }
            if (p.addend) {
#pragma clang loop unroll(full)
              for (int r = 0; r < 8; ++r) {
                const int64_t row = mw0 + i * 32 + acc_row(hb + r, half);
                av[r] = p.addend[(row < p.M ? row : p.M - 1) * p.ldadd + col];
              }
            }
            if (p.beta != 0.f) {
#pragma clang loop unroll(full)
              for (int r = 0; r < 8; ++r) {
                const int64_t row = mw0 + i * 32 + acc_row(hb + r, half);
                cv[r] = p.C[(row < p.M ? row : p.M - 1) * p.ldc + col];
              }
            }
#pragma clang loop unroll(full)
            for (int r = 0; r < 8; ++r) {
              const int64_t row = mw0 + i * 32 + acc_row(hb + r, half);
              if (row >= p.M) continue;
              float v = acc[i][j][hb + r] + bv;
              if (p.act == RS_ACT_RELU) v = fmaxf(v, 0.f);
              if (p.mask && !(mv[r] > 0.f)) v = 0.f;
              if (p.addend) v += av[r];
              if (p.beta != 0.f) v += p.beta * cv[r];
              p.C[row * p.ldc + col] = v;
            }
          }
          continue;
        }
      }
#pragma clang loop unroll(full)
      for (int r = 0; r < 16; ++r) {
        const int64_t row = mw0 + i * 32 + acc_row(r, half);
        if (row >= p.M) continue;
        float v = acc[i][j][r];
        if (SPLIT) {
          p.slab[zs * (p.slab_stride ? p.slab_stride : p.M * p.N) + row * p.N + col] = v;
        } else {
          v += bv;
          if (p.epi == 1) {
            const int64_t xo = row * p.ldx + col;
            p.aux[xo] = v;
            v = p.x0[xo] * v + p.xres[xo];
          }
          if (p.act == RS_ACT_RELU) v = fmaxf(v, 0.f);
          if (p.mask && !(p.mask[row * p.ldm + col] > 0.f)) v = 0.f;
          if (p.addend) v += p.addend[row * p.ldadd + col];
          float* cp = p.C + row * p.ldc + col;
          if (p.beta != 0.f) v += p.beta * (*cp);
          *cp = v;
        }
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, bool TA, bool TB, bool SPLIT>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmParams p_) {
  GemmParams p = p_;
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  constexpr int A_ELEMS = TA ? GEMM_BK * BM : BM * GEMM_KPAD;
  constexpr int B_ELEMS = TB ? BN * GEMM_KPAD : GEMM_BK * BN;
  constexpr int NA = BM * GEMM_BK / 4 / 256;  // float4 per thread per chunk
  constexpr int NB = BN * GEMM_BK / 4 / 256;
  static_assert(NA >= 1 && NB >= 1, "tile too small");
  __shared__ __attribute__((aligned(16))) float smem[2 * (A_ELEMS + B_ELEMS)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int half = lane >> 5;
  const int l32 = lane & 31;
  const int wm0 = (wave / WN) * (BM / WM);
  const int wn0 = (wave % WN) * (BN / WN);

  const GxTile tile = gemm_tile(p);
  const int64_t m0 = tile.m * BM;
  const int64_t n0 = tile.n * BN;
  int64_t kbeg = 0, kend = p.K;
  if (SPLIT) {
    kbeg = tile.z * p.k_per_split;
    kend = kbeg + p.k_per_split < p.K ? kbeg + p.k_per_split : p.K;
  }
  const int nchunks = kend > kbeg ? (int)((kend - kbeg + GEMM_BK - 1) / GEMM_BK) : 0;

  f32x4 ra[NA], rb[NB];

  auto load_chunk = [&](int c) {
    const int64_t k0 = kbeg + (int64_t)c * GEMM_BK;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int f = tid + 256 * i;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (!TA) {
        const int row = f >> 3, kq = f & 7;
        const int64_t gm = m0 + row, gk = k0 + 4 * kq;
        if (gm < p.M && gk < kend) v = *reinterpret_cast<const f32x4*>(p.A + gm * p.lda + gk);
      } else {
        const int krow = f / (BM / 4), mq = f % (BM / 4);
        const int64_t gk = k0 + krow, gm = m0 + 4 * mq;
        if (gk < kend && gm < p.M) {
          const int64_t ak = p.arow ? (int64_t)p.arow[gk] : gk;  // the stored row of contraction row gk
          v = gm == p.ones_row1 - 1 ? f32x4{1.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const f32x4*>(p.A + ak * p.lda + gm);
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int f = tid + 256 * i;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (TB) {
        const int row = f >> 3, kq = f & 7;
        const int64_t gn = n0 + row, gk = k0 + 4 * kq;
        if (gn < p.N && gk < kend) v = *reinterpret_cast<const f32x4*>(p.B + gn * p.ldb + gk);
      } else {
        const int krow = f / (BN / 4), nq = f % (BN / 4);
        const int64_t gk = k0 + krow, gn = n0 + 4 * nq;
        if (gk < kend && gn < p.N) v = *reinterpret_cast<const f32x4*>(p.B + gk * p.ldb + gn);
      }
      rb[i] = v;
    }
  };

  auto store_chunk = [&](int buf) {
    float* As = smem + buf * (A_ELEMS + B_ELEMS);
    float* Bs = As + A_ELEMS;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int f = tid + 256 * i;
      if (!TA) {
        const int row = f >> 3, kq = f & 7;
        *reinterpret_cast<f32x4*>(As + row * GEMM_KPAD + 4 * kq) = ra[i];
      } else {
        const int krow = f / (BM / 4), mq = f % (BM / 4);
        *reinterpret_cast<f32x4*>(As + krow * BM + 4 * mq) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int f = tid + 256 * i;
      if (TB) {
        const int row = f >> 3, kq = f & 7;
        *reinterpret_cast<f32x4*>(Bs + row * GEMM_KPAD + 4 * kq) = rb[i];
      } else {
        const int krow = f / (BN / 4), nq = f % (BN / 4);
        *reinterpret_cast<f32x4*>(Bs + krow * BN + 4 * nq) = rb[i];
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nchunks > 0) {
    load_chunk(0);
    store_chunk(0);
    __syncthreads();
  }
  for (int c = 0; c < nchunks; ++c) {
    if (c + 1 < nchunks) load_chunk(c + 1);
    const float* As = smem + (c & 1) * (A_ELEMS + B_ELEMS);
    const float* Bs = As + A_ELEMS;
#pragma unroll
    for (int kk = 0; kk < GEMM_BK; kk += 8) {
      f32x4 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm0 + i * 32 + l32;
        if (!TA) {
          a[i] = *reinterpret_cast<const f32x4*>(As + row * GEMM_KPAD + kk + 4 * half);
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) a[i][t] = As[(kk + 4 * half + t) * BM + row];
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn0 + j * 32 + l32;
        if (TB) {
          b[j] = *reinterpret_cast<const f32x4*>(Bs + col * GEMM_KPAD + kk + 4 * half);
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) b[j][t] = Bs[(kk + 4 * half + t) * BN + col];
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma32x32x2(a[i][t], b[j][t], acc[i][j]);
    }
    if (c + 1 < nchunks) store_chunk((c + 1) & 1);
    __syncthreads();
  }

  gemm_epilogue<TM, TN, SPLIT>(p, acc, m0 + wm0, n0 + wn0, half, l32, tile.z);
}

// ---- split-operand GEMM (precision 6 / 9) ------------------------------------------------------
// fp32 operands split exactly into three bf16 planes at staging (split.hpp) and multiplied on
// v_mfma_f32_32x32x16_bf16 with NP cross products; fp32 accumulation and the same epilogue.
// BK = 16 (one MFMA k-step) per LDS chunk, double-buffered, register prefetch one chunk ahead.
// Each operand keeps its global orientation in LDS: k-contiguous rows ([row][16 k], 32 B, the
// two 16-B halves swapped on rows 8-15 of every 16: conflict-free ds_read_b128) or k-major rows
// ([16 k][BM|BN], 8-row x 32-column subtiles with XOR-swizzled chunks, read with
// ds_read_b64_tr_b16): no transposition at staging.
constexpr int GX_BK = 16;

template <int R>  // k-major image: byte offset of 16-B chunk ch (8 columns) of k-row r
__device__ __forceinline__ int gx_moff(int r, int ch) {
  return 16 * R * (r >> 3) + 512 * (ch >> 2) + 64 * (r & 7) + 16 * ((ch & 3) ^ ((r >> 2) & 3));
}
__device__ __forceinline__ int gx_koff(int row, int h) {  // k-contiguous image: half h of row
  return row * 32 + 16 * (h ^ ((row >> 3) & 1));
}

// NWV = 4 waves (2 x 2 wave grid, 2 workgroups per CU) or 8 (4 x 2, one workgroup per CU: the
// 256 x 256 tile for large problems loads 1/3 fewer operand bytes per MFMA than 128 x 256)
template <int BM, int BN, bool TA, bool TB, bool SPLIT, int NP, int NWV = 4>
__global__ __launch_bounds__(64 * NWV, NWV == 4 ? 2 : 1) void gemm_x3_kernel(GemmParams p_) {
  GemmParams p = p_;
  constexpr int NTH = 64 * NWV, WGM = NWV / 2;  // threads; wave rows (2 wave columns)
  constexpr int TM = BM / WGM / 32, TN = BN / 64;
  constexpr int A_PLANE = BM * GX_BK * 2, B_PLANE = BN * GX_BK * 2;
  constexpr int BUF = 3 * (A_PLANE + B_PLANE);
  constexpr int NA = BM * GX_BK / 4 / NTH, NB = BN * GX_BK / 4 / NTH;  // float4 per thread per chunk
  static_assert(NA >= 1 && NB >= 1 && TM >= 1, "tile too small");
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  const int wm0 = (wave >> 1) * (BM / WGM), wn0 = (wave & 1) * (BN / 2);
  const GxTile tile = gemm_tile(p);
  const int64_t m0 = tile.m * BM, n0 = tile.n * BN;
  int64_t kbeg = 0, kend = p.K;
  if (SPLIT) {
    kbeg = tile.z * p.k_per_split;
    kend = kbeg + p.k_per_split < p.K ? kbeg + p.k_per_split : p.K;
  }
  const int nchunks = kend > kbeg ? (int)((kend - kbeg + GX_BK - 1) / GX_BK) : 0;

  f32x4 ra[NA], rb[NB];
  // a row-mapped op(A) (p.arow, the distinct-row weight gradients): the stored rows of chunk c + 1's
  // contraction rows are loaded one chunk ahead of its data loads, so the dependent index -> row
  // round trip is not paid inside the chunk's own prefetch window
  int32_t ai[TA ? NA : 1];
  auto idx_load = [&](int c) {
    if constexpr (TA) {
      if (p.arow) {  // (uniform; each lane's index load unconditional, rows past the slice clamped)
        const int64_t k0 = kbeg + (int64_t)c * GX_BK;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
          const int64_t gk = k0 + (tid + NTH * i) / (BM / 4);
          ai[i] = p.arow[gk < kend ? gk : kend - 1];
        }
      }
    }
  };
  auto load_chunk = [&](int c) {
    const int64_t k0 = kbeg + (int64_t)c * GX_BK;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int f = tid + NTH * i;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (!TA) {
        const int row = f >> 2, kq = f & 3;
        const int64_t gm = m0 + row, gk = k0 + 4 * kq;
        if (gm < p.M && gk < kend) v = *reinterpret_cast<const f32x4*>(p.A + gm * p.lda + gk);
      } else {
        const int krow = f / (BM / 4), mq = f % (BM / 4);
        const int64_t gk = k0 + krow, gm = m0 + 4 * mq;
        if (gk < kend && gm < p.M) {
          const int64_t ak = p.arow ? (int64_t)ai[i] : gk;  // the stored row of contraction row gk
          v = gm == p.ones_row1 - 1 ? f32x4{1.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const f32x4*>(p.A + ak * p.lda + gm);
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int f = tid + NTH * i;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (TB) {
        const int row = f >> 2, kq = f & 3;
        const int64_t gn = n0 + row, gk = k0 + 4 * kq;
        if (gn < p.N && gk < kend) v = *reinterpret_cast<const f32x4*>(p.B + gn * p.ldb + gk);
      } else {
        const int krow = f / (BN / 4), nq = f % (BN / 4);
        const int64_t gk = k0 + krow, gn = n0 + 4 * nq;
        if (gk < kend && gn < p.N) v = *reinterpret_cast<const f32x4*>(p.B + gk * p.ldb + gn);
      }
      rb[i] = v;
    }
  };
  auto put = [&](char* plane0, int plane_bytes, int off, f32x4 v) {
    const IbSplit s0 = ib_split2(v[0], v[1]), s1 = ib_split2(v[2], v[3]);
    *reinterpret_cast<u32x2*>(plane0 + off) = u32x2{s0.h, s1.h};
    *reinterpret_cast<u32x2*>(plane0 + plane_bytes + off) = u32x2{s0.m, s1.m};
    *reinterpret_cast<u32x2*>(plane0 + 2 * plane_bytes + off) = u32x2{s0.l, s1.l};
  };
  // weight gradient: column sums of op(B) = G (k-major rows, thread column group tid % (BN / 4))
  constexpr bool CS = TA && !TB && SPLIT;
  static_assert(!CS || NTH % (BN / 4) == 0, "column groups must not depend on the chunk slot");
  const bool do_cs = CS && p.colsum_row > 0 && tile.m == 0;
  f32x4 csum = {0.f, 0.f, 0.f, 0.f};
  auto store_chunk = [&](int buf) {
    char* As = smem + buf * BUF;
    char* Bs = As + 3 * A_PLANE;
    if constexpr (CS) {
      if (do_cs) {
#pragma unroll
        for (int i = 0; i < NB; ++i) csum += rb[i];
      }
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int f = tid + NTH * i;
      if (!TA) {
        const int row = f >> 2, kq = f & 3;
        put(As, A_PLANE, gx_koff(row, kq >> 1) + 8 * (kq & 1), ra[i]);
      } else {
        const int krow = f / (BM / 4), mq = f % (BM / 4);
        put(As, A_PLANE, gx_moff<BM>(krow, mq >> 1) + 8 * (mq & 1), ra[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int f = tid + NTH * i;
      if (TB) {
        const int row = f >> 2, kq = f & 3;
        put(Bs, B_PLANE, gx_koff(row, kq >> 1) + 8 * (kq & 1), rb[i]);
      } else {
        const int krow = f / (BN / 4), nq = f % (BN / 4);
        put(Bs, B_PLANE, gx_moff<BN>(krow, nq >> 1) + 8 * (nq & 1), rb[i]);
      }
    }
  };
  // fragment of the 32 rows (or columns) starting at r0 of an operand image: element j = k 8h + j
  auto frag_k = [&](const char* plane, int r0) -> u32x4 {
    return *reinterpret_cast<const u32x4*>(plane + gx_koff(r0 + l32, half));
  };
  const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  auto frag_m = [&](const char* plane, int R, int c0) -> u32x4 {  // R = BM or BN
    u32x4 a;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int r = 8 * half + 4 * b + qq;
      const int ch = c0 / 8 + 2 * (g & 1) + (pp >> 1);
      const int off = 16 * R * (r >> 3) + 512 * (ch >> 2) + 64 * (r & 7) + 16 * ((ch & 3) ^ ((r >> 2) & 3)) + 8 * (pp & 1);
      const ib_s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) ib_s16x4*)(plane + off));
      const u32x2 w2 = __builtin_bit_cast(u32x2, v);
      a[2 * b] = w2[0];
      a[2 * b + 1] = w2[1];
    }
    return a;
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nchunks > 0) {
    idx_load(0);
    load_chunk(0);
    store_chunk(0);
    if (nchunks > 1) idx_load(1);
    __syncthreads();
  }
  for (int c = 0; c < nchunks; ++c) {
    if (c + 1 < nchunks) {
      load_chunk(c + 1);
      if (c + 2 < nchunks) idx_load(c + 2);
    }
    const char* As = smem + (c & 1) * BUF;
    const char* Bs = As + 3 * A_PLANE;
    u32x4 a[TM][3];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        a[i][pl] = TA ? frag_m(As + pl * A_PLANE, BM, wm0 + 32 * i) : frag_k(As + pl * A_PLANE, wm0 + 32 * i);
#pragma unroll
    for (int j = 0; j < TN; ++j) {  // one B fragment live at a time
      u32x4 b[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        b[pl] = TB ? frag_k(Bs + pl * B_PLANE, wn0 + 32 * j) : frag_m(Bs + pl * B_PLANE, BN, wn0 + 32 * j);
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[i][j] = mfma_split<NP>(a[i], b, acc[i][j]);
    }
    if (c + 1 < nchunks) store_chunk((c + 1) & 1);
    __syncthreads();
  }
  if constexpr (CS) {
    if (do_cs) {  // the NTH / (BN / 4) partial sums of each column group, in thread order
      f32x4* red = reinterpret_cast<f32x4*>(smem);
      red[tid] = csum;
      __syncthreads();
      if (tid < BN / 4) {
        f32x4 t = red[tid];
        for (int r = 1; r < NTH / (BN / 4); ++r) t += red[tid + r * (BN / 4)];
        const int64_t col = n0 + 4 * tid;
        float* dst = p.slab + tile.z * (p.slab_stride ? p.slab_stride : p.M * p.N) + p.colsum_row * p.N;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (col + e < p.N) dst[col + e] = t[e];
      }
    }
  }
  gemm_epilogue<TM, TN, SPLIT>(p, acc, m0 + wm0, n0 + wn0, half, l32, tile.z);
}

// ---- plane-image GEMM (precision 6 / 9 on pre-split operands) -----------------------------------
// The operands arrive as bf16 plane images in HBM, written once per operand by plane_image_kernel
// (h, m, l of every fp32 element, split.hpp), laid out so that every (plane, 16-k chunk, 256-wide
// tile) is ONE contiguous 8 KB block that is byte for byte the LDS image the fragment reads
// expect. A 512-thread workgroup (8 waves, 4 x 2, each 64 x 128 of a 256 x 256 tile) streams the
// 48 KB of a chunk (A and B, three planes each) into a 3-stage LDS ring with global_load_lds
// (LDS-DMA: no VGPR staging, no split VALU, loads issued two chunks ahead), one barrier per chunk.
// Same MFMA sequence, k order and epilogue as gemm_x3_kernel: bitwise the same sums.
//   KC image of X [R][K] (k contiguous, e.g. the A of x W): block (pl, kc, tile) at
//     ((pl * KCn + kc) * Rp + 256 tile) * 32; row r of the tile = 32 B (k 0-7 | k 8-15, halves
//     swapped on rows with bit 3 set) -> fragment reads ds_read_b128 (gx_koff);
//   KM image of X [K][C] (k = row index, e.g. the B of x W): block (pl, kc, tile) at
//     ((pl * KCn + kc) * Cp / 32 + 8 tile) * 1024: eight 1 KB 32-column blocks of 16 k rows (two
//     8-row x 32-column subtiles, XOR-swizzled 16-B chunks) -> ds_read_b64_tr_b16 fragments.
// KCn = ceil(K / 16), Rp / Cp = rows / cols padded to 256; the padding is zeros.
constexpr int PG_T = 256;  // image padding unit (rows of a KC / columns of a KM image)

__device__ __forceinline__ int pg_moff(int r, int ch) {  // KM block: byte offset of chunk ch of k-row r
  return 1024 * (ch >> 2) + 512 * (r >> 3) + 64 * (r & 7) + 16 * ((ch & 3) ^ ((r >> 2) & 3));
}

// layout 0 (KC): image of X[rows][cols] with k = cols; layout 1 (KM): k = rows.
// KC: one thread per (row, 16-k chunk); KM: one wave per (16-k chunk, 32-column block).
__global__ __launch_bounds__(256) void plane_image_kc_kernel(const float* __restrict__ X, int64_t ldx,
                                                             int64_t R, int64_t K, int64_t Rp, int64_t KCn,
                                                             char* __restrict__ img) {
  const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t kc = blockIdx.y;
  if (row >= Rp) return;
  float v[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t k = kc * 16 + 4 * q;
    f32x4 x = {0.f, 0.f, 0.f, 0.f};
    if (row < R) {
      if (k + 3 < K) {
        x = *reinterpret_cast<const f32x4*>(X + row * ldx + k);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (k + e < K) x[e] = X[row * ldx + k + e];
      }
    }
    v[4 * q] = x[0];
    v[4 * q + 1] = x[1];
    v[4 * q + 2] = x[2];
    v[4 * q + 3] = x[3];
  }
  const int64_t plane = KCn * Rp * 32;
  char* dst = img + (kc * Rp + row) * 32;
  const int sw = (int)((row >> 3) & 1);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    u32x4 ph, pm, pl;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const IbSplit x = ib_split2(v[8 * h + 2 * w], v[8 * h + 2 * w + 1]);
      ph[w] = x.h;
      pm[w] = x.m;
      pl[w] = x.l;
    }
    const int off = 16 * (h ^ sw);
    *reinterpret_cast<u32x4*>(dst + off) = ph;
    *reinterpret_cast<u32x4*>(dst + plane + off) = pm;
    *reinterpret_cast<u32x4*>(dst + 2 * plane + off) = pl;
  }
}

__global__ __launch_bounds__(256) void plane_image_km_kernel(const float* __restrict__ X, int64_t ldx,
                                                             int64_t K, int64_t C, int64_t Cp, int64_t KCn,
                                                             char* __restrict__ img) {
  const int lane = threadIdx.x & 63;
  const int64_t cb = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // 32-column block
  const int64_t kc = blockIdx.y;
  if (cb * 32 >= Cp) return;
  const int r = lane >> 2, ch = lane & 3;
  const int64_t k = kc * 16 + r, c0 = cb * 32 + 8 * ch;
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = 0.f;
  if (k < K) {
    if (c0 + 7 < C) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(X + k * ldx + c0);
      const f32x4 b = *reinterpret_cast<const f32x4*>(X + k * ldx + c0 + 4);
      v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
      v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c0 + e < C) v[e] = X[k * ldx + c0 + e];
    }
  }
  u32x4 ph, pm, pl;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const IbSplit x = ib_split2(v[2 * w], v[2 * w + 1]);
    ph[w] = x.h;
    pm[w] = x.m;
    pl[w] = x.l;
  }
  const int64_t plane = KCn * Cp * 32;
  char* dst = img + (kc * (Cp / 32) + cb) * 1024 + pg_moff(r, ch);
  *reinterpret_cast<u32x4*>(dst) = ph;
  *reinterpret_cast<u32x4*>(dst + plane) = pm;
  *reinterpret_cast<u32x4*>(dst + 2 * plane) = pl;
}

struct PgemmImgs {
  const char* A;
  const char* B;
  int64_t a_plane, b_plane;  // bytes per plane of each image (KCn * padded extent * 32)
  int64_t a_slab, b_slab;    // bytes per (plane, chunk) = padded extent * 32
};

// one 8 KB block per wave-instruction group: 512 threads x 16 B; M0 holds the wave's LDS base
__device__ __forceinline__ void pg_dma(const char* __restrict__ src, uint32_t lds_wave, int lane) {
  const char* g = src + lane * 16;
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(lds_wave)
               : "memory");
}

// BM x BN tiles on NWV waves in a (NWV / WGN) x WGN grid, NS-stage ring: <256, 256, 8, 3> (each
// wave 64 x 128; 144 KB, one workgroup per CU), <128, 256, 4, 2> (64 x 128; 72 KB, two per CU: one's
// epilogue and prologue run beside the other's MFMAs) or <256, 256, 4, 3, WGN = 2> (each wave 128 x
// 128 at one wave per SIMD, 512 registers: a quarter of the LDS fragment reads and DMA issues per
// MFMA of the 64 x 128 wave tile)
template <int BM, int BN, int NWV, int NS, bool TA, bool TB, bool SPLIT, int NP, int WGN = 2, int OCC = 0>
__global__ __launch_bounds__(64 * NWV, OCC ? OCC : (NWV == 8 ? 1 : 2)) void pgemm_kernel(GemmParams p, PgemmImgs im) {
  constexpr int WGM = NWV / WGN;
  constexpr int TM = BM / WGM / 32, TN = BN / WGN / 32;
  constexpr int ABLK = BM * GX_BK * 2, BBLK = BN * GX_BK * 2, STAGE = 3 * (ABLK + BBLK);
  constexpr int NA = ABLK / 1024 / NWV, NB = BBLK / 1024 / NWV;  // 1 KB copies per wave per plane
  constexpr int PC = 3 * (NA + NB);                              // copies per wave per chunk
  static_assert(NA >= 1 && NB >= 1 && TM * 32 * WGM == BM && TN * 32 * WGN == BN && BN == 256, "pgemm tile");
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  const int wm0 = (wave / WGN) * (BM / WGM), wn0 = (wave % WGN) * (BN / WGN);
  const GxTile tile = gx_tile();
  const int64_t m0 = tile.m * BM, n0 = tile.n * BN;
  int64_t kbeg = 0, kend = p.K;
  if (SPLIT) {
    kbeg = tile.z * p.k_per_split;
    kend = kbeg + p.k_per_split < p.K ? kbeg + p.k_per_split : p.K;
  }
  const int nchunks = kend > kbeg ? (int)((kend - kbeg + GX_BK - 1) / GX_BK) : 0;
  const int64_t kc0 = kbeg / GX_BK;
  const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem);
  const uint32_t lds_wave = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)wave * 1024);
  // this wave's 1 KB pieces of each (plane) block: piece wave + NWV k
  const char* a_src = im.A + tile.m * ABLK + wave * 1024;
  const char* b_src = im.B + tile.n * BBLK + wave * 1024;
  auto issue = [&](int c) __attribute__((always_inline)) {
    const int64_t kc = kc0 + c;
    const uint32_t st = lds_wave + (uint32_t)((c % NS) * STAGE);
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int k = 0; k < NA; ++k)
        pg_dma(a_src + pl * im.a_plane + kc * im.a_slab + k * NWV * 1024, st + pl * ABLK + k * NWV * 1024, lane);
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int k = 0; k < NB; ++k)
        pg_dma(b_src + pl * im.b_plane + kc * im.b_slab + k * NWV * 1024, st + 3 * ABLK + pl * BBLK + k * NWV * 1024,
               lane);
  };
  auto frag_k = [&](const char* plane, int r0) -> u32x4 {
    return *reinterpret_cast<const u32x4*>(plane + gx_koff(r0 + l32, half));
  };
  const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  auto frag_m = [&](const char* plane, int c0) -> u32x4 {
    u32x4 a;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int r = 8 * half + 4 * b + qq;
      const int ch = c0 / 8 + 2 * (g & 1) + (pp >> 1);
      const ib_s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) ib_s16x4*)(plane + pg_moff(r, ch) + 8 * (pp & 1)));
      const u32x2 w2 = __builtin_bit_cast(u32x2, v);
      a[2 * b] = w2[0];
      a[2 * b + 1] = w2[1];
    }
    return a;
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // 32 x 32 subtiles of this wave that hold any output (wave-uniform): at N = 3344 the last tile
  // column has 16 valid columns, so its workgroups do 1/8 of the MFMAs
  const int64_t nrem = p.N - (n0 + wn0), mrem = p.M - (m0 + wm0);
  const int nj = nrem <= 0 ? 0 : (nrem >= 32 * TN ? TN : (int)((nrem + 31) / 32));
  const int ni = mrem <= 0 ? 0 : (mrem >= 32 * TM ? TM : (int)((mrem + 31) / 32));
  for (int c = 0; c < NS - 1 && c < nchunks; ++c) issue(c);
  for (int c = 0; c < nchunks; ++c) {
    // chunk c has landed once at most the copies of the NS - 2 younger chunks are in flight
    if constexpr (NS == 3) {
      static_assert(PC == 6 || PC == 12, "vmcnt immediate");
      if (c + 1 < nchunks) {
        if constexpr (PC == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();  // every wave's copies of chunk c are in LDS; stage (c + NS - 1) % NS is free
    if (c + NS - 1 < nchunks) issue(c + NS - 1);
    const char* As = smem + (c % NS) * STAGE;
    const char* Bs = As + 3 * ABLK;
    u32x4 a[TM][3];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        a[i][pl] = TA ? frag_m(As + pl * ABLK, wm0 + 32 * i) : frag_k(As + pl * ABLK, wm0 + 32 * i);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (j < nj) {  // 32-column subtiles wholly past N (the last tile column) issue no MFMAs
        u32x4 b[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          b[pl] = TB ? frag_k(Bs + pl * BBLK, wn0 + 32 * j) : frag_m(Bs + pl * BBLK, wn0 + 32 * j);
#pragma unroll
        for (int i = 0; i < TM; ++i)
          if (i < ni) acc[i][j] = mfma_split<NP>(a[i], b, acc[i][j]);
      }
    }
  }
  gemm_epilogue<TM, TN, SPLIT>(p, acc, m0 + wm0, n0 + wn0, half, l32, tile.z);
}

int64_t pimg_pad(int64_t n) { return ceil_div(n > 0 ? n : 1, PG_T) * PG_T; }
size_t pimg_bytes(int64_t K, int64_t extent) {
  return (size_t)3 * (size_t)ceil_div(K > 0 ? K : 1, GX_BK) * (size_t)pimg_pad(extent) * 32;
}

// image of X (rows x cols, leading dim ldx): layout 0 = KC (k = cols), 1 = KM (k = rows)
int plane_image_launch(const float* X, int64_t ldx, int64_t rows, int64_t cols, int layout, char* img,
                       hipStream_t st) {
  if (layout == 0) {
    const int64_t Rp = pimg_pad(rows), KCn = ceil_div(cols > 0 ? cols : 1, GX_BK);
    hipLaunchKernelGGL(plane_image_kc_kernel, dim3((unsigned)(Rp / 256), (unsigned)KCn), dim3(256), 0, st, X, ldx,
                       rows, cols, Rp, KCn, img);
  } else {
    const int64_t Cp = pimg_pad(cols), KCn = ceil_div(rows > 0 ? rows : 1, GX_BK);
    hipLaunchKernelGGL(plane_image_km_kernel, dim3((unsigned)(Cp / 128), (unsigned)KCn), dim3(256), 0, st, X, ldx,
                       rows, cols, Cp, KCn, img);
  }
  return check_launch("plane_image");
}

// Plane-GEMM tile: 128-row tiles (two workgroups per CU, default), RS_PGEMM_BM=256 (8 waves of 64 x
// 128, one workgroup per CU, 3-stage ring) or RS_PGEMM_BM=2564 (4 waves of 128 x 128 at one wave
// per SIMD, 3-stage ring): A/B measurements, DESIGN.md.
static int pgemm_cfg() {
  static int cfg = [] {
    const char* e = exp_env("RS_PGEMM_BM");
    const int v = e ? atoi(e) : 0;
    return v == 256 ? 1 : (v == 2564 ? 2 : 0);
  }();
  return cfg;
}
static int pgemm_bm() { return pgemm_cfg() ? 256 : 128; }

// C = epilogue(op(A) op(B)) from the images: A is KM when ta (A^T stored [K][M]) else KC ([M][K]);
// B is KC when tb ([N][K]) else KM ([K][N]).
template <bool SPLIT>
int pgemm_dispatch(int ta, int tb, GemmParams p, const char* Aimg, const char* Bimg, int64_t S, hipStream_t st) {
  PgemmImgs im;
  im.A = Aimg;
  im.B = Bimg;
  const int64_t KCn = ceil_div(p.K > 0 ? p.K : 1, GX_BK);
  im.a_slab = pimg_pad(p.M) * 32;
  im.b_slab = pimg_pad(p.N) * 32;
  im.a_plane = KCn * im.a_slab;
  im.b_plane = KCn * im.b_slab;
  const int bm = pgemm_bm();
  dim3 grid((unsigned)ceil_div(p.N, PG_T), (unsigned)ceil_div(p.M, bm), (unsigned)S);
#define RS_PG(TA_, TB_)                                                                                            \
  if (pgemm_cfg() == 2) {                                                                                          \
    if (p.prec == 6)                                                                                               \
      hipLaunchKernelGGL((pgemm_kernel<256, 256, 4, 3, TA_, TB_, SPLIT, 6, 2, 1>), grid, dim3(256), 0, st, p, im); \
    else                                                                                                           \
      hipLaunchKernelGGL((pgemm_kernel<256, 256, 4, 3, TA_, TB_, SPLIT, 9, 2, 1>), grid, dim3(256), 0, st, p, im); \
  } else if (bm == 256) {                                                                                          \
    if (p.prec == 6)                                                                                               \
      hipLaunchKernelGGL((pgemm_kernel<256, 256, 8, 3, TA_, TB_, SPLIT, 6>), grid, dim3(512), 0, st, p, im);       \
    else                                                                                                           \
      hipLaunchKernelGGL((pgemm_kernel<256, 256, 8, 3, TA_, TB_, SPLIT, 9>), grid, dim3(512), 0, st, p, im);       \
  } else {                                                                                                         \
    if (p.prec == 6)                                                                                               \
      hipLaunchKernelGGL((pgemm_kernel<128, 256, 4, 2, TA_, TB_, SPLIT, 6>), grid, dim3(256), 0, st, p, im);       \
    else                                                                                                           \
      hipLaunchKernelGGL((pgemm_kernel<128, 256, 4, 2, TA_, TB_, SPLIT, 9>), grid, dim3(256), 0, st, p, im);       \
  }
  if (!ta && !tb) { RS_PG(false, false) }
  else if (!ta && tb) { RS_PG(false, true) }
  else if (ta && !tb) { RS_PG(true, false) }
  else { RS_PG(true, true) }
#undef RS_PG
  return check_launch(SPLIT ? "pgemm_splitk" : "pgemm");
}

template <bool SPLIT>
static int dispatch(int ta, int tb, const GemmParams& p, dim3 gz, hipStream_t st) {
  // Split-operand GEMMs with a short K loop (K <= 256: the Dense layers) run on 64 x 64 tiles:
  // 8x the workgroups of the 128 x 256 tile, so a CU holds several at different phases and one's
  // prologue / epilogue traffic overlaps another's MFMAs (C3 tower forward 61 -> 53 us, dX 46 ->
  // 42 us, C3 step -1 %, C2 step 0.88 -> 0.81 ms)
  const bool short_k = p.prec != 0 && !SPLIT && p.K <= 256;
  // tile choice per problem (a grouped launch uses the tiles of its single-problem launches)
  const int64_t zh = p.ngroup > 1 ? (int64_t)gz.z / p.ngroup : (int64_t)gz.z;
  const bool wide = p.N > 64 && !short_k;
  const int BN = wide ? 128 : 64;
  // 128-row tiles unless that leaves the chip under-filled (< 256 workgroups): then 64 rows
  const bool tall = !short_k && ceil_div(p.M, 128) * ceil_div(p.N, BN) * zh >= 256;
  const int BM = tall ? 128 : 64;
  dim3 grid((unsigned)ceil_div(p.N, BN), (unsigned)ceil_div(p.M, BM), gz.z);
#define RS_GEMM_LAUNCH(TA_, TB_)                                                                    \
  if (tall && wide)                                                                                 \
    hipLaunchKernelGGL((gemm_f32_kernel<128, 128, 2, 2, TA_, TB_, SPLIT>), grid, dim3(256), 0, st, p); \
  else if (tall)                                                                                    \
    hipLaunchKernelGGL((gemm_f32_kernel<128, 64, 2, 2, TA_, TB_, SPLIT>), grid, dim3(256), 0, st, p);  \
  else if (wide)                                                                                    \
    hipLaunchKernelGGL((gemm_f32_kernel<64, 128, 2, 2, TA_, TB_, SPLIT>), grid, dim3(256), 0, st, p);  \
  else                                                                                              \
    hipLaunchKernelGGL((gemm_f32_kernel<64, 64, 2, 2, TA_, TB_, SPLIT>), grid, dim3(256), 0, st, p);
#if defined(RS_GEMM_X3_256)
// large problems: 256 x 256 tiles on 8 waves (each wave 64 x 128), one workgroup per CU
#define RS_GEMM_X3_BIG(TA_, TB_, NP_)                                                                  \
  if (p.M >= 256 && p.N >= 256 && ceil_div(p.M, 256) * ceil_div(p.N, 256) * zh >= 256) {   \
    dim3 g2((unsigned)ceil_div(p.N, 256), (unsigned)ceil_div(p.M, 256), gz.z);                          \
    hipLaunchKernelGGL((gemm_x3_kernel<256, 256, TA_, TB_, SPLIT, NP_, 8>), g2, dim3(512), 0, st, p);    \
  } else
#elif !defined(RS_GEMM_X3_M256) && !defined(RS_GEMM_X3_NOBIG)
// large problems: 128 x 256 tiles (each wave 64 x 128: half the LDS fragment reads per MFMA)
#define RS_GEMM_X3_BIG(TA_, TB_, NP_)                                                                  \
  if (tall && p.N >= 256 && ceil_div(p.M, 128) * ceil_div(p.N, 256) * zh >= 512) {          \
    dim3 g2((unsigned)ceil_div(p.N, 256), (unsigned)ceil_div(p.M, 128), gz.z);                          \
    hipLaunchKernelGGL((gemm_x3_kernel<128, 256, TA_, TB_, SPLIT, NP_>), g2, dim3(256), 0, st, p);       \
  } else
#elif defined(RS_GEMM_X3_M256)
#define RS_GEMM_X3_BIG(TA_, TB_, NP_)                                                                  \
  if (tall && p.M >= 256 && wide && ceil_div(p.M, 256) * ceil_div(p.N, 128) * zh >= 512) {  \
    dim3 g2((unsigned)ceil_div(p.N, 128), (unsigned)ceil_div(p.M, 256), gz.z);                          \
    hipLaunchKernelGGL((gemm_x3_kernel<256, 128, TA_, TB_, SPLIT, NP_>), g2, dim3(256), 0, st, p);       \
  } else
#else
#define RS_GEMM_X3_BIG(TA_, TB_, NP_)
#endif
#define RS_GEMM_X3(TA_, TB_, NP_)                                                                      \
  RS_GEMM_X3_BIG(TA_, TB_, NP_)                                                                        \
  if (tall && wide)                                                                                    \
    hipLaunchKernelGGL((gemm_x3_kernel<128, 128, TA_, TB_, SPLIT, NP_>), grid, dim3(256), 0, st, p);     \
  else if (tall)                                                                                       \
    hipLaunchKernelGGL((gemm_x3_kernel<128, 64, TA_, TB_, SPLIT, NP_>), grid, dim3(256), 0, st, p);      \
  else if (wide)                                                                                       \
    hipLaunchKernelGGL((gemm_x3_kernel<64, 128, TA_, TB_, SPLIT, NP_>), grid, dim3(256), 0, st, p);      \
  else                                                                                                 \
    hipLaunchKernelGGL((gemm_x3_kernel<64, 64, TA_, TB_, SPLIT, NP_>), grid, dim3(256), 0, st, p);
#define RS_GEMM_X3_NP(TA_, TB_) \
  if (p.prec == 6) { RS_GEMM_X3(TA_, TB_, 6) } else { RS_GEMM_X3(TA_, TB_, 9) }
  static const bool no_ws = exp_env("RS_GEMM_NO_WS") != nullptr;             // A/B switch (timing)
  if (!SPLIT && !no_ws && ws_ok(ta, tb, p)) {
    ws_dispatch(tb, p, st);
    return check_launch("gemm_ws");
  }
  static const bool no_skinny = exp_env("RS_GEMM_NO_SKINNY") != nullptr;   // A/B switch (timing)
  if (!SPLIT && !no_skinny && skinny_ok(ta, tb, p)) {
    skinny_dispatch(tb, p, st);
    return check_launch("gemm_skinny");
  }
  if (p.prec == 6 || p.prec == 9) {
    if (!ta && !tb) { RS_GEMM_X3_NP(false, false) }
    else if (!ta && tb) { RS_GEMM_X3_NP(false, true) }
    else if (ta && !tb) { RS_GEMM_X3_NP(true, false) }
    else { RS_GEMM_X3_NP(true, true) }
    return check_launch(SPLIT ? "gemm_x3_splitk" : "gemm_x3");
  }
#undef RS_GEMM_X3_NP
#undef RS_GEMM_X3
  if (!ta && !tb) { RS_GEMM_LAUNCH(false, false) }
  else if (!ta && tb) { RS_GEMM_LAUNCH(false, true) }
  else if (ta && !tb) { RS_GEMM_LAUNCH(true, false) }
  else { RS_GEMM_LAUNCH(true, true) }
#undef RS_GEMM_LAUNCH
  return check_launch(SPLIT ? "gemm_f32_splitk" : "gemm_f32");
}

static int validate(const char* fn, int ta, int tb, int64_t M, int64_t N, int64_t K,
                    const float* A, int64_t lda, const float* B, int64_t ldb, const float* C,
                    int64_t ldc) {
  RS_REQUIRE(M >= 0 && N >= 0 && K >= 0, "%s: negative size", fn);
  RS_REQUIRE((A || M * K == 0) && (B || K * N == 0) && (C || M * N == 0), "%s: null operand", fn);
  RS_REQUIRE((!A || aligned16(A)) && (!B || aligned16(B)), "%s: operands must be 16-byte aligned", fn);
  RS_REQUIRE(lda % 4 == 0 && ldb % 4 == 0, "%s: lda/ldb must be multiples of 4", fn);
  RS_REQUIRE(lda >= (ta ? M : K) && ldb >= (tb ? K : N) && ldc >= N, "%s: leading dim too small",
             fn);
  // the k-contiguous staging moves whole float4s along k; m/n-contiguous along m or n
  RS_REQUIRE(K % 4 == 0 || (ta && !tb), "%s: K must be a multiple of 4 for this layout", fn);
  RS_REQUIRE(!ta || M % 4 == 0, "%s: M must be a multiple of 4 when trans_a", fn);
  RS_REQUIRE(tb || N % 4 == 0, "%s: N must be a multiple of 4 when !trans_b", fn);
  return RS_OK;
}

static int64_t splitk_count(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = ceil_div(M, 128) * ceil_div(N, N > 64 ? 128 : 64);
  // ~2 workgroups per CU; a large output (the DCN-v2 dW, 27 x 27 tiles) takes at least 2 slices,
  // which makes it eligible for the 128 x 256 split tiles (c5 dW 2.45 -> 2.26 ms).
  // RS_SPLITK_WANT (timing switch: the workgroup target of small outputs; the slices, and so the
  // order of the fp32 sums, change with it). 256: the C3 tower dW + db (4 layers, both towers)
  // 273 -> 234 us against 512 (tools/gpu_r04_f.sh, profiles/r04_splitk_want.log); fewer slices
  // write and re-read fewer slab bytes, more leave CUs idle (128: 257 us, 64: 319 us)
  static const int64_t want_small = [] {
    const char* e = exp_env("RS_SPLITK_WANT");
    return e && atoi(e) > 0 ? (int64_t)atoi(e) : (int64_t)256;
  }();
  int64_t want = ceil_div(tiles >= 256 ? 1024 : want_small, tiles);
  int64_t maxs = ceil_div(K, 128);                       // >= 128 reduction rows per split
  int64_t s = want < maxs ? want : maxs;
  if (s < 1) s = 1;
  if (s > 1024) s = 1024;
  return s;
}

// Plane-image GEMM launchers used by the DCN-v2 stack (dcn2.hip): full epilogue control.
int pgemm_launch(int ta, int tb, int64_t M, int64_t N, int64_t K, const char* Aimg, const char* Bimg, float* C,
                 int64_t ldc, const float* bias, int epi, const float* x0, const float* xres, float* aux, int64_t ldx,
                 const float* addend, int64_t ldadd, hipStream_t st, int prec, float beta) {
  RS_REQUIRE(M >= 0 && N >= 0 && K >= 0 && Aimg && Bimg && (C || M * N == 0), "pgemm_launch: bad args");
  RS_REQUIRE(prec == RS_PREC_F32_SPLIT6 || prec == RS_PREC_F32_SPLIT9, "pgemm_launch: precision must be 6 or 9");
  if (M == 0 || N == 0) return RS_OK;
  GemmParams p{nullptr, nullptr, C, 0, 0, ldc, M, N, K, bias, 0, nullptr, 0, beta, K, nullptr,
               epi, x0, xres, aux, ldx, addend, ldadd, prec};
  return pgemm_dispatch<false>(ta, tb, p, Aimg, Bimg, 1, st);
}

// K slices: one workgroup per CU, so the time is ~ rounds(S) = ceil(tiles S / 256) rounds of K / S
// each, plus S slabs of M N floats written and read by the ordered reduction. Pick the S that
// minimises that model (measured constants: ~0.146 ns per k-row of a 256 x 256 round, ~5 TB/s
// for the slabs), with >= 256 reduction rows per slice.
static int64_t pgemm_splitk_count(int64_t M, int64_t N, int64_t K) {
  const int64_t bm = pgemm_bm(), slots = 256 * (PG_T / bm);     // resident workgroups chip-wide
  const int64_t tiles = ceil_div(M, bm) * ceil_div(N, PG_T);
  int64_t maxs = K / 256;
  if (maxs > 64) maxs = 64;
  int64_t best = 1;
  double best_t = 1e30;
  for (int64_t s = 1; s <= (maxs < 1 ? 1 : maxs); ++s) {
    const double rounds = (double)ceil_div(tiles * s, slots);
    // ~0.11 us per k per round of 256 x 256 tiles (measured: 1.82 ms for K = 16384 at s = 1), plus
    // the slabs' write + read at ~5 TB/s
    const double t = rounds * ((double)K / s) * 1.1e-7 + (s > 1 ? (double)s * M * N * 8.0 / 5e12 : 0.0);
    if (t < best_t * 0.995) {
      best_t = t;
      best = s;
    }
  }
  return best;
}
size_t pgemm_splitk_ws_bytes(int64_t M, int64_t N, int64_t K) {
  return align_up((size_t)pgemm_splitk_count(M, N, K) * (size_t)M * (size_t)N * sizeof(float), 256) + 256;
}
// C = op(A) op(B) (+ addend_scale * addend) with the K range split over workgroups, ordered slabs
int pgemm_splitk_launch(int ta, int tb, int64_t M, int64_t N, int64_t K, const char* Aimg, const char* Bimg,
                        float* C, const float* addend, float addend_scale, int prec, void* ws, size_t ws_bytes,
                        hipStream_t st) {
  RS_REQUIRE(M >= 0 && N >= 0 && K >= 0 && Aimg && Bimg && (C || M * N == 0), "pgemm_splitk_launch: bad args");
  RS_REQUIRE(prec == RS_PREC_F32_SPLIT6 || prec == RS_PREC_F32_SPLIT9, "pgemm_splitk_launch: precision 6 or 9");
  if (!ws || ws_bytes < pgemm_splitk_ws_bytes(M, N, K)) {
    set_error("pgemm_splitk_launch: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  if (M == 0 || N == 0) return RS_OK;
  const int64_t S = pgemm_splitk_count(M, N, K);
  const int64_t kps = ceil_div(ceil_div(K > 0 ? K : 1, S), GX_BK) * GX_BK;
  const int64_t Seff = K > 0 ? ceil_div(K, kps) : 1;
  float* slab = static_cast<float*>(ws);
  GemmParams p{nullptr, nullptr, C, 0, 0, N, M, N, K, nullptr, 0, nullptr, 0, 0.f, kps, slab,
               0, nullptr, nullptr, nullptr, 0, nullptr, 0, prec};
  const int rc = pgemm_dispatch<true>(ta, tb, p, Aimg, Bimg, Seff, st);
  if (rc) return rc;
  return launch_slab_reduce(slab, Seff, M * N, C, addend, addend_scale, st);
}

// ---- plane-pair GEMM (xgemm: precision 6 on pre-split operands, 16x16x32 MFMA) -----------------
// C[M][N] = sum_k A[m][k] B[n][k] with both fp32 operands split into bf16 planes (h, m, l;
// split.hpp) once per operand by ximg_kernel. The 16x16x32 MFMA sums 32 products over two 16-k
// halves, so one MFMA takes TWO cross products of a 16-k block: with A = [h | m] (lanes 0-31 read
// the h plane, lanes 32-63 the m plane) and B = [m | h] it adds h.m + m.h; [h | l] x [l | h] adds
// h.l + l.h and [h | m] x [h | m] adds h.h + m.m: the six products of precision 6 in 3 MFMAs, the
// same MFMA cycles per FLOP as six 16-k products, no split VALU in the loop, and each operand's
// three planes loaded once per 16-k block (6 B per element: half the L2 bytes per MFMA of
// splitting fp32 tiles at staging).
// Tile 256 x 256 on 8 waves (2 x 4, each 128 x 64 = 8 x 4 subtiles of 16 x 16), one workgroup per
// CU; a K-step is one 16-k block: 48 KB (A and B, three 8 KB plane blocks each) streamed by
// LDS-DMA (global_load_lds_dwordx4, 6 per wave) into a 3-slot ring two K-steps ahead, one raw
// s_barrier per K-step, the DMA waited with a counted vmcnt (never 0 in the loop).
//   Image of X viewed as [R][K] (R rows, contraction K): block (plane, 16-k block kb, 256-row tile
//   rt) = 8 KB at ((plane KB + kb) RT + rt) 8192; row r of the tile = 32 B (k 0-7 | k 8-15); the
//   fragment reads (lane l: row l & 15, half (l >> 4) & 1) are conflict-free on this image.
//   KB = ceil(K / 16), RT = ceil(R / 256); the padding is zeros.
constexpr int XG_BLK = 8192;
#ifndef XG_EPI_NI
#define XG_EPI_NI 4  // 16-row subtiles per epilogue batch
#endif
constexpr int XG_STAGE = 6 * XG_BLK;

__device__ __forceinline__ int64_t xg_rt_dev(int64_t R) { return (R + 255) / 256; }
int64_t xg_kb(int64_t K) { return ceil_div(K > 0 ? K : 1, 16); }
int64_t xg_rt(int64_t R) { return ceil_div(R > 0 ? R : 1, 256); }
size_t ximg_bytes(int64_t R, int64_t K) { return (size_t)3 * xg_kb(K) * xg_rt(R) * XG_BLK; }

// one thread per (row, 16-k block); TRANS: X is stored [K][R] (element (r, k) at X[k ld + r])
template <bool TRANS>
__global__ __launch_bounds__(256) void ximg_kernel(const float* __restrict__ X, int64_t ld, int64_t R, int64_t K,
                                                   int64_t RT, int64_t KB, char* __restrict__ img) {
  const int64_t rt = blockIdx.x, kb = blockIdx.y;
  const int t = threadIdx.x;
  const int64_t r = rt * 256 + t, k0 = kb * 16;
  float v[16];
  if (!TRANS) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t k = k0 + 4 * q;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      if (r < R) {
        if (k + 3 < K) {
          x = *reinterpret_cast<const f32x4*>(X + r * ld + k);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (k + e < K) x[e] = X[r * ld + k + e];
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * q + e] = x[e];
    }
  } else {
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = (r < R && k0 + e < K) ? X[(k0 + e) * ld + r] : 0.f;
  }
  const int64_t plane = KB * RT * XG_BLK;
  char* dst = img + (kb * RT + rt) * XG_BLK + t * 32;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    u32x4 ph, pm, pl;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const IbSplit s = ib_split2(v[8 * c + 2 * w], v[8 * c + 2 * w + 1]);
      ph[w] = s.h;
      pm[w] = s.m;
      pl[w] = s.l;
    }
    *reinterpret_cast<u32x4*>(dst + 16 * c) = ph;
    *reinterpret_cast<u32x4*>(dst + plane + 16 * c) = pm;
    *reinterpret_cast<u32x4*>(dst + 2 * plane + 16 * c) = pl;
  }
}

int ximg_launch(const float* X, int64_t ld, int64_t R, int64_t K, int trans, char* img, hipStream_t st) {
  const int64_t RT = xg_rt(R), KB = xg_kb(K);
  if (trans)
    hipLaunchKernelGGL(ximg_kernel<true>, dim3((unsigned)RT, (unsigned)KB), dim3(256), 0, st, X, ld, R, K, RT, KB, img);
  else
    hipLaunchKernelGGL(ximg_kernel<false>, dim3((unsigned)RT, (unsigned)KB), dim3(256), 0, st, X, ld, R, K, RT, KB, img);
  return check_launch("ximg");
}

// Both xgemm images of one [R][K] fp32 matrix from ONE read of it: img (rows R, contraction K: the
// A operand of X W) and img_t (rows K, contraction R: the operand of X^T G), byte for byte what
// ximg_kernel<false> / <true> write (padding included). Block (cb, rt): 256 rows x 32 columns (two
// 16-k blocks), read as whole 128-B row segments (8 lanes per row, 8 rows per wave instruction);
// each lane splits its 4 values into 8 B of each plane of the plain image, the tile goes through
// LDS, and thread (f, j) splits column f's 16 values of rows 16 j .. 16 j + 15 into the transposed
// image (32 columns x 32 B contiguous per plane). Blocks past the columns write the transposed
// image's zero padding rows. MODE 1 (the DCN-v2 cross backward, fused): the matrix is t = g * x0
// (never written), gx0 = base + g * u is written, and part[rt][k] = t's column sums over the
// block's rows (16-row groups in order, then the groups in order) for the bias gradient. MODE 2
// (a Dense layer's backward): the matrix is g = dy masked by y > 0 (y = x0, nullable: no mask),
// with the same column partials (the bias gradient).
template <int MODE>
__global__ __launch_bounds__(256) void ximg_dual_kernel(const float* __restrict__ X, const float* __restrict__ x0,
                                                        const float* __restrict__ u, const float* __restrict__ base,
                                                        float* __restrict__ gx0, int64_t R, int64_t K, int64_t KB,
                                                        int64_t RT, int64_t KBT, int64_t RTT, char* __restrict__ img,
                                                        char* __restrict__ img_t, float* __restrict__ part) {
  __shared__ float tile[256][33];
  const int64_t cb = blockIdx.x, rt = blockIdx.y;
  const int t = threadIdx.x;
  const int rsub = t >> 3, c4 = t & 7;
  const int64_t k = cb * 32 + 4 * c4;       // this lane's 4 columns
  const int64_t kb = cb * 2 + (c4 >> 2);    // their 16-k block
  const bool kin = k < K;                    // K % 4 == 0: a float4 is wholly inside or outside
  const int64_t plane = KB * RT * XG_BLK;
  char* dst0 = img + (kb * RT + rt) * XG_BLK + 8 * (c4 & 3);
#pragma unroll 2
  for (int ps = 0; ps < 8; ++ps) {
    const int rl = ps * 32 + rsub;
    const int64_t r = rt * 256 + rl;
    const bool in = kin && r < R;
    const int64_t o = in ? r * K + k : 0;
    f32x4 x = {0.f, 0.f, 0.f, 0.f};
    if (MODE == 2) {
      const f32x4 gv = *reinterpret_cast<const f32x4*>(X + o);
      const f32x4 yv = x0 ? *reinterpret_cast<const f32x4*>(x0 + o) : f32x4{1.f, 1.f, 1.f, 1.f};
      if (in) {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = yv[e] > 0.f ? gv[e] : 0.f;
      }
    } else if (MODE == 1) {
      const f32x4 gv = *reinterpret_cast<const f32x4*>(X + o);
      const f32x4 xv = *reinterpret_cast<const f32x4*>(x0 + o);
      const f32x4 uv = *reinterpret_cast<const f32x4*>(u + o);
      const f32x4 bv = base ? *reinterpret_cast<const f32x4*>(base + o) : f32x4{0.f, 0.f, 0.f, 0.f};
      if (in) {
        x = gv * xv;
        const f32x4 add = gv * uv;
        *reinterpret_cast<f32x4*>(gx0 + o) = base ? bv + add : add;
      }
    } else {
      const f32x4 xv = *reinterpret_cast<const f32x4*>(X + o);
      if (in) x = xv;
    }
    if (kb < KB) {
      const IbSplit s0 = ib_split2(x[0], x[1]), s1 = ib_split2(x[2], x[3]);
      char* dst = dst0 + rl * 32;
      *reinterpret_cast<u32x2*>(dst) = u32x2{s0.h, s1.h};
      *reinterpret_cast<u32x2*>(dst + plane) = u32x2{s0.m, s1.m};
      *reinterpret_cast<u32x2*>(dst + 2 * plane) = u32x2{s0.l, s1.l};
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) tile[rl][4 * c4 + e] = x[e];
  }
  __syncthreads();
  const int f = t & 31, j0 = t >> 5;
  const int64_t row = cb * 32 + f;  // row of the transposed image
  const int64_t planet = KBT * RTT * XG_BLK;
  float cs[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int j = j0 + 8 * h;
    float w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = tile[16 * j + i][f];
    cs[h] = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) cs[h] += w[i];
    const int64_t kbt = rt * 16 + j;
    if (kbt < KBT && row < RTT * 256) {
      char* dst = img_t + (kbt * RTT + row / 256) * XG_BLK + (row % 256) * 32;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        u32x4 ph, pm, pl;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const IbSplit sp = ib_split2(w[8 * c + 2 * q], w[8 * c + 2 * q + 1]);
          ph[q] = sp.h;
          pm[q] = sp.m;
          pl[q] = sp.l;
        }
        *reinterpret_cast<u32x4*>(dst + 16 * c) = ph;
        *reinterpret_cast<u32x4*>(dst + planet + 16 * c) = pm;
        *reinterpret_cast<u32x4*>(dst + 2 * planet + 16 * c) = pl;
      }
    }
  }
  if (MODE != 0 && cb * 32 < K) {
    __syncthreads();
    tile[j0][f] = cs[0];
    tile[j0 + 8][f] = cs[1];
    __syncthreads();
    if (t < 32 && cb * 32 + t < K) {
      float s = 0.f;
      for (int j = 0; j < 16; ++j) s += tile[j][t];
      part[rt * K + cb * 32 + t] = s;
    }
  }
}

// X [R][K] (K % 4 == 0, 16-B aligned, dense rows): img = ximg(X), img_t = ximg(X^T). Cross-backward
// form (u non-null): X = g, the images are those of t = g * x0, gx0 = base (nullable) + g * u,
// part [RT][K]. Masked form (part non-null, u null): the images and part of X * (x0 > 0) (x0
// nullable: X itself).
int ximg_dual_launch(const float* X, const float* x0, const float* u, const float* base, float* gx0, int64_t R,
                     int64_t K, char* img, char* img_t, float* part, hipStream_t st) {
  const int64_t KB = xg_kb(K), RT = xg_rt(R), KBT = xg_kb(R), RTT = xg_rt(K);
  const int64_t kc = ceil_div(K, 32), gx = kc > RTT * 8 ? kc : RTT * 8;
  const dim3 grid((unsigned)gx, (unsigned)RT);
  if (u)
    hipLaunchKernelGGL(ximg_dual_kernel<1>, grid, dim3(256), 0, st, X, x0, u, base, gx0, R, K, KB, RT, KBT, RTT,
                       img, img_t, part);
  else if (part)
    hipLaunchKernelGGL(ximg_dual_kernel<2>, grid, dim3(256), 0, st, X, x0, nullptr, nullptr, nullptr, R, K, KB, RT, KBT,
                       RTT, img, img_t, part);
  else
    hipLaunchKernelGGL(ximg_dual_kernel<0>, grid, dim3(256), 0, st, X, nullptr, nullptr, nullptr, nullptr, R, K, KB,
                       RT, KBT, RTT, img, img_t, nullptr);
  return check_launch("ximg_dual");
}

struct XgImgs {
  const char* A;
  const char* B;
  int64_t a_plane, b_plane;  // bytes per plane
  int64_t a_kb, b_kb;        // bytes per 16-k block (RT x 8 KB)
};

// Epilogue of one 16-column slice (subtile column j) of a wave's 128 x 64 tile: 32 values per lane
// (rows 16 i + 4 (lane >> 4) + e, column lane & 15). Every operand the epilogue reads (x0, x_l,
// mask, addend, C for beta) is loaded for all 32 values before any store, so the loads are in
// flight together: bias, DCN-v2 cross update (u -> aux, x0 * u + x_l), ReLU, mask, addend, beta * C;
// split mode writes the K-slice slab.
template <bool SPLIT, int I0, int NI>
__device__ __forceinline__ void xg_epilogue_col(const GemmParams& p, const f32x4 (&acc)[8][4], int j, int64_t row0,
                                                int64_t col, int fq, int64_t zs, int ib) {
  if (col >= p.N) return;
  float v[NI][4];
  bool ok[NI][4];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[i][e] = acc[ib + i][j][e];
      ok[i][e] = row0 + i * 16 + fq * 4 + e < p.M;
    }
  if (SPLIT) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (ok[i][e]) p.slab[zs * (p.slab_stride ? p.slab_stride : p.M * p.N) + (row0 + i * 16 + fq * 4 + e) * p.N + col] = v[i][e];
    return;
  }
  const float bv = p.bias ? p.bias[col] : 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) v[i][e] += bv;
  if (p.epi == 1) {
    float x0v[NI][4], xrv[NI][4];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t xo = (row0 + i * 16 + fq * 4 + e) * p.ldx + col;
        x0v[i][e] = ok[i][e] ? p.x0[xo] : 0.f;
        xrv[i][e] = ok[i][e] ? p.xres[xo] : 0.f;
      }
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t xo = (row0 + i * 16 + fq * 4 + e) * p.ldx + col;
        if (ok[i][e]) p.aux[xo] = v[i][e];
        v[i][e] = x0v[i][e] * v[i][e] + xrv[i][e];
      }
  }
  if (p.act == RS_ACT_RELU) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[i][e] = fmaxf(v[i][e], 0.f);
  }
  if (p.mask) {
    float mv[NI][4];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) mv[i][e] = ok[i][e] ? p.mask[(row0 + i * 16 + fq * 4 + e) * p.ldm + col] : 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (!(mv[i][e] > 0.f)) v[i][e] = 0.f;
  }
  if (p.addend) {
    float av[NI][4];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) av[i][e] = ok[i][e] ? p.addend[(row0 + i * 16 + fq * 4 + e) * p.ldadd + col] : 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[i][e] += av[i][e];
  }
  if (p.beta != 0.f) {
    float cv[NI][4];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) cv[i][e] = ok[i][e] ? p.C[(row0 + i * 16 + fq * 4 + e) * p.ldc + col] : 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[i][e] += p.beta * cv[i][e];
  }
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (ok[i][e]) p.C[(row0 + i * 16 + fq * 4 + e) * p.ldc + col] = v[i][e];
}

// V (A/B variants, RS_XGEMM_VAR): bit 0 s_setprio 1 around each K-step's MFMAs, bit 1 the next
// copies issued in three pairs spread over the MFMAs, bit 2 static priority 1 for waves 4-7
template <bool SPLIT, int V = 0>
__global__ __launch_bounds__(512, 1) void xgemm_kernel(GemmParams p, XgImgs im) {
  __shared__ __attribute__((aligned(1024))) char smem[3 * XG_STAGE];  // 3-slot ring of K-steps
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, hi = lane >> 5;
  GxTile tile;
  if (p.tile_n > 0) {  // tile-range launch: 1-D grid of tile_n tiles (x K slices)
    const int64_t tt = gx_xcd(blockIdx.x, gridDim.x);
    tile = gx_map(p.tile_lo + tt % p.tile_n, xg_rt_dev(p.N), xg_rt_dev(p.M));
    tile.z = tt / p.tile_n;
  } else {
    tile = gx_tile();
  }
  const int64_t m0 = tile.m * 256, n0 = tile.n * 256;
  int64_t kbeg = 0, kend = p.K;
  if (SPLIT) {
    kbeg = tile.z * p.k_per_split;
    kend = kbeg + p.k_per_split < p.K ? kbeg + p.k_per_split : p.K;
  }
  const int nsteps = kend > kbeg ? (int)((kend - kbeg + 15) / 16) : 0;
  const int64_t kb0 = kbeg / 16;
  const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem);
  const uint32_t lds_wave = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)wave * 1024);
  // wave w copies the 1 KB pieces w of the six 8 KB plane blocks of a K-step (A h, m, l, B h, m, l)
  const char* a_src = im.A + tile.m * XG_BLK + wave * 1024;
  const char* b_src = im.B + tile.n * XG_BLK + wave * 1024;
  auto piece = [&](int t, int q) __attribute__((always_inline)) {  // q: A h, m, l, B h, m, l
    const int64_t kb = kb0 + t;
    const uint32_t dst = lds_wave + (uint32_t)((t % 3) * XG_STAGE + q * XG_BLK);
    if (q < 3) pg_dma(a_src + q * im.a_plane + kb * im.a_kb, dst, lane);
    else pg_dma(b_src + (q - 3) * im.b_plane + kb * im.b_kb, dst, lane);
  };
  auto stage = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 6; ++q) piece(t, q);
  };
  // fragment reads: lane l takes row (l & 15) and 16-B half ((l >> 4) & 1) of the plane its lane
  // half selects; per-lane offsets of each kind (plane byte offset + row/half), A planes at 0..2,
  // B planes at 3..5 blocks of the stage
  const int rowoff = fr * 32 + 16 * ((lane >> 4) & 1);
  const int a_k0 = rowoff + (hi ? 1 : 0) * XG_BLK;                   // A [h | m]
  const int a_k1 = rowoff + (hi ? 2 : 0) * XG_BLK;                   // A [h | l]
  const int b_k0 = rowoff + (3 + (hi ? 0 : 1)) * XG_BLK;             // B [m | h]
  const int b_k1 = rowoff + (3 + (hi ? 0 : 2)) * XG_BLK;             // B [l | h]
  const int b_k2 = rowoff + (3 + (hi ? 1 : 0)) * XG_BLK;             // B [h | m]
  auto rd = [&](const char* base, int off) -> u32x4 { return *reinterpret_cast<const u32x4*>(base + off); };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // does this wave hold any output column (wave-uniform; the last tile column at N = 3,344 has 16)
  const bool live = n0 + wc * 64 < p.N;

  if ((V & 4) && wave >= 4) __builtin_amdgcn_s_setprio(1);
  if (nsteps > 0) stage(0);
  if (nsteps > 1) stage(1);
  for (int t = 0; t < nsteps; ++t) {
    // this K-step's copies have landed once only the next one's (if any) are in flight
    if (t + 1 < nsteps) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's copies of K-step t are in LDS; slot (t + 2) % 3 is free
    const bool more = t + 2 < nsteps;
    if (!(V & 2) && more) stage(t + 2);
    if (V & 1) __builtin_amdgcn_s_setprio(1);
    if (live) {
      const char* S = smem + (t % 3) * XG_STAGE;
      const char* SA = S + (wr * 128) * 32;
      const char* SB = S + (wc * 64) * 32;
      u32x4 b0[4], b1[4], b2[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        b0[j] = rd(SB + j * 512, b_k0);
        b1[j] = rd(SB + j * 512, b_k1);
        b2[j] = rd(SB + j * 512, b_k2);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if ((V & 2) && more && (i == 0 || i == 3 || i == 6)) {
          piece(t + 2, 2 * (i / 3));
          piece(t + 2, 2 * (i / 3) + 1);
        }
        const u32x4 a0 = rd(SA + i * 512, a_k0), a1 = rd(SA + i * 512, a_k1);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[i][j] = mfma16_bf16(a1, b1[j], acc[i][j]);  // h.l + l.h
          acc[i][j] = mfma16_bf16(a0, b0[j], acc[i][j]);  // h.m + m.h
          acc[i][j] = mfma16_bf16(a0, b2[j], acc[i][j]);  // h.h + m.m
        }
      }
    } else if ((V & 2) && more) {
      stage(t + 2);
    }
    if (V & 1) __builtin_amdgcn_s_setprio(0);
  }
  // epilogue: lane holds rows 4 (lane >> 4) + e, column lane & 15 of each 16 x 16 subtile
#pragma clang loop unroll(full)
  for (int j = 0; j < 4; ++j)
#pragma clang loop unroll(full)
    for (int i = 0; i < 8; i += XG_EPI_NI)
      xg_epilogue_col<SPLIT, 0, XG_EPI_NI>(p, acc, j, m0 + wr * 128 + i * 16, n0 + wc * 64 + j * 16 + fr, lane >> 4,
                                           tile.z, i);
}

static XgImgs xg_imgs(const GemmParams& p, const char* Aimg, const char* Bimg) {
  XgImgs im;
  im.A = Aimg;
  im.B = Bimg;
  im.a_kb = xg_rt(p.M) * XG_BLK;
  im.b_kb = xg_rt(p.N) * XG_BLK;
  im.a_plane = xg_kb(p.K) * im.a_kb;
  im.b_plane = xg_kb(p.K) * im.b_kb;
  return im;
}

template <bool SPLIT>
static int xgemm_dispatch(const GemmParams& p, const char* Aimg, const char* Bimg, int64_t S, hipStream_t st) {
  const XgImgs im = xg_imgs(p, Aimg, Bimg);
  dim3 grid((unsigned)xg_rt(p.N), (unsigned)xg_rt(p.M), (unsigned)S);
  const char* ev = exp_env("RS_XGEMM_VAR");
  switch (ev ? atoi(ev) : 0) {
#define RS_XV(v) case v: hipLaunchKernelGGL((xgemm_kernel<SPLIT, v>), grid, dim3(512), 0, st, p, im); break;
    RS_XV(1) RS_XV(2) RS_XV(3) RS_XV(4) RS_XV(5) RS_XV(6) RS_XV(7)
#undef RS_XV
    default: hipLaunchKernelGGL((xgemm_kernel<SPLIT, 0>), grid, dim3(512), 0, st, p, im);
  }
  return check_launch(SPLIT ? "xgemm_splitk" : "xgemm");
}

// C = epilogue(A B^T) from images: A = image of the [M][K] operand, B = image of the [N][K] operand
int xgemm_launch(int64_t M, int64_t N, int64_t K, const char* Aimg, const char* Bimg, float* C, int64_t ldc,
                 const float* bias, int act, int epi, const float* x0, const float* xres, float* aux, int64_t ldx,
                 const float* addend, int64_t ldadd, hipStream_t st, int prec, float beta) {
  RS_REQUIRE(M >= 0 && N >= 0 && K >= 0 && Aimg && Bimg && (C || M * N == 0), "xgemm_launch: bad args");
  RS_REQUIRE(prec == RS_PREC_F32_SPLIT6, "xgemm_launch: precision must be 6");
  if (M == 0 || N == 0) return RS_OK;
  GemmParams p{nullptr, nullptr, C, 0, 0, ldc, M, N, K, bias, act, nullptr, 0, beta, K, nullptr,
               epi, x0, xres, aux, ldx, addend, ldadd, prec};
  return xgemm_dispatch<false>(p, Aimg, Bimg, 1, st);
}

// Tail tiles of a tile-range launch (the last partial round): the K slices' sums in slab order,
// then the xgemm epilogue (bias, DCN-v2 cross update, ReLU, addend, beta C) on them. Block (c, t):
// 16 rows x 64 float4 columns of tail tile t.
__global__ __launch_bounds__(256) void xg_tail_fixup_kernel(GemmParams p, int64_t S) {
  const int64_t t = p.tile_lo + blockIdx.y;
  const GxTile tile = gx_map(t, xg_rt_dev(p.N), xg_rt_dev(p.M));
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), c4 = threadIdx.x & 63;
  const int64_t col = tile.n * 256 + 4 * c4;
  const int64_t stride = p.slab_stride;
#pragma unroll 1
  for (int rr = 0; rr < 4; ++rr) {
    const int64_t row = tile.m * 256 + r * 4 + rr;
    if (row >= p.M || col >= p.N) continue;
    f32x4 v = *reinterpret_cast<const f32x4*>(p.slab + row * p.N + col);
    for (int64_t z = 1; z < S; ++z) v += *reinterpret_cast<const f32x4*>(p.slab + z * stride + row * p.N + col);
    if (p.bias) v += *reinterpret_cast<const f32x4*>(p.bias + col);
    if (p.epi == 1) {
      const int64_t xo = row * p.ldx + col;
      *reinterpret_cast<f32x4*>(p.aux + xo) = v;
      v = *reinterpret_cast<const f32x4*>(p.x0 + xo) * v + *reinterpret_cast<const f32x4*>(p.xres + xo);
    }
    if (p.act == RS_ACT_RELU) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    if (p.addend) v += *reinterpret_cast<const f32x4*>(p.addend + row * p.ldadd + col);
    float* cp = p.C + row * p.ldc + col;
    if (p.beta != 0.f) v += p.beta * *reinterpret_cast<const f32x4*>(cp);
    *reinterpret_cast<f32x4*>(cp) = v;
  }
}

// The last partial round of a large xgemm (tiles % 256 <= 128 past >= 1 full round, K >= 1024,
// N % 4 == 0, 16-B aligned rows) re-run as S K slices (S = 256 / tail tiles), so that round's CUs
// are all busy for 1/S of a tile's time instead of half of them for a whole one; the slices meet
// in an ordered fixup that applies the epilogue. Workspace: xgemm_tail_ws_bytes (0 when not used).
static bool xg_tail_plan(int64_t M, int64_t N, int64_t K, int64_t* T0, int64_t* R, int64_t* S, int64_t* kps) {
  const int64_t tiles = xg_rt(M) * xg_rt(N);
  const int64_t r = tiles % 256;
  if (tiles < 256 || r == 0 || r > 128 || K < 1024 || N % 4 != 0) return false;
  int64_t s = 256 / r;
  if (s > 8) s = 8;
  *kps = ceil_div(ceil_div(K, s), 16) * 16;
  *S = ceil_div(K, *kps);
  *T0 = tiles - r;
  *R = r;
  return true;
}
size_t xgemm_tail_ws_bytes(int64_t M, int64_t N, int64_t K) {
  int64_t T0, R, S, kps;
  if (!xg_tail_plan(M, N, K, &T0, &R, &S, &kps)) return 0;
  return align_up((size_t)S * (size_t)M * (size_t)N * sizeof(float), 256) + 256;
}
int xgemm_launch_ws(int64_t M, int64_t N, int64_t K, const char* Aimg, const char* Bimg, float* C, int64_t ldc,
                    const float* bias, int act, int epi, const float* x0, const float* xres, float* aux, int64_t ldx,
                    const float* addend, int64_t ldadd, hipStream_t st, int prec, float beta, void* ws,
                    size_t wsb) {
  int64_t T0, R, S, kps;
  const bool aligned = ldc % 4 == 0 && (epi != 1 || ldx % 4 == 0) && (!addend || ldadd % 4 == 0) && aligned16(C) &&
                       (!bias || aligned16(bias)) && (!addend || aligned16(addend)) &&
                       (epi != 1 || (aligned16(x0) && aligned16(xres) && aligned16(aux)));
  if (!ws || !aligned || !xg_tail_plan(M, N, K, &T0, &R, &S, &kps) || wsb < xgemm_tail_ws_bytes(M, N, K))
    return xgemm_launch(M, N, K, Aimg, Bimg, C, ldc, bias, act, epi, x0, xres, aux, ldx, addend, ldadd, st, prec,
                        beta);
  RS_REQUIRE(prec == RS_PREC_F32_SPLIT6, "xgemm_launch: precision must be 6");
  GemmParams p{nullptr, nullptr, C, 0, 0, ldc, M, N, K, bias, act, nullptr, 0, beta, K, nullptr,
               epi, x0, xres, aux, ldx, addend, ldadd, prec};
  const XgImgs im = xg_imgs(p, Aimg, Bimg);
  p.tile_lo = 0;
  p.tile_n = T0;
  hipLaunchKernelGGL((xgemm_kernel<false, 0>), dim3((unsigned)T0), dim3(512), 0, st, p, im);
  int rc = check_launch("xgemm");
  if (rc) return rc;
  GemmParams q = p;
  q.tile_lo = T0;
  q.tile_n = R;
  q.k_per_split = kps;
  q.slab = static_cast<float*>(ws);
  q.slab_stride = M * N;
  hipLaunchKernelGGL((xgemm_kernel<true, 0>), dim3((unsigned)(R * S)), dim3(512), 0, st, q, im);
  rc = check_launch("xgemm_tail");
  if (rc) return rc;
  hipLaunchKernelGGL(xg_tail_fixup_kernel, dim3(16, (unsigned)R), dim3(256), 0, st, q, S);
  return check_launch("xgemm_tail_fixup");
}

// K slices for xgemm: one workgroup per CU; minimise rounds x (K / S) + the slab round trip,
// slices of >= 512 contraction rows (multiples of 16)
static int64_t xgemm_splitk_count(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = xg_rt(M) * xg_rt(N);
  int64_t maxs = K / 512;
  if (maxs > 32) maxs = 32;
  int64_t best = 1;
  double best_t = 1e30;
  for (int64_t s = 1; s <= (maxs < 1 ? 1 : maxs); ++s) {
    const double rounds = (double)ceil_div(tiles * s, 256);
    // ~0.11 us per k per round of 256 x 256 tiles (measured: 1.82 ms for K = 16384 at s = 1), plus
    // the slabs' write + read at ~5 TB/s
    const double t = rounds * ((double)K / s) * 1.1e-7 + (s > 1 ? (double)s * M * N * 8.0 / 5e12 : 0.0);
    if (t < best_t * 0.995) {
      best_t = t;
      best = s;
    }
  }
  return best;
}
size_t xgemm_splitk_ws_bytes(int64_t M, int64_t N, int64_t K) {
  return align_up((size_t)xgemm_splitk_count(M, N, K) * (size_t)M * (size_t)N * sizeof(float), 256) + 256;
}
// C = A B^T (+ addend_scale * addend) with the K range split over workgroups, ordered slabs
int xgemm_splitk_launch(int64_t M, int64_t N, int64_t K, const char* Aimg, const char* Bimg, float* C,
                        const float* addend, float addend_scale, int prec, void* ws, size_t ws_bytes, hipStream_t st) {
  RS_REQUIRE(M >= 0 && N >= 0 && K >= 0 && Aimg && Bimg && (C || M * N == 0), "xgemm_splitk_launch: bad args");
  RS_REQUIRE(prec == RS_PREC_F32_SPLIT6, "xgemm_splitk_launch: precision must be 6");
  if (!ws || ws_bytes < xgemm_splitk_ws_bytes(M, N, K)) {
    set_error("xgemm_splitk_launch: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  if (M == 0 || N == 0) return RS_OK;
  const int64_t S = xgemm_splitk_count(M, N, K);
  const int64_t kps = ceil_div(ceil_div(K > 0 ? K : 1, S), 16) * 16;
  const int64_t Seff = K > 0 ? ceil_div(K, kps) : 1;
  float* slab = static_cast<float*>(ws);
  GemmParams p{nullptr, nullptr, C, 0, 0, N, M, N, K, nullptr, 0, nullptr, 0, 0.f, kps, slab,
               0, nullptr, nullptr, nullptr, 0, nullptr, 0, prec};
  const int rc = xgemm_dispatch<true>(p, Aimg, Bimg, Seff, st);
  if (rc) return rc;
  return launch_slab_reduce(slab, Seff, M * N, C, addend, addend_scale, st);
}

// Internal launcher used by the DCN-v2 stack (dcn2.hip): full epilogue control.
int gemm_launch(int ta, int tb, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                const float* B, int64_t ldb, float* C, int64_t ldc, const float* bias, int epi,
                const float* x0, const float* xres, float* aux, int64_t ldx, const float* addend,
                int64_t ldadd, hipStream_t st, int prec, float beta) {
  int rc = validate("gemm_launch", ta, tb, M, N, K, A, lda, B, ldb, C, ldc);
  if (rc) return rc;
  if (M == 0 || N == 0) return RS_OK;
  GemmParams p{A, B, C, lda, ldb, ldc, M, N, K, bias, 0, nullptr, 0, beta, K, nullptr,
               epi, x0, xres, aux, ldx, addend, ldadd, prec};
  return dispatch<false>(ta, tb, p, dim3(1, 1, 1), st);
}

}  // namespace rs

using namespace rs;

extern "C" {

int rs_gemm_prec_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, const float* A,
                     int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                     const float* bias, int activation, const float* mask, int64_t ldm, float beta,
                     int precision, rs_stream_t stream) {
  int rc = validate("rs_gemm_f32", trans_a, trans_b, M, N, K, A, lda, B, ldb, C, ldc);
  if (rc) return rc;
  RS_REQUIRE(activation == RS_ACT_NONE || activation == RS_ACT_RELU, "rs_gemm_f32: bad activation");
  RS_REQUIRE(!mask || ldm >= N, "rs_gemm_f32: ldm too small");
  RS_REQUIRE(precision == RS_PREC_F32 || precision == RS_PREC_F32_SPLIT6 || precision == RS_PREC_F32_SPLIT9,
             "rs_gemm_f32: precision must be 0, 6 or 9");
  if (M == 0 || N == 0) return RS_OK;
  GemmParams p{A, B, C, lda, ldb, ldc, M, N, K, bias, activation, mask, ldm, beta, K, nullptr,
               0, nullptr, nullptr, nullptr, 0, nullptr, 0, precision};
  return dispatch<false>(trans_a, trans_b, p, dim3(1, 1, 1), as_stream(stream));
}

int rs_gemm_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, const float* A,
                int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                const float* bias, int activation, const float* mask, int64_t ldm, float beta,
                rs_stream_t stream) {
  return rs_gemm_prec_f32(trans_a, trans_b, M, N, K, A, lda, B, ldb, C, ldc, bias, activation, mask, ldm, beta,
                          RS_PREC_F32, stream);
}

size_t rs_plane_image_bytes(int64_t k_extent, int64_t extent) { return pimg_bytes(k_extent, extent); }

int rs_plane_image_f32(const float* X, int64_t ldx, int64_t rows, int64_t cols, int layout, void* img,
                       rs_stream_t stream) {
  RS_REQUIRE(rows > 0 && cols > 0 && ldx >= cols && (layout == 0 || layout == 1) && X && img,
             "rs_plane_image_f32: bad args");
  RS_REQUIRE(aligned16(X) && aligned16(img) && ldx % 4 == 0, "rs_plane_image_f32: 16-byte alignment");
  return plane_image_launch(X, ldx, rows, cols, layout, static_cast<char*>(img), as_stream(stream));
}

int rs_gemm_planes_prec_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, const void* Aimg,
                            const void* Bimg, float* C, int64_t ldc, const float* bias, int activation,
                            float beta, int precision, rs_stream_t stream) {
  RS_REQUIRE(ldc >= N, "rs_gemm_planes_prec_f32: ldc too small");
  RS_REQUIRE(activation == RS_ACT_NONE || activation == RS_ACT_RELU, "rs_gemm_planes_prec_f32: bad activation");
  RS_REQUIRE(precision == RS_PREC_F32_SPLIT6 || precision == RS_PREC_F32_SPLIT9,
             "rs_gemm_planes_prec_f32: precision must be 6 or 9");
  if (M == 0 || N == 0) return RS_OK;
  RS_REQUIRE(Aimg && Bimg && C, "rs_gemm_planes_prec_f32: null");
  GemmParams p{nullptr, nullptr, C, 0, 0, ldc, M, N, K, bias, activation, nullptr, 0, beta, K, nullptr,
               0, nullptr, nullptr, nullptr, 0, nullptr, 0, precision};
  return pgemm_dispatch<false>(trans_a, trans_b, p, static_cast<const char*>(Aimg), static_cast<const char*>(Bimg),
                               1, as_stream(stream));
}

size_t rs_gemm_planes_splitk_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  return pgemm_splitk_ws_bytes(M, N, K);
}

int rs_gemm_planes_splitk_prec_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, const void* Aimg,
                                   const void* Bimg, float* C, const float* addend, float addend_scale,
                                   int precision, void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  return pgemm_splitk_launch(trans_a, trans_b, M, N, K, static_cast<const char*>(Aimg),
                             static_cast<const char*>(Bimg), C, addend, addend_scale, precision, workspace,
                             workspace_bytes, as_stream(stream));
}

size_t rs_xgemm_image_bytes(int64_t rows, int64_t k_extent) { return ximg_bytes(rows, k_extent); }

int rs_xgemm_image_f32(const float* X, int64_t ldx, int64_t rows, int64_t k_extent, int trans, void* img,
                       rs_stream_t stream) {
  RS_REQUIRE(rows > 0 && k_extent > 0 && X && img && (trans == 0 || trans == 1), "rs_xgemm_image_f32: bad args");
  RS_REQUIRE(ldx >= (trans ? rows : k_extent), "rs_xgemm_image_f32: ldx too small");
  RS_REQUIRE(aligned16(img) && (trans || (aligned16(X) && ldx % 4 == 0)), "rs_xgemm_image_f32: 16-byte alignment");
  return ximg_launch(X, ldx, rows, k_extent, trans, static_cast<char*>(img), as_stream(stream));
}

size_t rs_xgemm_image_dual_workspace_bytes(int64_t rows, int64_t k_extent) {
  return align_up((size_t)xg_rt(rows) * (size_t)(k_extent > 0 ? k_extent : 1) * sizeof(float), 256) + 256;
}

int rs_xgemm_image_dual_f32(const float* X, const float* relu_y, int64_t rows, int64_t k_extent, void* img,
                            void* img_t, float* colsum, void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(rows > 0 && k_extent > 0 && k_extent % 4 == 0 && X && img && img_t, "rs_xgemm_image_dual_f32: bad args");
  RS_REQUIRE(aligned16(X) && aligned16(img) && aligned16(img_t) && (!relu_y || aligned16(relu_y)),
             "rs_xgemm_image_dual_f32: 16-byte alignment");
  hipStream_t st = as_stream(stream);
  if (!relu_y && !colsum)
    return ximg_dual_launch(X, nullptr, nullptr, nullptr, nullptr, rows, k_extent, static_cast<char*>(img),
                            static_cast<char*>(img_t), nullptr, st);
  if (!workspace || workspace_bytes < rs_xgemm_image_dual_workspace_bytes(rows, k_extent)) {
    set_error("rs_xgemm_image_dual_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  float* part = static_cast<float*>(workspace);
  int rc = ximg_dual_launch(X, relu_y, nullptr, nullptr, nullptr, rows, k_extent, static_cast<char*>(img),
                            static_cast<char*>(img_t), part, st);
  if (rc || !colsum) return rc;
  return launch_slab_reduce(part, xg_rt(rows), k_extent, colsum, nullptr, 0.f, st);
}

int rs_xgemm_prec_f32(int64_t M, int64_t N, int64_t K, const void* Aimg, const void* Bimg, float* C, int64_t ldc,
                      const float* bias, int activation, float beta, int precision, rs_stream_t stream) {
  RS_REQUIRE(ldc >= N, "rs_xgemm_prec_f32: ldc too small");
  RS_REQUIRE(activation == RS_ACT_NONE || activation == RS_ACT_RELU, "rs_xgemm_prec_f32: bad activation");
  return xgemm_launch(M, N, K, static_cast<const char*>(Aimg), static_cast<const char*>(Bimg), C, ldc, bias,
                      activation, 0, nullptr, nullptr, nullptr, 0, nullptr, 0, as_stream(stream), precision, beta);
}

size_t rs_xgemm_splitk_workspace_bytes(int64_t M, int64_t N, int64_t K) { return xgemm_splitk_ws_bytes(M, N, K); }

int rs_xgemm_splitk_prec_f32(int64_t M, int64_t N, int64_t K, const void* Aimg, const void* Bimg, float* C,
                             const float* addend, float addend_scale, int precision, void* workspace,
                             size_t workspace_bytes, rs_stream_t stream) {
  return xgemm_splitk_launch(M, N, K, static_cast<const char*>(Aimg), static_cast<const char*>(Bimg), C, addend,
                             addend_scale, precision, workspace, workspace_bytes, as_stream(stream));
}

size_t rs_gemm_splitk_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  return align_up((size_t)splitk_count(M, N, K) * (size_t)M * (size_t)N * sizeof(float), 256) + 256;
}

int rs_gemm_splitk_prec_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                            const float* A, int64_t lda, const float* B, int64_t ldb, float* C,
                            int64_t ldc, const float* addend, float addend_scale, int precision,
                            void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  int rc = validate("rs_gemm_splitk_f32", trans_a, trans_b, M, N, K, A, lda, B, ldb, C, ldc);
  if (rc) return rc;
  RS_REQUIRE(ldc == N, "rs_gemm_splitk_f32: C must be dense (ldc == N)");
  RS_REQUIRE(precision == RS_PREC_F32 || precision == RS_PREC_F32_SPLIT6 || precision == RS_PREC_F32_SPLIT9,
             "rs_gemm_splitk_f32: precision must be 0, 6 or 9");
  if (!workspace || workspace_bytes < rs_gemm_splitk_workspace_bytes(M, N, K)) {
    set_error("rs_gemm_splitk_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  if (M == 0 || N == 0) return RS_OK;
  hipStream_t st = as_stream(stream);
  const int64_t S = splitk_count(M, N, K);
  int64_t kps = ceil_div(ceil_div(K > 0 ? K : 1, S), GEMM_BK) * GEMM_BK;
  const int64_t Seff = K > 0 ? ceil_div(K, kps) : 1;
  float* slab = static_cast<float*>(workspace);
  GemmParams p{A, B, C, lda, ldb, ldc, M, N, K, nullptr, 0, nullptr, 0, 0.f, kps, slab,
               0, nullptr, nullptr, nullptr, 0, nullptr, 0, precision};
  rc = dispatch<true>(trans_a, trans_b, p, dim3(1, 1, (unsigned)Seff), st);
  if (rc) return rc;
  return launch_slab_reduce(slab, Seff, M * N, C, addend, addend_scale, st);
}

// split-operand weight gradients compute the bias row by column sums (colsum_row); the f32
// kernels keep the all-ones row of X^T
static bool wgrad_colsum(int precision) { return precision == RS_PREC_F32_SPLIT6 || precision == RS_PREC_F32_SPLIT9; }
static int64_t wgrad_splits(int64_t M, int64_t N, int64_t K, int precision) {
  return wgrad_colsum(precision) ? splitk_count(M, N, K) : splitk_count(M + 1, N, K);
}

// The large-batch dW kernel (gemm_ws.hip) when the shapes fit: the slices grow to a multiple of its
// 64-row chunk (never more slices than the workspace holds). Sets *seff to its slice count.
static bool wgrad_ws_try(const GemmParams& p, int64_t kps, int64_t* seff, hipStream_t st) {
  static const bool no_ws = exp_env("RS_GEMM_NO_WS") != nullptr;  // A/B switch (timing)
#ifdef RS_NO_WGWS  // A/B build: the gemm_x3 split-K weight gradients
  return false;
#endif
  if (no_ws || !wgrad_ws_ok(p)) return false;
  GemmParams q = p;
  q.k_per_split = wgrad_ws_kps(p, kps);  // >= kps rows: no more slices than the workspace holds
  *seff = ceil_div(p.K, q.k_per_split);
  wgrad_ws_dispatch(q, *seff, st);
  return true;
}

size_t rs_gemm_wgrad_bias_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  const int64_t s = std::max(wgrad_splits(M, N, K, RS_PREC_F32), wgrad_splits(M, N, K, RS_PREC_F32_SPLIT6));
  return std::max(rs_gemm_splitk_workspace_bytes(M + 1, N, K),
                  align_up((size_t)s * (size_t)(M + 1) * (size_t)N * sizeof(float), 256) + 256);
}

int rs_gemm_wgrad_bias_prec_f32(int64_t M, int64_t N, int64_t K, const float* X, int64_t ldx, const float* G,
                                int64_t ldg, float* dWdb, const float* W, float w_scale, const float* w_dscale,
                                int precision, void* workspace, size_t workspace_bytes, rs_stream_t stream,
                                void* queue) {
  int rc = validate("rs_gemm_wgrad_bias_prec_f32", 1, 0, M, N, K, X, ldx, G, ldg, dWdb, N);
  if (rc) return rc;
  RS_REQUIRE(precision == RS_PREC_F32 || precision == RS_PREC_F32_SPLIT6 || precision == RS_PREC_F32_SPLIT9,
             "rs_gemm_wgrad_bias_prec_f32: precision must be 0, 6 or 9");
  if (!workspace || workspace_bytes < rs_gemm_wgrad_bias_workspace_bytes(M, N, K)) {
    set_error("rs_gemm_wgrad_bias_prec_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  if (N == 0) return RS_OK;
  hipStream_t st = as_stream(stream);
  const int64_t M1 = M + 1;  // slab row M: the column sums of G (the bias gradient)
  const int64_t S = wgrad_splits(M, N, K, precision);
  int64_t kps = ceil_div(ceil_div(K > 0 ? K : 1, S), GEMM_BK) * GEMM_BK;
  int64_t Seff = K > 0 ? ceil_div(K, kps) : 1;
  float* slab = static_cast<float*>(workspace);
  GemmParams p{X, G, dWdb, ldx, ldg, N, M1, N, K, nullptr, 0, nullptr, 0, 0.f, kps, slab,
               0, nullptr, nullptr, nullptr, 0, nullptr, 0, precision, M + 1};
  if (wgrad_colsum(precision)) {  // M rows of X^T; the split kernels sum G's columns into row M
    p.M = M;
    p.ones_row1 = 0;
    p.colsum_row = M;
    p.slab_stride = M1 * N;
  }
  int64_t Seff_ws = Seff;
  if (wgrad_ws_try(p, kps, &Seff_ws, st)) {
    rc = check_launch("wgrad_ws");
    Seff = Seff_ws;
  } else {
    rc = dispatch<true>(1, 0, p, dim3(1, 1, (unsigned)Seff), st);
  }
  if (rc) return rc;
  // dW (rows 0..M-1) += w_scale * (*w_dscale) * W: the l2 kernel-regularizer gradient
  return launch_slab_reduce_strided(slab, Seff, M1 * N, M1 * N, dWdb, W, w_scale, st, w_dscale, W ? M * N : 0,
                                    static_cast<SlabQueue*>(queue));
}

int rs_gemm_group_prec_f32(int ngroup, int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                           const float* const* A, int64_t lda, const float* const* B, int64_t ldb, float* const* C,
                           int64_t ldc, const float* const* bias, int activation, const float* const* mask,
                           int64_t ldm, float beta, int precision, rs_stream_t stream) {
  return rs_gemm_group_img_prec_f32(ngroup, trans_a, trans_b, M, N, K, A, lda, B, ldb, C, ldc, bias, activation,
                                    mask, ldm, beta, precision, nullptr, stream);
}

static int gemm_group_impl(int ngroup, int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                           const float* const* A, int64_t lda, const float* const* B, int64_t ldb,
                           float* const* C, int64_t ldc, const float* const* bias, int activation,
                           const float* const* mask, int64_t ldm, float beta, int precision,
                           const void* const* b_img, const int32_t* const* mask_rows, const int64_t* const* m_dev,
                           rs_stream_t stream, const int32_t* const* a_rows = nullptr) {
  RS_REQUIRE(ngroup >= 1 && ngroup <= GEMM_GMAX && A && B && C, "rs_gemm_group_prec_f32: 1..%d problems",
             GEMM_GMAX);
  for (int g = 0; g < ngroup; ++g) {
    int rc = validate("rs_gemm_group_prec_f32", trans_a, trans_b, M, N, K, A[g], lda, B[g], ldb, C[g], ldc);
    if (rc) return rc;
  }
  RS_REQUIRE(activation == RS_ACT_NONE || activation == RS_ACT_RELU, "rs_gemm_group_prec_f32: bad activation");
  RS_REQUIRE(!mask || ldm >= N, "rs_gemm_group_prec_f32: ldm too small");
  RS_REQUIRE(precision == RS_PREC_F32 || precision == RS_PREC_F32_SPLIT6 || precision == RS_PREC_F32_SPLIT9,
             "rs_gemm_group_prec_f32: precision must be 0, 6 or 9");
  if (M == 0 || N == 0) return RS_OK;
  GemmParams p{A[0], B[0], C[0], lda, ldb, ldc, M, N, K, bias ? bias[0] : nullptr, activation,
               mask ? mask[0] : nullptr, ldm, beta, K, nullptr, 0, nullptr, nullptr, nullptr, 0, nullptr, 0,
               precision};
  p.ngroup = ngroup;
  p.zper = 1;
  for (int g = 0; g < ngroup; ++g) {
    p.gA[g] = A[g];
    p.gB[g] = B[g];
    p.gC[g] = C[g];
    p.gbias[g] = bias ? bias[g] : nullptr;
    p.gmask[g] = mask ? mask[g] : nullptr;
    p.gbimg[g] = b_img ? static_cast<const char*>(b_img[g]) : nullptr;
    RS_REQUIRE(!p.gbimg[g] || aligned16(p.gbimg[g]), "rs_gemm_group_img_prec_f32: image %d not 16-byte aligned", g);
  }
  // an image serves every problem or none (the kernels select per problem)
  for (int g = 1; g < ngroup; ++g)
    RS_REQUIRE(!p.gbimg[g] == !p.gbimg[0], "rs_gemm_group_img_prec_f32: images for some problems only");
  p.bimg = p.gbimg[0];
  if (mask_rows || m_dev || a_rows) {  // the distinct-row layers run on the weight-stationary kernel only
    for (int g = 0; g < ngroup; ++g) {
      p.gmrow[g] = mask_rows ? mask_rows[g] : nullptr;
      p.gmdev[g] = m_dev ? m_dev[g] : nullptr;
      p.garow[g] = a_rows ? a_rows[g] : nullptr;
      RS_REQUIRE(!a_rows || p.garow[g], "rs_gemm_group_rows_prec_f32: null A row map");
      RS_REQUIRE(!mask_rows || !mask || p.gmrow[g], "rs_gemm_group_rows_prec_f32: null mask row map");
    }
    p.mrow = mask ? p.gmrow[0] : nullptr;
    for (int g = 0; g < ngroup && !mask; ++g) p.gmrow[g] = nullptr;
    p.mdev = p.gmdev[0];
    p.arow = p.garow[0];
    if (!ws_ok(trans_a, trans_b, p)) {
      set_error("rs_gemm_group_rows_prec_f32: shape outside the weight-stationary kernel (precision 6 / 9, "
                "K and N in {64, 128, 256}, >= 32768 rows, no addend / beta, 16-B aligned rows)");
      return RS_ERR_UNSUPPORTED;
    }
    ws_dispatch(trans_b, p, as_stream(stream));
    return check_launch("gemm_ws");
  }
  return dispatch<false>(trans_a, trans_b, p, dim3(1, 1, (unsigned)ngroup), as_stream(stream));
}

int rs_gemm_group_img_prec_f32(int ngroup, int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                               const float* const* A, int64_t lda, const float* const* B, int64_t ldb,
                               float* const* C, int64_t ldc, const float* const* bias, int activation,
                               const float* const* mask, int64_t ldm, float beta, int precision,
                               const void* const* b_img, rs_stream_t stream) {
  return gemm_group_impl(ngroup, trans_a, trans_b, M, N, K, A, lda, B, ldb, C, ldc, bias, activation, mask, ldm, beta,
                         precision, b_img, nullptr, nullptr, stream);
}

int rs_gemm_group_rows_prec_f32(int ngroup, int trans_b, int64_t M, int64_t N, int64_t K, const float* const* A,
                                int64_t lda, const int32_t* const* a_rows, const float* const* B, int64_t ldb,
                                float* const* C, int64_t ldc, const float* const* bias, int activation,
                                const float* const* mask, int64_t ldm, const int32_t* const* mask_rows,
                                const int64_t* const* m_dev, int precision, rs_stream_t stream) {
  RS_REQUIRE(mask_rows || m_dev || a_rows, "rs_gemm_group_rows_prec_f32: no row map and no device row count");
  return gemm_group_impl(ngroup, 0, trans_b, M, N, K, A, lda, B, ldb, C, ldc, bias, activation, mask, ldm, 0.f,
                         precision, nullptr, mask_rows, m_dev, stream, a_rows);
}

size_t rs_gemm_wgrad_bias_group_workspace_bytes(int ngroup, int64_t M, int64_t N, int64_t K) {
  const int64_t M1 = M + 1;
  const int64_t s = std::max(wgrad_splits(M, N, K, RS_PREC_F32), wgrad_splits(M, N, K, RS_PREC_F32_SPLIT6));
  return align_up((size_t)ngroup * s * (size_t)M1 * (size_t)N * sizeof(float), 256) + 256;
}

static int wgrad_group_impl(int ngroup, int64_t M, int64_t N, int64_t K, const float* const* X, int64_t ldx,
                            const int32_t* const* x_rows, const float* const* G, int64_t ldg, float* dWdb,
                            int precision, void* workspace, size_t workspace_bytes, rs_stream_t stream, void* queue);

int rs_gemm_wgrad_bias_group_prec_f32(int ngroup, int64_t M, int64_t N, int64_t K, const float* const* X,
                                      int64_t ldx, const float* const* G, int64_t ldg, float* dWdb, int precision,
                                      void* workspace, size_t workspace_bytes, rs_stream_t stream, void* queue) {
  return wgrad_group_impl(ngroup, M, N, K, X, ldx, nullptr, G, ldg, dWdb, precision, workspace, workspace_bytes,
                          stream, queue);
}

int rs_gemm_wgrad_bias_group_rows_prec_f32(int ngroup, int64_t M, int64_t N, int64_t K, const float* const* X,
                                           int64_t ldx, const int32_t* const* x_rows, const float* const* G,
                                           int64_t ldg, float* dWdb, int precision, void* workspace,
                                           size_t workspace_bytes, rs_stream_t stream, void* queue) {
  RS_REQUIRE(x_rows, "rs_gemm_wgrad_bias_group_rows_prec_f32: null row maps");
  RS_REQUIRE(precision == RS_PREC_F32_SPLIT6 || precision == RS_PREC_F32_SPLIT9,
             "rs_gemm_wgrad_bias_group_rows_prec_f32: precision must be 6 or 9");
  for (int g = 0; g < ngroup; ++g)
    RS_REQUIRE(x_rows[g], "rs_gemm_wgrad_bias_group_rows_prec_f32: null row map %d", g);
  return wgrad_group_impl(ngroup, M, N, K, X, ldx, x_rows, G, ldg, dWdb, precision, workspace, workspace_bytes,
                          stream, queue);
}

static int wgrad_group_impl(int ngroup, int64_t M, int64_t N, int64_t K, const float* const* X, int64_t ldx,
                            const int32_t* const* x_rows, const float* const* G, int64_t ldg, float* dWdb,
                            int precision, void* workspace, size_t workspace_bytes, rs_stream_t stream, void* queue) {
  RS_REQUIRE(ngroup >= 1 && ngroup <= GEMM_GMAX && X && G, "rs_gemm_wgrad_bias_group_prec_f32: 1..%d problems",
             GEMM_GMAX);
  for (int g = 0; g < ngroup; ++g) {
    int rc = validate("rs_gemm_wgrad_bias_group_prec_f32", 1, 0, M, N, K, X[g], ldx, G[g], ldg, dWdb, N);
    if (rc) return rc;
  }
  RS_REQUIRE(precision == RS_PREC_F32 || precision == RS_PREC_F32_SPLIT6 || precision == RS_PREC_F32_SPLIT9,
             "rs_gemm_wgrad_bias_group_prec_f32: precision must be 0, 6 or 9");
  if (!workspace || workspace_bytes < rs_gemm_wgrad_bias_group_workspace_bytes(ngroup, M, N, K)) {
    set_error("rs_gemm_wgrad_bias_group_prec_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  if (N == 0) return RS_OK;
  hipStream_t st = as_stream(stream);
  const int64_t M1 = M + 1;  // row M of each problem: the column sums of G (the bias gradient)
  const int64_t S = wgrad_splits(M, N, K, precision);
  int64_t kps = ceil_div(ceil_div(K > 0 ? K : 1, S), GEMM_BK) * GEMM_BK;
  int64_t Seff = K > 0 ? ceil_div(K, kps) : 1;
  // slab layout [slice][problem][M1 N]: one ordered reduction over all problems writes the
  // contiguous [problem][M1][N] output with each problem's sums exactly those of its own launch
  float* slab = static_cast<float*>(workspace);
  GemmParams p{X[0], G[0], dWdb, ldx, ldg, N, M1, N, K, nullptr, 0, nullptr, 0, 0.f, kps, slab,
               0, nullptr, nullptr, nullptr, 0, nullptr, 0, precision, M + 1};
  p.slab_stride = (int64_t)ngroup * M1 * N;
  p.ngroup = ngroup;
  p.zper = Seff;
  if (wgrad_colsum(precision)) {
    p.M = M;
    p.ones_row1 = 0;
    p.colsum_row = M;
  }
  for (int g = 0; g < ngroup; ++g) {
    p.gA[g] = X[g];
    p.gB[g] = G[g];
    p.gC[g] = dWdb + (int64_t)g * M1 * N;
    p.gslab[g] = slab + (int64_t)g * M1 * N;
    p.garow[g] = x_rows ? x_rows[g] : nullptr;
  }
  p.arow = p.garow[0];
  int64_t Seff_ws = Seff;
  int rc;
  if (wgrad_ws_try(p, kps, &Seff_ws, st)) {
    rc = check_launch("wgrad_ws");
    Seff = Seff_ws;
  } else {
    rc = dispatch<true>(1, 0, p, dim3(1, 1, (unsigned)(ngroup * Seff)), st);
  }
  if (rc) return rc;
  return launch_slab_reduce_strided(slab, Seff, p.slab_stride, p.slab_stride, dWdb, nullptr, 0.f, st, nullptr, -1,
                                    static_cast<SlabQueue*>(queue));
}

int rs_gemm_splitk_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                       const float* A, int64_t lda, const float* B, int64_t ldb, float* C,
                       int64_t ldc, const float* addend, float addend_scale, void* workspace,
                       size_t workspace_bytes, rs_stream_t stream) {
  return rs_gemm_splitk_prec_f32(trans_a, trans_b, M, N, K, A, lda, B, ldb, C, ldc, addend, addend_scale,
                                 RS_PREC_F32, workspace, workspace_bytes, stream);
}

}  // extern "C"
