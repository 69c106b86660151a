// mlp.hip — a whole Dense stack in ONE launch per direction (the towers / the DCN deep net at small
// batches, where each per-layer GEMM launch is ~10 us of mostly fixed cost: C2's 4096 rows).
//
// Forward (rs_mlp_fwd_prec_f32) replaces the per-layer keras.layers.Dense forward
// (src/models.py:26-29,76-77) of MLPFn / MLPGroupFn: y_l = act_l(y_{l-1} W_l + b_l), y_0 = x,
// every y_l written (the backward's masks and weight-gradient operands). The backward's input-
// gradient chain (rs_mlp_bwd_chain_prec_f32) is the same machine run down the stack: g_{l-1} =
// (g_l W_l^T) masked by y_{l-1} > 0 (TF's ReluGrad of layer l - 1), every g_{l-1} written (the
// weight gradients' operands), ending in dL/dx = g_0 W_0^T.
//
// A 256-thread workgroup owns 32 rows of one stack and carries them through every stage: the rows
// live in LDS as exact three-term bf16 split planes (split.hpp; the 16-B chunks of a row XOR-
// swizzled by the row, so the 16x16x32 A-fragment reads are conflict-free), each wave computes all
// 32 rows x N/4 columns of a stage on v_mfma_f32_16x16x32_bf16 with the weights' fragments loaded
// from L2 (split in registers, the next 32-k chunk's loads in flight during this chunk's MFMAs),
// and the epilogue adds the bias, applies the ReLU or the mask, stores the stage's output and
// writes its split planes into the other LDS buffer for the next stage. Same split products as
// the per-layer GEMMs (mfma16_split_n); the order of the k additions differs.
#include "common.hpp"
#include "split.hpp"
#include <type_traits>

namespace rs {

constexpr int MLP_MAXL = 6, MLP_MAXG = 2, MLP_ROWS = 32;

struct MlpStage {
  const float* W[MLP_MAXG];     // [K][N] (forward) or [N][K] (the chain: W_l read transposed)
  const float* b[MLP_MAXG];     // bias [N] or null
  const float* mask[MLP_MAXG];  // [M][N]: output zeroed where mask <= 0, or null
  float* y[MLP_MAXG];           // [M][N] output, or null (not stored)
  int K, N, relu;
};
struct MlpParams {
  const float* x[MLP_MAXG];
  MlpStage s[MLP_MAXL];
  int L;
  int64_t M;
};

// element (row, k) of a 32 x 256 plane: 16-B chunk k / 8 swizzled by the row
__device__ __forceinline__ int mlp_off(int row, int k) { return row * 256 + ((((k >> 3) ^ row) & 31) << 3) + (k & 7); }

__device__ __forceinline__ void mlp_split1(float v, uint16_t& h, uint16_t& m, uint16_t& l) {
  const __bf16 bh = (__bf16)v;
  const float rh = v - (float)bh;
  const __bf16 bm = (__bf16)rh;
  const __bf16 bl = (__bf16)(rh - (float)bm);
  h = __builtin_bit_cast(uint16_t, bh);
  m = __builtin_bit_cast(uint16_t, bm);
  l = __builtin_bit_cast(uint16_t, bl);
}

template <typename T>
__device__ __forceinline__ T mlp_pick(const T (&a)[MLP_MAXG], int st) {
  T r = a[0];
#pragma unroll
  for (int i = 1; i < MLP_MAXG; ++i)
    if (st == i) r = a[i];
  return r;
}

// TRANS: the stage's B operand is W^T (the chain), so a lane's 8 k-consecutive weights are
// contiguous in memory (two 16-B loads) instead of a column walk
template <int NP, bool TRANS>
__global__ __launch_bounds__(256, 1) void mlp_chain_kernel(MlpParams p) {
  __shared__ __attribute__((aligned(16))) uint16_t act[2][3][MLP_ROWS * 256];  // 96 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  const int st = (int)blockIdx.y;
  const float* __restrict__ X = mlp_pick(p.x, st);
  const int64_t r0 = (int64_t)blockIdx.x * MLP_ROWS;
  const int64_t M = p.M;

  // the input rows, split into buffer 0 (rows past M are zero)
  {
    const int K0 = p.s[0].K, q = K0 / 4;
    for (int idx = tid; idx < MLP_ROWS * q; idx += 256) {
      const int row = idx / q, k = 4 * (idx - row * q);
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (r0 + row < M) v = *reinterpret_cast<const f32x4*>(X + (r0 + row) * K0 + k);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        uint16_t h, m, l;
        mlp_split1(v[e], h, m, l);
        const int o = mlp_off(row, k + e);
        act[0][0][o] = h;
        act[0][1][o] = m;
        act[0][2][o] = l;
      }
    }
  }
  __syncthreads();

  int cur = 0;
  for (int layer = 0; layer < p.L; ++layer) {
    const int K = p.s[layer].K, N = p.s[layer].N;
    const int nt = N / 64;  // 16-column tiles per wave (1, 2 or 4)
    const int c0 = wave * (N / 4);
    const float* __restrict__ W = mlp_pick(p.s[layer].W, st);
    const float* __restrict__ bias = mlp_pick(p.s[layer].b, st);
    const float* __restrict__ mask = mlp_pick(p.s[layer].mask, st);
    float* __restrict__ Y = mlp_pick(p.s[layer].y, st);
    f32x4 acc[2][4];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    // weight fragment of tile t, chunk c: B[32 c + 8 g + j][c0 + 16 t + i16], j < 8 (tiles past nt
    // read tile 0 and are never used); B = W, or W^T with W [N][K]
    float wf[2][4][8];
    auto wload = [&](int c, auto BUFI) __attribute__((always_inline)) {
      constexpr int bufi = decltype(BUFI)::value;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int tt = t < nt ? t : 0;
        if constexpr (TRANS) {
          const f32x4* src = reinterpret_cast<const f32x4*>(W + (int64_t)(c0 + 16 * tt + i16) * K + 32 * c + 8 * g);
          const f32x4 lo = src[0], hi = src[1];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            wf[bufi][t][j] = lo[j];
            wf[bufi][t][4 + j] = hi[j];
          }
        } else {
          const float* src = W + (int64_t)(32 * c + 8 * g) * N + c0 + 16 * tt + i16;
#pragma unroll
          for (int j = 0; j < 8; ++j) wf[bufi][t][j] = src[(int64_t)j * N];
        }
      }
    };
    const int nch = K / 32;
    // one 32-k chunk with the weight buffer index a compile-time constant (a run-time index would
    // send wf to LDS)
    auto chunk = [&](int c, auto BI) __attribute__((always_inline)) {
      constexpr int bi = decltype(BI)::value;
      // A fragments of both 16-row tiles from LDS: row 16 rt + i16, k 32 c + 8 g .. + 7
      u32x4 ap[2][3];
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          ap[rt][pl] = *reinterpret_cast<const u32x4*>(&act[cur][pl][mlp_off(16 * rt + i16, 32 * c + 8 * g)]);
      if (c + 1 < nch) wload(c + 1, std::integral_constant<int, bi ^ 1>{});
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (t < nt) {
          u32x4 bp[3];
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const IbSplit s = ib_split2(wf[bi][t][2 * w], wf[bi][t][2 * w + 1]);
            bp[0][w] = s.h;
            bp[1][w] = s.m;
            bp[2][w] = s.l;
          }
          const u32x4* const aa[2] = {ap[0], ap[1]};
          const u32x4* const bb[2] = {bp, bp};
          f32x4* const cc[2] = {&acc[0][t], &acc[1][t]};
          mfma16_split_n<NP, 2>(aa, bb, cc);
        }
      }
    };
    wload(0, std::integral_constant<int, 0>{});
    for (int c = 0; c < nch; c += 2) {
      chunk(c, std::integral_constant<int, 0>{});
      if (c + 1 < nch) chunk(c + 1, std::integral_constant<int, 1>{});
    }
    // epilogue: D[row 16 rt + 4 g + r][col c0 + 16 t + i16]
    const bool relu = p.s[layer].relu != 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t < nt) {
        const int n = c0 + 16 * t + i16;
        const float bv = bias ? bias[n] : 0.f;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * rt + 4 * g + r;
            const bool live = r0 + row < M;
            float v = acc[rt][t][r] + bv;
            if (relu) v = fmaxf(v, 0.f);
            if (mask && live && !(mask[(r0 + row) * N + n] > 0.f)) v = 0.f;
            if (Y && live) Y[(r0 + row) * N + n] = v;
            if (layer + 1 < p.L) {
              uint16_t h, m, l;
              mlp_split1(live ? v : 0.f, h, m, l);
              const int o = mlp_off(row, n);
              act[cur ^ 1][0][o] = h;
              act[cur ^ 1][1][o] = m;
              act[cur ^ 1][2][o] = l;
            }
          }
      }
    }
    __syncthreads();
    cur ^= 1;
  }
}

int mlp_launch(MlpParams& p, int G, bool trans, int precision, rs_stream_t stream) {
  if (p.M == 0) return RS_OK;
  const dim3 grid((unsigned)ceil_div(p.M, MLP_ROWS), (unsigned)G);
  hipStream_t st = as_stream(stream);
  if (precision == RS_PREC_F32_SPLIT6) {
    if (trans) hipLaunchKernelGGL((mlp_chain_kernel<6, true>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((mlp_chain_kernel<6, false>), grid, dim3(256), 0, st, p);
  } else {
    if (trans) hipLaunchKernelGGL((mlp_chain_kernel<9, true>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((mlp_chain_kernel<9, false>), grid, dim3(256), 0, st, p);
  }
  return check_launch(trans ? "mlp_bwd_chain" : "mlp_fwd");
}

bool mlp_width_ok(int64_t n) { return n == 64 || n == 128 || n == 256; }

}  // namespace rs

using namespace rs;

extern "C" {

int rs_mlp_fwd_prec_f32(int G, int L, const int64_t* dims, int64_t M, const float* const* x, const float* const* W,
                        const float* const* b, const int* relu, float* const* y, int precision, rs_stream_t stream) {
  RS_REQUIRE(G >= 1 && G <= MLP_MAXG && L >= 1 && L <= MLP_MAXL && dims && x && W && y && relu,
             "rs_mlp_fwd_prec_f32: 1..%d stacks of 1..%d layers", MLP_MAXG, MLP_MAXL);
  RS_REQUIRE(precision == RS_PREC_F32_SPLIT6 || precision == RS_PREC_F32_SPLIT9,
             "rs_mlp_fwd_prec_f32: precision must be 6 or 9");
  RS_REQUIRE(M >= 0, "rs_mlp_fwd_prec_f32: M < 0");
  RS_REQUIRE(dims[0] >= 32 && dims[0] <= 256 && dims[0] % 32 == 0, "rs_mlp_fwd_prec_f32: input width %lld",
             (long long)dims[0]);
  MlpParams p{};
  p.L = L;
  p.M = M;
  for (int l = 0; l < L; ++l) {
    RS_REQUIRE(mlp_width_ok(dims[l + 1]), "rs_mlp_fwd_prec_f32: layer %d width %lld (64, 128 or 256)", l,
               (long long)dims[l + 1]);
    p.s[l].K = (int)dims[l];
    p.s[l].N = (int)dims[l + 1];
    p.s[l].relu = relu[l] ? 1 : 0;
  }
  for (int s = 0; s < G; ++s) {
    RS_REQUIRE(x[s] && aligned16(x[s]), "rs_mlp_fwd_prec_f32: x[%d] null or not 16-byte aligned", s);
    p.x[s] = x[s];
    for (int l = 0; l < L; ++l) {
      RS_REQUIRE(W[s * L + l] && y[s * L + l], "rs_mlp_fwd_prec_f32: null W / y (stack %d layer %d)", s, l);
      p.s[l].W[s] = W[s * L + l];
      p.s[l].b[s] = b ? b[s * L + l] : nullptr;
      p.s[l].y[s] = y[s * L + l];
    }
  }
  return mlp_launch(p, G, false, precision, stream);
}

int rs_mlp_bwd_chain_prec_f32(int G, int L, const int64_t* dims, int64_t M, const float* const* g_top,
                              const float* const* W, const float* const* y, const int* relu, float* const* g,
                              int precision, rs_stream_t stream) {
  RS_REQUIRE(G >= 1 && G <= MLP_MAXG && L >= 1 && L <= MLP_MAXL && dims && g_top && W && y && relu && g,
             "rs_mlp_bwd_chain_prec_f32: 1..%d stacks of 1..%d layers", MLP_MAXG, MLP_MAXL);
  RS_REQUIRE(precision == RS_PREC_F32_SPLIT6 || precision == RS_PREC_F32_SPLIT9,
             "rs_mlp_bwd_chain_prec_f32: precision must be 6 or 9");
  RS_REQUIRE(M >= 0, "rs_mlp_bwd_chain_prec_f32: M < 0");
  bool dx_any = false;
  for (int s = 0; s < G; ++s) dx_any = dx_any || g[s * L] != nullptr;
  for (int l = 0; l <= L; ++l)
    RS_REQUIRE(mlp_width_ok(dims[l]) || (l == 0 && !dx_any), "rs_mlp_bwd_chain_prec_f32: width %d = %lld (64, 128 or 256)", l,
               (long long)dims[l]);
  // stage j runs layer l = L - 1 - j backwards: [M][dims[l + 1]] . W_l^T -> [M][dims[l]], masked
  // by y_{l-1} > 0 when layer l - 1 has a ReLU, into g[l - 1] (g[-1] = dL/dx, nullable: stage
  // skipped)
  MlpParams p{};
  p.M = M;
  int stages = 0;
  for (int l = L - 1; l >= 0; --l) {
    if (l == 0 && !dx_any) break;
    MlpStage& S = p.s[stages++];
    S.K = (int)dims[l + 1];
    S.N = (int)dims[l];
    S.relu = 0;
    for (int s = 0; s < G; ++s) {
      RS_REQUIRE(W[s * L + l], "rs_mlp_bwd_chain_prec_f32: null W (stack %d layer %d)", s, l);
      S.W[s] = W[s * L + l];
      S.b[s] = nullptr;
      if (l > 0 && relu[l - 1]) {
        RS_REQUIRE(y[s * L + l - 1], "rs_mlp_bwd_chain_prec_f32: null y (stack %d layer %d)", s, l - 1);
        S.mask[s] = y[s * L + l - 1];
      }
      S.y[s] = g[s * L + l];
      RS_REQUIRE(l == 0 || S.y[s], "rs_mlp_bwd_chain_prec_f32: null g (stack %d layer %d)", s, l - 1);
    }
  }
  p.L = stages;
  for (int s = 0; s < G; ++s) {
    RS_REQUIRE(g_top[s] && aligned16(g_top[s]), "rs_mlp_bwd_chain_prec_f32: g_top[%d] null or not 16-byte aligned",
               s);
    p.x[s] = g_top[s];
  }
  if (stages == 0) return RS_OK;
  return mlp_launch(p, G, true, precision, stream);
}

}  // extern "C"
