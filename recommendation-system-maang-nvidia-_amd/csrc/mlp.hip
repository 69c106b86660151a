// mlp.hip — a whole Dense stack's forward in ONE launch (the towers / the DCN deep net at small
// batches, where each per-layer GEMM launch is ~10 us of mostly fixed cost: C2's 4096 rows).
//
// Replaces the per-layer keras.layers.Dense forward (src/models.py:26-29,76-77) of MLPFn /
// MLPGroupFn: y_l = act_l(y_{l-1} W_l + b_l), y_0 = x, every y_l written (the backward's masks and
// weight-gradient operands). A 256-thread workgroup owns 32 rows of one stack and carries them
// through every layer: the activations live in LDS as exact three-term bf16 split planes (split.hpp;
// 16-B chunks of a row XOR-swizzled by the row, so the 16x16x32 A-fragment reads are conflict-free),
// each wave computes all 32 rows x N/4 columns of a layer on v_mfma_f32_16x16x32_bf16 with the
// weights' fragments loaded from L2 (split in registers, the next 32-k chunk's loads in flight
// during this chunk's MFMAs), and the epilogue adds the bias, applies the ReLU, stores y_l and
// writes its split planes into the other LDS buffer for the next layer. Same split products as
// the per-layer GEMMs (mfma16_split_n), fp32 accumulation; the order of the k additions differs.
#include "common.hpp"
#include "split.hpp"
#include <type_traits>

namespace rs {

constexpr int MLP_MAXL = 6, MLP_MAXG = 2, MLP_ROWS = 32;

struct MlpParams {
  const float* x[MLP_MAXG];
  const float* W[MLP_MAXG][MLP_MAXL];
  const float* b[MLP_MAXG][MLP_MAXL];
  float* y[MLP_MAXG][MLP_MAXL];
  int dims[MLP_MAXL + 1];
  int relu[MLP_MAXL];
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

template <int NP>
__global__ __launch_bounds__(256, 1) void mlp_fwd_kernel(MlpParams p) {
  __shared__ __attribute__((aligned(16))) uint16_t act[2][3][MLP_ROWS * 256];  // 96 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  const int st = (int)blockIdx.y;
  const float* __restrict__ X = p.x[0];
#pragma unroll
  for (int i = 1; i < MLP_MAXG; ++i)
    if (st == i) X = p.x[i];
  const int64_t r0 = (int64_t)blockIdx.x * MLP_ROWS;
  const int64_t M = p.M;

  // the input rows, split into buffer 0 (rows past M are zero)
  {
    const int K0 = p.dims[0], q = K0 / 4;
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
    const int K = p.dims[layer], N = p.dims[layer + 1];
    const int nt = N / 64;  // 16-column tiles per wave (1, 2 or 4)
    const int c0 = wave * (N / 4);
    const float* __restrict__ W = p.W[0][layer];
    const float* __restrict__ bias = p.b[0][layer];
    float* __restrict__ Y = p.y[0][layer];
#pragma unroll
    for (int i = 1; i < MLP_MAXG; ++i)
      if (st == i) {
        W = p.W[i][layer];
        bias = p.b[i][layer];
        Y = p.y[i][layer];
      }
    f32x4 acc[2][4];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    // weight fragment of tile t, chunk c: W[32 c + 8 g + j][c0 + 16 t + i16], j < 8 (tiles past nt
    // read tile 0 and are never used)
    float wf[2][4][8];
    auto wload = [&](int c, auto BUFI) __attribute__((always_inline)) {
      constexpr int bufi = decltype(BUFI)::value;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int tt = t < nt ? t : 0;
        const float* src = W + (int64_t)(32 * c + 8 * g) * N + c0 + 16 * tt + i16;
#pragma unroll
        for (int j = 0; j < 8; ++j) wf[bufi][t][j] = src[(int64_t)j * N];
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
    const bool relu = p.relu[layer] != 0;
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
            float v = acc[rt][t][r] + bv;
            if (relu) v = fmaxf(v, 0.f);
            if (r0 + row < M) Y[(r0 + row) * N + n] = v;
            if (layer + 1 < p.L) {
              uint16_t h, m, l;
              mlp_split1(r0 + row < M ? v : 0.f, h, m, l);
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
  p.dims[0] = (int)dims[0];
  for (int l = 0; l < L; ++l) {
    const int64_t n = dims[l + 1];
    RS_REQUIRE(n == 64 || n == 128 || n == 256, "rs_mlp_fwd_prec_f32: layer %d width %lld (64, 128 or 256)", l,
               (long long)n);
    p.dims[l + 1] = (int)n;
    p.relu[l] = relu[l] ? 1 : 0;
  }
  for (int s = 0; s < G; ++s) {
    RS_REQUIRE(x[s] && aligned16(x[s]), "rs_mlp_fwd_prec_f32: x[%d] null or not 16-byte aligned", s);
    p.x[s] = x[s];
    for (int l = 0; l < L; ++l) {
      RS_REQUIRE(W[s * L + l] && y[s * L + l], "rs_mlp_fwd_prec_f32: null W / y (stack %d layer %d)", s, l);
      p.W[s][l] = W[s * L + l];
      p.b[s][l] = b ? b[s * L + l] : nullptr;
      p.y[s][l] = y[s * L + l];
    }
  }
  if (M == 0) return RS_OK;
  const dim3 grid((unsigned)ceil_div(M, MLP_ROWS), (unsigned)G);
  hipStream_t st = as_stream(stream);
  if (precision == RS_PREC_F32_SPLIT6) hipLaunchKernelGGL((mlp_fwd_kernel<6>), grid, dim3(256), 0, st, p);
  else hipLaunchKernelGGL((mlp_fwd_kernel<9>), grid, dim3(256), 0, st, p);
  return check_launch("mlp_fwd");
}

}  // extern "C"
