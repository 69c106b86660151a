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
// The weights enter as fragment images (rs_mlp_weight_image_f32, once per step for both
// directions): every 16x16x32 B fragment of W (forward) and of W^T (chain) pre-split into its three
// bf16 planes, 1 KB per plane, so a wave loads a fragment with three coalesced 16-B loads and no
// split arithmetic (measured: splitting the weights in every workgroup made the stack kernels
// VALU-bound, ~4300 VALU per wave for 240 MFMAs). A 256-thread workgroup owns 16 (or 32) rows of one
// stack and carries them through every stage: the rows live in LDS as split planes (the 16-B
// chunks of a row XOR-swizzled by the row, so the A-fragment reads are conflict-free), each wave
// computes all rows x N/4 columns of a stage on v_mfma_f32_16x16x32_bf16 with the next chunk's
// fragments in flight, and the epilogue adds the bias, applies the ReLU or the mask (both loaded
// before the k loop), stores the stage's output and writes its split planes into the other LDS
// buffer for the next stage. Same split products as the per-layer GEMMs (mfma16_split_n); the order
// of the k additions differs.
#include "common.hpp"
#include "split.hpp"
#include <cstdlib>
#include <type_traits>

namespace rs {

constexpr int MLP_MAXL = 6, MLP_MAXG = 2;

struct MlpStage {
  const char* img[MLP_MAXG];    // the B operand's fragment image (K x N: W, or W^T for the chain)
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

// fragment image of a B operand [KB][NB]: fragment (c, t) (k rows 32 c .., columns 16 t ..), plane
// p, lane (i16, g) at ((c * NB / 16 + t) * 3 + p) KB + 16 lane: the bf16 terms of B[32 c + 8 g + j]
// [16 t + i16], j < 8, in pairs
constexpr int MLP_FRAG = 3 * 1024;

template <int NP, int R>
__global__ __launch_bounds__(256, R == 16 ? 2 : 1) void mlp_chain_kernel(MlpParams p) {
  constexpr int RT = R / 16;  // 16-row tiles per workgroup
  __shared__ __attribute__((aligned(16))) uint16_t act[2][3][R * 256];  // 48 or 96 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  const int st = (int)blockIdx.y;
  const float* __restrict__ X = mlp_pick(p.x, st);
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int64_t M = p.M;

  // the input rows, split into buffer 0 (rows past M are zero)
  {
    const int K0 = p.s[0].K, q = K0 / 4;
    for (int idx = tid; idx < R * q; idx += 256) {
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
    const char* __restrict__ WI = mlp_pick(p.s[layer].img, st);
    const float* __restrict__ bias = mlp_pick(p.s[layer].b, st);
    const float* __restrict__ mask = mlp_pick(p.s[layer].mask, st);
    float* __restrict__ Y = mlp_pick(p.s[layer].y, st);
    f32x4 acc[RT][4];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    // B fragments of this wave's tiles t (columns c0 + 16 t ..) for chunk c (tiles past nt read
    // tile 0 and are never used)
    constexpr int NB = 2;
    u32x4 wf[NB][4][3];
    const int t0 = c0 / 16, ntile = N / 16;
    auto wload = [&](int c, auto BUFI) __attribute__((always_inline)) {
      constexpr int bufi = decltype(BUFI)::value;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int tt = t < nt ? t : 0;
        const u32x4* src = reinterpret_cast<const u32x4*>(WI + (int64_t)(c * ntile + t0 + tt) * MLP_FRAG) + lane;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) wf[bufi][t][pl] = src[64 * pl];
      }
    };
    const int nch = K / 32;
    // one 32-k chunk with the weight buffer index a compile-time constant (a run-time index would
    // send wf to LDS)
    auto chunk = [&](int c, auto BI) __attribute__((always_inline)) {
      constexpr int bi = decltype(BI)::value;
      // A fragments of both 16-row tiles from LDS: row 16 rt + i16, k 32 c + 8 g .. + 7
      u32x4 ap[RT][3];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          ap[rt][pl] = *reinterpret_cast<const u32x4*>(&act[cur][pl][mlp_off(16 * rt + i16, 32 * c + 8 * g)]);
      if (c + NB - 1 < nch) wload(c + NB - 1, std::integral_constant<int, (bi + NB - 1) % NB>{});
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (t < nt) {
          const u32x4* aa[RT];
          const u32x4* bb[RT];
          f32x4* cc[RT];
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) {
            aa[rt] = ap[rt];
            bb[rt] = wf[bi][t];
            cc[rt] = &acc[rt][t];
          }
          mfma16_split_n<NP, RT>(aa, bb, cc);
        }
      }
    };
    // the epilogue's bias and mask values, loaded before the k loop (their latency hides under it)
    float bvp[4], mv[4][RT][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int n = c0 + 16 * (t < nt ? t : 0) + i16;
      bvp[t] = bias ? bias[n] : 0.f;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = r0 + 16 * rt + 4 * g + r;
          mv[t][rt][r] = mask && t < nt && row < M ? mask[row * N + n] : 1.f;
        }
    }
    wload(0, std::integral_constant<int, 0>{});
    for (int c = 0; c < nch; c += NB) {
      chunk(c, std::integral_constant<int, 0>{});
      if (c + 1 < nch) chunk(c + 1, std::integral_constant<int, 1>{});
    }
    // epilogue: D[row 16 rt + 4 g + r][col c0 + 16 t + i16]
    const bool relu = p.s[layer].relu != 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t < nt) {
        const int n = c0 + 16 * t + i16;
        const float bv = bvp[t];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * rt + 4 * g + r;
            const bool live = r0 + row < M;
            float v = acc[rt][t][r] + bv;
            if (relu) v = fmaxf(v, 0.f);
            if (!(mv[t][rt][r] > 0.f)) v = 0.f;
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

// ----- weight gradients of a whole stack in one launch ----------------------------------------
// dW_l = x_l^T g_l and db_l = column sums of g_l for every layer l of every stack, as 64 x 64
// output tiles (k x n), each tile's M rows split into S slices of ms rows. A workgroup stages a
// 128-row chunk of its slice of x_l[:, k-tile] and g_l[:, n-tile] into LDS transposed (rows k / n,
// 8 consecutive m per 16-B chunk, split planes: the operands of a 16x16x32 MFMA over m), four waves
// each own a 32 x 32 quarter of the tile; the next chunk's global loads are in flight during the
// MFMAs. The n-tiles of k-tile 0 also sum g's columns (fp32, fixed order). With S > 1 each slice
// writes its partial [K + 1][N] image (dW rows, then the db row) into a slab and the library's
// ordered slab reduction sums the S slabs and adds the l2 term (queued with the step's other
// reductions when a queue is given): deterministic, and one launch for all the stacks' layers.
// Output per layer: [K + 1][N], rows < K dW, row K db (rs_gemm_wgrad_bias_prec_f32's layout).
constexpr int WG_MAXP = MLP_MAXG * MLP_MAXL, WG_MAXS = 16, WG_CH = 64;

struct MlpWgradParams {
  const float* x[WG_MAXP];
  const float* g[WG_MAXP];
  float* out[WG_MAXP];
  const float* wreg[WG_MAXP];
  int64_t slab_off[WG_MAXP];
  int K[WG_MAXP], N[WG_MAXP], tile0[WG_MAXP + 1];
  int np, S;
  int64_t M, ms;
  float w_scale;
  const float* w_dscale;
  float* slab;
};

__device__ __forceinline__ int wg_off(int row, int ch) { return row * WG_CH + (((ch ^ row) & 7) << 3); }

template <int NP>
__global__ __launch_bounds__(256, 2) void mlp_wgrad_kernel(MlpWgradParams p) {
  __shared__ __attribute__((aligned(16))) uint16_t xt[3][64 * WG_CH];  // 24 KB
  __shared__ __attribute__((aligned(16))) uint16_t gt[3][64 * WG_CH];  // 24 KB
  __shared__ float csum[8][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  const int S = p.S;
  const int tile = (int)blockIdx.x / S, slice = (int)blockIdx.x - tile * S;
  int q = 0;
#pragma unroll
  for (int i = 1; i < WG_MAXP; ++i)
    if (i < p.np && tile >= p.tile0[i]) q = i;
  const int K = p.K[q], N = p.N[q], nn = N / 64;
  const int lt = tile - p.tile0[q], kt = lt / nn, ntl = lt - kt * nn;
  const float* __restrict__ X = p.x[q] + 64 * kt;
  const float* __restrict__ Gm = p.g[q] + 64 * ntl;
  const bool want_db = kt == 0;
  const int64_t mb0 = (int64_t)slice * p.ms;
  const int64_t mend = mb0 + p.ms < p.M ? mb0 + p.ms : p.M;
  const int nchunk = (int)((p.ms + WG_CH - 1) / WG_CH);
  // loader: 8 consecutive rows (mb) x 2 consecutive columns (c2) of each operand per thread
  const int c2 = tid & 31, mb = tid >> 5;
  f32x2 xv[8], gv[8];
  auto load = [&](int ch) __attribute__((always_inline)) {
    const int64_t m0 = mb0 + (int64_t)ch * WG_CH + 8 * mb;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = m0 + j < mend;
      xv[j] = ok ? *reinterpret_cast<const f32x2*>(X + (m0 + j) * K + 2 * c2) : f32x2{0.f, 0.f};
      gv[j] = ok ? *reinterpret_cast<const f32x2*>(Gm + (m0 + j) * N + 2 * c2) : f32x2{0.f, 0.f};
    }
  };
  f32x2 cs = {0.f, 0.f};
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wk = wave >> 1, wn = wave & 1;
  load(0);
  for (int ch = 0; ch < nchunk; ++ch) {
    // transposed split stores: column 2 c2 + e, the 8 rows of this thread as one 16-B chunk
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      u32x4 xh, xm, xl, gh, gm, gl;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const IbSplit sx = ib_split2(xv[2 * w][e], xv[2 * w + 1][e]);
        xh[w] = sx.h;
        xm[w] = sx.m;
        xl[w] = sx.l;
        const IbSplit sg = ib_split2(gv[2 * w][e], gv[2 * w + 1][e]);
        gh[w] = sg.h;
        gm[w] = sg.m;
        gl[w] = sg.l;
      }
      const int o = wg_off(2 * c2 + e, mb);
      *reinterpret_cast<u32x4*>(&xt[0][o]) = xh;
      *reinterpret_cast<u32x4*>(&xt[1][o]) = xm;
      *reinterpret_cast<u32x4*>(&xt[2][o]) = xl;
      *reinterpret_cast<u32x4*>(&gt[0][o]) = gh;
      *reinterpret_cast<u32x4*>(&gt[1][o]) = gm;
      *reinterpret_cast<u32x4*>(&gt[2][o]) = gl;
    }
    if (want_db) {
#pragma unroll
      for (int j = 0; j < 8; ++j) cs += gv[j];
    }
    __syncthreads();
    if (ch + 1 < nchunk) load(ch + 1);
#pragma unroll
    for (int c = 0; c < WG_CH / 32; ++c) {
      u32x4 ap[2][3], bp[2][3];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          ap[t][pl] = *reinterpret_cast<const u32x4*>(&xt[pl][wg_off(32 * wk + 16 * t + i16, 4 * c + g)]);
          bp[t][pl] = *reinterpret_cast<const u32x4*>(&gt[pl][wg_off(32 * wn + 16 * t + i16, 4 * c + g)]);
        }
      const u32x4* const aa[4] = {ap[0], ap[0], ap[1], ap[1]};
      const u32x4* const bb[4] = {bp[0], bp[1], bp[0], bp[1]};
      f32x4* const cc[4] = {&acc[0][0], &acc[0][1], &acc[1][0], &acc[1][1]};
      mfma16_split_n<NP, 4>(aa, bb, cc);
    }
    __syncthreads();
  }
  // the slice's column sums of g: csum[mb][n] then a fixed-order sum over mb
  if (want_db) {
#pragma unroll
    for (int e = 0; e < 2; ++e) csum[mb][2 * c2 + e] = cs[e];
  }
  __syncthreads();
  float dbv = 0.f;
  if (want_db && tid < 64) {
#pragma unroll
    for (int i = 0; i < 8; ++i) dbv += csum[i][tid];
  }
  // S == 1: the final values (+ the l2 term); else this slice's partial into its slab
  const bool direct = S == 1;
  float* __restrict__ out = direct ? p.out[q] : p.slab + p.slab_off[q] + (int64_t)slice * (K + 1) * N;
  const float* __restrict__ wreg = direct ? p.wreg[q] : nullptr;
  const float wsc = wreg ? p.w_scale * *p.w_dscale : 0.f;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = 64 * kt + 32 * wk + 16 * a + 4 * g + r, n = 64 * ntl + 32 * wn + 16 * b + i16;
        float v = acc[a][b][r];
        if (wreg) v += wsc * wreg[(int64_t)k * N + n];
        out[(int64_t)k * N + n] = v;
      }
  if (want_db && tid < 64) out[(int64_t)K * N + 64 * ntl + tid] = dbv;
}

int mlp_wgrad_plan(int G, int L, const int64_t* dims, int64_t M, int& ntiles, int& S, int64_t& ms) {
  ntiles = 0;
  for (int l = 0; l < L; ++l) ntiles += (int)(dims[l] / 64) * (int)(dims[l + 1] / 64);
  ntiles *= G;
  int64_t s = (M + 255) / 256;
  S = (int)(s < 1 ? 1 : s > WG_MAXS ? WG_MAXS : s);
  ms = ((M + S - 1) / S + WG_CH - 1) / WG_CH * WG_CH;
  if (ms == 0) ms = WG_CH;
  return 0;
}

// rows per workgroup: 16 (two workgroups resident per CU: more loads in flight; measured C2
// 0.416 vs 0.431 ms per step) or 32 (two 16-row tiles share every weight fragment); RS_MLP_ROWS
int mlp_rows() {
  const char* e = exp_env("RS_MLP_ROWS");
  return e && atoi(e) == 32 ? 32 : 16;
}

template <int NP>
void mlp_launch_r(const MlpParams& p, int G, int R, hipStream_t st) {
  const dim3 grid((unsigned)ceil_div(p.M, R), (unsigned)G);
  if (R == 16) hipLaunchKernelGGL((mlp_chain_kernel<NP, 16>), grid, dim3(256), 0, st, p);
  else hipLaunchKernelGGL((mlp_chain_kernel<NP, 32>), grid, dim3(256), 0, st, p);
}

int mlp_launch(MlpParams& p, int G, bool trans, int precision, rs_stream_t stream) {
  if (p.M == 0) return RS_OK;
  const int R = mlp_rows();
  hipStream_t st = as_stream(stream);
  if (precision == RS_PREC_F32_SPLIT6) mlp_launch_r<6>(p, G, R, st);
  else mlp_launch_r<9>(p, G, R, st);
  return check_launch(trans ? "mlp_bwd_chain" : "mlp_fwd");
}

// ----- weight fragment images ------------------------------------------------------------------
// per stack, per layer l: the forward image of W_l [K][N], then the chain image of W_l^T [N][K]
// (each K N 6 bytes); one thread writes one lane's three 16-B plane entries of one fragment
constexpr int MLP_IMG_JOBS = 2 * MLP_MAXG * MLP_MAXL;
struct MlpImageJobs {
  const float* W[MLP_IMG_JOBS];
  char* img[MLP_IMG_JOBS];
  int KB[MLP_IMG_JOBS], NB[MLP_IMG_JOBS], trans[MLP_IMG_JOBS];
  int64_t t0[MLP_IMG_JOBS + 1];
  int n;
};

__global__ __launch_bounds__(256) void mlp_image_kernel(MlpImageJobs jb) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= jb.t0[jb.n]) return;
  int q = 0;
  for (int k = 1; k < jb.n; ++k)
    if (i >= jb.t0[k]) q = k;
  const int64_t e = i - jb.t0[q];
  const int lane = (int)(e & 63), frag = (int)(e >> 6);
  const int KB = jb.KB[q], NB = jb.NB[q], ntile = NB / 16;
  const int c = frag / ntile, t = frag - c * ntile;
  const int g = lane >> 4, i16 = lane & 15;
  const int kb = 32 * c + 8 * g, nb = 16 * t + i16;
  const float* __restrict__ W = jb.W[q];
  float v[8];
  // B[kb + j][nb]: W[kb + j][nb] (forward, W [KB][NB]) or W[nb][kb + j] (chain, W [NB][KB])
  if (jb.trans[q]) {
    const f32x4* src = reinterpret_cast<const f32x4*>(W + (int64_t)nb * KB + kb);
    const f32x4 lo = src[0], hi = src[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = lo[j];
      v[4 + j] = hi[j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = W[(int64_t)(kb + j) * NB + nb];
  }
  u32x4 h, m, l;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const IbSplit sp = ib_split2(v[2 * w], v[2 * w + 1]);
    h[w] = sp.h;
    m[w] = sp.m;
    l[w] = sp.l;
  }
  u32x4* dst = reinterpret_cast<u32x4*>(jb.img[q] + (int64_t)frag * MLP_FRAG) + lane;
  dst[0] = h;
  dst[64] = m;
  dst[128] = l;
}

size_t mlp_layer_image_bytes(int64_t K, int64_t N) { return (size_t)K * N * 6; }

bool mlp_width_ok(int64_t n) { return n == 64 || n == 128 || n == 256; }

}  // namespace rs

using namespace rs;

extern "C" {

size_t rs_mlp_weight_image_bytes(int L, const int64_t* dims) {
  if (L < 1 || L > MLP_MAXL || !dims) return 0;
  size_t b = 0;
  for (int l = 0; l < L; ++l) b += 2 * mlp_layer_image_bytes(dims[l], dims[l + 1]);
  return b;
}

int rs_mlp_weight_image_f32(int G, int L, const int64_t* dims, const float* const* W, void* const* img,
                            rs_stream_t stream) {
  RS_REQUIRE(G >= 1 && G <= MLP_MAXG && L >= 1 && L <= MLP_MAXL && dims && W && img,
             "rs_mlp_weight_image_f32: 1..%d stacks of 1..%d layers", MLP_MAXG, MLP_MAXL);
  for (int l = 0; l <= L; ++l)
    RS_REQUIRE(dims[l] >= 32 && dims[l] <= 4096 && dims[l] % 32 == 0,
               "rs_mlp_weight_image_f32: width %d = %lld (a multiple of 32)", l, (long long)dims[l]);
  MlpImageJobs jb{};
  int64_t t = 0;
  for (int s = 0; s < G; ++s) {
    RS_REQUIRE(img[s] && aligned16(img[s]), "rs_mlp_weight_image_f32: img[%d] null or not 16-byte aligned", s);
    size_t off = 0;
    for (int l = 0; l < L; ++l) {
      const float* w = W[s * L + l];
      RS_REQUIRE(w && aligned16(w), "rs_mlp_weight_image_f32: W (stack %d layer %d) null or not 16-byte aligned", s,
                 l);
      for (int tr = 0; tr < 2; ++tr) {
        const int q = jb.n++;
        jb.W[q] = w;
        jb.img[q] = static_cast<char*>(img[s]) + off;
        jb.KB[q] = (int)(tr ? dims[l + 1] : dims[l]);
        jb.NB[q] = (int)(tr ? dims[l] : dims[l + 1]);
        jb.trans[q] = tr;
        jb.t0[q] = t;
        t += (int64_t)jb.KB[q] * jb.NB[q] / 8;
        off += mlp_layer_image_bytes(dims[l], dims[l + 1]);
      }
    }
  }
  jb.t0[jb.n] = t;
  hipLaunchKernelGGL(mlp_image_kernel, dim3((unsigned)ceil_div(t, 256)), dim3(256), 0, as_stream(stream), jb);
  return check_launch("mlp_image");
}

int rs_mlp_weight_images_f32(int n, const int64_t* K, const int64_t* N, const float* const* W, void* const* dst,
                             rs_stream_t stream) {
  RS_REQUIRE(n >= 1 && 2 * n <= MLP_IMG_JOBS && K && N && W && dst,
             "rs_mlp_weight_images_f32: 1..%d layers", MLP_IMG_JOBS / 2);
  MlpImageJobs jb{};
  int64_t t = 0;
  for (int i = 0; i < n; ++i) {
    RS_REQUIRE(K[i] >= 32 && K[i] <= 4096 && K[i] % 32 == 0 && N[i] >= 32 && N[i] <= 4096 && N[i] % 32 == 0,
               "rs_mlp_weight_images_f32: layer %d is %lld x %lld (multiples of 32)", i, (long long)K[i],
               (long long)N[i]);
    RS_REQUIRE(W[i] && aligned16(W[i]) && dst[i] && aligned16(dst[i]),
               "rs_mlp_weight_images_f32: layer %d: null or unaligned W / dst", i);
    for (int tr = 0; tr < 2; ++tr) {
      const int q = jb.n++;
      jb.W[q] = W[i];
      jb.img[q] = static_cast<char*>(dst[i]) + (tr ? mlp_layer_image_bytes(K[i], N[i]) : 0);
      jb.KB[q] = (int)(tr ? N[i] : K[i]);
      jb.NB[q] = (int)(tr ? K[i] : N[i]);
      jb.trans[q] = tr;
      jb.t0[q] = t;
      t += (int64_t)jb.KB[q] * jb.NB[q] / 8;
    }
  }
  jb.t0[jb.n] = t;
  hipLaunchKernelGGL(mlp_image_kernel, dim3((unsigned)ceil_div(t, 256)), dim3(256), 0, as_stream(stream), jb);
  return check_launch("mlp_images");
}

// the stage images of layer l of a stack image: forward, then chain
static const char* mlp_img(const void* base, int L, const int64_t* dims, int l, int chain) {
  size_t off = 0;
  for (int j = 0; j < l; ++j) off += 2 * mlp_layer_image_bytes(dims[j], dims[j + 1]);
  if (chain) off += mlp_layer_image_bytes(dims[l], dims[l + 1]);
  (void)L;
  return static_cast<const char*>(base) + off;
}

int rs_mlp_fwd_prec_f32(int G, int L, const int64_t* dims, int64_t M, const float* const* x, const void* const* img,
                        const float* const* b, const int* relu, float* const* y, int precision, rs_stream_t stream) {
  RS_REQUIRE(G >= 1 && G <= MLP_MAXG && L >= 1 && L <= MLP_MAXL && dims && x && img && y && relu,
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
      RS_REQUIRE(img[s] && y[s * L + l], "rs_mlp_fwd_prec_f32: null image / y (stack %d layer %d)", s, l);
      p.s[l].img[s] = mlp_img(img[s], L, dims, l, 0);
      p.s[l].b[s] = b ? b[s * L + l] : nullptr;
      p.s[l].y[s] = y[s * L + l];
    }
  }
  return mlp_launch(p, G, false, precision, stream);
}

int rs_mlp_bwd_chain_prec_f32(int G, int L, const int64_t* dims, int64_t M, const float* const* g_top,
                              const void* const* img, const float* const* y, const int* relu, float* const* g,
                              int precision, rs_stream_t stream) {
  RS_REQUIRE(G >= 1 && G <= MLP_MAXG && L >= 1 && L <= MLP_MAXL && dims && g_top && img && y && relu && g,
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
      RS_REQUIRE(img[s], "rs_mlp_bwd_chain_prec_f32: null image (stack %d)", s);
      S.img[s] = mlp_img(img[s], L, dims, l, 1);
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

size_t rs_mlp_wgrad_workspace_bytes(int G, int L, const int64_t* dims, int64_t M) {
  if (G < 1 || L < 1 || !dims) return 0;
  int ntiles, S;
  int64_t ms;
  mlp_wgrad_plan(G, L, dims, M, ntiles, S, ms);
  if (S == 1) return 0;
  size_t per = 0;
  for (int l = 0; l < L; ++l) per += (size_t)(dims[l] + 1) * dims[l + 1];
  return (size_t)G * S * per * sizeof(float);
}

int rs_mlp_wgrad_prec_f32(int G, int L, const int64_t* dims, int64_t M, const float* const* x, const float* const* g,
                          float* const* dWdb, const float* const* w_reg, float w_scale, const float* w_dscale,
                          int precision, void* workspace, size_t workspace_bytes, rs_stream_t stream, void* queue) {
  RS_REQUIRE(G >= 1 && G <= MLP_MAXG && L >= 1 && L <= MLP_MAXL && dims && x && g && dWdb,
             "rs_mlp_wgrad_prec_f32: 1..%d stacks of 1..%d layers", MLP_MAXG, MLP_MAXL);
  RS_REQUIRE(precision == RS_PREC_F32_SPLIT6 || precision == RS_PREC_F32_SPLIT9,
             "rs_mlp_wgrad_prec_f32: precision must be 6 or 9");
  RS_REQUIRE(M >= 0, "rs_mlp_wgrad_prec_f32: M < 0");
  for (int l = 0; l <= L; ++l)
    RS_REQUIRE(dims[l] >= 64 && dims[l] <= 4096 && dims[l] % 64 == 0,
               "rs_mlp_wgrad_prec_f32: width %d = %lld (a multiple of 64)", l, (long long)dims[l]);
  MlpWgradParams p{};
  int ntiles, S;
  int64_t ms;
  mlp_wgrad_plan(G, L, dims, M, ntiles, S, ms);
  if (S > 1 && (!workspace || workspace_bytes < rs_mlp_wgrad_workspace_bytes(G, L, dims, M))) {
    set_error("rs_mlp_wgrad_prec_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  p.np = G * L;
  p.S = S;
  p.M = M;
  p.ms = ms;
  p.w_scale = w_scale;
  p.w_dscale = w_dscale;
  p.slab = static_cast<float*>(workspace);
  int t0 = 0;
  int64_t off = 0;
  for (int s = 0; s < G; ++s)
    for (int l = 0; l < L; ++l) {
      const int i = s * L + l;
      // (no rows: x / g are never read and may be null)
      RS_REQUIRE(dWdb[i] && (M == 0 || (x[i] && g[i] && aligned16(x[i]) && aligned16(g[i]))),
                 "rs_mlp_wgrad_prec_f32: null or unaligned x / g / dWdb (stack %d layer %d)", s, l);
      p.x[i] = x[i];
      p.g[i] = g[i];
      p.out[i] = dWdb[i];
      p.wreg[i] = w_reg ? w_reg[i] : nullptr;
      RS_REQUIRE(!p.wreg[i] || w_dscale, "rs_mlp_wgrad_prec_f32: w_reg without w_dscale");
      p.K[i] = (int)dims[l];
      p.N[i] = (int)dims[l + 1];
      p.tile0[i] = t0;
      p.slab_off[i] = off;
      t0 += (int)(dims[l] / 64) * (int)(dims[l + 1] / 64);
      off += (int64_t)S * (dims[l] + 1) * dims[l + 1];
    }
  p.tile0[p.np] = t0;
  // M == 0 runs too: one slice of no rows writes dW = the l2 term (or 0) and db = 0
  const dim3 grid((unsigned)(ntiles * S));
  hipStream_t st = as_stream(stream);
  if (precision == RS_PREC_F32_SPLIT6) hipLaunchKernelGGL((mlp_wgrad_kernel<6>), grid, dim3(256), 0, st, p);
  else hipLaunchKernelGGL((mlp_wgrad_kernel<9>), grid, dim3(256), 0, st, p);
  int rc = check_launch("mlp_wgrad");
  if (rc || S == 1) return rc;
  for (int i = 0; i < p.np && rc == 0; ++i) {
    const int64_t cnt = (int64_t)(p.K[i] + 1) * p.N[i];
    rc = launch_slab_reduce_strided(p.slab + p.slab_off[i], S, cnt, cnt, p.out[i], p.wreg[i], w_scale, st,
                                    p.wreg[i] ? w_dscale : nullptr, p.wreg[i] ? (int64_t)p.K[i] * p.N[i] : 0,
                                    static_cast<SlabQueue*>(queue));
  }
  return rc;
}

}  // extern "C"
