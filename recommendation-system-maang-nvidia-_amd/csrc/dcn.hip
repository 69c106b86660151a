// dcn.hip — DCN (v1, vector weight) cross stack, fused over all L layers, fwd + bwd.
//
// Reference: DeepCrossNetwork.call, src/models.py:38-44 (weights built at :31-35):
//   xl_T = expand_dims(xl, 2); w_xl = tensordot(xl_T, w_i[d,1], axes=(1,0)); ct = squeeze
//   xl = x0 * ct + b_i + xl
// i.e. a per-row scalar s_l = x_l . w_l (a GEMV, not a GEMM: the reference's weight is [d,1]),
// and the concat tf.concat([u, i], 1) of src/models.py:128 producing x0.
// Memory-bound: one wave per row, the row (d = 2D floats) lives in registers across all L
// layers, each dot is a wave64 shuffle reduction; the TF graph makes 3 elementwise passes + a
// matmul per layer. Backward recomputes x_l from (x0, s_l) in registers and accumulates the
// weight/bias gradients per wave, then per workgroup into ordered slabs (no atomics).
#include "common.hpp"

#include <initializer_list>

namespace rs {

constexpr int DCN_VMAX = 8;  // d <= 512 (8 floats per lane)
constexpr int DCN_LMAX = 8;

template <int DCN_MAXV>
__global__ __launch_bounds__(256) void dcn_cross_vec_fwd_kernel(
    const float* __restrict__ u, const float* __restrict__ v, int64_t B, int64_t D, int L,
    const float* __restrict__ w, const float* __restrict__ bias, float* __restrict__ x0o,
    float* __restrict__ xlo, float* __restrict__ so) {
  const int lane = threadIdx.x & 63;
  const int64_t d = 2 * D;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); b < B; b += nw) {
    float x0[DCN_MAXV], xl[DCN_MAXV];
#pragma unroll
    for (int j = 0; j < DCN_MAXV; ++j) {
      const int64_t e = lane + 64 * j;
      float val = 0.f;
      if (e < d) val = (e < D) ? u[b * D + e] : v[b * D + (e - D)];
      x0[j] = val;
      xl[j] = val;
    }
    for (int l = 0; l < L; ++l) {
      float part = 0.f;
#pragma unroll
      for (int j = 0; j < DCN_MAXV; ++j) {
        const int64_t e = lane + 64 * j;
        if (e < d) part += xl[j] * w[l * d + e];
      }
      const float s = wave_sum(part);
#pragma unroll
      for (int j = 0; j < DCN_MAXV; ++j) {
        const int64_t e = lane + 64 * j;
        if (e < d) xl[j] = (x0[j] * s + bias[l * d + e]) + xl[j];
      }
      if (lane == 0) so[b * L + l] = s;
    }
#pragma unroll
    for (int j = 0; j < DCN_MAXV; ++j) {
      const int64_t e = lane + 64 * j;
      if (e < d) {
        x0o[b * d + e] = x0[j];
        xlo[b * d + e] = xl[j];
      }
    }
  }
}

// slab layout per workgroup: [2][L][d] (dw then db)
// ADD: add_u / add_v (another consumer's dL/du, dL/dv) are added last to the outputs
template <int DCN_MAXV, int DCN_MAXL, bool EXTRA, bool ADD = false>
__global__ __launch_bounds__(256) void dcn_cross_vec_bwd_kernel(
    const float* __restrict__ x0g, const float* __restrict__ sg, const float* __restrict__ w,
    const float* __restrict__ bias, int64_t B, int64_t D, int L, const float* __restrict__ g_xl,
    const float* __restrict__ g_x0_extra, float* __restrict__ g_u, float* __restrict__ g_v,
    float* __restrict__ slab, const float* __restrict__ add_u = nullptr, const float* __restrict__ add_v = nullptr) {
  extern __shared__ float red[];  // [4][2][L][d]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t d = 2 * D;
  const int64_t nw = (int64_t)gridDim.x * 4;
  float dw[DCN_MAXL][DCN_MAXV], db[DCN_MAXL][DCN_MAXV];
#pragma unroll
  for (int l = 0; l < DCN_MAXL; ++l)
#pragma unroll
    for (int j = 0; j < DCN_MAXV; ++j) dw[l][j] = db[l][j] = 0.f;

  // the next row's x0, g, s (and extra gradient) are loaded while the current row is computed,
  // unconditionally with the row / column / layer index clamped into range
  const int Lc = L > 0 ? L : 1;
  const float* sgp = L > 0 ? sg : x0g;
  float px0[DCN_MAXV], pg[DCN_MAXV], pex[DCN_MAXV], ps[DCN_MAXL];
  auto fetch = [&](int64_t bb) __attribute__((always_inline)) {
    if (bb >= B) bb = B - 1;
#pragma unroll
    for (int l = 0; l < DCN_MAXL; ++l) ps[l] = sgp[bb * Lc + (l < Lc ? l : Lc - 1)];
#pragma unroll
    for (int j = 0; j < DCN_MAXV; ++j) {
      int64_t e = lane + 64 * j;
      if (e >= d) e = d - 1;
      px0[j] = x0g[bb * d + e];
      pg[j] = g_xl[bb * d + e];
      if constexpr (EXTRA) pex[j] = g_x0_extra[bb * d + e];
    }
  };
  const int64_t bstart = (int64_t)blockIdx.x * 4 + wave;
  if (bstart < B) fetch(bstart);
  for (int64_t b = bstart; b < B; b += nw) {
    float x0[DCN_MAXV], xs[DCN_MAXL + 1][DCN_MAXV], g[DCN_MAXV], gx0[DCN_MAXV], s[DCN_MAXL], ex[DCN_MAXV];
#pragma unroll
    for (int l = 0; l < DCN_MAXL; ++l) s[l] = (l < L) ? ps[l] : 0.f;
#pragma unroll
    for (int j = 0; j < DCN_MAXV; ++j) {
      const int64_t e = lane + 64 * j;
      x0[j] = (e < d) ? px0[j] : 0.f;
      xs[0][j] = x0[j];
      g[j] = (e < d) ? pg[j] : 0.f;
      gx0[j] = 0.f;
      ex[j] = EXTRA ? pex[j] : 0.f;
    }
    fetch(b + nw);
    // recompute x_1..x_{L-1} exactly as the forward did
#pragma unroll
    for (int l = 0; l < DCN_MAXL; ++l) {
      if (l >= L) break;
#pragma unroll
      for (int j = 0; j < DCN_MAXV; ++j) {
        const int64_t e = lane + 64 * j;
        xs[l + 1][j] = (e < d) ? (x0[j] * s[l] + bias[l * d + e]) + xs[l][j] : 0.f;
      }
    }
#pragma unroll
    for (int l = DCN_MAXL - 1; l >= 0; --l) {
      if (l >= L) continue;
      float part = 0.f;
#pragma unroll
      for (int j = 0; j < DCN_MAXV; ++j) part += g[j] * x0[j];
      const float t = wave_sum(part);  // dLoss/ds_l
#pragma unroll
      for (int j = 0; j < DCN_MAXV; ++j) {
        const int64_t e = lane + 64 * j;
        gx0[j] += g[j] * s[l];
        dw[l][j] += t * xs[l][j];
        db[l][j] += g[j];
        g[j] = (e < d) ? g[j] + t * w[l * d + e] : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < DCN_MAXV; ++j) {
      const int64_t e = lane + 64 * j;
      if (e < d) {
        float out = gx0[j] + g[j];
        if constexpr (EXTRA) out += ex[j];
        if (e < D) g_u[b * D + e] = ADD ? out + add_u[b * D + e] : out;
        else g_v[b * D + (e - D)] = ADD ? out + add_v[b * D + (e - D)] : out;
      }
    }
  }
  // combine the 4 waves in a fixed order, then one slab row per workgroup
  const int64_t per = 2 * (int64_t)L * d;
#pragma unroll
  for (int l = 0; l < DCN_MAXL; ++l) {
    if (l >= L) break;
#pragma unroll
    for (int j = 0; j < DCN_MAXV; ++j) {
      const int64_t e = lane + 64 * j;
      if (e < d) {
        red[wave * per + l * d + e] = dw[l][j];
        red[wave * per + (L + l) * d + e] = db[l][j];
      }
    }
  }
  __syncthreads();
  for (int64_t i = threadIdx.x; i < per; i += 256)
    slab[(int64_t)blockIdx.x * per + i] = ((red[i] + red[per + i]) + red[2 * per + i]) + red[3 * per + i];
}

// ---- d = 256 (the reference's 2 x 128 concat) on float4 lanes ---------------------------------
// Lane l owns columns 4l .. 4l + 3 (u for lanes < 32, v above), so a row moves as one 16-B access
// per lane instead of four dword accesses; the layer weights and biases stay in registers across
// rows, and NR rows per wave are processed together so their dot-product shuffle chains overlap.
// Same per-element arithmetic as the kernels above ((x0 s + b) + x_l, the backward's recompute of
// x_l bitwise the forward's); the dots sum in lane-column order instead (fp32 rounding only).
template <int ML, int NR>
__global__ __launch_bounds__(256) void dcn_cross_vec_fwd4_kernel(
    const float* __restrict__ u, const float* __restrict__ v, int64_t B, int L, const float* __restrict__ w,
    const float* __restrict__ bias, float* __restrict__ x0o, float* __restrict__ xlo, float* __restrict__ so) {
  constexpr int D = 128, d = 256;
  const int lane = threadIdx.x & 63;
  const float* src = lane < 32 ? u : v;
  const int cs = 4 * (lane & 31);  // column within u or v
  f32x4 wr[ML], br[ML];
#pragma unroll
  for (int l = 0; l < ML; ++l) {
    const int lc = l < L ? l : 0;
    wr[l] = *reinterpret_cast<const f32x4*>(w + lc * d + 4 * lane);
    br[l] = *reinterpret_cast<const f32x4*>(bias + lc * d + 4 * lane);
  }
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t b0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * NR; b0 < B; b0 += nw * NR) {
    f32x4 x0[NR], xl[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int64_t b = b0 + r < B ? b0 + r : B - 1;
      x0[r] = *reinterpret_cast<const f32x4*>(src + b * D + cs);
      xl[r] = x0[r];
    }
#pragma unroll
    for (int l = 0; l < ML; ++l) {
      if (l >= L) break;
      float sr[NR];
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        float part = xl[r][0] * wr[l][0];
        part += xl[r][1] * wr[l][1];
        part += xl[r][2] * wr[l][2];
        part += xl[r][3] * wr[l][3];
        sr[r] = part;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int r = 0; r < NR; ++r) sr[r] += __shfl_xor(sr[r], o, 64);
#pragma unroll
      for (int r = 0; r < NR; ++r) {
#pragma unroll
        for (int c = 0; c < 4; ++c) xl[r][c] = (x0[r][c] * sr[r] + br[l][c]) + xl[r][c];
        if (lane == 0 && b0 + r < B) so[(b0 + r) * L + l] = sr[r];
      }
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      if (b0 + r < B) {
        *reinterpret_cast<f32x4*>(x0o + (b0 + r) * d + 4 * lane) = x0[r];
        *reinterpret_cast<f32x4*>(xlo + (b0 + r) * d + 4 * lane) = xl[r];
      }
    }
  }
}

// slab layout per workgroup: [2][L][256] (dw then db), as dcn_cross_vec_bwd_kernel
template <int ML, int NR, bool EXTRA, bool ADD = false>
__global__ __launch_bounds__(256) void dcn_cross_vec_bwd4_kernel(
    const float* __restrict__ x0g, const float* __restrict__ sg, const float* __restrict__ w,
    const float* __restrict__ bias, int64_t B, int L, const float* __restrict__ g_xl,
    const float* __restrict__ g_x0_extra, float* __restrict__ g_u, float* __restrict__ g_v,
    float* __restrict__ slab, const float* __restrict__ add_u = nullptr, const float* __restrict__ add_v = nullptr) {
  constexpr int D = 128, d = 256;
  extern __shared__ float red[];  // [4][2][L][d]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  f32x4 wr[ML], br[ML], dw[ML], db[ML];
#pragma unroll
  for (int l = 0; l < ML; ++l) {
    const int lc = l < L ? l : 0;
    wr[l] = *reinterpret_cast<const f32x4*>(w + lc * d + 4 * lane);
    br[l] = *reinterpret_cast<const f32x4*>(bias + lc * d + 4 * lane);
    dw[l] = f32x4{0.f, 0.f, 0.f, 0.f};
    db[l] = dw[l];
  }
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t b0 = ((int64_t)blockIdx.x * 4 + wave) * NR; b0 < B; b0 += nw * NR) {
    f32x4 x0[NR], g[NR], gx0[NR], ex[NR], ad[NR];
    f32x4 xs[NR][ML];
    float s[NR][ML];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int64_t b = b0 + r < B ? b0 + r : B - 1;
      x0[r] = *reinterpret_cast<const f32x4*>(x0g + b * d + 4 * lane);
      g[r] = *reinterpret_cast<const f32x4*>(g_xl + b * d + 4 * lane);
      if constexpr (EXTRA) ex[r] = *reinterpret_cast<const f32x4*>(g_x0_extra + b * d + 4 * lane);
      // the addend is loaded with the row (in flight during the recompute), added last
      if constexpr (ADD) ad[r] = *reinterpret_cast<const f32x4*>((lane < 32 ? add_u : add_v) + b * D + 4 * (lane & 31));
#pragma unroll
      for (int l = 0; l < ML; ++l) s[r][l] = sg[b * L + (l < L ? l : 0)];
      gx0[r] = f32x4{0.f, 0.f, 0.f, 0.f};
      // a row past B (clamped) contributes nothing to dw / db
      if (b0 + r >= B) g[r] = gx0[r];
    }
    // recompute x_0 .. x_{L-1} exactly as the forward did
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      xs[r][0] = x0[r];
#pragma unroll
      for (int l = 0; l + 1 < ML; ++l) {
        if (l + 1 >= L) break;
#pragma unroll
        for (int c = 0; c < 4; ++c) xs[r][l + 1][c] = (x0[r][c] * s[r][l] + br[l][c]) + xs[r][l][c];
      }
    }
#pragma unroll
    for (int l = ML - 1; l >= 0; --l) {
      if (l >= L) continue;
      float t[NR];
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        float part = g[r][0] * x0[r][0];
        part += g[r][1] * x0[r][1];
        part += g[r][2] * x0[r][2];
        part += g[r][3] * x0[r][3];
        t[r] = part;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int r = 0; r < NR; ++r) t[r] += __shfl_xor(t[r], o, 64);  // dLoss/ds_l
#pragma unroll
      for (int r = 0; r < NR; ++r) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          gx0[r][c] += g[r][c] * s[r][l];
          dw[l][c] += t[r] * xs[r][l][c];
          db[l][c] += g[r][c];
          g[r][c] = g[r][c] + t[r] * wr[l][c];
        }
      }
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      if (b0 + r < B) {
        f32x4 out = gx0[r] + g[r];
        if constexpr (EXTRA) out += ex[r];
        if constexpr (ADD) out += ad[r];
        float* dst = lane < 32 ? g_u : g_v;
        *reinterpret_cast<f32x4*>(dst + (b0 + r) * D + 4 * (lane & 31)) = out;
      }
    }
  }
  // combine the 4 waves in a fixed order, then one slab row per workgroup
  const int64_t per = 2 * (int64_t)L * d;
#pragma unroll
  for (int l = 0; l < ML; ++l) {
    if (l >= L) break;
    *reinterpret_cast<f32x4*>(red + wave * per + l * d + 4 * lane) = dw[l];
    *reinterpret_cast<f32x4*>(red + wave * per + (L + l) * d + 4 * lane) = db[l];
  }
  __syncthreads();
  for (int64_t i = threadIdx.x; i < per; i += 256)
    slab[(int64_t)blockIdx.x * per + i] = ((red[i] + red[per + i]) + red[2 * per + i]) + red[3 * per + i];
}

static bool dcn_vec4_ok(int64_t D, int L, std::initializer_list<const void*> ptrs) {
  if (D != 128 || L > 4) return false;
  for (const void* q : ptrs)
    if (q && !aligned16(q)) return false;
  return true;
}

static int64_t dcn_blocks(int64_t B) {
  int64_t nb = ceil_div(B, 4);  // one row per wave up to 1024 workgroups, then grid-stride
  if (nb < 1) nb = 1;
  if (nb > 1024) nb = 1024;
  return nb;
}

}  // namespace rs

using namespace rs;

extern "C" {

int rs_dcn_cross_vec_fwd_f32(const float* u, const float* v, int64_t B, int64_t D, int L,
                             const float* w, const float* b, float* x0, float* xl, float* s,
                             rs_stream_t stream) {
  RS_REQUIRE(B >= 0 && D > 0 && L >= 0, "rs_dcn_cross_vec_fwd_f32: bad sizes");
  RS_REQUIRE(2 * D <= 64 * DCN_VMAX && L <= DCN_LMAX, "rs_dcn_cross_vec_fwd_f32: d <= 512, L <= 8");
  RS_REQUIRE(u && v && x0 && xl && (L == 0 || (w && b && s)), "rs_dcn_cross_vec_fwd_f32: null");
  if (B == 0) return RS_OK;
  int64_t nb = ceil_div(B, 4);
  if (nb > 256 * 32) nb = 256 * 32;
  const int nv = (int)ceil_div(2 * D, 64);
  hipStream_t st = as_stream(stream);
  if (L > 0 && dcn_vec4_ok(D, L, {u, v, w, b, x0, xl})) {
    int64_t nb4 = ceil_div(B, 8);
    if (nb4 > 256 * 32) nb4 = 256 * 32;
    hipLaunchKernelGGL((dcn_cross_vec_fwd4_kernel<4, 2>), dim3((unsigned)nb4), dim3(256), 0, st, u, v, B, L, w, b,
                       x0, xl, s);
    return check_launch("dcn_cross_vec_fwd4");
  }
#define RS_DCN_FWD(NV) \
  hipLaunchKernelGGL((dcn_cross_vec_fwd_kernel<NV>), dim3((unsigned)nb), dim3(256), 0, st, u, v, B, D, L, w, b, x0, xl, s)
  if (nv <= 1) RS_DCN_FWD(1);
  else if (nv <= 2) RS_DCN_FWD(2);
  else if (nv <= 4) RS_DCN_FWD(4);
  else RS_DCN_FWD(8);
#undef RS_DCN_FWD
  return check_launch("dcn_cross_vec_fwd");
}

size_t rs_dcn_cross_vec_bwd_workspace_bytes(int64_t B, int64_t D, int L) {
  return align_up((size_t)dcn_blocks(B) * 2 * (size_t)(L > 0 ? L : 1) * 2 * (size_t)D * sizeof(float), 256) +
         256;
}

static int dcn_vec_bwd_impl(const float* x0, const float* s, const float* w, const float* b,
                             int64_t B, int64_t D, int L, const float* g_xl,
                             const float* g_x0_extra, float* g_u, float* g_v, float* g_w,
                             float* g_b, void* workspace, size_t workspace_bytes,
                             rs_stream_t stream, const float* add_u, const float* add_v, void* queue) {
  RS_REQUIRE(B >= 0 && D > 0 && L >= 0, "rs_dcn_cross_vec_bwd_f32: bad sizes");
  RS_REQUIRE(2 * D <= 64 * DCN_VMAX && L <= DCN_LMAX, "rs_dcn_cross_vec_bwd_f32: d <= 512, L <= 8");
  RS_REQUIRE(x0 && g_xl && g_u && g_v && (L == 0 || (s && w && b && g_w && g_b)),
             "rs_dcn_cross_vec_bwd_f32: null");
  if (!workspace || workspace_bytes < rs_dcn_cross_vec_bwd_workspace_bytes(B, D, L)) {
    set_error("rs_dcn_cross_vec_bwd_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  const int64_t d = 2 * D;
  if (B == 0) {
    if (L > 0) {
      RS_HIP(hipMemsetAsync(g_w, 0, L * d * sizeof(float), st));
      RS_HIP(hipMemsetAsync(g_b, 0, L * d * sizeof(float), st));
    }
    return RS_OK;
  }
  const int64_t nb = dcn_blocks(B);
  const int64_t per = 2 * (int64_t)L * d;
  const size_t shm = (size_t)4 * (per > 0 ? per : 1) * sizeof(float);
  RS_REQUIRE(shm <= 160 * 1024, "rs_dcn_cross_vec_bwd_f32: L*d too large for LDS");
  float* slab = static_cast<float*>(workspace);
  const int nv = (int)ceil_div(d, 64);
  const bool add = add_u != nullptr;
  if (L > 0 && dcn_vec4_ok(D, L, {x0, w, b, g_xl, g_x0_extra, g_u, g_v, workspace, add_u, add_v})) {
#define RS_DCN_BWD4(EX, AD)                                                                                      \
  hipLaunchKernelGGL((dcn_cross_vec_bwd4_kernel<4, 2, EX, AD>), dim3((unsigned)nb), dim3(256), shm, st, x0, s, w, b, \
                     B, L, g_xl, g_x0_extra, g_u, g_v, slab, add_u, add_v)
    if (g_x0_extra && add) RS_DCN_BWD4(true, true);
    else if (g_x0_extra) RS_DCN_BWD4(true, false);
    else if (add) RS_DCN_BWD4(false, true);
    else RS_DCN_BWD4(false, false);
#undef RS_DCN_BWD4
  } else {
#define RS_DCN_BWDK(NV, ML, EX, AD)                                                                          \
  hipLaunchKernelGGL((dcn_cross_vec_bwd_kernel<NV, ML, EX, AD>), dim3((unsigned)nb), dim3(256), shm, st, x0, s, \
                     w, b, B, D, L, g_xl, g_x0_extra, g_u, g_v, slab, add_u, add_v)
#define RS_DCN_BWD(NV, ML)                                          \
  do {                                                              \
    if (g_x0_extra && add) RS_DCN_BWDK(NV, ML, true, true);         \
    else if (g_x0_extra) RS_DCN_BWDK(NV, ML, true, false);          \
    else if (add) RS_DCN_BWDK(NV, ML, false, true);                 \
    else RS_DCN_BWDK(NV, ML, false, false);                         \
  } while (0)
  if (L <= 4) {
    if (nv <= 1) RS_DCN_BWD(1, 4);
    else if (nv <= 2) RS_DCN_BWD(2, 4);
    else if (nv <= 4) RS_DCN_BWD(4, 4);
    else RS_DCN_BWD(8, 4);
  } else {
    if (nv <= 1) RS_DCN_BWD(1, 8);
    else if (nv <= 2) RS_DCN_BWD(2, 8);
    else if (nv <= 4) RS_DCN_BWD(4, 8);
    else RS_DCN_BWD(8, 8);
  }
#undef RS_DCN_BWD
#undef RS_DCN_BWDK
  }
  int rc = check_launch("dcn_cross_vec_bwd");
  if (rc || L == 0) return rc;
  // reduce [nb][2][L][d] -> dw (first L*d) and db (next L*d), slab order
  SlabQueue* q = static_cast<SlabQueue*>(queue);
  rc = launch_slab_reduce_strided(slab, nb, per, L * d, g_w, nullptr, 0.f, st, nullptr, -1, q);
  if (rc) return rc;
  return launch_slab_reduce_strided(slab + L * d, nb, per, L * d, g_b, nullptr, 0.f, st, nullptr, -1, q);
}

int rs_dcn_cross_vec_bwd_f32(const float* x0, const float* s, const float* w, const float* b, int64_t B, int64_t D,
                             int L, const float* g_xl, const float* g_x0_extra, float* g_u, float* g_v, float* g_w,
                             float* g_b, void* workspace, size_t workspace_bytes, rs_stream_t stream,
                             void* queue) {
  return dcn_vec_bwd_impl(x0, s, w, b, B, D, L, g_xl, g_x0_extra, g_u, g_v, g_w, g_b, workspace, workspace_bytes,
                          stream, nullptr, nullptr, queue);
}

int rs_dcn_cross_vec_bwd_add_f32(const float* x0, const float* s, const float* w, const float* b, int64_t B,
                                 int64_t D, int L, const float* g_xl, const float* g_x0_extra, const float* add_u,
                                 const float* add_v, float* g_u, float* g_v, float* g_w, float* g_b, void* workspace,
                                 size_t workspace_bytes, rs_stream_t stream, void* queue) {
  RS_REQUIRE(add_u && add_v, "rs_dcn_cross_vec_bwd_add_f32: null addend");
  return dcn_vec_bwd_impl(x0, s, w, b, B, D, L, g_xl, g_x0_extra, g_u, g_v, g_w, g_b, workspace, workspace_bytes,
                          stream, add_u, add_v, queue);
}

}  // extern "C"
