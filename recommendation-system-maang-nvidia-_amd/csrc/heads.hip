// heads.hip — DCN output concat + rating/CTR heads (fwd, bwd) and the two Ranking losses.
//
// Reference: z = tf.concat([xl, deep_out], 1) (src/models.py:50); rating_head = Dense(1),
// ctr_head = Dense(1, 'sigmoid') (src/models.py:119-120, applied at :131);
// rating_task = tfrs.tasks.Ranking(MSE), ctr_task = tfrs.tasks.Ranking(BCE) with
// sample_weight = class_weights[y] (src/models.py:122-123,138-145).
// The concat is never materialised: each head is a GEMV over the two row halves, one wave per
// row. Losses are ordered two-stage sums (fp64 partials); their per-row derivatives are written
// in the forward so the heads backward is one fused pass (dz = dr w_r + dlogit w_c).
#include "common.hpp"

#include <cmath>

namespace rs {

constexpr int HV = 16;  // (dx + dh) <= 1024 floats per row

__global__ __launch_bounds__(256) void heads_fwd_kernel(const float* __restrict__ xl, int64_t dx,
                                                        const float* __restrict__ h, int64_t dh,
                                                        int64_t B, const float* __restrict__ w_r,
                                                        const float* __restrict__ b_r,
                                                        const float* __restrict__ w_c,
                                                        const float* __restrict__ b_c,
                                                        float* __restrict__ rating,
                                                        float* __restrict__ ctr) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t dz = dx + dh;
  if (dz <= 64 * 8) {
    // one batch of 8 columns per lane covers the row: the lane's weights and its columns' source
    // (xl or h, offset) are fixed for every row, so they are loaded / formed once per wave; per
    // row only the 8 z values are read (same values, same order as the general loop below)
    float wrv[8], wcv[8];
    int off[8];
    bool fromx[8], live[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      int64_t e = lane + 64 * u;
      live[u] = e < dz;
      if (e >= dz) e = dz - 1;
      fromx[u] = e < dx;
      off[u] = (int)(fromx[u] ? e : e - dx);
      wrv[u] = w_r[e];
      wcv[u] = w_c[e];
    }
    for (int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); b < B; b += nw) {
      const float* xr = xl + b * dx;
      const float* hr = h + b * dh;
      float zv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) zv[u] = fromx[u] ? xr[off[u]] : hr[off[u]];
      float pr = 0.f, pc = 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (live[u]) {
          pr += zv[u] * wrv[u];
          pc += zv[u] * wcv[u];
        }
      }
      pr = wave_sum(pr);
      pc = wave_sum(pc);
      if (lane == 0) {
        rating[b] = pr + b_r[0];
        const float t = pc + b_c[0];
        ctr[b] = 1.f / (1.f + expf(-t));
      }
    }
    return;
  }
  for (int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); b < B; b += nw) {
    float pr = 0.f, pc = 0.f;
    // 8 columns per lane per batch: their loads (column clamped into the row) issued together,
    // then the products added in the column order of the one-at-a-time loop
    for (int64_t e0 = lane; e0 < dz; e0 += 64 * 8) {
      float zv[8], wrv[8], wcv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        int64_t e = e0 + 64 * u;
        if (e >= dz) e = dz - 1;
        zv[u] = e < dx ? xl[b * dx + e] : h[b * dh + (e - dx)];
        wrv[u] = w_r[e];
        wcv[u] = w_c[e];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (e0 + 64 * u < dz) {
          pr += zv[u] * wrv[u];
          pc += zv[u] * wcv[u];
        }
      }
    }
    pr = wave_sum(pr);
    pc = wave_sum(pc);
    if (lane == 0) {
      rating[b] = pr + b_r[0];
      const float t = pc + b_c[0];
      ctr[b] = 1.f / (1.f + expf(-t));
    }
  }
}

// Columns [c0, c0 + cw) of z = [xl || h] per launch (rows wider than 64*HV run as several
// column chunks). Per workgroup slab: [g_wr (cw) | g_wc (cw) | g_br | g_bc].
template <int NV>
__global__ __launch_bounds__(256) void heads_bwd_kernel(
    const float* __restrict__ xl, int64_t dx, const float* __restrict__ h, int64_t dh, int64_t B,
    const float* __restrict__ w_r, const float* __restrict__ w_c, const float* __restrict__ ctr,
    const float* __restrict__ g_rating, const float* __restrict__ g_ctr,
    const float* __restrict__ unit_r, const float* __restrict__ unit_c,
    const float* __restrict__ gs_rat, const float* __restrict__ gs_ctr, float* __restrict__ g_xl,
    float* __restrict__ g_h, int64_t c0, int64_t cw, float* __restrict__ slab, float wsr = 1.f, float wsc = 1.f,
    float* __restrict__ g_ret = nullptr, float w_ret = 0.f, int relu_h = 0) {
  extern __shared__ float red[];  // [4][2*cw + 2]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t dz = c0 + cw;  // last column (exclusive) of this chunk
  const int64_t nw = (int64_t)gridDim.x * 4;
  // the loss weighting's backward folded in (rs_heads_bwd_combine_f32): the per-task upstream
  // scalars are g * w_task (the products loss_combine_bwd_kernel formed), and the retrieval
  // term's gradient g * w_ret is written once
  const float sr = gs_rat ? gs_rat[0] * wsr : 0.f;
  const float sc = gs_ctr ? gs_ctr[0] * wsc : 0.f;
  if (g_ret && blockIdx.x == 0 && threadIdx.x == 0 && c0 == 0) g_ret[0] = gs_rat[0] * w_ret;
  float awr[NV], awc[NV], abr = 0.f, abc = 0.f;
  float wr[NV], wc[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int64_t e = c0 + lane + 64 * j;
    awr[j] = awc[j] = 0.f;
    wr[j] = e < dz ? w_r[e] : 0.f;
    wc[j] = e < dz ? w_c[e] : 0.f;
  }
  // the next row's per-row scalars and z values are loaded while the current row is computed:
  // every load unconditional (absent per-row terms read the ctr row and are scaled by 0; the
  // column is clamped into the chunk), so hipcc does not wait on them at a branch join
  const float* grp = g_rating ? g_rating : ctr;
  const float* urp = (unit_r && gs_rat) ? unit_r : ctr;
  const float* gcp = g_ctr ? g_ctr : ctr;
  const float* ucp = (unit_c && gs_ctr) ? unit_c : ctr;
  const float fgr = g_rating ? 1.f : 0.f, fur = (unit_r && gs_rat) ? sr : 0.f;
  const float fgc = g_ctr ? 1.f : 0.f, fuc = (unit_c && gs_ctr) ? sc : 0.f;
  const float* zp[NV];
  int64_t zs[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    int64_t e = c0 + lane + 64 * j;
    if (e >= dz) e = dz - 1;
    zp[j] = e < dx ? xl + e : h + (e - dx);
    zs[j] = e < dx ? dx : dh;
  }
  float q_gr, q_ur, q_gc, q_uc, q_p, qz[NV];
  auto fetch = [&](int64_t bb) __attribute__((always_inline)) {
    if (bb >= B) bb = B - 1;
    q_gr = grp[bb];
    q_ur = urp[bb];
    q_gc = gcp[bb];
    q_uc = ucp[bb];
    q_p = ctr[bb];
#pragma unroll
    for (int j = 0; j < NV; ++j) qz[j] = zp[j][bb * zs[j]];
  };
  const int64_t bstart = (int64_t)blockIdx.x * 4 + wave;
  if (bstart < B) fetch(bstart);
  for (int64_t b = bstart; b < B; b += nw) {
    const float dr = (0.f + fgr * q_gr) + fur * q_ur;
    const float dp = (0.f + fgc * q_gc) + fuc * q_uc;
    const float p = q_p;
    float z[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) z[j] = qz[j];
    fetch(b + nw);
    const float dt = dp * (p * (1.f - p));
    abr += dr;
    abc += dt;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int64_t e = c0 + lane + 64 * j;
      if (e < dz) {
        awr[j] += dr * z[j];
        awc[j] += dt * z[j];
        const float gz = dr * wr[j] + dt * wc[j];
        if (e < dx) g_xl[b * dx + e] = gz;
        else g_h[b * dh + (e - dx)] = (relu_h && !(z[j] > 0.f)) ? 0.f : gz;  // ReluGrad of h's top layer
      }
    }
  }
  const int64_t per = 2 * cw + 2;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int64_t e = lane + 64 * j;  // local column
    if (e < cw) {
      red[wave * per + e] = awr[j];
      red[wave * per + cw + e] = awc[j];
    }
  }
  if (lane == 0) {
    red[wave * per + 2 * cw] = abr;
    red[wave * per + 2 * cw + 1] = abc;
  }
  __syncthreads();
  for (int64_t i = threadIdx.x; i < per; i += 256)
    slab[(int64_t)blockIdx.x * per + i] = ((red[i] + red[per + i]) + red[2 * per + i]) + red[3 * per + i];
}

static int64_t heads_blocks(int64_t B) {
  int64_t nb = ceil_div(B, 4);  // one row per wave up to 1024 workgroups, then grid-stride
  if (nb < 1) nb = 1;
  if (nb > 1024) nb = 1024;
  return nb;
}

// ---- ranking losses --------------------------------------------------------------------
constexpr float kKerasEps = 1e-7f;  // keras.backend.epsilon()

// One row's terms {(r-y)^2, sw*bce, bce, sw}; writes unit_r and the raw dbce/dp.
__device__ __forceinline__ void rank_row(const float* __restrict__ r, const float* __restrict__ p,
                                         const float* __restrict__ y, const float* __restrict__ yi, int64_t b,
                                         int64_t B, int use_cw, float cw0, float cw1, int mode,
                                         float* __restrict__ unit_r, float* __restrict__ dbce, double (&a)[4]) {
  const float diff = r[b] - y[b];
  a[0] = (double)diff * diff;
  unit_r[b] = 2.f * diff / (float)B;
  const float yv = yi[b];
  const float sw = use_cw ? (yv == 1.f ? cw1 : cw0) : 1.f;
  const float pv = p[b];
  const float pc = fminf(fmaxf(pv, kKerasEps), 1.f - kKerasEps);
  const float bce = -(yv * logf(pc + kKerasEps) + (1.f - yv) * logf(1.f - pc + kKerasEps));
  // clip_by_value passes the gradient where eps <= p <= 1 - eps
  const bool pass = (pv >= kKerasEps) && (pv <= 1.f - kKerasEps);
  const float g = pass ? (-yv / (pc + kKerasEps) + (1.f - yv) / (1.f - pc + kKerasEps)) : 0.f;
  // mode 0 (per-sample weights) scales the unit gradient here (ranking_unit_c_kernel's product);
  // mode 1 needs the batch's mean weight first (ranking_unit_c_kernel after the final)
  dbce[b] = mode == 0 ? g * sw / (float)B : g;
  a[1] = (double)sw * bce;
  a[2] = bce;
  a[3] = sw;
}

// The partial of 256-row block blk = {sum (r-y)^2, sum sw*bce, sum bce, sum sw} by ONE wave: lane l
// adds rows 256 blk + l + 64 j in j order, then a butterfly over the wave (xor 32 .. 1). Both the
// multi-workgroup pass and the one-workgroup kernel use it, so their partials are bitwise equal.
__device__ __forceinline__ void rank_block(const float* __restrict__ r, const float* __restrict__ p,
                                           const float* __restrict__ y, const float* __restrict__ yi, int64_t blk,
                                           int64_t B, int use_cw, float cw0, float cw1, int mode,
                                           float* __restrict__ unit_r, float* __restrict__ dbce, double (&s)[4]) {
  const int lane = threadIdx.x & 63;
  s[0] = s[1] = s[2] = s[3] = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t b = blk * 256 + lane + 64 * j;
    if (b < B) {
      double a[4];
      rank_row(r, p, y, yi, b, B, use_cw, cw0, cw1, mode, unit_r, dbce, a);
#pragma unroll
      for (int k = 0; k < 4; ++k) s[k] += a[k];
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) s[k] = wave_sum_d(s[k]);
}

// partial[blk], one 256-row block per wave (four per workgroup)
__global__ __launch_bounds__(256) void ranking_partial_kernel(
    const float* __restrict__ r, const float* __restrict__ p, const float* __restrict__ y,
    const float* __restrict__ yi, int64_t B, int use_cw, float cw0, float cw1,
    float* __restrict__ unit_r, float* __restrict__ dbce, double* __restrict__ part, int mode) {
  const int64_t blk = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blk * 256 >= B) return;
  double s[4];
  rank_block(r, p, y, yi, blk, B, use_cw, cw0, cw1, mode, unit_r, dbce, s);
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < 4; ++k) part[blk * 4 + k] = s[k];
}

// the task weighting of compute_loss (src/models.py:147) on the final losses: total[0] = w_ret ret +
// w_rat rating (+ w_ctr ctr), fp32 left to right (loss_combine_kernel's form), total[1] = total[0]
// + reg (the train step's loss + sum(model.losses), reg nullable: + 0)
struct RankCombine {
  const float* ret;
  const float* reg;
  float w_ret, w_rat, w_ctr;
  int use_ctr;
  float* total;
  float* total_reg;
};
__device__ inline void rank_combine(const RankCombine& c, float l0, float l1) {
  if (!c.total) return;
  const float t = (c.w_ret * c.ret[0] + c.w_rat * l0) + (c.use_ctr ? c.w_ctr * l1 : 0.f);
  c.total[0] = t;
  if (c.total_reg) c.total_reg[0] = c.reg ? t + c.reg[0] : t;
}

__global__ __launch_bounds__(256) void ranking_final_kernel(const double* __restrict__ part,
                                                            int64_t nb, int64_t B, int mode,
                                                            float* __restrict__ loss,
                                                            float* __restrict__ scal, RankCombine cmb = {}) {
  __shared__ double red[4][256];
  double a[4] = {0, 0, 0, 0};
  for (int64_t i = threadIdx.x; i < nb; i += 256)
    for (int k = 0; k < 4; ++k) a[k] += part[i * 4 + k];
  for (int k = 0; k < 4; ++k) red[k][threadIdx.x] = a[k];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
      for (int k = 0; k < 4; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double invB = 1.0 / (double)B;
    loss[0] = (float)(red[0][0] * invB);
    if (mode == 0) loss[1] = (float)(red[1][0] * invB);
    else loss[1] = (float)((red[2][0] * invB) * (red[3][0] * invB));
    scal[0] = (float)(red[3][0] * invB);  // mean sample weight
    rank_combine(cmb, loss[0], loss[1]);
  }
}

// Small batches (B <= 64 x 256): the partial pass, the final and (mode 1) the unit-gradient scaling
// in ONE workgroup of 16 waves (each wave a 256-row block at a time, all blocks' loads in flight
// together), the same per-block partials and final tree as the multi-launch path (bitwise).
__global__ __launch_bounds__(1024) void ranking_single_kernel(
    const float* __restrict__ r, const float* __restrict__ p, const float* __restrict__ y,
    const float* __restrict__ yi, int64_t B, int use_cw, float cw0, float cw1, int mode,
    float* __restrict__ unit_r, float* __restrict__ dbce, float* __restrict__ loss, RankCombine cmb) {
  __shared__ double red[4][256];
  __shared__ double part[64][4];
  __shared__ float scal_s;
  const int64_t nb = (B + 255) / 256;
  const int wave = threadIdx.x >> 6;
  for (int64_t blk = wave; blk < nb; blk += 16) {
    double s[4];
    rank_block(r, p, y, yi, blk, B, use_cw, cw0, cw1, mode, unit_r, dbce, s);
    if ((threadIdx.x & 63) == 0)
      for (int k = 0; k < 4; ++k) part[blk][k] = s[k];
  }
  __syncthreads();
  // ranking_final_kernel's tree (nb <= 64 <= 256: one partial per thread at most)
  if (threadIdx.x < 256) {
    double a[4] = {0, 0, 0, 0};
    if ((int64_t)threadIdx.x < nb)
      for (int k = 0; k < 4; ++k) a[k] = 0.0 + part[threadIdx.x][k];
    for (int k = 0; k < 4; ++k) red[k][threadIdx.x] = a[k];
  }
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
      for (int k = 0; k < 4; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double invB = 1.0 / (double)B;
    const float l0 = (float)(red[0][0] * invB);
    const float l1 = mode == 0 ? (float)(red[1][0] * invB) : (float)((red[2][0] * invB) * (red[3][0] * invB));
    loss[0] = l0;
    loss[1] = l1;
    scal_s = (float)(red[3][0] * invB);
    rank_combine(cmb, l0, l1);
  }
  if (mode != 0) {
    __syncthreads();
    const float f = scal_s;
    for (int64_t b = threadIdx.x; b < B; b += 1024) dbce[b] = dbce[b] * f / (float)B;
  }
}

// mode 1 only (Keras 3 rank-1 broadcasting: the batch's mean weight scales every row)
__global__ void ranking_unit_c_kernel(int64_t B, const float* __restrict__ scal, float* __restrict__ dbce) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  dbce[b] = dbce[b] * scal[0] / (float)B;
}

// compute_loss's task weighting (src/models.py:147): total = w_ret ret + w_rat rating + w_ctr ctr
// (fp32, left to right); the backward hands each term g * w.
__global__ void loss_combine_kernel(const float* __restrict__ ret, const float* __restrict__ rat,
                                    const float* __restrict__ ctr, float w0, float w1, float w2,
                                    float* __restrict__ total) {
  if (threadIdx.x == 0) total[0] = (w0 * ret[0] + w1 * rat[0]) + (ctr ? w2 * ctr[0] : 0.f);
}
__global__ void loss_combine_bwd_kernel(const float* __restrict__ g, float w0, float w1, float w2,
                                        float* __restrict__ grads) {
  if (threadIdx.x < 3) grads[threadIdx.x] = g[0] * (threadIdx.x == 0 ? w0 : (threadIdx.x == 1 ? w1 : w2));
}

}  // namespace rs


using namespace rs;

extern "C" {

int rs_heads_fwd_f32(const float* xl, int64_t dx, const float* h, int64_t dh, int64_t B,
                     const float* w_r, const float* b_r, const float* w_c, const float* b_c,
                     float* rating, float* ctr, rs_stream_t stream) {
  RS_REQUIRE(B >= 0 && dx >= 0 && dh >= 0 && dx + dh > 0, "rs_heads_fwd_f32: bad sizes");
  RS_REQUIRE((dx == 0 || xl) && (dh == 0 || h) && w_r && b_r && w_c && b_c && rating && ctr,
             "rs_heads_fwd_f32: null");
  if (B == 0) return RS_OK;
  int64_t nb = ceil_div(B, 4);
  if (nb > 256 * 32) nb = 256 * 32;
  hipLaunchKernelGGL(heads_fwd_kernel, dim3((unsigned)nb), dim3(256), 0, as_stream(stream), xl, dx, h, dh,
                     B, w_r, b_r, w_c, b_c, rating, ctr);
  return check_launch("heads_fwd");
}

size_t rs_heads_bwd_workspace_bytes(int64_t B, int64_t dx, int64_t dh) {
  const int64_t cw = (dx + dh) < 64 * HV ? (dx + dh) : 64 * HV;
  return align_up((size_t)heads_blocks(B) * (size_t)(2 * cw + 2) * sizeof(float), 256) + 256;
}

static int heads_bwd_impl(const float* xl, int64_t dx, const float* h, int64_t dh, int64_t B,
                          const float* w_r, const float* w_c, const float* ctr,
                          const float* g_rating, const float* g_ctr, const float* unit_r,
                          const float* unit_c, const float* gs_rat, const float* gs_ctr,
                          float* g_xl, float* g_h, float* g_wr, float* g_br, float* g_wc,
                          float* g_bc, void* workspace, size_t workspace_bytes, rs_stream_t stream,
                          void* queue, float wsr, float wsc, float* g_ret, float w_ret, int relu_h = 0) {
  const int64_t dz = dx + dh;
  RS_REQUIRE(B >= 0 && dx >= 0 && dh >= 0 && dz > 0, "rs_heads_bwd_f32: bad sizes");
  RS_REQUIRE(w_r && w_c && ctr && g_wr && g_br && g_wc && g_bc && (dx == 0 || (xl && g_xl)) &&
                 (dh == 0 || (h && g_h)),
             "rs_heads_bwd_f32: null");
  if (!workspace || workspace_bytes < rs_heads_bwd_workspace_bytes(B, dx, dh)) {
    set_error("rs_heads_bwd_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  const int64_t nb = heads_blocks(B);
  float* slab = static_cast<float*>(workspace);
  // one column chunk: the slab serves one set of reductions, which may be queued; several chunks
  // reuse the slab, so their reductions launch at once
  SlabQueue* one = dz <= 64 * HV ? static_cast<SlabQueue*>(queue) : nullptr;
  for (int64_t c0 = 0; c0 < dz; c0 += 64 * HV) {
    const int64_t cw = dz - c0 < 64 * HV ? dz - c0 : 64 * HV;
    const int64_t per = 2 * cw + 2;
    const size_t shm = (size_t)4 * per * sizeof(float);
    const int nv = (int)ceil_div(cw, 64);
#define RS_HEADS_BWD(NV)                                                                                  \
  hipLaunchKernelGGL((heads_bwd_kernel<NV>), dim3((unsigned)nb), dim3(256), shm, st, xl, dx, h, dh, B, w_r, w_c, \
                     ctr, g_rating, g_ctr, unit_r, unit_c, gs_rat, gs_ctr, g_xl, g_h, c0, cw, slab, wsr, wsc, g_ret, w_ret, \
                     relu_h)
    if (nv <= 2) RS_HEADS_BWD(2);
    else if (nv <= 4) RS_HEADS_BWD(4);
    else if (nv <= 8) RS_HEADS_BWD(8);
    else RS_HEADS_BWD(16);
#undef RS_HEADS_BWD
    int rc = check_launch("heads_bwd");
    if (rc) return rc;
    rc = launch_slab_reduce_strided(slab, nb, per, cw, g_wr + c0, nullptr, 0.f, st, nullptr, -1, one);
    if (rc) return rc;
    rc = launch_slab_reduce_strided(slab + cw, nb, per, cw, g_wc + c0, nullptr, 0.f, st, nullptr, -1, one);
    if (rc) return rc;
    if (c0 == 0) {
      rc = launch_slab_reduce_strided(slab + 2 * cw, nb, per, 1, g_br, nullptr, 0.f, st, nullptr, -1, one);
      if (rc) return rc;
      rc = launch_slab_reduce_strided(slab + 2 * cw + 1, nb, per, 1, g_bc, nullptr, 0.f, st, nullptr, -1, one);
      if (rc) return rc;
    }
  }
  return RS_OK;
}

int rs_heads_bwd_f32(const float* xl, int64_t dx, const float* h, int64_t dh, int64_t B,
                     const float* w_r, const float* w_c, const float* ctr,
                     const float* g_rating, const float* g_ctr, const float* unit_r,
                     const float* unit_c, const float* gs_rat, const float* gs_ctr,
                     float* g_xl, float* g_h, float* g_wr, float* g_br, float* g_wc,
                     float* g_bc, void* workspace, size_t workspace_bytes, rs_stream_t stream,
                     void* queue) {
  return heads_bwd_impl(xl, dx, h, dh, B, w_r, w_c, ctr, g_rating, g_ctr, unit_r, unit_c, gs_rat, gs_ctr, g_xl, g_h,
                        g_wr, g_br, g_wc, g_bc, workspace, workspace_bytes, stream, queue, 1.f, 1.f, nullptr, 0.f);
}

int rs_heads_bwd_combine_f32(const float* xl, int64_t dx, const float* h, int64_t dh, int64_t B, const float* w_r,
                             const float* w_c, const float* ctr, const float* unit_r, const float* unit_c,
                             const float* g_total, float w_ret, float w_rat, float w_ctr, int flags, float* g_ret,
                             float* g_xl, float* g_h, float* g_wr, float* g_br, float* g_wc, float* g_bc,
                             void* workspace, size_t workspace_bytes, rs_stream_t stream, void* queue) {
  RS_REQUIRE(g_total && g_ret && unit_r && unit_c, "rs_heads_bwd_combine_f32: null");
  RS_REQUIRE((flags & ~3) == 0, "rs_heads_bwd_combine_f32: unknown flags %d", flags);
  return heads_bwd_impl(xl, dx, h, dh, B, w_r, w_c, ctr, nullptr, nullptr, unit_r, unit_c, g_total,
                        (flags & RS_HEADS_USE_CTR) ? g_total : nullptr, g_xl, g_h, g_wr, g_br, g_wc, g_bc, workspace,
                        workspace_bytes, stream, queue, w_rat, w_ctr, g_ret, w_ret, (flags & RS_HEADS_RELU_H) ? 1 : 0);
}

size_t rs_ranking_losses_workspace_bytes(int64_t B) {
  return align_up((size_t)ceil_div(B > 0 ? B : 1, 256) * 4 * sizeof(double), 256) + 512;
}

static int ranking_impl(const char* fn, const float* rating_pred, const float* ctr_pred, const float* rating,
                        const float* y_implicit, int64_t B, int use_class_weights, float cw0, float cw1, int ctr_mode,
                        float* loss, float* unit_r, float* unit_c, const RankCombine& cmb, void* workspace,
                        size_t workspace_bytes, hipStream_t st) {
  RS_REQUIRE(B > 0, "%s: B must be > 0", fn);
  RS_REQUIRE(rating_pred && ctr_pred && rating && y_implicit && loss && unit_r && unit_c, "%s: null", fn);
  RS_REQUIRE(ctr_mode == 0 || ctr_mode == 1, "%s: ctr_mode must be 0 or 1", fn);
  if (!workspace || workspace_bytes < rs_ranking_losses_workspace_bytes(B)) {
    set_error("%s: workspace too small", fn);
    return RS_ERR_WORKSPACE;
  }
  const int64_t nb = ceil_div(B, 256);
  if (nb <= 64) {  // one launch: partials, final, weighting (and the mode-1 scaling) in one workgroup
    hipLaunchKernelGGL(ranking_single_kernel, dim3(1), dim3(1024), 0, st, rating_pred, ctr_pred, rating, y_implicit,
                       B, use_class_weights, cw0, cw1, ctr_mode, unit_r, unit_c, loss, cmb);
    return check_launch("ranking_single");
  }
  Carve c(workspace, workspace_bytes);
  double* part = c.take<double>(nb * 4);
  float* scal = c.take<float>(4);
  hipLaunchKernelGGL(ranking_partial_kernel, dim3((unsigned)ceil_div(nb, 4)), dim3(256), 0, st, rating_pred, ctr_pred,
                     rating, y_implicit, B, use_class_weights, cw0, cw1, unit_r, unit_c, part, ctr_mode);
  int rc = check_launch("ranking_partial");
  if (rc) return rc;
  hipLaunchKernelGGL(ranking_final_kernel, dim3(1), dim3(256), 0, st, part, nb, B, ctr_mode, loss, scal, cmb);
  rc = check_launch("ranking_final");
  if (rc || ctr_mode == 0) return rc;
  hipLaunchKernelGGL(ranking_unit_c_kernel, dim3((unsigned)nb), dim3(256), 0, st, B, scal, unit_c);
  return check_launch("ranking_unit_c");
}

int rs_ranking_losses_f32(const float* rating_pred, const float* ctr_pred, const float* rating,
                          const float* y_implicit, int64_t B, int use_class_weights, float cw0,
                          float cw1, int ctr_mode, float* loss, float* unit_r, float* unit_c,
                          void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  return ranking_impl("rs_ranking_losses_f32", rating_pred, ctr_pred, rating, y_implicit, B, use_class_weights, cw0,
                      cw1, ctr_mode, loss, unit_r, unit_c, RankCombine{}, workspace, workspace_bytes,
                      as_stream(stream));
}

int rs_ranking_losses_combine_f32(const float* rating_pred, const float* ctr_pred, const float* rating,
                                  const float* y_implicit, int64_t B, int use_class_weights, float cw0, float cw1,
                                  int ctr_mode, const float* ret, const float* reg, float w_ret, float w_rat,
                                  float w_ctr, int use_ctr, float* loss, float* total, float* total_reg,
                                  float* unit_r, float* unit_c, void* workspace, size_t workspace_bytes,
                                  rs_stream_t stream) {
  RS_REQUIRE(ret && total, "rs_ranking_losses_combine_f32: null");
  return ranking_impl("rs_ranking_losses_combine_f32", rating_pred, ctr_pred, rating, y_implicit, B,
                      use_class_weights, cw0, cw1, ctr_mode, loss, unit_r, unit_c,
                      RankCombine{ret, reg, w_ret, w_rat, w_ctr, use_ctr ? 1 : 0, total, total_reg}, workspace, workspace_bytes,
                      as_stream(stream));
}

int rs_loss_combine_f32(const float* ret, const float* rating, const float* ctr, float w_ret, float w_rat,
                        float w_ctr, float* total, rs_stream_t stream) {
  RS_REQUIRE(ret && rating && total, "rs_loss_combine_f32: null");
  hipLaunchKernelGGL(loss_combine_kernel, dim3(1), dim3(64), 0, as_stream(stream), ret, rating, ctr, w_ret, w_rat,
                     w_ctr, total);
  return check_launch("loss_combine");
}

int rs_loss_combine_bwd_f32(const float* g, float w_ret, float w_rat, float w_ctr, float* grads,
                            rs_stream_t stream) {
  RS_REQUIRE(g && grads, "rs_loss_combine_bwd_f32: null");
  hipLaunchKernelGGL(loss_combine_bwd_kernel, dim3(1), dim3(64), 0, as_stream(stream), g, w_ret, w_rat, w_ctr, grads);
  return check_launch("loss_combine_bwd");
}

}  // extern "C"
