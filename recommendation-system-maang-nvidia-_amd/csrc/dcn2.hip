// dcn2.hip — DCN-v2 matrix cross stack (BASELINE config 5; SURVEY §7 hard parts: an extension,
// the reference's cross weight is a [d,1] vector — see dcn.hip for the reference semantics).
//
//   u_l = x_l W_l + b_l ;  x_{l+1} = x0 ⊙ u_l + x_l        (W_l: [d, d] Keras layout [in][out])
//
// Forward: one GEMM per layer (f32 MFMA, or split bf16 at precision 6 / 9: gemm.hip) with the cross epilogue fused (gemm.hip, epi = 1: the
// epilogue stores u_l for the backward and writes x0 ⊙ u_l + x_l), so a layer is a single pass
// over [B, d]. Backward per layer, given g = dL/dx_{l+1}:
//   t = g ⊙ x0 ; dL/dx0 += g ⊙ u_l          (one vectorised elementwise pass)
//   db_l = colsum(t) ; dW_l = x_l^T t        (ordered column sums; split-K GEMM with ordered slabs)
//   dL/dx_l = t W_l^T + g                    (GEMM with the residual fused as an addend epilogue)
// The d x d GEMMs are the genuinely dense contraction of the path: MFMA-bound at d = 3,344.
#include "common.hpp"
#include "split.hpp"

namespace rs {

// t = g * x0 ; gx0 = base + g * u   (base nullable = 0; gx0 may alias base)
__global__ __launch_bounds__(256) void cross_mat_bwd_elem_kernel(
    const f32x4* __restrict__ g, const f32x4* __restrict__ x0, const f32x4* __restrict__ u,
    int64_t n4, f32x4* __restrict__ t, const f32x4* base, f32x4* gx0) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const f32x4 gv = g[i];
    t[i] = gv * x0[i];
    const f32x4 add = gv * u[i];
    gx0[i] = base ? base[i] + add : add;
  }
}

__global__ __launch_bounds__(256) void add2_kernel(const f32x4* __restrict__ a, const f32x4* b,
                                                   f32x4* out, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
    out[i] = a[i] + (b ? b[i] : f32x4{0.f, 0.f, 0.f, 0.f});
}

static unsigned elem_blocks(int64_t n4) {
  int64_t b = ceil_div(n4, 256 * 4);
  if (b < 1) b = 1;
  if (b > 4096) b = 4096;
  return (unsigned)b;
}

}  // namespace rs

using namespace rs;

extern "C" {

int rs_dcn_cross_mat_fwd_prec_f32(const float* x0, int64_t B, int64_t d, int L, const float* W,
                                  const float* b, float* xs, float* us, int precision, rs_stream_t stream) {
  RS_REQUIRE(B >= 0 && d > 0 && L >= 0, "rs_dcn_cross_mat_fwd_f32: bad sizes");
  RS_REQUIRE(d % 4 == 0, "rs_dcn_cross_mat_fwd_f32: d must be a multiple of 4 (pad x0)");
  RS_REQUIRE(x0 && (L == 0 || (W && b && xs && us)), "rs_dcn_cross_mat_fwd_f32: null");
  hipStream_t st = as_stream(stream);
  for (int l = 0; l < L; ++l) {
    const float* xin = l == 0 ? x0 : xs + (int64_t)(l - 1) * B * d;
    float* xout = xs + (int64_t)l * B * d;
    float* u = us + (int64_t)l * B * d;
    int rc = gemm_launch(0, 0, B, d, d, xin, d, W + (int64_t)l * d * d, d, xout, d, b + (int64_t)l * d, 1, x0,
                         xin, u, d, nullptr, 0, st, precision);
    if (rc) return rc;
  }
  return RS_OK;
}

int rs_dcn_cross_mat_fwd_f32(const float* x0, int64_t B, int64_t d, int L, const float* W,
                             const float* b, float* xs, float* us, rs_stream_t stream) {
  return rs_dcn_cross_mat_fwd_prec_f32(x0, B, d, L, W, b, xs, us, RS_PREC_F32, stream);
}

size_t rs_dcn_cross_mat_bwd_workspace_bytes(int64_t B, int64_t d, int L) {
  (void)L;
  Carve c(nullptr, 0);
  c.take<float>((size_t)B * d);  // t
  c.take<float>((size_t)B * d);  // g ping
  c.take<float>((size_t)B * d);  // g pong
  c.take<char>(rs_gemm_splitk_workspace_bytes(d, d, B));
  c.take<char>(rs_colsum_workspace_bytes(B, d));
  return c.off + 256;
}

int rs_dcn_cross_mat_bwd_prec_f32(const float* x0, const float* xs, const float* us, const float* W,
                                  int64_t B, int64_t d, int L, const float* g_xl,
                                  const float* g_x0_extra, float* g_x0, float* g_W, float* g_b, int precision,
                                  void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(B >= 0 && d > 0 && L >= 0 && d % 4 == 0, "rs_dcn_cross_mat_bwd_f32: bad sizes");
  RS_REQUIRE(x0 && g_xl && g_x0 && (L == 0 || (xs && us && W && g_W && g_b)),
             "rs_dcn_cross_mat_bwd_f32: null");
  const size_t need = rs_dcn_cross_mat_bwd_workspace_bytes(B, d, L);
  if (!workspace || workspace_bytes < need) {
    set_error("rs_dcn_cross_mat_bwd_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  const int64_t n4 = B * d / 4;
  const unsigned eb = elem_blocks(n4);
  if (B == 0) {
    if (L > 0) {
      RS_HIP(hipMemsetAsync(g_W, 0, (size_t)L * d * d * sizeof(float), st));
      RS_HIP(hipMemsetAsync(g_b, 0, (size_t)L * d * sizeof(float), st));
    }
    return RS_OK;
  }
  Carve c(workspace, workspace_bytes);
  float* t = c.take<float>((size_t)B * d);
  float* gp[2] = {c.take<float>((size_t)B * d), c.take<float>((size_t)B * d)};
  const size_t skb = rs_gemm_splitk_workspace_bytes(d, d, B);
  char* skws = c.take<char>(skb);
  const size_t csb = rs_colsum_workspace_bytes(B, d);
  char* csws = c.take<char>(csb);

  const float* g = g_xl;
  for (int l = L - 1; l >= 0; --l) {
    const float* xin = l == 0 ? x0 : xs + (int64_t)(l - 1) * B * d;
    const float* u = us + (int64_t)l * B * d;
    const float* base = (l == L - 1) ? g_x0_extra : g_x0;
    hipLaunchKernelGGL(cross_mat_bwd_elem_kernel, dim3(eb), dim3(256), 0, st, (const f32x4*)g, (const f32x4*)x0,
                       (const f32x4*)u, n4, (f32x4*)t, (const f32x4*)base, (f32x4*)g_x0);
    int rc = check_launch("cross_mat_bwd_elem");
    if (rc) return rc;
    rc = rs_relu_bwd_colsum_f32(t, nullptr, B, d, nullptr, g_b + (int64_t)l * d, csws, csb, stream, nullptr);
    if (rc) return rc;
    rc = rs_gemm_splitk_prec_f32(1, 0, d, d, B, xin, d, t, d, g_W + (int64_t)l * d * d, d, nullptr, 0.f,
                                 precision, skws, skb, stream);
    if (rc) return rc;
    // dL/dx_l = t W_l^T + dL/dx_{l+1}; at l = 0 the epilogue also adds the direct terms already
    // in g_x0 (beta = 1: (t W^T + g) + g_x0, the order of the former separate add)
    float* gnew = l == 0 ? g_x0 : gp[l & 1];
    rc = gemm_launch(0, 1, B, d, d, t, d, W + (int64_t)l * d * d, d, gnew, d, nullptr, 0, nullptr, nullptr,
                     nullptr, 0, g, d, st, precision, l == 0 ? 1.f : 0.f);
    if (rc) return rc;
    g = gnew;
  }
  if (L > 0) return RS_OK;
  // no cross layer: dL/dx0 = the residual gradient plus the caller's extra term
  hipLaunchKernelGGL(add2_kernel, dim3(eb), dim3(256), 0, st, (const f32x4*)g_xl, (const f32x4*)g_x0_extra,
                     (f32x4*)g_x0, n4);
  return check_launch("cross_mat_add");
}

// ---- plane-image path (precision 6): operands split once per GEMM into xgemm images (gemm.hip),
// GEMMs on the plane-pair kernel (two cross products per 16x16x32 MFMA, 256 x 256 tiles, LDS-DMA
// ring): forward x_l W_l from the images of x_l and W_l^T; backward dW_l = x_l^T t from the image of
// x_l^T (written by the forward and kept) and of t^T, dL/dx_l = t W_l^T + g from the images of t and
// W_l. Same sums as the split-at-staging path up to the order of the fp32 additions (both within a
// few fp32 ulps of the exact products).
size_t rs_dcn_cross_mat_planes_bytes(int64_t B, int64_t d, int L) {
  return (size_t)(L > 0 ? L : 0) * align_up(ximg_bytes(d, B), 256);  // image of x_l^T, kept for the backward
}

size_t rs_dcn_cross_mat_fwd_planes_workspace_bytes(int64_t B, int64_t d) {
  Carve c(nullptr, 0);
  c.take<char>(ximg_bytes(B, d));  // x_l
  c.take<char>(ximg_bytes(d, d));  // W_l^T
  c.take<char>(xgemm_tail_ws_bytes(B, d, d));  // the GEMM's last round split over K
  return c.off + 256;
}

int rs_dcn_cross_mat_fwd_planes_f32(const float* x0, int64_t B, int64_t d, int L, const float* W, const float* b,
                                    float* xs, float* us, void* ximg, int precision, void* workspace,
                                    size_t workspace_bytes, rs_stream_t stream) {
  return rs_dcn_cross_mat_fwd_planes_x0img_f32(x0, B, d, L, W, b, xs, us, ximg, nullptr, precision, workspace,
                                               workspace_bytes, stream);
}

int rs_dcn_cross_mat_fwd_planes_x0img_f32(const float* x0, int64_t B, int64_t d, int L, const float* W,
                                          const float* b, float* xs, float* us, void* ximg, void* x0_img,
                                          int precision, void* workspace, size_t workspace_bytes,
                                          rs_stream_t stream) {
  RS_REQUIRE(B >= 0 && d > 0 && L >= 0 && d % 4 == 0, "rs_dcn_cross_mat_fwd_planes_f32: bad sizes");
  RS_REQUIRE(precision == RS_PREC_F32_SPLIT6, "rs_dcn_cross_mat_fwd_planes_f32: precision must be 6");
  RS_REQUIRE(x0 && (L == 0 || (W && b && xs && us && ximg)), "rs_dcn_cross_mat_fwd_planes_f32: null");
  RS_REQUIRE(aligned16(x0) && (L == 0 || (aligned16(W) && aligned16(xs) && aligned16(ximg))),
             "rs_dcn_cross_mat_fwd_planes_f32: 16-byte alignment");
  if (B == 0 || L == 0) return RS_OK;
  if (!workspace || workspace_bytes < rs_dcn_cross_mat_fwd_planes_workspace_bytes(B, d)) {
    set_error("rs_dcn_cross_mat_fwd_planes_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  Carve c(workspace, workspace_bytes);
  char* ximg_x = c.take<char>(ximg_bytes(B, d));
  char* ximg_wt = c.take<char>(ximg_bytes(d, d));
  const size_t twb = xgemm_tail_ws_bytes(B, d, d);
  char* tws = c.take<char>(twb);
  const size_t xt_bytes = align_up(ximg_bytes(d, B), 256);
  for (int l = 0; l < L; ++l) {
    const float* xin = l == 0 ? x0 : xs + (int64_t)(l - 1) * B * d;
    float* xout = xs + (int64_t)l * B * d;
    float* u = us + (int64_t)l * B * d;
    // x_l's image (A of x_l W) and its transpose's (kept for dW_l = x_l^T t) from one read; x0's
    // plain image goes to the caller's x0_img when given (the DCN-v2 deep tower reuses it)
    char* a_img = (l == 0 && x0_img) ? static_cast<char*>(x0_img) : ximg_x;
    int rc = ximg_dual_launch(xin, nullptr, nullptr, nullptr, nullptr, B, d, a_img,
                              static_cast<char*>(ximg) + (size_t)l * xt_bytes, nullptr, st);
    if (rc) return rc;
    rc = ximg_launch(W + (int64_t)l * d * d, d, d, d, 1, ximg_wt, st);
    if (rc) return rc;
    rc = xgemm_launch_ws(B, d, d, a_img, ximg_wt, xout, d, b + (int64_t)l * d, RS_ACT_NONE, 1, x0, xin, u, d, nullptr,
                         0, st, precision, 0.f, tws, twb);
    if (rc) return rc;
  }
  return RS_OK;
}

size_t rs_dcn_cross_mat_bwd_planes_workspace_bytes(int64_t B, int64_t d, int L) {
  if (L == 0 || B == 0) return rs_dcn_cross_mat_bwd_workspace_bytes(B, d, L);  // the row path's degenerate cases
  Carve c(nullptr, 0);
  c.take<float>((size_t)B * d);    // g ping
  c.take<float>((size_t)B * d);    // g pong
  c.take<char>(ximg_bytes(B, d));  // t
  c.take<char>(ximg_bytes(d, B));  // t^T
  c.take<char>(ximg_bytes(d, d));  // W_l
  c.take<char>(xgemm_splitk_ws_bytes(d, d, B));
  c.take<float>((size_t)ceil_div(B, 256) * d);  // column-sum partials of t (per 256-row block)
  c.take<char>(xgemm_tail_ws_bytes(B, d, d));    // the dX GEMM's last round split over K
  return c.off + 256;
}

int rs_dcn_cross_mat_bwd_planes_f32(const float* x0, const float* xs, const float* us, const float* W,
                                    const void* ximg, int64_t B, int64_t d, int L, const float* g_xl,
                                    const float* g_x0_extra, float* g_x0, float* g_W, float* g_b, int precision,
                                    void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(B >= 0 && d > 0 && L >= 0 && d % 4 == 0, "rs_dcn_cross_mat_bwd_planes_f32: bad sizes");
  RS_REQUIRE(precision == RS_PREC_F32_SPLIT6, "rs_dcn_cross_mat_bwd_planes_f32: precision must be 6");
  RS_REQUIRE(x0 && g_xl && g_x0 && (L == 0 || (xs && us && W && ximg && g_W && g_b)),
             "rs_dcn_cross_mat_bwd_planes_f32: null");
  if (L == 0 || B == 0)
    return rs_dcn_cross_mat_bwd_prec_f32(x0, xs, us, W, B, d, L, g_xl, g_x0_extra, g_x0, g_W, g_b, RS_PREC_F32,
                                         workspace, workspace_bytes, stream);
  const size_t need = rs_dcn_cross_mat_bwd_planes_workspace_bytes(B, d, L);
  if (!workspace || workspace_bytes < need) {
    set_error("rs_dcn_cross_mat_bwd_planes_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  Carve c(workspace, workspace_bytes);
  float* gp[2] = {c.take<float>((size_t)B * d), c.take<float>((size_t)B * d)};
  char* img_t = c.take<char>(ximg_bytes(B, d));
  char* img_tt = c.take<char>(ximg_bytes(d, B));
  char* img_w = c.take<char>(ximg_bytes(d, d));
  const size_t skb = xgemm_splitk_ws_bytes(d, d, B);
  char* skws = c.take<char>(skb);
  const int64_t nrb = ceil_div(B, 256);
  float* cpart = c.take<float>((size_t)nrb * d);
  const size_t twb = xgemm_tail_ws_bytes(B, d, d);
  char* tws = c.take<char>(twb);
  const size_t xt_bytes = align_up(ximg_bytes(d, B), 256);

  const float* g = g_xl;
  for (int l = L - 1; l >= 0; --l) {
    const float* u = us + (int64_t)l * B * d;
    const float* base = (l == L - 1) ? g_x0_extra : g_x0;
    // t = dL/dx_{l+1} * x0 as the images of t and t^T, dL/dx0 = base + g * u, and t's column
    // partials, from one read of g, x0, u and base (t itself is never written)
    int rc = ximg_dual_launch(g, x0, u, base, g_x0, B, d, img_t, img_tt, cpart, st);
    if (rc) return rc;
    rc = launch_slab_reduce(cpart, nrb, d, g_b + (int64_t)l * d, nullptr, 0.f, st);  // db_l (ordered)
    if (rc) return rc;
    // dW_l = x_l^T t (K = B split over workgroups, ordered slabs)
    rc = xgemm_splitk_launch(d, d, B, static_cast<const char*>(ximg) + (size_t)l * xt_bytes, img_tt,
                             g_W + (int64_t)l * d * d, nullptr, 0.f, precision, skws, skb, st);
    if (rc) return rc;
    rc = ximg_launch(W + (int64_t)l * d * d, d, d, d, 0, img_w, st);
    if (rc) return rc;
    // dL/dx_l = t W_l^T + dL/dx_{l+1} (+ g_x0 at l = 0, beta = 1, as the row path)
    float* gnew = l == 0 ? g_x0 : gp[l & 1];
    rc = xgemm_launch_ws(B, d, d, img_t, img_w, gnew, d, nullptr, RS_ACT_NONE, 0, nullptr, nullptr, nullptr, 0, g, d,
                         st, precision, l == 0 ? 1.f : 0.f, tws, twb);
    if (rc) return rc;
    g = gnew;
  }
  return RS_OK;
}

int rs_dcn_cross_mat_bwd_f32(const float* x0, const float* xs, const float* us, const float* W,
                             int64_t B, int64_t d, int L, const float* g_xl,
                             const float* g_x0_extra, float* g_x0, float* g_W, float* g_b,
                             void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  return rs_dcn_cross_mat_bwd_prec_f32(x0, xs, us, W, B, d, L, g_xl, g_x0_extra, g_x0, g_W, g_b, RS_PREC_F32,
                                       workspace, workspace_bytes, stream);
}

}  // extern "C"
