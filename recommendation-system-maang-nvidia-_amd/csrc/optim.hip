// optim.hip — multi-tensor dense Adagrad with per-tensor clip-by-norm.
//
// Reference: model.compile(optimizer=keras.optimizers.Adagrad(ExponentialDecay(lr, 1000, 0.96,
// staircase=True), clipnorm=1.0)) (src/trainer.py:157-163), Keras >= 2.11 semantics:
//   g <- tf.clip_by_norm(g, clipnorm) = g * clipnorm / max(||g||_2, clipnorm)   (per variable)
//   acc += g*g ; var -= lr_t * g / sqrt(acc + epsilon)    (initial_accumulator_value = 0.1)
//   lr_t = lr0 * decay_rate ^ floor(iterations / decay_steps)
// All ~30 dense variables are updated by two launches (norm partials; update, each workgroup
// forming its tensor's norm from the partials) driven by a device-resident slot table, so the whole step is graph-capturable; the
// learning rate is computed on the device from the iteration counter (graph replay safe).
#include "common.hpp"

#include <cmath>

namespace rs {

// Partial blocks per tensor for the norm: enough that the largest tensor (the 45M-element DCN-v2
// cross stack) streams at HBM rate, never fewer than 32. Depends only on max_numel, so the
// workspace size and the reduction order are fixed for a given model.
static int opt_nb(int64_t max_numel) {
  int64_t nb = ceil_div(max_numel > 0 ? max_numel : 1, (int64_t)256 * 64);
  return (int)(nb < 32 ? 32 : (nb > 1024 ? 1024 : nb));
}

__global__ __launch_bounds__(256) void adagrad_norm_partial_kernel(const rs_dense_slot* __restrict__ slots,
                                                                   double* __restrict__ part, int nb) {
  __shared__ double red[256];
  const rs_dense_slot sl = slots[blockIdx.y];
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < sl.numel; i += (int64_t)nb * 256) {
    const float g = sl.grad[i];
    acc += (double)g * g;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(int64_t)blockIdx.y * nb + blockIdx.x] = red[0];
}

// the clip denominator of tensor t from its nb partials, by one wave: lane j sums partials j,
// j + 64, ... in order, then a fixed xor tree (the order depends only on nb, so the norm is
// reproducible run to run). Every update workgroup forms its tensor's denominator itself (a few
// L2-resident loads) instead of a separate launch doing it once.
__device__ inline float adagrad_denom(const double* __restrict__ part, int t, int nb, float clipnorm, int lane) {
  double s = 0.0;
  for (int b = lane; b < nb; b += 64) s += part[(int64_t)t * nb + b];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float l2 = s > 0.0 ? (float)sqrt(s) : 0.f;
  return fmaxf(l2, clipnorm);
}

__global__ __launch_bounds__(256) void adagrad_update_kernel(const rs_dense_slot* __restrict__ slots,
                                                             const double* __restrict__ part, int nb,
                                                             const int64_t* __restrict__ iteration,
                                                             float lr0, float decay_rate,
                                                             int64_t decay_steps, float clipnorm,
                                                             float eps) {
  __shared__ float dn_s;
  const rs_dense_slot sl = slots[blockIdx.y];
  const float step = (float)iteration[0];
  const float lr = lr0 * powf(decay_rate, floorf(step / (float)decay_steps));
  const bool clip = clipnorm > 0.f;
  if (clip) {
    if (threadIdx.x < 64) {
      const float d = adagrad_denom(part, blockIdx.y, nb, clipnorm, threadIdx.x);
      if (threadIdx.x == 0) dn_s = d;
    }
    __syncthreads();
  }
  const float dn = clip ? dn_s : 1.f;
  auto upd = [&](float g, float& a, float& p) __attribute__((always_inline)) {
    if (clip) g = (g * clipnorm) / dn;
    a = a + g * g;
    p -= lr * g / sqrtf(a + eps);
  };
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i0 = 0;
  if (((reinterpret_cast<uintptr_t>(sl.param) | reinterpret_cast<uintptr_t>(sl.grad) |
        reinterpret_cast<uintptr_t>(sl.accum)) & 15u) == 0) {
    // float4 lanes over the bulk (the same elementwise arithmetic), then the scalar tail
    const int64_t n4 = sl.numel / 4;
    f32x4* P = reinterpret_cast<f32x4*>(sl.param);
    f32x4* A = reinterpret_cast<f32x4*>(sl.accum);
    const f32x4* G = reinterpret_cast<const f32x4*>(sl.grad);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
      const f32x4 g = G[i];
      const f32x4 a4 = A[i], p4 = P[i];
      float a[4] = {a4[0], a4[1], a4[2], a4[3]}, p[4] = {p4[0], p4[1], p4[2], p4[3]};
#pragma unroll
      for (int e = 0; e < 4; ++e) upd(g[e], a[e], p[e]);
      A[i] = f32x4{a[0], a[1], a[2], a[3]};
      P[i] = f32x4{p[0], p[1], p[2], p[3]};
    }
    i0 = 4 * n4;
  }
  for (int64_t i = i0 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < sl.numel; i += stride) {
    float a = sl.accum[i], p = sl.param[i];
    upd(sl.grad[i], a, p);
    sl.accum[i] = a;
    sl.param[i] = p;
  }
}

}  // namespace rs

using namespace rs;

extern "C" {

size_t rs_adagrad_dense_workspace_bytes(int ntensors, int64_t max_numel) {
  return align_up((size_t)ntensors * opt_nb(max_numel) * sizeof(double), 256) +
         align_up((size_t)ntensors * sizeof(float), 256) + 256;
}

int rs_adagrad_dense_f32(const rs_dense_slot* slots, int ntensors, int64_t max_numel,
                         const int64_t* iteration, float lr0, float decay_rate,
                         int64_t decay_steps, float clipnorm, float epsilon, void* workspace,
                         size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(ntensors >= 0 && max_numel >= 0, "rs_adagrad_dense_f32: bad sizes");
  RS_REQUIRE(ntensors <= 65535, "rs_adagrad_dense_f32: too many tensors");
  RS_REQUIRE(slots && iteration, "rs_adagrad_dense_f32: null");
  RS_REQUIRE(decay_steps > 0, "rs_adagrad_dense_f32: decay_steps must be > 0");
  if (ntensors == 0) return RS_OK;
  if (!workspace || workspace_bytes < rs_adagrad_dense_workspace_bytes(ntensors, max_numel)) {
    set_error("rs_adagrad_dense_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  Carve c(workspace, workspace_bytes);
  const int nb = opt_nb(max_numel);
  double* part = c.take<double>((size_t)ntensors * nb);
  if (clipnorm > 0.f) {
    hipLaunchKernelGGL(adagrad_norm_partial_kernel, dim3(nb, ntensors), dim3(256), 0, st, slots, part, nb);
    int rc = check_launch("adagrad_norm_partial");
    if (rc) return rc;
  }
  int64_t bx = ceil_div(max_numel > 0 ? max_numel : 1, 256 * 4);
  if (bx > 2048) bx = 2048;
  hipLaunchKernelGGL(adagrad_update_kernel, dim3((unsigned)bx, ntensors), dim3(256), 0, st, slots, part, nb,
                     iteration, lr0, decay_rate, decay_steps, clipnorm, epsilon);
  return check_launch("adagrad_update");
}

}  // extern "C"
