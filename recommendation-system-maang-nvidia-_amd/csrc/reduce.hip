// reduce.hip — ABI plumbing + ordered (bitwise reproducible) reductions shared by the kernels.
//
// Every cross-workgroup sum in this library is a two-stage ordered reduction: each workgroup
// writes a partial "slab" whose element→thread assignment depends only on the launch shape,
// then one pass sums the slabs in an order fixed by the launch shape. No float atomics anywhere, so a rerun on the
// same inputs is bit-identical (the reference's TF kernels make no such promise; the build
// adds it so replicas under data parallelism stay identical).
#include "common.hpp"

#include <string>

namespace rs {

static thread_local char g_err[512] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return RS_ERR_HIP;
  }
  return RS_OK;
}

// out[i] = sum_{s<S} slab[s*stride + i] (+ addend_scale * addend[i]) in one launch, in a fixed
// order that depends only on (S, count): T threads share each output (T = the power of two that
// leaves each thread <= 8 slabs); thread j of an output sums slabs j, j+T, j+2T, ... into four
// interleaved accumulators, and the T partials meet in a fixed LDS tree. Every load of a thread
// is independent, so a reduction over hundreds of slabs costs two or three memory round trips,
// not hundreds.
template <int T>
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* __restrict__ slab, int64_t S,
                                                          int64_t stride, int64_t count,
                                                          float* __restrict__ out,
                                                          const float* __restrict__ addend,
                                                          float addend_scale, const float* __restrict__ dscale,
                                                          int64_t addend_count) {
  constexpr int OW = 256 / T;  // outputs per workgroup; adjacent lanes take adjacent outputs
  const int t = threadIdx.x;
  const int o = t % OW, j = t / OW;
  const int64_t i = (int64_t)blockIdx.x * OW + o;
  float acc = 0.f;
  if (i < count) {
    const float* p = slab + i;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int64_t s = j;
    for (; s + 3 * T < S; s += 4 * T) {
      a0 += p[s * stride];
      a1 += p[(s + T) * stride];
      a2 += p[(s + 2 * T) * stride];
      a3 += p[(s + 3 * T) * stride];
    }
    if (s < S) a0 += p[s * stride];
    if (s + T < S) a1 += p[(s + T) * stride];
    if (s + 2 * T < S) a2 += p[(s + 2 * T) * stride];
    acc = (a0 + a1) + (a2 + a3);
  }
  if constexpr (T > 1) {
    __shared__ float red[256];
    red[t] = acc;
    __syncthreads();
#pragma unroll
    for (int h = T / 2; h > 0; h >>= 1) {
      if (j < h) red[t] += red[t + h * OW];
      __syncthreads();
    }
    acc = red[o];
  }
  if (j == 0 && i < count) {
    if (addend && i < addend_count) acc += (dscale ? addend_scale * dscale[0] : addend_scale) * addend[i];
    out[i] = acc;
  }
}

// float4 form (count, stride multiples of 4, 16-B aligned): each lane sums 4 adjacent outputs
// with exactly the slab sequence and tree of slab_reduce_kernel<T> per component (bitwise the
// same sums), so 256 / T lanes of a slab read 16 * 256 / T contiguous bytes (whole 128-B lines
// at T <= 32) instead of 4 * 256 / T.
template <int T>
__global__ __launch_bounds__(256) void slab_reduce4_kernel(const f32x4* __restrict__ slab, int64_t S,
                                                           int64_t stride4, int64_t count4,
                                                           f32x4* __restrict__ out,
                                                           const f32x4* __restrict__ addend,
                                                           float addend_scale, const float* __restrict__ dscale,
                                                           int64_t addend_count4) {
  constexpr int OW = 256 / T;
  const int t = threadIdx.x;
  const int o = t % OW, j = t / OW;
  const int64_t i = (int64_t)blockIdx.x * OW + o;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (i < count4) {
    const f32x4* p = slab + i;
    f32x4 a0 = acc, a1 = acc, a2 = acc, a3 = acc;
    int64_t s = j;
    for (; s + 3 * T < S; s += 4 * T) {
      a0 += p[s * stride4];
      a1 += p[(s + T) * stride4];
      a2 += p[(s + 2 * T) * stride4];
      a3 += p[(s + 3 * T) * stride4];
    }
    if (s < S) a0 += p[s * stride4];
    if (s + T < S) a1 += p[(s + T) * stride4];
    if (s + 2 * T < S) a2 += p[(s + 2 * T) * stride4];
    acc = (a0 + a1) + (a2 + a3);
  }
  if constexpr (T > 1) {
    __shared__ f32x4 red[256];
    red[t] = acc;
    __syncthreads();
#pragma unroll
    for (int h = T / 2; h > 0; h >>= 1) {
      if (j < h) red[t] += red[t + h * OW];
      __syncthreads();
    }
    acc = red[o];
  }
  if (j == 0 && i < count4) {
    if (addend && i < addend_count4) acc += (dscale ? addend_scale * dscale[0] : addend_scale) * addend[i];
    out[i] = acc;
  }
}

// ---- deferred reductions --------------------------------------------------------------------
// Between rs_reductions_defer(1) and rs_reductions_flush the second stages of the library's ordered
// reductions (weight and bias gradients: split-K slabs, column-sum partials) are queued instead of
// launched one by one, and the flush runs them all in one launch: each workgroup serves one job
// with the runtime T of that job and exactly the slab sequence, accumulators and LDS tree of
// slab_reduce_kernel<T> / slab_reduce4_kernel<T> (bitwise the same sums). At small batches a
// training step is launch-bound (~4.5 us per launch), and a step queues ~13 of these.
struct SlabJob {
  const float* slab;
  float* out;
  const float* addend;
  const float* dscale;
  int64_t S, stride, count, addend_count;  // in floats, or in float4 for vec jobs
  float addend_scale;
  int T, vec, block0;
};
constexpr int kMaxSlabJobs = 36;  // kernel arguments stay under 4 KB
struct SlabJobs {
  SlabJob j[kMaxSlabJobs];
  int n;
};

__global__ __launch_bounds__(256) void slab_reduce_batch_kernel(SlabJobs jobs) {
  int k = 0;
  for (int q = 1; q < jobs.n; ++q)
    if ((int)blockIdx.x >= jobs.j[q].block0) k = q;
  const SlabJob& jb = jobs.j[k];
  const int T = jb.T, OW = 256 / T;
  const int t = threadIdx.x;
  const int o = t % OW, jj = t / OW;
  const int64_t i = (int64_t)(blockIdx.x - jb.block0) * OW + o;
  const int64_t S = jb.S, stride = jb.stride;
  __shared__ f32x4 red[256];
  if (jb.vec) {
    const f32x4* p = reinterpret_cast<const f32x4*>(jb.slab) + i;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (i < jb.count) {
      f32x4 a0 = acc, a1 = acc, a2 = acc, a3 = acc;
      int64_t s = jj;
      for (; s + 3 * T < S; s += 4 * T) {
        a0 += p[s * stride];
        a1 += p[(s + T) * stride];
        a2 += p[(s + 2 * T) * stride];
        a3 += p[(s + 3 * T) * stride];
      }
      if (s < S) a0 += p[s * stride];
      if (s + T < S) a1 += p[(s + T) * stride];
      if (s + 2 * T < S) a2 += p[(s + 2 * T) * stride];
      acc = (a0 + a1) + (a2 + a3);
    }
    if (T > 1) {
      red[t] = acc;
      __syncthreads();
      for (int h = T / 2; h > 0; h >>= 1) {
        if (jj < h) red[t] += red[t + h * OW];
        __syncthreads();
      }
      acc = red[o];
    }
    if (jj == 0 && i < jb.count) {
      const f32x4* ad = reinterpret_cast<const f32x4*>(jb.addend);
      if (ad && i < jb.addend_count) acc += (jb.dscale ? jb.addend_scale * jb.dscale[0] : jb.addend_scale) * ad[i];
      reinterpret_cast<f32x4*>(jb.out)[i] = acc;
    }
  } else {
    const float* p = jb.slab + i;
    float acc = 0.f;
    if (i < jb.count) {
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
      int64_t s = jj;
      for (; s + 3 * T < S; s += 4 * T) {
        a0 += p[s * stride];
        a1 += p[(s + T) * stride];
        a2 += p[(s + 2 * T) * stride];
        a3 += p[(s + 3 * T) * stride];
      }
      if (s < S) a0 += p[s * stride];
      if (s + T < S) a1 += p[(s + T) * stride];
      if (s + 2 * T < S) a2 += p[(s + 2 * T) * stride];
      acc = (a0 + a1) + (a2 + a3);
    }
    if (T > 1) {
      float* rs_ = reinterpret_cast<float*>(red);
      rs_[t] = acc;
      __syncthreads();
      for (int h = T / 2; h > 0; h >>= 1) {
        if (jj < h) rs_[t] += rs_[t + h * OW];
        __syncthreads();
      }
      acc = rs_[o];
    }
    if (jj == 0 && i < jb.count) {
      if (jb.addend && i < jb.addend_count)
        acc += (jb.dscale ? jb.addend_scale * jb.dscale[0] : jb.addend_scale) * jb.addend[i];
      jb.out[i] = acc;
    }
  }
}

// The queue lives in caller-owned host memory (rs_reduction_queue_bytes): the library holds no
// state between calls. One queue serves one training loop (one backward at a time); its jobs are
// bound to the stream they were queued on.
constexpr uint64_t kQueueMagic = 0x7273517565756531ull;  // "rsQueue1"
struct SlabQueue {
  uint64_t magic;
  hipStream_t stream;
  int blocks;
  SlabJobs jobs;
};

static int flush_queue(SlabQueue* q) {
  if (q->jobs.n == 0) return RS_OK;
  hipLaunchKernelGGL(slab_reduce_batch_kernel, dim3((unsigned)q->blocks), dim3(256), 0, q->stream, q->jobs);
  q->jobs.n = 0;
  q->blocks = 0;
  return check_launch("slab_reduce_batch");
}

int launch_slab_reduce_strided(const float* slab, int64_t S, int64_t stride, int64_t count,
                               float* out, const float* addend, float addend_scale,
                               hipStream_t st, const float* addend_dscale, int64_t addend_count,
                               SlabQueue* q) {
  if (count <= 0) return RS_OK;
  if (addend_count < 0 || addend_count > count) addend_count = count;
  int T = 1;
  while (T < 256 && (int64_t)T * 8 < S) T <<= 1;
  if (q) {
    if (q->magic != kQueueMagic) {
      set_error("deferred reduction: the queue was not initialised (rs_reduction_queue_init)");
      return RS_ERR_INVALID_ARG;
    }
    if (q->jobs.n == kMaxSlabJobs || (q->jobs.n > 0 && st != q->stream)) {
      const int rc = flush_queue(q);  // on the stream its jobs were queued on
      if (rc) return rc;
    }
    q->stream = st;
    const bool vec = count % 4 == 0 && stride % 4 == 0 && addend_count % 4 == 0 && aligned16(slab) &&
                     aligned16(out) && (!addend || aligned16(addend));
    const int64_t c = vec ? count / 4 : count;
    SlabJob& jb = q->jobs.j[q->jobs.n++];
    jb = SlabJob{slab, out, addend, addend_dscale, S, vec ? stride / 4 : stride, c,
                 vec ? addend_count / 4 : addend_count, addend_scale, T, vec ? 1 : 0, q->blocks};
    q->blocks += (int)ceil_div(c, 256 / T);
    return RS_OK;
  }
  if (count % 4 == 0 && stride % 4 == 0 && addend_count % 4 == 0 && aligned16(slab) && aligned16(out) &&
      (!addend || aligned16(addend))) {
    const dim3 grid4((unsigned)ceil_div(count / 4, 256 / T));
#define RS_SLAB4(T_)                                                                                        \
  case T_:                                                                                                  \
    hipLaunchKernelGGL(slab_reduce4_kernel<T_>, grid4, dim3(256), 0, st, reinterpret_cast<const f32x4*>(slab), \
                       S, stride / 4, count / 4, reinterpret_cast<f32x4*>(out),                             \
                       reinterpret_cast<const f32x4*>(addend), addend_scale, addend_dscale, addend_count / 4); \
    break;
    switch (T) {
      RS_SLAB4(1) RS_SLAB4(2) RS_SLAB4(4) RS_SLAB4(8) RS_SLAB4(16) RS_SLAB4(32) RS_SLAB4(64) RS_SLAB4(128)
      RS_SLAB4(256)
    }
#undef RS_SLAB4
    return check_launch("slab_reduce4");
  }
  const dim3 grid((unsigned)ceil_div(count, 256 / T));
#define RS_SLAB(T_)                                                                                 \
  case T_:                                                                                          \
    hipLaunchKernelGGL(slab_reduce_kernel<T_>, grid, dim3(256), 0, st, slab, S, stride, count, out, \
                       addend, addend_scale, addend_dscale, addend_count);                          \
    break;
  switch (T) {
    RS_SLAB(1) RS_SLAB(2) RS_SLAB(4) RS_SLAB(8) RS_SLAB(16) RS_SLAB(32) RS_SLAB(64) RS_SLAB(128)
    RS_SLAB(256)
  }
#undef RS_SLAB
  return check_launch("slab_reduce");
}

int launch_slab_reduce(const float* slab, int64_t S, int64_t count, float* out,
                       const float* addend, float addend_scale, hipStream_t st) {
  return launch_slab_reduce_strided(slab, S, count, count, out, addend, addend_scale, st);
}

}  // namespace rs

extern "C" {

size_t rs_reduction_queue_bytes(void) { return sizeof(rs::SlabQueue); }

static rs::SlabQueue* queue_of(void* queue, const char* fn) {
  auto* q = static_cast<rs::SlabQueue*>(queue);
  if (!q || reinterpret_cast<uintptr_t>(q) % alignof(rs::SlabQueue) != 0 || q->magic != rs::kQueueMagic) {
    rs::set_error("%s: not an initialised reduction queue", fn);
    return nullptr;
  }
  return q;
}

int rs_reduction_queue_init(void* queue, size_t bytes) {
  RS_REQUIRE(queue && bytes >= sizeof(rs::SlabQueue) && reinterpret_cast<uintptr_t>(queue) % alignof(rs::SlabQueue) == 0,
             "rs_reduction_queue_init: need %zu bytes aligned to %zu", sizeof(rs::SlabQueue), alignof(rs::SlabQueue));
  auto* q = static_cast<rs::SlabQueue*>(queue);
  q->magic = rs::kQueueMagic;
  q->stream = nullptr;
  q->blocks = 0;
  q->jobs.n = 0;
  return RS_OK;
}

int rs_reduction_queue_pending(const void* queue) {
  auto* q = queue_of(const_cast<void*>(queue), "rs_reduction_queue_pending");
  return q ? q->jobs.n : RS_ERR_INVALID_ARG;
}

int rs_reduction_queue_flush(void* queue, rs_stream_t stream) {
  auto* q = queue_of(queue, "rs_reduction_queue_flush");
  if (!q) return RS_ERR_INVALID_ARG;
  if (q->jobs.n > 0 && rs::as_stream(stream) != q->stream) {
    rs::set_error("rs_reduction_queue_flush: the queued reductions belong to another stream");
    return RS_ERR_INVALID_ARG;
  }
  return rs::flush_queue(q);
}

}  // extern "C"

namespace rs {

// ---- sum of squares (two-stage, fp64 partials) ------------------------------------------
__global__ __launch_bounds__(256) void sumsq_partial_kernel(const float* __restrict__ x,
                                                            int64_t n, double* __restrict__ part) {
  __shared__ double red[256];
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float v = x[i];
    acc += (double)v * (double)v;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// Single workgroup: ordered tree over the partials; out_f = scale*sum (fp32), out_d fp64.
__global__ __launch_bounds__(256) void final_sum_kernel(const double* __restrict__ part, int64_t np,
                                                        double scale, float* __restrict__ out_f,
                                                        double* __restrict__ out_d) {
  __shared__ double red[256];
  // eight independent accumulators per thread (eight loads in flight, not one dependent chain:
  // at B = 65536 the 16,384 partials took ~20 us one at a time), combined in a fixed order
  double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int64_t i0 = threadIdx.x; i0 < np; i0 += 256 * 8) {
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = i0 + 256 * j < np ? part[i0 + 256 * j] : 0.0;
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += v[j];
  }
  red[threadIdx.x] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (out_f) out_f[0] = (float)(scale * red[0]);
    if (out_d) out_d[0] = scale * red[0];
  }
}

int launch_final_sum(const double* part, int64_t np, double scale, float* out_f, double* out_d,
                     hipStream_t st) {
  hipLaunchKernelGGL(final_sum_kernel, dim3(1), dim3(256), 0, st, part, np, scale, out_f, out_d);
  return check_launch("final_sum");
}

// sum of squares of up to 8 tensors in one partial pass: the blocks walk the concatenation
struct SumsqJobs {
  const float* x[8];
  int64_t start[9];  // prefix sums of the element counts
  int n;
};
__global__ __launch_bounds__(256) void sumsq_multi_partial_kernel(SumsqJobs jobs, double* __restrict__ part) {
  __shared__ double red[256];
  double acc = 0.0;
  const int64_t total = jobs.start[jobs.n];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    int t = 0;
#pragma unroll
    for (int k = 1; k < 8; ++k)
      if (k < jobs.n && i >= jobs.start[k]) t = k;
    const float v = jobs.x[t][i - jobs.start[t]];
    acc += (double)v * (double)v;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

int64_t sumsq_blocks(int64_t n) {
  int64_t b = ceil_div(n, 256 * 8);
  if (b < 1) b = 1;
  if (b > 1024) b = 1024;
  return b;
}

// rows x cols with a row stride; same partial/final structure as the contiguous form
__global__ __launch_bounds__(256) void sumsq2d_partial_kernel(const float* __restrict__ x, int64_t rows,
                                                              int64_t cols, int64_t ld,
                                                              double* __restrict__ part) {
  __shared__ double red[256];
  double acc = 0.0;
  const int64_t n = rows * cols;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / cols, c = i - r * cols;
    const float v = x[r * ld + c];
    acc += (double)v * (double)v;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

int launch_sumsq_2d(const float* x, int64_t rows, int64_t cols, int64_t ld, double* part, double scale,
                    float* out_f, hipStream_t st) {
  if (ld == cols) return launch_sumsq(x, rows * cols, part, scale, out_f, st);
  int64_t nb = sumsq_blocks(rows * cols);
  hipLaunchKernelGGL(sumsq2d_partial_kernel, dim3((unsigned)nb), dim3(256), 0, st, x, rows, cols, ld, part);
  int rc = check_launch("sumsq2d_partial");
  if (rc) return rc;
  return launch_final_sum(part, nb, scale, out_f, nullptr, st);
}

// part must hold sumsq_blocks(n) doubles; out_f[0] = scale * sum(x^2).
int launch_sumsq(const float* x, int64_t n, double* part, double scale, float* out_f,
                 hipStream_t st) {
  int64_t nb = sumsq_blocks(n);
  hipLaunchKernelGGL(sumsq_partial_kernel, dim3((unsigned)nb), dim3(256), 0, st, x, n, part);
  int rc = check_launch("sumsq_partial");
  if (rc) return rc;
  return launch_final_sum(part, nb, scale, out_f, nullptr, st);
}

// ---- relu backward + ordered column sums ---------------------------------------------------
// rows per workgroup of the float4 pass (256 columns per workgroup)
static int64_t colsum4_rows_per_block(int64_t M, int64_t N) {
  const int64_t cb = ceil_div(N, 256);
  int64_t nrb = ceil_div(1024, cb);
  if (nrb > ceil_div(M > 0 ? M : 1, 16)) nrb = ceil_div(M > 0 ? M : 1, 16);
  if (nrb < 1) nrb = 1;
  return ceil_div(M > 0 ? M : 1, nrb);
}
// rows per workgroup in the column-sum pass: enough workgroups to fill the chip at small M
static int64_t colsum_rows_per_block(int64_t M, int64_t N) {
  const int64_t cb = ceil_div(N, 64);
  int64_t nrb = ceil_div(1024, cb);
  if (nrb > ceil_div(M > 0 ? M : 1, 16)) nrb = ceil_div(M > 0 ? M : 1, 16);
  if (nrb < 1) nrb = 1;
  return ceil_div(M > 0 ? M : 1, nrb);
}

__global__ __launch_bounds__(256) void relu_bwd_colsum_kernel(
    const float* __restrict__ dy, const float* __restrict__ y, int64_t M, int64_t N,
    int64_t kColRows, float* __restrict__ g, float* __restrict__ part) {
  __shared__ float red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + tx;
  const int64_t r0 = (int64_t)blockIdx.y * kColRows;
  float acc = 0.f;
  if (col < N) {
    const int64_t rend = (r0 + kColRows < M) ? r0 + kColRows : M;
    for (int64_t r = r0 + ty; r < rend; r += 4) {
      float v = dy[r * N + col];
      if (y && !(y[r * N + col] > 0.f)) v = 0.f;
      if (g) g[r * N + col] = v;
      acc += v;
    }
  }
  red[ty][tx] = acc;
  __syncthreads();
  if (ty == 0 && col < N) {
    part[(int64_t)blockIdx.y * N + col] = ((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx];
  }
}

// float4 form (N % 4 == 0, 16-B aligned rows): each lane owns 4 adjacent columns, so a wave
// moves 1 KB per load instruction and 4 rows' loads per array are in flight per thread; row
// blocks sized for ~1024 workgroups (colsum4_rows_per_block). Within a row block every column
// sums rows r0 + ty + 4 j in order, then the fixed 4-way tree; blocks are reduced in order.
__global__ __launch_bounds__(256) void relu_bwd_colsum4_kernel(
    const f32x4* __restrict__ dy, const f32x4* __restrict__ y, int64_t M, int64_t N4,
    int64_t kColRows, f32x4* __restrict__ g, float* __restrict__ part) {
  __shared__ f32x4 red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t c4 = (int64_t)blockIdx.x * 64 + tx;
  const int64_t r0 = (int64_t)blockIdx.y * kColRows;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  auto step = [&](f32x4 v, f32x4 m, int64_t o) __attribute__((always_inline)) {
    if (y) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (!(m[e] > 0.f)) v[e] = 0.f;
    }
    if (g) g[o] = v;
    acc += v;
  };
  if (c4 < N4) {
    const int64_t rend = (r0 + kColRows < M) ? r0 + kColRows : M;
    int64_t r = r0 + ty;
    for (; r + 12 < rend; r += 16) {
      f32x4 v[4], m[4] = {};
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = dy[(r + 4 * j) * N4 + c4];
      if (y) {
#pragma unroll
        for (int j = 0; j < 4; ++j) m[j] = y[(r + 4 * j) * N4 + c4];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) step(v[j], m[j], (r + 4 * j) * N4 + c4);
    }
    for (; r < rend; r += 4) step(dy[r * N4 + c4], y ? y[r * N4 + c4] : f32x4{}, r * N4 + c4);
  }
  red[ty][tx] = acc;
  __syncthreads();
  if (ty == 0 && c4 < N4) {
    const f32x4 s = ((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx];
    *reinterpret_cast<f32x4*>(part + (int64_t)blockIdx.y * N4 * 4 + 4 * c4) = s;
  }
}

}  // namespace rs

using namespace rs;

extern "C" {

int rs_abi_version(void) { return 2; }
const char* rs_last_error(void) { return rs::g_err; }

size_t rs_sum_squares_workspace_bytes(int64_t n) {
  return align_up((size_t)sumsq_blocks(n) * sizeof(double), 256) + 256;
}

size_t rs_sum_squares_multi_workspace_bytes(int ntensors, const int64_t* n) {
  int64_t tot = 0;
  for (int k = 0; k < ntensors; ++k) tot += n[k];
  return rs_sum_squares_workspace_bytes(tot);
}

int rs_sum_squares_multi_f32(int ntensors, const float* const* x, const int64_t* n, float scale, float* out,
                             void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(ntensors >= 1 && ntensors <= 8 && x && n && out, "rs_sum_squares_multi_f32: 1..8 tensors");
  SumsqJobs jobs{};
  jobs.n = ntensors;
  jobs.start[0] = 0;
  for (int k = 0; k < ntensors; ++k) {
    RS_REQUIRE(n[k] >= 0 && (n[k] == 0 || x[k]), "rs_sum_squares_multi_f32: bad tensor %d", k);
    jobs.x[k] = x[k];
    jobs.start[k + 1] = jobs.start[k] + n[k];
  }
  if (!workspace || workspace_bytes < rs_sum_squares_multi_workspace_bytes(ntensors, n)) {
    set_error("rs_sum_squares_multi_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  const int64_t nb = sumsq_blocks(jobs.start[ntensors]);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(sumsq_multi_partial_kernel, dim3((unsigned)nb), dim3(256), 0, st, jobs,
                     static_cast<double*>(workspace));
  int rc = check_launch("sumsq_multi_partial");
  if (rc) return rc;
  return launch_final_sum(static_cast<double*>(workspace), nb, (double)scale, out, nullptr, st);
}

int rs_sum_squares_f32(const float* x, int64_t n, float scale, float* out, void* workspace,
                       size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(n >= 0 && out, "rs_sum_squares_f32: bad args");
  RS_REQUIRE(n == 0 || x, "rs_sum_squares_f32: null x");
  if (workspace_bytes < rs_sum_squares_workspace_bytes(n) || !workspace) {
    set_error("rs_sum_squares_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  return launch_sumsq(x, n, static_cast<double*>(workspace), (double)scale, out,
                      as_stream(stream));
}

size_t rs_colsum_workspace_bytes(int64_t M, int64_t N) {
  // partial rows of whichever pass runs (the float4 one needs the operands' alignment, known
  // only at the call): the larger of the two
  int64_t nrb = ceil_div(M > 0 ? M : 1, colsum_rows_per_block(M, N));
  if (N % 4 == 0) {
    const int64_t n4 = ceil_div(M > 0 ? M : 1, colsum4_rows_per_block(M, N));
    if (n4 > nrb) nrb = n4;
  }
  return align_up((size_t)nrb * (size_t)N * sizeof(float), 256) + 256;
}

int rs_relu_bwd_colsum_f32(const float* dy, const float* y, int64_t M, int64_t N, float* g,
                           float* colsum, void* workspace, size_t workspace_bytes,
                           rs_stream_t stream, void* queue) {
  RS_REQUIRE(M >= 0 && N > 0 && dy && colsum, "rs_relu_bwd_colsum_f32: bad args");
  if (!workspace || workspace_bytes < rs_colsum_workspace_bytes(M, N)) {
    set_error("rs_relu_bwd_colsum_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  float* part = static_cast<float*>(workspace);
  // the float4 pass also stores f32x4 partials into the caller's workspace: it must be 16-B
  // aligned too. (The two passes split rows into different blocks, so the sums' bits depend on
  // which one runs — documented at the declaration.)
  const bool v4 = N % 4 == 0 && aligned16(dy) && (!y || aligned16(y)) && (!g || aligned16(g)) &&
                  aligned16(workspace);
  const int64_t rpb = v4 ? colsum4_rows_per_block(M, N) : colsum_rows_per_block(M, N);
  int64_t nrb = ceil_div(M > 0 ? M : 1, rpb);
  if (M == 0) {
    RS_HIP(hipMemsetAsync(colsum, 0, N * sizeof(float), st));
    return RS_OK;
  }
  if (v4) {
    dim3 grid((unsigned)ceil_div(N / 4, 64), (unsigned)nrb);
    hipLaunchKernelGGL(relu_bwd_colsum4_kernel, grid, dim3(256), 0, st, reinterpret_cast<const f32x4*>(dy),
                       reinterpret_cast<const f32x4*>(y), M, N / 4, rpb, reinterpret_cast<f32x4*>(g), part);
  } else {
    dim3 grid((unsigned)ceil_div(N, 64), (unsigned)nrb);
    hipLaunchKernelGGL(relu_bwd_colsum_kernel, grid, dim3(256), 0, st, dy, y, M, N, rpb, g, part);
  }
  int rc = check_launch("relu_bwd_colsum");
  if (rc) return rc;
  return launch_slab_reduce_strided(part, nrb, N, N, colsum, nullptr, 0.f, st, nullptr, -1,
                                    static_cast<SlabQueue*>(queue));
}

__global__ void iteration_increment_kernel(int64_t* it) { it[0] += 1; }

int rs_iteration_increment(int64_t* iteration, rs_stream_t stream) {
  RS_REQUIRE(iteration, "rs_iteration_increment: null");
  hipLaunchKernelGGL(iteration_increment_kernel, dim3(1), dim3(1), 0, as_stream(stream), iteration);
  return check_launch("iteration_increment");
}

}  // extern "C"
