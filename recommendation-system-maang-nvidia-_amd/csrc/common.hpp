// common.hpp — shared helpers for the gfx950 kernels of librecsys_hip.so.
// Wave64 reductions, MFMA wrappers, status/error plumbing for the C-ABI.
#pragma once
#include <cstring>
#include <cstdint>
#include <cstdio>
#include <cstdarg>
#include <hip/hip_runtime.h>
#include "../../include/recsys_hip.h"

namespace rs {

// A/B and timing switches read from the environment exist only in experiment builds
// (make EXPERIMENTS=1, i.e. -DRS_EXPERIMENTS): a release library ignores every RS_* variable, so
// its kernel selection depends on the call's arguments alone (tests/test_abi.py checks that no
// switch name is left in the release binary).
#ifdef RS_EXPERIMENTS
}  // namespace rs
#include <cstdlib>
namespace rs {
inline const char* exp_env(const char* name) { return getenv(name); }
#else
inline const char* exp_env(const char*) { return nullptr; }
#endif

// ----- status plumbing (host) ---------------------------------------------------------
void set_error(const char* fmt, ...);
int check_launch(const char* what);

#define RS_REQUIRE(cond, ...)                 \
  do {                                        \
    if (!(cond)) {                            \
      ::rs::set_error(__VA_ARGS__);           \
      return RS_ERR_INVALID_ARG;              \
    }                                         \
  } while (0)

#define RS_HIP(call)                                                          \
  do {                                                                        \
    hipError_t e_ = (call);                                                   \
    if (e_ != hipSuccess) {                                                   \
      ::rs::set_error("%s failed: %s", #call, hipGetErrorString(e_));         \
      return RS_ERR_HIP;                                                      \
    }                                                                         \
  } while (0)

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
inline hipStream_t as_stream(rs_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Bump allocator over a caller-provided workspace (256-B aligned carve-outs).
struct Carve {
  char* base;
  size_t size;
  size_t off = 0;
  Carve(void* b, size_t s) : base(static_cast<char*>(b)), size(s) {}
  template <typename T>
  T* take(size_t count) {
    off = align_up(off, 256);
    T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
    off += count * sizeof(T);
    return p;
  }
  bool ok() const { return off <= size; }
};

// ----- shared launchers (reduce.hip) ----------------------------------------------------
int launch_slab_reduce(const float* slab, int64_t S, int64_t count, float* out,
                       const float* addend, float addend_scale, hipStream_t st);
// q (nullable): a caller-owned deferred-reduction queue (rs_reduction_queue_*, reduce.hip). With a
// queue the reduction is appended to it instead of launched (the caller guarantees the slab stays
// allocated and untouched until rs_reduction_queue_flush); without one it launches now.
struct SlabQueue;
int launch_slab_reduce_strided(const float* slab, int64_t S, int64_t stride, int64_t count,
                               float* out, const float* addend, float addend_scale, hipStream_t st,
                               const float* addend_dscale = nullptr, int64_t addend_count = -1,
                               SlabQueue* q = nullptr);
int launch_final_sum(const double* part, int64_t np, double scale, float* out_f, double* out_d,
                     hipStream_t st);
int64_t sumsq_blocks(int64_t n);
int gemm_launch(int ta, int tb, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                const float* B, int64_t ldb, float* C, int64_t ldc, const float* bias, int epi,
                const float* x0, const float* xres, float* aux, int64_t ldx, const float* addend,
                int64_t ldadd, hipStream_t st, int prec = 0, float beta = 0.f);
// plane-image GEMM (gemm.hip): images of fp32 operands (layout 0 = KC: k = cols, 1 = KM: k = rows)
size_t pimg_bytes(int64_t K, int64_t extent);
int plane_image_launch(const float* X, int64_t ldx, int64_t rows, int64_t cols, int layout, char* img,
                       hipStream_t st);
int pgemm_launch(int ta, int tb, int64_t M, int64_t N, int64_t K, const char* Aimg, const char* Bimg, float* C,
                 int64_t ldc, const float* bias, int epi, const float* x0, const float* xres, float* aux, int64_t ldx,
                 const float* addend, int64_t ldadd, hipStream_t st, int prec, float beta);
size_t pgemm_splitk_ws_bytes(int64_t M, int64_t N, int64_t K);
int pgemm_splitk_launch(int ta, int tb, int64_t M, int64_t N, int64_t K, const char* Aimg, const char* Bimg,
                        float* C, const float* addend, float addend_scale, int prec, void* ws, size_t ws_bytes,
                        hipStream_t st);
// plane-pair GEMM (gemm.hip, xgemm): images of X viewed as [rows][k] (trans: X stored [k][rows])
size_t ximg_bytes(int64_t R, int64_t K);
int ximg_launch(const float* X, int64_t ld, int64_t R, int64_t K, int trans, char* img, hipStream_t st);
int ximg_dual_launch(const float* X, const float* x0, const float* u, const float* base, float* gx0, int64_t R,
                     int64_t K, char* img, char* img_t, float* part, hipStream_t st);
int xgemm_launch(int64_t M, int64_t N, int64_t K, const char* Aimg, const char* Bimg, float* C, int64_t ldc,
                 const float* bias, int act, int epi, const float* x0, const float* xres, float* aux, int64_t ldx,
                 const float* addend, int64_t ldadd, hipStream_t st, int prec, float beta);
// xgemm_launch with the last partial round split over K when a workspace of xgemm_tail_ws_bytes
// is given (same results up to the fp32 association of the K halves)
size_t xgemm_tail_ws_bytes(int64_t M, int64_t N, int64_t K);
int xgemm_launch_ws(int64_t M, int64_t N, int64_t K, const char* Aimg, const char* Bimg, float* C, int64_t ldc,
                    const float* bias, int act, int epi, const float* x0, const float* xres, float* aux, int64_t ldx,
                    const float* addend, int64_t ldadd, hipStream_t st, int prec, float beta, void* ws, size_t wsb);
size_t xgemm_splitk_ws_bytes(int64_t M, int64_t N, int64_t K);
int xgemm_splitk_launch(int64_t M, int64_t N, int64_t K, const char* Aimg, const char* Bimg, float* C,
                        const float* addend, float addend_scale, int prec, void* ws, size_t ws_bytes, hipStream_t st);
int launch_sumsq(const float* x, int64_t n, double* part, double scale, float* out_f,
                 hipStream_t st);
int launch_sumsq_2d(const float* x, int64_t rows, int64_t cols, int64_t ld, double* part, double scale,
                    float* out_f, hipStream_t st);

// ----- device helpers -------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// v_mfma_f32_32x32x2_f32: lane l supplies A[l&31][l>>5], B[l>>5][l&31];
// acc reg r of lane l holds D[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31].
__device__ __forceinline__ f32x16 mfma32x32x2(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int acc_row(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

// Last-workgroup tickets without an agent-scope release fence. That fence writes back the XCD's
// L2 (buffer_wbl2) and costs the whole grid ~30 ns per workgroup that issues it (measured: the
// C3 row finalize, 16384 workgroups, 50 -> 538 us). Only the partials the last workgroup reads
// need publishing, so they are written with agent-coherent stores (sc1: performed past the XCD's
// L2), the writer waits for their completion (vmcnt(0), the wait the release sequence ends with)
// before its ticket increment, and the last workgroup reads them with agent-coherent loads.
__device__ __forceinline__ void ticket_publish(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the ticket count before this arrival (call from the thread that published)
__device__ __forceinline__ unsigned int ticket_arrive(unsigned int* done) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ticket_collect(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Completion ticket of a grid whose last workgroup finishes a reduction, two levels deep: the
// arrivals of one address serialise (~9 ns each: +150 us for 16384 workgroups on one counter),
// so workgroups arrive on their group's counter (gs <= 64 per group at up to 65536 workgroups;
// counters 128 B apart) and each group's last arrives on the top counter. The counters live in
// TICKET_BYTES, zeroed before the grid (ticket_zero, by an earlier kernel of the sequence) and
// left zeroed. Returns, in every thread, whether this is the grid's last workgroup.
constexpr int TICKET_MAX_GROUPS = 1024;
constexpr size_t TICKET_WORDS = 32 * (1 + TICKET_MAX_GROUPS);
__device__ __forceinline__ void ticket_zero(unsigned int* done, int tid, int nthreads) {
  for (int k = tid; k <= TICKET_MAX_GROUPS; k += nthreads) done[32 * k] = 0u;
}
__device__ __forceinline__ bool ticket_last(unsigned int* done, int64_t blk, int64_t nb) {
  __shared__ int last;
  if (threadIdx.x == 0) {
    const int64_t gs = nb > 64 * (int64_t)TICKET_MAX_GROUPS ? (nb + TICKET_MAX_GROUPS - 1) / TICKET_MAX_GROUPS : 64;
    const int64_t g = blk / gs, ng = (nb + gs - 1) / gs;
    const int64_t n_in = nb - g * gs < gs ? nb - g * gs : gs;
    unsigned int* cg = done + 32 * (1 + g);
    int l = 0;
    if (ticket_arrive(cg) == (unsigned int)(n_in - 1)) {
      __hip_atomic_store(cg, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      l = ticket_arrive(done) == (unsigned int)(ng - 1);
      if (l) __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    last = l;
  }
  __syncthreads();
  return last != 0;
}

}  // namespace rs
