// metrics.hip — ranking-metric suite over top-K lists and the L2 row normalisation of the
// cosine index.
//
// rs_rank_metrics_i64 replaces AdvancedMetrics (src/evaluation.py:22-104) on integer item rows:
// recall@k, precision@k, NDCG@k, MAP@k for up to 8 cut-offs, MRR over the whole list, catalogue
// coverage and per-list diversity, with the reference's exact definitions (first occurrence of
// the true item; precision = 1/len(top_k) on a hit; NDCG's ideal DCG = 1; MAP@k = 1/rank on a
// hit; diversity = |set(list)| / len(list), 0 for lists of length <= 1). One wave per list: the
// list is staged in LDS, the true item is found with a ballot per 64 entries, duplicates are
// counted against the earlier entries, and coverage sets one bit per item in a bitmap. Means
// are ordered (fixed-tree) sums of the per-list values: bit-identical across runs.
//
// rs_l2_normalize_rows_f32 is faiss.normalize_L2 (src/trainer.py:241,
// app/recommendation_service.py:70): x *= 1/sqrt(sum x^2) when the sum is > 0. One wave per row.
#include "common.hpp"

#include <cmath>

namespace rs {

constexpr int RM_MAXK = 8;     // cut-offs per call
constexpr int RM_MAXLEN = 1024;  // list length

struct RmCuts {
  int k[RM_MAXK];
};

__global__ __launch_bounds__(256) void rank_metrics_row_kernel(const int64_t* __restrict__ pred, int64_t U, int Kmax,
                                                               const int32_t* __restrict__ lens,
                                                               const int64_t* __restrict__ truth, RmCuts cuts,
                                                               int nks, int64_t n_items,
                                                               double* __restrict__ per_row,
                                                               uint32_t* __restrict__ cover) {
  __shared__ int64_t row_s[4][RM_MAXLEN];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t u = (int64_t)blockIdx.x * 4 + w;
  if (u >= U) return;
  const int64_t* p = pred + u * Kmax;
  int K = lens ? lens[u] : Kmax;
  if (K > Kmax) K = Kmax;
  if (K < 0) K = 0;
  const int64_t t = truth[u];
  int pos = -1;
  for (int c = 0; c < K; c += 64) {
    const int j = c + lane;
    const int64_t v = j < K ? p[j] : (int64_t)-1;
    if (j < K) {
      row_s[w][j] = v;
      if (v >= 0 && v < n_items) atomicOr(&cover[v >> 5], 1u << (v & 31));
    }
    const uint64_t m = __ballot(j < K && v == t);
    if (pos < 0 && m) pos = c + __ffsll((unsigned long long)m) - 1;
  }
  __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own LDS writes, in order
  // distinct entries: an entry counts if no earlier entry equals it
  int uniq = 0;
  for (int c = 0; c < K; c += 64) {
    const int j = c + lane;
    int first = 0;
    if (j < K) {
      const int64_t v = row_s[w][j];
      first = 1;
      for (int i = 0; i < j; ++i)
        if (row_s[w][i] == v) {
          first = 0;
          break;
        }
    }
    uniq += __popcll(__ballot(first));
  }
  if (lane == 0) {
    const int nm = 4 * nks + 2;
    double* o = per_row + u * nm;
    for (int i = 0; i < nks; ++i) {
      const int k = cuts.k[i];
      const bool hit = pos >= 0 && pos < k;
      const int len = k < K ? k : K;  // len(pred[:k])
      o[4 * i + 0] = hit ? 1.0 : 0.0;
      o[4 * i + 1] = hit ? 1.0 / (double)len : 0.0;
      o[4 * i + 2] = hit ? 1.0 / log2((double)pos + 2.0) : 0.0;
      o[4 * i + 3] = hit ? 1.0 / (double)(pos + 1) : 0.0;
    }
    o[4 * nks] = pos >= 0 ? 1.0 / (double)(pos + 1) : 0.0;
    o[4 * nks + 1] = K > 1 ? (double)uniq / (double)K : 0.0;
  }
}

// out[m] = (sum over rows of per_row[:, m]) / U, ordered: thread t sums rows t, t+256, ...; then
// a fixed tree. Block nm+1 counts the coverage bits.
__global__ __launch_bounds__(256) void rank_metrics_reduce_kernel(const double* __restrict__ per_row, int64_t U,
                                                                  int nm, const uint32_t* __restrict__ cover,
                                                                  int64_t nwords, int64_t n_items,
                                                                  double* __restrict__ out) {
  __shared__ double red[256];
  const int m = blockIdx.x;
  double acc = 0.0;
  if (m < nm) {
    for (int64_t r = threadIdx.x; r < U; r += 256) acc += per_row[r * nm + m];
  } else {
    for (int64_t i = threadIdx.x; i < nwords; i += 256) acc += (double)__popc(cover[i]);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (m < nm) out[m] = U > 0 ? red[0] / (double)U : 0.0;
    else out[m] = n_items > 0 ? red[0] / (double)n_items : 0.0;
  }
}

__global__ __launch_bounds__(256) void l2_normalize_rows_kernel(const float* __restrict__ x, int64_t n, int64_t D,
                                                                float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const float* xr = x + r * D;
  float ss = 0.f;
  for (int64_t j = lane; j < D; j += 64) ss += xr[j] * xr[j];
  ss = wave_sum(ss);
  const float inv = ss > 0.f ? 1.f / sqrtf(ss) : 1.f;
  float* orow = out + r * D;
  for (int64_t j = lane; j < D; j += 64) orow[j] = ss > 0.f ? xr[j] * inv : xr[j];
}

}  // namespace rs

using namespace rs;

extern "C" {

size_t rs_rank_metrics_workspace_bytes(int64_t U, int nks, int64_t n_items) {
  const int64_t nm = 4 * (int64_t)(nks > 0 ? nks : 0) + 2;
  return align_up((size_t)(U > 0 ? U : 1) * nm * sizeof(double), 256) +
         align_up((size_t)((n_items > 0 ? n_items : 1) + 31) / 32 * sizeof(uint32_t), 256) + 256;
}

int rs_rank_metrics_i64(const int64_t* pred, int64_t U, int K, const int32_t* lens, const int64_t* truth,
                        const int32_t* ks, int nks,
                        int64_t n_items, double* out, void* workspace, size_t workspace_bytes,
                        rs_stream_t stream) {
  RS_REQUIRE(U >= 0 && K >= 1 && K <= RM_MAXLEN && n_items >= 0, "rs_rank_metrics_i64: bad sizes");
  RS_REQUIRE(nks >= 0 && nks <= RM_MAXK, "rs_rank_metrics_i64: at most %d cut-offs", RM_MAXK);
  RS_REQUIRE(out && (U == 0 || (pred && truth)) && (nks == 0 || ks), "rs_rank_metrics_i64: null");
  RmCuts cuts = {};
  for (int i = 0; i < nks; ++i) {
    RS_REQUIRE(ks[i] >= 1, "rs_rank_metrics_i64: cut-offs must be >= 1");
    cuts.k[i] = ks[i];
  }
  if (!workspace || workspace_bytes < rs_rank_metrics_workspace_bytes(U, nks, n_items)) {
    set_error("rs_rank_metrics_i64: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  const int nm = 4 * nks + 2;
  Carve c(workspace, workspace_bytes);
  double* per_row = c.take<double>((size_t)(U > 0 ? U : 1) * nm);
  const int64_t nwords = ((n_items > 0 ? n_items : 1) + 31) / 32;
  uint32_t* cover = c.take<uint32_t>(nwords);
  RS_HIP(hipMemsetAsync(cover, 0, nwords * sizeof(uint32_t), st));
  if (U > 0) {
    hipLaunchKernelGGL(rank_metrics_row_kernel, dim3((unsigned)ceil_div(U, 4)), dim3(256), 0, st, pred, U, K, lens,
                       truth,
                       cuts, nks, n_items, per_row, cover);
    int rc = check_launch("rank_metrics_row");
    if (rc) return rc;
  }
  hipLaunchKernelGGL(rank_metrics_reduce_kernel, dim3((unsigned)(nm + 1)), dim3(256), 0, st, per_row, U, nm, cover,
                     nwords, n_items, out);
  return check_launch("rank_metrics_reduce");
}

int rs_l2_normalize_rows_f32(const float* x, int64_t n, int64_t D, float* out, rs_stream_t stream) {
  RS_REQUIRE(n >= 0 && D > 0, "rs_l2_normalize_rows_f32: bad sizes");
  RS_REQUIRE(n == 0 || (x && out), "rs_l2_normalize_rows_f32: null");
  if (n == 0) return RS_OK;
  hipLaunchKernelGGL(l2_normalize_rows_kernel, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, as_stream(stream), x,
                     n, D, out);
  return check_launch("l2_normalize_rows");
}

}  // extern "C"
