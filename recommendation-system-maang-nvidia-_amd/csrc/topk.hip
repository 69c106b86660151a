// topk.hip — exact brute-force inner-product top-K over an item table (row-sharded capable).
//
// Reference: ProductionTrainer._evaluate (src/trainer.py:204-212: sims = np.dot(user_embs,
// item_embs.T); np.argpartition(-sim, k)[:k]) and the FAISS IndexFlatIP search of
// _build_faiss / RecommendationService (src/trainer.py:240-243,
// app/recommendation_service.py:71-72). Output order is the build contract of SURVEY A.8:
// (-score, index) ascending, so the result is a deterministic function of the scores.
//
// Stage 1 (scan): one wave owns 32 queries (lane = query) and a contiguous slice of items;
// 32-item tiles are staged through LDS with coalesced 1-KB loads and scored with
// v_mfma_f32_32x32x2_f32 (exact fp32: on dyadic-grid data every score is exact, so indices
// are bit-exact vs the CPU oracle); each lane keeps its query's running top-k list in LDS and
// only inserts items that beat the list's current k-th entry (after warm-up a rare event).
// Stage 2 (merge): groups of sorted lists are bitonic-sorted in LDS by (-score, index) until
// one list per query remains. The caller adds `index_base` (the shard's first global row)
// so per-GPU shards merge by plain concatenation + one more stage-2 pass.
#include "common.hpp"

#include <cmath>

namespace rs {

constexpr int TK_KMAX = 128;
constexpr int TK_MERGE = 4096;  // entries sorted per merge workgroup

__device__ __forceinline__ bool tk_better(float s, int64_t i, float ts, int64_t ti) {
  return s > ts || (s == ts && i < ti);
}

template <int D>
__global__ __launch_bounds__(64) void topk_scan_kernel(const float* __restrict__ Q, int64_t nq,
                                                       const float* __restrict__ items, int64_t N,
                                                       int k, int64_t per_split,
                                                       float* __restrict__ cand_s,
                                                       int32_t* __restrict__ cand_i,
                                                       int64_t nsplit) {
  constexpr int KPAD = D + 4;
  __shared__ __attribute__((aligned(16))) float tile[32 * KPAD];
  __shared__ float ls[32][TK_KMAX];
  __shared__ int32_t li[32][TK_KMAX];
  const int lane = threadIdx.x, half = lane >> 5, l32 = lane & 31;
  const int64_t q = (int64_t)blockIdx.x * 32 + l32;
  const int64_t split = blockIdx.y;
  const int64_t i0 = split * per_split;
  const int64_t i1 = (i0 + per_split < N) ? i0 + per_split : N;

  float qf[D / 2];
#pragma unroll
  for (int g = 0; g < D / 8; ++g) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (q < nq) v = *reinterpret_cast<const f32x4*>(Q + q * D + 8 * g + 4 * half);
#pragma unroll
    for (int t = 0; t < 4; ++t) qf[4 * g + t] = v[t];
  }
  for (int j = half; j < k; j += 2) {
    ls[l32][j] = -INFINITY;
    li[l32][j] = 0x7fffffff;
  }
  __syncthreads();

  for (int64_t base = i0; base < i1; base += 32) {
    // stage 32 item rows (coalesced 16-B pieces)
    for (int f = lane; f < 32 * D / 4; f += 64) {
      const int row = f / (D / 4), c4 = f % (D / 4);
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (base + row < i1) v = *reinterpret_cast<const f32x4*>(items + (base + row) * D + 4 * c4);
      *reinterpret_cast<f32x4*>(tile + row * KPAD + 4 * c4) = v;
    }
    __syncthreads();
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const float* trow = tile + l32 * KPAD + 4 * half;
#pragma unroll
    for (int g = 0; g < D / 8; ++g) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(trow + 8 * g);
#pragma unroll
      for (int t = 0; t < 4; ++t) acc = mfma32x32x2(a[t], qf[4 * g + t], acc);
    }
    // acc[r] = score(q, base + acc_row(r, half)); the two halves insert in turn
    for (int h = 0; h < 2; ++h) {
      if (half == h && q < nq) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t item = base + acc_row(r, h);
          const float s = acc[r];
          if (item < i1 && tk_better(s, item, ls[l32][k - 1], li[l32][k - 1])) {
            int pos = k - 1;
            while (pos > 0 && tk_better(s, item, ls[l32][pos - 1], li[l32][pos - 1])) {
              ls[l32][pos] = ls[l32][pos - 1];
              li[l32][pos] = li[l32][pos - 1];
              --pos;
            }
            ls[l32][pos] = s;
            li[l32][pos] = (int32_t)item;
          }
        }
      }
      __syncthreads();
    }
  }
  if (q < nq) {
    for (int j = half; j < k; j += 2) {
      cand_s[(q * nsplit + split) * k + j] = ls[l32][j];
      cand_i[(q * nsplit + split) * k + j] = li[l32][j];
    }
  }
}

// Merge `group` sorted lists of k entries per query into one (bitonic sort of <= 4096 entries).
template <typename IdxT>
__device__ __forceinline__ IdxT tk_sentinel() { return (IdxT)(sizeof(IdxT) == 4 ? 0x7fffffffLL : 0x7fffffffffffffffLL); }

template <typename IdxT>
__global__ __launch_bounds__(256) void topk_merge_kernel(const float* __restrict__ in_s,
                                                         const IdxT* __restrict__ in_i,
                                                         int64_t nlists, int k, int group,
                                                         int64_t nout, float* __restrict__ out_s,
                                                         IdxT* __restrict__ out_i,
                                                         float* __restrict__ fin_s,
                                                         int64_t* __restrict__ fin_i,
                                                         int64_t index_base) {
  __shared__ float ss[TK_MERGE];
  __shared__ IdxT si[TK_MERGE];
  const int64_t q = blockIdx.y, o = blockIdx.x;
  const int64_t l0 = o * group;
  int64_t l1 = l0 + group;
  if (l1 > nlists) l1 = nlists;
  const int m = (int)((l1 - l0) * k);
  int P = 1;
  while (P < m) P <<= 1;
  const IdxT SENT = tk_sentinel<IdxT>();
  for (int e = threadIdx.x; e < P; e += 256) {
    if (e < m) {
      ss[e] = in_s[(q * nlists + l0) * k + e];
      si[e] = in_i[(q * nlists + l0) * k + e];
    } else {
      ss[e] = -INFINITY;
      si[e] = SENT;
    }
  }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int e = threadIdx.x; e < P; e += 256) {
        const int partner = e ^ stride;
        if (partner > e) {
          const bool desc = (e & size) == 0;  // blocks alternate direction; final pass: best first
          const bool pb = tk_better(ss[partner], (int64_t)si[partner], ss[e], (int64_t)si[e]);
          if (pb == desc) {
            const float ts = ss[e];
            const IdxT ti = si[e];
            ss[e] = ss[partner];
            si[e] = si[partner];
            ss[partner] = ts;
            si[partner] = ti;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int j = threadIdx.x; j < k; j += 256) {
    if (fin_s) {
      fin_s[q * k + j] = ss[j];
      fin_i[q * k + j] = si[j] == SENT ? (int64_t)-1 : (int64_t)si[j] + index_base;
    } else {
      out_s[(q * nout + o) * k + j] = ss[j];
      out_i[(q * nout + o) * k + j] = si[j];
    }
  }
}

template <typename IdxT>
static int merge_rounds(float* s0, IdxT* i0, float* s1, IdxT* i1, int64_t nq, int64_t nl, int k,
                        int64_t index_base, float* out_s, int64_t* out_i, hipStream_t st) {
  const int group = TK_MERGE / k;
  while (true) {
    const int64_t nout = ceil_div(nl, group);
    const bool last = nout == 1;
    hipLaunchKernelGGL((topk_merge_kernel<IdxT>), dim3((unsigned)nout, (unsigned)nq), dim3(256), 0, st, s0,
                       i0, nl, k, group, nout, s1, i1, last ? out_s : nullptr,
                       last ? out_i : nullptr, index_base);
    int rc = check_launch("topk_merge");
    if (rc || last) return rc;
    float* ts = s0; s0 = s1; s1 = ts;
    IdxT* ti = i0; i0 = i1; i1 = ti;
    nl = nout;
  }
}

static int64_t topk_nsplit(int64_t nq, int64_t N) {
  const int64_t qb = ceil_div(nq, 32);
  int64_t s = ceil_div(1024, qb);           // ~4 single-wave workgroups per CU
  const int64_t maxs = ceil_div(N, 256);    // >= 256 items per slice
  if (s > maxs) s = maxs;
  if (s < 1) s = 1;
  return s;
}

template <int D>
static int topk_impl(const float* Q, int64_t nq, const float* items, int64_t N, int k,
                     int64_t index_base, float* out_s, int64_t* out_i, void* ws, size_t wsb,
                     hipStream_t st) {
  const int64_t ns = topk_nsplit(nq, N);
  const int64_t per = ceil_div(ceil_div(N, ns), 32) * 32;
  const int64_t nse = ceil_div(N, per);
  Carve c(ws, wsb);
  float* s0 = c.take<float>(nq * nse * k);
  int32_t* i0 = c.take<int32_t>(nq * nse * k);
  float* s1 = c.take<float>(nq * nse * k);
  int32_t* i1 = c.take<int32_t>(nq * nse * k);
  hipLaunchKernelGGL((topk_scan_kernel<D>), dim3((unsigned)ceil_div(nq, 32), (unsigned)nse), dim3(64), 0, st, Q,
                     nq, items, N, k, per, s0, i0, nse);
  int rc = check_launch("topk_scan");
  if (rc) return rc;
  return merge_rounds<int32_t>(s0, i0, s1, i1, nq, nse, k, index_base, out_s, out_i, st);
}

}  // namespace rs

using namespace rs;

extern "C" {

size_t rs_topk_ip_workspace_bytes(int64_t nq, int64_t N, int64_t D, int k) {
  (void)D;
  const int64_t ns = topk_nsplit(nq > 0 ? nq : 1, N > 0 ? N : 1);
  const int64_t per = ceil_div(ceil_div(N > 0 ? N : 1, ns), 32) * 32;
  const int64_t nse = ceil_div(N > 0 ? N : 1, per);
  const size_t e = (size_t)(nq > 0 ? nq : 1) * nse * (k > 0 ? k : 1);
  return 2 * (align_up(e * 4, 256) + align_up(e * 4, 256)) + 1024;
}

int rs_topk_ip_f32(const float* queries, int64_t nq, const float* items, int64_t N, int64_t D,
                   int k, int64_t index_base, float* out_scores, int64_t* out_index,
                   void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(nq >= 0 && N > 0 && k > 0, "rs_topk_ip_f32: bad sizes");
  RS_REQUIRE(k <= TK_KMAX, "rs_topk_ip_f32: k must be <= %d", TK_KMAX);
  RS_REQUIRE(k <= N, "rs_topk_ip_f32: k must be <= N");
  RS_REQUIRE(N < ((int64_t)1 << 31) - 1, "rs_topk_ip_f32: N must be < 2^31 per call (shard it)");
  RS_REQUIRE(queries && items && out_scores && out_index, "rs_topk_ip_f32: null");
  RS_REQUIRE(aligned16(queries) && aligned16(items), "rs_topk_ip_f32: 16-byte alignment");
  if (nq == 0) return RS_OK;
  if (!workspace || workspace_bytes < rs_topk_ip_workspace_bytes(nq, N, D, k)) {
    set_error("rs_topk_ip_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  switch (D) {
    case 32: return topk_impl<32>(queries, nq, items, N, k, index_base, out_scores, out_index, workspace, workspace_bytes, st);
    case 64: return topk_impl<64>(queries, nq, items, N, k, index_base, out_scores, out_index, workspace, workspace_bytes, st);
    case 128: return topk_impl<128>(queries, nq, items, N, k, index_base, out_scores, out_index, workspace, workspace_bytes, st);
    default:
      set_error("rs_topk_ip_f32: D=%lld not compiled (32, 64, 128)", (long long)D);
      return RS_ERR_UNSUPPORTED;
  }
}

size_t rs_topk_merge_workspace_bytes(int64_t nq, int64_t nlists, int k) {
  const size_t e = (size_t)(nq > 0 ? nq : 1) * (nlists > 0 ? nlists : 1) * (k > 0 ? k : 1);
  return 2 * (align_up(e * 4, 256) + align_up(e * 8, 256)) + 1024;
}

int rs_topk_merge_f32(const float* in_scores, const int64_t* in_index, int64_t nq, int64_t nlists,
                      int k, float* out_scores, int64_t* out_index, void* workspace,
                      size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(nq >= 0 && nlists > 0 && k > 0 && k <= TK_KMAX, "rs_topk_merge_f32: bad sizes");
  RS_REQUIRE(in_scores && in_index && out_scores && out_index, "rs_topk_merge_f32: null");
  if (nq == 0) return RS_OK;
  if (!workspace || workspace_bytes < rs_topk_merge_workspace_bytes(nq, nlists, k)) {
    set_error("rs_topk_merge_f32: workspace too small");
    return RS_ERR_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  const size_t e = (size_t)nq * nlists * k;
  Carve c(workspace, workspace_bytes);
  float* s0 = c.take<float>(e);
  int64_t* i0 = c.take<int64_t>(e);
  float* s1 = c.take<float>(e);
  int64_t* i1 = c.take<int64_t>(e);
  RS_HIP(hipMemcpyAsync(s0, in_scores, e * sizeof(float), hipMemcpyDeviceToDevice, st));
  RS_HIP(hipMemcpyAsync(i0, in_index, e * sizeof(int64_t), hipMemcpyDeviceToDevice, st));
  return merge_rounds<int64_t>(s0, i0, s1, i1, nq, nlists, k, 0, out_scores, out_index, st);
}

}  // extern "C"
