// gemm.hpp — the GEMM launch parameters shared by gemm.hip and gemm_skinny.hip.
#pragma once
#include "common.hpp"

namespace rs {

constexpr int GEMM_BK = 32;
constexpr int GEMM_GMAX = 4;  // problems per grouped launch
constexpr int GEMM_KPAD = GEMM_BK + 4;

struct GemmParams {
  const float* A;
  const float* B;
  float* C;
  int64_t lda, ldb, ldc;
  int64_t M, N, K;
  const float* bias;
  int act;
  const float* mask;
  int64_t ldm;
  float beta;
  int64_t k_per_split;
  float* slab;  // split mode: [gridDim.z][M][N]
  // DCN-v2 cross epilogue (epi == 1): u = acc + bias -> aux[m, n]; C = x0[m, n] * u + xres[m, n]
  int epi;
  const float* x0;
  const float* xres;
  float* aux;
  int64_t ldx;  // leading dim of x0 / xres / aux
  // addend epilogue (any epi): v += addend[m * ldadd + n]
  const float* addend;
  int64_t ldadd;
  int prec;  // RS_PREC_F32 (f32 MFMA) or RS_PREC_F32_SPLIT6 / 9 (gemm_x3_kernel)
  // trans_a only: 1 + the index of a synthetic all-ones row of op(A) (a multiple of 4, = the real
  // M), 0 = none: row ones_row1 - 1 of C is then the column sums of op(B) (a Dense bias gradient
  // computed by its weight-gradient GEMM)
  int64_t ones_row1;
  // split mode: floats between K slices of the slab (0 = M N)
  int64_t slab_stride;
  // grouped launch (ngroup > 1, gemm_f32 / gemm_x3 kernels): ngroup problems of this one shape in
  // one grid, z = g zper + K slice; problem g reads A, B and writes C / slab from the g-th entries
  // (bias / mask: nullable per problem as for a single launch)
  int ngroup;
  int64_t zper;
  const float* gA[GEMM_GMAX];
  const float* gB[GEMM_GMAX];
  float* gC[GEMM_GMAX];
  const float* gbias[GEMM_GMAX];
  const float* gmask[GEMM_GMAX];
  float* gslab[GEMM_GMAX];
  // tile-range launch (xgemm, tile_n > 0): a 1-D grid over tiles [tile_lo, tile_lo + tile_n) of the
  // gx_map order (x K slices in split mode); 0 = the whole grid
  int64_t tile_lo, tile_n;
  // split-mode weight gradients (gemm_x3_kernel, trans_a, !trans_b; 0 = off): the workgroups of row
  // tile 0 also sum their op(B) chunks' columns into slab row colsum_row of their K slice (the
  // Dense bias gradient, without the extra row tile an all-ones row of op(A) costs)
  int64_t colsum_row;
  // the skinny kernel's weight operand as a fragment image (rs_mlp_weight_image_f32's layout: B
  // fragment (c, t) = 3 planes x 1 KB at (c N / 16 + t) 3 KB), or null: B read and split per chunk
  const char* bimg;
  const char* gbimg[GEMM_GMAX];
  // distinct-row Dense layers (rs_gemm_group_rows_prec_f32 / rs_gemm_wgrad_bias_group_rows_prec_f32;
  // null = off): arow, trans_a split kernels: op(A)'s contraction row k is row arow[k] of the stored
  // A (the weight gradient of a layer whose input rows are shared by several batch rows); mrow,
  // gemm_ws_kernel: the mask of output row m is row mrow[m] of the mask matrix; mdev, gemm_ws_kernel:
  // the row count read from device memory (<= M; the grid is sized for M)
  const int32_t* arow;
  const int32_t* garow[GEMM_GMAX];
  const int32_t* mrow;
  const int32_t* gmrow[GEMM_GMAX];
  const int64_t* mdev;
  const int64_t* gmdev[GEMM_GMAX];
};

// gemm_skinny.hip: the Dense layers' forward / dX kernel for large batches (envelope and launch)
bool skinny_ok(int ta, int tb, const GemmParams& p);
void skinny_dispatch(int tb, const GemmParams& p, hipStream_t st);
// gemm_ws.hip: the weight-stationary forward / dX kernel for large batches (envelope and launch)
bool ws_ok(int ta, int tb, const GemmParams& p);
void ws_dispatch(int tb, const GemmParams& p, hipStream_t st);
// gemm_ws.hip: the large-batch weight-gradient kernel (split-K slabs + column sums, as gemm_x3's)
bool wgrad_ws_ok(const GemmParams& p);
void wgrad_ws_dispatch(const GemmParams& p, int64_t slices, hipStream_t st);
int64_t wgrad_ws_kps(const GemmParams& p, int64_t kps_min);

}  // namespace rs
