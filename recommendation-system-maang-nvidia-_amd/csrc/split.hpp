// split.hpp — fp32 operands on the bf16 matrix cores: exact three-term bf16 splits.
//
// x = h + m + l with h = bf16(x), m = bf16(x - h), l = x - h - m: each difference is exact in
// fp32 and l fits bf16's 8-bit significand, so the split is exact (for |x| above ~2^-110; the
// embeddings and activations of this path are far above that). A product x.y is the sum of the
// cross products of the terms, each exact in the fp32 accumulator of v_mfma_f32_32x32x16_bf16:
// NP = 9 sums all nine (the fp32 products exactly), NP = 6 drops m.l, l.m and l.l (< 2^-23 of
// |x.y|, one fp32 ulp). Used by inbatch.hip and gemm.hip (include/recsys_hip.h RS_PREC_*).
#pragma once
#include "common.hpp"

namespace rs {

typedef __bf16 ib_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 ib_bf16x2 __attribute__((ext_vector_type(2)));
typedef short ib_s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t ib_pk(float a, float b) {
  const ib_bf16x2 r = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ float ib_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float ib_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
// (a, b) -> packed bf16 pairs h, m, l with a = h + m + l and b likewise, exactly
struct IbSplit {
  uint32_t h, m, l;
};
__device__ __forceinline__ IbSplit ib_split2(float a, float b) {
  IbSplit r;
  r.h = ib_pk(a, b);
  const float ra = a - ib_lo(r.h), rb = b - ib_hi(r.h);
  r.m = ib_pk(ra, rb);
  r.l = ib_pk(ra - ib_lo(r.m), rb - ib_hi(r.m));
  return r;
}
// the same split on a float pair, the differences as packed fp32 (v_pk_add_f32): 9 VALU per pair
typedef float f32x2 __attribute__((ext_vector_type(2)));
// (the empty asm keeps hipcc from re-deriving the low half by a second v_cvt_pk_bf16_f32 of the
// first element alone: one VALU per stage)
__device__ __forceinline__ IbSplit ib_split2v(f32x2 x) {
  IbSplit r;
  r.h = ib_pk(x[0], x[1]);
  asm("" : "+v"(r.h));
  const f32x2 rx = x - f32x2{ib_lo(r.h), ib_hi(r.h)};
  r.m = ib_pk(rx[0], rx[1]);
  asm("" : "+v"(r.m));
  const f32x2 lx = rx - f32x2{ib_lo(r.m), ib_hi(r.m)};
  r.l = ib_pk(lx[0], lx[1]);
  return r;
}
__device__ __forceinline__ f32x16 mfma_bf16(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(ib_bf16x8, a), __builtin_bit_cast(ib_bf16x8, b),
                                                  c, 0, 0, 0);
}
// c += sum of the NP cross products of the split operands, smallest terms first
template <int NP>
__device__ __forceinline__ f32x16 mfma_split(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x16 c) {
  if constexpr (NP == 9) {
    c = mfma_bf16(a[2], b[2], c);
    c = mfma_bf16(a[2], b[1], c);
    c = mfma_bf16(a[1], b[2], c);
  }
  c = mfma_bf16(a[1], b[1], c);
  c = mfma_bf16(a[2], b[0], c);
  c = mfma_bf16(a[0], b[2], c);
  c = mfma_bf16(a[1], b[0], c);
  c = mfma_bf16(a[0], b[1], c);
  c = mfma_bf16(a[0], b[0], c);
  return c;
}
__device__ __forceinline__ f32x4 mfma16_bf16(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(ib_bf16x8, a), __builtin_bit_cast(ib_bf16x8, b),
                                                  c, 0, 0, 0);
}
// N independent accumulators c[i] += a[i] . b[i] over the NP cross products, product-major (each
// accumulator sees the same product order as mfma16_split; consecutive MFMAs are independent)
template <int NP, int N>
__device__ __forceinline__ void mfma16_split_n(const u32x4* const (&a)[N], const u32x4* const (&b)[N],
                                               f32x4* const (&c)[N]) {
  constexpr int ia[9] = {2, 2, 1, 1, 2, 0, 1, 0, 0}, ib[9] = {2, 1, 2, 1, 0, 2, 0, 1, 0};
#pragma unroll
  for (int k = 9 - NP; k < 9; ++k)
#pragma unroll
    for (int i = 0; i < N; ++i) *c[i] = mfma16_bf16(a[i][ia[k]], b[i][ib[k]], *c[i]);
}

// Plane images of 32-row x 128-column fp32 tiles (the in-batch and top-k kernels, D = 128): per
// tile three 8 KB planes (h, m, l). A plane is 8-row x 32-column subtiles of 512 B with the 16-B
// chunks of a subtile row XOR-swizzled by bits 2-3 of the row; ibx_off is the byte offset of
// chunk ch (8 bf16) of row r. Row reads (ds_read_b128: the A operand of an S = X Y^T product)
// and transposed reads (ds_read_b64_tr_b16: X^T as an operand) are conflict-free, and each kind
// needs only two per-lane base addresses, the rest being instruction offsets.
constexpr int IBX_D = 128;
constexpr int IBX_ROWB = 2 * IBX_D;        // bytes per plane row
constexpr int IBX_PLANE = 32 * IBX_ROWB;   // one plane image of a 32-row tile
constexpr int IBX_BUF = 3 * IBX_PLANE;     // h, m, l planes
__device__ __forceinline__ int ibx_off(int r, int ch) {
  return 2048 * (r >> 3) + 512 * (ch >> 2) + 64 * (r & 7) + 16 * ((ch & 3) ^ ((r >> 2) & 3));
}
// split-store 4 consecutive columns (c4 = column / 4) of row r of a tile image
__device__ __forceinline__ void ibx_put4(char* img, int r, int c4, f32x4 v) {
  const IbSplit s0 = ib_split2(v[0], v[1]), s1 = ib_split2(v[2], v[3]);
  const int off = ibx_off(r, c4 >> 1) + 8 * (c4 & 1);
  *reinterpret_cast<u32x2*>(img + off) = u32x2{s0.h, s1.h};
  *reinterpret_cast<u32x2*>(img + IBX_PLANE + off) = u32x2{s0.m, s1.m};
  *reinterpret_cast<u32x2*>(img + 2 * IBX_PLANE + off) = u32x2{s0.l, s1.l};
}

}  // namespace rs
