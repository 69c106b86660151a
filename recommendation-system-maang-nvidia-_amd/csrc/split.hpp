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

}  // namespace rs
