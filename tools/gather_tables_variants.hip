// Variants of the two-table gather (gather_tables_wave_kernel in csrc/embedding.hip) for an
// in-process A/B (tools/ab_gather_tables.py); not part of the product.
// NTL / NTS: non-temporal load / store hints; RPW rows per wave iteration (all in flight).
#include <hip/hip_runtime.h>
#include <cstdint>

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Jobs2 {
  const float* table[2];
  const int64_t* ids[2];
  float* out[2];
  int64_t n[2];
  int64_t wstart[3];
};

template <int RPW, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void gt_var(Jobs2 jobs) {
  constexpr int QPR = 32, RPI = 64 / QPR, NI = RPW / RPI;
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int sub = lane / QPR, q = lane % QPR;
  for (int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < jobs.wstart[2]; w += nwaves) {
    const int j = w >= jobs.wstart[1] ? 1 : 0;
    const f32x4* t4 = reinterpret_cast<const f32x4*>(jobs.table[j]);
    f32x4* o4 = reinterpret_cast<f32x4*>(jobs.out[j]);
    const int64_t n = jobs.n[j];
    const int64_t r0 = (w - jobs.wstart[j]) * RPW;
    int64_t ida = -1, idb = -1;
    if (lane < RPW && r0 + lane < n) ida = jobs.ids[j][r0 + lane];
    if (RPW > 64 && lane + 64 < RPW && r0 + 64 + lane < n) idb = jobs.ids[j][r0 + 64 + lane];
    f32x4 v[NI];
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int rr = u * RPI + sub;
      const int64_t id = rr < 64 ? __shfl(ida, rr) : __shfl(idb, rr - 64);
      v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (id >= 0) v[u] = NTL ? __builtin_nontemporal_load(t4 + id * QPR + q) : t4[id * QPR + q];
    }
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int64_t row = r0 + u * RPI + sub;
      if (row < n) {
        if (NTS) __builtin_nontemporal_store(v[u], o4 + row * QPR + q);
        else o4[row * QPR + q] = v[u];
      }
    }
  }
}

template <int RPW, bool NTL, bool NTS>
static void launch(Jobs2 j, int blocks_cap, hipStream_t st) {
  j.wstart[0] = 0;
  j.wstart[1] = (j.n[0] + RPW - 1) / RPW;
  j.wstart[2] = j.wstart[1] + (j.n[1] + RPW - 1) / RPW;
  int64_t blocks = (j.wstart[2] + 3) / 4;
  if (blocks_cap > 0 && blocks > blocks_cap) blocks = blocks_cap;
  hipLaunchKernelGGL((gt_var<RPW, NTL, NTS>), dim3((unsigned)blocks), dim3(256), 0, st, j);
}

extern "C" int gather_tables_variant(int which, const float* t0, const int64_t* i0, float* o0, int64_t n0,
                                     const float* t1, const int64_t* i1, float* o1, int64_t n1, int blocks_cap,
                                     hipStream_t st) {
  Jobs2 j{};
  j.table[0] = t0; j.ids[0] = i0; j.out[0] = o0; j.n[0] = n0;
  j.table[1] = t1; j.ids[1] = i1; j.out[1] = o1; j.n[1] = n1;
  switch (which) {
    case 0: launch<64, true, false>(j, blocks_cap, st); break;    // = product kernel
    case 1: launch<64, false, false>(j, blocks_cap, st); break;
    case 2: launch<64, true, true>(j, blocks_cap, st); break;
    case 3: launch<64, false, true>(j, blocks_cap, st); break;
    case 4: launch<32, true, false>(j, blocks_cap, st); break;
    case 5: launch<32, false, true>(j, blocks_cap, st); break;
    case 6: launch<128, true, false>(j, blocks_cap, st); break;
    case 7: launch<128, false, true>(j, blocks_cap, st); break;
    case 8: launch<16, false, true>(j, blocks_cap, st); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
