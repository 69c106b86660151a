// Gather-kernel variants for an in-process A/B (tools/ab_gather.py); not part of the product.
#include <hip/hip_runtime.h>
#include <cstdint>

typedef float f32x4 __attribute__((ext_vector_type(4)));

// RIF: 16-B pieces in flight per thread; NT_LOAD / NT_STORE: non-temporal hints.
template <int RIF, bool NT_LOAD, bool NT_STORE>
__global__ __launch_bounds__(256) void gather_v(const float* __restrict__ table, int64_t qpr,
                                                const int64_t* __restrict__ ids, int64_t total,
                                                float* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const f32x4* t4 = reinterpret_cast<const f32x4*>(table);
  f32x4* o4 = reinterpret_cast<f32x4*>(out);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride * RIF) {
    f32x4 v[RIF];
    int64_t idx[RIF];
#pragma unroll
    for (int u = 0; u < RIF; ++u) {
      idx[u] = i + u * stride;
      if (idx[u] < total) {
        const int64_t row = idx[u] / qpr, q = idx[u] - row * qpr;
        const f32x4* src = t4 + ids[row] * qpr + q;
        v[u] = NT_LOAD ? __builtin_nontemporal_load(src) : *src;
      }
    }
#pragma unroll
    for (int u = 0; u < RIF; ++u)
      if (idx[u] < total) {
        if (NT_STORE) __builtin_nontemporal_store(v[u], o4 + idx[u]);
        else o4[idx[u]] = v[u];
      }
  }
}

// Row-blocked: each wave copies whole rows, ROWS rows in flight per wave (D = 128: a half-wave
// moves one 512-B row per instruction, so ROWS/2 instructions per batch).
template <int ROWS>
__global__ __launch_bounds__(256) void gather_rows_blocked(const float* __restrict__ table, int64_t qpr,
                                                           const int64_t* __restrict__ ids, int64_t n,
                                                           float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int per_inst = 64 / (int)qpr;  // rows per wave-instruction (2 for D=128)
  const f32x4* t4 = reinterpret_cast<const f32x4*>(table);
  f32x4* o4 = reinterpret_cast<f32x4*>(out);
  const int sub = lane / (int)qpr, q = lane % (int)qpr;
  for (int64_t r0 = wave * ROWS; r0 < n; r0 += nwaves * ROWS) {
    f32x4 v[ROWS / 2];
    int64_t rr[ROWS / 2];
#pragma unroll
    for (int u = 0; u < ROWS / 2; ++u) {
      rr[u] = r0 + u * per_inst + sub;
      if (rr[u] < n) v[u] = __builtin_nontemporal_load(t4 + ids[rr[u]] * qpr + q);
    }
#pragma unroll
    for (int u = 0; u < ROWS / 2; ++u)
      if (rr[u] < n) o4[rr[u] * qpr + q] = v[u];
  }
}

// Compile-time row width (shift instead of a 64-bit divide), 32-bit index math.
template <int QPR, int RIF>
__global__ __launch_bounds__(256) void gather_q(const float* __restrict__ table, const int64_t* __restrict__ ids,
                                                int total, float* __restrict__ out) {
  const int stride = gridDim.x * blockDim.x;
  const f32x4* t4 = reinterpret_cast<const f32x4*>(table);
  f32x4* o4 = reinterpret_cast<f32x4*>(out);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride * RIF) {
    f32x4 v[RIF];
#pragma unroll
    for (int u = 0; u < RIF; ++u) {
      const int idx = i + u * stride;
      if (idx < total) v[u] = __builtin_nontemporal_load(t4 + ids[idx / QPR] * QPR + (idx % QPR));
    }
#pragma unroll
    for (int u = 0; u < RIF; ++u) {
      const int idx = i + u * stride;
      if (idx < total) o4[idx] = v[u];
    }
  }
}

// Wave loads 64 ids at once (one per lane), then streams those rows: 64/QPR rows per
// instruction, BATCH instructions in flight before the stores; ids broadcast by readlane.
template <int QPR, int BATCH>
__global__ __launch_bounds__(256) void gather_w(const float* __restrict__ table, const int64_t* __restrict__ ids,
                                                int n, float* __restrict__ out) {
  constexpr int RPI = 64 / QPR;  // rows per instruction
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const f32x4* t4 = reinterpret_cast<const f32x4*>(table);
  f32x4* o4 = reinterpret_cast<f32x4*>(out);
  const int sub = lane / QPR, q = lane % QPR;
  for (int r0 = wave * 64; r0 < n; r0 += nwaves * 64) {
    const int64_t my_id = (r0 + lane < n) ? ids[r0 + lane] : 0;
    for (int b0 = 0; b0 < 64; b0 += BATCH * RPI) {
      f32x4 v[BATCH];
#pragma unroll
      for (int u = 0; u < BATCH; ++u) {
        const int rr = b0 + u * RPI + sub;
        const int64_t id = __shfl(my_id, rr);
        if (r0 + rr < n) v[u] = __builtin_nontemporal_load(t4 + id * QPR + q);
      }
#pragma unroll
      for (int u = 0; u < BATCH; ++u) {
        const int rr = b0 + u * RPI + sub;
        if (r0 + rr < n) o4[(int64_t)(r0 + rr) * QPR + q] = v[u];
      }
    }
  }
}

// Generalised wave variant: RPW rows per wave iteration, all in flight.
template <int QPR, int RPW>
__global__ __launch_bounds__(256) void gather_wr(const float* __restrict__ table, const int64_t* __restrict__ ids,
                                                 int n, float* __restrict__ out) {
  constexpr int RPI = 64 / QPR;
  constexpr int NI = RPW / RPI;
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const f32x4* t4 = reinterpret_cast<const f32x4*>(table);
  f32x4* o4 = reinterpret_cast<f32x4*>(out);
  const int sub = lane / QPR, q = lane % QPR;
  for (int r0 = wave * RPW; r0 < n; r0 += nwaves * RPW) {
    const int64_t my_id = (lane < RPW && r0 + lane < n) ? ids[r0 + lane] : 0;
    f32x4 v[NI];
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int rr = u * RPI + sub;
      const int64_t id = __shfl(my_id, rr);
      if (r0 + rr < n) v[u] = __builtin_nontemporal_load(t4 + id * QPR + q);
    }
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int rr = u * RPI + sub;
      if (r0 + rr < n) o4[(int64_t)(r0 + rr) * QPR + q] = v[u];
    }
  }
}

extern "C" int gather_variant(int which, const float* table, int64_t dim, const int64_t* ids, int64_t n,
                              float* out, int blocks, hipStream_t st) {
  const int64_t qpr = dim / 4, total = n * qpr;
  dim3 g(blocks), b(256);
  switch (which) {
    case 0: hipLaunchKernelGGL((gather_v<4, true, false>), g, b, 0, st, table, qpr, ids, total, out); break;
    case 1: hipLaunchKernelGGL((gather_v<8, true, false>), g, b, 0, st, table, qpr, ids, total, out); break;
    case 2: hipLaunchKernelGGL((gather_v<8, true, true>), g, b, 0, st, table, qpr, ids, total, out); break;
    case 3: hipLaunchKernelGGL((gather_v<8, false, false>), g, b, 0, st, table, qpr, ids, total, out); break;
    case 4: hipLaunchKernelGGL((gather_v<16, true, false>), g, b, 0, st, table, qpr, ids, total, out); break;
    case 5: hipLaunchKernelGGL((gather_rows_blocked<8>), g, b, 0, st, table, qpr, ids, n, out); break;
    case 6: hipLaunchKernelGGL((gather_rows_blocked<16>), g, b, 0, st, table, qpr, ids, n, out); break;
    case 7: hipLaunchKernelGGL((gather_q<32, 4>), g, b, 0, st, table, ids, (int)total, out); break;
    case 8: hipLaunchKernelGGL((gather_q<32, 8>), g, b, 0, st, table, ids, (int)total, out); break;
    case 9: hipLaunchKernelGGL((gather_w<32, 8>), g, b, 0, st, table, ids, (int)n, out); break;
    case 10: hipLaunchKernelGGL((gather_w<32, 16>), g, b, 0, st, table, ids, (int)n, out); break;
    case 11: hipLaunchKernelGGL((gather_w<32, 32>), g, b, 0, st, table, ids, (int)n, out); break;
    case 12: hipLaunchKernelGGL((gather_wr<32, 16>), g, b, 0, st, table, ids, (int)n, out); break;
    case 13: hipLaunchKernelGGL((gather_wr<32, 32>), g, b, 0, st, table, ids, (int)n, out); break;
    case 14: hipLaunchKernelGGL((gather_wr<32, 64>), g, b, 0, st, table, ids, (int)n, out); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
