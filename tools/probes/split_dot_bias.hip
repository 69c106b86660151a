// Probe (round 5): the signed error of one long dot product sum_u P_u U_u (n = 4096 terms, the
// in-batch col pass's dC sums at C2: P ~ 2^-12 (1 + 4 % noise) > 0, U ~ 0.05 + 0.01 N(0,1)) on the
// 16x16x32 bf16 MFMA over the exact three-plane splits (6 products, the kernels' order), in
// several accumulation arrangements, against the exact fp64 sum. Mean signed error in units of
// 2^-24 |sum| over many trials; a non-zero mean is a bias common to every output of such sums.
// Build: hipcc --offload-arch=gfx950 -O2 split_dot_bias.hip -o split_dot_bias
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r = x - (float)h;
  m = (__bf16)r;
  l = (__bf16)(r - (float)m);
}

// mode 0: running accumulator, classes mm, lh, hl, mh, hm, hh per 32-term tile (the kernels' order)
// mode 1: per-tile fresh accumulator (same order), then a fp32 VALU add into the running sum
// mode 2: hh into the running accumulator, the five small classes into a second running one
// mode 3: the f32 MFMA 32x32x2 on the unsplit values (the precision-0 kernels' instruction)
// mode 4: running accumulator, hh first then the small classes
__global__ void probe(int mode, int n, int ntrial, const float* P, const float* U, float* out) {
  const int lane = threadIdx.x;
  for (int t = blockIdx.x; t < ntrial; t += gridDim.x) {
    const float* p = P + (int64_t)t * n;
    const float* u = U + (int64_t)t * n;
    if (mode == 3) {
      f32x16 acc = {};
      for (int k = 0; k < n; k += 2) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(p[k + (lane >> 5)], u[k + (lane >> 5)], acc, 0, 0, 0);
      if (lane == 0) out[t] = acc[0];
      continue;
    }
    f32x4 run = {}, run2 = {};
    for (int k0 = 0; k0 < n; k0 += 32) {
      bf16x8 a[3], b[3];
      for (int e = 0; e < 8; ++e) {
        const int k = k0 + 8 * (lane >> 4) + e;
        __bf16 h, m, l;
        split3(p[k], h, m, l);
        a[0][e] = h; a[1][e] = m; a[2][e] = l;
        split3(u[k], h, m, l);
        b[0][e] = h; b[1][e] = m; b[2][e] = l;
      }
      const int ia[6] = {1, 2, 0, 1, 0, 0}, ib[6] = {1, 0, 2, 0, 1, 0};
      if (mode == 0) {
        for (int c = 0; c < 6; ++c) run = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ia[c]], b[ib[c]], run, 0, 0, 0);
      } else if (mode == 1) {
        f32x4 tmp = {};
        for (int c = 0; c < 6; ++c) tmp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ia[c]], b[ib[c]], tmp, 0, 0, 0);
        run += tmp;
      } else if (mode == 2) {
        for (int c = 0; c < 5; ++c) run2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ia[c]], b[ib[c]], run2, 0, 0, 0);
        run = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], run, 0, 0, 0);
      } else {
        for (int c = 5; c >= 0; --c) run = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ia[c]], b[ib[c]], run, 0, 0, 0);
      }
    }
    if (mode == 2) run += run2;
    if (lane == 0) out[t] = run[0];
  }
}

int main() {
  const int n = 4096, T = 2048;
  std::mt19937_64 rng(7);
  std::normal_distribution<double> nd(0.0, 1.0);
  std::uniform_real_distribution<double> ud(0.0, 1.0);
  const char* names[5] = {"running, small classes first", "fresh per 32-term tile + add", "hh / small classes apart",
                          "f32 MFMA 32x32x2 unsplit", "running, hh first"};
  for (int sc = 0; sc < 2; ++sc) {
    std::vector<float> P((size_t)n * T), U((size_t)n * T);
    std::vector<double> ex(T);
    for (int t = 0; t < T; ++t) {
      double s = 0;
      for (int k = 0; k < n; ++k) {
        const float pv = (float)(std::ldexp(1.0, -12) * (1.0 + 0.04 * ud(rng)));
        const float uv = sc == 0 ? (float)(0.05 + 0.01 * nd(rng)) : (float)(0.05 * nd(rng));
        P[(size_t)t * n + k] = pv;
        U[(size_t)t * n + k] = uv;
        s += (double)pv * (double)uv;
      }
      ex[t] = s;
    }
    float *dP, *dU, *dO;
    (void)hipMalloc(&dP, P.size() * 4); (void)hipMalloc(&dU, U.size() * 4); (void)hipMalloc(&dO, T * 4);
    (void)hipMemcpy(dP, P.data(), P.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dU, U.data(), U.size() * 4, hipMemcpyHostToDevice);
    std::vector<float> o(T);
    printf("U %s\n", sc == 0 ? "0.05 + 0.01 N(0,1) (one sign: a tower output's bias)" : "0.05 N(0,1) (mixed signs)");
    for (int mode = 0; mode < 5; ++mode) {
      hipLaunchKernelGGL(probe, dim3(512), dim3(64), 0, 0, mode, n, T, dP, dU, dO);
      (void)hipMemcpy(o.data(), dO, T * 4, hipMemcpyDeviceToHost);
      double ms = 0, ma = 0;
      for (int t = 0; t < T; ++t) {
        const double e = ((double)o[t] - ex[t]) / (std::fabs(ex[t]) * std::ldexp(1.0, -24));
        ms += e;
        ma += std::fabs(e);
      }
      printf("  %-32s mean err %+8.3f  mean |err| %7.3f  (units of 2^-24 |sum|)\n", names[mode], ms / T, ma / T);
    }
    (void)hipFree(dP); (void)hipFree(dU); (void)hipFree(dO);
  }
  return 0;
}
