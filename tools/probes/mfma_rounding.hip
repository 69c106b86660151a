// Probe: how the gfx950 MFMAs round their fp32 accumulation. Each trial feeds one MFMA with
// A[i][k] = a_k, B[k][j] = b_k (the same k mapping on both operands, so every output element is
// c + sum_k a_k b_k whatever the lane layout) and compares the result with that sum computed in
// fp64 and rounded to fp32 to nearest-even and toward zero. Prints the counts and the mean signed
// error in ulps. Build: hipcc --offload-arch=gfx950 -O2 mfma_rounding.hip -o /tmp/mfma_rounding
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

// kind 0: 16x16x32 bf16 (k = 8 (lane / 16) + e); kind 1: 32x32x2 f32 (k = lane / 32);
// kind 2: 16x16x4 f32 (k = lane / 16)
__global__ void probe(int kind, int ntrial, const float* a, const float* b, const float* c, float* out) {
  const int lane = threadIdx.x;
  for (int t = blockIdx.x; t < ntrial; t += gridDim.x) {
    const float* at = a + t * 32;
    const float* bt = b + t * 32;
    if (kind == 0) {
      bf16x8 av, bv;
      for (int e = 0; e < 8; ++e) {
        av[e] = (__bf16)at[8 * (lane >> 4) + e];
        bv[e] = (__bf16)bt[8 * (lane >> 4) + e];
      }
      f32x4 acc = {c[t], c[t], c[t], c[t]};
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
      if (lane == 0) out[t] = acc[0];
    } else if (kind == 1) {
      f32x16 acc;
      for (int r = 0; r < 16; ++r) acc[r] = c[t];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(at[lane >> 5], bt[lane >> 5], acc, 0, 0, 0);
      if (lane == 0) out[t] = acc[0];
    } else {
      f32x4 acc = {c[t], c[t], c[t], c[t]};
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(at[lane >> 4], bt[lane >> 4], acc, 0, 0, 0);
      if (lane == 0) out[t] = acc[0];
    }
  }
}

static float bf16_round(float x) {  // RNE to bf16
  uint32_t u;
  memcpy(&u, &x, 4);
  u = (u + 0x7fff + ((u >> 16) & 1)) & 0xffff0000u;
  memcpy(&x, &u, 4);
  return x;
}
static float rtz(double v) {
  float f = (float)v;
  if (std::fabs((double)f) > std::fabs(v)) f = std::nextafter(f, 0.f);
  return f;
}

int main() {
  const int N = 1 << 16;
  const char* names[3] = {"16x16x32_bf16", "32x32x2_f32", "16x16x4_f32"};
  const int nk[3] = {32, 2, 4};
  const int regimes[4][2] = {{2, 10}, {18, 26}, {22, 30}, {26, 34}};
  for (int kind = 0; kind < 3; ++kind) {
   for (int rg = 0; rg < 4; ++rg) {
    for (int sign = 0; sign < 2; ++sign) {
      std::mt19937_64 rng(1234 + kind + 10 * sign);
      std::uniform_real_distribution<double> u(0.0, 1.0);
      std::vector<float> a(N * 32, 0.f), b(N * 32, 0.f), c(N), out(N);
      for (int t = 0; t < N; ++t) {
        c[t] = (float)(0.5 + 0.5 * u(rng));
        for (int k = 0; k < nk[kind]; ++k) {
          // products of 2^-12 .. 2^-4 of c: many bits below c's ulp
          float av = (float)((1.0 + u(rng)) * std::ldexp(1.0, -(int)(u(rng) * (regimes[rg][1] - regimes[rg][0])) - regimes[rg][0]));
          float bv = (float)((1.0 + u(rng)) * std::ldexp(1.0, -2));
          if (sign && u(rng) < 0.5) av = -av;
          if (kind == 0) { av = bf16_round(av); bv = bf16_round(bv); }
          a[t * 32 + k] = av;
          b[t * 32 + k] = bv;
        }
      }
      float *da, *db, *dc, *dout;
      hipMalloc(&da, a.size() * 4); hipMalloc(&db, b.size() * 4); hipMalloc(&dc, N * 4); hipMalloc(&dout, N * 4);
      hipMemcpy(da, a.data(), a.size() * 4, hipMemcpyHostToDevice);
      hipMemcpy(db, b.data(), b.size() * 4, hipMemcpyHostToDevice);
      hipMemcpy(dc, c.data(), N * 4, hipMemcpyHostToDevice);
      hipLaunchKernelGGL(probe, dim3(1024), dim3(64), 0, 0, kind, N, da, db, dc, dout);
      hipMemcpy(out.data(), dout, N * 4, hipMemcpyDeviceToHost);
      long rne = 0, rz = 0, other = 0;
      double sum_ulp = 0, sum_abs = 0;
      for (int t = 0; t < N; ++t) {
        double s = c[t];
        for (int k = 0; k < nk[kind]; ++k) s += (double)a[t * 32 + k] * (double)b[t * 32 + k];
        const float fr = (float)s, fz = rtz(s);
        if (out[t] == fr) ++rne;
        if (out[t] == fz) ++rz;
        if (out[t] != fr && out[t] != fz) ++other;
        const double ulp = std::ldexp(1.0, std::ilogb(s) - 23);
        sum_ulp += ((double)out[t] - s) / ulp;
        sum_abs += std::fabs(((double)out[t] - s) / ulp);
      }
      printf("products 2^-%d..2^-%d of c  ", regimes[rg][0], regimes[rg][1] + 2);
      printf("%-14s %s: RNE match %ld  RTZ match %ld  neither %ld  of %d; mean err %+.4f ulp, mean |err| %.4f ulp\n",
             names[kind], sign ? "mixed-sign" : "positive  ", rne, rz, other, N, sum_ulp / N, sum_abs / N);
      hipFree(da); hipFree(db); hipFree(dc); hipFree(dout);
    }
   }
  }
  return 0;
}
