// Y = L^-1 J^T micro-benchmark (contact.cuh formY, the LCP rows' massed
// columns): n = 33 dofs, m = 24 rows, one problem per 64-lane wave in LDS,
// (blocked: formYWide; halves: formY's two-half form for <= 32 columns)
// against the row-at-a-time loop it replaced (kept here as the reference:
// the results must be bit-identical).  Clocks per call, solo and at 2048
// waves (two per SIMD).  Prints JSON.
#include <cstdio>
#include <vector>
#include "../../nimblephysics_amd/csrc/model.h"
#include "../../nimblephysics_amd/csrc/spatial.cuh"
#include "../../nimblephysics_amd/csrc/wave.cuh"
#include "../../nimblephysics_amd/csrc/stamp.cuh"
#include "../../nimblephysics_amd/csrc/chol_wave.cuh"
#include "../../nimblephysics_amd/csrc/contact.cuh"

__device__ double hr(unsigned k) {
  k ^= k >> 16; k *= 0x7feb352dU; k ^= k >> 15; k *= 0x846ca68bU; k ^= k >> 16;
  return (k & 0xffffff) / double(0x1000000) - 0.5;
}

// the row-at-a-time loop (r05..r06n)
__device__ void formYRows(double* Y, const double* Lm, const double* dinv, int n, int m, int lane) {
  for (int j = lane; j < m; j += WAVE) {
    for (int i = 0; i < n; i++) {
      double acc = Y[i * m + j];
      const double* Li = Lm + tri(i, 0);
      int k = 0;
      for (; k + 8 <= i; k += 8) {
        double lv[8], yv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) { lv[u] = Li[k + u]; yv[u] = Y[(k + u) * m + j]; }
#pragma unroll
        for (int u = 0; u < 8; u++) asm volatile("" : "+v"(lv[u]), "+v"(yv[u]));
#pragma unroll
        for (int u = 0; u < 8; u++) acc -= lv[u] * yv[u];
      }
      for (; k < i; k++) acc -= Li[k] * Y[k * m + j];
      Y[i * m + j] = acc * dinv[i];
    }
  }
  WSYNC();
}

extern "C" __global__ void __launch_bounds__(64) formy_bench(double* out, int n, int m, int variant) {
  __shared__ double Lm[33 * 34 / 2], dinv[33], Y[33 * 24];
  const int lane = threadIdx.x, w = blockIdx.x;
  for (int t = lane; t < n * (n + 1) / 2; t += 64) Lm[t] = hr(w * 7919u + t) * 0.1;
  for (int t = lane; t < n; t += 64) { dinv[t] = 1.0 / (1.0 + 0.5 * hr(w * 31u + t + 5000u)); Lm[tri(t, t)] = 1.0 / dinv[t]; }
  for (int t = lane; t < n * m; t += 64) Y[t] = hr(w * 131u + t + 90000u);
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  if (variant == 0) formYRows(Y, Lm, dinv, n, m, lane);
  else if (variant == 1) formYWide(Y, Y, Lm, dinv, n, m, lane);
  else formY(Y, Y, Lm, dinv, n, m, lane);
  const long long t1 = __builtin_amdgcn_s_memtime();
  for (int t = lane; t < n * m; t += 64) out[(size_t)w * (n * m + 1) + 1 + t] = Y[t];
  if (lane == 0) out[(size_t)w * (n * m + 1)] = (double)(t1 - t0);
}

int main() {
  const int n = 33, m = 24, rec = n * m + 1;
  double* d;
  hipMalloc(&d, (size_t)2048 * rec * sizeof(double));
  std::vector<double> h[3];
  std::printf("{");
  const char* names[3] = {"rows", "blocked", "halves"};
  for (int v = 0; v < 3; v++) {
    for (int B : {1, 2048}) {
      for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(formy_bench, dim3(B), dim3(64), 0, 0, d, n, m, v);
      hipDeviceSynchronize();
      std::vector<double> o((size_t)B * rec);
      hipMemcpy(o.data(), d, o.size() * sizeof(double), hipMemcpyDeviceToHost);
      double clk = 0;
      for (int w = 0; w < B; w++) clk += o[(size_t)w * rec];
      std::printf("%s\"%s_%s\": %.0f", (v || B > 1) ? ", " : "", names[v], B == 1 ? "solo" : "2048", clk / B);
      if (B == 2048) h[v] = o;
    }
  }
  size_t diff = 0, diff2 = 0;
  for (size_t i = 0; i < h[0].size(); i++) {
    if (i % rec && h[0][i] != h[1][i]) diff++;
    if (i % rec && h[0][i] != h[2][i]) diff2++;
  }
  std::printf(", \"elements_differing\": %zu, \"elements_differing_halves\": %zu}\n", diff, diff2);
  return 0;
}
