// PGS sweep latency micro-benchmark (the LCP fallback of the forward's
// cascade, lcp_wave.cuh wavePgsR): one 24-row contact-layout problem per
// 64-lane wave (8 contacts: a normal row and two friction rows each, A =
// J J^T + 1e-3 I from a fixed pseudo-random J), the PGS fallback from x = 0
// at shift 1e-4; clocks per solve and per row step (sweeps x rows), solo
// (one wave on the GPU) and at 1024 waves.  Prints JSON.
#include <cstdio>
#include <vector>

#include "../../nimblephysics_amd/csrc/lcp_wave.cuh"

__device__ double hrand(unsigned k) {
  k ^= k >> 16; k *= 0x7feb352dU; k ^= k >> 15; k *= 0x846ca68bU; k ^= k >> 16;
  return (k & 0xffffff) / double(0x1000000) - 0.5;
}

extern "C" __global__ void __launch_bounds__(64) pgs_bench(double* out, int n, int sweepsCap) {
  __shared__ double A[24 * 24];
  const int lane = threadIdx.x, w = blockIdx.x;
  // J: 24 x 12, A = J J^T + 1e-3 I
  for (int t = lane; t < n * n; t += 64) {
    const int i = t / n, j = t % n;
    double acc = i == j ? 1e-3 : 0.0;
    for (int k = 0; k < 12; k++) acc += hrand(w * 7919u + i * 131u + k) * hrand(w * 7919u + j * 131u + k);
    A[t] = acc;
  }
  __syncthreads();
  const bool live = lane < n;
  const int c = lane / 3, r = lane % 3;
  double x[1] = {0.0};
  const double b[1] = {live ? hrand(w * 31u + lane + 100000u) : 0.0};
  const double lo[1] = {live ? (r == 0 ? 0.0 : -0.8) : 0.0}, hi[1] = {live ? (r == 0 ? 1e30 : 0.8) : 0.0};
  const int fi[1] = {live && r ? 3 * c : -1};
  double dbg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const long long t0 = __builtin_amdgcn_s_memtime();
  const bool ok = wavePgsR<true, false, 1>(n, spc<true>(A), x, b, lo, hi, fi, lane, dbg, 1e-4, nullptr);
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    out[w * 4 + 0] = (double)(t1 - t0);
    out[w * 4 + 1] = dbg[0] + 1;  // sweeps (the first one plus the iterations)
    out[w * 4 + 2] = ok ? 1 : 0;
    out[w * 4 + 3] = dbg[1];
  }
  (void)sweepsCap;
}

int main() {
  const int n = 24;
  double* d;
  hipMalloc(&d, 1024 * 4 * sizeof(double));
  std::printf("{");
  for (int B : {1, 1024}) {
    for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(pgs_bench, dim3(B), dim3(64), 0, 0, d, n, 30);
    hipDeviceSynchronize();
    std::vector<double> h(B * 4);
    hipMemcpy(h.data(), d, B * 4 * sizeof(double), hipMemcpyDeviceToHost);
    double clk = 0, sw = 0, contact = 0;
    for (int w = 0; w < B; w++) { clk += h[w * 4]; sw += h[w * 4 + 1]; contact += h[w * 4 + 3]; }
    std::printf("%s\"%s\": {\"clk_per_solve\": %.0f, \"sweeps\": %.2f, \"clk_per_row_step\": %.1f, \"contact_layout\": %.2f}",
                B == 1 ? "" : ", ", B == 1 ? "solo" : "batch_1024", clk / B, sw / B, clk / sw / n, contact / B);
  }
  std::printf("}\n");
  return 0;
}
