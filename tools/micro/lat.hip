// Latency probes for the dependent-chain primitives the wave LCP kernels use.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../nimblephysics_amd/csrc/wave.cuh"

#define N 1024
__global__ void __launch_bounds__(64) probe(double* out, double a, double b, int k) {
  const int lane = threadIdx.x;
  double x = lane * 1e-3;
  long long t0, t1;
  // 1: dependent fp64 FMA
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) x = fma(x, a, b);
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[0] = (double)(t1 - t0) / N;
  // 2: readlane -> fma (lane-k broadcast chain)
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) x = fma(rdl(x, k), a, x);
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[1] = (double)(t1 - t0) / N;
  // 3: masked fma (lane > i%48) -> readlane  (solveL1 step)
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) {
    const int kk = i & 31;
    const double bk = rdl(x, kk);
    if (lane > kk && lane < 40) x -= a * bk;
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[2] = (double)(t1 - t0) / N;
  // 4: dependent fp64 add
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) x = x + b;
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[3] = (double)(t1 - t0) / N;
  // 5: dependent fp64 division
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) x = b / x;
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[4] = (double)(t1 - t0) / N;
  // 6: waveSum chain
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) x = waveSum(x) * 1e-3;
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[5] = (double)(t1 - t0) / N;
  // 7: independent fma throughput (8 chains)
  double y[8];
  for (int u = 0; u < 8; u++) y[u] = x + u;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) {
#pragma unroll
    for (int u = 0; u < 8; u++) y[u] = fma(y[u], a, b);
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[6] = (double)(t1 - t0) / (8 * N);
  // 8: LDS round trip chain
  __shared__ double s[64];
  s[lane] = x;
  t0 = __builtin_amdgcn_s_memtime();
  int idx = lane;
  for (int i = 0; i < N; i++) {
    const double v = s[idx];
    idx = ((int)v & 0) + ((idx + 1) & 63);
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[7] = (double)(t1 - t0) / N;
  // 9: waveMin chain
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) x = waveMin(x) + b;
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[8] = (double)(t1 - t0) / N;
  // 10: s_memtime rate vs wall: spin 1M memtime ticks
  for (int u = 0; u < 8; u++) x += y[u];
  out[16 + lane] = x + idx;
}

int main() {
  double* d;
  hipMalloc(&d, 128 * sizeof(double));
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 2; rep++) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, 0.999, 1e-3, 5);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
  }
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double h[16];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[] = {"fma chain", "readlane->fma", "solveL1 step", "add chain", "div chain", "waveSum chain",
                      "fma throughput", "LDS read chain", "waveMin chain"};
  for (int i = 0; i < 9; i++) printf("%-16s %8.1f clk\n", nm[i], h[i]);
  printf("kernel %.3f ms\n", ms);
  return 0;
}
