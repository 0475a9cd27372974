// Latency probes (dependent chains) for LDS loads, scalar (K$) loads and
// vector global loads on gfx950; one wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#define N 256
__global__ void __launch_bounds__(64) probe(double* out, const int* __restrict__ gidx, int k) {
  __shared__ int lds[1024];
  const int lane = threadIdx.x;
  for (int i = lane; i < 1024; i += 64) lds[i] = (i * 7 + 3) & 1023;
  __syncthreads();
  long long t0, t1;
  // 1: dependent LDS load chain (uniform address)
  int p = k;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) p = lds[p];
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[0] = (double)(t1 - t0) / N;
  // 2: dependent LDS load chain (per-lane address)
  int q = (k + lane) & 1023;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) q = lds[q];
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[1] = (double)(t1 - t0) / N;
  // 3: dependent scalar load chain
  int sp = __builtin_amdgcn_readfirstlane(k);
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) sp = __builtin_amdgcn_readfirstlane(gidx[sp]);
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[2] = (double)(t1 - t0) / N;
  // 4: dependent vector global load chain (per-lane)
  int g = (k + lane) & 1023;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) g = gidx[g];
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[3] = (double)(t1 - t0) / N;
  // 5: s_memtime vs s_memrealtime (100 MHz) over a spin
  long long r0 = __builtin_amdgcn_s_memrealtime();
  t0 = __builtin_amdgcn_s_memtime();
  double x = lane;
  for (int i = 0; i < 20000; i++) x = fma(x, 1.0000001, 1e-9);
  t1 = __builtin_amdgcn_s_memtime();
  long long r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) { out[4] = (double)(t1 - t0) / ((double)(r1 - r0) / 100.0); out[5] = x; }
  (void)p; (void)q; (void)sp; (void)g;
  if (lane == 0) out[6] = p + q + sp + g;
}
int main() {
  int h[1024];
  for (int i = 0; i < 1024; i++) h[i] = (i * 13 + 5) & 1023;
  int* d; double* o;
  hipMalloc(&d, sizeof(h)); hipMalloc(&o, 8 * sizeof(double));
  hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, o, d, 5);
  double r[8];
  hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
  const char* nm[] = {"LDS load chain (uniform addr)", "LDS load chain (per-lane addr)", "scalar load chain (K$)",
                      "global load chain (per-lane)", "s_memtime ticks per us"};
  for (int i = 0; i < 5; i++) printf("%-34s %8.1f\n", nm[i], r[i]);
  return 0;
}
