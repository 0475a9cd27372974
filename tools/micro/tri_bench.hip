// Triangular-solve step costs (Dantzig's solveL1 / solveL1T): the bare
// readlane -> fp64 FMA chain against the WaveDantzig solves on an LDS factor,
// one wave per workgroup, shader clocks per solve and per step.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o dbg/tri_bench tools/micro/tri_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../nimblephysics_amd/csrc/lcp_wave.cuh"

#define STEPS 1024
template <int R, bool kPL = false>
__global__ void __launch_bounds__(64) tri(double* out, int m, int reps) {
  extern __shared__ double ldsbuf[];
  const int lane = threadIdx.x;
  const int ld = m | 1;
  const int nL = dantzigLDoubles(m, kPL);
  for (int t = lane; t < nL; t += 64) ldsbuf[t] = 1e-3 * ((t * 7919) % 97 - 48) / 97.0;
  __syncthreads();
  WaveDantzig<R, false, kPL> D;
  D.n = m;
  D.lane = lane;
  D.ldL = ld;
  D.L = ldsbuf;
  D.degen = false;
  double B[R];
  for (int s = 0; s < R; s++) B[s] = 1.0 + 1e-3 * (lane + 64 * s);
  long long t0, t1;
  double a = out[7], x = lane * 1e-3;
  // 1: readlane -> fma chain
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < STEPS; i++) x = fma(-a, rdl(x, i & 63), x);
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[0] = (double)(t1 - t0) / STEPS;
  // 2: readlane -> fma chain, 8 steps unrolled, lane index uniform per step
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < STEPS; i += 8) {
#pragma unroll
    for (int u = 0; u < 8; u++) x = fma(-a, rdl(x, (i + u) & 63), x);
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[1] = (double)(t1 - t0) / STEPS;
  // 3: solveL1 (m steps a call)
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; r++) D.solveL1(B, m);
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[2] = (double)(t1 - t0) / reps;
  // 4: solveL1T
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; r++) D.solveL1T(B, m);
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[3] = (double)(t1 - t0) / reps;
  // 6, 7: the predicated sweeps (a degenerate factor)
  D.degen = true;
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; r++) D.solveL1(B, m);
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[6] = (double)(t1 - t0) / reps;
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; r++) D.solveL1T(B, m);
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[7] = (double)(t1 - t0) / reps;
  // 5: empty timer pair
  t0 = __builtin_amdgcn_s_memtime();
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[4] = (double)(t1 - t0);
  if (lane == 0) out[5] = x + B[0];
  if (lane == 0 && out[5] == 12345.0) out[8] = 1;
}

int main() {
  double* d;
  (void)hipMalloc(&d, 64 * sizeof(double));
  double h[16] = {0, 0, 0, 0, 0, 0, 0, 1e-3};
  for (int R = 1; R <= 2; R++) {
    const int ms[] = {21, 24, 64, 90, 96};
    for (int pk = 0; pk < 2; pk++)
    for (int m : ms) {
      if ((R == 1 && m > 64) || (R == 2 && m < 64)) continue;
      (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
      const size_t lds = (size_t)dantzigLDoubles(m, pk) * sizeof(double);
      const void* f = R == 1 ? (pk ? (const void*)tri<1, true> : (const void*)tri<1>)
                             : (pk ? (const void*)tri<2, true> : (const void*)tri<2>);
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (R == 1 && pk) hipLaunchKernelGGL((tri<1, true>), dim3(1), dim3(64), lds, 0, d, m, 20);
      else if (R == 1) hipLaunchKernelGGL((tri<1>), dim3(1), dim3(64), lds, 0, d, m, 20);
      else if (pk) hipLaunchKernelGGL((tri<2, true>), dim3(1), dim3(64), lds, 0, d, m, 20);
      else hipLaunchKernelGGL((tri<2>), dim3(1), dim3(64), lds, 0, d, m, 20);
      (void)hipDeviceSynchronize();
      double o[16];
      (void)hipMemcpy(o, d, sizeof(o), hipMemcpyDeviceToHost);
      printf("%s R=%d m=%3d: chain step %.1f (unrolled %.1f) | solveL1 %.0f clk = %.1f/step | solveL1T %.0f clk = %.1f/step | predicated %.1f / %.1f per step | timer %.0f\n",
             pk ? "packed" : "square", R, m, o[0], o[1], o[2], o[2] / m, o[3], o[3] / m, o[6] / m, o[7] / m, o[4]);
    }
  }
  return 0;
}
