// Per-row cost probes of the PGS sweep step (one wave, uncontended).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../nimblephysics_amd/csrc/wave.cuh"

#define SW 29
__global__ void __launch_bounds__(64) probe(double* out, const double* Ag, int n, unsigned long long bounding,
                                            unsigned long long order) {
  __shared__ double A[24 * 24];
  const int lane = threadIdx.x;
  for (int t = lane; t < n * n; t += 64) A[t] = Ag[t];
  __syncthreads();
  const int col = lane < n ? lane : 0;
  double r = lane * 1e-3, xn = 0.1, hB = 1.0, lB = -1.0, diag = 1.0, dummyAct = 1.0, hi = 0.5;
  const int findex = lane >= 8 && lane < 24 ? (lane - 8) / 2 : -1;
  long long t0, t1;
  // V1: full row step as in wavePgs (scaled sweeps), rows from registers (no LDS)
  double Arow = A[col];
  t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < SW; it++) {
    const double xs = xn;
    for (int idx = 0; idx < n; idx++) {
      if (!((order >> idx) & 1ull)) continue;
      double nx = r + diag * xs;
      nx = nx > hB ? hB : (nx < lB ? lB : nx);
      const double dx = rdl(nx - xs, idx);
      if (lane == idx) xn = nx;
      if ((bounding >> idx) & 1ull) {
        const double nxi = rdl(nx, idx);
        if (findex == idx) { hB = hi * nxi; lB = -hB; }
      }
      r -= (Arow * dummyAct) * dx;
    }
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[0] = (double)(t1 - t0) / (SW * n);
  // V2: no clamp
  t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < SW; it++) {
    const double xs = xn;
    for (int idx = 0; idx < n; idx++) {
      double nx = r + diag * xs;
      const double dx = rdl(nx - xs, idx);
      if (lane == idx) xn = nx;
      r -= (Arow * dummyAct) * dx;
    }
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[1] = (double)(t1 - t0) / (SW * n);
  // V3: clamp, no bounding branch, no order branch
  t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < SW; it++) {
    const double xs = xn;
    for (int idx = 0; idx < n; idx++) {
      double nx = r + diag * xs;
      nx = nx > hB ? hB : (nx < lB ? lB : nx);
      const double dx = rdl(nx - xs, idx);
      if (lane == idx) xn = nx;
      r -= (Arow * dummyAct) * dx;
    }
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[2] = (double)(t1 - t0) / (SW * n);
  // V4: V3 with fmin/fmax clamp
  t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < SW; it++) {
    const double xs = xn;
    for (int idx = 0; idx < n; idx++) {
      double nx = fmin(fmax(r + diag * xs, lB), hB);
      const double dx = rdl(nx - xs, idx);
      if (lane == idx) xn = nx;
      r -= (Arow * dummyAct) * dx;
    }
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[3] = (double)(t1 - t0) / (SW * n);
  // V5: V3 fully unrolled by 8 (no loop overhead)
  t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < SW; it++) {
    const double xs = xn;
#pragma unroll 8
    for (int idx = 0; idx < 24; idx++) {
      double nx = r + diag * xs;
      nx = nx > hB ? hB : (nx < lB ? lB : nx);
      const double dx = rdl(nx - xs, idx);
      if (lane == idx) xn = nx;
      r -= (Arow * dummyAct) * dx;
    }
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[4] = (double)(t1 - t0) / (SW * 24);
  // V6: only readlane chain: r -= A*rdl(r, idx)
  t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < SW; it++) {
    for (int idx = 0; idx < n; idx++) {
      const double dx = rdl(r, idx);
      r -= Arow * dx;
    }
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[5] = (double)(t1 - t0) / (SW * n);
  // V7: branch-free row: order folded into an SGPR lane mask, bounds updated every row
  const double dxsBase = 0.0;
  (void)dxsBase;
  t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < SW; it++) {
    const double xs = xn;
    const double dxs = diag * xs;
#pragma unroll 8
    for (int idx = 0; idx < 24; idx++) {
      const bool on = (order >> idx) & 1ull;
      double nx = r + dxs;
      const double t = nx < lB ? lB : nx;
      nx = nx > hB ? hB : t;
      double dx = rdl(nx - xs, idx);
      dx = on ? dx : 0.0;
      if (on && lane == idx) xn = nx;
      const double nxi = rdl(nx, idx);
      const bool fm = findex == idx;
      const double hn = hi * nxi;
      hB = fm ? hn : hB;
      lB = fm ? -hn : lB;
      r -= (Arow * dummyAct) * dx;
    }
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[6] = (double)(t1 - t0) / (SW * 24);
  // V8: unrolled, branch on bounding only
  t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < SW; it++) {
    const double xs = xn;
    const double dxs = diag * xs;
#pragma unroll 8
    for (int idx = 0; idx < 24; idx++) {
      const bool on = (order >> idx) & 1ull;
      double nx = r + dxs;
      const double t = nx < lB ? lB : nx;
      nx = nx > hB ? hB : t;
      double dx = rdl(nx - xs, idx);
      dx = on ? dx : 0.0;
      if (on && lane == idx) xn = nx;
      if ((bounding >> idx) & 1ull) {
        const double nxi = rdl(nx, idx);
        if (findex == idx) { hB = hi * nxi; lB = -hB; }
      }
      r -= (Arow * dummyAct) * dx;
    }
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[7] = (double)(t1 - t0) / (SW * 24);
  // V9: contact-layout row (as wavePgs fast path): box from the last normal's x (SGPR)
  const unsigned long long normals = 0x249249ull;
  const double lo = -hi;
  double xN = 0.0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < SW; it++) {
    const double xs = xn;
    for (int i0 = 0; i0 < n; i0 += 4) {
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int idx = i0 + u;
        if (idx < n) {
          double h = hi, l = lo;
          if (!((normals >> idx) & 1ull)) { h = hi * xN; l = lo * xN; }
          double nx = r + diag * xs;
          const double t = nx < l ? l : nx;
          nx = nx > h ? h : t;
          const double dx = rdl(nx - xs, idx);
          if ((normals >> idx) & 1ull) xN = rdl(nx, idx);
          if (lane == idx) xn = nx;
          r -= (Arow * dummyAct) * dx;
        }
      }
    }
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[8] = (double)(t1 - t0) / (SW * n);
  out[16 + lane] = r + xn + hB + lB + xN;
}

int main() {
  double* d; double* A;
  hipMalloc(&d, 128 * sizeof(double));
  hipMalloc(&A, 24 * 24 * sizeof(double));
  double h[576];
  for (int i = 0; i < 576; i++) h[i] = 1e-3 * ((i * 37) % 17);
  hipMemcpy(A, h, sizeof(h), hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, A, 24, 0x249249ull, 0xFFFFFFull);
    hipDeviceSynchronize();
  }
  hipMemcpy(h, d, 16 * sizeof(double), hipMemcpyDeviceToHost);
  const char* nm[] = {"full row", "no clamp", "clamp, no branches", "fmin/fmax clamp", "unrolled x8", "readlane chain",
                      "branch-free", "unrolled, bounding br", "contact layout"};
  for (int i = 0; i < 9; i++) printf("%-22s %8.1f clk/row\n", nm[i], h[i]);
  return 0;
}
