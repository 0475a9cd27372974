// Cholesky factorisation M = L L^T of the packed lower triangle of the
// joint-space mass matrix and the solves with it, one world per 64-lane
// wave (lane i = row i).  Used by the forward (ddq, impulses) and the
// backward (Minv products); stands in for the reference's articulated-body
// forward dynamics (dart/dynamics/Skeleton.cpp:13034) with the same result.
#pragma once
#include "spatial.cuh"
#include "wave.cuh"
#ifndef WAVE
#define WAVE 64
#endif

// In-place Cholesky of the packed lower triangle at A (row i at i(i+1)/2):
// left-looking (Crout) with one lane per row, one barrier per column.  The
// per-element subtraction order (k ascending) is that of the right-looking
// factorisation.  A column's scale is 1/L_jj from the hardware reciprocal
// square root refined by two Newton steps (L_jj = a_jj / sqrt(a_jj) =
// a_jj * rsq), so the column costs one multiply per lane instead of a square
// root and two divisions on its critical path (tools/micro/chol_bench.hip:
// 49.7k -> 39.5k clocks for n = 33; the factor differs from the divided one
// in the last bits only).
__device__ __forceinline__ double rsqrtRefined(double a) {
  double y = __builtin_amdgcn_rsq(a);
  y = y * (1.5 - 0.5 * a * y * y);
  return y * (1.5 - 0.5 * a * y * y);
}
__device__ __forceinline__ void choleskyLds(double* A, double* dinv, int n, int lane) {
  for (int j = 0; j < n; j++) {
    double sum = 0.0;
    if (lane >= j && lane < n) {
      const int ri = tri(lane, 0), rj = tri(j, 0);
      sum = A[ri + j];
      // blocks of 8: the sixteen loads issued before the multiply-adds
      int k = 0;
      for (; k + 8 <= j; k += 8) {
        double a[8], c[8];
#pragma unroll
        for (int u = 0; u < 8; u++) { a[u] = A[ri + k + u]; c[u] = A[rj + k + u]; }
#pragma unroll
        for (int u = 0; u < 8; u++) asm volatile("" : "+v"(a[u]), "+v"(c[u]));
#pragma unroll
        for (int u = 0; u < 8; u++) sum -= a[u] * c[u];
      }
      for (; k < j; k++) sum -= A[ri + k] * A[rj + k];
    }
    const double ajj = rdl(sum, j);
    const double y = rsqrtRefined(ajj);
    if (lane == j) { A[tri(j, j)] = ajj * y; dinv[j] = y; }
    else if (lane > j && lane < n) A[tri(lane, j)] = sum * y;
    WSYNC();
  }
}

// (A register-resident variant -- row i in VGPRs of lane i, row j broadcast
// through LDS per column -- measured 3x slower inside the forward kernel:
// fully unrolled it costs instruction-cache misses, and its rows spill when
// inlined.  The LDS form above is the one used.)
__device__ __forceinline__ void cholesky(double* A, double* dinv, int n, int lane) { choleskyLds(A, dinv, n, lane); }

// Solve L L^T x = b for K right-hand sides at once, held in registers (row i
// on lane i): the K independent dependency chains interleave.  dinv[k] =
// 1 / L_kk.  The L entries and reciprocals of 8 steps are loaded ahead of
// their readlane -> FMA chain (LDS latency paid once per 8 steps).
template <int K>
__device__ __forceinline__ void cholSolveReg(const double* Lm, const double* dinv, double (&x)[K], int n, int lane) {
  for (int k = 0; k < n; k++) {
    const double dk = dinv[k];
    const double lk = (lane > k && lane < n) ? Lm[tri(lane, k)] : 0.0;
#pragma unroll
    for (int q = 0; q < K; q++) {
      const double xk = rdl(x[q], k) * dk;
      if (lane == k) x[q] = xk;
      else if (lane > k) x[q] -= lk * xk;
    }
  }
  for (int k = n - 1; k >= 0; k--) {
    const double dk = dinv[k];
    const double lk = lane < k ? Lm[tri(k, lane)] : 0.0;
#pragma unroll
    for (int q = 0; q < K; q++) {
      const double xk = rdl(x[q], k) * dk;
      if (lane == k) x[q] = xk;
      else if (lane < k) x[q] -= lk * xk;
    }
  }
}
// (Loading the L entries of 8 steps ahead of the readlane chain, as the
// Dantzig solves do, measured slower here: 19.8k -> 22.7k clocks for the
// 33-dof unconstrained solve.)

__device__ __forceinline__ void cholSolve(const double* Lm, const double* dinv, double* x, int n, int lane) {
  double xr[1] = {lane < n ? x[lane] : 0.0};
  cholSolveReg<1>(Lm, dinv, xr, n, lane);
  WSYNC();
  if (lane < n) x[lane] = xr[0];
  WSYNC();
}
