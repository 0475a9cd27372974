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
// factorisation.
__device__ __forceinline__ void choleskyLds(double* A, double* dinv, int n, int lane) {
  for (int j = 0; j < n; j++) {
    double sum = 0.0;
    if (lane >= j && lane < n) {
      const int ri = tri(lane, 0), rj = tri(j, 0);
      sum = A[ri + j];
#pragma unroll 8
      for (int k = 0; k < j; k++) sum -= A[ri + k] * A[rj + k];
    }
    const double djj = sqrt(rdl(sum, j));
    if (lane == j) { A[tri(j, j)] = djj; dinv[j] = 1.0 / djj; }
    else if (lane > j && lane < n) A[tri(lane, j)] = sum / djj;
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

__device__ __forceinline__ void cholSolve(const double* Lm, const double* dinv, double* x, int n, int lane) {
  double xr[1] = {lane < n ? x[lane] : 0.0};
  cholSolveReg<1>(Lm, dinv, xr, n, lane);
  WSYNC();
  if (lane < n) x[lane] = xr[0];
  WSYNC();
}
