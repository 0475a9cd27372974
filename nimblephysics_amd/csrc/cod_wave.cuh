// Complete orthogonal decomposition (column-pivoted Householder QR + RZ)
// of a small LDS matrix, lane-parallel over one 64-lane wave.
#pragma once
#include "wave.cuh"
#ifndef WAVE
#define WAVE 64
#endif

// ---------------------------------------------------------------------------
// Complete orthogonal decomposition (Eigen::CompleteOrthogonalDecomposition,
// used by the reference for Q^+ b at ConstrainedGroupGradientMatrices.cpp:270
// and BackpropSnapshot.cpp:2747): column-pivoted Householder QR, rank =
// #{|R_kk| > eps * min(m,n) * max|R_kk|}, then RZ on the leading r rows.
// Factorisation is lane-parallel over columns / rows; solves are per lane.
// A is m x n with leading dimension ld; reflectors are stored in place.
// ---------------------------------------------------------------------------
struct Cod {
  double* A;
  int m, n, ld, kmax;
  int* perm;        // n
  double* vd;       // kmax  QR reflector heads
  double* vn;       // kmax  QR reflector norms (<= 0: skipped)
  double* zd;       // m     RZ reflector heads
  double* zn;       // m     RZ reflector norms
  int* rank;        // 1
};

// carve a Cod workspace from `w` (needs 6*max(m,n) + 8 doubles + the v vector)
__device__ inline double* carveCod(double* w, double* A, int m, int n, int ld, Cod& c) {
  const int mx = m > n ? m : n;
  c.A = A; c.m = m; c.n = n; c.ld = ld; c.kmax = m < n ? m : n;
  c.vd = w; w += mx;
  c.vn = w; w += mx;
  c.zd = w; w += mx;
  c.zn = w; w += mx;
  c.perm = reinterpret_cast<int*>(w); w += (mx + 1) / 2 + 1;
  c.rank = reinterpret_cast<int*>(w); w += 2;
  return w;
}

// Lane-parallel factorisation: column norms live in registers (lane j =
// column j), the pivot is a wave arg-max (first index among equal maxima, as
// the sequential scan), alpha and |v|^2 are wave reductions, and the
// reflector pass (lane = column) also recomputes the next step's partial
// column norms (same sums as a fresh recomputation).  Requires n <= 64.
// Factorises the m x n matrix A (leading dimension ld) in place; ws is the
// carveCod workspace, v a further m doubles of scratch.
template <bool kLds>
__device__ void codFactor(typename Space<kLds>::dptr Ain, typename Space<kLds>::dptr wsIn, int m_, int n_, int ld_,
                          typename Space<kLds>::dptr vIn, int lane, double* prof = nullptr) {
#ifdef NIMBLE_STAGE_TIMING
  const long long tc0 = (long long)__builtin_amdgcn_s_memtime();
#else
  (void)prof;
#endif
  Cod c;
  carveCod((double*)wsIn, (double*)Ain, uni(m_), uni(n_), uni(ld_), c);
  double* v = (double*)vIn;
  double* A = c.A;
  const int m = c.m, n = c.n, ld = c.ld;
  if (lane < n) c.perm[lane] = lane;
  double norm = 0.0;  // partial norm of column `lane` over rows >= k
  if (lane < n) {
#pragma unroll 8
    for (int i = 0; i < m; i++) norm += A[i * ld + lane] * A[i * ld + lane];
  }
  WSYNC();
  double maxPivot = 0.0;
  for (int k = 0; k < c.kmax; k++) {
    // pivot: largest remaining norm, lowest index on ties
    const double cand = (lane >= k && lane < n) ? norm : -1.0;
    const double best = -waveMin(-cand);
    const int p = waveFirst(lane >= k && lane < n && cand == best);
    if (p != k) {
      for (int i = lane; i < m; i += WAVE) {
        const double t = A[i * ld + k]; A[i * ld + k] = A[i * ld + p]; A[i * ld + p] = t;
      }
      const double nk = rdl(norm, k), np = rdl(norm, p);
      if (lane == k) norm = np;
      else if (lane == p) norm = nk;
      if (lane == 0) { int t = c.perm[k]; c.perm[k] = c.perm[p]; c.perm[p] = t; }
    }
    WSYNC();
    const double akk = A[k * ld + k];
    const double colv = (lane >= k && lane < m) ? A[lane * ld + k] : 0.0;
    double alpha = sqrt(waveSum(colv * colv));
    if (alpha == 0.0) {
      if (lane == 0) c.vn[k] = -1.0;
      // fresh norms of the remaining columns over rows >= k+1
      if (lane > k && lane < n) {
        double nrm = 0.0;
#pragma unroll 8
        for (int i = k + 1; i < m; i++) nrm += A[i * ld + lane] * A[i * ld + lane];
        norm = nrm;
      }
      WSYNC();
      continue;
    }
    if (akk > 0) alpha = -alpha;
    const double vi = (lane == k) ? colv - alpha : colv;
    if (lane >= k && lane < m) v[lane] = vi;
    const double vnorm = waveSum(vi * vi);
    WSYNC();
    if (lane >= k && lane < n) {
      double nrm = 0.0;
      if (vnorm > 0) {
        double sc = 0;
#pragma unroll 8
        for (int i = k; i < m; i++) sc += v[i] * A[i * ld + lane];
        sc = 2 * sc / vnorm;
#pragma unroll 8
        for (int i = k; i < m; i++) {
          const double a = A[i * ld + lane] - sc * v[i];
          A[i * ld + lane] = a;
          if (i > k) nrm += a * a;
        }
      } else {
#pragma unroll 8
        for (int i = k + 1; i < m; i++) nrm += A[i * ld + lane] * A[i * ld + lane];
      }
      norm = nrm;
    }
    WSYNC();
    maxPivot = fmax(maxPivot, fabs(A[k * ld + k]));
    if (lane > k && lane < m) A[lane * ld + k] = v[lane];
    if (lane == 0) { c.vd[k] = v[k]; c.vn[k] = vnorm; }
    WSYNC();
  }
#ifdef NIMBLE_STAGE_TIMING
  const long long tc1 = (long long)__builtin_amdgcn_s_memtime();
#endif
  const double thr = 2.220446049250313e-16 * c.kmax * maxPivot;
  int r = 0;
  for (int k = 0; k < c.kmax; k++)
    if (fabs(A[k * ld + k]) > thr) r++;
  r = uni(r);
  if (lane == 0) *c.rank = r;
  // RZ: reflect row i over columns {i} U {r..n-1}; row i's trailing part is
  // kept as the reflector
  for (int i = r - 1; i >= 0 && r < n; i--) {
    const double aii = unid(A[i * ld + i]);
    const double tj = (lane >= r && lane < n) ? A[i * ld + lane] : 0.0;
    const double tail = waveSum(tj * tj);
    double al = sqrt(aii * aii + tail);
    if (aii > 0) al = -al;
    const double vi = aii - al;
    const double vnz = vi * vi + tail;
    WSYNC();
    if (lane == 0) { c.zd[i] = vi; c.zn[i] = vnz; }
    if (vnz != 0) {
      for (int row = lane; row <= i; row += WAVE) {
        double sc = A[row * ld + i] * vi;
#pragma unroll 4
        for (int j = r; j < n; j++) sc += A[row * ld + j] * A[i * ld + j];
        sc = 2 * sc / vnz;
        A[row * ld + i] -= sc * vi;
        if (row < i)
#pragma unroll 4
          for (int j = r; j < n; j++) A[row * ld + j] -= sc * A[i * ld + j];
      }
    }
    WSYNC();
  }
  WSYNC();
#ifdef NIMBLE_STAGE_TIMING
  if (prof && lane == 0) {
    prof[0] += (double)(tc1 - tc0);
    prof[1] += (double)((long long)__builtin_amdgcn_s_memtime() - tc1);
    prof[2] = r;
  }
#endif
}
