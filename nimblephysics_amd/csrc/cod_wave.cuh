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

// Register-resident column-pivoted QR for m <= R rows: lane j keeps column
// j in R registers for the whole factorisation.  Columns never move between
// lanes; each lane carries its column's current slot `pos` instead, so a
// pivot swap is two slot exchanges rather than a column copy, and ties go to
// the lowest slot, as in the sequential scan.  Per step the pivot lane
// stages its column in `vb` (LDS, >= R doubles), every lane reads it back
// as the Householder vector (broadcast reads), and the reflector application
// and the next step's partial norms are unpredicated per-lane FMA chains
// (inactive lanes scale by 0).  alpha = sqrt(partial norm of the pivot
// column), which the previous step recomputed over rows >= k.  The pivot
// column is final after its step and is written to slot k of A right away
// (R part by the pivot lane, reflector tail lane-parallel), so A ends in
// the layout of the LDS factorisation, with perm / vd / vn.  Cost per step:
// ~4R dependent-free VALU ops per lane plus two LDS round trips, instead of
// 2(m-k) LDS round trips.
#ifdef NIMBLE_COD_PROFILE
// per-phase clocks of codQrRegs, 8 per workgroup (tools/micro/cod_bench.hip
// only): 0 pivot search + slot swap, 1 pivot-column broadcast + reflector
// head, 2 reflector application + next partial norms, 3 write-back
__device__ double* g_codProf;
#define COD_PROF_BEGIN long long codT_ = (long long)__builtin_amdgcn_s_memtime()
#define COD_PROF(k)                                                                    \
  do {                                                                                 \
    const long long t_ = (long long)__builtin_amdgcn_s_memtime();                     \
    if (lane == 0) g_codProf[blockIdx.x * 8 + (k)] += (double)(t_ - codT_);            \
    codT_ = t_;                                                                        \
  } while (0)
#else
#define COD_PROF_BEGIN do { } while (0)
#define COD_PROF(k) do { } while (0)
#endif

template <bool kLds, int R>
__device__ void codQrRegs(typename Space<kLds>::dptr A, Cod& c, typename Space<kLds>::dptr vb, int lane) {
  const int m = c.m, n = c.n, ld = c.ld;
  const bool col = lane < n;
  const int cl = col ? lane : 0;
  double a[R];
#pragma unroll
  for (int i = 0; i < R; i++) {
    double v = A[(i < m ? i : 0) * ld + cl];
    a[i] = (col && i < m) ? v : 0.0;
  }
  double norm = 0.0;
#pragma unroll
  for (int i = 0; i < R; i++) norm += a[i] * a[i];
  int pos = lane;
  WSYNC();  // every column is in registers: A may now be overwritten
  COD_PROF_BEGIN;
  for (int k = 0; k < c.kmax; k++) {
    const bool cand = col && pos >= k;
    const double best = -waveMin(cand ? -norm : 1.0);
    const unsigned long long tie = __ballot(cand && norm == best);
    int pl = __ffsll((long long)tie) - 1;
    if (__popcll(tie) > 1) {
      // lowest slot among equal maxima
      const int ps = (int)waveMin((tie >> lane) & 1ull ? (double)pos : 1e9);
      pl = waveFirst(((tie >> lane) & 1ull) && pos == ps);
    }
    const int ppos = rdli(pos, pl);
    if (ppos != k) {
      const int q = waveFirst(col && pos == k);
      if (lane == q) pos = ppos;
      if (lane == pl) pos = k;
    }
    COD_PROF(0);
    if (lane == pl) {
#pragma unroll
      for (int i = 0; i < R; i++) vb[i] = a[i];
    }
    WSYNC();
    if (best == 0.0) {
      // zero column: no reflector; the column stays, fresh partial norms
      // over rows >= k+1
      if (lane == 0) c.vn[k] = -1.0;
      if (lane < m) A[lane * ld + k] = vb[lane];
      double nrm = 0.0;
#pragma unroll
      for (int i = 0; i < R; i++) {
        const double t = i > k ? a[i] : 0.0;
        nrm += t * t;
      }
      norm = nrm;
      WSYNC();
      continue;
    }
    const double akk = vb[k];
    double alpha = sqrt(best);
    if (akk > 0) alpha = -alpha;
    const double vk = akk - alpha;
    WSYNC();
    if (lane <= k) vb[lane] = lane == k ? vk : 0.0;
    WSYNC();
    double v[R];
#pragma unroll
    for (int i = 0; i < R; i++) v[i] = vb[i];
    COD_PROF(1);
    double vn0 = 0.0, vn1 = 0.0, sc0 = 0.0, sc1 = 0.0;
#pragma unroll
    for (int i = 0; i < R; i += 2) {
      vn0 += v[i] * v[i];
      sc0 += v[i] * a[i];
      if (i + 1 < R) { vn1 += v[i + 1] * v[i + 1]; sc1 += v[i + 1] * a[i + 1]; }
    }
    const double vnorm = unid(vn0 + vn1);
    const bool act = col && pos >= k;
    const double sc = act && vnorm > 0 ? 2 * (sc0 + sc1) / vnorm : 0.0;
    double nrm = 0.0;
#pragma unroll
    for (int i = 0; i < R; i++) {
      a[i] -= sc * v[i];
      const double t = i > k ? a[i] : 0.0;
      nrm += t * t;
    }
    norm = nrm;
    COD_PROF(2);
    // slot k is final: R part from the pivot lane, reflector tail below.
    // The pivot lane stores its whole column, unconditionally (a uniform
    // condition per element had become a branch per element): the rows it
    // does not own (> k, or past m) go to one sink, the RZ pass's reflector
    // heads, which nothing reads before that pass writes them
    if (lane == pl) {
      const auto sink = sp<kLds>(c.zd);
#pragma unroll
      for (int i = 0; i < R; i++) {
        auto dst = i <= k && i < m ? &A[i * ld + k] : sink;
        *dst = a[i];
      }
    }
    if (lane > k && lane < m) A[lane * ld + k] = vb[lane];
    if (lane == 0) { c.vd[k] = vk; c.vn[k] = vnorm; }
    WSYNC();
    COD_PROF(3);
  }
  if (col) {
    if (pos >= c.kmax) {
#pragma unroll
      for (int i = 0; i < R; i++)
        if (i < m) A[i * ld + pos] = a[i];
    }
    c.perm[pos] = lane;
  }
}

// Lane-parallel factorisation: column norms live in registers (column j on
// lane j & 63, slot j >> 6; R = 2 for the 65..128-column clamping sets), the
// pivot is a wave arg-max (first index among equal maxima, as the sequential
// scan), alpha and |v|^2 are wave reductions, and the reflector pass (lane =
// column) also recomputes the next step's partial column norms (same sums as
// a fresh recomputation).  Factorises the m x n matrix A (leading dimension
// ld, n <= 64 R) in place; ws is the carveCod workspace, v a further m
// doubles of scratch.  Inlined into its callers: as a called function its
// prologue saved 44 callee-saved VGPRs to per-lane scratch on every call
// (forward writes 29.1 -> 24.6 KB/world measured, WRITE_SIZE).
template <bool kLds, int R>
__device__ __forceinline__ void codFactorR(typename Space<kLds>::dptr Ain, typename Space<kLds>::dptr wsIn, int m_, int n_, int ld_,
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
  double maxPivot = 0.0;
  // the step the rank-revealing stop ended the QR at (kmax: no stop); the
  // diagonal past it is unreduced and not R's, so the rank count below
  // does not read it
  int stopK = c.kmax;
#ifndef NIMBLE_COD_LDS_ONLY
  if (m <= 24 && n <= 64) {
    WSYNC();
    codQrRegs<kLds, 24>(Ain, c, vIn, lane);
    WSYNC();
    goto rankAndRz;
  }
#endif
  {
  double norm[R];  // partial norm of column `row` over rows >= k
#pragma unroll
  for (int s = 0; s < R; s++) {
    const int j = rowAt(s, lane);
    norm[s] = 0.0;
    if (j < n) {
      c.perm[j] = j;
#pragma unroll 8
      for (int i = 0; i < m; i++) norm[s] += A[i * ld + j] * A[i * ld + j];
    }
  }
  WSYNC();
  COD_PROF_BEGIN;
  // Rank-revealing stop: the pivot's partial norm is |R_kk| and, with column
  // pivoting, bounds every later |R_jj|; once it is within the rank threshold
  // (eps kmax max|R_jj|, the rule below) the rank is k, and the remaining
  // steps would only rotate rows >= k, which the rank-k solves and the RZ
  // pass never read (their reflectors are marked skipped).  The clamping
  // sets of the flat-foot mesh worlds have rank <= the 33 dofs at 93-99
  // rows: most of the factorisation was these steps.
  double maxPiv = 0.0;
  for (int k = 0; k < c.kmax; k++) {
    // pivot: largest remaining norm, lowest index on ties
    double cand[R], neg[R];
#pragma unroll
    for (int s = 0; s < R; s++) {
      const int j = rowAt(s, lane);
      cand[s] = (j >= k && j < n) ? norm[s] : -1.0;
      neg[s] = -cand[s];
    }
    const double best = -waveMinR(neg);
    {
      const double piv = sqrt(best > 0.0 ? best : 0.0);
      if (k > 0 && piv <= 2.220446049250313e-16 * c.kmax * maxPiv) {
        for (int kk = k + lane; kk < c.kmax; kk += WAVE) c.vn[kk] = -1.0;
        WSYNC();
        stopK = k;
        break;
      }
      maxPiv = piv > maxPiv ? piv : maxPiv;
    }
    bool isBest[R];
#pragma unroll
    for (int s = 0; s < R; s++) isBest[s] = rowAt(s, lane) >= k && rowAt(s, lane) < n && cand[s] == best;
    const int p = waveFirstR(isBest);
    if (p != k) {
      for (int i = lane; i < m; i += WAVE) {
        const double t = A[i * ld + k]; A[i * ld + k] = A[i * ld + p]; A[i * ld + p] = t;
      }
      const double nk = rdlR(norm, k), np = rdlR(norm, p);
      setR(norm, k, lane, np);
      setR(norm, p, lane, nk);
      if (lane == 0) { int t = c.perm[k]; c.perm[k] = c.perm[p]; c.perm[p] = t; }
    }
    WSYNC();
    COD_PROF(0);
    const double akk = A[k * ld + k];
    double colv[R], sq[R];
#pragma unroll
    for (int s = 0; s < R; s++) {
      const int i = rowAt(s, lane);
      colv[s] = (i >= k && i < m) ? A[i * ld + k] : 0.0;
      sq[s] = colv[s] * colv[s];
    }
    double alpha = sqrt(waveSumR(sq));
    if (alpha == 0.0) {
      if (lane == 0) c.vn[k] = -1.0;
      // fresh norms of the remaining columns over rows >= k+1
#pragma unroll
      for (int s = 0; s < R; s++) {
        const int j = rowAt(s, lane);
        if (j > k && j < n) {
          double nrm = 0.0;
#pragma unroll 8
          for (int i = k + 1; i < m; i++) nrm += A[i * ld + j] * A[i * ld + j];
          norm[s] = nrm;
        }
      }
      WSYNC();
      continue;
    }
    if (akk > 0) alpha = -alpha;
    double vi[R];
#pragma unroll
    for (int s = 0; s < R; s++) {
      const int i = rowAt(s, lane);
      vi[s] = (i == k) ? colv[s] - alpha : colv[s];
      if (i >= k && i < m) v[i] = vi[s];
      sq[s] = vi[s] * vi[s];
    }
    const double vnorm = waveSumR(sq);
    WSYNC();
    COD_PROF(1);
    if (R == 2 && vnorm > 0 && n > WAVE) {
      // both slots in one pass over the rows: two independent dot / norm
      // chains per lane, the same operations per column in the same order as
      // the slot loop below (the same factor bit for bit).  An inactive slot
      // (a factored column, or past n) reads column k and stores into a
      // per-lane sink -- the RZ reflector heads, not written before the RZ
      // pass -- so no store is predicated (n > 64: zd holds > 64; with fewer
      // columns the second slot is idle and the slot loop below skips it).  Row
      // k is peeled off: it is updated but not part of the next step's norms.
      const int j0 = lane, j1 = lane + WAVE;
      const bool a0 = j0 >= k && j0 < n, a1 = j1 >= k && j1 < n;
      const int c0 = a0 ? j0 : k, c1 = a1 ? j1 : k;
      double* const sink = c.zd + lane;
      // (the store address of row i: the column's element or the sink)
      auto at0 = [&](int i) { return a0 ? A + i * ld + c0 : sink; };
      auto at1 = [&](int i) { return a1 ? A + i * ld + c1 : sink; };
      double s0 = 0, s1 = 0;
      int i = k;
      for (; i + 8 <= m; i += 8) {
        double x0[8], x1[8], vv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) { vv[u] = v[i + u]; x0[u] = A[(i + u) * ld + c0]; x1[u] = A[(i + u) * ld + c1]; }
#pragma unroll
        for (int u = 0; u < 8; u++) { s0 += vv[u] * x0[u]; s1 += vv[u] * x1[u]; }
      }
      for (; i < m; i++) { const double vi = v[i]; s0 += vi * A[i * ld + c0]; s1 += vi * A[i * ld + c1]; }
      COD_PROF(4);
      s0 = 2 * s0 / vnorm;
      s1 = 2 * s1 / vnorm;
      {
        const double vk = v[k];
        double x0 = A[k * ld + c0], x1 = A[k * ld + c1];
        asm volatile("" : "+v"(x0), "+v"(x1));
        *at0(k) = x0 - s0 * vk;
        *at1(k) = x1 - s1 * vk;
      }
      double n0 = 0.0, n1 = 0.0;
      i = k + 1;
      for (; i + 8 <= m; i += 8) {
        double x0[8], x1[8], vv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) { vv[u] = v[i + u]; x0[u] = A[(i + u) * ld + c0]; x1[u] = A[(i + u) * ld + c1]; }
#pragma unroll
        for (int u = 0; u < 8; u++) asm volatile("" : "+v"(x0[u]), "+v"(x1[u]), "+v"(vv[u]));
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const double b0 = x0[u] - s0 * vv[u];
          const double b1 = x1[u] - s1 * vv[u];
          *at0(i + u) = b0;
          *at1(i + u) = b1;
          n0 += b0 * b0;
          n1 += b1 * b1;
        }
      }
      for (; i < m; i++) {
        const double vi = v[i];
        double x0 = A[i * ld + c0], x1 = A[i * ld + c1];
        asm volatile("" : "+v"(x0), "+v"(x1));
        const double b0 = x0 - s0 * vi;
        const double b1 = x1 - s1 * vi;
        *at0(i) = b0;
        *at1(i) = b1;
        n0 += b0 * b0;
        n1 += b1 * b1;
      }
      if (a0) norm[0] = n0;
      if (a1) norm[R - 1] = n1;
    } else
#pragma unroll
    for (int s = 0; s < R; s++) {
      const int j = rowAt(s, lane);
      if (j >= k && j < n) {
        double nrm = 0.0;
        if (vnorm > 0) {
          double sc = 0;
#pragma unroll 8
          for (int i = k; i < m; i++) sc += v[i] * A[i * ld + j];
          sc = 2 * sc / vnorm;
          // eight rows' loads before their stores (A and v may alias for the
          // compiler: element by element, every load would wait for the
          // previous store); same operations in the same order
          int i = k;
          for (; i + 8 <= m; i += 8) {
            double av[8], vv[8];
#pragma unroll
            for (int u = 0; u < 8; u++) { av[u] = A[(i + u) * ld + j]; vv[u] = v[i + u]; }
#pragma unroll
            for (int u = 0; u < 8; u++) asm volatile("" : "+v"(av[u]), "+v"(vv[u]));
#pragma unroll
            for (int u = 0; u < 8; u++) {
              const double a = av[u] - sc * vv[u];
              A[(i + u) * ld + j] = a;
              const double t = i + u > k ? a : 0.0;  // (adds +0: the same sum)
              nrm += t * t;
            }
          }
          for (; i < m; i++) {
            const double a = A[i * ld + j] - sc * v[i];
            A[i * ld + j] = a;
            if (i > k) nrm += a * a;
          }
        } else {
#pragma unroll 8
          for (int i = k + 1; i < m; i++) nrm += A[i * ld + j] * A[i * ld + j];
        }
        norm[s] = nrm;
      }
    }
    WSYNC();
    COD_PROF(2);
    for (int i = lane; i < m; i += WAVE)
      if (i > k) A[i * ld + k] = v[i];
    if (lane == 0) { c.vd[k] = v[k]; c.vn[k] = vnorm; }
    WSYNC();
    COD_PROF(3);
  }
  }
rankAndRz:
#ifdef NIMBLE_STAGE_TIMING
  const long long tc1 = (long long)__builtin_amdgcn_s_memtime();
#endif
  // max |R_kk| and rank = #{|R_kk| > eps * kmax * max|R_kk|}, row k = R_kk
  double dkk[R], ndkk[R];
#pragma unroll
  for (int s = 0; s < R; s++) {
    const int k = rowAt(s, lane);
    dkk[s] = k < stopK ? fabs(A[k * ld + k]) : 0.0;
    ndkk[s] = -dkk[s];
  }
  maxPivot = -waveMinR(ndkk);
  const double thr = 2.220446049250313e-16 * c.kmax * maxPivot;
  int r = 0;
#pragma unroll
  for (int s = 0; s < R; s++) r += __popcll(__ballot(rowAt(s, lane) < c.kmax && dkk[s] > thr));
  if (lane == 0) *c.rank = r;
  // RZ: reflect row i over columns {i} U {r..n-1}; row i's trailing part is
  // kept as the reflector
  for (int i = r - 1; i >= 0 && r < n; i--) {
    const double aii = unid(A[i * ld + i]);
    double tj[R];
#pragma unroll
    for (int s = 0; s < R; s++) {
      const int j = rowAt(s, lane);
      const double t = (j >= r && j < n) ? A[i * ld + j] : 0.0;
      tj[s] = t * t;
    }
    const double tail = waveSumR(tj);
    double al = sqrt(aii * aii + tail);
    if (aii > 0) al = -al;
    const double vi = aii - al;
    const double vnz = vi * vi + tail;
    WSYNC();
    if (lane == 0) { c.zd[i] = vi; c.zn[i] = vnz; }
    if (vnz != 0) {
      for (int row = lane; row <= i; row += WAVE) {
        double sc = A[row * ld + i] * vi;
        // blocks of 4: the eight loads issued before the multiply-adds
        int j = r;
        for (; j + 4 <= n; j += 4) {
          double a[4], c[4];
#pragma unroll
          for (int u = 0; u < 4; u++) { a[u] = A[row * ld + j + u]; c[u] = A[i * ld + j + u]; }
#pragma unroll
          for (int u = 0; u < 4; u++) asm volatile("" : "+v"(a[u]), "+v"(c[u]));
#pragma unroll
          for (int u = 0; u < 4; u++) sc += a[u] * c[u];
        }
        for (; j < n; j++) sc += A[row * ld + j] * A[i * ld + j];
        sc = 2 * sc / vnz;
        A[row * ld + i] -= sc * vi;
        if (row < i) {
          // blocks of 4 as above: the loads before the stores (A's two rows
          // may alias for the compiler: element by element, every load would
          // wait for the previous store); the same update per element
          int j = r;
          for (; j + 4 <= n; j += 4) {
            double a[4], c[4];
#pragma unroll
            for (int u = 0; u < 4; u++) { a[u] = A[row * ld + j + u]; c[u] = A[i * ld + j + u]; }
#pragma unroll
            for (int u = 0; u < 4; u++) asm volatile("" : "+v"(a[u]), "+v"(c[u]));
#pragma unroll
            for (int u = 0; u < 4; u++) A[row * ld + j + u] = a[u] - sc * c[u];
          }
          for (; j < n; j++) A[row * ld + j] -= sc * A[i * ld + j];
        }
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

template <bool kLds>
__device__ void codFactor(typename Space<kLds>::dptr Ain, typename Space<kLds>::dptr wsIn, int m_, int n_, int ld_,
                          typename Space<kLds>::dptr vIn, int lane, double* prof = nullptr) {
  codFactorR<kLds, 1>(Ain, wsIn, m_, n_, ld_, vIn, lane, prof);
}
