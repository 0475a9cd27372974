// Wave-parallel LCP kernels for one world per 64-lane wave.  Vectors of the
// LCP live row-distributed in registers (row i on lane i & 63, slot i >> 6:
// R = 1 slot for <= 64 rows, R = 2 for the 65..128-row problems), matrices
// in LDS (or the world's HBM workspace);
// the sequential structure of the reference algorithms (pivot order, sweep
// order, tie-breaking) is kept exactly, only the inner vector work is spread
// over the lanes:
//   * wavePgs       PgsBoxedLcpSolver::solve (PgsBoxedLcpSolver.cpp:85)
//   * waveDantzig   dSolveLCP (dart/external/odelcpsolver/lcp.cpp:780) with
//                   _dLDLTAddTL / _dLDLTRemove (matrix.cpp:286, :374), early
//                   termination as the contact solver uses it
//   * waveLcpValid  LCPUtils::isLCPSolutionValid (LCPUtils.cpp:14)
//   * codSolveWave  COD min-norm solve on a codFactor()ed matrix
// All functions must be entered by the whole wave (uniform control flow).
// The *R templates take the row-distributed arrays; the scalar forms are
// their R = 1 instances.
#pragma once
#include <type_traits>
#include "wave.cuh"
#include "cod_wave.cuh"

#define LCP_INF __builtin_inf()

// optional per-phase clock accounting (tools/lcp_bench: -DLCP_PROFILE)
#ifdef LCP_PROFILE
#define LP_BEGIN() const long long lp0_ = (long long)__builtin_amdgcn_s_memtime()
#define LP_END(acc, k) (acc)[k] += (long long)__builtin_amdgcn_s_memtime() - lp0_
#else
#define LP_BEGIN() do { } while (0)
#define LP_END(acc, k) do { } while (0)
#endif

// ---------------------------------------------------------------------------
// Residual form: lane j keeps r_j = b_j - sum_k A_jk x_k; a sweep step on
// row i needs only r_i + A_ii x_i (= b_i - sum_{k!=i} A_ik x_k) on lane i,
// then every lane applies r_j -= A_ji * dx_i.  No cross-lane reduction on the
// critical path (the reference recomputes the row sum; results agree to
// rounding).  A is symmetric and read by rows (conflict-free LDS access);
// the reference's in-place row scaling (1/A_jj) is applied lane-locally,
// A_ji / A_jj = A_ij * dummy_j, so A is never written.
// `shift` is added to A's diagonal on the fly (A + cfm I without a copy);
// `cancel` (LDS int, optional) is polled after every sweep and ends the
// solve early with `false` when set.  With `ld` / `idx` the problem is the
// principal submatrix A[idx][idx] of a matrix with leading dimension ld
// (lane j holds idx_j), read in place (LCPUtils::removeFriction without a
// gathered copy).
//
// Contact-layout rows clamp with v_max_f64 / v_min_f64 (their box is never
// inverted: l = -h <= 0 <= h); for operands that are not NaN that is the
// reference's compare-and-assign chain, two dependent operations instead of
// six on the sweep's critical path.  A NaN anywhere leaves a non-finite
// residual behind (maxNum would otherwise swallow it), so a solve that ends
// with one is re-run from its inputs with the reference's chain (kExact).
// The box scale of a contact-layout row: 1 for a normal row, x_N (its
// normal's newest x) for a friction row, selected on the scalar unit, so the
// row's box is one multiply (hi * 1 = hi exactly) instead of a multiply, a
// per-lane select and the canonicalisation fmin / fmax need for a selected
// operand, all on the sweep's dependent chain.  (Opaque to the optimiser,
// which would otherwise fold x * (c ? 1 : y) back into c ? x : x * y.)
__device__ __forceinline__ double boxScale(bool normal, double xN) {
  double sc = normal ? 1.0 : xN;
  NIMBLE_OPAQUE_SGPR(sc);
  return sc;
}

template <bool kLds, bool kMapped, int R, bool kExact = false>
__device__ bool wavePgsR(int n, typename Space<kLds>::cdptr Ain, double (&x)[R], const double (&bIn)[R],
                         const double (&lo)[R], const double (&hi)[R], const int (&findex)[R], int lane,
                         double* dbg = nullptr, double shift = 0.0, const int* cancel = nullptr, int ld = -1,
                         const int* idxIn = nullptr, int* tally = nullptr) {
  n = uni(n);
  if (n == 0) return true;
  // executed work for the roofline (tally: LDS ints [1] sweeps, [2] FLOPs;
  // the residual set-up and every sweep are n rows of n multiply-adds plus
  // the row's clamp, ~12 operations)
  auto account = [&](int sweeps) {
    if (tally && lane == 0) {
      __hip_atomic_fetch_add(tally + 1, sweeps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_add(tally + 2, (sweeps + 1) * (2 * n * n + 12 * n), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  };
  double xEntry[R];
#pragma unroll
  for (int s = 0; s < R; s++) xEntry[s] = x[s];
  // (kExact = false) a non-finite residual or iterate: re-run exactly
  auto nonFinite = [&](const double (&rv)[R], const double (&xv)[R]) {
    bool bad = false;
#pragma unroll
    for (int s = 0; s < R; s++) bad = bad || (rowAt(s, lane) < n && !(isfinite(rv[s]) && isfinite(xv[s])));
    return __ballot(bad) != 0ull;
  };
  ld = kMapped ? uni(ld) : n;
  int idx[R];
  double b[R];
#pragma unroll
  for (int s = 0; s < R; s++) {
    idx[s] = kMapped ? idxIn[s] : rowAt(s, lane);
    b[s] = bIn[s];
  }
  const double* A = (const double*)Ain;
  const double deltaXThr = 1e-6, relTol = 1e-3, epsDiv = 1e-9;
#ifdef LCP_PROFILE
  const long long tp0 = (long long)__builtin_amdgcn_s_memtime();
#endif
  bool act[R];
  int col[R];
  double diagRaw[R];
  unsigned long long order[R];
  bool inOrder[R];
  const int idx0 = rdliR(idx, 0);
#pragma unroll
  for (int s = 0; s < R; s++) {
    act[s] = rowAt(s, lane) < n;
    col[s] = act[s] ? idx[s] : idx0;  // idle lanes read a valid address, use 0
    diagRaw[s] = act[s] ? A[col[s] * ld + col[s]] + shift : 1.0;
    order[s] = __ballot(act[s] && diagRaw[s] >= epsDiv);
    inOrder[s] = act[s] && ((order[s] >> lane) & 1ull);
  }
  // rows whose x bounds friction rows (their update refreshes those bounds)
  unsigned long long bounding[R];
#pragma unroll
  for (int s = 0; s < R; s++) bounding[s] = 0ull;
  for (int i = 0; i < n; i++) {
    bool hit = false;
#pragma unroll
    for (int s = 0; s < R; s++) hit = hit || findex[s] == i;
    if (__ballot(hit)) bounding[i >> 6] |= 1ull << (i & 63);
  }
  double r[R];
#pragma unroll
  for (int s = 0; s < R; s++) r[s] = act[s] ? b[s] : 0.0;
  for (int k = 0; k < n; k++) {
    const double xk = rdlR(x, k);
    const int rk = kMapped ? rdliR(idx, k) : k;
#pragma unroll
    for (int s = 0; s < R; s++) {
      const double a0 = A[rk * ld + col[s]];
      if (act[s]) r[s] -= (k == rowAt(s, lane) ? a0 + shift : a0) * xk;
    }
  }
  // Contact layout (the forward's rows: each contact is a normal row
  // followed by 0 or 2 friction rows with findex = that normal and
  // lo = -hi), every row in order: the friction box of row i is
  // +-hi_i * x_N with x_N the newest x of the last normal row, which the
  // sweep carries as one scalar -- no per-lane box registers.
  bool contactRows = true;
  unsigned long long normals[R];
#pragma unroll
  for (int s = 0; s < R; s++) {
    const int row = rowAt(s, lane);
    contactRows = contactRows && order[s] == __ballot(act[s]);
    const int f1 = gatherRi(findex, row > 0 ? row - 1 : 0), f2 = gatherRi(findex, row > 1 ? row - 2 : 0);
    const bool ok = !act[s] || findex[s] < 0 ||
                    (lo[s] == -hi[s] &&
                     ((findex[s] == row - 1 && f1 < 0) || (findex[s] == row - 2 && f1 == row - 2 && f2 < 0)));
    contactRows = contactRows && !__ballot(!ok);
    normals[s] = __ballot(act[s] && findex[s] < 0);
  }
  if (dbg && lane == 0) dbg[1] = contactRows ? 1 : 0;
#ifdef LCP_PROFILE
  const long long tp1 = (long long)__builtin_amdgcn_s_memtime();
#endif
  // current box of each row; friction rows track hi * x[findex]
  double hB[R], lB[R];
#pragma unroll
  for (int s = 0; s < R; s++) {
    hB[s] = hi[s];
    lB[s] = lo[s];
    const double xf = gatherR(x, findex[s] >= 0 ? findex[s] : 0);
    if (findex[s] >= 0) { hB[s] = hi[s] * xf; lB[s] = -hB[s]; }
  }
  // Each lane's x changes only at its own row of a sweep, so within a sweep
  // row i still holds its sweep-start value x0 when it is visited, and the
  // reference's per-row "moved" test can be evaluated for all rows at once
  // after the sweep (same operands, same outcome).  The row loop then
  // carries only clamp -> readlane -> residual update.  Rows of A
  // (symmetric, row i lane j = A_ji) are loaded one 4-row group ahead, so
  // the load latency is off the dependent chain.
  double x0[R], xn[R], act1[R];
#pragma unroll
  for (int s = 0; s < R; s++) {
    x0[s] = x[s];
    xn[s] = x[s];
    act1[s] = act[s] ? 1.0 : 0.0;
  }
  const int nLast = n - 1;
  auto rowAtI = [&](int i) { return kMapped ? rdliR(idx, i < n ? i : nLast) : (i < n ? i : nLast); };
  // (slot of row i: wave-uniform; with R = 1 always 0)
  auto pick = [&](const double (&v)[R], int i) -> double {
    if constexpr (R == 1) return v[0];
    else return (i >> 6) ? v[1] : v[0];
  };
  typedef double Grp[4][R];
  auto loadGroup = [&](Grp& G, int i0) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int ro = rowAtI(i0 + u) * ld;
#pragma unroll
      for (int s = 0; s < R; s++) G[u][s] = A[ro + col[s]];
    }
  };
  {
    auto row1 = [&](int i, const double (&cur)[R]) {
      const double rr = pick(r, i), xs0 = pick(x0, i), dg = pick(diagRaw, i);
      double nx = 0.0;
      if (bitR(order, i)) {
        const double hb = pick(hB, i), lb = pick(lB, i);
        nx = (rr + dg * xs0) / dg;
        nx = nx > hb ? hb : (nx < lb ? lb : nx);
      }
      const double dx = rdl(nx - xs0, i & 63);
      setR(xn, i, lane, nx);
      if (bitR(bounding, i)) {
        const double nxi = rdl(nx, i & 63);
#pragma unroll
        for (int s = 0; s < R; s++)
          if (findex[s] == i) { hB[s] = hi[s] * nxi; lB[s] = -hB[s]; }
      }
#pragma unroll
      for (int s = 0; s < R; s++) r[s] -= (cur[s] * act1[s]) * dx;
    };
    double xN = 0.0;
    // (the row kind is a scalar bit: the branch never waits on VALU results;
    // x_N is only consumed by VALU multiplies, never by SALU)
    auto row1c = [&](int i, const double (&cur)[R]) {
      const bool nrm = bitR(normals, i);
      const double sc = boxScale(nrm, xN);
      const double h = pick(hi, i) * sc, l = pick(lo, i) * sc;
      const double rr = pick(r, i), xs0 = pick(x0, i), dg = pick(diagRaw, i);
      double nx = (rr + dg * xs0) / dg;
      if constexpr (kExact) {
        const double t = nx < l ? l : nx;
        nx = nx > h ? h : t;
      } else {
        nx = fmin(fmax(nx, l), h);
      }
      const double dx = rdl(nx - xs0, i & 63);
      {
        // (unconditional readlane, scalar select: no branch per row)
        const double xi = rdl(nx, i & 63);
        xN = nrm ? xi : xN;
      }
      setR(xn, i, lane, nx);
#pragma unroll
      for (int s = 0; s < R; s++) r[s] -= (cur[s] * act1[s]) * dx;
    };
    Grp C, N;
    loadGroup(C, 0);
    if (contactRows) {
      int i0 = 0;
      for (; i0 + 4 <= n; i0 += 4) {
        loadGroup(N, i0 + 4);
        row1c(i0, C[0]);
        row1c(i0 + 1, C[1]);
        row1c(i0 + 2, C[2]);
        row1c(i0 + 3, C[3]);
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
          for (int s = 0; s < R; s++) C[u][s] = N[u][s];
      }
      if (i0 < n) {
        row1c(i0, C[0]);
        if (i0 + 1 < n) row1c(i0 + 1, C[1]);
        if (i0 + 2 < n) row1c(i0 + 2, C[2]);
      }
    } else {
      int i0 = 0;
      for (; i0 + 4 <= n; i0 += 4) {
        loadGroup(N, i0 + 4);
        row1(i0, C[0]);
        row1(i0 + 1, C[1]);
        row1(i0 + 2, C[2]);
        row1(i0 + 3, C[3]);
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
          for (int s = 0; s < R; s++) C[u][s] = N[u][s];
      }
      if (i0 < n) {
        row1(i0, C[0]);
        if (i0 + 1 < n) row1(i0 + 1, C[1]);
        if (i0 + 2 < n) row1(i0 + 2, C[2]);
      }
    }
    // the shift's share of the diagonal updates, deferred: a row's residual
    // is not read again before its own row in the next sweep
    if (shift != 0.0)
#pragma unroll
      for (int s = 0; s < R; s++)
        if (act[s]) r[s] -= shift * (xn[s] - x0[s]);
  }
#ifdef LCP_PROFILE
  const long long tp2 = (long long)__builtin_amdgcn_s_memtime();
  if (dbg && lane == 0) { dbg[2] = (double)(tp1 - tp0); dbg[3] = (double)(tp2 - tp1); }
#endif
  {
    bool moved = false;
#pragma unroll
    for (int s = 0; s < R; s++) moved = moved || (inOrder[s] && fabs(xn[s] - x0[s]) > deltaXThr);
    if (!__ballot(moved)) {
      if constexpr (!kExact) {
        if (contactRows && nonFinite(r, xn)) {
#pragma unroll
          for (int s = 0; s < R; s++) x[s] = xEntry[s];
          account(1);
          return wavePgsR<kLds, kMapped, R, true>(n, Ain, x, bIn, lo, hi, findex, lane, dbg, shift, cancel, ld, idxIn,
                                                  tally);
        }
      }
#pragma unroll
      for (int s = 0; s < R; s++) x[s] = xn[s];
      account(1);
      return true;
    }
  }
  // row scaling of the reference, lane-local: A'_jk = A_jk * dummy_j
  double diag[R], dummyAct[R];
#pragma unroll
  for (int s = 0; s < R; s++) {
    const double dummy = inOrder[s] ? 1.0 / diagRaw[s] : 1.0;
    if (inOrder[s]) { b[s] *= dummy; r[s] *= dummy; }
    diag[s] = inOrder[s] ? diagRaw[s] * dummy : diagRaw[s];
    dummyAct[s] = act[s] ? dummy : 0.0;
  }
  bool possible = false;
  int sweeps = 1;
  for (int iter = 1; iter < 30; iter++) {
    sweeps++;
    double xs[R];
#pragma unroll
    for (int s = 0; s < R; s++) xs[s] = xn[s];
    auto row = [&](int i, const double (&cur)[R]) {
      if (!bitR(order, i)) return;
      const double hb = pick(hB, i), lb = pick(lB, i);
      double nx = pick(r, i) + pick(diag, i) * pick(xs, i);
      nx = nx > hb ? hb : (nx < lb ? lb : nx);
      const double dx = rdl(nx - pick(xs, i), i & 63);
      setR(xn, i, lane, nx);
      if (bitR(bounding, i)) {
        const double nxi = rdl(nx, i & 63);
#pragma unroll
        for (int s = 0; s < R; s++)
          if (findex[s] == i) { hB[s] = hi[s] * nxi; lB[s] = -hB[s]; }
      }
#pragma unroll
      for (int s = 0; s < R; s++) r[s] -= (cur[s] * dummyAct[s]) * dx;
    };
    double xN = 0.0;
    auto rowc = [&](int i, const double (&cur)[R]) {
      const bool nrm = bitR(normals, i);
      const double sc = boxScale(nrm, xN);
      const double h = pick(hi, i) * sc, l = pick(lo, i) * sc;
      double nx = pick(r, i) + pick(diag, i) * pick(xs, i);
      if constexpr (kExact) {
        const double t = nx < l ? l : nx;
        nx = nx > h ? h : t;
      } else {
        nx = fmin(fmax(nx, l), h);
      }
      const double dx = rdl(nx - pick(xs, i), i & 63);
      {
        // (unconditional readlane, scalar select: no branch per row)
        const double xi = rdl(nx, i & 63);
        xN = nrm ? xi : xN;
      }
      setR(xn, i, lane, nx);
#pragma unroll
      for (int s = 0; s < R; s++) r[s] -= (cur[s] * dummyAct[s]) * dx;
    };
    Grp C, N;
    loadGroup(C, 0);
    // (full groups of four rows straight-line: a branch per row cost more
    // than the row; the last, partial group row by row)
    if (contactRows) {
      int i0 = 0;
      for (; i0 + 4 <= n; i0 += 4) {
        loadGroup(N, i0 + 4);
        rowc(i0, C[0]);
        rowc(i0 + 1, C[1]);
        rowc(i0 + 2, C[2]);
        rowc(i0 + 3, C[3]);
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
          for (int s = 0; s < R; s++) C[u][s] = N[u][s];
      }
      if (i0 < n) {
        rowc(i0, C[0]);
        if (i0 + 1 < n) rowc(i0 + 1, C[1]);
        if (i0 + 2 < n) rowc(i0 + 2, C[2]);
      }
    } else {
      int i0 = 0;
      for (; i0 + 4 <= n; i0 += 4) {
        loadGroup(N, i0 + 4);
        row(i0, C[0]);
        row(i0 + 1, C[1]);
        row(i0 + 2, C[2]);
        row(i0 + 3, C[3]);
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
          for (int s = 0; s < R; s++) C[u][s] = N[u][s];
      }
      if (i0 < n) {
        row(i0, C[0]);
        if (i0 + 1 < n) row(i0 + 1, C[1]);
        if (i0 + 2 < n) row(i0 + 2, C[2]);
      }
    }
    if (shift != 0.0)
#pragma unroll
      for (int s = 0; s < R; s++) r[s] -= (shift * dummyAct[s]) * (xn[s] - xs[s]);
    bool far = false;
#pragma unroll
    for (int s = 0; s < R; s++) far = far || (inOrder[s] && fabs(xn[s]) > epsDiv && fabs((xn[s] - xs[s]) / xn[s]) > relTol);
    possible = !__ballot(far);
    if (dbg && lane == 0) dbg[0] = iter;
    if (possible) break;
    if (cancel && uni(__hip_atomic_load(cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))) break;
  }
#ifdef LCP_PROFILE
  if (dbg && lane == 0) dbg[4] = (double)((long long)__builtin_amdgcn_s_memtime() - tp2);
#endif
  if constexpr (!kExact) {
    if (contactRows && nonFinite(r, xn)) {
#pragma unroll
      for (int s = 0; s < R; s++) x[s] = xEntry[s];
      account(sweeps);
      return wavePgsR<kLds, kMapped, R, true>(n, Ain, x, bIn, lo, hi, findex, lane, dbg, shift, cancel, ld, idxIn,
                                              tally);
    }
  }
#pragma unroll
  for (int s = 0; s < R; s++) x[s] = xn[s];
  account(sweeps);
  return possible;
}

// the one-row-per-lane form (rows <= 64)
template <bool kLds, bool kMapped = false>
__device__ bool wavePgs(int n, typename Space<kLds>::cdptr Ain, double& x, double b, double lo, double hi, int findex,
                        int lane, double* dbg = nullptr, double shift = 0.0, const int* cancel = nullptr, int ld = -1,
                        int idx = -1) {
  double xa[1] = {x};
  const double ba[1] = {b}, la[1] = {lo}, ha[1] = {hi};
  const int fa[1] = {findex}, ia[1] = {idx};
  const bool ok = wavePgsR<kLds, kMapped, 1>(n, Ain, xa, ba, la, ha, fa, lane, dbg, shift, cancel, ld, ia);
  x = xa[0];
  return ok;
}

// ---------------------------------------------------------------------------
template <bool kLds, int R>
__device__ bool waveLcpValidR(int m, typename Space<kLds>::cdptr Ain, double cfm, const double (&x)[R],
                              const double (&b)[R], const double (&hi)[R], const double (&lo)[R], const int (&fi)[R],
                              bool ignoreFriction, int lane) {
  m = uni(m);
  const double* A = (const double*)Ain;
  double v[R];
#pragma unroll
  for (int s = 0; s < R; s++) v[s] = -b[s];
#pragma unroll 4
  for (int j = 0; j < m; j++) {
    const double xj = rdlR(x, j);
#pragma unroll
    for (int s = 0; s < R; s++) {
      const int row = rowAt(s, lane);
      if (row < m) v[s] += (A[j * m + row] + (row == j ? cfm : 0.0)) * xj;  // A symmetric: row j
    }
  }
  bool bad = false;
#pragma unroll
  for (int s = 0; s < R; s++) {
    const double xf = gatherR(x, fi[s] >= 0 ? fi[s] : 0);
    if (rowAt(s, lane) < m) {
      bool ok = true;
      double up = hi[s], low = lo[s];
      bool done = false;
      if (fi[s] != -1) {
        if (ignoreFriction) { ok = (x[s] == 0); done = true; }
        up *= xf;
        low *= xf;
      }
      if (!done) {
        const double tol = 1e-5;
        if (fabs(low) < tol && fabs(up) < tol && fabs(x[s]) < tol) {
        } else if (fabs(x[s] - low) < tol) {
          if (v[s] < -tol) ok = false;
        } else if (fabs(x[s] - up) < tol) {
          if (v[s] > tol) ok = false;
        } else if (x[s] > low && x[s] < up) {
          if (fabs(v[s]) > tol) ok = false;
        } else {
          ok = false;
        }
      }
      bad = bad || !ok;
    }
  }
  return __ballot(bad) == 0ull;
}

template <bool kLds>
__device__ bool waveLcpValid(int m, typename Space<kLds>::cdptr Ain, double cfm, double x, double b, double hi,
                             double lo, int fi, bool ignoreFriction, int lane) {
  const double xa[1] = {x}, ba[1] = {b}, ha[1] = {hi}, la[1] = {lo};
  const int fa[1] = {fi};
  return waveLcpValidR<kLds, 1>(m, Ain, cfm, xa, ba, ha, la, fa, ignoreFriction, lane);
}

// ---------------------------------------------------------------------------
// x (row-distributed, length c.n) = min-norm least-squares solution for rhs
// (row-distributed, length c.m).  scr: >= n doubles.
// (A, ws, m, n, ld) as given to carveCod + codFactor
template <bool kLds, int R>
__device__ void codSolveWaveR(typename Space<kLds>::dptr Ain, typename Space<kLds>::dptr wsIn, int m_, int n_, int ld_,
                              const double (&rhsIn)[R], typename Space<kLds>::dptr scrIn, int lane, double (&out)[R]) {
  Cod c;
  carveCod((double*)wsIn, (double*)Ain, uni(m_), uni(n_), uni(ld_), c);
  double* scr = (double*)scrIn;
  const double* A = c.A;
  const int m = c.m, n = c.n, ld = c.ld;
  double rhs[R];
#pragma unroll
  for (int s = 0; s < R; s++) rhs[s] = rhsIn[s];
  for (int k = 0; k < c.kmax; k++) {
    const double vnorm = unid(c.vn[k]);
    if (!(vnorm > 0)) continue;
    const double vk = c.vd[k];
    double v[R], t[R];
#pragma unroll
    for (int s = 0; s < R; s++) {
      const int row = rowAt(s, lane);
      v[s] = row == k ? vk : ((row > k && row < m) ? A[row * ld + k] : 0.0);
      t[s] = v[s] * rhs[s];
    }
    double sc = waveSumR(t);
    sc = 2 * sc / vnorm;
#pragma unroll
    for (int s = 0; s < R; s++) {
      const int row = rowAt(s, lane);
      if (row >= k && row < m) rhs[s] -= sc * v[s];
    }
  }
  const int r = uni(*c.rank);
  double z[R], acc[R];
#pragma unroll
  for (int s = 0; s < R; s++) { z[s] = 0.0; acc[s] = 0.0; }
  for (int i = r - 1; i >= 0; i--) {
    const double zi = (rdlR(rhs, i) - rdlR(acc, i)) / A[i * ld + i];
    setR(z, i, lane, zi);
#pragma unroll
    for (int s = 0; s < R; s++) {
      const int row = rowAt(s, lane);
      if (row < i) acc[s] += A[row * ld + i] * zi;
    }
  }
  if (r < n) {
    for (int i = 0; i < r; i++) {
      const double vn = unid(c.zn[i]);
      if (vn == 0) continue;
      const double zd = c.zd[i];
      double t[R];
#pragma unroll
      for (int s = 0; s < R; s++) {
        const int row = rowAt(s, lane);
        t[s] = (row >= r && row < n) ? z[s] * A[i * ld + row] : 0.0;
      }
      double sc = rdlR(z, i) * zd + waveSumR(t);
      sc = 2 * sc / vn;
#pragma unroll
      for (int s = 0; s < R; s++) {
        const int row = rowAt(s, lane);
        if (row == i) z[s] -= sc * zd;
        if (row >= r && row < n) z[s] -= sc * A[i * ld + row];
      }
    }
  }
  WSYNC();
#pragma unroll
  for (int s = 0; s < R; s++)
    if (rowAt(s, lane) < n) scr[c.perm[rowAt(s, lane)]] = z[s];
  WSYNC();
#pragma unroll
  for (int s = 0; s < R; s++) out[s] = rowAt(s, lane) < n ? scr[rowAt(s, lane)] : 0.0;
  WSYNC();
}

template <bool kLds>
__device__ double codSolveWave(typename Space<kLds>::dptr Ain, typename Space<kLds>::dptr wsIn, int m_, int n_, int ld_,
                               double rhs, typename Space<kLds>::dptr scrIn, int lane) {
  const double ra[1] = {rhs};
  double out[1];
  codSolveWaveR<kLds, 1>(Ain, wsIn, m_, n_, ld_, ra, scrIn, lane, out);
  return out[0];
}

// ---------------------------------------------------------------------------
// kPk: A held as its packed lower triangle (element (a, b), a >= b, at
// a (a + 1) / 2 + b): the wide kernels' LDS stage holds it beside L, where
// the full matrix does not fit (same values, so the same results).
// kPL: L (unit lower) held packed too, in panels of 8 rows: panel q (rows
// 8 q .. 8 q + 7) holds columns 0 .. 8 q + 7 column-major, element (i, j) at
// panel(q) + 8 j + (i & 7) -- each row's i entries, then zeros to the end of
// its panel; the panels 8 doubles apart modulo 32 to spread their LDS banks
// -- 40 KB instead of 74 KB at 96 rows, which lets the wide kernel's stage
// hold Dantzig's factor beside the classification's COD from the start of the
// cascade.  Both solves read eight consecutive steps' elements at constant
// strides (L: a row's eight columns 8 apart; L^T: a column's eight rows of a
// panel, contiguous), immediate offsets from one address.
//
// The zeros are what the triangular solves read instead of a mask: in either
// layout every element at or right of the diagonal is +0, and so is every
// row >= n_C (the packed panels hold rows up to n, one past the last: a zero
// row every column of which exists).  The buffer is zeroed when Dantzig
// starts; the factor's updates -- a row appended at n_C, ldltAddTL, a row
// and column removed -- only ever write strictly lower elements of rows
// < n_C (the square layout's shifts move zeros into zeros, the packed one's
// keep each row's padding where it is), and the removal zeroes the row it
// leaves behind at the new n_C.  So a lane that must not change in a step
// multiplies +0 instead of selecting it.
__host__ __device__ __forceinline__ int dantzigLPanel(int q) { return 32 * q * (q + 1) + 8 * q; }
__host__ __device__ __forceinline__ int dantzigLPackedEl(int i, int j) { return dantzigLPanel(i >> 3) + 8 * j + (i & 7); }
__host__ __device__ __forceinline__ int dantzigLDoubles(int n, bool packed) {
  return packed ? dantzigLPanel((n + 8) >> 3) + 8 : n * (n | 1);
}
template <int R, bool kPk = false, bool kPL = false>
struct WaveDantzig {
  int n, nC, nN, lane, ldL;
  bool degen;  // the factor has given a non-finite solve (solveAny)
  // offset of row i of L (i wave-uniform or per lane)
  // element (i, j) of L, and the stride between a row's consecutive columns
  static constexpr int kCs = kPL ? 8 : 1;
  __device__ __forceinline__ int lel(int i, int j) const { return kPL ? dantzigLPackedEl(i, j) : i * ldL + j; }
  // A: the problem matrix (n x n, symmetric), read in place: slot i of the
  // permuted problem is original row p_i (row i's register p), so the
  // permuted entry (i, j) is A[p_i n + p_j] and a swap of two slots is a
  // swap of registers -- the same values the reference's physically
  // permuted matrix holds (dLCP's row / column swaps), without moving them
  const double* A;
  double* L;    // n x ldL, ldL odd (LDS bank-conflict-free columns), or packed (kPL)
  double* scr;  // >= n doubles
  double x[R], b[R], w[R], lo[R], hi[R], d[R], deltaX[R], deltaW[R], Dell[R], ell[R];
  int findex[R], p[R], C[R], state[R];
#ifdef LCP_PROFILE
  long long prof[8];
#endif

  __device__ __forceinline__ int row(int s) const { return rowAt(s, lane); }
  __device__ __forceinline__ void swapReg(double (&v)[R], int i1, int i2) {
    const double a = rdlR(v, i1), c = rdlR(v, i2);
#pragma unroll
    for (int s = 0; s < R; s++) {
      if (row(s) == i1) v[s] = c;
      else if (row(s) == i2) v[s] = a;
    }
  }
  __device__ __forceinline__ void swapRegI(int (&v)[R], int i1, int i2) {
    const int a = rdliR(v, i1), c = rdliR(v, i2);
#pragma unroll
    for (int s = 0; s < R; s++) {
      if (row(s) == i1) v[s] = c;
      else if (row(s) == i2) v[s] = a;
    }
  }
  // permuted-matrix accessors: row slot i (wave-uniform), column of this
  // lane's slot s / of its C entry / the diagonal
  // (cross-lane reads are kept out of lane-divergent expressions: callers
  // take the row offset first, then index with it)
  // `ro` is the row token of rowOff: the row's offset (full) or index (packed)
  __device__ __forceinline__ int rowOff(int i) const { return kPk ? rdliR(p, i) : rdliR(p, i) * n; }
  __device__ __forceinline__ double Ael(int ro, int c) const {
    if (kPk) {
      const int a = ro > c ? ro : c, b = ro > c ? c : ro;
      return A[a * (a + 1) / 2 + b];
    }
    return A[ro + c];
  }
  __device__ __forceinline__ double ArowAt(int ro, int s) const { return Ael(ro, row(s) < n ? p[s] : 0); }
  __device__ __forceinline__ double Adiag(int i) const {
    const int pi = rdliR(p, i);
    return kPk ? A[pi * (pi + 1) / 2 + pi] : A[pi * n + pi];
  }
  // p of the slot this lane's C entry (slot s) names
  __device__ __forceinline__ int pOfC(int s) const { return gatherRi(p, C[s] & (64 * R - 1)); }
  __device__ __forceinline__ void swapProblem(int i1, int i2) {
    if (i1 == i2) return;
    LP_BEGIN();
    swapReg(x, i1, i2); swapReg(b, i1, i2); swapReg(w, i1, i2); swapReg(lo, i1, i2); swapReg(hi, i1, i2);
    swapRegI(p, i1, i2); swapRegI(state, i1, i2); swapRegI(findex, i1, i2);
    LP_END(prof, 0);
  }
  // L x = B (unit lower), B row-distributed, first m entries, in blocks of
  // eight steps.  A block's L entries are loaded together ahead of its
  // dependent readlane -> FMA chain (LDS latency paid once per 8 steps), so
  // a step is a readlane and unpredicated FMAs: no exec-mask update that
  // would wait on a vector compare, no per-step select, and no branch (a
  // taken branch per step cost more than the step).  A lane that must not
  // change in a step reads a stored +0 (see dantzigLPanel): its own row's
  // elements right of the diagonal, or -- a row already final or past m --
  // zeros the offsets point it at, chosen once per block (lOff: the offset
  // of the row's element 0 for L, the column's offset in its row for L^T).
  // Blocks are 8-aligned, so all steps of a block read their b_k from one
  // register slot S (compile time: no slot select on the chain), and only
  // the slots holding rows the block can change are updated -- rows > k for
  // L, rows < k for L^T; the reference's loops touch no other row either.
  // The last, partial block pads its steps past m with b_k = +0 on zero
  // elements (B - 0 * 0 is B bit for bit).  0 * b_k leaves a lane unchanged
  // only for finite b_k; a non-finite b_k (degenerate factor) re-runs the
  // solve predicated, exactly as the reference's loop.
  // kOnly: update slot S alone (the other slot's updates are deferred, see
  // solveL1 / solveL1T).  kPred: a lane keeps its B where the reference's
  // loop does not touch it (the result selected, not the multiplier zeroed:
  // the form for non-finite b_k, where 0 * b_k is not 0)
  template <int S, bool kFull, bool kT, bool kOnly = false, bool kPred = false>
  __device__ __forceinline__ void solveBlock(double (&B)[R], int m, int k0, const int (&lOff)[R]) {
    // steps: k = k0 + u (L) or k = k0 + 7 - u (L^T, k0 the block's lowest row)
    double Lk[R][8];
#pragma unroll
    for (int s = 0; s < R; s++) {
      if ((kT ? s > S : s < S) || (kOnly && s != S)) continue;
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int k = kT ? k0 + 7 - u : k0 + u;
        // a padded step's element: zero for every lane (L: column m - 1 of
        // the square factor, the rows' own padding in the packed one; L^T:
        // the square factor's row 0, the packed one's (zero) row k >= m)
        const int kc = kFull || k < m ? k : (kPL ? k : kT ? 0 : m - 1);
        // (L^T: the row's element 0 from the block's panel, its k - k0 known
        // at compile time)
        const int rb = kPL ? dantzigLPanel(k0 >> 3) + (kc - k0) : kc * ldL;
        Lk[s][u] = kT ? L[rb + lOff[s]] : L[lOff[s] + kc * kCs];
      }
    }
    // keep the loads unconditional and batched: all issued before any is
    // consumed (one barrier per block -- a barrier per load made the wave
    // wait for each load in turn)
#pragma unroll
    for (int s = 0; s < R; s++) {
      if ((kT ? s > S : s < S) || (kOnly && s != S)) continue;
#pragma unroll
      for (int u = 0; u < 8; u++) asm volatile("" : "+v"(Lk[s][u]));
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int k = kT ? k0 + 7 - u : k0 + u;
      const bool live = kFull || k < m;
      double bk = rdl(B[S], (live ? k : k0) & 63);
      if (!kFull) bk = live ? bk : 0.0;
#pragma unroll
      for (int s = 0; s < R; s++) {
        if ((kT ? s > S : s < S) || (kOnly && s != S)) continue;
        if (kPred) {
          const double t = B[s] - Lk[s][u] * bk;
          B[s] = (kT ? row(s) < k : row(s) > k) && row(s) < m && k < m ? t : B[s];
        } else {
          B[s] -= Lk[s][u] * bk;
        }
      }
    }
  }
  // The deferred updates of slot D by the steps of blocks [kb0, kb1) (8-
  // aligned; steps past m padded as in solveBlock) of slot 1 - D's solve, in
  // the solve's step order: the same multiply-subtract per element as
  // solveBlock's, with every b_k already final -- so an independent chain
  // per lane of dependent FMAs instead of readlane -> FMA steps (the two
  // slots' chains made an R = 2 step ~95 clocks against ~75 for R = 1).
  // Every row of slot D is on the changing side of these steps (L: rows
  // >= 64 > k; L^T: rows < 64 <= k), rows past m read zeros (lOff).
  template <int D, bool kT, bool kPred = false>
  __device__ __forceinline__ void deferredSlot(double (&B)[R], int m, int kb0, int kb1, const int (&lOff)[R]) {
    constexpr int Sb = 1 - D;
    for (int b = 0; b < (kb1 - kb0) / 8; b++) {
      const int k0 = kT ? kb1 - 8 - 8 * b : kb0 + 8 * b;
      double lv[8], bk[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int k = kT ? k0 + 7 - u : k0 + u;
        lv[u] = kT ? L[(kPL ? dantzigLPanel(k0 >> 3) + 7 - u : (k < m ? k : 0) * ldL) + lOff[D]]
                   : L[lOff[D] + k * kCs];
        bk[u] = rdl(B[Sb], k & 63);
        bk[u] = k < m ? bk[u] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; u++) asm volatile("" : "+v"(lv[u]));
#pragma unroll
      for (int u = 0; u < 8; u++) {
        if (kPred) {
          const int k = kT ? k0 + 7 - u : k0 + u;
          const double t = B[D] - lv[u] * bk[u];
          B[D] = (kT ? row(D) < k : row(D) > k) && row(D) < m && k < m ? t : B[D];
        } else {
          B[D] -= lv[u] * bk[u];
        }
      }
    }
  }
  // per-block offsets onto stored zeros (solveBlock): L -- the lane's own
  // row while it can still change (rows k0 .. m - 1), else the block's first
  // row, whose padding covers the block's columns (packed; the square
  // factor's fixed offsets need no per-block choice); L^T -- a column, the
  // lane's own while its row can still change (rows < k0 + 8, < m), else
  // the block's last column, right of every row of the block
  __device__ __forceinline__ void fwdOffsets(int m, int k0, const int (&own)[R], int (&o)[R]) const {
#pragma unroll
    for (int s = 0; s < R; s++) o[s] = !kPL || (row(s) >= k0 && row(s) < m) ? own[s] : lel(k0, 0);
  }
  __device__ __forceinline__ void bwdColumns(int m, int k0, const int (&own)[R], int (&c)[R]) const {
#pragma unroll
    for (int s = 0; s < R; s++) c[s] = !kPL || (row(s) < k0 + 8 && row(s) < m) ? own[s] : (k0 + 7) * kCs;
  }
  template <bool kFull, bool kT, bool kPred>
  __device__ __forceinline__ void solveBlockAt(double (&B)[R], int m, int k0, const int (&lOff)[R]) {
    if (R == 1 || k0 < 64) solveBlock<0, kFull, kT, false, kPred>(B, m, k0, lOff);
    else solveBlock<R - 1, kFull, kT, false, kPred>(B, m, k0, lOff);
  }
  template <bool kPred>
  __device__ __forceinline__ void sweepL1(double (&B)[R], int m) {
    int rowOffL[R], o[R];
#pragma unroll
    for (int s = 0; s < R; s++)
      // (rows past m: a zero row -- the square factor's row 0, the packed
      // one's row m)
      rowOffL[s] = lel(row(s) < m ? row(s) : (kPL ? m : 0), 0);
    int k0 = 0;
    if constexpr (R == 2) {
      // rows 0..63 first, slot 0 alone; slot 1's updates by those steps
      // deferred to one pass; then rows 64.. on slot 1 (its own steps)
      const int kA = m < 64 ? m : 64;
      for (; k0 + 8 <= kA; k0 += 8) {
        fwdOffsets(m, k0, rowOffL, o);
        solveBlock<0, true, false, true, kPred>(B, m, k0, o);
      }
      if (m <= 64) {
        if (k0 < m) {
          fwdOffsets(m, k0, rowOffL, o);
          solveBlock<0, false, false, true, kPred>(B, m, k0, o);
        }
      } else {
        deferredSlot<1, false, kPred>(B, m, 0, 64, rowOffL);
        for (; k0 + 8 <= m; k0 += 8) {
          fwdOffsets(m, k0, rowOffL, o);
          solveBlock<1, true, false, false, kPred>(B, m, k0, o);
        }
        if (k0 < m) {
          fwdOffsets(m, k0, rowOffL, o);
          solveBlock<1, false, false, false, kPred>(B, m, k0, o);
        }
      }
    } else {
      for (; k0 + 8 <= m; k0 += 8) {
        fwdOffsets(m, k0, rowOffL, o);
        solveBlockAt<true, false, kPred>(B, m, k0, o);
      }
      if (k0 < m) {
        fwdOffsets(m, k0, rowOffL, o);
        solveBlockAt<false, false, kPred>(B, m, k0, o);
      }
    }
  }
  // L^T: the blocks from the last row up, the partial one first (8-aligned
  // below it)
  template <bool kPred>
  __device__ __forceinline__ void sweepL1T(double (&B)[R], int m) {
    int colL[R], c[R];
#pragma unroll
    for (int s = 0; s < R; s++)
      // (rows past m: the square factor's column m - 1, zero in every row < m)
      colL[s] = (row(s) < m ? row(s) : (kPL ? 0 : m - 1)) * kCs;
    bool wide = false;
    if constexpr (R == 2) wide = m > 64;
    if (wide) {
      // rows 64.. first, slot 1 alone; slot 0's updates by those steps
      // deferred to one pass (its rows are all below them); then rows 0..63
      int k0 = (m - 1) & ~7;
      bwdColumns(m, k0, colL, c);
      if (k0 + 8 > m) solveBlock<R - 1, false, true, true, kPred>(B, m, k0, c);
      else solveBlock<R - 1, true, true, true, kPred>(B, m, k0, c);
      for (k0 -= 8; k0 >= 64; k0 -= 8) {
        bwdColumns(m, k0, colL, c);
        solveBlock<R - 1, true, true, true, kPred>(B, m, k0, c);
      }
      if constexpr (R == 2) deferredSlot<0, true, kPred>(B, m, 64, ((m - 1) & ~7) + 8, colL);
      for (k0 = 56; k0 >= 0; k0 -= 8) {
        bwdColumns(m, k0, colL, c);
        solveBlock<0, true, true, false, kPred>(B, m, k0, c);
      }
    } else if (m > 0) {
      int k0 = (m - 1) & ~7;  // lowest row of the top block
      bwdColumns(m, k0, colL, c);
      if (k0 + 8 > m) solveBlockAt<false, true, kPred>(B, m, k0, c);
      else solveBlockAt<true, true, kPred>(B, m, k0, c);
      for (k0 -= 8; k0 >= 0; k0 -= 8) {
        bwdColumns(m, k0, colL, c);
        solveBlockAt<true, true, kPred>(B, m, k0, c);
      }
    }
  }
  // A non-finite b_k (a degenerate factor: an infinite d after a zero
  // pivot) makes 0 * b_k a NaN where the reference's loop leaves a row
  // alone, so such a solve is re-run exactly as the reference's loop when
  // the unpredicated sweep's result is non-finite (finite b_k give the same
  // bits either way: a skipped lane's +0 * b_k adds a signed zero only).
  // R = 1 (the one-row kernel: <= 64 rows, degenerate factors rare, and
  // every variant of the sweep costs registers the kernel does not have):
  // the unblocked loop.  R = 2 (the wide kernel's 65..128-row problems,
  // whose failing Dantzig runs go degenerate for dozens of pivots): the
  // blocked predicated sweep, taken directly when B arrives non-finite or
  // once the factor has shown itself degenerate (`degen`, sticky for the
  // rest of the solve) -- measured r05m..v5: 96-row problem 4.39M -> 2.35M
  // clocks, the one-row kernel unchanged.
  template <bool kT>
  __device__ __forceinline__ void solveAny(double (&B)[R], int m) {
    m = uni(m);
    if constexpr (R == 2) {
      bool bad = false;
#pragma unroll
      for (int s = 0; s < R; s++) bad = bad || (row(s) < m && !isfinite(B[s]));
      if (degen || __ballot(bad)) {
        if (kT) sweepL1T<true>(B, m);
        else sweepL1<true>(B, m);
        return;
      }
    }
    double B0[R];
#pragma unroll
    for (int s = 0; s < R; s++) B0[s] = B[s];
    if (kT) sweepL1T<false>(B, m);
    else sweepL1<false>(B, m);
    bool nonFinite = false;
#pragma unroll
    for (int s = 0; s < R; s++) nonFinite = nonFinite || (row(s) < m && !isfinite(B[s]));
    if (__ballot(nonFinite)) {
      degen = true;
#pragma unroll
      for (int s = 0; s < R; s++) B[s] = B0[s];
      if constexpr (R == 2) {
        if (kT) sweepL1T<true>(B, m);
        else sweepL1<true>(B, m);
      } else if (kT) {
        for (int k = m - 1; k >= 0; k--) {
          const double bk = rdlR(B, k);
#pragma unroll
          for (int s = 0; s < R; s++)
            if (row(s) < k) B[s] -= L[lel(k, row(s))] * bk;
        }
      } else {
        for (int k = 0; k < m; k++) {
          const double bk = rdlR(B, k);
#pragma unroll
          for (int s = 0; s < R; s++)
            if (row(s) > k && row(s) < m) B[s] -= L[lel(row(s), k)] * bk;
        }
      }
    }
  }
  __device__ __forceinline__ void solveL1(double (&B)[R], int m) {
    LP_BEGIN();
    solveAny<false>(B, m);
    LP_END(prof, 1);
  }
  __device__ __forceinline__ void solveL1T(double (&B)[R], int m) {
    LP_BEGIN();
    solveAny<true>(B, m);
    LP_END(prof, 2);
  }
  __device__ __forceinline__ double sumC(const double (&u)[R], const double (&v)[R]) const {
    double t[R];
#pragma unroll
    for (int s = 0; s < R; s++) t[s] = row(s) < nC ? u[s] * v[s] : 0.0;
    return waveSumR(t);
  }
  __device__ __forceinline__ void transferToC(int i) {
    const double Aii = Adiag(i);
    if (nC > 0) {
#pragma unroll
      for (int s = 0; s < R; s++)
        if (row(s) < nC) L[lel(nC, row(s))] = ell[s];
      const double dd = sumC(ell, Dell);
      setR(d, nC, lane, 1.0 / (Aii - dd));
    } else {
      setR(d, 0, lane, 1.0 / Aii);
    }
    swapProblem(nC, i);
    setRi(C, nC, lane, nC);
    nC++;
  }
  __device__ __forceinline__ void loadDell(int i) {
    const int ro = rowOff(i);
#pragma unroll
    for (int s = 0; s < R; s++) {
      const int pc = pOfC(s);
      Dell[s] = row(s) < nC ? Ael(ro, pc) : 0.0;
    }
  }
  __device__ __forceinline__ void transferFromNtoC(int i) {
    const double Aii = Adiag(i);
    if (nC > 0) {
      loadDell(i);
      solveL1(Dell, nC);
#pragma unroll
      for (int s = 0; s < R; s++) {
        ell[s] = row(s) < nC ? Dell[s] * d[s] : 0.0;
        if (row(s) < nC) L[lel(nC, row(s))] = ell[s];
      }
      const double dd = sumC(ell, Dell);
      setR(d, nC, lane, 1.0 / (Aii - dd));
    } else {
      setR(d, 0, lane, 1.0 / Aii);
    }
    swapProblem(nC, i);
    setRi(C, nC, lane, nC);
    nN--;
    nC++;
  }
  // _dLDLTAddTL on the sub-factorisation starting at (r, r); `a` holds
  // element j at row r + j
  __device__ __forceinline__ void ldltAddTL(int r, int m2, const double (&a)[R]) {
    if (m2 < 2) return;
    const double r2 = 0.70710678118654752440;
    int j0[R];
    double W1[R], W2[R];
#pragma unroll
    for (int s = 0; s < R; s++) {
      j0[s] = row(s) - r;
      W1[s] = 0.0;
      W2[s] = 0.0;
      if (j0[s] >= 1 && j0[s] < m2) { W1[s] = a[s] * r2; W2[s] = W1[s]; }
    }
    const double a0 = rdlR(a, r);
    const double W11 = (0.5 * a0 + 1) * r2;
    const double W21 = (0.5 * a0 - 1) * r2;
    double alpha1 = 1.0, alpha2 = 1.0;
    {
      double dee = rdlR(d, r);
      double alphanew = alpha1 + (W11 * W11) * dee;
      dee /= alphanew;
      const double gamma1 = W11 * dee;
      dee *= alpha1;
      alpha1 = alphanew;
      alphanew = alpha2 - (W21 * W21) * dee;
      dee /= alphanew;
      alpha2 = alphanew;
      const double k1 = 1.0 - W21 * gamma1;
      const double k2 = W21 * gamma1 * W11 - W21;
#pragma unroll
      for (int s = 0; s < R; s++)
        if (j0[s] >= 1 && j0[s] < m2) {
          const double Wp = W1[s];
          const double el = L[lel(r + j0[s], r)];
          W1[s] = Wp - W11 * el;
          W2[s] = k1 * Wp + k2 * el;
        }
    }
    for (int j = 1; j < m2; j++) {
      const double k1 = rdlR(W1, r + j), k2 = rdlR(W2, r + j);
      double dee = rdlR(d, r + j);
      double alphanew = alpha1 + (k1 * k1) * dee;
      dee /= alphanew;
      const double gamma1 = k1 * dee;
      dee *= alpha1;
      alpha1 = alphanew;
      alphanew = alpha2 - (k2 * k2) * dee;
      dee /= alphanew;
      const double gamma2 = k2 * dee;
      dee *= alpha2;
      setR(d, r + j, lane, dee);
      alpha2 = alphanew;
#pragma unroll
      for (int s = 0; s < R; s++)
        if (j0[s] > j && j0[s] < m2) {
          double el = L[lel(r + j0[s], r + j)];
          double Wp = W1[s] - k1 * el;
          el += gamma1 * Wp;
          W1[s] = Wp;
          Wp = W2[s] - k2 * el;
          el -= gamma2 * Wp;
          W2[s] = Wp;
          L[lel(r + j0[s], r + j)] = el;
        }
    }
  }
  __device__ __forceinline__ void ldltRemove(int r, int n2) {
    LP_BEGIN();
    if (r != n2 - 1) {
      double a[R];
      if (r == 0) {
        const int ro = rowOff(rdliR(C, 0));
#pragma unroll
        for (int s = 0; s < R; s++) {
          const int pc = pOfC(s);
          a[s] = row(s) < n2 ? -Ael(ro, pc) : 0.0;  // A symmetric
          if (row(s) == 0) a[s] += 1.0;
        }
        ldltAddTL(0, n2, a);
      } else {
        double t[R], sacc[R];
#pragma unroll
        for (int s = 0; s < R; s++) {
          t[s] = row(s) < r ? L[lel(r, row(s))] / d[s] : 0.0;
          sacc[s] = 0.0;
        }
        const int ro = rowOff(rdliR(C, r));
        int pc[R];
#pragma unroll
        for (int s = 0; s < R; s++) pc[s] = pOfC(s);
        for (int k = 0; k < r; k++) {
          const double tk = rdlR(t, k);
#pragma unroll
          for (int s = 0; s < R; s++)
            if (row(s) >= r && row(s) < n2) sacc[s] += L[lel(row(s), k)] * tk;
        }
#pragma unroll
        for (int s = 0; s < R; s++) {
          a[s] = 0.0;
          if (row(s) >= r && row(s) < n2) a[s] = sacc[s] - Ael(ro, pc[s]);  // A symmetric
          if (row(s) == r) a[s] += 1.0;
        }
        ldltAddTL(r, n2 - r, a);
      }
    }
    WSYNC();
    if (r < n2 - 1) {
      if (kPL) {
        // row and column r out of the packed triangle, lane = column: new
        // (i, j) = old (i + 1, j + [j >= r]) for rows i >= r (the rows above
        // keep their place).  Eight rows per batch: all their reads, a wave
        // barrier, then their writes -- a lane's source element is another
        // lane's destination one row later, so the batch's reads must be
        // done before any of its writes, and the next batch's sources (old
        // rows >= i0 + 9) lie past every destination of this one
        for (int i0 = r; i0 < n2 - 1; i0 += 8) {
          double v[8][R];
#pragma unroll
          for (int u = 0; u < 8; u++) {
            const int i = i0 + u;
            const int src = i + 1 < n2 ? i + 1 : n2 - 1;
#pragma unroll
            for (int s = 0; s < R; s++) {
              const int j = row(s);
              v[u][s] = (i < n2 - 1 && j < i) ? L[lel(src, j + (j >= r ? 1 : 0))] : 0.0;
            }
          }
          WSYNC();
#pragma unroll
          for (int u = 0; u < 8; u++) {
            const int i = i0 + u;
#pragma unroll
            for (int s = 0; s < R; s++) {
              const int j = row(s);
              if (i < n2 - 1 && j < i) L[lel(i, j)] = v[u][s];
            }
          }
          WSYNC();
        }
      } else {
#pragma unroll
        for (int s = 0; s < R; s++)
          if (row(s) < n2)
            for (int j = r; j < n2 - 1; j++) L[row(s) * ldL + j] = L[row(s) * ldL + j + 1];
        WSYNC();
#pragma unroll
        for (int s = 0; s < R; s++)
          if (row(s) < n2)
            for (int i = r; i < n2 - 1; i++) L[i * ldL + row(s)] = L[(i + 1) * ldL + row(s)];
      }
      WSYNC();
      double dn[R];
#pragma unroll
      for (int s = 0; s < R; s++) dn[s] = d[s];
      shiftDownR(dn, lane);
#pragma unroll
      for (int s = 0; s < R; s++)
        if (row(s) >= r && row(s) < n2 - 1) d[s] = dn[s];
    }
    // the row left behind at the new n_C: zero again (dantzigLPanel)
#pragma unroll
    for (int s = 0; s < R; s++)
      if (row(s) < n2 - 1) L[lel(n2 - 1, row(s))] = 0.0;
    WSYNC();
    LP_END(prof, 3);
  }
  __device__ __forceinline__ void transferFromCtoN(int i) {
    bool hitI[R], hitLast[R];
#pragma unroll
    for (int s = 0; s < R; s++) {
      hitI[s] = row(s) < nC && C[s] == i;
      hitLast[s] = row(s) < nC && C[s] == nC - 1;
    }
    const int j = waveFirstR(hitI);
    if (j >= 0) {
      const int k = waveFirstR(hitLast);
      ldltRemove(j, nC);
      const int Cj = rdliR(C, j);
      setRi(C, k, lane, Cj);
      int Cn[R];
#pragma unroll
      for (int s = 0; s < R; s++) Cn[s] = C[s];
      shiftDownRi(Cn, lane);
#pragma unroll
      for (int s = 0; s < R; s++)
        if (row(s) >= j && row(s) < nC - 1) C[s] = Cn[s];
    }
    swapProblem(i, nC - 1);
    nN++;
    nC--;
  }
  __device__ __forceinline__ void solve1(int i, int dir, bool onlyTransfer) {
    if (nC > 0) {
      loadDell(i);
      solveL1(Dell, nC);
#pragma unroll
      for (int s = 0; s < R; s++) ell[s] = row(s) < nC ? Dell[s] * d[s] : 0.0;
      if (!onlyTransfer) {
        double tmp[R];
#pragma unroll
        for (int s = 0; s < R; s++) tmp[s] = ell[s];
        solveL1T(tmp, nC);
        WSYNC();
#pragma unroll
        for (int s = 0; s < R; s++)
          if (row(s) < nC) scr[C[s]] = dir > 0 ? -tmp[s] : tmp[s];
        WSYNC();
#pragma unroll
        for (int s = 0; s < R; s++)
          if (row(s) < nC) deltaX[s] = scr[row(s)];
        WSYNC();
      }
    }
  }
  __device__ __forceinline__ double AiC(int i, const double (&q)[R]) {
    const int ro = rowOff(i);
    double t[R];
#pragma unroll
    for (int s = 0; s < R; s++) t[s] = row(s) < nC ? ArowAt(ro, s) * q[s] : 0.0;
    return waveSumR(t);
  }
  __device__ __forceinline__ double AiN(int i, const double (&q)[R]) {
    const int ro = rowOff(i);
    double t[R];
#pragma unroll
    for (int s = 0; s < R; s++) t[s] = (row(s) >= nC && row(s) < nC + nN) ? ArowAt(ro, s) * q[s] : 0.0;
    return waveSumR(t);
  }
};

// A (n x n, symmetric, read only), L (dantzigLDoubles(n, kPL) scratch), scr (>= n); problem
// vectors row-distributed; returns success and x (row-distributed).
// kLds: A on chip; kLdsL: L and scr on chip (default: with A)
template <bool kLds, int R, bool kPk = false, bool kLdsL = kLds, bool kPL = false>
__device__ bool waveDantzigR(int n, typename Space<kLds>::cdptr Ain, typename Space<kLdsL>::dptr Lin,
                             typename Space<kLdsL>::dptr scrIn, double (&xOut)[R], const double (&b)[R],
                             const double (&lo)[R], const double (&hi)[R], const int (&findex)[R], int lane,
                             double* dbg = nullptr, const int* cancel = nullptr, int* tally = nullptr) {
  n = uni(n);
  const double* A = (const double*)Ain;
  double* Lbuf = (double*)Lin;
  double* scr = (double*)scrIn;
  WaveDantzig<R, kPk, kPL> D;
  int pivots = 0;
  // executed work for the roofline (tally: LDS ints [0] pivots, [2] FLOPs):
  // per row the w_i dot product (2n), per pivot the two triangular solves on
  // the clamped set (2 n_C^2), the N-rows' column update (2 n_N n_C), its
  // dot products and the ratio tests (~6n)
  int flops = 0;
  auto account = [&]() {
    if (tally && lane == 0) {
      __hip_atomic_fetch_add(tally, pivots, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_add(tally + 2, flops, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  };
  D.n = n; D.nC = 0; D.nN = 0; D.lane = lane; D.ldL = n | 1; D.degen = false;
  D.A = A; D.L = Lbuf; D.scr = scr;
#pragma unroll
  for (int s = 0; s < R; s++) {
    D.x[s] = 0.0; D.b[s] = b[s]; D.w[s] = 0.0; D.lo[s] = lo[s]; D.hi[s] = hi[s]; D.d[s] = 0.0;
    D.deltaX[s] = 0.0; D.deltaW[s] = 0.0; D.Dell[s] = 0.0; D.ell[s] = 0.0;
    D.findex[s] = findex[s]; D.p[s] = rowAt(s, lane); D.C[s] = 0; D.state[s] = 0;
  }
#ifdef LCP_PROFILE
  for (int k = 0; k < 8; k++) D.prof[k] = 0;
#endif
  for (int k = lane; k < dantzigLDoubles(n, kPL); k += 64) Lbuf[k] = 0.0;
  {
    bool unb = false;
#pragma unroll
    for (int s = 0; s < R; s++)
      unb = unb || (rowAt(s, lane) < n && findex[s] < 0 && lo[s] == -LCP_INF && hi[s] == LCP_INF);
    if (__ballot(unb)) return false;
  }
  {
    int numAtEnd = 0;
    for (int k = n - 1; k >= 0; k--)
      if (rdliR(D.findex, k) >= 0) { D.swapProblem(k, n - 1 - numAtEnd); numAtEnd++; }
  }
  WSYNC();
  bool hitFirstFriction = false;
  for (int i = 0; i < n; i++) {
    D.nC = uni(D.nC);
    D.nN = uni(D.nN);
    if (!hitFirstFriction && rdliR(D.findex, i) >= 0) {
      WSYNC();
#pragma unroll
      for (int s = 0; s < R; s++)
        if (rowAt(s, lane) < n) scr[D.p[s]] = D.x[s];
      WSYNC();
#pragma unroll
      for (int s = 0; s < R; s++)
        if (rowAt(s, lane) >= i && rowAt(s, lane) < n) {
          const double wfk = scr[D.findex[s]];
          if (wfk == 0) { D.hi[s] = 0; D.lo[s] = 0; }
          else { D.hi[s] = fabs(D.hi[s] * wfk); D.lo[s] = -D.hi[s]; }
        }
      WSYNC();
      hitFirstFriction = true;
    }
    flops += 2 * n;
    LP_BEGIN();
    const double wi = D.AiC(i, D.x) + D.AiN(i, D.x) - rdlR(D.b, i);
    LP_END(D.prof, 4);
    setR(D.w, i, lane, wi);
    const double loi = rdlR(D.lo, i), hii = rdlR(D.hi, i);
    if (loi == 0 && wi >= 0) {
      D.nN++;
      setRi(D.state, i, lane, 0);
    } else if (hii == 0 && wi <= 0) {
      D.nN++;
      setRi(D.state, i, lane, 1);
    } else if (wi == 0) {
      D.solve1(i, 0, true);
      D.transferToC(i);
    } else {
      for (;;) {
        D.nC = uni(D.nC);
        D.nN = uni(D.nN);
        const double wiNow = rdlR(D.w, i);
        int dir;
        double dirf;
        if (wiNow <= 0) { dir = 1; dirf = 1.0; } else { dir = -1; dirf = -1.0; }
        D.solve1(i, dir, false);
        const int nC = D.nC, nN = D.nN;
        bool inN[R];
        LP_BEGIN();
        {
          // every lane accumulates (no exec mask per step); only N rows keep it
          int colA[R];
          double acc[R];
#pragma unroll
          for (int s = 0; s < R; s++) {
            const int row = rowAt(s, lane);
            inN[s] = row >= nC && row < nC + nN;
            colA[s] = row < n ? D.p[s] : 0;
            acc[s] = 0.0;
          }
          // eight C entries per block: their readlanes and A loads issued
          // together, then the multiply-adds in j order (A symmetric: row j);
          // the last, partial block pads with +0 * -0 terms (acc + -0 is acc
          // bit for bit), so no term is a branch of its own
          // (Mc: the register slots holding N rows, a compile-time mask --
          // the others' sums are never read, so their loads and multiply-adds
          // are skipped: with two slots, a pivot at row i <= 64 has no N row
          // in slot 1, one with n_C >= 64 none in slot 0)
          auto block = [&](auto Mc, int j0, bool full) {
            constexpr int M = decltype(Mc)::value;
            double dx[8], av[R][8];
            int ro[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
              const int j = full || j0 + u < nC ? j0 + u : 0;
              dx[u] = rdlR(D.deltaX, j);
              ro[u] = D.rowOff(j);
            }
#pragma unroll
            for (int u = 0; u < 8; u++)
#pragma unroll
              for (int s = 0; s < R; s++)
                if ((M >> s) & 1) av[s][u] = D.Ael(ro[u], colA[s]);
#pragma unroll
            for (int s = 0; s < R; s++)
#pragma unroll
              for (int u = 0; u < 8; u++)
                if ((M >> s) & 1) asm volatile("" : "+v"(av[s][u]));
            if (!full) {
#pragma unroll
              for (int u = 0; u < 8; u++) {
                const bool live = j0 + u < nC;
                dx[u] = live ? dx[u] : -0.0;
#pragma unroll
                for (int s = 0; s < R; s++)
                  if ((M >> s) & 1) av[s][u] = live ? av[s][u] : 0.0;
              }
            }
#pragma unroll
            for (int u = 0; u < 8; u++)
#pragma unroll
              for (int s = 0; s < R; s++)
                if ((M >> s) & 1) acc[s] += av[s][u] * dx[u];
          };
          auto blocks = [&](auto Mc) {
            int j0 = 0;
            for (; j0 + 8 <= nC; j0 += 8) block(Mc, j0, true);
            if (j0 < nC) block(Mc, j0, false);
          };
#ifdef LCP_PROFILE
          const long long lpm_ = (long long)__builtin_amdgcn_s_memtime();
#endif
          const bool nIn0 = nN > 0 && nC < 64, nIn1 = R > 1 && nN > 0 && nC + nN > 64;
          if constexpr (R == 1) {
            if (nIn0) blocks(std::integral_constant<int, 1>{});
          } else {
            if (nIn0 && nIn1) blocks(std::integral_constant<int, 3>{});
            else if (nIn1) blocks(std::integral_constant<int, 2>{});
            else if (nIn0) blocks(std::integral_constant<int, 1>{});
          }
#ifdef LCP_PROFILE
          D.prof[6] += (long long)__builtin_amdgcn_s_memtime() - lpm_;
#endif
          const int roI = D.rowOff(i);
#pragma unroll
          for (int s = 0; s < R; s++) {
            const double aij = D.ArowAt(roI, s);
            if (inN[s]) D.deltaW[s] = acc[s] + (dir > 0 ? aij : -aij);
          }
        }
        const double dwi = D.AiC(i, D.deltaX) + D.Adiag(i) * dirf;
        setR(D.deltaW, i, lane, dwi);
        int cmd = 1, si = 0;
        double s = -wiNow / dwi;
        const double xi = rdlR(D.x, i), hiI = rdlR(D.hi, i), loI = rdlR(D.lo, i);
        if (dir > 0) {
          if (hiI < LCP_INF) { const double s2 = (hiI - xi) * dirf; if (s2 < s) { s = s2; cmd = 3; } }
        } else {
          if (loI > -LCP_INF) { const double s2 = (loI - xi) * dirf; if (s2 < s) { s = s2; cmd = 2; } }
        }
        {
          // the N-side (cmd 4) and C-side (cmd 5/6) ratio tests of the
          // reference over disjoint rows: one division and one reduction;
          // on equal minima the N side wins, as in the reference's order
          bool cand4[R], anyR[R], tmin[R];
          int typ[R];
          double rr[R], key[R];
#pragma unroll
          for (int q = 0; q < R; q++) {
            const int row = rowAt(q, lane);
            cand4[q] = false;
            typ[q] = 0;
            double num = 0.0, den = 1.0;
            if (inN[q]) {
              const bool dirOk = !D.state[q] ? D.deltaW[q] < 0 : D.deltaW[q] > 0;
              if (dirOk && !(D.lo[q] == 0 && D.hi[q] == 0)) { cand4[q] = true; num = -D.w[q]; den = D.deltaW[q]; }
            } else if (row < nC) {
              if (D.deltaX[q] < 0 && D.lo[q] > -LCP_INF) { num = D.lo[q] - D.x[q]; den = D.deltaX[q]; typ[q] = 5; }
              if (D.deltaX[q] > 0 && D.hi[q] < LCP_INF) { num = D.hi[q] - D.x[q]; den = D.deltaX[q]; typ[q] = 6; }
            }
            rr[q] = num / den;
            anyR[q] = cand4[q] || typ[q];
            key[q] = anyR[q] ? rr[q] : LCP_INF;
          }
          const double mm = waveMinR(key);
          if (mm < s) {
            s = mm;
#pragma unroll
            for (int q = 0; q < R; q++) tmin[q] = cand4[q] && rr[q] == mm;
            const int s4i = waveFirstR(tmin);
            if (s4i >= 0) {
              cmd = 4;
              si = s4i;
            } else {
#pragma unroll
              for (int q = 0; q < R; q++) tmin[q] = typ[q] && rr[q] == mm;
              si = waveFirstR(tmin);
              cmd = rdliR(typ, si);
            }
          }
        }
        pivots++;
        flops += 2 * nC * nC + 2 * nN * nC + 6 * n;
        if (dbg && lane == 0) { dbg[0] = pivots; dbg[1] = i; }
        LP_END(D.prof, 5);
#ifdef LCP_PROFILE
        if (dbg && lane == 0)
          for (int k = 0; k < 8; k++) dbg[2 + k] = (double)D.prof[k];
#endif
        if (s <= 0.0) {
          account();
          return false;
        }
        // `cancel` (LDS int, optional): polled once per pivot; a set flag
        // abandons the solve (the caller no longer needs it)
        if (cancel && uni(__hip_atomic_load(cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))) {
          account();
          return false;
        }
#pragma unroll
        for (int q = 0; q < R; q++) {
          const int row = rowAt(q, lane);
          if (row < nC) D.x[q] += s * D.deltaX[q];
          if (row == i) D.x[q] += s * dirf;
          if (inN[q]) D.w[q] += s * D.deltaW[q];
          if (row == i) D.w[q] += s * dwi;
        }
#ifdef LCP_PROFILE
        const long long lpt_ = (long long)__builtin_amdgcn_s_memtime();
#endif
        switch (cmd) {
          case 1:
            setR(D.w, i, lane, 0.0);
            D.transferToC(i);
            break;
          case 2:
            setR(D.x, i, lane, rdlR(D.lo, i));
            setRi(D.state, i, lane, 0);
            D.nN++;
            break;
          case 3:
            setR(D.x, i, lane, rdlR(D.hi, i));
            setRi(D.state, i, lane, 1);
            D.nN++;
            break;
          case 4:
            setR(D.w, si, lane, 0.0);
            D.transferFromNtoC(si);
            break;
          case 5:
            setR(D.x, si, lane, rdlR(D.lo, si));
            setRi(D.state, si, lane, 0);
            D.transferFromCtoN(si);
            break;
          case 6:
            setR(D.x, si, lane, rdlR(D.hi, si));
            setRi(D.state, si, lane, 1);
            D.transferFromCtoN(si);
            break;
        }
#ifdef LCP_PROFILE
        D.prof[7] += (long long)__builtin_amdgcn_s_memtime() - lpt_;
#endif
        if (cmd <= 3) break;
      }
    }
  }
  WSYNC();
#pragma unroll
  for (int s = 0; s < R; s++)
    if (rowAt(s, lane) < n) scr[D.p[s]] = D.x[s];
  WSYNC();
#pragma unroll
  for (int s = 0; s < R; s++) xOut[s] = rowAt(s, lane) < n ? scr[rowAt(s, lane)] : 0.0;
  WSYNC();
  account();
  return true;
}

template <bool kLds>
__device__ bool waveDantzig(int n, typename Space<kLds>::cdptr Ain, typename Space<kLds>::dptr Lin,
                            typename Space<kLds>::dptr scrIn, double& xOut, double b, double lo, double hi,
                            int findex, int lane, double* dbg = nullptr, const int* cancel = nullptr) {
  double xa[1];
  const double ba[1] = {b}, la[1] = {lo}, ha[1] = {hi};
  const int fa[1] = {findex};
  const bool ok = waveDantzigR<kLds, 1>(n, Ain, Lin, scrIn, xa, ba, la, ha, fa, lane, dbg, cancel);
  xOut = xa[0];
  return ok;
}

// ---------------------------------------------------------------------------
// LCPUtils::reduce (LCPUtils.cpp:144) with mergeLCPColumns (:346), without
// moving data.  A merge of column b into column a (the first pair, in (a, b)
// order, whose columns differ by < 1e-4 in squared norm, with |b_a - b_b| <
// 1e-4 and equal findex / hi / lo) deletes row and column b and doubles column
// a, so the reduced problem is always the principal submatrix of the input
// over the surviving rows, each column j scaled by a power of two scl_j:
//   A_r[r][s] = (A[i][j] + shift [i == j]) * scl_j,  i = act_r, j = act_s.
// `shift` is a CFM the caller has already (virtually) added to A's diagonal
// (the PGS fallback reduces A + cfm I).  Row i holds original row i's b, lo,
// hi and findex.  Gives (wave-uniform) the mask of surviving rows; row i
// gets scl (its column scale, 1 for a removed row) and rep (the surviving row
// row i was merged into).  `maxMerges` = 0 only reports whether a merge
// exists (mask != the full mask).
// ---------------------------------------------------------------------------
template <bool kLds, int R>
__device__ void waveReduceR(int m, typename Space<kLds>::cdptr Ain, double shift, const double (&b)[R],
                            const double (&lo)[R], const double (&hi)[R], const int (&fi)[R], int lane,
                            double (&scl)[R], int (&rep)[R], unsigned long long (&alive)[R], int maxMerges = 128) {
  m = uni(m);
  const double* A = (const double*)Ain;
  constexpr int kNone = 64 * R;
  int col[R];
#pragma unroll
  for (int s = 0; s < R; s++) {
    const int lo64 = 64 * s;
    alive[s] = m >= lo64 + 64 ? ~0ull : (m > lo64 ? ((1ull << (m - lo64)) - 1ull) : 0ull);
    scl[s] = 1.0;
    rep[s] = rowAt(s, lane);
    col[s] = rowAt(s, lane) < m ? rowAt(s, lane) : 0;
  }
  for (int merges = 0; merges <= maxMerges; merges++) {
    // findex in terms of surviving rows (the reference remaps fIndex on
    // every merge; comparing representatives is the same test)
    int frow[R], hitC[R];
    bool me[R];
#pragma unroll
    for (int s = 0; s < R; s++) {
      const int fr = gatherRi(rep, fi[s] >= 0 ? fi[s] : 0);
      frow[s] = fi[s] >= 0 ? fr : -1;
      me[s] = rowAt(s, lane) < m && bitR(alive, rowAt(s, lane));
      hitC[s] = kNone;
    }
    // Norms of the scaled surviving columns: a pair whose norms differ by
    // more than the distance bound (plus the rounding of both norms and of
    // the distance sum, a relative 1e-12 margin, far above m eps) cannot
    // pass the distance test (||a - c|| >= | ||a|| - ||c|| |), so its O(m)
    // row loop is skipped; the pairs that are compared are compared exactly
    // as before.  (On the HBM-pool worlds every row loop is m dependent L2
    // reads per lane: up to ~0.7M clocks per reduce at 96 rows.)
    double nrm[R];
#pragma unroll
    for (int s = 0; s < R; s++) nrm[s] = 0.0;
    for (int i = 0; i < m; i++) {
      const bool ai = bitR(alive, i);
#pragma unroll
      for (int s = 0; s < R; s++) {
        const double aa = (A[i * m + col[s]] + (i == rowAt(s, lane) ? shift : 0.0)) * scl[s];
        nrm[s] += ai ? aa * aa : 0.0;
      }
    }
#pragma unroll
    for (int s = 0; s < R; s++) nrm[s] = sqrt(nrm[s]);
    for (int c = 1; c < m; c++) {
      if (!bitR(alive, c)) continue;
      const double bc = rdlR(b, c), loc = rdlR(lo, c), hic = rdlR(hi, c), sc = rdlR(scl, c);
      const double nrc = rdlR(nrm, c);
      const int fc = rdliR(frow, c);
      bool cand[R], anyCand = false;
#pragma unroll
      for (int s = 0; s < R; s++) {
        const bool far = fabs(nrm[s] - nrc) - 1e-12 * (nrm[s] + nrc) > 1.0000001e-2;
        cand[s] = me[s] && rowAt(s, lane) < c && hitC[s] == kNone && fabs(b[s] - bc) < 1e-4 && frow[s] == fc &&
                  hi[s] == hic && lo[s] == loc && !far;
        anyCand = anyCand || cand[s];
      }
      if (__ballot(anyCand)) {
        double dd[R];
#pragma unroll
        for (int s = 0; s < R; s++) dd[s] = 0.0;
        for (int i = 0; i < m; i++) {
          if (!bitR(alive, i)) continue;
          const double ac = (A[i * m + c] + (i == c ? shift : 0.0)) * sc;
#pragma unroll
          for (int s = 0; s < R; s++) {
            const double aa = (A[i * m + col[s]] + (i == rowAt(s, lane) ? shift : 0.0)) * scl[s];
            dd[s] += (aa - ac) * (aa - ac);
          }
        }
#pragma unroll
        for (int s = 0; s < R; s++)
          if (cand[s] && dd[s] < 1e-4) hitC[s] = c;
      }
    }
    bool hit[R];
#pragma unroll
    for (int s = 0; s < R; s++) hit[s] = hitC[s] < kNone;
    const int a = waveFirstR(hit);
    if (a < 0 || merges == maxMerges) {
      if (a >= 0) {
        const int cb = rdliR(hitC, a);
        alive[cb >> 6] &= ~(1ull << (cb & 63));  // report only
      }
      break;
    }
    const int cb = rdliR(hitC, a);
    alive[cb >> 6] &= ~(1ull << (cb & 63));
#pragma unroll
    for (int s = 0; s < R; s++) {
      if (rowAt(s, lane) == a) scl[s] *= 2.0;
      if (rep[s] == cb) rep[s] = a;
    }
  }
}

template <bool kLds>
__device__ unsigned long long waveReduce(int m, typename Space<kLds>::cdptr Ain, double shift, double b, double lo,
                                         double hi, int fi, int lane, double& scl, int& rep, int maxMerges = 64) {
  const double ba[1] = {b}, la[1] = {lo}, ha[1] = {hi};
  const int fa[1] = {fi};
  double sa[1];
  int ra[1];
  unsigned long long al[1];
  waveReduceR<kLds, 1>(m, Ain, shift, ba, la, ha, fa, lane, sa, ra, al, maxMerges);
  scl = sa[0];
  rep = ra[0];
  return al[0];
}

// rank of original row `row` among the surviving rows (its reduced index)
__device__ __forceinline__ int reducedIndex(unsigned long long alive, int row) {
  return __popcll(alive & ((1ull << row) - 1ull));
}

// the reduced problem's row-held vectors: row r gets the values of the r-th
// surviving row (its findex as a reduced index); returns the reduced size
template <int R>
__device__ __forceinline__ int reducedVectorsR(const unsigned long long (&alive)[R], const int (&rep)[R], int lane,
                                               double (&b)[R], double (&lo)[R], double (&hi)[R], int (&fi)[R],
                                               int (&act)[R]) {
  const int mr = popR(alive);
  // act_r: the r-th set bit of alive
#pragma unroll
  for (int s = 0; s < R; s++) act[s] = 0;
  {
    int r = 0;
#pragma unroll
    for (int q = 0; q < R; q++) {
      unsigned long long a = alive[q];
      while (a) {
        const int i = 64 * q + __ffsll((long long)a) - 1;
        setRi(act, r, lane, i);
        a &= a - 1ull;
        r++;
      }
    }
  }
  double nb[R], nlo[R], nhi[R];
  int nfi[R];
#pragma unroll
  for (int s = 0; s < R; s++) {
    const int src = rowAt(s, lane) < mr ? act[s] : 0;
    nb[s] = gatherR(b, src);
    nlo[s] = gatherR(lo, src);
    nhi[s] = gatherR(hi, src);
    nfi[s] = gatherRi(fi, src);
  }
#pragma unroll
  for (int s = 0; s < R; s++) {
    const int frep = gatherRi(rep, nfi[s] >= 0 ? nfi[s] : 0);
    const bool in = rowAt(s, lane) < mr;
    b[s] = in ? nb[s] : 0.0;
    lo[s] = in ? nlo[s] : 0.0;
    hi[s] = in ? nhi[s] : 0.0;
    fi[s] = (in && nfi[s] >= 0) ? rankR(alive, frep) : -1;
  }
  return mr;
}

__device__ __forceinline__ int reducedVectors(unsigned long long alive, int rep, int lane, double& b, double& lo,
                                              double& hi, int& fi, int& act) {
  const unsigned long long al[1] = {alive};
  const int ra[1] = {rep};
  double ba[1] = {b}, la[1] = {lo}, ha[1] = {hi};
  int fa[1] = {fi}, aa[1];
  const int mr = reducedVectorsR<1>(al, ra, lane, ba, la, ha, fa, aa);
  b = ba[0]; lo = la[0]; hi = ha[0]; fi = fa[0]; act = aa[0];
  return mr;
}

// Dantzig's view of the reduced matrix: ODE's dLCP reads only the lower
// triangle of the (row-major) A it is given (swapRowsAndCols / GETA,
// lcp.cpp:144, matrix.cpp:371), i.e. the symmetric S[r][s] =
// A_r[max(r,s)][min(r,s)] = A[i][j] * scl_{act_min(r,s)}; written to M
// (mr x mr).  PGS reads rows (PgsBoxedLcpSolver.cpp:139): its copy is the
// transpose T[s][r] = A_r[r][s] (wavePgs reads row i, lane j as A_ji).
template <bool kLds, int R>
__device__ void reducedMatrixR(int m, typename Space<kLds>::cdptr Ain, double shift,
                               const unsigned long long (&alive)[R], const int (&act)[R], const double (&scl)[R],
                               typename Space<kLds>::dptr Mout, bool forPgs, int lane) {
  m = uni(m);
  const int mr = popR(alive);
  const double* A = (const double*)Ain;
  double* M = (double*)Mout;
  double sclAct[R];  // scale of the row's reduced column / row
#pragma unroll
  for (int s = 0; s < R; s++) sclAct[s] = gatherR(scl, rowAt(s, lane) < mr ? act[s] : 0);
  for (int r = 0; r < mr; r++) {
    const int i = rdliR(act, r);
    const double si = rdlR(sclAct, r);
#pragma unroll
    for (int s = 0; s < R; s++) {
      const int row = rowAt(s, lane);
      if (row < mr) {
        const int j = act[s];
        const double v = A[i * m + j] + (i == j ? shift : 0.0);
        // forPgs: T[r][row] = A_r[row][r] = (A[j][i] + ...) * scl_i
        // Dantzig: S[r][row] = A[i][j] * scl_{act_min(r, row)}
        M[r * mr + row] = forPgs ? v * si : v * (r < row ? si : sclAct[s]);
      }
    }
  }
  WSYNC();
}

template <bool kLds>
__device__ void reducedMatrix(int m, typename Space<kLds>::cdptr Ain, double shift, unsigned long long alive,
                              int act, double scl, typename Space<kLds>::dptr Mout, bool forPgs, int lane) {
  const unsigned long long al[1] = {alive};
  const int aa[1] = {act};
  const double sa[1] = {scl};
  reducedMatrixR<kLds, 1>(m, Ain, shift, al, aa, sa, Mout, forPgs, lane);
}
