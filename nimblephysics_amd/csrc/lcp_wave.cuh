// Wave-parallel LCP kernels for one world per 64-lane wave.  Vectors of the
// (<= 48-row) LCP live one element per lane in registers, matrices in LDS;
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
#pragma once
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
template <bool kLds, bool kMapped = false>
__device__ bool wavePgs(int n, typename Space<kLds>::cdptr Ain, double& x, double b, double lo, double hi, int findex,
                        int lane, double* dbg = nullptr, double shift = 0.0, const int* cancel = nullptr, int ld = -1,
                        int idx = -1) {
  n = uni(n);
  if (n == 0) return true;
  ld = kMapped ? uni(ld) : n;
  if (!kMapped) idx = lane;
  const double* A = (const double*)Ain;
  const double deltaXThr = 1e-6, relTol = 1e-3, epsDiv = 1e-9;
#ifdef LCP_PROFILE
  const long long tp0 = (long long)__builtin_amdgcn_s_memtime();
#endif
  const bool act = lane < n;
  const int col = act ? idx : rdli(idx, 0);  // idle lanes read a valid address, use 0
  const double diagRaw = act ? A[col * ld + col] + shift : 1.0;
  const unsigned long long order = __ballot(act && diagRaw >= epsDiv);
  const bool inOrder = act && ((order >> lane) & 1ull);
  // rows whose x bounds friction rows (their update refreshes those bounds)
  unsigned long long bounding = 0;
  for (int i = 0; i < n; i++)
    if (__ballot(findex == i)) bounding |= 1ull << i;
  double r = act ? b : 0.0;
  for (int k = 0; k < n; k++) {
    const double xk = rdl(x, k);
    const double a0 = A[(kMapped ? rdli(idx, k) : k) * ld + col];
    if (act) r -= (k == lane ? a0 + shift : a0) * xk;
  }
  // Contact layout (the forward's rows: each contact is a normal row
  // followed by 0 or 2 friction rows with findex = that normal and
  // lo = -hi), every row in order: the friction box of row i is
  // +-hi_i * x_N with x_N the newest x of the last normal row, which the
  // sweep carries as one scalar -- no per-lane box registers.
  bool contactRows = order == __ballot(act);
  {
    const int f1 = __shfl(findex, lane > 0 ? lane - 1 : 0), f2 = __shfl(findex, lane > 1 ? lane - 2 : 0);
    const bool ok = !act || findex < 0 ||
                    (lo == -hi && ((findex == lane - 1 && f1 < 0) || (findex == lane - 2 && f1 == lane - 2 && f2 < 0)));
    contactRows = contactRows && !__ballot(!ok);
  }
  const unsigned long long normals = __ballot(act && findex < 0);
  if (dbg && lane == 0) dbg[1] = contactRows ? 1 : 0;
#ifdef LCP_PROFILE
  const long long tp1 = (long long)__builtin_amdgcn_s_memtime();
#endif
  // current box of each row; friction rows track hi * x[findex]
  double hB = hi, lB = lo;
  if (findex >= 0) { hB = hi * __shfl(x, findex); lB = -hB; }
  // Each lane's x changes only at its own row of a sweep, so within a sweep
  // lane i still holds its sweep-start value x0 when row i is visited, and
  // the reference's per-row "moved" test can be evaluated for all rows at
  // once after the sweep (same operands, same outcome).  The row loop then
  // carries only clamp -> readlane -> residual update.  Rows of A (symmetric,
  // row i lane j = A_ji) are loaded one 4-row group ahead, so LDS latency is
  // off the dependent chain.
  const double x0 = x;
  const double act1 = act ? 1.0 : 0.0;
  double xn = x;
  const int nLast = n - 1;
#define PGS_ROW_AT(i) ((kMapped ? rdli(idx, (i) < n ? (i) : nLast) : ((i) < n ? (i) : nLast)) * ld + col)
#define PGS_LOAD_GROUP(R, i0)               \
  double R##0 = A[PGS_ROW_AT(i0)];         \
  double R##1 = A[PGS_ROW_AT((i0) + 1)];   \
  double R##2 = A[PGS_ROW_AT((i0) + 2)];   \
  double R##3 = A[PGS_ROW_AT((i0) + 3)]
  {
    auto row1 = [&](int i, double cur) {
      double nx = 0.0;
      if ((order >> i) & 1ull) {
        nx = (r + diagRaw * x0) / diagRaw;
        nx = nx > hB ? hB : (nx < lB ? lB : nx);
      }
      const double dx = rdl(nx - x0, i);
      if (lane == i) xn = nx;
      if ((bounding >> i) & 1ull) {
        const double nxi = rdl(nx, i);
        if (findex == i) { hB = hi * nxi; lB = -hB; }
      }
      r -= (cur * act1) * dx;
    };
    double xN = 0.0;
    // (the row kind is a scalar bit: the branch never waits on VALU results;
    // x_N is only consumed by VALU multiplies, never by SALU)
    auto row1c = [&](int i, double cur) {
      double h = hi, l = lo;
      if (!((normals >> i) & 1ull)) { h = hi * xN; l = lo * xN; }
      double nx = (r + diagRaw * x0) / diagRaw;
      const double t = nx < l ? l : nx;
      nx = nx > h ? h : t;
      const double dx = rdl(nx - x0, i);
      if ((normals >> i) & 1ull) xN = rdl(nx, i);
      if (lane == i) xn = nx;
      r -= (cur * act1) * dx;
    };
    PGS_LOAD_GROUP(C, 0);
    if (contactRows) {
      for (int i0 = 0; i0 < n; i0 += 4) {
        PGS_LOAD_GROUP(N, i0 + 4);
        row1c(i0, C0);
        if (i0 + 1 < n) row1c(i0 + 1, C1);
        if (i0 + 2 < n) row1c(i0 + 2, C2);
        if (i0 + 3 < n) row1c(i0 + 3, C3);
        C0 = N0; C1 = N1; C2 = N2; C3 = N3;
      }
    } else {
      for (int i0 = 0; i0 < n; i0 += 4) {
        PGS_LOAD_GROUP(N, i0 + 4);
        row1(i0, C0);
        if (i0 + 1 < n) row1(i0 + 1, C1);
        if (i0 + 2 < n) row1(i0 + 2, C2);
        if (i0 + 3 < n) row1(i0 + 3, C3);
        C0 = N0; C1 = N1; C2 = N2; C3 = N3;
      }
    }
    // the shift's share of the diagonal updates, deferred: lane i's residual
    // is not read again before its own row in the next sweep
    if (shift != 0.0 && act) r -= shift * (xn - x0);
  }
#ifdef LCP_PROFILE
  const long long tp2 = (long long)__builtin_amdgcn_s_memtime();
  if (dbg && lane == 0) { dbg[2] = (double)(tp1 - tp0); dbg[3] = (double)(tp2 - tp1); }
#endif
  if (!__ballot(inOrder && fabs(xn - x0) > deltaXThr)) { x = xn; return true; }
  // row scaling of the reference, lane-local: A'_jk = A_jk * dummy_j
  const double dummy = inOrder ? 1.0 / diagRaw : 1.0;
  if (inOrder) { b *= dummy; r *= dummy; }
  const double diag = inOrder ? diagRaw * dummy : diagRaw;
  const double dummyAct = act ? dummy : 0.0;
  bool possible = false;
  for (int iter = 1; iter < 30; iter++) {
    const double xs = xn;
    auto row = [&](int idx, double cur) {
      if (!((order >> idx) & 1ull)) return;
      double nx = r + diag * xs;
      nx = nx > hB ? hB : (nx < lB ? lB : nx);
      const double dx = rdl(nx - xs, idx);
      if (lane == idx) xn = nx;
      if ((bounding >> idx) & 1ull) {
        const double nxi = rdl(nx, idx);
        if (findex == idx) { hB = hi * nxi; lB = -hB; }
      }
      r -= (cur * dummyAct) * dx;
    };
    double xN = 0.0;
    auto rowc = [&](int idx, double cur) {
      double h = hi, l = lo;
      if (!((normals >> idx) & 1ull)) { h = hi * xN; l = lo * xN; }
      double nx = r + diag * xs;
      const double t = nx < l ? l : nx;
      nx = nx > h ? h : t;
      const double dx = rdl(nx - xs, idx);
      if ((normals >> idx) & 1ull) xN = rdl(nx, idx);
      if (lane == idx) xn = nx;
      r -= (cur * dummyAct) * dx;
    };
    PGS_LOAD_GROUP(C, 0);
    if (contactRows) {
      for (int i0 = 0; i0 < n; i0 += 4) {
        PGS_LOAD_GROUP(N, i0 + 4);
        rowc(i0, C0);
        if (i0 + 1 < n) rowc(i0 + 1, C1);
        if (i0 + 2 < n) rowc(i0 + 2, C2);
        if (i0 + 3 < n) rowc(i0 + 3, C3);
        C0 = N0; C1 = N1; C2 = N2; C3 = N3;
      }
    } else {
      for (int i0 = 0; i0 < n; i0 += 4) {
        PGS_LOAD_GROUP(N, i0 + 4);
        row(i0, C0);
        if (i0 + 1 < n) row(i0 + 1, C1);
        if (i0 + 2 < n) row(i0 + 2, C2);
        if (i0 + 3 < n) row(i0 + 3, C3);
        C0 = N0; C1 = N1; C2 = N2; C3 = N3;
      }
    }
    if (shift != 0.0) r -= (shift * dummyAct) * (xn - xs);
    possible = !__ballot(inOrder && fabs(xn) > epsDiv && fabs((xn - xs) / xn) > relTol);
    if (dbg && lane == 0) dbg[0] = iter;
    if (possible) break;
    if (cancel && uni(__hip_atomic_load(cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))) break;
  }
#undef PGS_LOAD_GROUP
#undef PGS_ROW_AT
#ifdef LCP_PROFILE
  if (dbg && lane == 0) dbg[4] = (double)((long long)__builtin_amdgcn_s_memtime() - tp2);
#endif
  x = xn;
  return possible;
}

// ---------------------------------------------------------------------------
template <bool kLds>
__device__ bool waveLcpValid(int m, typename Space<kLds>::cdptr Ain, double cfm, double x, double b, double hi,
                             double lo, int fi, bool ignoreFriction, int lane) {
  m = uni(m);
  const double* A = (const double*)Ain;
  double v = -b;
#pragma unroll 4
  for (int j = 0; j < m; j++) {
    const double xj = rdl(x, j);
    if (lane < m) v += (A[j * m + lane] + (lane == j ? cfm : 0.0)) * xj;  // A symmetric: row j
  }
  const double xf = __shfl(x, fi >= 0 ? fi : 0);
  bool ok = true;
  if (lane < m) {
    double up = hi, low = lo;
    bool done = false;
    if (fi != -1) {
      if (ignoreFriction) { ok = (x == 0); done = true; }
      up *= xf;
      low *= xf;
    }
    if (!done) {
      const double tol = 1e-5;
      if (fabs(low) < tol && fabs(up) < tol && fabs(x) < tol) {
      } else if (fabs(x - low) < tol) {
        if (v < -tol) ok = false;
      } else if (fabs(x - up) < tol) {
        if (v > tol) ok = false;
      } else if (x > low && x < up) {
        if (fabs(v) > tol) ok = false;
      } else {
        ok = false;
      }
    }
  }
  return __ballot(!ok) == 0ull;
}

// ---------------------------------------------------------------------------
// x (lane-distributed, length c.n) = min-norm least-squares solution for rhs
// (lane-distributed, length c.m).  scr: >= n doubles of LDS.
// (A, ws, m, n, ld) as given to carveCod + codFactor
template <bool kLds>
__device__ double codSolveWave(typename Space<kLds>::dptr Ain, typename Space<kLds>::dptr wsIn, int m_, int n_, int ld_,
                               double rhs, typename Space<kLds>::dptr scrIn, int lane) {
  Cod c;
  carveCod((double*)wsIn, (double*)Ain, uni(m_), uni(n_), uni(ld_), c);
  double* scr = (double*)scrIn;
  const double* A = c.A;
  const int m = c.m, n = c.n, ld = c.ld;
  for (int k = 0; k < c.kmax; k++) {
    const double vnorm = unid(c.vn[k]);
    if (!(vnorm > 0)) continue;
    const double vk = c.vd[k];
    const double v = lane == k ? vk : ((lane > k && lane < m) ? A[lane * ld + k] : 0.0);
    double sc = waveSum(v * rhs);
    sc = 2 * sc / vnorm;
    if (lane >= k && lane < m) rhs -= sc * v;
  }
  const int r = uni(*c.rank);
  double z = 0.0, acc = 0.0;
  for (int i = r - 1; i >= 0; i--) {
    const double zi = (rdl(rhs, i) - rdl(acc, i)) / A[i * ld + i];
    if (lane == i) z = zi;
    if (lane < i) acc += A[lane * ld + i] * zi;
  }
  if (r < n) {
    for (int i = 0; i < r; i++) {
      const double vn = unid(c.zn[i]);
      if (vn == 0) continue;
      const double zd = c.zd[i];
      const double t = (lane >= r && lane < n) ? z * A[i * ld + lane] : 0.0;
      double sc = rdl(z, i) * zd + waveSum(t);
      sc = 2 * sc / vn;
      if (lane == i) z -= sc * zd;
      if (lane >= r && lane < n) z -= sc * A[i * ld + lane];
    }
  }
  WSYNC();
  if (lane < n) scr[c.perm[lane]] = z;
  WSYNC();
  const double out = lane < n ? scr[lane] : 0.0;
  WSYNC();
  return out;
}

// ---------------------------------------------------------------------------
struct WaveDantzig {
  int n, nC, nN, lane, ldL;
  // A: the problem matrix (n x n, symmetric, LDS), read in place: slot i of
  // the permuted problem is original row p_i (lane i's register p), so the
  // permuted entry (i, j) is A[p_i n + p_j] and a swap of two slots is a
  // swap of registers -- the same values the reference's physically
  // permuted matrix holds (dLCP's row / column swaps), without moving them
  const double* A;
  double* L;    // n x ldL, ldL odd (LDS bank-conflict-free columns)
  double* scr;  // >= n doubles (LDS)
  double x, b, w, lo, hi, d, deltaX, deltaW, Dell, ell;
  int findex, p, C, state;
#ifdef LCP_PROFILE
  long long prof[8];
#endif

  __device__ __forceinline__ void swapReg(double& v, int i1, int i2) {
    const double a = rdl(v, i1), c = rdl(v, i2);
    if (lane == i1) v = c;
    else if (lane == i2) v = a;
  }
  __device__ __forceinline__ void swapRegI(int& v, int i1, int i2) {
    const int a = rdli(v, i1), c = rdli(v, i2);
    if (lane == i1) v = c;
    else if (lane == i2) v = a;
  }
  // permuted-matrix accessors: row slot i (wave-uniform), column of this
  // lane's slot / of its C entry / the diagonal
  __device__ __forceinline__ int rowOff(int i) const { return rdli(p, i) * n; }
  __device__ __forceinline__ double Arow(int i) const { return A[rowOff(i) + (lane < n ? p : 0)]; }
  __device__ __forceinline__ double Adiag(int i) const {
    const int pi = rdli(p, i);
    return A[pi * n + pi];
  }
  // p of the slot this lane's C entry names
  __device__ __forceinline__ int pOfC() const { return __shfl(p, C & 63); }
  __device__ __forceinline__ void swapProblem(int i1, int i2) {
    if (i1 == i2) return;
    LP_BEGIN();
    swapReg(x, i1, i2); swapReg(b, i1, i2); swapReg(w, i1, i2); swapReg(lo, i1, i2); swapReg(hi, i1, i2);
    swapRegI(p, i1, i2); swapRegI(state, i1, i2); swapRegI(findex, i1, i2);
    LP_END(prof, 0);
  }
  // L x = B (unit lower), B lane-distributed, first m entries.  The L
  // entries of each lane are loaded 8 at a time ahead of the dependent
  // readlane -> FMA chain (LDS latency paid once per 8 steps) with the
  // triangle mask folded into them (0 where a lane must not change), so a
  // step is a readlane and one unpredicated FMA: no exec-mask update that
  // would wait on a vector compare.  0 * b_k leaves a lane unchanged only
  // for finite b_k; a non-finite b_k (degenerate factor) re-runs the solve
  // predicated, exactly as the reference's loop.
  __device__ __forceinline__ void solveL1(double& B, int m) {
    m = uni(m);
    LP_BEGIN();
    const double B0 = B;
    const int row = (lane < m ? lane : 0) * ldL;
    for (int k0 = 0; k0 < m; k0 += 8) {
      double Lk[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        double v = L[row + (k0 + u < m ? k0 + u : 0)];
        asm volatile("" : "+v"(v));  // keep the load unconditional (batched)
        Lk[u] = (lane > k0 + u && lane < m) ? v : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; u++)
        if (k0 + u < m) B -= Lk[u] * rdl(B, k0 + u);
    }
    if (__ballot(lane < m && !isfinite(B))) {
      B = B0;
      for (int k = 0; k < m; k++) {
        const double bk = rdl(B, k);
        if (lane > k && lane < m) B -= L[lane * ldL + k] * bk;
      }
    }
    LP_END(prof, 1);
  }
  // L^T x = B
  __device__ __forceinline__ void solveL1T(double& B, int m) {
    m = uni(m);
    LP_BEGIN();
    const double B0 = B;
    const int col = lane < m ? lane : 0;
    for (int k0 = m - 1; k0 >= 0; k0 -= 8) {
      double Lk[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        double v = L[(k0 - u >= 0 ? k0 - u : 0) * ldL + col];
        asm volatile("" : "+v"(v));
        Lk[u] = lane < k0 - u ? v : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; u++)
        if (k0 - u >= 0) B -= Lk[u] * rdl(B, k0 - u);
    }
    if (__ballot(lane < m && !isfinite(B))) {
      B = B0;
      for (int k = m - 1; k >= 0; k--) {
        const double bk = rdl(B, k);
        if (lane < k) B -= L[k * ldL + lane] * bk;
      }
    }
    LP_END(prof, 2);
  }
  __device__ __forceinline__ void transferToC(int i) {
    const double Aii = Adiag(i);
    if (nC > 0) {
      if (lane < nC) L[nC * ldL + lane] = ell;
      const double dd = waveSum(lane < nC ? ell * Dell : 0.0);
      if (lane == nC) d = 1.0 / (Aii - dd);
    } else {
      if (lane == 0) d = 1.0 / Aii;
    }
    swapProblem(nC, i);
    if (lane == nC) C = nC;
    nC++;
  }
  __device__ __forceinline__ void transferFromNtoC(int i) {
    const double Aii = Adiag(i);
    if (nC > 0) {
      const int pc = pOfC();
      Dell = lane < nC ? A[rowOff(i) + pc] : 0.0;
      solveL1(Dell, nC);
      ell = lane < nC ? Dell * d : 0.0;
      if (lane < nC) L[nC * ldL + lane] = ell;
      const double dd = waveSum(lane < nC ? ell * Dell : 0.0);
      if (lane == nC) d = 1.0 / (Aii - dd);
    } else {
      if (lane == 0) d = 1.0 / Aii;
    }
    swapProblem(nC, i);
    if (lane == nC) C = nC;
    nN--;
    nC++;
  }
  // _dLDLTAddTL on the sub-factorisation starting at (r, r); `a` holds
  // element j at lane r + j
  __device__ __forceinline__ void ldltAddTL(int r, int m2, double a) {
    if (m2 < 2) return;
    const double r2 = 0.70710678118654752440;
    const int j0 = lane - r;
    double W1 = 0.0, W2 = 0.0;
    if (j0 >= 1 && j0 < m2) { W1 = a * r2; W2 = W1; }
    const double a0 = rdl(a, r);
    const double W11 = (0.5 * a0 + 1) * r2;
    const double W21 = (0.5 * a0 - 1) * r2;
    double alpha1 = 1.0, alpha2 = 1.0;
    {
      double dee = rdl(d, r);
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
      if (j0 >= 1 && j0 < m2) {
        const double Wp = W1;
        const double el = L[(r + j0) * ldL + r];
        W1 = Wp - W11 * el;
        W2 = k1 * Wp + k2 * el;
      }
    }
    for (int j = 1; j < m2; j++) {
      const double k1 = rdl(W1, r + j), k2 = rdl(W2, r + j);
      double dee = rdl(d, r + j);
      double alphanew = alpha1 + (k1 * k1) * dee;
      dee /= alphanew;
      const double gamma1 = k1 * dee;
      dee *= alpha1;
      alpha1 = alphanew;
      alphanew = alpha2 - (k2 * k2) * dee;
      dee /= alphanew;
      const double gamma2 = k2 * dee;
      dee *= alpha2;
      if (lane == r + j) d = dee;
      alpha2 = alphanew;
      if (j0 > j && j0 < m2) {
        double el = L[(r + j0) * ldL + r + j];
        double Wp = W1 - k1 * el;
        el += gamma1 * Wp;
        W1 = Wp;
        Wp = W2 - k2 * el;
        el -= gamma2 * Wp;
        W2 = Wp;
        L[(r + j0) * ldL + r + j] = el;
      }
    }
  }
  __device__ __forceinline__ void ldltRemove(int r, int n2) {
    LP_BEGIN();
    if (r != n2 - 1) {
      const int pc = pOfC();
      if (r == 0) {
        const int C0 = rdli(C, 0);
        double a = lane < n2 ? -A[rowOff(C0) + pc] : 0.0;  // A symmetric
        if (lane == 0) a += 1.0;
        ldltAddTL(0, n2, a);
      } else {
        const double t = lane < r ? L[r * ldL + lane] / d : 0.0;
        const int Cr = rdli(C, r);
        double a = 0.0;
        double s = 0.0;
        for (int k = 0; k < r; k++) {
          const double tk = rdl(t, k);
          if (lane >= r && lane < n2) s += L[lane * ldL + k] * tk;
        }
        if (lane >= r && lane < n2) a = s - A[rowOff(Cr) + pc];  // A symmetric
        if (lane == r) a += 1.0;
        ldltAddTL(r, n2 - r, a);
      }
    }
    WSYNC();
    if (r < n2 - 1) {
      if (lane < n2)
        for (int j = r; j < n2 - 1; j++) L[lane * ldL + j] = L[lane * ldL + j + 1];
      WSYNC();
      if (lane < n2)
        for (int i = r; i < n2 - 1; i++) L[i * ldL + lane] = L[(i + 1) * ldL + lane];
      WSYNC();
      const double dn = shiftDown1(d, lane);
      if (lane >= r && lane < n2 - 1) d = dn;
    }
    LP_END(prof, 3);
  }
  __device__ __forceinline__ void transferFromCtoN(int i) {
    const int j = waveFirst(lane < nC && C == i);
    if (j >= 0) {
      const int k = waveFirst(lane < nC && C == nC - 1);
      ldltRemove(j, nC);
      const int Cj = rdli(C, j);
      if (lane == k) C = Cj;
      const int Cn = shiftDown1i(C, lane);
      if (lane >= j && lane < nC - 1) C = Cn;
    }
    swapProblem(i, nC - 1);
    nN++;
    nC--;
  }
  __device__ __forceinline__ void solve1(int i, int dir, bool onlyTransfer) {
    if (nC > 0) {
      const int pc = pOfC();
      Dell = lane < nC ? A[rowOff(i) + pc] : 0.0;
      solveL1(Dell, nC);
      ell = lane < nC ? Dell * d : 0.0;
      if (!onlyTransfer) {
        double tmp = ell;
        solveL1T(tmp, nC);
        WSYNC();
        if (lane < nC) scr[C] = dir > 0 ? -tmp : tmp;
        WSYNC();
        if (lane < nC) deltaX = scr[lane];
        WSYNC();
      }
    }
  }
  __device__ __forceinline__ double AiC(int i, double q) { return waveSum(lane < nC ? Arow(i) * q : 0.0); }
  __device__ __forceinline__ double AiN(int i, double q) {
    return waveSum((lane >= nC && lane < nC + nN) ? Arow(i) * q : 0.0);
  }
};

// A (n x n LDS, symmetric, read only), L (n x (n|1) LDS scratch), scr (>= n
// LDS); problem vectors lane-distributed; returns success and x
// (lane-distributed).
template <bool kLds>
__device__ bool waveDantzig(int n, typename Space<kLds>::cdptr Ain, typename Space<kLds>::dptr Lin,
                            typename Space<kLds>::dptr scrIn, double& xOut, double b, double lo, double hi,
                            int findex, int lane, double* dbg = nullptr, const int* cancel = nullptr) {
  n = uni(n);
  const double* A = (const double*)Ain;
  double* Lbuf = (double*)Lin;
  double* scr = (double*)scrIn;
  WaveDantzig D;
  int pivots = 0;
  D.n = n; D.nC = 0; D.nN = 0; D.lane = lane; D.ldL = n | 1;
  D.A = A; D.L = Lbuf; D.scr = scr;
  D.x = 0.0; D.b = b; D.w = 0.0; D.lo = lo; D.hi = hi; D.d = 0.0;
  D.deltaX = 0.0; D.deltaW = 0.0; D.Dell = 0.0; D.ell = 0.0;
  D.findex = findex; D.p = lane; D.C = 0; D.state = 0;
#ifdef LCP_PROFILE
  for (int k = 0; k < 8; k++) D.prof[k] = 0;
#endif
  for (int k = lane; k < n * (n | 1); k += 64) Lbuf[k] = 0.0;
  if (__ballot(lane < n && findex < 0 && lo == -LCP_INF && hi == LCP_INF)) return false;
  {
    int numAtEnd = 0;
    for (int k = n - 1; k >= 0; k--)
      if (rdli(D.findex, k) >= 0) { D.swapProblem(k, n - 1 - numAtEnd); numAtEnd++; }
  }
  WSYNC();
  bool hitFirstFriction = false;
  for (int i = 0; i < n; i++) {
    D.nC = uni(D.nC);
    D.nN = uni(D.nN);
    if (!hitFirstFriction && rdli(D.findex, i) >= 0) {
      WSYNC();
      if (lane < n) scr[D.p] = D.x;
      WSYNC();
      if (lane >= i && lane < n) {
        const double wfk = scr[D.findex];
        if (wfk == 0) { D.hi = 0; D.lo = 0; }
        else { D.hi = fabs(D.hi * wfk); D.lo = -D.hi; }
      }
      WSYNC();
      hitFirstFriction = true;
    }
    LP_BEGIN();
    const double wi = D.AiC(i, D.x) + D.AiN(i, D.x) - rdl(D.b, i);
    LP_END(D.prof, 4);
    if (lane == i) D.w = wi;
    const double loi = rdl(D.lo, i), hii = rdl(D.hi, i);
    if (loi == 0 && wi >= 0) {
      D.nN++;
      if (lane == i) D.state = 0;
    } else if (hii == 0 && wi <= 0) {
      D.nN++;
      if (lane == i) D.state = 1;
    } else if (wi == 0) {
      D.solve1(i, 0, true);
      D.transferToC(i);
    } else {
      for (;;) {
        D.nC = uni(D.nC);
        D.nN = uni(D.nN);
        const double wiNow = rdl(D.w, i);
        int dir;
        double dirf;
        if (wiNow <= 0) { dir = 1; dirf = 1.0; } else { dir = -1; dirf = -1.0; }
        D.solve1(i, dir, false);
        const int nC = D.nC, nN = D.nN;
        const bool inN = lane >= nC && lane < nC + nN;
        LP_BEGIN();
        {
          // every lane accumulates (no exec mask per step); only N lanes keep it
          const int colA = lane < n ? D.p : 0;
          double acc = 0.0;
#pragma unroll 4
          for (int j = 0; j < nC; j++) {
            const double dxj = rdl(D.deltaX, j);
            acc += A[D.rowOff(j) + colA] * dxj;  // A symmetric: row j
          }
          const double aij = D.Arow(i);
          if (inN) D.deltaW = acc + (dir > 0 ? aij : -aij);
        }
        const double dwi = D.AiC(i, D.deltaX) + D.Adiag(i) * dirf;
        if (lane == i) D.deltaW = dwi;
        int cmd = 1, si = 0;
        double s = -wiNow / dwi;
        const double xi = rdl(D.x, i), hiI = rdl(D.hi, i), loI = rdl(D.lo, i);
        if (dir > 0) {
          if (hiI < LCP_INF) { const double s2 = (hiI - xi) * dirf; if (s2 < s) { s = s2; cmd = 3; } }
        } else {
          if (loI > -LCP_INF) { const double s2 = (loI - xi) * dirf; if (s2 < s) { s = s2; cmd = 2; } }
        }
        {
          // the N-side (cmd 4) and C-side (cmd 5/6) ratio tests of the
          // reference over disjoint lanes: one division and one reduction;
          // on equal minima the N side wins, as in the reference's order
          bool cand4 = false;
          int typ = 0;
          double num = 0.0, den = 1.0;
          if (inN) {
            const bool dirOk = !D.state ? D.deltaW < 0 : D.deltaW > 0;
            if (dirOk && !(D.lo == 0 && D.hi == 0)) { cand4 = true; num = -D.w; den = D.deltaW; }
          } else if (lane < nC) {
            if (D.deltaX < 0 && D.lo > -LCP_INF) { num = D.lo - D.x; den = D.deltaX; typ = 5; }
            if (D.deltaX > 0 && D.hi < LCP_INF) { num = D.hi - D.x; den = D.deltaX; typ = 6; }
          }
          const double r = num / den;
          const bool any = cand4 || typ;
          const double mm = waveMin(any ? r : LCP_INF);
          if (mm < s) {
            s = mm;
            const int s4i = waveFirst(cand4 && r == mm);
            if (s4i >= 0) {
              cmd = 4;
              si = s4i;
            } else {
              si = waveFirst(typ && r == mm);
              cmd = rdli(typ, si);
            }
          }
        }
        pivots++;
        if (dbg && lane == 0) { dbg[0] = pivots; dbg[1] = i; }
        LP_END(D.prof, 5);
#ifdef LCP_PROFILE
        if (dbg && lane == 0)
          for (int k = 0; k < 8; k++) dbg[2 + k] = (double)D.prof[k];
#endif
        if (s <= 0.0) return false;
        // `cancel` (LDS int, optional): polled once per pivot; a set flag
        // abandons the solve (the caller no longer needs it)
        if (cancel && uni(__hip_atomic_load(cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))) return false;
        if (lane < nC) D.x += s * D.deltaX;
        if (lane == i) D.x += s * dirf;
        if (inN) D.w += s * D.deltaW;
        if (lane == i) D.w += s * dwi;
        switch (cmd) {
          case 1:
            if (lane == i) D.w = 0;
            D.transferToC(i);
            break;
          case 2:
            if (lane == i) { D.x = D.lo; D.state = 0; }
            D.nN++;
            break;
          case 3:
            if (lane == i) { D.x = D.hi; D.state = 1; }
            D.nN++;
            break;
          case 4:
            if (lane == si) D.w = 0;
            D.transferFromNtoC(si);
            break;
          case 5:
            if (lane == si) { D.x = D.lo; D.state = 0; }
            D.transferFromCtoN(si);
            break;
          case 6:
            if (lane == si) { D.x = D.hi; D.state = 1; }
            D.transferFromCtoN(si);
            break;
        }
        if (cmd <= 3) break;
      }
    }
  }
  WSYNC();
  if (lane < n) scr[D.p] = D.x;
  WSYNC();
  xOut = lane < n ? scr[lane] : 0.0;
  WSYNC();
  return true;
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
// (the PGS fallback reduces A + cfm I).  Lane i holds original row i's b, lo,
// hi and findex.  Returns (wave-uniform) the mask of surviving rows; lane i
// gets scl (its column scale, 1 for a removed row) and rep (the surviving row
// row i was merged into).  `maxMerges` = 0 only reports whether a merge
// exists (return value != the full mask).
// ---------------------------------------------------------------------------
template <bool kLds>
__device__ unsigned long long waveReduce(int m, typename Space<kLds>::cdptr Ain, double shift, double b, double lo,
                                         double hi, int fi, int lane, double& scl, int& rep, int maxMerges = 64) {
  m = uni(m);
  const double* A = (const double*)Ain;
  unsigned long long alive = m >= 64 ? ~0ull : ((1ull << m) - 1ull);
  scl = 1.0;
  rep = lane;
  const int col = lane < m ? lane : 0;
  for (int merges = 0; merges <= maxMerges; merges++) {
    // findex in terms of surviving rows (the reference remaps fIndex on
    // every merge; comparing representatives is the same test)
    const int fr = __shfl(rep, fi >= 0 ? fi : 0);
    const int frow = fi >= 0 ? fr : -1;
    const bool me = lane < m && ((alive >> lane) & 1ull);
    int hitC = 64;
    for (int c = 1; c < m; c++) {
      if (!((alive >> c) & 1ull)) continue;
      const double bc = rdl(b, c), loc = rdl(lo, c), hic = rdl(hi, c), sc = rdl(scl, c);
      const int fc = rdli(frow, c);
      bool cand = me && lane < c && hitC == 64 && fabs(b - bc) < 1e-4 && frow == fc && hi == hic && lo == loc;
      if (__ballot(cand)) {
        double dd = 0.0;
        for (int i = 0; i < m; i++) {
          if (!((alive >> i) & 1ull)) continue;
          const double aa = (A[i * m + col] + (i == lane ? shift : 0.0)) * scl;
          const double ac = (A[i * m + c] + (i == c ? shift : 0.0)) * sc;
          dd += (aa - ac) * (aa - ac);
        }
        if (cand && dd < 1e-4) hitC = c;
      }
    }
    const int a = waveFirst(hitC < 64);
    if (a < 0 || merges == maxMerges) {
      if (a >= 0) alive &= ~(1ull << rdli(hitC, a));  // report only
      break;
    }
    const int cb = rdli(hitC, a);
    alive &= ~(1ull << cb);
    if (lane == a) scl *= 2.0;
    if (rep == cb) rep = a;
  }
  return alive;
}

// rank of original row `row` among the surviving rows (its reduced index)
__device__ __forceinline__ int reducedIndex(unsigned long long alive, int row) {
  return __popcll(alive & ((1ull << row) - 1ull));
}

// the reduced problem's lane-held vectors: lane r gets the values of the r-th
// surviving row (its findex as a reduced index); returns the reduced size
__device__ __forceinline__ int reducedVectors(unsigned long long alive, int rep, int lane, double& b, double& lo,
                                              double& hi, int& fi, int& act) {
  const int mr = __popcll(alive);
  // act_r: the r-th set bit of alive
  act = 0;
  {
    unsigned long long a = alive;
    for (int r = 0; r < mr; r++) {
      const int i = __ffsll((long long)a) - 1;
      if (lane == r) act = i;
      a &= a - 1ull;
    }
  }
  const int src = lane < mr ? act : 0;
  const double nb = __shfl(b, src), nlo = __shfl(lo, src), nhi = __shfl(hi, src);
  const int nfi = __shfl(fi, src);
  const int frep = __shfl(rep, nfi >= 0 ? nfi : 0);
  b = lane < mr ? nb : 0.0;
  lo = lane < mr ? nlo : 0.0;
  hi = lane < mr ? nhi : 0.0;
  fi = (lane < mr && nfi >= 0) ? reducedIndex(alive, frep) : -1;
  return mr;
}

// Dantzig's view of the reduced matrix: ODE's dLCP reads only the lower
// triangle of the (row-major) A it is given (swapRowsAndCols / GETA,
// lcp.cpp:144, matrix.cpp:371), i.e. the symmetric S[r][s] =
// A_r[max(r,s)][min(r,s)] = A[i][j] * scl_{act_min(r,s)}; written to M
// (mr x mr).  PGS reads rows (PgsBoxedLcpSolver.cpp:139): its copy is the
// transpose T[s][r] = A_r[r][s] (wavePgs reads row i, lane j as A_ji).
template <bool kLds>
__device__ void reducedMatrix(int m, typename Space<kLds>::cdptr Ain, double shift, unsigned long long alive,
                              int act, double scl, typename Space<kLds>::dptr Mout, bool forPgs, int lane) {
  m = uni(m);
  const int mr = __popcll(alive);
  const double* A = (const double*)Ain;
  double* M = (double*)Mout;
  const double sclAct = __shfl(scl, lane < mr ? act : 0);  // scale of the lane's reduced column / row
  for (int r = 0; r < mr; r++) {
    const int i = rdli(act, r);
    const double si = rdl(sclAct, r);
    if (lane < mr) {
      const int j = act;
      const double v = A[i * m + j] + (i == j ? shift : 0.0);
      // forPgs: T[r][lane] = A_r[lane][r] = (A[j][i] + ...) * scl_i
      // Dantzig: S[r][lane] = A[i][j] * scl_{act_min(r, lane)}
      M[r * mr + lane] = forPgs ? v * si : v * (r < lane ? si : sclAct);
    }
  }
  WSYNC();
}
