// ORACLE / TEST INFRASTRUCTURE ONLY -- see nimble_oracle.cpp header.
//
// Restatements of
//  * the ODE Dantzig boxed-LCP solver used by the reference
//    (dart/external/odelcpsolver/lcp.cpp:780 dSolveLCP with the dLCP "fast"
//    index-set manipulator :314-770, LDL^T updates matrix.cpp:286 _dLDLTAddTL
//    and :374 _dLDLTRemove).  Pinned against the reference's own compiled
//    solver (oracle/_ref/libodelcp.so) in tests/test_oracle_lcp.py;
//  * the PGS fallback (dart/constraint/PgsBoxedLcpSolver.cpp:85);
//  * Eigen::CompleteOrthogonalDecomposition::solve (min-norm least squares)
//    used by the reference for Q^{-1} b (ConstrainedGroupGradientMatrices.cpp:270).
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "oracle_lcp.hpp"

namespace oracle {

static const double kInf = std::numeric_limits<double>::infinity();

//------------------------------------------------------------------------------
// Complete orthogonal decomposition solve (column-pivoted Householder QR,
// rank by |R_ii| > eps * min(m,n) * max|R_ii|, then RZ on the trapezoid).
// A is m x n row-major.  x (n) = minimum-norm least-squares solution.
void codSolve(const double* Ain, int m, int nCols, const double* b, double* x) {
  const int n = nCols;
  std::vector<double> A(Ain, Ain + m * n);
  std::vector<int> perm(n);
  for (int j = 0; j < n; j++) perm[j] = j;
  std::vector<double> rhs(b, b + m);
  const int kmax = std::min(m, n);
  std::vector<double> colNorm(n);
  for (int j = 0; j < n; j++) {
    double s = 0;
    for (int i = 0; i < m; i++) s += A[i * n + j] * A[i * n + j];
    colNorm[j] = s;
  }
  double maxPivot = 0;
  for (int k = 0; k < kmax; k++) {
    // pivot: largest remaining column norm
    int p = k;
    double best = -1;
    for (int j = k; j < n; j++) {
      double s = 0;
      for (int i = k; i < m; i++) s += A[i * n + j] * A[i * n + j];
      colNorm[j] = s;
      if (s > best) { best = s; p = j; }
    }
    if (p != k) {
      for (int i = 0; i < m; i++) std::swap(A[i * n + k], A[i * n + p]);
      std::swap(perm[k], perm[p]);
    }
    // Householder on column k, rows k..m-1
    double alpha = 0;
    for (int i = k; i < m; i++) alpha += A[i * n + k] * A[i * n + k];
    alpha = std::sqrt(alpha);
    if (alpha == 0.0) continue;
    if (A[k * n + k] > 0) alpha = -alpha;
    std::vector<double> v(m, 0.0);
    for (int i = k; i < m; i++) v[i] = A[i * n + k];
    v[k] -= alpha;
    double vn = 0;
    for (int i = k; i < m; i++) vn += v[i] * v[i];
    if (vn > 0) {
      for (int j = k; j < n; j++) {
        double s = 0;
        for (int i = k; i < m; i++) s += v[i] * A[i * n + j];
        s = 2 * s / vn;
        for (int i = k; i < m; i++) A[i * n + j] -= s * v[i];
      }
      double s = 0;
      for (int i = k; i < m; i++) s += v[i] * rhs[i];
      s = 2 * s / vn;
      for (int i = k; i < m; i++) rhs[i] -= s * v[i];
    }
    maxPivot = std::max(maxPivot, std::fabs(A[k * n + k]));
  }
  const double thr = std::numeric_limits<double>::epsilon() * kmax * maxPivot;
  int r = 0;
  for (int k = 0; k < kmax; k++)
    if (std::fabs(A[k * n + k]) > thr) r++;
  // R is upper-trapezoidal r x n (rows 0..r-1).  Min-norm solution of
  // R y = c (c = rhs[0..r-1]): y = R^T (R R^T)^{-1} c via RZ (Householder from
  // the right zeroing R[0:r, r:n]).
  std::vector<double> R(r * n, 0.0);
  for (int i = 0; i < r; i++)
    for (int j = i; j < n; j++) R[i * n + j] = A[i * n + j];
  // RZ: for i = r-1..0, reflect row i over columns {i} U {r..n-1}
  std::vector<std::vector<double>> Zv(r);
  std::vector<double> Zvn(r, 0.0);
  for (int i = r - 1; i >= 0 && r < n; i--) {
    double alpha = R[i * n + i] * R[i * n + i];
    for (int j = r; j < n; j++) alpha += R[i * n + j] * R[i * n + j];
    alpha = std::sqrt(alpha);
    if (R[i * n + i] > 0) alpha = -alpha;
    std::vector<double> v(n, 0.0);
    v[i] = R[i * n + i] - alpha;
    for (int j = r; j < n; j++) v[j] = R[i * n + j];
    double vn = v[i] * v[i];
    for (int j = r; j < n; j++) vn += v[j] * v[j];
    Zv[i] = v;
    Zvn[i] = vn;
    if (vn == 0) continue;
    for (int row = 0; row <= i; row++) {
      double s = R[row * n + i] * v[i];
      for (int j = r; j < n; j++) s += R[row * n + j] * v[j];
      s = 2 * s / vn;
      R[row * n + i] -= s * v[i];
      for (int j = r; j < n; j++) R[row * n + j] -= s * v[j];
    }
  }
  // solve T z = c (T = R[0:r,0:r] upper triangular)
  std::vector<double> z(n, 0.0);
  for (int i = r - 1; i >= 0; i--) {
    double s = rhs[i];
    for (int j = i + 1; j < r; j++) s -= R[i * n + j] * z[j];
    z[i] = s / R[i * n + i];
  }
  // y = Z^T [z; 0]: apply reflections in reverse order of construction
  for (int i = 0; i < r && r < n; i++) {
    if (Zvn[i] == 0) continue;
    const std::vector<double>& v = Zv[i];
    double s = z[i] * v[i];
    for (int j = r; j < n; j++) s += z[j] * v[j];
    s = 2 * s / Zvn[i];
    z[i] -= s * v[i];
    for (int j = r; j < n; j++) z[j] -= s * v[j];
  }
  for (int j = 0; j < n; j++) x[perm[j]] = z[j];
}

void pinvSolve(const double* A, const double* b, double* x, int n, double* pinvOut) {
  codSolve(A, n, n, b, x);
  if (pinvOut) {
    std::vector<double> e(n), col(n);
    for (int c = 0; c < n; c++) {
      std::fill(e.begin(), e.end(), 0.0);
      e[c] = 1.0;
      codSolve(A, n, n, e.data(), col.data());
      for (int r = 0; r < n; r++) pinvOut[r * n + c] = col[r];
    }
  }
}

//------------------------------------------------------------------------------
// Dantzig (dSolveLCP) restated on a full, explicitly permuted matrix.
namespace {
struct Dantzig {
  int n, nC = 0, nN = 0, nub;
  std::vector<double> A;  // n x n full symmetric, permuted in place
  double *x, *b, *w, *lo, *hi;
  int* findex;
  std::vector<int> p, C;
  std::vector<char> state;
  std::vector<double> L, d, Dell, ell, tmp;

  double& Aat(int i, int j) { return A[i * n + j]; }

  void swapProblem(int i1, int i2) {
    if (i1 == i2) return;
    for (int k = 0; k < n; k++) std::swap(A[i1 * n + k], A[i2 * n + k]);
    for (int k = 0; k < n; k++) std::swap(A[k * n + i1], A[k * n + i2]);
    std::swap(x[i1], x[i2]);
    std::swap(b[i1], b[i2]);
    std::swap(w[i1], w[i2]);
    std::swap(lo[i1], lo[i2]);
    std::swap(hi[i1], hi[i2]);
    std::swap(p[i1], p[i2]);
    std::swap(state[i1], state[i2]);
    if (findex) std::swap(findex[i1], findex[i2]);
  }
  // L is unit lower triangular n x n (row-major), d holds 1/D
  void solveL1(double* B, int m) {  // L x = B
    for (int i = 0; i < m; i++) {
      double s = B[i];
      for (int k = 0; k < i; k++) s -= L[i * n + k] * B[k];
      B[i] = s;
    }
  }
  void solveL1T(double* B, int m) {  // L^T x = B
    for (int i = m - 1; i >= 0; i--) {
      double s = B[i];
      for (int k = i + 1; k < m; k++) s -= L[k * n + i] * B[k];
      B[i] = s;
    }
  }
  void transferToC(int i) {
    if (nC > 0) {
      for (int j = 0; j < nC; j++) L[nC * n + j] = ell[j];
      double dd = 0;
      for (int j = 0; j < nC; j++) dd += ell[j] * Dell[j];
      d[nC] = 1.0 / (Aat(i, i) - dd);
    } else {
      d[0] = 1.0 / Aat(i, i);
    }
    swapProblem(nC, i);
    C[nC] = nC;
    nC++;
  }
  void transferFromNtoC(int i) {
    if (nC > 0) {
      for (int j = 0; j < nC; j++) Dell[j] = Aat(i, C[j]);
      solveL1(Dell.data(), nC);
      for (int j = 0; j < nC; j++) L[nC * n + j] = ell[j] = Dell[j] * d[j];
      double dd = 0;
      for (int j = 0; j < nC; j++) dd += ell[j] * Dell[j];
      d[nC] = 1.0 / (Aat(i, i) - dd);
    } else {
      d[0] = 1.0 / Aat(i, i);
    }
    swapProblem(nC, i);
    C[nC] = nC;
    nN--;
    nC++;
  }
  // _dLDLTAddTL (matrix.cpp:286) on the sub-factorization starting at (r,r)
  void ldltAddTL(double* Lsub, double* dsub, const double* a, int m) {
    if (m < 2) return;
    std::vector<double> W1(m), W2(m);
    W1[0] = W2[0] = 0.0;
    for (int j = 1; j < m; j++) W1[j] = W2[j] = a[j] * M_SQRT1_2;
    double W11 = (0.5 * a[0] + 1) * M_SQRT1_2;
    double W21 = (0.5 * a[0] - 1) * M_SQRT1_2;
    double alpha1 = 1.0, alpha2 = 1.0;
    {
      double dee = dsub[0];
      double alphanew = alpha1 + (W11 * W11) * dee;
      dee /= alphanew;
      double gamma1 = W11 * dee;
      dee *= alpha1;
      alpha1 = alphanew;
      alphanew = alpha2 - (W21 * W21) * dee;
      dee /= alphanew;
      alpha2 = alphanew;
      double k1 = 1.0 - W21 * gamma1;
      double k2 = W21 * gamma1 * W11 - W21;
      for (int p2 = 1; p2 < m; p2++) {
        double Wp = W1[p2];
        double el = Lsub[p2 * n];
        W1[p2] = Wp - W11 * el;
        W2[p2] = k1 * Wp + k2 * el;
      }
    }
    for (int j = 1; j < m; j++) {
      double k1 = W1[j], k2 = W2[j];
      double dee = dsub[j];
      double alphanew = alpha1 + (k1 * k1) * dee;
      dee /= alphanew;
      double gamma1 = k1 * dee;
      dee *= alpha1;
      alpha1 = alphanew;
      alphanew = alpha2 - (k2 * k2) * dee;
      dee /= alphanew;
      double gamma2 = k2 * dee;
      dee *= alpha2;
      dsub[j] = dee;
      alpha2 = alphanew;
      for (int p2 = j + 1; p2 < m; p2++) {
        double el = Lsub[p2 * n + j];
        double Wp = W1[p2] - k1 * el;
        el += gamma1 * Wp;
        W1[p2] = Wp;
        Wp = W2[p2] - k2 * el;
        el -= gamma2 * Wp;
        W2[p2] = Wp;
        Lsub[p2 * n + j] = el;
      }
    }
  }
  // _dLDLTRemove (matrix.cpp:374) + _dRemoveRowCol
  void ldltRemove(int r, int n2) {
    if (r != n2 - 1) {
      if (r == 0) {
        std::vector<double> a(n2);
        for (int i = 0; i < n2; i++) a[i] = -Aat(C[i], C[0]);
        a[0] += 1.0;
        ldltAddTL(L.data(), d.data(), a.data(), n2);
      } else {
        std::vector<double> t(r), a(n2 - r);
        for (int i = 0; i < r; i++) t[i] = L[r * n + i] / d[i];
        for (int i = 0; i < n2 - r; i++) {
          double s = 0;
          for (int k = 0; k < r; k++) s += L[(r + i) * n + k] * t[k];
          a[i] = s - Aat(C[r + i], C[r]);
        }
        a[0] += 1.0;
        ldltAddTL(L.data() + r * n + r, d.data() + r, a.data(), n2 - r);
      }
    }
    // remove row/col r from L (n2 x n2) and d
    if (r < n2 - 1) {
      for (int i = 0; i < n2; i++)
        for (int j = r; j < n2 - 1; j++) L[i * n + j] = L[i * n + j + 1];
      for (int i = r; i < n2 - 1; i++)
        for (int j = 0; j < n2; j++) L[i * n + j] = L[(i + 1) * n + j];
      for (int i = r; i < n2 - 1; i++) d[i] = d[i + 1];
    }
  }
  void transferFromCtoN(int i) {
    int j = 0, lastIdx = -1;
    for (; j < nC; j++) {
      if (C[j] == nC - 1) lastIdx = j;
      if (C[j] == i) {
        ldltRemove(j, nC);
        int k;
        if (lastIdx == -1) {
          for (k = j + 1; k < nC; k++)
            if (C[k] == nC - 1) break;
        } else {
          k = lastIdx;
        }
        C[k] = C[j];
        for (int t = j; t < nC - 1; t++) C[t] = C[t + 1];
        break;
      }
    }
    swapProblem(i, nC - 1);
    nN++;
    nC--;
  }
  void solve1(double* a, int i, int dir, bool onlyTransfer) {
    if (nC > 0) {
      for (int j = 0; j < nC; j++) Dell[j] = Aat(i, C[j]);
      solveL1(Dell.data(), nC);
      for (int j = 0; j < nC; j++) ell[j] = Dell[j] * d[j];
      if (!onlyTransfer) {
        for (int j = 0; j < nC; j++) tmp[j] = ell[j];
        solveL1T(tmp.data(), nC);
        if (dir > 0)
          for (int j = 0; j < nC; j++) a[C[j]] = -tmp[j];
        else
          for (int j = 0; j < nC; j++) a[C[j]] = tmp[j];
      }
    }
  }
  double AiC_qC(int i, const double* q) { double s = 0; for (int j = 0; j < nC; j++) s += Aat(i, j) * q[j]; return s; }
  double AiN_qN(int i, const double* q) { double s = 0; for (int j = nC; j < nC + nN; j++) s += Aat(i, j) * q[j]; return s; }
};
}  // namespace

bool dantzigSolveLCP(int n, double* Ain /* n x n, row-major, no padding */, double* x, double* b, double* wOut,
                     int nub, double* lo, double* hi, int* findex, bool earlyTermination) {
  Dantzig D;
  D.n = n;
  D.nub = nub;
  D.A.assign(Ain, Ain + n * n);
  std::vector<double> wloc(n, 0.0);
  D.x = x; D.b = b; D.w = wOut ? wOut : wloc.data(); D.lo = lo; D.hi = hi; D.findex = findex;
  D.p.resize(n); D.C.assign(n, 0); D.state.assign(n, 0);
  D.L.assign(n * n, 0.0); D.d.assign(n, 0.0); D.Dell.assign(n, 0.0); D.ell.assign(n, 0.0); D.tmp.assign(n, 0.0);
  for (int k = 0; k < n; k++) { x[k] = 0.0; D.p[k] = k; }
  // unbounded variables first (none for contact LCPs: nub stays 0)
  for (int k = D.nub; k < n; k++) {
    if (findex && findex[k] >= 0) continue;
    if (lo[k] == -kInf && hi[k] == kInf) { D.swapProblem(D.nub, k); D.nub++; }
  }
  if (D.nub > 0) return false;  // not used by the contact solver
  // friction-indexed rows to the end (lcp.cpp:520)
  if (findex) {
    int numAtEnd = 0;
    for (int k = n - 1; k >= D.nub; k--)
      if (findex[k] >= 0) { D.swapProblem(k, n - 1 - numAtEnd); numAtEnd++; }
  }
  std::vector<double> delta_x(n, 0.0), delta_w(n, 0.0);
  double* w = D.w;
  bool hitFirstFriction = false;
  for (int i = D.nub; i < n; i++) {
    bool sError = false;
    if (!hitFirstFriction && findex && findex[i] >= 0) {
      for (int j = 0; j < n; j++) delta_w[D.p[j]] = x[j];
      for (int k = i; k < n; k++) {
        double wfk = delta_w[findex[k]];
        if (wfk == 0) { hi[k] = 0; lo[k] = 0; }
        else { hi[k] = std::fabs(hi[k] * wfk); lo[k] = -hi[k]; }
      }
      hitFirstFriction = true;
    }
    w[i] = D.AiC_qC(i, x) + D.AiN_qN(i, x) - b[i];
    if (lo[i] == 0 && w[i] >= 0) {
      D.nN++;
      D.state[i] = 0;
    } else if (hi[i] == 0 && w[i] <= 0) {
      D.nN++;
      D.state[i] = 1;
    } else if (w[i] == 0) {
      D.solve1(delta_x.data(), i, 0, true);
      D.transferToC(i);
    } else {
      for (;;) {
        int dir;
        double dirf;
        if (w[i] <= 0) { dir = 1; dirf = 1.0; } else { dir = -1; dirf = -1.0; }
        D.solve1(delta_x.data(), i, dir, false);
        // pN = A_NC * qC
        for (int k = 0; k < D.nN; k++) delta_w[D.nC + k] = D.AiC_qC(D.nC + k, delta_x.data());
        for (int k = 0; k < D.nN; k++) delta_w[D.nC + k] += dir > 0 ? D.Aat(i, D.nC + k) : -D.Aat(i, D.nC + k);
        delta_w[i] = D.AiC_qC(i, delta_x.data()) + D.Aat(i, i) * dirf;
        int cmd = 1, si = 0;
        double s = -w[i] / delta_w[i];
        if (dir > 0) {
          if (hi[i] < kInf) { double s2 = (hi[i] - x[i]) * dirf; if (s2 < s) { s = s2; cmd = 3; } }
        } else {
          if (lo[i] > -kInf) { double s2 = (lo[i] - x[i]) * dirf; if (s2 < s) { s = s2; cmd = 2; } }
        }
        for (int k = 0; k < D.nN; k++) {
          const int idx = D.nC + k;
          if (!D.state[idx] ? delta_w[idx] < 0 : delta_w[idx] > 0) {
            if (lo[idx] == 0 && hi[idx] == 0) continue;
            double s2 = -w[idx] / delta_w[idx];
            if (s2 < s) { s = s2; cmd = 4; si = idx; }
          }
        }
        for (int k = D.nub; k < D.nC; k++) {
          const int idx = k;
          if (delta_x[idx] < 0 && lo[idx] > -kInf) {
            double s2 = (lo[idx] - x[idx]) / delta_x[idx];
            if (s2 < s) { s = s2; cmd = 5; si = idx; }
          }
          if (delta_x[idx] > 0 && hi[idx] < kInf) {
            double s2 = (hi[idx] - x[idx]) / delta_x[idx];
            if (s2 < s) { s = s2; cmd = 6; si = idx; }
          }
        }
        if (s <= 0.0) {
          if (earlyTermination) return false;
          for (int t = i; t < n; t++) { x[t] = 0; w[t] = 0; }
          sError = true;
          break;
        }
        for (int k = 0; k < D.nC; k++) x[k] += s * delta_x[k];
        x[i] += s * dirf;
        for (int k = 0; k < D.nN; k++) w[D.nC + k] += s * delta_w[D.nC + k];
        w[i] += s * delta_w[i];
        switch (cmd) {
          case 1: w[i] = 0; D.transferToC(i); break;
          case 2: x[i] = lo[i]; D.state[i] = 0; D.nN++; break;
          case 3: x[i] = hi[i]; D.state[i] = 1; D.nN++; break;
          case 4: w[si] = 0; D.transferFromNtoC(si); break;
          case 5: x[si] = lo[si]; D.state[si] = 0; D.transferFromCtoN(si); break;
          case 6: x[si] = hi[si]; D.state[si] = 1; D.transferFromCtoN(si); break;
        }
        if (cmd <= 3) break;
      }
    }
    if (sError) break;
  }
  // unpermute
  std::vector<double> t(x, x + n);
  for (int j = 0; j < n; j++) x[D.p[j]] = t[j];
  t.assign(w, w + n);
  for (int j = 0; j < n; j++) w[D.p[j]] = t[j];
  return true;
}

// PgsBoxedLcpSolver::solve (PgsBoxedLcpSolver.cpp:85) with an explicit
// PgsBoxedLcpSolver::Option (no randomisation); pgsSolveLCP uses the default
// Option (30 iterations, deltaX 1e-6, relative 1e-3, eps 1e-9) the contact
// solver runs with.
bool pgsSolveLCPOpt(int n, double* A /* n x n */, double* x, double* b, double* lo, double* hi, const int* findex,
                    int maxIter, double deltaXThr, double relTol, double epsDiv) {
  std::vector<int> order;
  bool possible = true;
  for (int i = 0; i < n; i++) {
    if (A[i * n + i] < epsDiv) { x[i] = 0.0; continue; }
    order.push_back(i);
    const double old = x[i];
    double nx = b[i];
    for (int j = 0; j < n; j++) if (j != i) nx -= A[i * n + j] * x[j];
    nx /= A[i * n + i];
    if (findex[i] >= 0) {
      const double h = hi[i] * x[findex[i]], l = -h;
      x[i] = nx > h ? h : (nx < l ? l : nx);
    } else {
      x[i] = nx > hi[i] ? hi[i] : (nx < lo[i] ? lo[i] : nx);
    }
    if (possible && std::fabs(x[i] - old) > deltaXThr) possible = false;
  }
  if (possible) return true;
  for (int idx : order) {
    const double dummy = 1.0 / A[idx * n + idx];
    b[idx] *= dummy;
    for (int j = 0; j < n; j++) A[idx * n + j] *= dummy;
  }
  for (int iter = 1; iter < maxIter; iter++) {
    possible = true;
    for (int idx : order) {
      double nx = b[idx];
      const double old = x[idx];
      for (int j = 0; j < n; j++) if (j != idx) nx -= A[idx * n + j] * x[j];
      if (findex[idx] >= 0) {
        const double h = hi[idx] * x[findex[idx]], l = -h;
        x[idx] = nx > h ? h : (nx < l ? l : nx);
      } else {
        x[idx] = nx > hi[idx] ? hi[idx] : (nx < lo[idx] ? lo[idx] : nx);
      }
      if (possible && std::fabs(x[idx]) > epsDiv) {
        if (std::fabs((x[idx] - old) / x[idx]) > relTol) possible = false;
      }
    }
    if (possible) break;
  }
  return possible;
}

bool pgsSolveLCP(int n, double* A, double* x, double* b, double* lo, double* hi, const int* findex) {
  return pgsSolveLCPOpt(n, A, x, b, lo, hi, findex, 30, 1e-6, 1e-3, 1e-9);
}

}  // namespace oracle
