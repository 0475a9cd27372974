// ORACLE / TEST INFRASTRUCTURE ONLY -- C entry points for tests/ (ctypes).
#include <cstring>
#include <vector>

#include "oracle.hpp"
#include "oracle_lcp.hpp"

using namespace oracle;

struct OracleSnap { Snapshot s; };

extern "C" {

void* oracle_world_create(const nimble_world_desc* d) { return new World(d); }
void oracle_world_destroy(void* w) { delete static_cast<World*>(w); }

// Batched loop over independent worlds (the CPU baseline is this loop).
// lcp_cache: [batch][NIMBLE_MAX_LCP + 1], element 0 = cached size (-1 = empty)
void* oracle_snapshots_create(int batch) { return new std::vector<OracleSnap>(batch); }
void oracle_snapshots_destroy(void* s) { delete static_cast<std::vector<OracleSnap>*>(s); }

int oracle_forward(void* wp, int batch, const double* state, const double* tau, double* lcpCache,
                   double* next, void* snaps) {
  World& w = *static_cast<World*>(wp);
  auto& S = *static_cast<std::vector<OracleSnap>*>(snaps);
  const int n = w.n;
  for (int b = 0; b < batch; b++) {
    double* cache = lcpCache + (size_t)b * (NIMBLE_MAX_LCP + 1);
    std::vector<double> c;
    int sz = (int)cache[0];
    if (sz >= 0) c.assign(cache + 1, cache + 1 + sz);
    else c.clear();
    std::vector<double>* cp = &c;
    bool empty = sz < 0;
    if (empty) c.clear();
    step(w, state + (size_t)b * 2 * n, tau + (size_t)b * n, *cp, next + (size_t)b * 2 * n, S[b].s);
    cache[0] = (double)c.size();
    for (size_t i = 0; i < c.size(); i++) cache[1 + i] = c[i];
  }
  return 0;
}

// oracle_forward with the LCP path of selected worlds replayed
// (ForcedLcp): forcedX [batch][NIMBLE_MAX_LCP + 1] (element 0 = rows, < 0 =
// solve normally), flags [batch][3] = (short-circuit, cfm, friction removed).
// Returns the number of forced worlds whose row count did not match.
int oracle_forward_forced(void* wp, int batch, const double* state, const double* tau, double* lcpCache,
                          double* next, void* snaps, const double* forcedX, const double* flags) {
  World& w = *static_cast<World*>(wp);
  auto& S = *static_cast<std::vector<OracleSnap>*>(snaps);
  const int n = w.n;
  int mismatched = 0;
  for (int b = 0; b < batch; b++) {
    double* cache = lcpCache + (size_t)b * (NIMBLE_MAX_LCP + 1);
    std::vector<double> c;
    const int sz = (int)cache[0];
    if (sz >= 0) c.assign(cache + 1, cache + 1 + sz);
    const double* fx = forcedX + (size_t)b * (NIMBLE_MAX_LCP + 1);
    ForcedLcp f;
    if ((int)fx[0] >= 0) {
      f.m = (int)fx[0];
      f.x = fx + 1;
      f.shortCircuit = flags[b * 3 + 0] != 0.0;
      f.cfm = flags[b * 3 + 1];
      f.ignoredFriction = flags[b * 3 + 2] != 0.0;
      tForcedLcp = &f;
    }
    step(w, state + (size_t)b * 2 * n, tau + (size_t)b * n, c, next + (size_t)b * 2 * n, S[b].s);
    tForcedLcp = nullptr;
    if (f.mismatch) mismatched++;
    cache[0] = (double)c.size();
    for (size_t i = 0; i < c.size(); i++) cache[1 + i] = c[i];
  }
  return mismatched;
}

// Collision detection only (kinematics + collide + the constraint filter's
// depth / normal tests): contact count per world, no LCP, no size limit.
// unsupported[b] = 1 when a narrow-phase branch not restated was hit.
void oracle_detect(void* wp, int batch, const double* state, int* counts, int* unsupported) {
  World& w = *static_cast<World*>(wp);
  const int n = w.n;
  for (int b = 0; b < batch; b++) {
    const double* q = state + (size_t)b * 2 * n;
    Kin<double> k;
    k.compute(w, q, q + n);
    std::vector<Contact> cs;
    int unsup = 0;
    collide(w, k, cs, &unsup);
    int kept = 0;
    for (const Contact& c : cs) {
      if (c.normal[0] * c.normal[0] + c.normal[1] * c.normal[1] + c.normal[2] * c.normal[2] < 1e-12) continue;
      if (c.depth < 0.0 || c.depth > w.clipDepth) continue;
      kept++;
    }
    counts[b] = kept;
    if (unsupported) unsupported[b] = unsup;
  }
}

int oracle_backward(void* wp, int batch, void* snaps, const double* gradNext, double* gradState, double* gradTau) {
  World& w = *static_cast<World*>(wp);
  auto& S = *static_cast<std::vector<OracleSnap>*>(snaps);
  const int n = w.n;
  for (int b = 0; b < batch; b++)
    backprop(w, S[b].s, gradNext + (size_t)b * 2 * n, gradState + (size_t)b * 2 * n, gradTau + (size_t)b * n);
  return 0;
}

// getJacobianOfConstraintForce (BackpropSnapshot.cpp:2723) per world:
// out [batch][maxRows][3n], row r = d f_c[r] / d(q, v, tau), zero past n_c
int oracle_constraint_force_jacobians(void* wp, int batch, void* snaps, double* out, int maxRows) {
  World& w = *static_cast<World*>(wp);
  auto& S = *static_cast<std::vector<OracleSnap>*>(snaps);
  const int n = w.n;
  std::vector<double> pp(n * n), pv(n * n), vp(n * n), vv(n * n), fv(n * n), dfc;
  for (int b = 0; b < batch; b++) {
    double* o = out + (size_t)b * maxRows * 3 * n;
    std::fill(o, o + (size_t)maxRows * 3 * n, 0.0);
    if (S[b].s.numClamping == 0) continue;
    stepJacobians(w, S[b].s, pp.data(), pv.data(), vp.data(), vv.data(), fv.data(), &dfc);
    const int nc = S[b].s.numClamping < maxRows ? S[b].s.numClamping : maxRows;
    std::copy(dfc.begin(), dfc.begin() + (size_t)nc * 3 * n, o);
  }
  return 0;
}

// getStateJacobian [2n][2n] = [[posPos, velPos], [posVel, velVel]]
// (BackpropSnapshot.cpp:1230) and d(next)/d(tau) [2n][n] = [0; forceVel]
int oracle_jacobians(void* wp, int batch, void* snaps, double* stateJac, double* forceJac) {
  World& w = *static_cast<World*>(wp);
  auto& S = *static_cast<std::vector<OracleSnap>*>(snaps);
  const int n = w.n;
  std::vector<double> pp(n * n), pv(n * n), vp(n * n), vv(n * n), fv(n * n);
  for (int b = 0; b < batch; b++) {
    stepJacobians(w, S[b].s, pp.data(), pv.data(), vp.data(), vv.data(), fv.data());
    double* J = stateJac + (size_t)b * 4 * n * n;
    double* F = forceJac + (size_t)b * 2 * n * n;
    for (int r = 0; r < n; r++)
      for (int c = 0; c < n; c++) {
        J[r * 2 * n + c] = pp[r * n + c];
        J[r * 2 * n + n + c] = vp[r * n + c];
        J[(n + r) * 2 * n + c] = pv[r * n + c];
        J[(n + r) * 2 * n + n + c] = vv[r * n + c];
        F[r * n + c] = 0.0;
        F[(n + r) * n + c] = fv[r * n + c];
      }
  }
  return 0;
}

// Debug getters (single world)
void oracle_mass_matrix(void* wp, const double* q, double* M) {
  World& w = *static_cast<World*>(wp);
  std::vector<double> v(w.n, 0.0);
  Kin<double> k; k.compute(w, q, v.data());
  w.massMatrix(k, M);
}
void oracle_coriolis_gravity(void* wp, const double* q, const double* v, double* C) {
  World& w = *static_cast<World*>(wp);
  Kin<double> k; k.compute(w, q, v);
  w.coriolisGravity(k, C);
}
void oracle_forward_dynamics(void* wp, const double* q, const double* v, const double* tau, double* ddq) {
  World& w = *static_cast<World*>(wp);
  Kin<double> k; k.compute(w, q, v);
  forwardDynamicsABA(w, k, q, v, tau, ddq);
}
void oracle_body_transforms(void* wp, const double* q, double* T /* nb x 12 */) {
  World& w = *static_cast<World*>(wp);
  std::vector<double> v(w.n, 0.0);
  Kin<double> k; k.compute(w, q, v.data());
  for (int b = 0; b < w.nb; b++)
    for (int r = 0; r < 3; r++) {
      for (int c = 0; c < 3; c++) T[b * 12 + r * 4 + c] = k.Tw[b].R(r, c);
      T[b * 12 + r * 4 + 3] = k.Tw[b].p[r];
    }
}
void oracle_jacobian_of_c(void* wp, const double* q, const double* v, int wrtPos, double* dC) {
  static_cast<World*>(wp)->jacobianOfC(q, v, wrtPos != 0, dC);
}
int oracle_num_contacts(void* snaps, int b) {
  return (int)(*static_cast<std::vector<OracleSnap>*>(snaps))[b].s.contacts.size();
}
// contacts of world b after a forward: per contact [point3, normal3, depth, type, bodyA, bodyB]
int oracle_contacts(void* snaps, int b, double* out, int maxc) {
  const auto& cs = (*static_cast<std::vector<OracleSnap>*>(snaps))[b].s.contacts;
  int k = 0;
  for (const auto& c : cs) {
    if (k >= maxc) break;
    double* o = out + 10 * k;
    for (int i = 0; i < 3; i++) { o[i] = c.point[i]; o[3 + i] = c.normal[i]; }
    o[6] = c.depth; o[7] = c.type; o[8] = c.bodyA; o[9] = c.bodyB;
    k++;
  }
  return k;
}
// LCP classification of world b: mapping per row (-1 clamping, -2 not clamping, >=0 upper bound)
int oracle_lcp_debug(void* snaps, int b, int* mapping, double* x, int maxRows) {
  const auto& s = (*static_cast<std::vector<OracleSnap>*>(snaps))[b].s;
  int m = s.numRows < maxRows ? s.numRows : maxRows;
  for (int i = 0; i < m; i++) { mapping[i] = s.mapping[i]; x[i] = s.lcpX[i]; }
  return s.numRows;
}
// LCP path flags of world b: [shortCircuit, ignoredFriction, cfm, numClamping, numUpperBound]
void oracle_lcp_flags(void* snaps, int b, double* out) {
  const auto& s = (*static_cast<std::vector<OracleSnap>*>(snaps))[b].s;
  out[0] = s.shortCircuit ? 1 : 0;
  out[1] = s.ignoredFriction ? 1 : 0;
  out[2] = s.cfm;
  out[3] = s.numClamping;
  out[4] = s.numUpperBound;
  out[5] = s.unsupportedContacts;
  out[6] = s.lcpReduced ? 1 : 0;
}
// clamping impulses f_c of world b; returns numClamping
int oracle_lcp_fc(void* snaps, int b, double* fc, int maxc) {
  const auto& s = (*static_cast<std::vector<OracleSnap>*>(snaps))[b].s;
  for (int i = 0; i < s.numClamping && i < maxc; i++) fc[i] = s.fc[i];
  return s.numClamping;
}
// J^T columns of world b's LCP rows (n x m row-major); returns m
int oracle_lcp_cols(void* snaps, int b, double* out, int maxElems) {
  const auto& s = (*static_cast<std::vector<OracleSnap>*>(snaps))[b].s;
  if ((int)s.Aall.size() > maxElems) return -1;
  for (size_t i = 0; i < s.Aall.size(); i++) out[i] = s.Aall[i];
  return s.numRows;
}
// LCP problem of world b (before the solve): A (m x m), b, lo, hi, findex; returns m
int oracle_lcp_problem(void* snaps, int b, double* A, double* bb, double* lo, double* hi, int* fi, int maxRows) {
  const auto& s = (*static_cast<std::vector<OracleSnap>*>(snaps))[b].s;
  const int m = s.numRows;
  if (m > maxRows) return -1;
  for (int i = 0; i < m * m; i++) A[i] = s.lcpA[i] - ((i / m == i % m) ? s.cfm : 0.0);
  for (int i = 0; i < m; i++) { bb[i] = s.lcpB[i]; lo[i] = s.lcpLo[i]; hi[i] = s.lcpHi[i]; fi[i] = s.lcpFIndex[i]; }
  return m;
}
// Dantzig restatement on a raw problem (A n x n row-major); returns success
int oracle_dantzig(int n, const double* A, const double* b, const double* lo, const double* hi, const int* findex,
                   double* x, int earlyTermination) {
  std::vector<double> Ac(A, A + n * n), bc(b, b + n), loc(lo, lo + n), hic(hi, hi + n);
  std::vector<int> fi(findex, findex + n);
  return dantzigSolveLCP(n, Ac.data(), x, bc.data(), nullptr, 0, loc.data(), hic.data(), fi.data(),
                         earlyTermination != 0) ? 1 : 0;
}
void codSolveC(const double* A, int m, int n, const double* b, double* x);
void oracle_cod_solve(const double* A, int m, int n, const double* b, double* x) { codSolveC(A, m, n, b, x); }
int oracle_box_box(const double* size1, const double* T1, const double* size2, const double* T2, double* out);
}
namespace oracle {
void codSolve(const double* A, int m, int n, const double* b, double* x);
bool pgsSolveLCP(int n, double* A, double* x, double* b, double* lo, double* hi, const int* findex);
bool pgsSolveLCPOpt(int n, double* A, double* x, double* b, double* lo, double* hi, const int* findex, int maxIter,
                    double deltaXThr, double relTol, double epsDiv);
bool lcpValid(const std::vector<double>& A, const std::vector<double>& x, const std::vector<double>& b,
              const std::vector<double>& hi, const std::vector<double>& lo, const std::vector<int>& fi,
              bool ignoreFriction);
std::vector<double> guessSolution(const std::vector<double>& A, const std::vector<double>& b,
                                  const std::vector<int>& fi);
std::vector<int> lcpReduce(std::vector<double>& A, std::vector<double>& X, std::vector<double>& b,
                           std::vector<double>& hi, std::vector<double>& lo, std::vector<int>& fi);
struct LcpCascade {
  bool reduced = false, ignoredFriction = false;
  double cfm = 0.0;
  int path = 0;
};
LcpCascade lcpFallbackCascade(const std::vector<double>& A, const std::vector<double>& b,
                              const std::vector<double>& lo, const std::vector<double>& hi,
                              const std::vector<int>& fi, const std::vector<double>& warm, double fallbackCfm,
                              std::vector<double>& X);
}  // namespace oracle

static std::vector<double> vec(const double* p, int n) { return std::vector<double>(p, p + n); }

extern "C" {
// LCPUtils::reduce on a raw problem (A m x m row-major); writes the reduced
// problem (A as mr x mr) and map (original row -> reduced row); returns mr
int oracle_lcp_reduce(int m, const double* A, const double* x, const double* b, const double* hi, const double* lo,
                      const int* fi, double* Ao, double* xo, double* bo, double* hio, double* loo, int* fio, int* map) {
  std::vector<double> Av = vec(A, m * m), xv = vec(x, m), bv = vec(b, m), hv = vec(hi, m), lv = vec(lo, m);
  std::vector<int> fv(fi, fi + m);
  const std::vector<int> mp = oracle::lcpReduce(Av, xv, bv, hv, lv, fv);
  const int mr = (int)bv.size();
  for (int i = 0; i < mr * mr; i++) Ao[i] = Av[i];
  for (int i = 0; i < mr; i++) { xo[i] = xv[i]; bo[i] = bv[i]; hio[i] = hv[i]; loo[i] = lv[i]; fio[i] = fv[i]; }
  for (int i = 0; i < m; i++) map[i] = mp[i];
  return mr;
}
// PgsBoxedLcpSolver::solve restated (default options); x in/out
int oracle_pgs(int n, const double* A, double* x, const double* b, const double* lo, const double* hi,
               const int* fi) {
  std::vector<double> Av = vec(A, n * n), bv = vec(b, n), lv = vec(lo, n), hv = vec(hi, n);
  return oracle::pgsSolveLCP(n, Av.data(), x, bv.data(), lv.data(), hv.data(), fi) ? 1 : 0;
}
// PgsBoxedLcpSolver::solve with PgsBoxedLcpSolver::Option(maxIter, deltaX, relTol, epsDiv, false)
int oracle_pgs_opt(int n, const double* A, double* x, const double* b, const double* lo, const double* hi,
                   const int* fi, int maxIter, double deltaX, double relTol, double epsDiv) {
  std::vector<double> Av = vec(A, n * n), bv = vec(b, n), lv = vec(lo, n), hv = vec(hi, n);
  return oracle::pgsSolveLCPOpt(n, Av.data(), x, bv.data(), lv.data(), hv.data(), fi, maxIter, deltaX, relTol, epsDiv)
             ? 1 : 0;
}
int oracle_lcp_valid(int m, const double* A, const double* x, const double* b, const double* hi, const double* lo,
                     const int* fi, int ignoreFriction) {
  return oracle::lcpValid(vec(A, m * m), vec(x, m), vec(b, m), vec(hi, m), vec(lo, m), std::vector<int>(fi, fi + m),
                          ignoreFriction != 0) ? 1 : 0;
}
void oracle_guess_solution(int m, const double* A, const double* b, const int* fi, double* x) {
  const std::vector<double> g = oracle::guessSolution(vec(A, m * m), vec(b, m), std::vector<int>(fi, fi + m));
  for (int i = 0; i < m; i++) x[i] = g[i];
}
// the fallback cascade of BoxedLcpConstraintSolver::solveLcp; x: in warm
// start, out solution; info: [path, reduced, ignoredFriction, cfm]
void oracle_lcp_cascade(int m, const double* A, const double* b, const double* lo, const double* hi, const int* fi,
                        double* x, double fallbackCfm, double* info) {
  std::vector<double> X;
  const oracle::LcpCascade r = oracle::lcpFallbackCascade(vec(A, m * m), vec(b, m), vec(lo, m), vec(hi, m),
                                                          std::vector<int>(fi, fi + m), vec(x, m), fallbackCfm, X);
  for (int i = 0; i < m; i++) x[i] = X[i];
  info[0] = r.path; info[1] = r.reduced ? 1 : 0; info[2] = r.ignoredFriction ? 1 : 0; info[3] = r.cfm;
}
}
void codSolveC(const double* A, int m, int n, const double* b, double* x) { oracle::codSolve(A, m, n, b, x); }
namespace oracle {
bool classifyLcp(int m, const double* A, const double* b, const double* lo, const double* hi, const int* fi,
                 double* X);
}
namespace oracle {
void lcpPathFromA(int m, const double* A, const double* b, const double* lo, const double* hi, const int* fi,
                  const double* warm, double fallbackCfm, double* flags, int* mapping);
}
// the whole LCP path (short-circuit, cascade, final classification) on a raw
// problem (tests: ambiguity probe of classification / friction-removed splits)
extern "C" void oracle_lcp_path(int m, const double* A, const double* b, const double* lo, const double* hi,
                                const int* fi, const double* warm, double fallbackCfm, double* flags, int* mapping) {
  oracle::lcpPathFromA(m, A, b, lo, hi, fi, warm, fallbackCfm, flags, mapping);
}
// the short-circuit classification on a raw problem (tests: ambiguity probe)
extern "C" int oracle_classify(int m, const double* A, const double* b, const double* lo, const double* hi,
                               const int* fi, double* x) {
  return oracle::classifyLcp(m, A, b, lo, hi, fi, x) ? 1 : 0;
}
