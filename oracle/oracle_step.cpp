// ORACLE / TEST INFRASTRUCTURE ONLY -- see nimble_oracle.cpp header.
//
// World::step (dart/simulation/World.cpp:221) and BackpropSnapshot::backprop
// (dart/neural/BackpropSnapshot.cpp:121) restated on plain dense matrices.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "oracle.hpp"
#include "oracle_lcp.hpp"

namespace oracle {

using Mat = std::vector<double>;

static void matmul(const double* A, const double* B, double* C, int r, int k, int c) {
  for (int i = 0; i < r; i++)
    for (int j = 0; j < c; j++) {
      double s = 0;
      for (int t = 0; t < k; t++) s += A[i * k + t] * B[t * c + j];
      C[i * c + j] = s;
    }
}
static void matvec(const double* A, const double* x, double* y, int r, int c) {
  for (int i = 0; i < r; i++) {
    double s = 0;
    for (int j = 0; j < c; j++) s += A[i * c + j] * x[j];
    y[i] = s;
  }
}
static void matTvec(const double* A, const double* x, double* y, int r, int c) {
  for (int j = 0; j < c; j++) {
    double s = 0;
    for (int i = 0; i < r; i++) s += A[i * c + j] * x[i];
    y[j] = s;
  }
}

// Cholesky solve for SPD A (n x n)
void cholSolve(const double* A, const double* b, double* x, int n) {
  std::vector<double> L(n * n, 0.0);
  for (int j = 0; j < n; j++) {
    double s = A[j * n + j];
    for (int k = 0; k < j; k++) s -= L[j * n + k] * L[j * n + k];
    L[j * n + j] = std::sqrt(s);
    for (int i = j + 1; i < n; i++) {
      double t = A[i * n + j];
      for (int k = 0; k < j; k++) t -= L[i * n + k] * L[j * n + k];
      L[i * n + j] = t / L[j * n + j];
    }
  }
  std::vector<double> y(n);
  for (int i = 0; i < n; i++) {
    double s = b[i];
    for (int k = 0; k < i; k++) s -= L[i * n + k] * y[k];
    y[i] = s / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = y[i];
    for (int k = i + 1; k < n; k++) s -= L[k * n + i] * x[k];
    x[i] = s / L[i * n + i];
  }
}

static void inverseSPD(const double* A, double* Ainv, int n) {
  std::vector<double> e(n), col(n);
  for (int c = 0; c < n; c++) {
    std::fill(e.begin(), e.end(), 0.0);
    e[c] = 1.0;
    cholSolve(A, e.data(), col.data(), n);
    for (int r = 0; r < n; r++) Ainv[r * n + c] = col[r];
  }
  for (int r = 0; r < n; r++)
    for (int c = r + 1; c < n; c++) {
      double m = 0.5 * (Ainv[r * n + c] + Ainv[c * n + r]);
      Ainv[r * n + c] = Ainv[c * n + r] = m;
    }
}

//------------------------------------------------------------------------------
void step(const World& w, const double* state, const double* tau, std::vector<double>& lcpCache,
          double* nextState, Snapshot& snap) {
  const int n = w.n;
  const double* q = state;
  const double* v = state + n;
  snap.q.assign(q, q + n);
  snap.v.assign(v, v + n);
  snap.tau.assign(tau, tau + n);

  Kin<double> k;
  k.compute(w, q, v);

  // Skeleton::computeForwardDynamics + integrateVelocities (World.cpp:226-233)
  std::vector<double> ddq(n, 0.0), v1(n);
  forwardDynamicsABA(w, k, q, v, tau, ddq.data());
  for (int i = 0; i < n; i++) v1[i] = v[i] + w.dt * ddq[i];
  snap.preConstraintV = v1;

  // runConstraintEngine (World.cpp:254): collision + LCP + impulses
  std::vector<Contact> contacts;
  collide(w, k, contacts, &snap.unsupportedContacts);
  solveContacts(w, k, q, v, tau, v1, contacts, lcpCache, snap);

  // integratePositions(initialVelocity) (World.cpp:300)
  std::vector<double> q1(n);
  if (w.parallelPosVel) w.integratePositionsExplicit(q, v, w.dt, q1.data());
  else w.integratePositionsExplicit(q, v1.data(), w.dt, q1.data());
  for (int i = 0; i < n; i++) { nextState[i] = q1[i]; nextState[n + i] = v1[i]; }
  snap.postQ = q1;
  snap.postV = v1;
}

//------------------------------------------------------------------------------
// BackpropSnapshot::backprop (BackpropSnapshot.cpp:121) with
// exploreAlternateStrategies == false: form posPos, posVel, velPos, velVel,
// forceVel and multiply their transposes into the upstream gradient.
// The five Jacobian blocks of the step (BackpropSnapshot::getPosPosJacobian
// :1263, getPosVelJacobian :762, getVelPosJacobian :1338, getVelVelJacobian
// :643, getControlForceVelJacobian :482), row-major n x n each.
void stepJacobians(const World& w, const Snapshot& snap, double* posPosOut, double* posVelOut, double* velPosOut,
                   double* velVelOut, double* forceVelOut, std::vector<double>* dFcOut) {
  const int n = w.n;
  const double dt = w.dt;
  const double* q = snap.q.data();
  const double* v = snap.v.data();
  const double* tau = snap.tau.data();

  Kin<double> k;
  k.compute(w, q, v);
  Mat M(n * n), Minv(n * n), C(n);
  w.massMatrix(k, M.data());
  inverseSPD(M.data(), Minv.data(), n);
  w.coriolisGravity(k, C.data());

  // Constraint matrices (BackpropSnapshot::getClampingConstraintMatrix etc.)
  const int nc = snap.numClamping, nu = snap.numUpperBound;
  Mat Ac, Aub, AcubE;  // n x nc, n x nu
  Mat Qfacinv;         // pinv(Q) nc x nc
  buildClampingMatrices(w, snap, Ac, Aub, AcubE);

  // z = dt (tau - C - D v - K (q - q0 + dt v)) + A_c_ub_E f_c
  Mat z(n), y(n);
  for (int i = 0; i < n; i++) {
    double springF = w.spring[i] * (q[i] - w.restPos[i] + dt * v[i]);
    double dampF = w.damping[i] * v[i];
    z[i] = dt * (tau[i] - C[i] - dampF - springF);
  }
  for (int i = 0; i < n; i++)
    for (int c = 0; c < nc; c++) z[i] += AcubE[i * nc + c] * snap.fc[c];
  matvec(Minv.data(), z.data(), y.data(), n, n);

  // getJacobianOfMinv(z, POSITION) = -Minv d(M y)/dq   (Skeleton.cpp:2024)
  Mat dMy(n * n), dM(n * n);
  w.jacobianOfMy(q, y.data(), dMy.data());
  matmul(Minv.data(), dMy.data(), dM.data(), n, n, n);
  for (auto& x : dM) x = -x;

  Mat dCq(n * n), dCv(n * n);
  w.jacobianOfC(q, v, true, dCq.data());
  w.jacobianOfC(q, v, false, dCv.data());

  Mat posVel(n * n), velVel(n * n), forceVel(n * n);
  if (nc == 0) {
    // BackpropSnapshot::getVelVelJacobian, A_c empty branch (:698)
    for (int r = 0; r < n; r++)
      for (int c = 0; c < n; c++) {
        double s = 0;
        for (int t = 0; t < n; t++) s += Minv[r * n + t] * dCv[t * n + c];
        velVel[r * n + c] = (r == c ? 1.0 : 0.0) - dt * Minv[r * n + c] * w.damping[c]
                            - dt * dt * Minv[r * n + c] * w.spring[c] - dt * s;
        forceVel[r * n + c] = dt * Minv[r * n + c];
      }
    // getVelJacobianWrt(POSITION) with A_c empty (:1095)
    for (int r = 0; r < n; r++)
      for (int c = 0; c < n; c++) {
        double s = 0;
        for (int t = 0; t < n; t++) s += Minv[r * n + t] * dCq[t * n + c];
        posVel[r * n + c] = dM[r * n + c] - dt * s - Minv[r * n + c] * dt * w.spring[c];
      }
  } else {
    constrainedJacobians(w, k, snap, M, Minv, C, dCq, dCv, dM, Ac, Aub, AcubE, posVel, velVel, forceVel, dFcOut);
  }

  Mat posPos(n * n), velPos(n * n);
  w.posPosJac(q, v, posPos.data());
  w.velPosJac(q, v, velPos.data());
  // bounce approximation (BackpropSnapshot.cpp:1131) is identity without
  // restitution; restitution is not enabled on the hot path.
  std::copy(posPos.begin(), posPos.end(), posPosOut);
  std::copy(posVel.begin(), posVel.end(), posVelOut);
  std::copy(velPos.begin(), velPos.end(), velPosOut);
  std::copy(velVel.begin(), velVel.end(), velVelOut);
  std::copy(forceVel.begin(), forceVel.end(), forceVelOut);
}

// BackpropSnapshot::backprop (:161-183): the transposed blocks times the
// upstream gradient, then clipLossGradientsToBounds.
void backprop(const World& w, const Snapshot& snap, const double* gradNext, double* gradState, double* gradTau) {
  const int n = w.n;
  const double* q = snap.q.data();
  const double* v = snap.v.data();
  const double* tau = snap.tau.data();
  const double* gp = gradNext;
  const double* gv = gradNext + n;
  Mat posPos(n * n), posVel(n * n), velPos(n * n), velVel(n * n), forceVel(n * n);
  stepJacobians(w, snap, posPos.data(), posVel.data(), velPos.data(), velVel.data(), forceVel.data());

  std::vector<double> lp(n), lv(n), lt(n), tmp(n);
  matTvec(posPos.data(), gp, lp.data(), n, n);
  matTvec(posVel.data(), gv, tmp.data(), n, n);
  for (int i = 0; i < n; i++) lp[i] += tmp[i];
  matTvec(velPos.data(), gp, lv.data(), n, n);
  matTvec(velVel.data(), gv, tmp.data(), n, n);
  for (int i = 0; i < n; i++) lv[i] += tmp[i];
  matTvec(forceVel.data(), gv, lt.data(), n, n);

  // clipLossGradientsToBounds (BackpropSnapshot.cpp:425)
  for (int j = 0; j < n; j++) {
    if (q[j] == w.posLo[j] && lp[j] > 0) lp[j] = 0;
    if (q[j] == w.posHi[j] && lp[j] < 0) lp[j] = 0;
    if (v[j] == w.velLo[j] && lv[j] > 0) lv[j] = 0;
    if (v[j] == w.velHi[j] && lv[j] < 0) lv[j] = 0;
    if (tau[j] == w.forceLo[j] && lt[j] > 0) lt[j] = 0;
    if (tau[j] == w.forceHi[j] && lt[j] < 0) lt[j] = 0;
  }
  for (int i = 0; i < n; i++) { gradState[i] = lp[i]; gradState[n + i] = lv[i]; gradTau[i] = lt[i]; }
}

}  // namespace oracle
