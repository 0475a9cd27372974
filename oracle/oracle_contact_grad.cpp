// ORACLE / TEST INFRASTRUCTURE ONLY -- see nimble_oracle.cpp header.
//
// Position derivatives of the contact constraint terms, restating
//  * DifferentiableContactConstraint::getConstraintForcesJacobian
//    (dart/neural/DifferentiableContactConstraint.cpp:1654): d(J^T e_i)/dq =
//    multiple_r * (dS_r/dq_k . wrench + S_r . dwrench/dq_k), with the screw
//    gradient ad(S_pos_k, S_r) (:1226, FreeJoint::getScrewAxisGradientForForce
//    FreeJoint.cpp:1193), the contact position gradient (:328) and the force
//    direction gradient (:594 normal, :1092 tangent basis);
//  * BackpropSnapshot::getJacobianOfConstraintForce (BackpropSnapshot.cpp:2723)
//    = dQ_b + Q^+ dB, getJacobianOfLCPConstraintMatrixClampingSubset (:2889)
//    including the pseudo-inverse gradient branch, and
//    getJacobianOfLCPOffsetClampingSubset (:3181) for POSITION.
// Supported contact types: VERTEX_FACE and FACE_VERTEX (box-box face
// contacts), SPHERE_BOX and BOX_SPHERE (capsule/sphere-box, the SPHERE_TO_BOX
// / BOX_TO_SPHERE branches of :328 and :594) and EDGE_EDGE (the EDGE_A /
// EDGE_B branches, :412 / :429 and :708 / :722).
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "oracle_lcp.hpp"

namespace oracle {

void codSolve(const double* A, int m, int n, const double* b, double* x);

using Mat = std::vector<double>;
enum { CT_FACE_VERTEX = 1, CT_VERTEX_FACE = 2, CT_EDGE_EDGE = 3, CT_SPHERE_BOX = 4, CT_BOX_SPHERE = 5, CT_SPHERE_SPHERE = 6,
       CT_SPHERE_PIPE = 7, CT_PIPE_SPHERE = 8, CT_PIPE_PIPE = 9 };

static void cross3(const double* a, const double* b, double* o) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

// World screw axis for position (Joint::getWorldAxisScrewForPosition,
// Joint.cpp:1167 with FreeJoint's position-space Jacobian FreeJoint.cpp:790;
// BallJoint's, BallJoint.cpp:282, is its rotational half)
static void positionScrew(const World& w, const Kin<double>& k, const double* q, int dof, double* Z) {
  const int b = w.dofBody[dof];
  const Body& B = w.bodies[b];
  const int c = dof - B.dof0;
  V6<double> xi;
  for (int i = 0; i < 6; i++) xi[i] = 0.0;
  if (B.jtype == NIMBLE_JOINT_FREE || B.jtype == NIMBLE_JOINT_BALL) {
    const double* th = q + B.dof0;
    V3<double> t{{th[0], th[1], th[2]}};
    if (c < 3) {
      // J_r e_c = column c of expMapJac(th)^T
      double t2 = th[0] * th[0] + th[1] * th[1] + th[2] * th[2];
      double tt = std::sqrt(t2);
      M3<double> K = skew(t), K2 = mul(K, K), J;
      double a, bb;
      if (tt < 1.0e-3) { a = 0.5; bb = 1.0 / 6.0; }  // expMapJac small-angle branch
      else { a = (1 - std::cos(tt)) / t2; bb = (tt - std::sin(tt)) / (t2 * tt); }
      for (int i = 0; i < 9; i++) J.m[i] = ((i % 4) == 0 ? 1.0 : 0.0) + a * K.m[i] + bb * K2.m[i];
      // expMapJac(th)^T column c = row c of expMapJac
      for (int i = 0; i < 3; i++) xi[i] = J(c, i);
    } else {
      M3<double> R = expMapRot(t);
      for (int i = 0; i < 3; i++) xi[3 + i] = R(c - 3, i);  // R^T e
    }
    V6<double> z = AdT(compose(k.Tw[b], B.Tcj), xi);
    for (int i = 0; i < 6; i++) Z[i] = z[i];
  } else {
    V6<double> sl;
    for (int i = 0; i < 6; i++) sl[i] = k.Sj[b](i, c);
    V6<double> z = AdT(k.Tw[b], sl);
    for (int i = 0; i < 6; i++) Z[i] = z[i];
  }
}

static void velocityScrew(const World& w, const Kin<double>& k, int dof, double* S) {
  const int b = w.dofBody[dof];
  V6<double> sl;
  for (int i = 0; i < 6; i++) sl[i] = k.Sj[b](i, dof - w.bodies[b].dof0);
  V6<double> s = AdT(k.Tw[b], sl);
  for (int i = 0; i < 6; i++) S[i] = s[i];
}

// ContactConstraint::getTangentBasisMatrixODEGradient (ContactConstraint.cpp:772)
static void tangentBasisGradient(const double* n, const double* g, double* T0, double* T1) {
  const double ez[3] = {0, 0, 1}, ex[3] = {1, 0, 0}, ey[3] = {0, 1, 0};
  const double* cr = ez;
  double t[3];
  cross3(cr, n, t);
  if (t[0] * t[0] + t[1] * t[1] + t[2] * t[2] < 1e-12) {
    cr = ex; cross3(cr, n, t);
    if (t[0] * t[0] + t[1] * t[1] + t[2] * t[2] < 1e-12) {
      cr = ey; cross3(cr, n, t);
      if (t[0] * t[0] + t[1] * t[1] + t[2] * t[2] < 1e-12) { cr = ez; cross3(cr, n, t); }
    }
  }
  double tn = std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
  for (int i = 0; i < 3; i++) t[i] /= tn;
  double gc[3];
  cross3(cr, g, gc);
  for (int i = 0; i < 3; i++) gc[i] /= tn;
  double gt[3];
  if (std::fabs(tn - 1.0) > 1e-6) {
    double dd = gc[0] * t[0] + gc[1] * t[1] + gc[2] * t[2];
    for (int i = 0; i < 3; i++) gt[i] = gc[i] - dd * t[i];
  } else {
    for (int i = 0; i < 3; i++) gt[i] = gc[i];
  }
  double a[3], b[3];
  cross3(g, t, a);
  cross3(n, gt, b);
  for (int i = 0; i < 3; i++) { T0[i] = gt[i]; T1[i] = a[i] + b[i]; }
}

// math::getContactPointGradient (dart/math/Geometry.cpp:1129) with radii 1:
// derivative of the midpoint of the edges' closest approach
static void contactPointGradient(const double* pA, const double* dpA, const double* uA, const double* duA,
                                 const double* pB, const double* dpB, const double* uB, const double* duB,
                                 double* out, double rA = 1.0, double rB = 1.0) {
  double p[3], d_p[3];
  for (int i = 0; i < 3; i++) { p[i] = pB[i] - pA[i]; d_p[i] = dpB[i] - dpA[i]; }
  auto dot = [](const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
  const double uaub = dot(uA, uB);
  const double d_uaub = dot(duA, uB) + dot(uA, duB);
  const double q1 = dot(uA, p);
  const double d_q1 = dot(duA, p) + dot(uA, d_p);
  const double q2 = -dot(uB, p);
  const double d_q2 = -dot(duB, p) - dot(uB, d_p);
  const double d = 1 - uaub * uaub;
  const double d_d = -2 * d_uaub * uaub;
  if (d <= 0) {
    for (int i = 0; i < 3; i++) out[i] = (dpA[i] * rB + dpB[i] * rA) / (rA + rB);
    return;
  }
  const double e = 1.0 / d;
  const double d_e = -(1.0 / (d * d)) * d_d;
  const double alpha = (q1 + uaub * q2) * e;
  const double d_alpha = (q1 + uaub * q2) * d_e + (d_q1 + d_uaub * q2 + uaub * d_q2) * e;
  const double beta = (uaub * q1 + q2) * e;
  const double d_beta = (uaub * q1 + q2) * d_e + (d_uaub * q1 + uaub * d_q1 + d_q2) * e;
  for (int i = 0; i < 3; i++)
    out[i] = ((dpA[i] + alpha * duA[i] + d_alpha * uA[i]) * rB + (dpB[i] + beta * duB[i] + d_beta * uB[i]) * rA) /
             (rA + rB);
}

// G_i = d(J^T e_i)/dq  (n x n) for constraint row i
static void constraintForcesJacobian(const World& w, const Kin<double>& k, const Snapshot& snap, int row, Mat& G) {
  const int n = w.n;
  G.assign(n * n, 0.0);
  const Contact& c = snap.contacts[snap.rowContact[row]];
  const int dirIdx = snap.rowDirIdx[row];
  const double* d = &snap.rowDir[3 * row];
  const double* p = c.point;
  double wr[6];
  cross3(p, d, wr);
  wr[3] = d[0]; wr[4] = d[1]; wr[5] = d[2];
  auto parentOf = [&](int dof, int body) { return body >= 0 && w.isAncestorOrSelf(w.dofBody[dof], body); };
  for (int kk = 0; kk < n; kk++) {
    double Z[6];
    positionScrew(w, k, snap.q.data(), kk, Z);
    // d wrench / d q_k
    double dp[3] = {0, 0, 0}, dd[3] = {0, 0, 0};
    const bool pa = parentOf(kk, c.bodyA), pb = parentOf(kk, c.bodyB);
    if (pa && pb) { std::fprintf(stderr, "oracle: self-collision gradients not supported\n"); std::abort(); }
    int type = 0;  // 0 none, 1 vertex, 2 face, 3 sphere-to-box, 4 box-to-sphere (getDofContactType :116)
    if (pa || pb) {
      if (c.type == CT_EDGE_EDGE) type = pa ? 5 : 6;  // EDGE_A / EDGE_B
      else if (c.type == CT_SPHERE_SPHERE) type = pa ? 7 : 8;  // SPHERE_A / SPHERE_B
      else if (c.type == CT_SPHERE_PIPE) type = pa ? 9 : 10;  // SPHERE_TO_PIPE / PIPE_TO_SPHERE
      else if (c.type == CT_PIPE_SPHERE) type = pa ? 10 : 9;
      else if (c.type == CT_PIPE_PIPE) type = pa ? 11 : 12;  // PIPE_A / PIPE_B
      // getDofContactType (:166-172, :213-219): PIPE_TO_VERTEX 13,
      // VERTEX_TO_PIPE 14, PIPE_TO_EDGE 15, EDGE_TO_PIPE 16
      else if (c.type == CT_PIPE_VERTEX) type = pa ? 13 : 14;
      else if (c.type == CT_VERTEX_PIPE) type = pa ? 14 : 13;
      else if (c.type == CT_PIPE_EDGE) type = pa ? 15 : 16;
      else if (c.type == CT_EDGE_PIPE) type = pa ? 16 : 15;
      else if (c.type == CT_SPHERE_BOX) type = pa ? 3 : 4;
      else if (c.type == CT_BOX_SPHERE) type = pa ? 4 : 3;
      else if (c.type == CT_VERTEX_FACE) type = pa ? 1 : 2;
      else type = pa ? 2 : 1;
    }
    const double wv[3] = {Z[0], Z[1], Z[2]}, vv[3] = {Z[3], Z[4], Z[5]};
    // math::gradientWrtTheta(worldTwist, x, 0) (dart/math/Geometry.cpp:968)
    auto gwt = [&](const double* x, double* out) {
      if (std::sqrt(wv[0] * wv[0] + wv[1] * wv[1] + wv[2] * wv[2]) > 1e-6) {
        cross3(wv, x, out);
        for (int i = 0; i < 3; i++) out[i] += vv[i];
      } else {
        for (int i = 0; i < 3; i++) out[i] = vv[i];
      }
    };
    // remove the components along the locked box faces (:356-372)
    auto lockProject = [&](double* x) {
      for (int f = 0; f < 3; f++) {
        if (!c.faceLocked[f]) continue;
        const double* fn = c.faceNormal + 3 * f;
        const double d0 = fn[0] * x[0] + fn[1] * x[1] + fn[2] * x[2];
        for (int i = 0; i < 3; i++) x[i] -= fn[i] * d0;
      }
    };
    if (type == 3 || type == 4) {
      double sg[3], dn[3];
      gwt(c.sphereCenter, sg);
      const double* nrm = c.normal;
      double dist2 = 0;
      for (int i = 0; i < 3; i++) dist2 += (c.sphereCenter[i] - p[i]) * (c.sphereCenter[i] - p[i]);
      const double norm = std::sqrt(dist2);
      if (type == 3) {  // SPHERE_TO_BOX
        for (int i = 0; i < 3; i++) dp[i] = sg[i];
        lockProject(dp);
        double cpg[3], spg[3];
        for (int i = 0; i < 3; i++) { cpg[i] = dp[i]; spg[i] = sg[i]; }
        if (norm > 1e-5)
          for (int i = 0; i < 3; i++) { cpg[i] /= norm; spg[i] /= norm; }
        for (int i = 0; i < 3; i++) dn[i] = c.type == CT_BOX_SPHERE ? cpg[i] - spg[i] : spg[i] - cpg[i];
      } else {  // BOX_TO_SPHERE
        double neg[3];
        for (int i = 0; i < 3; i++) neg[i] = -sg[i];
        lockProject(neg);
        double pg[3];
        gwt(p, pg);
        for (int i = 0; i < 3; i++) dp[i] = pg[i] + neg[i];
        double cpg[3];
        for (int i = 0; i < 3; i++) cpg[i] = dp[i];
        if (norm > 1e-5)
          for (int i = 0; i < 3; i++) cpg[i] /= norm;
        for (int i = 0; i < 3; i++) dn[i] = c.type == CT_BOX_SPHERE ? cpg[i] : -cpg[i];
      }
      const double dnn = dn[0] * nrm[0] + dn[1] * nrm[1] + dn[2] * nrm[2];
      for (int i = 0; i < 3; i++) dn[i] -= dnn * nrm[i];
      // getContactForceGradient (:1092)
      if (dirIdx == 0 || dn[0] * dn[0] + dn[1] * dn[1] + dn[2] * dn[2] <= 1e-12) {
        for (int i = 0; i < 3; i++) dd[i] = dn[i];
      } else {
        double T0[3], T1[3];
        tangentBasisGradient(c.normal, dn, T0, T1);
        for (int i = 0; i < 3; i++) dd[i] = dirIdx == 1 ? T0[i] : T1[i];
      }
    } else if (type == 7 || type == 8) {
      // SPHERE_A / SPHERE_B: the contact point moves with its sphere's centre
      // weighted by the other radius (:343 / :348); the normal by the centre's
      // motion over the centre distance, projected off the normal (:625 / :634)
      const bool A = type == 7;
      const double* cen = A ? c.sphereCenter : c.centerB;
      const double wt = (A ? c.radiusB : c.radiusA) / (c.radiusA + c.radiusB);
      double g[3], dn[3];
      gwt(cen, g);
      for (int i = 0; i < 3; i++) dp[i] = wt * g[i];
      double dist2 = 0;
      for (int i = 0; i < 3; i++) dist2 += (c.sphereCenter[i] - c.centerB[i]) * (c.sphereCenter[i] - c.centerB[i]);
      const double norm = std::sqrt(dist2);
      for (int i = 0; i < 3; i++) dn[i] = g[i] / norm;
      const double dnn = dn[0] * c.normal[0] + dn[1] * c.normal[1] + dn[2] * c.normal[2];
      for (int i = 0; i < 3; i++) dn[i] = (A ? 1.0 : -1.0) * (dn[i] - dnn * c.normal[i]);
      if (dirIdx == 0 || dn[0] * dn[0] + dn[1] * dn[1] + dn[2] * dn[2] <= 1e-12) {
        for (int i = 0; i < 3; i++) dd[i] = dn[i];
      } else {
        double T0[3], T1[3];
        tangentBasisGradient(c.normal, dn, T0, T1);
        for (int i = 0; i < 3; i++) dd[i] = dirIdx == 1 ? T0[i] : T1[i];
      }
    } else if (type == 9 || type == 10) {
      // SPHERE_TO_PIPE (:484 point, :819 normal): the sphere centre's motion,
      // its off-axis part weighted by the pipe radius; PIPE_TO_SPHERE (:496,
      // :837): the motion of the axis point closest to the sphere centre
      // (math::closestPointOnLineGradient, Geometry.cpp:4427)
      const double* dir = c.pipeDir;
      double g[3], dn[3];
      if (type == 9) {
        gwt(c.sphereCenter, g);
        const double par = dir[0] * g[0] + dir[1] * g[1] + dir[2] * g[2];
        const double wt = c.pipeRadius / (c.sphereRadius + c.pipeRadius);
        for (int i = 0; i < 3; i++) { dp[i] = par * dir[i] + wt * (g[i] - par * dir[i]); dn[i] = g[i] - par * dir[i]; }
      } else {
        double fg[3], dg[3];
        gwt(c.pipeFixed, fg);
        cross3(wv, dir, dg);  // gradientWrtThetaPureRotation
        double off = 0, dOff = 0, gOff = 0, dGOff = 0;
        for (int i = 0; i < 3; i++) {
          off += dir[i] * c.pipeFixed[i];
          dOff += dg[i] * c.pipeFixed[i] + dir[i] * fg[i];
          gOff += dir[i] * c.sphereCenter[i];
          dGOff += dg[i] * c.sphereCenter[i];
        }
        const double rel = gOff - off, dRel = dGOff - dOff;
        for (int i = 0; i < 3; i++) g[i] = fg[i] + rel * dg[i] + dRel * dir[i];
        const double wt = c.sphereRadius / (c.sphereRadius + c.pipeRadius);
        for (int i = 0; i < 3; i++) { dp[i] = wt * g[i]; dn[i] = g[i]; }
      }
      double dist2 = 0;
      for (int i = 0; i < 3; i++) dist2 += (c.pipeClosest[i] - c.sphereCenter[i]) * (c.pipeClosest[i] - c.sphereCenter[i]);
      const double norm = std::sqrt(dist2);
      for (int i = 0; i < 3; i++) dn[i] /= norm;
      const double dnn = dn[0] * c.normal[0] + dn[1] * c.normal[1] + dn[2] * c.normal[2];
      const bool plus = type == 9 ? c.type == CT_SPHERE_PIPE : c.type == CT_PIPE_SPHERE;
      for (int i = 0; i < 3; i++) dn[i] = (plus ? 1.0 : -1.0) * (dn[i] - dnn * c.normal[i]);
      if (dirIdx == 0 || dn[0] * dn[0] + dn[1] * dn[1] + dn[2] * dn[2] <= 1e-12) {
        for (int i = 0; i < 3; i++) dd[i] = dn[i];
      } else {
        double T0[3], T1[3];
        tangentBasisGradient(c.normal, dn, T0, T1);
        for (int i = 0; i < 3; i++) dd[i] = dirIdx == 1 ? T0[i] : T1[i];
      }
    } else if (type == 13 || type == 14) {
      // VERTEX_TO_PIPE (:408 point: the vertex moves; :940 normal) /
      // PIPE_TO_VERTEX (:334 point fixed; :967 normal): the axis point
      // closest to the vertex through math::closestPointOnLineGradient
      double g[3] = {0, 0, 0}, cg[3], dn[3], fg[3] = {0, 0, 0}, dg[3] = {0, 0, 0};
      if (type == 14) {
        gwt(p, g);
        for (int i = 0; i < 3; i++) dp[i] = g[i];
      } else {
        gwt(c.pipeFixed, fg);
        cross3(wv, c.pipeDir, dg);  // gradientWrtThetaPureRotation
      }
      double off = 0, dOff = 0, gOff = 0, dGOff = 0;
      for (int i = 0; i < 3; i++) {
        off += c.pipeDir[i] * c.pipeFixed[i];
        dOff += dg[i] * c.pipeFixed[i] + c.pipeDir[i] * fg[i];
        gOff += c.pipeDir[i] * p[i];
        dGOff += dg[i] * p[i] + c.pipeDir[i] * g[i];
      }
      const double rel = gOff - off, dRel = dGOff - dOff;
      for (int i = 0; i < 3; i++) cg[i] = fg[i] + rel * dg[i] + dRel * c.pipeDir[i];
      double dist2 = 0;
      for (int i = 0; i < 3; i++) dist2 += (c.pipeClosest[i] - p[i]) * (c.pipeClosest[i] - p[i]);
      const double norm = std::sqrt(dist2);
      for (int i = 0; i < 3; i++) dn[i] = (cg[i] - g[i]) / norm;
      const double dnn = dn[0] * c.normal[0] + dn[1] * c.normal[1] + dn[2] * c.normal[2];
      const double sg = c.type == CT_PIPE_VERTEX ? 1.0 : -1.0;
      for (int i = 0; i < 3; i++) dn[i] = sg * (dn[i] - dnn * c.normal[i]);
      if (dirIdx == 0 || dn[0] * dn[0] + dn[1] * dn[1] + dn[2] * dn[2] <= 1e-12) {
        for (int i = 0; i < 3; i++) dd[i] = dn[i];
      } else {
        double T0[3], T1[3];
        tangentBasisGradient(c.normal, dn, T0, T1);
        for (int i = 0; i < 3; i++) dd[i] = dirIdx == 1 ? T0[i] : T1[i];
      }
    } else if (type == 15 || type == 16) {
      // PIPE_TO_EDGE / EDGE_TO_PIPE (:538 / :555 point, :1029 / :1075 normal):
      // math::getContactPointGradient of the edge and the pipe axis with
      // radii (0, 1) -- the contact point -- and (1, 0)
      const bool pipeMoves = type == 15;
      double fg[3], dg[3], zero[3] = {0, 0, 0}, other[3], dn[3];
      gwt(pipeMoves ? c.pipeFixed : c.edgeAFixed, fg);
      cross3(wv, pipeMoves ? c.pipeDir : c.edgeADir, dg);
      const double* dpE = pipeMoves ? zero : fg; const double* duE = pipeMoves ? zero : dg;
      const double* dpP = pipeMoves ? fg : zero; const double* duP = pipeMoves ? dg : zero;
      contactPointGradient(c.edgeAFixed, dpE, c.edgeADir, duE, c.pipeFixed, dpP, c.pipeDir, duP, dp, 0.0, 1.0);
      contactPointGradient(c.edgeAFixed, dpE, c.edgeADir, duE, c.pipeFixed, dpP, c.pipeDir, duP, other, 1.0, 0.0);
      double dist2 = 0;
      for (int i = 0; i < 3; i++) dist2 += (c.edgeAClosest[i] - c.pipeClosest[i]) * (c.edgeAClosest[i] - c.pipeClosest[i]);
      const double norm = std::sqrt(dist2);
      for (int i = 0; i < 3; i++) dn[i] = (other[i] - dp[i]) / norm;
      const double dnn = dn[0] * c.normal[0] + dn[1] * c.normal[1] + dn[2] * c.normal[2];
      const double sg = c.type == CT_PIPE_EDGE ? 1.0 : -1.0;
      for (int i = 0; i < 3; i++) dn[i] = sg * (dn[i] - dnn * c.normal[i]);
      if (dirIdx == 0 || dn[0] * dn[0] + dn[1] * dn[1] + dn[2] * dn[2] <= 1e-12) {
        for (int i = 0; i < 3; i++) dd[i] = dn[i];
      } else {
        double T0[3], T1[3];
        tangentBasisGradient(c.normal, dn, T0, T1);
        for (int i = 0; i < 3; i++) dd[i] = dirIdx == 1 ? T0[i] : T1[i];
      }
    } else if (type == 11 || type == 12) {
      // PIPE_A / PIPE_B (:510 / :529 point, :862 / :901 normal): the moving
      // axis's fixed point and direction through math::getContactPointGradient
      // with the contact's (normalised) radii; the normal from the two
      // closest points' gradients (radii 0/1 and 1/0) over their distance
      const bool A = type == 11;
      double fg[3], dg[3], zero[3] = {0, 0, 0}, ca[3], cb[3], dn[3];
      gwt(A ? c.edgeAFixed : c.edgeBFixed, fg);
      cross3(wv, A ? c.edgeADir : c.edgeBDir, dg);
      const double* dpA = A ? fg : zero; const double* duA = A ? dg : zero;
      const double* dpB = A ? zero : fg; const double* duB = A ? zero : dg;
      contactPointGradient(c.edgeAFixed, dpA, c.edgeADir, duA, c.edgeBFixed, dpB, c.edgeBDir, duB, dp, c.radiusA,
                           c.radiusB);
      contactPointGradient(c.edgeAFixed, dpA, c.edgeADir, duA, c.edgeBFixed, dpB, c.edgeBDir, duB, ca, 0.0, 1.0);
      contactPointGradient(c.edgeAFixed, dpA, c.edgeADir, duA, c.edgeBFixed, dpB, c.edgeBDir, duB, cb, 1.0, 0.0);
      double dist2 = 0;
      for (int i = 0; i < 3; i++) dist2 += (c.edgeAClosest[i] - c.edgeBClosest[i]) * (c.edgeAClosest[i] - c.edgeBClosest[i]);
      const double norm = std::sqrt(dist2);
      for (int i = 0; i < 3; i++) dn[i] = (ca[i] - cb[i]) / norm;
      const double dnn = dn[0] * c.normal[0] + dn[1] * c.normal[1] + dn[2] * c.normal[2];
      for (int i = 0; i < 3; i++) dn[i] -= dnn * c.normal[i];
      if (dirIdx == 0 || dn[0] * dn[0] + dn[1] * dn[1] + dn[2] * dn[2] <= 1e-12) {
        for (int i = 0; i < 3; i++) dd[i] = dn[i];
      } else {
        double T0[3], T1[3];
        tangentBasisGradient(c.normal, dn, T0, T1);
        for (int i = 0; i < 3; i++) dd[i] = dirIdx == 1 ? T0[i] : T1[i];
      }
    } else if (type == 1) {
      // math::gradientWrtTheta(worldTwist, contactPos, 0)
      if (std::sqrt(wv[0] * wv[0] + wv[1] * wv[1] + wv[2] * wv[2]) > 1e-6) {
        cross3(wv, p, dp);
        for (int i = 0; i < 3; i++) dp[i] += vv[i];
      } else {
        for (int i = 0; i < 3; i++) dp[i] = vv[i];
      }
    } else if (type == 5 || type == 6) {
      // EDGE_A / EDGE_B (:412, :429): the contact point moves with the
      // closest approach of the two edges (math::getContactPointGradient,
      // Geometry.cpp:1129), the normal with the moving edge's direction
      // (:708, :722; not renormalised, as in the reference)
      const bool A = type == 5;
      double fg[3], dg[3], zero[3] = {0, 0, 0};
      gwt(A ? c.edgeAFixed : c.edgeBFixed, fg);
      cross3(wv, A ? c.edgeADir : c.edgeBDir, dg);  // gradientWrtThetaPureRotation
      contactPointGradient(c.edgeAFixed, A ? fg : zero, c.edgeADir, A ? dg : zero, c.edgeBFixed, A ? zero : fg,
                           c.edgeBDir, A ? zero : dg, dp);
      double nb[3];
      cross3(c.edgeBDir, c.edgeADir, nb);
      const double sign = (nb[0] * c.normal[0] + nb[1] * c.normal[1] + nb[2] * c.normal[2] < 0) ? -1.0 : 1.0;
      double dn[3];
      if (A) cross3(c.edgeBDir, dg, dn);
      else cross3(dg, c.edgeADir, dn);
      for (int i = 0; i < 3; i++) dn[i] *= sign;
      if (dirIdx == 0 || dn[0] * dn[0] + dn[1] * dn[1] + dn[2] * dn[2] <= 1e-12) {
        for (int i = 0; i < 3; i++) dd[i] = dn[i];
      } else {
        double T0[3], T1[3];
        tangentBasisGradient(c.normal, dn, T0, T1);
        for (int i = 0; i < 3; i++) dd[i] = dirIdx == 1 ? T0[i] : T1[i];
      }
    } else if (type == 2) {
      double dn[3];
      cross3(wv, c.normal, dn);  // gradientWrtThetaPureRotation
      if (dirIdx == 0 || dn[0] * dn[0] + dn[1] * dn[1] + dn[2] * dn[2] <= 1e-12) {
        for (int i = 0; i < 3; i++) dd[i] = dn[i];
      } else {
        double T0[3], T1[3];
        tangentBasisGradient(c.normal, dn, T0, T1);
        for (int i = 0; i < 3; i++) dd[i] = dirIdx == 1 ? T0[i] : T1[i];
      }
    }
    double dwr[6], t1[3], t2[3];
    cross3(p, dd, t1);
    cross3(dp, d, t2);
    for (int i = 0; i < 3; i++) { dwr[i] = t1[i] + t2[i]; dwr[3 + i] = dd[i]; }
    for (int r = 0; r < n; r++) {
      const bool ra = parentOf(r, c.bodyA), rb = parentOf(r, c.bodyB);
      double mult = (ra && rb) ? 0.0 : (ra ? 1.0 : (rb ? -1.0 : 0.0));
      if (mult == 0.0) continue;
      double S[6];
      velocityScrew(w, k, r, S);
      double val = 0;
      // screw-axis gradient: k's joint at or above r's joint
      const int bk = w.dofBody[kk], br = w.dofBody[r];
      if (w.isAncestorOrSelf(bk, br)) {
        // (a multi-dof joint's axes move with its own coordinates; a 1-dof
        // joint's axis does not, and a translational joint's pure
        // translations give ad(Z, S) = 0 either way)
        if (bk != br || w.bodies[bk].ndof > 1) {
          V6<double> zz, ss;
          for (int i = 0; i < 6; i++) { zz[i] = Z[i]; ss[i] = S[i]; }
          V6<double> g = ad(zz, ss);
          for (int i = 0; i < 6; i++) val += g[i] * wr[i];
        }
      }
      for (int i = 0; i < 6; i++) val += S[i] * dwr[i];
      G[r * n + kk] = mult * val;
    }
  }
}

void positionConstraintTerms(const World& w, const Snapshot& snap, const Mat& Minv, const Mat& C, const Mat& dCq,
                             const Mat& Ac, const Mat& Aub, const Mat& AcubE, const Mat& Qin, Mat& dFcPos,
                             Mat& dAcf) {
  const int n = w.n, m = snap.numRows, nc = snap.numClamping, nu = snap.numUpperBound;
  const double dt = w.dt;
  Kin<double> k;
  k.compute(w, snap.q.data(), snap.v.data());
  // per-row G matrices for clamping / upper-bound rows
  std::vector<Mat> Gc(nc), Gu(nu);
  for (int j = 0; j < m; j++) {
    if (snap.mapping[j] == CM_CLAMPING) constraintForcesJacobian(w, k, snap, j, Gc[snap.clampingIndex[j]]);
    else if (snap.mapping[j] >= 0) constraintForcesJacobian(w, k, snap, j, Gu[snap.upperBoundIndex[j]]);
  }
  auto dAc = [&](const Mat& f0) {  // getJacobianOfClampingConstraints: sum f0_i G_i
    Mat R(n * n, 0.0);
    for (int i = 0; i < nc; i++)
      if (f0[i] != 0.0) for (int t = 0; t < n * n; t++) R[t] += f0[i] * Gc[i][t];
    return R;
  };
  auto dAub = [&](const Mat& f0) {
    Mat R(n * n, 0.0);
    for (int i = 0; i < nu; i++)
      if (f0[i] != 0.0) for (int t = 0; t < n * n; t++) R[t] += f0[i] * Gu[i][t];
    return R;
  };
  auto dAcT = [&](const Mat& v0) {  // getJacobianOfClampingConstraintsTranspose: nc x n
    Mat R(nc * n, 0.0);
    for (int i = 0; i < nc; i++)
      for (int kk = 0; kk < n; kk++) {
        double s = 0;
        for (int r = 0; r < n; r++) s += Gc[i][r * n + kk] * v0[r];
        R[i * n + kk] = s;
      }
    return R;
  };
  auto dAubT = [&](const Mat& v0) {
    Mat R(nu * n, 0.0);
    for (int i = 0; i < nu; i++)
      for (int kk = 0; kk < n; kk++) {
        double s = 0;
        for (int r = 0; r < n; r++) s += Gu[i][r * n + kk] * v0[r];
        R[i * n + kk] = s;
      }
    return R;
  };
  auto mv = [&](const Mat& A, const Mat& x, int rows, int cols) {
    Mat y(rows, 0.0);
    for (int r = 0; r < rows; r++) { double s = 0; for (int c = 0; c < cols; c++) s += A[r * cols + c] * x[c]; y[r] = s; }
    return y;
  };
  auto mm = [&](const Mat& A, const Mat& B, int r, int kk, int c) {
    Mat Cm(r * c, 0.0);
    for (int i = 0; i < r; i++)
      for (int t = 0; t < kk; t++) {
        double a = A[i * kk + t];
        if (a == 0.0) continue;
        for (int j = 0; j < c; j++) Cm[i * c + j] += a * B[t * c + j];
      }
    return Cm;
  };
  auto tr = [&](const Mat& A, int r, int c) {
    Mat T(r * c);
    for (int i = 0; i < r; i++) for (int j = 0; j < c; j++) T[j * r + i] = A[i * c + j];
    return T;
  };
  auto jacMinv = [&](const Mat& x) {  // getJacobianOfMinv(x, POSITION) = -Minv d(M Minv x)/dq
    Mat y = mv(Minv, x, n, n);
    Mat dMy(n * n);
    w.jacobianOfMy(snap.q.data(), y.data(), dMy.data());
    Mat R = mm(Minv, dMy, n, n, n);
    for (auto& v : R) v = -v;
    return R;
  };
  Mat f = snap.fc;
  Mat E = snap.E;
  Mat Ef = mv(E, f, nu, nc);
  // dA_c f + dA_ub E f
  dAcf = dAc(f);
  {
    Mat t = dAub(Ef);
    for (int i = 0; i < n * n; i++) dAcf[i] += t[i];
  }
  // dB (POSITION), getJacobianOfLCPOffsetClampingSubset:
  //   -bounce .* (dA_c^T(v_f) + A_c^T dt (dMinv_f - Minv dC - Minv K))
  Mat fext(n);
  for (int i = 0; i < n; i++) {
    double springF = w.spring[i] * (snap.q[i] - w.restPos[i] + dt * snap.v[i]);
    fext[i] = snap.tau[i] - C[i] - w.damping[i] * snap.v[i] - springF;
  }
  Mat dMinvF = jacMinv(fext);
  Mat inner(n * n);
  {
    Mat MdC = mm(Minv, dCq, n, n, n);
    for (int r = 0; r < n; r++)
      for (int c = 0; c < n; c++) inner[r * n + c] = dMinvF[r * n + c] - MdC[r * n + c] - Minv[r * n + c] * w.spring[c];
  }
  Mat dB = dAcT(snap.preConstraintV);
  {
    Mat AcT = tr(Ac, n, nc);
    Mat t = mm(AcT, inner, nc, n, n);
    for (int i = 0; i < nc; i++)
      for (int c = 0; c < n; c++) dB[i * n + c] = -snap.bounceDiag[i] * (dB[i * n + c] + dt * t[i * n + c]);
  }
  // Q pseudo-inverse and Q^+ dB
  const Mat& Q = Qin;
  Mat Qinv(nc * nc);
  {
    Mat e(nc), col(nc);
    for (int c = 0; c < nc; c++) {
      std::fill(e.begin(), e.end(), 0.0);
      e[c] = 1.0;
      codSolve(Q.data(), nc, nc, e.data(), col.data());
      for (int r = 0; r < nc; r++) Qinv[r * nc + c] = col[r];
    }
  }
  auto Qsolve = [&](const Mat& R, int cols) {  // column-wise COD solve
    Mat out(nc * cols), bb(nc), xx(nc);
    for (int c = 0; c < cols; c++) {
      for (int r = 0; r < nc; r++) bb[r] = R[r * cols + c];
      codSolve(Q.data(), nc, nc, bb.data(), xx.data());
      for (int r = 0; r < nc; r++) out[r * cols + c] = xx[r];
    }
    return out;
  };
  Mat AcT = tr(Ac, n, nc);
  Mat AubT = tr(Aub, n, nu);
  auto dQ = [&](const Mat& rhs) {  // nc x n
    Mat AcubErhs = mv(AcubE, rhs, n, nc);
    Mat MA = mv(Minv, AcubErhs, n, n);
    Mat R = dAcT(MA);
    Mat J = jacMinv(AcubErhs);
    Mat inner2 = dAc(rhs);
    if (nu > 0) {
      Mat Erhs = mv(E, rhs, nu, nc);
      Mat t = dAub(Erhs);
      for (int i = 0; i < n * n; i++) inner2[i] += t[i];
    }
    Mat MI = mm(Minv, inner2, n, n, n);
    for (int i = 0; i < n * n; i++) J[i] += MI[i];
    Mat t2 = mm(AcT, J, nc, n, n);
    for (int i = 0; i < nc * n; i++) R[i] += t2[i];
    return R;
  };
  auto dQT = [&](const Mat& rhs) {  // nc x n
    Mat Acrhs = mv(Ac, rhs, n, nc);
    Mat MA = mv(Minv, Acrhs, n, n);
    Mat J = jacMinv(Acrhs);
    Mat MI = mm(Minv, dAc(rhs), n, n, n);
    for (int i = 0; i < n * n; i++) J[i] += MI[i];
    Mat R = dAcT(MA);
    Mat t2 = mm(AcT, J, nc, n, n);
    for (int i = 0; i < nc * n; i++) R[i] += t2[i];
    if (nu > 0) {
      Mat U = dAubT(MA);
      Mat t3 = mm(AubT, J, nu, n, n);
      for (int i = 0; i < nu * n; i++) U[i] += t3[i];
      Mat ET = tr(E, nu, nc);
      Mat t4 = mm(ET, U, nc, nu, n);
      for (int i = 0; i < nc * n; i++) R[i] += t4[i];
    }
    return R;
  };
  Mat b(nc, 0.0);
  for (int j = 0; j < m; j++)
    if (snap.mapping[j] == CM_CLAMPING) b[snap.clampingIndex[j]] = snap.lcpB[j];
  // imprecision map I - Q Q^+
  Mat imp(nc * nc);
  double impNorm = 0;
  {
    Mat QQ = mm(Q, Qinv, nc, nc, nc);
    for (int r = 0; r < nc; r++)
      for (int c = 0; c < nc; c++) {
        imp[r * nc + c] = (r == c ? 1.0 : 0.0) - QQ[r * nc + c];
        impNorm += imp[r * nc + c] * imp[r * nc + c];
      }
  }
  Mat Qb(nc);
  codSolve(Q.data(), nc, nc, b.data(), Qb.data());
  Mat dQb = Qsolve(dQ(Qb), n);
  for (auto& v : dQb) v = -v;
  if (impNorm >= 1e-18) {
    // full pseudo-inverse gradient (mathoverflow 29511), BackpropSnapshot.cpp:2960
    Mat impb = mv(imp, b, nc, nc);
    Mat QinvT = tr(Qinv, nc, nc);
    Mat t1 = Qsolve(mm(QinvT, dQT(impb), nc, nc, n), n);
    Mat IQQ(nc * nc);
    Mat QiQ = mm(Qinv, Q, nc, nc, nc);
    for (int r = 0; r < nc; r++)
      for (int c = 0; c < nc; c++) IQQ[r * nc + c] = (r == c ? 1.0 : 0.0) - QiQ[r * nc + c];
    Mat t2 = mm(IQQ, dQT(mv(QinvT, Qb, nc, nc)), nc, nc, n);
    for (int i = 0; i < nc * n; i++) dQb[i] += t1[i] + t2[i];
  }
  Mat QdB = Qsolve(dB, n);
  dFcPos.assign(nc * n, 0.0);
  for (int i = 0; i < nc * n; i++) dFcPos[i] = dQb[i] + QdB[i];
}

}  // namespace oracle
