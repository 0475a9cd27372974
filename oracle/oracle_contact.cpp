// ORACLE / TEST INFRASTRUCTURE ONLY -- see nimble_oracle.cpp header.
//
// Contacts on the timestep hot path, restated:
//  * box-box narrow phase: dart/collision/dart/DARTCollide.cpp:764 dBoxBox
//    (Nimble's variant: 15 separating axes with the 1.05 fudge factor on edge
//    axes, incident-face clipping intersectRectQuad :513, all clipped points
//    kept, contact typing VERTEX_FACE / FACE_VERTEX / EDGE_EDGE);
//  * detector loop + filter: DARTCollisionDetector.cpp:127, postProcess :357,
//    CollisionFilter.cpp:105;
//  * ContactConstraint (dart/constraint/ContactConstraint.cpp): spatial normals
//    :115-200, getInformation :393, tangent basis :705;
//  * BoxedLcpConstraintSolver::buildLcpInputs / solveLcp
//    (BoxedLcpConstraintSolver.cpp:175, :330) with the gradient short-circuit;
//  * ConstrainedGroupGradientMatrices::constructMatrices (:482) and
//    opportunisticallyStandardizeResults (:218);
//  * LCPUtils (LCPUtils.cpp): isLCPSolutionValid, guessSolution, reduce,
//    removeFriction;
//  * BackpropSnapshot Jacobian pieces for the clamping set
//    (BackpropSnapshot.cpp:980 getVelJacobianWrt, :2723
//    getJacobianOfConstraintForce, :3181 getJacobianOfLCPOffsetClampingSubset).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>

#include "oracle_lcp.hpp"

namespace oracle {

void codSolve(const double* A, int m, int n, const double* b, double* x);
bool pgsSolveLCP(int n, double* A, double* x, double* b, double* lo, double* hi, const int* findex);

static const double kInf = std::numeric_limits<double>::infinity();
enum { CT_FACE_VERTEX = 1, CT_VERTEX_FACE = 2, CT_EDGE_EDGE = 3, CT_SPHERE_SPHERE = 6, CT_SPHERE_PIPE = 7,
       CT_PIPE_SPHERE = 8, CT_PIPE_PIPE = 9 };

//------------------------------------------------------------------------------
// dBoxBox restatement.  R? are 3x3 row-major world rotations, p? centres,
// A/B half sizes.  Appends contacts (normal from box 2 into box 1).
static int boxBox(const double* p1, const double* R1, const double* A, const double* p2, const double* R2,
                  const double* B, double clipDepth, std::vector<Contact>& out, int s1, int s2, int b1, int b2) {
  const double fudge = 1.05;
  auto col = [](const double* R, int c, double* o) { o[0] = R[c]; o[1] = R[3 + c]; o[2] = R[6 + c]; };
  double p[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  double pp[3];
  for (int i = 0; i < 3; i++) pp[i] = R1[i] * p[0] + R1[3 + i] * p[1] + R1[6 + i] * p[2];  // R1^T p
  double Rm[3][3], Q[3][3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      Rm[i][j] = R1[i] * R2[j] + R1[3 + i] * R2[3 + j] + R1[6 + i] * R2[6 + j];  // R1^T R2
      Q[i][j] = std::fabs(Rm[i][j]);
    }
  double s = -1e12;
  int invertNormal = 0, code = 0;
  int normalCol = -1, normalBox = 0;  // face normal = column of R1 (box 1) or R2 (box 2)
  double normalC[3] = {0, 0, 0};
  auto tstFace = [&](double e1, double e2, int box, int colIdx, int cc) {
    double s2v = std::fabs(e1) - e2;
    if (s2v > s) { s = s2v; normalBox = box; normalCol = colIdx; invertNormal = e1 < 0; code = cc; }
  };
  tstFace(pp[0], A[0] + B[0] * Q[0][0] + B[1] * Q[0][1] + B[2] * Q[0][2], 1, 0, 1);
  tstFace(pp[1], A[1] + B[0] * Q[1][0] + B[1] * Q[1][1] + B[2] * Q[1][2], 1, 1, 2);
  tstFace(pp[2], A[2] + B[0] * Q[2][0] + B[1] * Q[2][1] + B[2] * Q[2][2], 1, 2, 3);
  for (int j = 0; j < 3; j++) {
    double c2[3];
    col(R2, j, c2);
    double e1 = c2[0] * p[0] + c2[1] * p[1] + c2[2] * p[2];
    double e2 = A[0] * Q[0][j] + A[1] * Q[1][j] + A[2] * Q[2][j] + B[j];
    tstFace(e1, e2, 2, j, 4 + j);
  }
  auto tstEdge = [&](double e1, double e2, double n1, double n2, double n3, int cc) {
    double s2v = std::fabs(e1) - e2;
    double l = std::sqrt(n1 * n1 + n2 * n2 + n3 * n3);
    if (l > 0) {
      s2v /= l;
      if (s2v * fudge > s) {
        s = s2v; normalCol = -1; normalC[0] = n1 / l; normalC[1] = n2 / l; normalC[2] = n3 / l;
        invertNormal = e1 < 0; code = cc;
      }
    }
  };
  const double R11 = Rm[0][0], R12 = Rm[0][1], R13 = Rm[0][2], R21 = Rm[1][0], R22 = Rm[1][1], R23 = Rm[1][2],
               R31 = Rm[2][0], R32 = Rm[2][1], R33 = Rm[2][2];
  const double Q11 = Q[0][0], Q12 = Q[0][1], Q13 = Q[0][2], Q21 = Q[1][0], Q22 = Q[1][1], Q23 = Q[1][2],
               Q31 = Q[2][0], Q32 = Q[2][1], Q33 = Q[2][2];
  tstEdge(pp[2] * R21 - pp[1] * R31, A[1] * Q31 + A[2] * Q21 + B[1] * Q13 + B[2] * Q12, 0, -R31, R21, 7);
  tstEdge(pp[2] * R22 - pp[1] * R32, A[1] * Q32 + A[2] * Q22 + B[0] * Q13 + B[2] * Q11, 0, -R32, R22, 8);
  tstEdge(pp[2] * R23 - pp[1] * R33, A[1] * Q33 + A[2] * Q23 + B[0] * Q12 + B[1] * Q11, 0, -R33, R23, 9);
  tstEdge(pp[0] * R31 - pp[2] * R11, A[0] * Q31 + A[2] * Q11 + B[1] * Q23 + B[2] * Q22, R31, 0, -R11, 10);
  tstEdge(pp[0] * R32 - pp[2] * R12, A[0] * Q32 + A[2] * Q12 + B[0] * Q23 + B[2] * Q21, R32, 0, -R12, 11);
  tstEdge(pp[0] * R33 - pp[2] * R13, A[0] * Q33 + A[2] * Q13 + B[0] * Q22 + B[1] * Q21, R33, 0, -R13, 12);
  tstEdge(pp[1] * R11 - pp[0] * R21, A[0] * Q21 + A[1] * Q11 + B[1] * Q33 + B[2] * Q32, -R21, R11, 0, 13);
  tstEdge(pp[1] * R12 - pp[0] * R22, A[0] * Q22 + A[1] * Q12 + B[0] * Q33 + B[2] * Q31, -R22, R12, 0, 14);
  tstEdge(pp[1] * R13 - pp[0] * R23, A[0] * Q23 + A[1] * Q13 + B[0] * Q32 + B[1] * Q31, -R23, R13, 0, 15);
  if (!code) return 0;
  if (s > 0.0) return 0;
  double normal[3];
  if (normalCol >= 0) {
    col(normalBox == 1 ? R1 : R2, normalCol, normal);
  } else {
    for (int i = 0; i < 3; i++) normal[i] = R1[i * 3] * normalC[0] + R1[i * 3 + 1] * normalC[1] + R1[i * 3 + 2] * normalC[2];
    double l = std::sqrt(normal[0] * normal[0] + normal[1] * normal[1] + normal[2] * normal[2]);
    for (int i = 0; i < 3; i++) normal[i] /= l;
  }
  if (invertNormal) for (int i = 0; i < 3; i++) normal[i] = -normal[i];

  if (code > 6) {
    // edge-edge (DARTCollide.cpp:992)
    double pa[3] = {p1[0], p1[1], p1[2]}, pb[3] = {p2[0], p2[1], p2[2]};
    for (int j = 0; j < 3; j++) {
      double c1[3]; col(R1, j, c1);
      double v = normal[0] * c1[0] + normal[1] * c1[1] + normal[2] * c1[2];
      double sign = (v > -1e-10) ? 1.0 : -1.0;
      for (int i = 0; i < 3; i++) pa[i] += sign * A[j] * c1[i];
    }
    for (int j = 0; j < 3; j++) {
      double c2[3]; col(R2, j, c2);
      double v = normal[0] * c2[0] + normal[1] * c2[1] + normal[2] * c2[2];
      double sign = (v > -1e-3) ? -1.0 : 1.0;
      for (int i = 0; i < 3; i++) pb[i] += sign * B[j] * c2[i];
    }
    double ua[3], ub[3];
    col(R1, (code - 7) / 3, ua);
    col(R2, (code - 7) % 3, ub);
    // dLineClosestApproach
    double pd[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]};
    double uaub = ua[0] * ub[0] + ua[1] * ub[1] + ua[2] * ub[2];
    double q1 = ua[0] * pd[0] + ua[1] * pd[1] + ua[2] * pd[2];
    double q2 = -(ub[0] * pd[0] + ub[1] * pd[1] + ub[2] * pd[2]);
    double dd = 1 - uaub * uaub, alpha = 0, beta = 0;
    if (dd > 0) { dd = 1.0 / dd; alpha = (q1 + uaub * q2) * dd; beta = (uaub * q1 + q2) * dd; }
    const double paFixed[3] = {pa[0], pa[1], pa[2]}, pbFixed[3] = {pb[0], pb[1], pb[2]};
    for (int i = 0; i < 3; i++) { pa[i] += ua[i] * alpha; pb[i] += ub[i] * beta; }
    const double pen = -s;
    if (pen > clipDepth) return 0;
    Contact c{};
    c.shapeA = s1; c.shapeB = s2; c.bodyA = b1; c.bodyB = b2;
    for (int i = 0; i < 3; i++) { c.point[i] = 0.5 * (pa[i] + pb[i]); c.normal[i] = -normal[i]; }
    c.depth = pen;
    c.type = CT_EDGE_EDGE;
    // edge metadata (DARTCollide.cpp:1046): fixed points before the closest
    // approach, unit edge directions
    const double la = std::sqrt(ua[0] * ua[0] + ua[1] * ua[1] + ua[2] * ua[2]);
    const double lb = std::sqrt(ub[0] * ub[0] + ub[1] * ub[1] + ub[2] * ub[2]);
    for (int i = 0; i < 3; i++) {
      c.edgeAFixed[i] = paFixed[i]; c.edgeADir[i] = ua[i] / la;
      c.edgeBFixed[i] = pbFixed[i]; c.edgeBDir[i] = ub[i] / lb;
    }
    out.push_back(c);
    return 1;
  }
  // face-something (DARTCollide.cpp:1060)
  const double *Ra, *Rb, *pa, *pb, *Sa, *Sb;
  bool flip;
  if (code <= 3) { Ra = R1; Rb = R2; pa = p1; pb = p2; Sa = A; Sb = B; flip = false; }
  else { Ra = R2; Rb = R1; pa = p2; pb = p1; Sa = B; Sb = A; flip = true; }
  double normal2[3], nr[3], anr[3];
  for (int i = 0; i < 3; i++) normal2[i] = code <= 3 ? normal[i] : -normal[i];
  for (int i = 0; i < 3; i++) nr[i] = Rb[i] * normal2[0] + Rb[3 + i] * normal2[1] + Rb[6 + i] * normal2[2];
  for (int i = 0; i < 3; i++) anr[i] = std::fabs(nr[i]);
  int lanr, a1, a2;
  if (anr[1] > anr[0]) {
    if (anr[1] > anr[2]) { a1 = 0; lanr = 1; a2 = 2; } else { a1 = 0; a2 = 1; lanr = 2; }
  } else {
    if (anr[0] > anr[2]) { lanr = 0; a1 = 1; a2 = 2; } else { a1 = 0; a2 = 1; lanr = 2; }
  }
  double center[3];
  for (int i = 0; i < 3; i++)
    center[i] = nr[lanr] < 0 ? pb[i] - pa[i] + Sb[lanr] * Rb[i * 3 + lanr] : pb[i] - pa[i] - Sb[lanr] * Rb[i * 3 + lanr];
  int codeN = code <= 3 ? code - 1 : code - 4;
  int code1, code2;
  if (codeN == 0) { code1 = 1; code2 = 2; } else if (codeN == 1) { code1 = 0; code2 = 2; } else { code1 = 0; code2 = 1; }
  auto inner = [](const double* R, int ca, const double* Rb2, int cb) {
    return R[ca] * Rb2[cb] + R[3 + ca] * Rb2[3 + cb] + R[6 + ca] * Rb2[6 + cb];
  };
  double c1 = center[0] * Ra[code1] + center[1] * Ra[3 + code1] + center[2] * Ra[6 + code1];
  double c2 = center[0] * Ra[code2] + center[1] * Ra[3 + code2] + center[2] * Ra[6 + code2];
  double m11 = inner(Ra, code1, Rb, a1), m12 = inner(Ra, code1, Rb, a2);
  double m21 = inner(Ra, code2, Rb, a1), m22 = inner(Ra, code2, Rb, a2);
  double quad[8];
  {
    double k1 = m11 * Sb[a1], k2 = m21 * Sb[a1], k3 = m12 * Sb[a2], k4 = m22 * Sb[a2];
    quad[0] = c1 - k1 - k3; quad[1] = c2 - k2 - k4;
    quad[2] = c1 - k1 + k3; quad[3] = c2 - k2 + k4;
    quad[4] = c1 + k1 + k3; quad[5] = c2 + k2 + k4;
    quad[6] = c1 + k1 - k3; quad[7] = c2 + k2 - k4;
  }
  double rect[2] = {Sa[code1], Sa[code2]};
  // intersectRectQuad (DARTCollide.cpp:513)
  double ret[16], buffer[16];
  int nq = 4, nrr = 0;
  double* q = quad;
  double* r = ret;
  for (int dir = 0; dir <= 1; dir++) {
    for (int sign = -1; sign <= 1; sign += 2) {
      double* pq = q;
      double* pr = r;
      nrr = 0;
      bool done = false;
      for (int i = nq; i > 0; i--) {
        if (sign * pq[dir] < rect[dir]) {
          pr[0] = pq[0]; pr[1] = pq[1]; pr += 2; nrr++;
          if (nrr & 8) { q = r; done = true; break; }
        }
        double* nextq = (i > 1) ? pq + 2 : q;
        if ((sign * pq[dir] < rect[dir]) ^ (sign * nextq[dir] < rect[dir])) {
          pr[1 - dir] = pq[1 - dir] + (nextq[1 - dir] - pq[1 - dir]) / (nextq[dir] - pq[dir]) * (sign * rect[dir] - pq[dir]);
          pr[dir] = sign * rect[dir];
          pr += 2; nrr++;
          if (nrr & 8) { q = r; done = true; break; }
        }
        pq += 2;
      }
      if (done) goto clipped;
      q = r;
      r = (q == ret) ? buffer : ret;
      nq = nrr;
    }
  }
clipped:
  if (q != ret) for (int i = 0; i < nrr * 2; i++) ret[i] = q[i];
  int nPts = nrr;
  if (nPts < 1) return 0;
  double point[24], dep[8];
  double det1 = 1.0 / (m11 * m22 - m12 * m21);
  m11 *= det1; m12 *= det1; m21 *= det1; m22 *= det1;
  int cnum = 0;
  for (int j = 0; j < nPts; j++) {
    double k1 = m22 * (ret[j * 2] - c1) - m12 * (ret[j * 2 + 1] - c2);
    double k2 = -m21 * (ret[j * 2] - c1) + m11 * (ret[j * 2 + 1] - c2);
    for (int i = 0; i < 3; i++) point[cnum * 3 + i] = center[i] + k1 * Rb[i * 3 + a1] + k2 * Rb[i * 3 + a2];
    dep[cnum] = Sa[codeN] - (normal2[0] * point[cnum * 3] + normal2[1] * point[cnum * 3 + 1] + normal2[2] * point[cnum * 3 + 2]);
    if (dep[cnum] >= 0) { ret[cnum * 2] = ret[j * 2]; ret[cnum * 2 + 1] = ret[j * 2 + 1]; cnum++; }
  }
  if (cnum < 1) return 0;
  for (int j = 0; j < cnum; j++) {
    Contact c{};
    c.shapeA = s1; c.shapeB = s2; c.bodyA = b1; c.bodyB = b2;
    for (int i = 0; i < 3; i++) { c.point[i] = point[j * 3 + i] + pa[i]; c.normal[i] = -normal[i]; }
    c.depth = dep[j];
    double xx = ret[j * 2], yy = ret[j * 2 + 1];
    bool onEdgeX = std::fabs(xx) == rect[0];
    bool onEdgeY = std::fabs(yy) == rect[1];
    if (onEdgeX && onEdgeY) {
      if (flip) { c.type = CT_FACE_VERTEX; for (int i = 0; i < 3; i++) c.point[i] += c.normal[i] * c.depth; }
      else { c.type = CT_VERTEX_FACE; for (int i = 0; i < 3; i++) c.point[i] -= c.normal[i] * c.depth; }
    } else if (!onEdgeX && !onEdgeY) {
      c.type = flip ? CT_VERTEX_FACE : CT_FACE_VERTEX;
    } else {
      // on an edge of the reference face but not at a corner
      // (DARTCollide.cpp:1318): edge A along the reference face edge through
      // its nearest corner, edge B along the nearest edge of the incident face
      c.type = CT_EDGE_EDGE;
      const double faceX = xx > 0 ? rect[0] : -rect[0], faceY = yy > 0 ? rect[1] : -rect[1];
      double eaF[3], eaD[3], ebF[3], ebD[3];
      for (int i = 0; i < 3; i++)
        eaF[i] = (pa[i] + Sa[codeN] * normal[i]) + faceX * Ra[i * 3 + code1] + faceY * Ra[i * 3 + code2];
      {
        double d[3], l = 0;
        for (int i = 0; i < 3; i++) { d[i] = c.point[i] - eaF[i]; l += d[i] * d[i]; }
        l = std::sqrt(l);
        for (int i = 0; i < 3; i++) eaD[i] = d[i] / l;
      }
      double other[3], o1[3], o2[3];
      for (int i = 0; i < 3; i++) { other[i] = Rb[i * 3 + lanr]; o1[i] = Rb[i * 3 + a1]; o2[i] = Rb[i * 3 + a2]; }
      if (other[0] * normal[0] + other[1] * normal[1] + other[2] * normal[2] < 0)
        for (int i = 0; i < 3; i++) other[i] = -other[i];
      double faceCenter[3];
      for (int i = 0; i < 3; i++) faceCenter[i] = pb[i] - Sb[lanr] * other[i];
      const double ifx = (o1[0] * c.point[0] + o1[1] * c.point[1] + o1[2] * c.point[2]) -
                         (o1[0] * pb[0] + o1[1] * pb[1] + o1[2] * pb[2]);
      const double ify = (o2[0] * c.point[0] + o2[1] * c.point[1] + o2[2] * c.point[2]) -
                         (o2[0] * pb[0] + o2[1] * pb[1] + o2[2] * pb[2]);
      const double sx = ifx == 0 ? 1.0 : ifx / std::fabs(ifx), sy = ify == 0 ? 1.0 : ify / std::fabs(ify);
      double nearB[3], otherB[3];
      for (int i = 0; i < 3; i++) nearB[i] = (sx * Sb[a1]) * o1[i] + (sy * Sb[a2]) * o2[i] + faceCenter[i];
      const double distX = std::fabs(std::fabs(ifx) - Sb[a1]), distY = std::fabs(std::fabs(ify) - Sb[a2]);
      if (distX < distY)
        for (int i = 0; i < 3; i++) otherB[i] = (sx * Sb[a1]) * o1[i] + (-1 * sy * Sb[a2]) * o2[i] + faceCenter[i];
      else
        for (int i = 0; i < 3; i++) otherB[i] = (-1 * sx * Sb[a1]) * o1[i] + (sy * Sb[a2]) * o2[i] + faceCenter[i];
      {
        double l = 0;
        for (int i = 0; i < 3; i++) { ebD[i] = nearB[i] - otherB[i]; l += ebD[i] * ebD[i]; }
        l = std::sqrt(l);
        for (int i = 0; i < 3; i++) { ebD[i] /= l; ebF[i] = nearB[i]; }
      }
      for (int i = 0; i < 3; i++) {
        c.edgeAFixed[i] = flip ? ebF[i] : eaF[i]; c.edgeADir[i] = flip ? ebD[i] : eaD[i];
        c.edgeBFixed[i] = flip ? eaF[i] : ebF[i]; c.edgeBDir[i] = flip ? eaD[i] : ebD[i];
      }
    }
    out.push_back(c);
  }
  return cnum;
}

}  // namespace oracle

// Raw box-box entry for known-answer fixtures (collideBoxBox signature:
// full sizes + world transforms [R|p] 3x4 row-major).  Output per contact:
// point3, normal3, depth, type.
extern "C" int oracle_box_box(const double* size1, const double* T1, const double* size2, const double* T2,
                              double* out) {
  double A[3] = {0.5 * size1[0], 0.5 * size1[1], 0.5 * size1[2]};
  double B[3] = {0.5 * size2[0], 0.5 * size2[1], 0.5 * size2[2]};
  double R1[9], R2[9], p1[3], p2[3];
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) { R1[r * 3 + c] = T1[r * 4 + c]; R2[r * 3 + c] = T2[r * 4 + c]; }
    p1[r] = T1[r * 4 + 3];
    p2[r] = T2[r * 4 + 3];
  }
  std::vector<oracle::Contact> cs;
  oracle::boxBox(p1, R1, A, p2, R2, B, 1e12, cs, 0, 1, 0, 1);
  // per contact: point3 normal3 depth type | edgeAFixed3 edgeADir3 edgeBFixed3 edgeBDir3
  for (size_t k = 0; k < cs.size(); k++) {
    double* o = out + 20 * k;
    for (int i = 0; i < 3; i++) { o[i] = cs[k].point[i]; o[3 + i] = cs[k].normal[i]; }
    o[6] = cs[k].depth;
    o[7] = cs[k].type;
    for (int i = 0; i < 3; i++) {
      o[8 + i] = cs[k].edgeAFixed[i]; o[11 + i] = cs[k].edgeADir[i];
      o[14 + i] = cs[k].edgeBFixed[i]; o[17 + i] = cs[k].edgeBDir[i];
    }
  }
  return (int)cs.size();
}

namespace oracle {

// collideSphereSphere (DARTCollide.cpp:1812): one SPHERE_SPHERE contact at
// the radius-weighted point between the centres, normal from centre 1 to 0
int sphereSphere(const double* c0, double r0, const double* c1, double r1, double clip, int shape1, int shape2,
                 int body1, int body2, std::vector<Contact>& out) {
  const double rsum = r0 + r1;
  double nrm[3];
  for (int i = 0; i < 3; i++) nrm[i] = c0[i] - c1[i];
  double nsq = nrm[0] * nrm[0] + nrm[1] * nrm[1] + nrm[2] * nrm[2];
  if (nsq > rsum * rsum) return 0;
  const double w0 = r0 / rsum, w1 = r1 / rsum;
  Contact c{};
  for (int i = 0; i < 3; i++) c.point[i] = w1 * c0[i] + w0 * c1[i];
  if (nsq < 1e-6) {  // DART_COLLISION_EPS: coincident centres, zero normal
    for (int i = 0; i < 3; i++) nrm[i] = 0.0;
    c.depth = rsum;
  } else {
    nsq = std::sqrt(nsq);
    for (int i = 0; i < 3; i++) nrm[i] *= 1.0 / nsq;
    c.depth = rsum - nsq;
  }
  if (c.depth > clip) return 0;
  c.type = CT_SPHERE_SPHERE;
  for (int i = 0; i < 3; i++) { c.normal[i] = nrm[i]; c.sphereCenter[i] = c0[i]; c.centerB[i] = c1[i]; }
  c.radiusA = w0 * rsum;
  c.radiusB = w1 * rsum;
  c.shapeA = shape1; c.shapeB = shape2; c.bodyA = body1; c.bodyB = body2;
  out.push_back(c);
  return 1;
}

// Sphere (centre c0, radius rs) against a capsule (radius rc, height h along
// the local z of Tc): dDistPointToSegment (DARTCollide.cpp:384) to the
// capsule's axis segment, SPHERE_SPHERE when the closest point is a segment
// end (alpha within 1e-8 of 0 or 1), else SPHERE_PIPE / PIPE_SPHERE.
int sphereCapsule(const double* c0, double rs, const Iso<double>& Tc, double rc, double h, bool sphereFirst,
                  double clip, int shape1, int shape2, int body1, int body2, std::vector<Contact>& out) {
  double ua[3], ub[3], v[3], wv[3];
  for (int i = 0; i < 3; i++) {
    ua[i] = Tc.R.m[3 * i + 2] * (-(h / 2)) + Tc.p[i];
    ub[i] = Tc.R.m[3 * i + 2] * (h / 2) + Tc.p[i];
  }
  for (int i = 0; i < 3; i++) { v[i] = ub[i] - ua[i]; wv[i] = c0[i] - ua[i]; }
  auto nrm3 = [](const double* a) { return std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]); };
  double alpha, dist, d[3];
  const double c1 = wv[0] * v[0] + wv[1] * v[1] + wv[2] * v[2];
  const double c2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
  if (c1 <= 0) {
    alpha = 0;
    for (int i = 0; i < 3; i++) d[i] = c0[i] - ua[i];
  } else if (c2 <= c1) {
    alpha = 1;
    for (int i = 0; i < 3; i++) d[i] = c0[i] - ub[i];
  } else {
    alpha = c1 / c2;
    for (int i = 0; i < 3; i++) d[i] = c0[i] - (ua[i] + alpha * v[i]);
  }
  dist = nrm3(d);
  const double r0 = sphereFirst ? rs : rc, r1 = sphereFirst ? rc : rs;  // object 1 / object 2
  if (!(dist < r0 + r1)) return 0;
  double cl[3];
  for (int i = 0; i < 3; i++) cl[i] = ua[i] + v[i] * alpha;
  const double rsum = r0 + r1, w0 = r0 / rsum, w1 = r1 / rsum;
  Contact c{};
  c.depth = rsum - dist;
  if (c.depth > clip) return 0;
  const double* p1 = sphereFirst ? c0 : cl;  // object 1's centre / closest point
  const double* p2 = sphereFirst ? cl : c0;
  double n[3];
  for (int i = 0; i < 3; i++) { c.point[i] = p1[i] * w1 + p2[i] * w0; n[i] = p1[i] - p2[i]; }
  const double nn = nrm3(n);
  for (int i = 0; i < 3; i++) c.normal[i] = nn > 0 ? n[i] / nn : n[i];  // Eigen normalized()
  c.radiusA = w0 * rsum;
  c.radiusB = w1 * rsum;
  if (std::fabs(alpha) < 1e-8 || std::fabs(1 - alpha) < 1e-8) {
    c.type = CT_SPHERE_SPHERE;
    for (int i = 0; i < 3; i++) { c.sphereCenter[i] = p1[i]; c.centerB[i] = p2[i]; }
  } else {
    c.type = sphereFirst ? CT_SPHERE_PIPE : CT_PIPE_SPHERE;
    c.sphereRadius = sphereFirst ? c.radiusA : c.radiusB;
    c.pipeRadius = sphereFirst ? c.radiusB : c.radiusA;
    const double vn = nrm3(v);
    for (int i = 0; i < 3; i++) {
      c.sphereCenter[i] = c0[i];
      c.pipeClosest[i] = cl[i];
      c.pipeFixed[i] = ua[i];
      c.pipeDir[i] = vn > 0 ? v[i] / vn : v[i];
    }
  }
  c.shapeA = shape1; c.shapeB = shape2; c.bodyA = body1; c.bodyB = body2;
  out.push_back(c);
  return 1;
}

// collideCapsuleCapsule (DARTCollide.cpp:4183): closest approach of the two
// axis segments; SPHERE_SPHERE / SPHERE_PIPE / PIPE_SPHERE when a closest
// point is a segment end (within 1e-8), else PIPE_PIPE
int capsuleCapsule(const Iso<double>& T0, double r0, double h0, const Iso<double>& T1, double r1, double h1,
                   double clip, int shape1, int shape2, int body1, int body2, std::vector<Contact>& out) {
  using std::sqrt;
  using std::fabs;
  double pa[3], pb[3], ua[3], ub[3];
  for (int i = 0; i < 3; i++) {
    pa[i] = T0.R.m[3 * i + 2] * (-(h0 / 2)) + T0.p[i];
    pb[i] = T0.R.m[3 * i + 2] * (h0 / 2) + T0.p[i];
    ua[i] = T1.R.m[3 * i + 2] * (-(h1 / 2)) + T1.p[i];
    ub[i] = T1.R.m[3 * i + 2] * (h1 / 2) + T1.p[i];
  }
  // dSegmentsClosestApproach (DARTCollide.cpp:301)
  double u[3], v[3], w[3];
  for (int i = 0; i < 3; i++) { u[i] = pb[i] - pa[i]; v[i] = ub[i] - ua[i]; w[i] = pa[i] - ua[i]; }
  const double a = u[0] * u[0] + u[1] * u[1] + u[2] * u[2], b = u[0] * v[0] + u[1] * v[1] + u[2] * v[2];
  const double c = v[0] * v[0] + v[1] * v[1] + v[2] * v[2], d = u[0] * w[0] + u[1] * w[1] + u[2] * w[2];
  const double e = v[0] * w[0] + v[1] * w[1] + v[2] * w[2];
  const double D = a * c - b * b;
  double sN, sD = D, tN, tD = D;
  if (D < 1e-15) {
    sN = 0.0; sD = 1.0; tN = e; tD = c;
  } else {
    sN = b * e - c * d;
    tN = a * e - b * d;
    if (sN < 0.0) { sN = 0.0; tN = e; tD = c; }
    else if (sN > sD) { sN = sD; tN = e + b; tD = c; }
  }
  if (tN < 0.0) {
    tN = 0.0;
    if (-d < 0.0) sN = 0.0;
    else if (-d > a) sN = sD;
    else { sN = -d; sD = a; }
  } else if (tN > tD) {
    tN = tD;
    if ((-d + b) < 0.0) sN = 0;
    else if ((-d + b) > a) sN = sD;
    else { sN = -d + b; sD = a; }
  }
  double alpha = fabs(sN) < 1e-15 ? 0.0 : sN / sD;
  double beta = fabs(tN) < 1e-15 ? 0.0 : tN / tD;
  if (alpha < 0) alpha = 0;
  if (alpha > 1) alpha = 1;
  if (beta < 0) beta = 0;
  if (beta > 1) beta = 1;
  double c0[3], c1[3], dd[3];
  for (int i = 0; i < 3; i++) { c0[i] = pa[i] + u[i] * alpha; c1[i] = ua[i] + v[i] * beta; dd[i] = c0[i] - c1[i]; }
  const double dist = sqrt(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2]);
  const double rsum = r0 + r1;
  if (!(dist <= rsum)) return 0;
  const double w0 = r0 / rsum, w1 = r1 / rsum;
  const double depth = rsum - dist;
  if (depth > clip) return 0;
  const bool s0 = fabs(alpha) < 1e-8 || fabs(1 - alpha) < 1e-8, s1 = fabs(beta) < 1e-8 || fabs(1 - beta) < 1e-8;
  const double un = sqrt(a), vn = sqrt(c);
  double point[3], nrm[3], dirA[3], dirB[3];
  for (int i = 0; i < 3; i++) {
    point[i] = c0[i] * w1 + c1[i] * w0;
    nrm[i] = dist > 0 ? dd[i] / dist : dd[i];
    dirA[i] = un > 0 ? u[i] / un : u[i];
    dirB[i] = vn > 0 ? v[i] / vn : v[i];
  }
  Contact ct{};
  ct.depth = depth;
  for (int i = 0; i < 3; i++) { ct.point[i] = point[i]; ct.normal[i] = nrm[i]; }
  ct.radiusA = w0 * rsum;
  ct.radiusB = w1 * rsum;
  if (s0 && s1) {
    ct.type = CT_SPHERE_SPHERE;
    for (int i = 0; i < 3; i++) { ct.sphereCenter[i] = c0[i]; ct.centerB[i] = c1[i]; }
  } else if (s0 || s1) {
    ct.type = s0 ? CT_SPHERE_PIPE : CT_PIPE_SPHERE;
    ct.sphereRadius = s0 ? w0 * rsum : w1 * rsum;
    ct.pipeRadius = s0 ? w1 * rsum : w0 * rsum;
    for (int i = 0; i < 3; i++) {
      ct.sphereCenter[i] = s0 ? c0[i] : c1[i];
      ct.pipeClosest[i] = s0 ? c1[i] : c0[i];
      ct.pipeFixed[i] = s0 ? ua[i] : pa[i];
      ct.pipeDir[i] = s0 ? dirB[i] : dirA[i];
    }
  } else {
    ct.type = CT_PIPE_PIPE;
    ct.radiusA = w0;
    ct.radiusB = w1;
    for (int i = 0; i < 3; i++) {
      ct.edgeAFixed[i] = pa[i]; ct.edgeAClosest[i] = c0[i]; ct.edgeADir[i] = dirA[i];
      ct.edgeBFixed[i] = ua[i]; ct.edgeBClosest[i] = c1[i]; ct.edgeBDir[i] = dirB[i];
    }
  }
  ct.shapeA = shape1; ct.shapeB = shape2; ct.bodyA = body1; ct.bodyB = body2;
  out.push_back(ct);
  return 1;
}

void collide(const World& w, const Kin<double>& k, std::vector<Contact>& out, int* unsupported) {
  out.clear();
  int unsup = 0;
  const int ns = (int)w.shapes.size();
  for (int i = 0; i + 1 < ns; i++) {
    for (int j = i + 1; j < ns; j++) {
      const Shape& S1 = w.shapes[i];
      const Shape& S2 = w.shapes[j];
      const Body& B1 = w.bodies[S1.body];
      const Body& B2 = w.bodies[S2.body];
      // BodyNodeCollisionFilter (CollisionFilter.cpp:105)
      if (S1.body == S2.body) continue;
      if (!B1.mobile && !B2.mobile) continue;
      if (B1.skel == B2.skel) continue;  // self-collision check disabled by default
      Iso<double> T1 = compose(k.Tw[S1.body], S1.T);
      Iso<double> T2 = compose(k.Tw[S2.body], S2.T);
      std::vector<Contact> pair;
      if (S1.type == NIMBLE_SHAPE_BOX && S2.type == NIMBLE_SHAPE_BOX) {
        double A[3] = {0.5 * S1.size[0], 0.5 * S1.size[1], 0.5 * S1.size[2]};
        double Bh[3] = {0.5 * S2.size[0], 0.5 * S2.size[1], 0.5 * S2.size[2]};
        boxBox(T1.p.x, T1.R.m, A, T2.p.x, T2.R.m, Bh, w.clipDepth, pair, i, j, S1.body, S2.body);
      } else if (S1.type == NIMBLE_SHAPE_BOX && S2.type == NIMBLE_SHAPE_CAPSULE) {
        // collideBoxCapsule (DARTCollide.cpp:4422); capsule size = (radius, height)
        capsuleBox(T1, S1.size, T2, S2.size[0], S2.size[1], true, w.clipDepth, i, j, S1.body, S2.body, pair, &unsup);
      } else if (S1.type == NIMBLE_SHAPE_CAPSULE && S2.type == NIMBLE_SHAPE_BOX) {
        // collideCapsuleBox (:4533)
        capsuleBox(T2, S2.size, T1, S1.size[0], S1.size[1], false, w.clipDepth, i, j, S1.body, S2.body, pair, &unsup);
      } else if (S1.type == NIMBLE_SHAPE_SPHERE && S2.type == NIMBLE_SHAPE_BOX) {
        sphereBoxPair(T2, S2.size, T1.p.x, S1.size[0], false, w.clipDepth, i, j, S1.body, S2.body, pair);
      } else if (S1.type == NIMBLE_SHAPE_BOX && S2.type == NIMBLE_SHAPE_SPHERE) {
        sphereBoxPair(T1, S1.size, T2.p.x, S2.size[0], true, w.clipDepth, i, j, S1.body, S2.body, pair);
      } else if (S1.type == NIMBLE_SHAPE_SPHERE && S2.type == NIMBLE_SHAPE_SPHERE) {
        sphereSphere(T1.p.x, S1.size[0], T2.p.x, S2.size[0], w.clipDepth, i, j, S1.body, S2.body, pair);
      } else if (S1.type == NIMBLE_SHAPE_SPHERE && S2.type == NIMBLE_SHAPE_CAPSULE) {
        sphereCapsule(T1.p.x, S1.size[0], T2, S2.size[0], S2.size[1], true, w.clipDepth, i, j, S1.body, S2.body, pair);
      } else if (S1.type == NIMBLE_SHAPE_CAPSULE && S2.type == NIMBLE_SHAPE_SPHERE) {
        sphereCapsule(T2.p.x, S2.size[0], T1, S1.size[0], S1.size[1], false, w.clipDepth, i, j, S1.body, S2.body,
                      pair);
      } else if (S1.type == NIMBLE_SHAPE_CAPSULE && S2.type == NIMBLE_SHAPE_CAPSULE) {
        capsuleCapsule(T1, S1.size[0], S1.size[1], T2, S2.size[0], S2.size[1], w.clipDepth, i, j, S1.body, S2.body,
                       pair);
      } else if (S1.type == NIMBLE_SHAPE_MESH && S2.type == NIMBLE_SHAPE_BOX) {
        meshBox(T1, S1, T2, S2.size, true, w.clipDepth, i, j, S1.body, S2.body, pair, &unsup);
      } else if (S1.type == NIMBLE_SHAPE_BOX && S2.type == NIMBLE_SHAPE_MESH) {
        meshBox(T2, S2, T1, S1.size, false, w.clipDepth, i, j, S1.body, S2.body, pair, &unsup);
      } else {
        std::fprintf(stderr, "oracle: shape pair (%d,%d) not supported\n", S1.type, S2.type);
        std::abort();
      }
      // postProcess (DARTCollisionDetector.cpp:357): drop repeated points
      for (const Contact& c : pair) {
        bool close = false;
        for (const Contact& t : out) {
          double dd = 0;
          for (int m = 0; m < 3; m++) dd += (c.point[m] - t.point[m]) * (c.point[m] - t.point[m]);
          if (std::sqrt(dd) < 3.0e-12) { close = true; break; }
        }
        if (!close) out.push_back(c);
      }
    }
  }
  if (unsupported) *unsupported = unsup;
}

//------------------------------------------------------------------------------
// Constraint rows.  One row = (contact, direction); generalized force column
// J^T e = sum over reactive bodies of +-S_w . [p x d; d] (world frame), the
// quantity DifferentiableContactConstraint::getConstraintForces (:231)
// computes and the impulse test of ContactConstraint::applyUnitImpulse
// (:525) realises.
struct Row {
  int contact, dir;  // dir 0 = normal, 1,2 = tangents
  double d[3];       // world direction for body A (body B gets -d)
};

static void tangentBasis(const double* n, double* t1, double* t2) {
  // ContactConstraint::getTangentBasisMatrixODE (:705), first dir = UnitZ
  auto cr = [](const double* a, const double* b, double* o) {
    o[0] = a[1] * b[2] - a[2] * b[1]; o[1] = a[2] * b[0] - a[0] * b[2]; o[2] = a[0] * b[1] - a[1] * b[0];
  };
  const double ez[3] = {0, 0, 1}, ex[3] = {1, 0, 0}, ey[3] = {0, 1, 0};
  double t[3];
  cr(ez, n, t);
  if (t[0] * t[0] + t[1] * t[1] + t[2] * t[2] < 1e-12) {
    cr(ex, n, t);
    if (t[0] * t[0] + t[1] * t[1] + t[2] * t[2] < 1e-12) {
      cr(ey, n, t);
      if (t[0] * t[0] + t[1] * t[1] + t[2] * t[2] < 1e-12) cr(ez, n, t);
    }
  }
  double l = std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
  for (int i = 0; i < 3; i++) t1[i] = t[i] / l;
  cr(n, t1, t2);
}

static bool reactive(const World& w, int b) {
  if (!w.bodies[b].mobile) return false;
  for (int a = b; a >= 0; a = w.bodies[a].parent)
    if (w.bodies[a].ndof > 0) return true;
  return false;
}

static void rowForce(const World& w, const Kin<double>& k, const Contact& c, const double* d, double* col) {
  const int n = w.n;
  for (int i = 0; i < n; i++) col[i] = 0.0;
  for (int side = 0; side < 2; side++) {
    const int body = side == 0 ? c.bodyA : c.bodyB;
    if (!reactive(w, body)) continue;
    const double sgn = side == 0 ? 1.0 : -1.0;
    double wr[6];
    wr[0] = c.point[1] * d[2] - c.point[2] * d[1];
    wr[1] = c.point[2] * d[0] - c.point[0] * d[2];
    wr[2] = c.point[0] * d[1] - c.point[1] * d[0];
    wr[3] = d[0]; wr[4] = d[1]; wr[5] = d[2];
    for (int dof = 0; dof < n; dof++) {
      const int b = w.dofBody[dof];
      if (!w.isAncestorOrSelf(b, body)) continue;
      const Body& B = w.bodies[b];
      const int kk = dof - B.dof0;
      // world screw axis = Ad_{Tw_b} S_local
      V6<double> sl;
      for (int i = 0; i < 6; i++) sl[i] = k.Sj[b](i, kk);
      V6<double> sw = AdT(k.Tw[b], sl);
      double s = 0;
      for (int i = 0; i < 6; i++) s += sw[i] * wr[i];
      col[dof] += sgn * s;
    }
  }
}

//------------------------------------------------------------------------------
// LCPUtils::isLCPSolutionValid (LCPUtils.cpp:14)
bool lcpValid(const std::vector<double>& A, const std::vector<double>& x, const std::vector<double>& b,
                     const std::vector<double>& hi, const std::vector<double>& lo, const std::vector<int>& fi,
                     bool ignoreFriction) {
  const int m = (int)x.size();
  for (int i = 0; i < m; i++) {
    double v = -b[i];
    for (int j = 0; j < m; j++) v += A[i * m + j] * x[j];
    double up = hi[i], low = lo[i];
    if (fi[i] != -1) {
      if (ignoreFriction) { if (x[i] != 0) return false; continue; }
      up *= x[fi[i]];
      low *= x[fi[i]];
    }
    const double tol = 1e-5;
    if (std::fabs(low) < tol && std::fabs(up) < tol && std::fabs(x[i]) < tol) {
    } else if (std::fabs(x[i] - low) < tol) {
      if (v < -tol) return false;
    } else if (std::fabs(x[i] - up) < tol) {
      if (v > tol) return false;
    } else if (x[i] > low && x[i] < up) {
      if (std::fabs(v) > tol) return false;
    } else {
      return false;
    }
  }
  return true;
}

// LCPUtils::guessSolution (LCPUtils.cpp:69)
std::vector<double> guessSolution(const std::vector<double>& A, const std::vector<double>& b,
                                         const std::vector<int>& fi) {
  const int m = (int)b.size();
  std::vector<int> cl;
  for (int i = 0; i < m; i++) {
    if (fi[i] == -1) { if (b[i] > 0) cl.push_back(i); }
    else cl.push_back(i);
  }
  std::vector<double> x(m, 0.0);
  const int k = (int)cl.size();
  if (k == 0) return x;
  std::vector<double> Ar(k * k), br(k), xr(k);
  for (int r = 0; r < k; r++) {
    br[r] = b[cl[r]];
    for (int c = 0; c < k; c++) Ar[r * k + c] = A[cl[r] * m + cl[c]];
  }
  codSolve(Ar.data(), k, k, br.data(), xr.data());
  for (int i = 0; i < k; i++) x[cl[i]] = xr[i];
  return x;
}

// LCPUtils::reduce (LCPUtils.cpp:144) with mergeLCPColumns (:346): while
// some column pair (a < b, first in (a, b) order) of the current problem has
// ||A_a - A_b||^2 < 1e-4, |b_a - b_b| < 1e-4 and equal findex / hi / lo,
// merge b into a: row and column b are deleted, column a is doubled, findex
// entries pointing at b point at a, later indices shift down.  The problem is
// reduced in place (A row-major, the new size on return); the returned map
// sends each original row to its reduced row, i.e. mapOut * x_reduced is
// x_full[i] = x_reduced[map[i]] (mapOut's columns are sums of unit columns).
struct LcpCascade {
  bool reduced = false, ignoredFriction = false;
  double cfm = 0.0;
  int path = 0;  // 0 Dantzig, 1 PGS (CFM), 2 frictionless PGS
};

std::vector<int> lcpReduce(std::vector<double>& A, std::vector<double>& X, std::vector<double>& b,
                           std::vector<double>& hi, std::vector<double>& lo, std::vector<int>& fi) {
  const int m0 = (int)b.size();
  std::vector<int> map(m0);
  for (int i = 0; i < m0; i++) map[i] = i;
  for (;;) {
    const int n = (int)b.size();
    int ca = -1, cb = -1;
    for (int a = 0; a < n - 1 && ca < 0; a++)
      for (int c = a + 1; c < n; c++) {
        double dd = 0;
        for (int i = 0; i < n; i++) dd += (A[i * n + a] - A[i * n + c]) * (A[i * n + a] - A[i * n + c]);
        if (dd < 1e-4 && std::fabs(b[a] - b[c]) < 1e-4 && fi[a] == fi[c] && hi[a] == hi[c] && lo[a] == lo[c]) {
          ca = a; cb = c;
          break;
        }
      }
    if (ca < 0) break;
    // mergeLCPColumns(ca, cb)
    std::vector<double> nA((n - 1) * (n - 1));
    for (int i = 0, ni = 0; i < n; i++) {
      if (i == cb) continue;
      for (int j = 0, nj = 0; j < n; j++) {
        if (j == cb) continue;
        nA[ni * (n - 1) + nj] = j == ca ? A[i * n + j] * 2.0 : A[i * n + j];
        nj++;
      }
      ni++;
    }
    auto drop = [&](auto& v) { v.erase(v.begin() + cb); };
    drop(X); drop(b); drop(hi); drop(lo); drop(fi);
    for (int& f : fi) f = f == cb ? ca : (f > cb ? f - 1 : f);
    for (int& r : map) r = r == cb ? ca : (r > cb ? r - 1 : r);
    A.swap(nA);
  }
  return map;
}

// BoxedLcpConstraintSolver::solveLcp's fallbacks once the gradient
// short-circuit failed (BoxedLcpConstraintSolver.cpp:459-687): Dantzig with
// early termination on the reduced problem (LCPUtils::reduce), validity on
// the full one; else CFM on the diagonal and PGS on the reduced A + cfm I from
// the warm start, validity; else LCPUtils::removeFriction and PGS on the
// normal rows from zero.  NaNs zero the solution.  X: the solution (in: the
// warm start, which is also mXBackup).
LcpCascade lcpFallbackCascade(const std::vector<double>& A, const std::vector<double>& b,
                              const std::vector<double>& lo, const std::vector<double>& hi,
                              const std::vector<int>& fi, const std::vector<double>& warm, double fallbackCfm,
                              std::vector<double>& X) {
  const int m = (int)b.size();
  LcpCascade res;
  X = warm;
  bool success = false;
  {
    std::vector<double> Ad = A, xr = X, bd = b, lod = lo, hid = hi;
    std::vector<int> fid = fi;
    const std::vector<int> map = lcpReduce(Ad, xr, bd, hid, lod, fid);
    const int mr = (int)bd.size();
    if (mr < m) res.reduced = true;
    // the reduced A is not symmetric (merged columns are doubled); ODE's dLCP
    // only ever reads the lower triangle of the row-major matrix it is given
    // (swapRowsAndCols, lcp.cpp:144; GETA, matrix.cpp:371) -- checked against
    // the reference's compiled solver in tests/test_lcp_utils.py -- so the
    // restatement gets that triangle mirrored
    for (int r = 0; r < mr; r++)
      for (int c = r + 1; c < mr; c++) Ad[r * mr + c] = Ad[c * mr + r];
    std::vector<double> xd(mr, 0.0);
    success = dantzigSolveLCP(mr, Ad.data(), xd.data(), bd.data(), nullptr, 0, lod.data(), hid.data(), fid.data(), true);
    if (success) {
      for (int i = 0; i < m; i++) X[i] = xd[map[i]];
      if (!lcpValid(A, X, b, hi, lo, fi, false)) success = false;
    }
  }
  for (double xv : X) if (std::isnan(xv)) { success = false; std::fill(X.begin(), X.end(), 0.0); break; }
  if (success) return res;
  res.path = 1;
  res.cfm = fallbackCfm;
  std::vector<double> Acfm = A;
  for (int i = 0; i < m; i++) Acfm[i * m + i] += fallbackCfm;
  {
    std::vector<double> Ad = Acfm, xd = warm, bd = b, lod = lo, hid = hi;
    std::vector<int> fid = fi;
    const std::vector<int> map = lcpReduce(Ad, xd, bd, hid, lod, fid);
    const int mr = (int)bd.size();
    if (mr < m) res.reduced = true;
    success = pgsSolveLCP(mr, Ad.data(), xd.data(), bd.data(), lod.data(), hid.data(), fid.data());
    if (success) {
      for (int i = 0; i < m; i++) X[i] = xd[map[i]];
      if (!lcpValid(Acfm, X, b, hi, lo, fi, false)) success = false;
    }
  }
  if (!success) {
    res.path = 2;
    res.ignoredFriction = true;
    std::vector<int> keep;
    for (int i = 0; i < m; i++) if (fi[i] == -1) keep.push_back(i);
    const int k2 = (int)keep.size();
    std::vector<double> Ar(k2 * k2), br(k2), xr(k2, 0.0), lor(k2), hir(k2);
    std::vector<int> fir(k2, -1);
    for (int r = 0; r < k2; r++) {
      br[r] = b[keep[r]]; lor[r] = lo[keep[r]]; hir[r] = hi[keep[r]];
      for (int c = 0; c < k2; c++) Ar[r * k2 + c] = Acfm[keep[r] * m + keep[c]];
    }
    pgsSolveLCP(k2, Ar.data(), xr.data(), br.data(), lor.data(), hir.data(), fir.data());
    std::fill(X.begin(), X.end(), 0.0);
    for (int r = 0; r < k2; r++) X[keep[r]] = xr[r];
  }
  for (double xv : X) if (std::isnan(xv)) { std::fill(X.begin(), X.end(), 0.0); break; }
  return res;
}

// ---- ConstrainedGroupGradientMatrices (the per-step "gradient matrices") ----
struct GradMats {
  const World* w;
  int m = 0;  // constraint dim
  std::vector<double> X, hi, lo, B, aColNorms, A;
  std::vector<int> fi;
  double cfm = 0;
  bool ignoreFriction = false;
  // Q from A's entries (A_cc + A_cu E: the same matrix as A_c^T Minv A_cubE,
  // the device's form) instead of J and Minv: the classification probe of
  // oracle_classify, which has A only
  bool qFromA = false;
  const std::vector<double>* allCols;      // n x m   (col j = J^T e_j)
  const std::vector<double>* massedCols;   // n x m   (col j = Minv J^T e_j)
  const std::vector<double>* Minv;         // n x n
  std::vector<double> restitution;         // per row (0 without bounce)
  std::vector<double> penVel;
  // outputs
  std::vector<int> mapping, clampIdx, ubIdx;
  int nc = 0, nu = 0;
  std::vector<double> fc, relVel, E, clampA;
  bool standardized = false;

  void construct() {
    const int n = w ? w->n : 0;
    mapping.assign(m, CM_NOT_CLAMPING);
    clampIdx.assign(m, -1);
    ubIdx.assign(m, -1);
    nc = nu = 0;
    const double TH = 1e-6;
    for (int j = 0; j < m; j++) {
      if (aColNorms[j] < 1e-9) { mapping[j] = CM_NOT_CLAMPING; continue; }
      const double f = X[j];
      double up = hi[j], low = lo[j];
      const int fp = fi[j];
      if (fp != -1) { up *= X[fp]; low *= X[fp]; }
      if (std::fabs(f) < TH) {
        if (fp != -1) {
          if (std::fabs(X[fp]) < TH) mapping[j] = CM_NOT_CLAMPING;
          else if (ignoreFriction) mapping[j] = CM_NOT_CLAMPING;
          else { mapping[j] = CM_CLAMPING; clampIdx[j] = nc++; }
        } else {
          mapping[j] = CM_NOT_CLAMPING;
        }
        continue;
      }
      const double tie = 1e-5;
      if ((f > low + tie && f < up - tie) || (low - f > 1e-2 || f - up > 1e-2)) {
        mapping[j] = CM_CLAMPING; clampIdx[j] = nc++;
      } else if (fp != -1 && std::fabs(X[fp]) > 1e-9 && aColNorms[fp] > 1e-9 &&
                 (fp > j || mapping[fp] == CM_CLAMPING)) {
        mapping[j] = fp; ubIdx[j] = nu++;
      } else {
        mapping[j] = CM_NOT_CLAMPING;
      }
    }
    fc.assign(nc, 0.0);
    relVel.assign(nc, 0.0);
    E.assign(nu * nc, 0.0);
    clampA.assign(nc * nc, 0.0);
    for (int j = 0; j < m; j++) {
      if (mapping[j] == CM_CLAMPING) { fc[clampIdx[j]] = X[j]; relVel[clampIdx[j]] = B[j]; }
    }
    for (int j = 0; j < m; j++) {
      if (mapping[j] >= 0) {
        const int fp = mapping[j];
        const double up = X[fp] * hi[j], low = X[fp] * lo[j];
        E[ubIdx[j] * nc + clampIdx[fp]] = std::fabs(X[j] - up) < std::fabs(X[j] - low) ? hi[j] : lo[j];
      }
    }
    for (int r = 0; r < m; r++)
      if (mapping[r] == CM_CLAMPING)
        for (int c = 0; c < m; c++)
          if (mapping[c] == CM_CLAMPING) clampA[clampIdx[r] * nc + clampIdx[c]] = A[r * m + c];
    (void)n;
    standardize();
  }
  // opportunisticallyStandardizeResults (ConstrainedGroupGradientMatrices.cpp:218)
  bool standardize() {
    standardized = true;
    if (m == 0) return true;
    const int n = w ? w->n : 0;
    if (nc == 0) {
      std::vector<double> zero(m, 0.0);
      if (lcpValid(A, zero, B, hi, lo, fi, ignoreFriction)) { X = zero; return true; }
      standardized = false;
      return false;
    }
    std::vector<double> Q(nc * nc, 0.0);
    if (nu == 0) {
      Q = clampA;
    } else if (qFromA) {
      for (int r = 0; r < m; r++) {
        if (mapping[r] != CM_CLAMPING) continue;
        for (int c = 0; c < m; c++) {
          if (mapping[c] != CM_CLAMPING) continue;
          double v = A[r * m + c];
          for (int u = 0; u < m; u++)
            if (mapping[u] == c) v += E[ubIdx[u] * nc + clampIdx[c]] * A[r * m + u];
          Q[clampIdx[r] * nc + clampIdx[c]] = v;
        }
      }
      for (int c = 0; c < nc; c++) Q[c * nc + c] += cfm;
    } else {
      // Q = A_c^T Minv (A_c + A_ub E) + cfm I
      std::vector<double> AcubE(n * nc, 0.0);
      for (int j = 0; j < m; j++) {
        if (mapping[j] == CM_CLAMPING)
          for (int i = 0; i < n; i++) AcubE[i * nc + clampIdx[j]] += (*allCols)[i * m + j];
      }
      for (int j = 0; j < m; j++)
        if (mapping[j] >= 0)
          for (int c = 0; c < nc; c++) {
            const double e = E[ubIdx[j] * nc + c];
            if (e != 0) for (int i = 0; i < n; i++) AcubE[i * nc + c] += (*allCols)[i * m + j] * e;
          }
      std::vector<double> MA(n * nc, 0.0);
      for (int i = 0; i < n; i++)
        for (int c = 0; c < nc; c++) {
          double s = 0;
          for (int t = 0; t < n; t++) s += (*Minv)[i * n + t] * AcubE[t * nc + c];
          MA[i * nc + c] = s;
        }
      for (int j = 0; j < m; j++)
        if (mapping[j] == CM_CLAMPING)
          for (int c = 0; c < nc; c++) {
            double s = 0;
            for (int i = 0; i < n; i++) s += (*allCols)[i * m + j] * MA[i * nc + c];
            Q[clampIdx[j] * nc + c] = s;
          }
      for (int c = 0; c < nc; c++) Q[c * nc + c] += cfm;
    }
    std::vector<double> f(nc);
    codSolve(Q.data(), nc, nc, relVel.data(), f.data());
    const std::vector<double> orig = fc;
    bool anyNewlyNot = false;
    std::vector<double> nx(m, 0.0);
    for (int i = 0; i < m; i++) {
      if (clampIdx[i] != -1) {
        nx[i] = f[clampIdx[i]];
        if (std::fabs(f[clampIdx[i]]) < 1e-6 && std::fabs(X[i]) > 1e-6 && fi[i] == -1) anyNewlyNot = true;
      }
      if (ubIdx[i] != -1) {
        const int fp = fi[i];
        const double om = orig[clampIdx[fp]] / X[i];
        const double clean = std::fabs(om - hi[i]) < std::fabs(om - lo[i]) ? hi[i] : lo[i];
        nx[i] = f[clampIdx[fp]] * clean;
      }
    }
    if (lcpValid(A, nx, B, hi, lo, fi, ignoreFriction)) {
      X = nx;
      fc = f;
      if (anyNewlyNot) construct();
      return true;
    }
    standardized = false;
    return false;
  }
};

//------------------------------------------------------------------------------
thread_local ForcedLcp* tForcedLcp = nullptr;

void solveContacts(const World& w, const Kin<double>& k, const double* q, const double* v, const double* tau,
                   std::vector<double>& v1, const std::vector<Contact>& contactsIn,
                   std::vector<double>& lcpCache, Snapshot& snap) {
  (void)q; (void)v; (void)tau;
  const int n = w.n;
  snap.numRows = 0;
  snap.numClamping = 0;
  snap.numUpperBound = 0;
  snap.contacts.clear();
  snap.shortCircuit = false;
  snap.ignoredFriction = false;
  snap.lcpReduced = false;
  snap.cfm = 0.0;
  // ConstraintSolver::updateConstraints (ConstraintSolver.cpp:520)
  std::vector<Contact> contacts;
  for (const Contact& c : contactsIn) {
    if (c.normal[0] * c.normal[0] + c.normal[1] * c.normal[1] + c.normal[2] * c.normal[2] < 1e-12) continue;
    if (c.depth < 0.0) continue;
    if (c.depth > w.clipDepth) continue;
    if (!reactive(w, c.bodyA) && !reactive(w, c.bodyB)) continue;  // ContactConstraint::update
    contacts.push_back(c);
  }
  snap.contacts = contacts;
  if (contacts.empty()) return;
  if ((int)contacts.size() > NIMBLE_MAX_CONTACTS) {
    std::fprintf(stderr, "oracle: %zu contacts exceed NIMBLE_MAX_CONTACTS\n", contacts.size());
    std::abort();
  }
  // rows (ContactConstraint: 3 rows with friction, else 1)
  std::vector<Row> rows;
  std::vector<double> lo, hi, bounce, rest, pen;
  std::vector<int> fi;
  for (int ci = 0; ci < (int)contacts.size(); ci++) {
    const Contact& c = contacts[ci];
    const double mu = std::min(w.bodies[c.bodyA].friction, w.bodies[c.bodyB].friction);
    const double restC = w.bodies[c.bodyA].restitution * w.bodies[c.bodyB].restitution;
    const bool frictionOn = mu > 1e-3;
    const int base = (int)rows.size();
    Row r0{ci, 0, {c.normal[0], c.normal[1], c.normal[2]}};
    rows.push_back(r0);
    lo.push_back(0.0); hi.push_back(kInf); fi.push_back(-1);
    if (frictionOn) {
      double t1[3], t2[3];
      tangentBasis(c.normal, t1, t2);
      rows.push_back(Row{ci, 1, {t1[0], t1[1], t1[2]}});
      rows.push_back(Row{ci, 2, {t2[0], t2[1], t2[2]}});
      lo.push_back(-mu); hi.push_back(mu); fi.push_back(base);
      lo.push_back(-mu); hi.push_back(mu); fi.push_back(base);
    }
    // restitution is only "on" above DART_RESTITUTION_COEFF_THRESHOLD
    rest.push_back(restC > 1e-3 ? restC : 0.0);
    if (frictionOn) { rest.push_back(0); rest.push_back(0); }
  }
  const int m = (int)rows.size();
  snap.numRows = m;
  std::vector<double> allCols(n * m), massed(n * m);
  // Minv via the mass matrix
  std::vector<double> M(n * n), Minv(n * n);
  w.massMatrix(k, M.data());
  invertSmall(M.data(), Minv.data(), n);
  for (int j = 0; j < m; j++) {
    const Contact& c = contacts[rows[j].contact];
    std::vector<double> col(n);
    rowForce(w, k, c, rows[j].d, col.data());
    for (int i = 0; i < n; i++) allCols[i * m + j] = col[i];
  }
  for (int i = 0; i < n; i++)
    for (int j = 0; j < m; j++) {
      double s = 0;
      for (int t = 0; t < n; t++) s += Minv[i * n + t] * allCols[t * m + j];
      massed[i * m + j] = s;
    }
  // A = J Minv J^T ; b = -J v1 (+ bouncing / penetration correction)
  std::vector<double> A(m * m), b(m);
  for (int r = 0; r < m; r++)
    for (int c = 0; c < m; c++) {
      double s = 0;
      for (int i = 0; i < n; i++) s += allCols[i * m + r] * massed[i * m + c];
      A[r * m + c] = s;
    }
  for (int r = 0; r < m; r++)
    for (int c = r + 1; c < m; c++) A[c * m + r] = A[r * m + c];  // upper triangle copied down
  pen.assign(m, 0.0);
  for (int r = 0; r < m; r++) {
    double s = 0;
    for (int i = 0; i < n; i++) s += allCols[i * m + r] * v1[i];
    b[r] = -s;
  }
  for (int r = 0; r < m; r++) {
    if (rows[r].dir != 0) continue;
    const Contact& c = contacts[rows[r].contact];
    double bv = c.depth - 0.0;  // mErrorAllowance = 0
    if (bv < 0.0) bv = 0.0;
    else { bv *= 0.01 / w.dt; if (bv > 1e-3) bv = 1e-3; }
    if (!w.penetrationCorrection) bv = 0;
    pen[r] = bv;
    if (rest[r] > 0) {
      const double rv = b[r] * rest[r];
      if (rv > 1e-1 && rv > bv) { bv = rv > 1e2 ? 1e2 : rv; pen[r] = 0.0; }
      else rest[r] = 0.0;  // getCoefficientOfRestitution returns 0 unless bounced
    }
    b[r] += bv;
  }
  std::vector<double> aColNorms(m);
  for (int j = 0; j < m; j++) {
    double s = 0;
    for (int i = 0; i < m; i++) s += A[i * m + j] * A[i * m + j];
    aColNorms[j] = s;
  }
  // cached LCP solution (BoxedLcpConstraintSolver::mX)
  std::vector<double> X;
  if ((int)lcpCache.size() != m) X = guessSolution(A, b, fi);
  else X = lcpCache;

  GradMats gm;
  gm.w = &w; gm.m = m; gm.hi = hi; gm.lo = lo; gm.fi = fi; gm.B = b; gm.aColNorms = aColNorms; gm.A = A;
  gm.allCols = &allCols; gm.massedCols = &massed; gm.Minv = &Minv; gm.restitution = rest; gm.penVel = pen;
  ForcedLcp* forced = tForcedLcp;
  if (forced != nullptr && forced->m != m) { forced->mismatch = true; forced = nullptr; }
  bool success, shortCircuit;
  if (forced != nullptr) {
    // replay: the given path's final solution in place of the solve
    X.assign(forced->x, forced->x + m);
    success = shortCircuit = forced->shortCircuit;
    if (shortCircuit) {
      gm.X = X; gm.cfm = 0.0; gm.ignoreFriction = false;
      gm.construct();
      if (gm.standardized) X = gm.X;
    }
  } else {
    gm.X = X; gm.cfm = 0.0; gm.ignoreFriction = false;
    gm.construct();
    success = gm.standardized;
    shortCircuit = success;
    if (success) X = gm.X;
  }
  std::vector<double> Acfm = A;
  double cfm = 0.0;
  bool ignoredFriction = false;
  if (!success && forced != nullptr) {
    cfm = forced->cfm;
    ignoredFriction = forced->ignoredFriction;
    if (cfm != 0.0)
      for (int i = 0; i < m; i++) Acfm[i * m + i] += cfm;
  } else if (!success) {
    const std::vector<double> warm = X;  // mX == mXBackup (cache or guess)
    const LcpCascade r = lcpFallbackCascade(A, b, lo, hi, fi, warm, w.fallbackCfm, X);
    cfm = r.cfm;
    ignoredFriction = r.ignoredFriction;
    snap.lcpReduced = r.reduced;
    if (cfm != 0.0)
      for (int i = 0; i < m; i++) Acfm[i * m + i] += cfm;
  }
  if (!shortCircuit) {
    gm.X = X; gm.A = Acfm; gm.cfm = cfm; gm.ignoreFriction = ignoredFriction;
    gm.construct();
    if (gm.standardized) X = gm.X;
  }
  lcpCache = X;
  // applyConstraintImpulses + computeImpulseForwardDynamics: v1 += Minv J^T x
  for (int i = 0; i < n; i++) {
    double s = 0;
    for (int j = 0; j < m; j++) s += massed[i * m + j] * X[j];
    v1[i] += s;
  }
  // snapshot for the backward pass
  snap.Aall = allCols;
  snap.rowContact.clear(); snap.rowDirIdx.clear(); snap.rowDir.clear();
  for (const Row& r : rows) {
    snap.rowContact.push_back(r.contact); snap.rowDirIdx.push_back(r.dir);
    for (int i = 0; i < 3; i++) snap.rowDir.push_back(r.d[i]);
  }
  snap.massedImpulse = massed;
  snap.lcpA = gm.A; snap.lcpB = b; snap.lcpLo = lo; snap.lcpHi = hi; snap.lcpX = gm.X; snap.lcpFIndex = fi;
  snap.aColNorms = aColNorms;
  snap.mapping = gm.mapping; snap.clampingIndex = gm.clampIdx; snap.upperBoundIndex = gm.ubIdx;
  snap.numClamping = gm.nc; snap.numUpperBound = gm.nu;
  snap.fc = gm.fc;
  snap.E = gm.E;
  snap.cfm = gm.cfm;
  snap.ignoredFriction = gm.ignoreFriction;
  snap.shortCircuit = shortCircuit;
  snap.bounceDiag.assign(gm.nc, 1.0);
  snap.penetrationVel.assign(gm.nc, 0.0);
  for (int j = 0; j < m; j++)
    if (gm.mapping[j] == CM_CLAMPING) {
      snap.bounceDiag[gm.clampIdx[j]] = 1.0 + rest[j];
      snap.penetrationVel[gm.clampIdx[j]] = pen[j];
    }
}

//------------------------------------------------------------------------------
// The gradient short-circuit's classification + standardisation alone
// (ConstrainedGroupGradientMatrices::constructMatrices :482, :218) on a raw
// problem with warm start X, Q from A's entries: test infrastructure, the
// probe of whether a world's short-circuit outcome flips under 1e-15
// perturbations of A.  Returns standardized; X receives the standardised x.
bool classifyLcp(int m, const double* A, const double* b, const double* lo, const double* hi, const int* fi,
                 double* X) {
  GradMats gm;
  gm.w = nullptr;
  gm.m = m;
  gm.A.assign(A, A + m * m);
  gm.B.assign(b, b + m);
  gm.lo.assign(lo, lo + m);
  gm.hi.assign(hi, hi + m);
  gm.fi.assign(fi, fi + m);
  gm.X.assign(X, X + m);
  gm.aColNorms.assign(m, 0.0);
  for (int j = 0; j < m; j++) {
    double s = 0;
    for (int i = 0; i < m; i++) s += A[i * m + j] * A[i * m + j];
    gm.aColNorms[j] = s;
  }
  gm.qFromA = true;
  gm.construct();
  for (int j = 0; j < m; j++) X[j] = gm.X[j];
  return gm.standardized;
}

// The LCP part of solveContacts above on a raw problem (tests: the ambiguity
// probe of path splits that are neither at the short-circuit nor at
// Dantzig's outcome): the short-circuit classification from the warm start,
// else BoxedLcpConstraintSolver's fallback cascade from it, then the final
// classification, with Q from A's entries.  flags = [shortCircuit,
// ignoredFriction, cfm, numClamping, numUpperBound, lcpReduced]; mapping gets
// the final per-row classification.
void lcpPathFromA(int m, const double* A, const double* b, const double* lo, const double* hi, const int* fi,
                  const double* warm, double fallbackCfm, double* flags, int* mapping) {
  GradMats gm;
  gm.w = nullptr;
  gm.m = m;
  gm.A.assign(A, A + m * m);
  gm.B.assign(b, b + m);
  gm.lo.assign(lo, lo + m);
  gm.hi.assign(hi, hi + m);
  gm.fi.assign(fi, fi + m);
  gm.aColNorms.assign(m, 0.0);
  for (int j = 0; j < m; j++) {
    double s = 0;
    for (int i = 0; i < m; i++) s += A[i * m + j] * A[i * m + j];
    gm.aColNorms[j] = s;
  }
  gm.qFromA = true;
  std::vector<double> X(warm, warm + m);
  gm.X = X; gm.cfm = 0.0; gm.ignoreFriction = false;
  gm.construct();
  const bool shortCircuit = gm.standardized;
  bool reduced = false;
  if (!shortCircuit) {
    const std::vector<double> w0 = X;  // mX == mXBackup
    const LcpCascade r = lcpFallbackCascade(gm.A, gm.B, gm.lo, gm.hi, gm.fi, w0, fallbackCfm, X);
    reduced = r.reduced;
    std::vector<double> Acfm(A, A + m * m);
    if (r.cfm != 0.0)
      for (int i = 0; i < m; i++) Acfm[i * m + i] += r.cfm;
    gm.X = X; gm.A = Acfm; gm.cfm = r.cfm; gm.ignoreFriction = r.ignoredFriction;
    gm.construct();
  }
  flags[0] = shortCircuit ? 1 : 0;
  flags[1] = gm.ignoreFriction ? 1 : 0;
  flags[2] = gm.cfm;
  flags[3] = gm.nc;
  flags[4] = gm.nu;
  flags[5] = reduced ? 1 : 0;
  for (int j = 0; j < m; j++) mapping[j] = gm.mapping[j];
}

void buildClampingMatrices(const World& w, const Snapshot& snap, std::vector<double>& Ac, std::vector<double>& Aub,
                           std::vector<double>& AcubE) {
  const int n = w.n, m = snap.numRows, nc = snap.numClamping, nu = snap.numUpperBound;
  Ac.assign(n * nc, 0.0);
  Aub.assign(n * nu, 0.0);
  AcubE.assign(n * nc, 0.0);
  for (int j = 0; j < m; j++) {
    if (snap.mapping[j] == CM_CLAMPING)
      for (int i = 0; i < n; i++) Ac[i * nc + snap.clampingIndex[j]] = snap.Aall[i * m + j];
    else if (snap.mapping[j] >= 0)
      for (int i = 0; i < n; i++) Aub[i * nu + snap.upperBoundIndex[j]] = snap.Aall[i * m + j];
  }
  for (int i = 0; i < n; i++)
    for (int c = 0; c < nc; c++) {
      double s = Ac[i * nc + c];
      for (int u = 0; u < nu; u++) s += Aub[i * nu + u] * snap.E[u * nc + c];
      AcubE[i * nc + c] = s;
    }
}

// Position-dependent constraint terms (dA_c f_c, dF_c wrt position) --
// oracle_contact_grad.cpp.
void positionConstraintTerms(const World& w, const Snapshot& snap, const std::vector<double>& Minv,
                             const std::vector<double>& C, const std::vector<double>& dCq,
                             const std::vector<double>& Ac, const std::vector<double>& Aub,
                             const std::vector<double>& AcubE, const std::vector<double>& Qpinv,
                             std::vector<double>& dFcPos, std::vector<double>& dAcf);

void constrainedJacobians(const World& w, const Kin<double>& k, const Snapshot& snap, const std::vector<double>& M,
                          const std::vector<double>& Minv, const std::vector<double>& C,
                          const std::vector<double>& dCq, const std::vector<double>& dCv,
                          const std::vector<double>& dM, const std::vector<double>& Ac,
                          const std::vector<double>& Aub, const std::vector<double>& AcubE,
                          std::vector<double>& posVel, std::vector<double>& velVel, std::vector<double>& forceVel,
                          std::vector<double>* dFcOut) {
  (void)k; (void)M; (void)Aub;
  const int n = w.n, nc = snap.numClamping;
  const double dt = w.dt;
  // Q = A_c^T Minv A_c_ub_E + cfm I (BackpropSnapshot.cpp:2747)
  std::vector<double> MA(n * nc), Q(nc * nc);
  for (int i = 0; i < n; i++)
    for (int c = 0; c < nc; c++) {
      double s = 0;
      for (int t = 0; t < n; t++) s += Minv[i * n + t] * AcubE[t * nc + c];
      MA[i * nc + c] = s;
    }
  for (int r = 0; r < nc; r++)
    for (int c = 0; c < nc; c++) {
      double s = 0;
      for (int i = 0; i < n; i++) s += Ac[i * nc + r] * MA[i * nc + c];
      Q[r * nc + c] = s + (r == c ? snap.cfm : 0.0);
    }
  auto Qsolve = [&](const std::vector<double>& rhs /* nc x cols */, int cols, std::vector<double>& out) {
    out.assign(nc * cols, 0.0);
    std::vector<double> bb(nc), xx(nc);
    for (int c = 0; c < cols; c++) {
      for (int r = 0; r < nc; r++) bb[r] = rhs[r * cols + c];
      codSolve(Q.data(), nc, nc, bb.data(), xx.data());
      for (int r = 0; r < nc; r++) out[r * cols + c] = xx[r];
    }
  };
  // dB wrt velocity (getJacobianOfLCPOffsetClampingSubset, VELOCITY):
  //   -bounce .* A_c^T (I - dt Minv (dC_v + D + dt K))
  std::vector<double> inner(n * n), dBv(nc * n), dBf(nc * n);
  for (int r = 0; r < n; r++)
    for (int c = 0; c < n; c++) {
      double s = 0;
      for (int t = 0; t < n; t++) {
        double mat = dCv[t * n + c] + (t == c ? w.damping[c] + dt * w.spring[c] : 0.0);
        s += Minv[r * n + t] * mat;
      }
      inner[r * n + c] = (r == c ? 1.0 : 0.0) - dt * s;
    }
  for (int r = 0; r < nc; r++)
    for (int c = 0; c < n; c++) {
      double s = 0, sf = 0;
      for (int i = 0; i < n; i++) { s += Ac[i * nc + r] * inner[i * n + c]; sf += Ac[i * nc + r] * Minv[i * n + c]; }
      dBv[r * n + c] = -snap.bounceDiag[r] * s;
      dBf[r * n + c] = -snap.bounceDiag[r] * dt * sf;
    }
  std::vector<double> dFv, dFf;
  Qsolve(dBv, n, dFv);
  Qsolve(dBf, n, dFf);
  // velVel = I + Minv (A_c_ub_E dF_c - dt dC_v) - dt Minv D - dt^2 Minv K
  // forceVel = Minv (A_c_ub_E dF_c + dt I)
  std::vector<double> T1(n * n), T2(n * n);
  for (int i = 0; i < n; i++)
    for (int c = 0; c < n; c++) {
      double s1 = 0, s2 = 0;
      for (int r = 0; r < nc; r++) { s1 += AcubE[i * nc + r] * dFv[r * n + c]; s2 += AcubE[i * nc + r] * dFf[r * n + c]; }
      T1[i * n + c] = s1 - dt * dCv[i * n + c];
      T2[i * n + c] = s2 + (i == c ? dt : 0.0);
    }
  for (int r = 0; r < n; r++)
    for (int c = 0; c < n; c++) {
      double s1 = 0, s2 = 0;
      for (int t = 0; t < n; t++) { s1 += Minv[r * n + t] * T1[t * n + c]; s2 += Minv[r * n + t] * T2[t * n + c]; }
      velVel[r * n + c] = (r == c ? 1.0 : 0.0) + s1 - dt * Minv[r * n + c] * w.damping[c] -
                          dt * dt * Minv[r * n + c] * w.spring[c];
      forceVel[r * n + c] = s2;
    }
  // position: dM + Minv (A_c_ub_E dF_c + dA_c f + dA_ub E f - dt dC) - dt Minv K
  std::vector<double> dFq, dAcf;
  positionConstraintTerms(w, snap, Minv, C, dCq, Ac, Aub, AcubE, Q, dFq, dAcf);
  if (dFcOut) {
    // getJacobianOfConstraintForce (BackpropSnapshot.cpp:2723): rows f_c[r],
    // columns POSITION | VELOCITY | FORCE
    dFcOut->assign((size_t)nc * 3 * n, 0.0);
    for (int r = 0; r < nc; r++)
      for (int c = 0; c < n; c++) {
        (*dFcOut)[(size_t)r * 3 * n + c] = dFq[r * n + c];
        (*dFcOut)[(size_t)r * 3 * n + n + c] = dFv[r * n + c];
        (*dFcOut)[(size_t)r * 3 * n + 2 * n + c] = dFf[r * n + c];
      }
  }
  std::vector<double> T3(n * n);
  for (int i = 0; i < n; i++)
    for (int c = 0; c < n; c++) {
      double s = 0;
      for (int r = 0; r < nc; r++) s += AcubE[i * nc + r] * dFq[r * n + c];
      T3[i * n + c] = s + dAcf[i * n + c] - dt * dCq[i * n + c];
    }
  for (int r = 0; r < n; r++)
    for (int c = 0; c < n; c++) {
      double s = 0;
      for (int t = 0; t < n; t++) s += Minv[r * n + t] * T3[t * n + c];
      posVel[r * n + c] = dM[r * n + c] + s - Minv[r * n + c] * dt * w.spring[c];
    }
}

}  // namespace oracle

// One shape pair through the same dispatch as collide() (the collide<Shape1,
// Shape2> functions of DARTCollide.cpp): shape types / sizes as in
// nimble_world_desc, world transforms 3x4 row-major.  Output per contact:
// point3, normal3, depth, type (this package's numbering); returns the count,
// or -1 - count when a branch that is not restated was taken.
extern "C" int oracle_collide_pair(int type1, const double* size1, const double* T1r, int type2, const double* size2,
                                   const double* T2r, double clip, double* out, int maxc) {
  using namespace oracle;
  Iso<double> T1, T2;
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) { T1.R(r, c) = T1r[r * 4 + c]; T2.R(r, c) = T2r[r * 4 + c]; }
    T1.p[r] = T1r[r * 4 + 3];
    T2.p[r] = T2r[r * 4 + 3];
  }
  std::vector<Contact> pair;
  int unsup = 0;
  if (type1 == NIMBLE_SHAPE_BOX && type2 == NIMBLE_SHAPE_BOX) {
    double A[3] = {0.5 * size1[0], 0.5 * size1[1], 0.5 * size1[2]};
    double Bh[3] = {0.5 * size2[0], 0.5 * size2[1], 0.5 * size2[2]};
    boxBox(T1.p.x, T1.R.m, A, T2.p.x, T2.R.m, Bh, clip, pair, 0, 1, 0, 1);
  } else if (type1 == NIMBLE_SHAPE_BOX && type2 == NIMBLE_SHAPE_CAPSULE) {
    capsuleBox(T1, size1, T2, size2[0], size2[1], true, clip, 0, 1, 0, 1, pair, &unsup);
  } else if (type1 == NIMBLE_SHAPE_CAPSULE && type2 == NIMBLE_SHAPE_BOX) {
    capsuleBox(T2, size2, T1, size1[0], size1[1], false, clip, 0, 1, 0, 1, pair, &unsup);
  } else if (type1 == NIMBLE_SHAPE_SPHERE && type2 == NIMBLE_SHAPE_BOX) {
    sphereBoxPair(T2, size2, T1.p.x, size1[0], false, clip, 0, 1, 0, 1, pair);
  } else if (type1 == NIMBLE_SHAPE_BOX && type2 == NIMBLE_SHAPE_SPHERE) {
    sphereBoxPair(T1, size1, T2.p.x, size2[0], true, clip, 0, 1, 0, 1, pair);
  } else if (type1 == NIMBLE_SHAPE_SPHERE && type2 == NIMBLE_SHAPE_SPHERE) {
    sphereSphere(T1.p.x, size1[0], T2.p.x, size2[0], clip, 0, 1, 0, 1, pair);
  } else if (type1 == NIMBLE_SHAPE_SPHERE && type2 == NIMBLE_SHAPE_CAPSULE) {
    sphereCapsule(T1.p.x, size1[0], T2, size2[0], size2[1], true, clip, 0, 1, 0, 1, pair);
  } else if (type1 == NIMBLE_SHAPE_CAPSULE && type2 == NIMBLE_SHAPE_SPHERE) {
    sphereCapsule(T2.p.x, size2[0], T1, size1[0], size1[1], false, clip, 0, 1, 0, 1, pair);
  } else if (type1 == NIMBLE_SHAPE_CAPSULE && type2 == NIMBLE_SHAPE_CAPSULE) {
    capsuleCapsule(T1, size1[0], size1[1], T2, size2[0], size2[1], clip, 0, 1, 0, 1, pair);
  } else {
    return -1;
  }
  const int k = (int)pair.size() < maxc ? (int)pair.size() : maxc;
  for (int c = 0; c < k; c++) {
    for (int i = 0; i < 3; i++) { out[8 * c + i] = pair[c].point[i]; out[8 * c + 3 + i] = pair[c].normal[i]; }
    out[8 * c + 6] = pair[c].depth;
    out[8 * c + 7] = pair[c].type;
  }
  return unsup ? -1 - k : k;
}
