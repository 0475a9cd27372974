// Contact handling for the gfx950 timestep: box-box narrow phase, contact
// constraint rows, the boxed LCP with Nimble's gradient short-circuit
// (classification + least-squares standardisation), Dantzig / PGS fallbacks,
// and the constraint impulses.
//
// Reference behaviour (see oracle/ for the CPU restatement and its pins):
//   dart/collision/dart/DARTCollide.cpp:764 dBoxBox, :513 intersectRectQuad
//   dart/collision/dart/DARTCollisionDetector.cpp:127 (pair loop), :357 postProcess
//   dart/constraint/ConstraintSolver.cpp:520 updateConstraints
//   dart/constraint/ContactConstraint.cpp:393 getInformation, :705 tangent basis
//   dart/constraint/BoxedLcpConstraintSolver.cpp:175 buildLcpInputs, :330 solveLcp
//   dart/neural/ConstrainedGroupGradientMatrices.cpp:482 constructMatrices,
//     :218 opportunisticallyStandardizeResults
//   dart/external/odelcpsolver/lcp.cpp:780 dSolveLCP
//   dart/constraint/PgsBoxedLcpSolver.cpp:85
//
// GPU structure: the pair tests run one pair per lane; the small dense LCP
// algebra (m <= 48 rows) runs on LDS-resident matrices.  The sequential
// pivoting of Dantzig and the Householder sweeps of the COD solve are driven
// by lane 0 while lanes 1..63 wait at the next barrier -- for the <= 24-row
// problems of the benchmark models this is a small fraction of the step.
#pragma once
#include "model.h"
#include "spatial.cuh"
#include "pool_sizes.h"
#include "capsule.cuh"
#include "mesh.cuh"

#define CT_FACE_VERTEX 1
#define CT_VERTEX_FACE 2
#define CT_EDGE_EDGE 3
#include "stamp.cuh"

#define CM_CLAMPING (-1)
#define CM_NOT_CLAMPING (-2)


// ---------------------------------------------------------------------------
// dBoxBox (one pair, one lane).  R1/R2 row-major 3x3, A/B half sizes.
// Writes up to 8 contact records to `out`; returns the count.
// ---------------------------------------------------------------------------
__device__ int deviceBoxBox(const double* p1, const double* R1, const double* A, const double* p2,
                            const double* R2, const double* B, double clipDepth, int b1, int b2, double* out) {
  // keep the separating-axis / clipping arithmetic unfused so that exact
  // comparisons (edge classification) agree with the CPU restatement
#pragma clang fp contract(off)
  const double fudge = 1.05;
  double p[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  double pp[3];
  for (int i = 0; i < 3; i++) pp[i] = R1[i] * p[0] + R1[3 + i] * p[1] + R1[6 + i] * p[2];
  double Rm[9], Qm[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      Rm[i * 3 + j] = R1[i] * R2[j] + R1[3 + i] * R2[3 + j] + R1[6 + i] * R2[6 + j];
      Qm[i * 3 + j] = fabs(Rm[i * 3 + j]);
    }
  double s = -1e12;
  int invertNormal = 0, code = 0, normalCol = -1, normalBox = 0;
  double normalC[3] = {0, 0, 0};
  for (int i = 0; i < 3; i++) {
    double e1 = pp[i];
    double e2 = A[i] + B[0] * Qm[i * 3] + B[1] * Qm[i * 3 + 1] + B[2] * Qm[i * 3 + 2];
    double s2 = fabs(e1) - e2;
    if (s2 > s) { s = s2; normalBox = 1; normalCol = i; invertNormal = e1 < 0; code = 1 + i; }
  }
  for (int j = 0; j < 3; j++) {
    double e1 = R2[j] * p[0] + R2[3 + j] * p[1] + R2[6 + j] * p[2];
    double e2 = A[0] * Qm[j] + A[1] * Qm[3 + j] + A[2] * Qm[6 + j] + B[j];
    double s2 = fabs(e1) - e2;
    if (s2 > s) { s = s2; normalBox = 2; normalCol = j; invertNormal = e1 < 0; code = 4 + j; }
  }
  const double R11 = Rm[0], R12 = Rm[1], R13 = Rm[2], R21 = Rm[3], R22 = Rm[4], R23 = Rm[5], R31 = Rm[6],
               R32 = Rm[7], R33 = Rm[8];
  const double Q11 = Qm[0], Q12 = Qm[1], Q13 = Qm[2], Q21 = Qm[3], Q22 = Qm[4], Q23 = Qm[5], Q31 = Qm[6],
               Q32 = Qm[7], Q33 = Qm[8];
  const double E1[9] = {pp[2] * R21 - pp[1] * R31, pp[2] * R22 - pp[1] * R32, pp[2] * R23 - pp[1] * R33,
                        pp[0] * R31 - pp[2] * R11, pp[0] * R32 - pp[2] * R12, pp[0] * R33 - pp[2] * R13,
                        pp[1] * R11 - pp[0] * R21, pp[1] * R12 - pp[0] * R22, pp[1] * R13 - pp[0] * R23};
  const double E2[9] = {A[1] * Q31 + A[2] * Q21 + B[1] * Q13 + B[2] * Q12,
                        A[1] * Q32 + A[2] * Q22 + B[0] * Q13 + B[2] * Q11,
                        A[1] * Q33 + A[2] * Q23 + B[0] * Q12 + B[1] * Q11,
                        A[0] * Q31 + A[2] * Q11 + B[1] * Q23 + B[2] * Q22,
                        A[0] * Q32 + A[2] * Q12 + B[0] * Q23 + B[2] * Q21,
                        A[0] * Q33 + A[2] * Q13 + B[0] * Q22 + B[1] * Q21,
                        A[0] * Q21 + A[1] * Q11 + B[1] * Q33 + B[2] * Q32,
                        A[0] * Q22 + A[1] * Q12 + B[0] * Q33 + B[2] * Q31,
                        A[0] * Q23 + A[1] * Q13 + B[0] * Q32 + B[1] * Q31};
  const double NN[27] = {0, -R31, R21, 0, -R32, R22, 0, -R33, R23,
                         R31, 0, -R11, R32, 0, -R12, R33, 0, -R13,
                         -R21, R11, 0, -R22, R12, 0, -R23, R13, 0};
  for (int t = 0; t < 9; t++) {
    double s2 = fabs(E1[t]) - E2[t];
    const double n1 = NN[3 * t], n2 = NN[3 * t + 1], n3 = NN[3 * t + 2];
    double l = sqrt(n1 * n1 + n2 * n2 + n3 * n3);
    if (l > 0) {
      s2 /= l;
      if (s2 * fudge > s) {
        s = s2; normalCol = -1; normalC[0] = n1 / l; normalC[1] = n2 / l; normalC[2] = n3 / l;
        invertNormal = E1[t] < 0; code = 7 + t;
      }
    }
  }
  if (!code || s > 0.0) return 0;
  double normal[3];
  if (normalCol >= 0) {
    const double* R = normalBox == 1 ? R1 : R2;
    normal[0] = R[normalCol]; normal[1] = R[3 + normalCol]; normal[2] = R[6 + normalCol];
  } else {
    for (int i = 0; i < 3; i++) normal[i] = R1[i * 3] * normalC[0] + R1[i * 3 + 1] * normalC[1] + R1[i * 3 + 2] * normalC[2];
    double l = sqrt(normal[0] * normal[0] + normal[1] * normal[1] + normal[2] * normal[2]);
    for (int i = 0; i < 3; i++) normal[i] /= l;
  }
  if (invertNormal) for (int i = 0; i < 3; i++) normal[i] = -normal[i];
  if (code > 6) {
    double pa[3] = {p1[0], p1[1], p1[2]}, pb[3] = {p2[0], p2[1], p2[2]};
    for (int j = 0; j < 3; j++) {
      double v = normal[0] * R1[j] + normal[1] * R1[3 + j] + normal[2] * R1[6 + j];
      double sign = (v > -1e-10) ? 1.0 : -1.0;
      for (int i = 0; i < 3; i++) pa[i] += sign * A[j] * R1[i * 3 + j];
    }
    for (int j = 0; j < 3; j++) {
      double v = normal[0] * R2[j] + normal[1] * R2[3 + j] + normal[2] * R2[6 + j];
      double sign = (v > -1e-3) ? -1.0 : 1.0;
      for (int i = 0; i < 3; i++) pb[i] += sign * B[j] * R2[i * 3 + j];
    }
    const int ca = (code - 7) / 3, cb = (code - 7) % 3;
    double ua[3] = {R1[ca], R1[3 + ca], R1[6 + ca]}, ub[3] = {R2[cb], R2[3 + cb], R2[6 + cb]};
    double pd[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]};
    double uaub = dot3(ua, ub), q1 = dot3(ua, pd), q2 = -dot3(ub, pd);
    double dd = 1 - uaub * uaub, alpha = 0, beta = 0;
    if (dd > 0) { dd = 1.0 / dd; alpha = (q1 + uaub * q2) * dd; beta = (uaub * q1 + q2) * dd; }
    // edge metadata (DARTCollide.cpp:1046): fixed points before the closest
    // approach, unit directions
    double* e = out + CREC;
    {
      const double la = sqrt(dot3(ua, ua)), lb = sqrt(dot3(ub, ub));
      for (int i = 0; i < 3; i++) { e[i] = pa[i]; e[3 + i] = ua[i] / la; e[6 + i] = pb[i]; e[9 + i] = ub[i] / lb; }
    }
    for (int i = 0; i < 3; i++) { pa[i] += ua[i] * alpha; pb[i] += ub[i] * beta; }
    if (-s > clipDepth) return 0;
    for (int i = 0; i < 3; i++) { out[i] = 0.5 * (pa[i] + pb[i]); out[3 + i] = -normal[i]; }
    out[6] = -s; out[7] = CT_EDGE_EDGE; out[8] = b1; out[9] = b2;
    return 1;
  }
  const double *Ra, *Rb, *pa, *pb, *Sa, *Sb;
  const bool flip = code > 3;
  if (!flip) { Ra = R1; Rb = R2; pa = p1; pb = p2; Sa = A; Sb = B; }
  else { Ra = R2; Rb = R1; pa = p2; pb = p1; Sa = B; Sb = A; }
  double normal2[3], nr[3], anr[3];
  for (int i = 0; i < 3; i++) normal2[i] = flip ? -normal[i] : normal[i];
  for (int i = 0; i < 3; i++) nr[i] = Rb[i] * normal2[0] + Rb[3 + i] * normal2[1] + Rb[6 + i] * normal2[2];
  for (int i = 0; i < 3; i++) anr[i] = fabs(nr[i]);
  int lanr, a1, a2;
  if (anr[1] > anr[0]) {
    if (anr[1] > anr[2]) { a1 = 0; lanr = 1; a2 = 2; } else { a1 = 0; a2 = 1; lanr = 2; }
  } else {
    if (anr[0] > anr[2]) { lanr = 0; a1 = 1; a2 = 2; } else { a1 = 0; a2 = 1; lanr = 2; }
  }
  double center[3];
  for (int i = 0; i < 3; i++)
    center[i] = nr[lanr] < 0 ? pb[i] - pa[i] + Sb[lanr] * Rb[i * 3 + lanr] : pb[i] - pa[i] - Sb[lanr] * Rb[i * 3 + lanr];
  const int codeN = flip ? code - 4 : code - 1;
  const int code1 = codeN == 0 ? 1 : 0, code2 = codeN == 2 ? 1 : 2;
  double c1 = center[0] * Ra[code1] + center[1] * Ra[3 + code1] + center[2] * Ra[6 + code1];
  double c2 = center[0] * Ra[code2] + center[1] * Ra[3 + code2] + center[2] * Ra[6 + code2];
  double m11 = Ra[code1] * Rb[a1] + Ra[3 + code1] * Rb[3 + a1] + Ra[6 + code1] * Rb[6 + a1];
  double m12 = Ra[code1] * Rb[a2] + Ra[3 + code1] * Rb[3 + a2] + Ra[6 + code1] * Rb[6 + a2];
  double m21 = Ra[code2] * Rb[a1] + Ra[3 + code2] * Rb[3 + a1] + Ra[6 + code2] * Rb[6 + a1];
  double m22 = Ra[code2] * Rb[a2] + Ra[3 + code2] * Rb[3 + a2] + Ra[6 + code2] * Rb[6 + a2];
  double quad[8];
  {
    double k1 = m11 * Sb[a1], k2 = m21 * Sb[a1], k3 = m12 * Sb[a2], k4 = m22 * Sb[a2];
    quad[0] = c1 - k1 - k3; quad[1] = c2 - k2 - k4;
    quad[2] = c1 - k1 + k3; quad[3] = c2 - k2 + k4;
    quad[4] = c1 + k1 + k3; quad[5] = c2 + k2 + k4;
    quad[6] = c1 + k1 - k3; quad[7] = c2 + k2 - k4;
  }
  double rect[2] = {Sa[code1], Sa[code2]};
  // intersectRectQuad with ping-pong buffers (bufA/bufB), as in the reference
  double bufA[16], bufB[16];
  for (int i = 0; i < 8; i++) bufB[i] = quad[i];
  // q starts at quad (kept in bufB), r at ret (bufA)
  double* q = bufB;
  double* r = bufA;
  int nq = 4, nrr = 0;
  bool stop = false;
  for (int dir = 0; dir <= 1 && !stop; dir++) {
    for (int sign = -1; sign <= 1 && !stop; sign += 2) {
      double* pq = q;
      double* pr = r;
      nrr = 0;
      for (int i = nq; i > 0; i--) {
        if (sign * pq[dir] < rect[dir]) {
          pr[0] = pq[0]; pr[1] = pq[1]; pr += 2; nrr++;
          if (nrr & 8) { q = r; stop = true; break; }
        }
        double* nextq = (i > 1) ? pq + 2 : q;
        if ((sign * pq[dir] < rect[dir]) ^ (sign * nextq[dir] < rect[dir])) {
          pr[1 - dir] = pq[1 - dir] + (nextq[1 - dir] - pq[1 - dir]) / (nextq[dir] - pq[dir]) * (sign * rect[dir] - pq[dir]);
          pr[dir] = sign * rect[dir];
          pr += 2; nrr++;
          if (nrr & 8) { q = r; stop = true; break; }
        }
        pq += 2;
      }
      if (stop) break;
      q = r;
      r = (q == bufA) ? bufB : bufA;
      nq = nrr;
    }
  }
  double* ret = q;  // final polygon
  if (nrr < 1) return 0;
  double det1 = 1.0 / (m11 * m22 - m12 * m21);
  m11 *= det1; m12 *= det1; m21 *= det1; m22 *= det1;
  int cnum = 0;
  for (int j = 0; j < nrr; j++) {
    double k1 = m22 * (ret[j * 2] - c1) - m12 * (ret[j * 2 + 1] - c2);
    double k2 = -m21 * (ret[j * 2] - c1) + m11 * (ret[j * 2 + 1] - c2);
    double pt[3];
    for (int i = 0; i < 3; i++) pt[i] = center[i] + k1 * Rb[i * 3 + a1] + k2 * Rb[i * 3 + a2];
    double dep = Sa[codeN] - dot3(normal2, pt);
    if (dep >= 0) {
      double* o = out + PBREC * cnum;
      double xx = ret[j * 2], yy = ret[j * 2 + 1];
      for (int i = 0; i < 3; i++) { o[i] = pt[i] + pa[i]; o[3 + i] = -normal[i]; }
      o[6] = dep;
      bool onX = fabs(xx) == rect[0], onY = fabs(yy) == rect[1];
      int type;
      if (onX && onY) {
        if (flip) { type = CT_FACE_VERTEX; for (int i = 0; i < 3; i++) o[i] += o[3 + i] * dep; }
        else { type = CT_VERTEX_FACE; for (int i = 0; i < 3; i++) o[i] -= o[3 + i] * dep; }
      } else if (!onX && !onY) {
        type = flip ? CT_VERTEX_FACE : CT_FACE_VERTEX;
      } else {
        // on an edge of the reference face, not at a corner
        // (DARTCollide.cpp:1318): edge A along that face edge through its
        // nearest corner, edge B along the nearest incident-face edge
        type = CT_EDGE_EDGE;
        const double faceX = xx > 0 ? rect[0] : -rect[0], faceY = yy > 0 ? rect[1] : -rect[1];
        double eaF[3], eaD[3], ebF[3], ebD[3];
        for (int i = 0; i < 3; i++)
          eaF[i] = (pa[i] + Sa[codeN] * normal[i]) + faceX * Ra[i * 3 + code1] + faceY * Ra[i * 3 + code2];
        {
          double l = 0;
          for (int i = 0; i < 3; i++) { eaD[i] = o[i] - eaF[i]; l += eaD[i] * eaD[i]; }
          l = sqrt(l);
          for (int i = 0; i < 3; i++) eaD[i] /= l;
        }
        double other[3], o1[3], o2[3];
        for (int i = 0; i < 3; i++) { other[i] = Rb[i * 3 + lanr]; o1[i] = Rb[i * 3 + a1]; o2[i] = Rb[i * 3 + a2]; }
        if (dot3(other, normal) < 0)
          for (int i = 0; i < 3; i++) other[i] = -other[i];
        double faceCenter[3];
        for (int i = 0; i < 3; i++) faceCenter[i] = pb[i] - Sb[lanr] * other[i];
        const double ifx = dot3(o1, o) - dot3(o1, pb), ify = dot3(o2, o) - dot3(o2, pb);
        const double sx = ifx == 0 ? 1.0 : ifx / fabs(ifx), sy = ify == 0 ? 1.0 : ify / fabs(ify);
        double nearB[3], otherB[3];
        for (int i = 0; i < 3; i++) nearB[i] = (sx * Sb[a1]) * o1[i] + (sy * Sb[a2]) * o2[i] + faceCenter[i];
        const double distX = fabs(fabs(ifx) - Sb[a1]), distY = fabs(fabs(ify) - Sb[a2]);
        if (distX < distY)
          for (int i = 0; i < 3; i++) otherB[i] = (sx * Sb[a1]) * o1[i] + (-1 * sy * Sb[a2]) * o2[i] + faceCenter[i];
        else
          for (int i = 0; i < 3; i++) otherB[i] = (-1 * sx * Sb[a1]) * o1[i] + (sy * Sb[a2]) * o2[i] + faceCenter[i];
        {
          double l = 0;
          for (int i = 0; i < 3; i++) { ebD[i] = nearB[i] - otherB[i]; l += ebD[i] * ebD[i]; }
          l = sqrt(l);
          for (int i = 0; i < 3; i++) { ebD[i] /= l; ebF[i] = nearB[i]; }
        }
        double* e = o + CREC;
        for (int i = 0; i < 3; i++) {
          e[i] = flip ? ebF[i] : eaF[i]; e[3 + i] = flip ? ebD[i] : eaD[i];
          e[6 + i] = flip ? eaF[i] : ebF[i]; e[9 + i] = flip ? eaD[i] : ebD[i];
        }
      }
      o[7] = type; o[8] = b1; o[9] = b2;
      cnum++;
    }
  }
  return cnum;
}

// ContactConstraint::getTangentBasisMatrixODE (ContactConstraint.cpp:705)
__device__ void tangentBasisODE(const double* n, double* t1, double* t2) {
#pragma clang fp contract(off)
  const double ez[3] = {0, 0, 1}, ex[3] = {1, 0, 0}, ey[3] = {0, 1, 0};
  double t[3];
  cross3(ez, n, t);
  if (dot3(t, t) < 1e-12) {
    cross3(ex, n, t);
    if (dot3(t, t) < 1e-12) {
      cross3(ey, n, t);
      if (dot3(t, t) < 1e-12) cross3(ez, n, t);
    }
  }
  double l = sqrt(dot3(t, t));
  for (int i = 0; i < 3; i++) t1[i] = t[i] / l;
  cross3(n, t1, t2);
}

// ---------------------------------------------------------------------------
// Per-world LCP workspace, carved at run time for the actual row count m.
// It lives in LDS when it fits the model's LDS pool and otherwise in the
// world's snapshot tail in HBM (same code, different base pointer).
// ---------------------------------------------------------------------------

struct FwdPool {
  double *cols, *massed, *A, *M1, *M2;
  double *lo, *hi, *b, *X, *aCol, *rest, *pen, *relVel, *fc, *Eval, *nx, *fsol, *xc, *xh, *xh2, *xp, *xf, *dvec;
  int *fi, *mapping, *clampIdx, *ubIdx, *rowC, *rowDir, *clampRow, *cl;
  double* scr;  // >= 10 m + 2 n + 16
};

// (rows first: J^T, the rows' directions, boxes and restitution and the int
// vectors take the pool's first n m + 10 m doubles, which in the one-row
// kernel lie clear of the dynamics buffers -- the helper's early rows, EA_*)
__device__ inline void carveFwd(double* base, int m, int n, FwdPool& P) {
  double* p = base;
  P.cols = p; p += n * m;
  P.massed = P.cols;  // Y = L^-1 J^T overwrites J^T in place
  // plain member assignments (no pointer-to-member tables) keep the
  // pointers' provenance visible, so LDS-laundered bases stay LDS
  P.lo = p; p += m;
  P.hi = p; p += m;
  P.rest = p; p += m;
  P.dvec = p; p += 3 * m;
  int* ip = reinterpret_cast<int*>(p);
  P.fi = ip; ip += m;
  P.rowC = ip; ip += m;
  P.rowDir = ip; ip += m;
  P.mapping = ip; ip += m;
  P.clampIdx = ip; ip += m;
  P.ubIdx = ip; ip += m;
  P.clampRow = ip; ip += m;
  P.cl = ip; ip += m;
  p += 4 * m;
  P.A = p; p += m * m;
  P.M1 = p; p += m * m;
  P.M2 = p; p += m * (m | 1);  // Dantzig's L with an odd leading dimension
  P.b = p; p += m;
  P.X = p; p += m;
  P.aCol = p; p += m;
  P.pen = p; p += m;
  P.relVel = p; p += m;
  P.fc = p; p += m;
  P.Eval = p; p += m;
  P.nx = p; p += m;
  P.fsol = p; p += m;
  P.xc = p; p += m;
  P.xh = p; p += m;   // the helper wave's Dantzig solution
  P.xh2 = p; p += m;  // ... and its scratch
  // (aliases, see the task board: the PGS fallback's solution overwrites
  // its warm start once read, the frictionless PGS's solution the
  // penetration-correction terms, dead after the row setup)
  P.xp = P.xc;
  P.xf = P.pen;
  P.scr = p;
}

#include "lcp_wave.cuh"

// A = Y^T Y (m x m, Y n x m row-major) with v_mfma_f64_16x16x4f64, one 16 x
// 16 tile of A per MFMA chain over ceil(n / 4) k-steps (the upper tiles,
// mirrored).  Operand lanes: A/B lane l = row / column l % 16 of the tile, k
// = l / 16; result element e of lane l = tile row l / 16 + 4 e, column l % 16
// (the f64 layout).  All 64 lanes must be active.  For the Atlas LCP (n = 33,
// m = 24) this takes 5.3k clocks against 9.9k for the 8 x 8 VALU lane tiles
// (tools/micro/mfma_gram.hip, profiles/r02e_mfma_gram_micro.json).
typedef double nimble_double4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void gramMfma(const double* Y, double* A, int n, int m, int lane) {
  const int i16 = lane & 15, kq = lane >> 4;
  const int T = (m + 15) >> 4;
  for (int ti = 0; ti < T; ti++)
    for (int tj = ti; tj < T; tj++) {
      nimble_double4 acc = {0.0, 0.0, 0.0, 0.0};
      const int ri = ti * 16 + i16, cj = tj * 16 + i16;
#pragma unroll 3
      for (int k0 = 0; k0 < n; k0 += 4) {
        const int k = k0 + kq;
        const double a = (k < n && ri < m) ? Y[k * m + ri] : 0.0;
        const double b = (k < n && cj < m) ? Y[k * m + cj] : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
      }
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int r = ti * 16 + kq + 4 * e, c = tj * 16 + i16;
        if (r < m && c < m && r <= c) {
          A[r * m + c] = acc[e];
          A[c * m + r] = acc[e];
        }
      }
    }
}

// ---------------------------------------------------------------------------
// Contact-stage LDS header (at Layout::ct) and snapshot layout.
// ---------------------------------------------------------------------------
#define H_NCON 0
#define H_M 1
#define H_STATUS 2
#define H_NDROP 3
#define H_FLAG 4
#define H_NC 5
#define H_NU 6
#define H_STD 7
#define H_CFM 8
#define H_SC 9
#define H_IGN 10
#define H_K 11
#define H_CODOK 12  // M1 + scr hold the COD of the final clamping Q
#define H_HELPER 13 // 2 doubles = 4 ints: helper state (HS_*), unused x3
#define H_COLLIDE 15  // 2 ints: collision-detection hand-off between the waves (CS_*)
#define H_PAIRCNT 16   // 16 per-pair counts of the current chunk
// the LCP solvers' executed-work tally (2 doubles = 4 ints: Dantzig pivots,
// PGS sweeps, FLOPs, unused), in the pair counts' dead tail past the board
#define H_TALLY 24
// the LCP task board (BD_*, 16 ints): the pair counts are collision-time
// scratch, dead once the contacts are final, when the board is first used
#define H_BOARD H_PAIRCNT

// ---------------------------------------------------------------------------
// Helper wave.  The forward kernel runs two waves per world: wave 0 does the
// step; wave 1 (the helper) detects the contacts (collideWorld, below) and
// then shares the LCP cascade of BoxedLcpConstraintSolver::solve with wave 0.
// The reference's cascade is a priority order over independent computations
// on the same inputs A, b, lo, hi, findex (none of them writes those):
//   C  the short-circuit classification (devConstruct, from the warm start)
//   D  Dantzig on A (LCPUtils::reduce first: taken here only when it merges
//      no column; otherwise wave 0 runs the reduced Dantzig itself)
//   P  PGS on (reduced) A + cfm I from the warm start
//   F  PGS on the normal rows only (LCPUtils::removeFriction), from zero
// and its answer is the first of C, D, P, F that succeeds (and validates).
// D needs only A, so the helper starts it as soon as A is built, while wave 0
// computes the warm start and runs C; whichever wave is free then claims P
// (once the warm start is final) and F.  Results are written to their own LDS
// vectors (xh, xp, xf) and taken in the reference's order, so the answer is
// the same whichever wave computed it and however the work interleaved; a
// computation made moot by a higher-priority success is cancelled (polled
// per pivot / sweep).  Protocol per world: wave 0 posts TASK (board cleared)
// or SKIP exactly once, the helper answers DONE once it has stopped touching
// the pool, wave 0 resets to IDLE.
// ---------------------------------------------------------------------------
#define HS_IDLE 0
#define HS_TASK 1
#define HS_SKIP 2
#define HS_DONE 3
#define HS_POST 4      // (one-row kernel) wave 0's post-answer share for the helper, see contactLcp
#define HS_POSTDONE 5  // ... done
#define BD_G 0        // warm start final (P.xc): 1
#define BD_D 1        // Dantzig: 0 running, 1 ok + valid, 2 failed, 3 not run (reduce merges)
#define BD_PCLAIM 2   // PGS fallback: 0 unclaimed, 1 wave 0, 2 helper
#define BD_P 3        //   0 pending, 1 ok + valid, 2 failed
#define BD_PDUP 4     //   its reduce merged columns
#define BD_FCLAIM 5   // frictionless PGS: claim as BD_PCLAIM
#define BD_F 6        //   0 pending, 1 done
#define BD_STOPD 7    // cancel flags: Dantzig,
#define BD_STOPP 8    //   PGS fallback,
#define BD_STOPF 9    //   frictionless PGS
#define BD_INTS 10
__device__ __forceinline__ int* helperFlags(double* ct) { return reinterpret_cast<int*>(ct + H_HELPER); }
__device__ __forceinline__ void helperPost(double* ct, int state, int lane) {
  // release: the task's LDS inputs are visible before the state changes
  if (lane == 0) __hip_atomic_store(helperFlags(ct), state, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int helperState(double* ct) {
  return uni(__hip_atomic_load(helperFlags(ct), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
// Deadlock guard of every wait between the two waves: a wait that outlasts
// kSpinTicks of the constant 100 MHz real-time counter (1 s: more than two
// hundred times the slowest world's whole step, ~8.4M clocks = 3.5 ms, so
// never a slow but live partner) gives up instead of hanging the device or
// trapping: it raises the world's protocol flag (helperFlags(ct)[3], set
// into the snapshot status as ST_PROTOCOL by wave 0, a status that makes the
// step raise).  A wait also gives up as soon as the partner has raised the
// flag, so one expiry ends every wait of the world at once.  After a failure
// neither wave relies on the other: wave 0 abandons the world's contact step
// without touching anything the helper may still write (protocolAbort: the
// contact header and list, the pool and the board's vectors stay the
// helper's), the helper leaves at its next wait, every wave reaches its exit
// and the launch drains.  The clock is read once per 64 polls.
constexpr long long kSpinTicks = 100000000ll;
__device__ __forceinline__ long long spinClock() { return (long long)__builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ bool spinExpired(long long t0, int it) {
  return (it & 63) == 63 && spinClock() - t0 > kSpinTicks;
}
// (the flag is polled inside the waits while the other wave may raise it:
// atomic accesses, so that the poll is re-read every time and, under the
// host emulation, lane 0's observation is the whole wave's)
__device__ __forceinline__ void protocolFail(double* ct) {
  __hip_atomic_store(helperFlags(ct) + 3, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ bool protocolFailed(double* ct) {
  return uni(__hip_atomic_load(helperFlags(ct) + 3, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0;
}
// The wait sites, for the guard's test switch: NIMBLE_AMD_GUARD_TEST
// (capi.cpp, tests only) puts a mask of sites into helperFlags(ct)[2] for the
// worlds it targets, and a wait at a masked site expires at once -- a partner
// that is late at exactly that point -- so every failure path runs on purpose
// (tests/test_gpu_guard.py, tests/test_wave_emu.py).  0 in every other run.
#define GW_HELPER_GO 1      // helper: wave 0's CS_GO (body transforms final; one-row kernel)
#define GW_COLLIDE_DONE 2   // wave 0: the helper's CS_DONE (contacts detected; one-row kernel)
#define GW_MERGED 4         // wave 0: the helper out of the pool before a reduced Dantzig (on chip)
#define GW_BOARD 8          // wave 0: the task board's answer (Dantzig / PGS fallback / frictionless)
#define GW_NAN 16           // wave 0: the helper out of the pool before the fallbacks (NaN answer)
#define GW_COLLECT 32       // wave 0: the helper out of the pool before construct 2
#define GW_HELPER_TASK 64   // helper: wave 0's TASK or SKIP
#define GW_HELPER_WARM 128  // helper: the final warm start for the PGS fallback
#define GW_HELPER_IDLE 256  // helper: wave 0 took its DONE
#define GW_RETIRE 512       // wave 0: the helper's DONE at the world's end
#define GW_ONE_ROW_ONLY 1024  // (modifier) the sites in the one-row kernel only, not in the wide kernel
#define GW_EARLY_B 2048       // helper: wave 0 has formed b (early rows, one-row kernel)
#define GW_EARLY_DYN 32768    // helper: wave 0's dynamics done (early rows)
#define GW_EARLY_ROWS 4096    // wave 0: the helper's early rows
#define GW_EARLY_A 8192       // wave 0: the helper's A = Y^T Y
#define GW_POST 16384         // wave 0: the helper's post-answer share (impulse, snapshot rows)
__device__ __forceinline__ bool guardForced(double* ct, int site) { return (uni(helperFlags(ct)[2]) & site) != 0; }
// spin with s_sleep until pred(state); -1 when the guard expired (or was
// forced at `site`, or the partner failed)
template <class Pred>
__device__ __forceinline__ int helperWait(double* ct, Pred pred, int site) {
  if (guardForced(ct, site)) {
    protocolFail(ct);
    return -1;
  }
  const long long t0 = spinClock();
  for (int it = 0;; it++) {
    const int st = helperState(ct);
    if (pred(st)) return st;
    if (protocolFailed(ct) || spinExpired(t0, it)) {
      protocolFail(ct);
      return -1;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
__device__ __forceinline__ int* board(double* ct) { return reinterpret_cast<int*>(ct + H_BOARD); }
__device__ __forceinline__ int* tallyOf(double* ct) { return reinterpret_cast<int*>(ct + H_TALLY); }
__device__ __forceinline__ int boardGet(double* ct, int k) {
  return uni(__hip_atomic_load(board(ct) + k, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void boardSet(double* ct, int k, int v, int lane) {
  // release: a result's LDS vector is visible before its state
  if (lane == 0) __hip_atomic_store(board(ct) + k, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// claim task slot k for `who` (1 wave 0, 2 helper); true for the one winner
__device__ __forceinline__ bool boardClaim(double* ct, int k, int who, int lane) {
  int won = 0;
  if (lane == 0) {
    int expect = 0;
    won = __hip_atomic_compare_exchange_strong(board(ct) + k, &expect, who, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE,
                                               __HIP_MEMORY_SCOPE_WORKGROUP) ? 1 : 0;
  }
  return rdli(won, 0) != 0;
}

// board mode (helperFlags(ct)[1], set by wave 0 before it posts the task):
// 0 the pool in LDS at L.pool (one row per lane), 1 the wide kernel's HBM
// pool (two rows per lane) with Dantzig's factor at the start of its LDS
// stage (which begins at L.pool)
#define HB_LDS_POOL 0
#define HB_WIDE 1
// wave 0 posts the cascade's task (board cleared, mode, warm start final or not)
__device__ __forceinline__ void boardPost(double* ct, int mode, bool warmFinal, int lane) {
  if (lane < BD_INTS) board(ct)[lane] = 0;
  if (lane == 0) helperFlags(ct)[1] = mode;
  if (warmFinal) boardSet(ct, BD_G, 1, lane);
  helperPost(ct, HS_TASK, lane);
}

// Collision detection on the helper wave.  collideWorld only reads the
// body transforms (kinematics) and writes the contact header / list and its
// own scratch clear of the dynamics buffers, so it overlaps wave 0's composite
// inertias, mass matrix, Cholesky factor and unconstrained velocity.  Per
// world: wave 0 posts CS_GO after the kinematics, the helper answers CS_DONE,
// wave 0 takes the contacts and resets to CS_IDLE before the next world.
#define CS_IDLE 0
#define CS_GO 1
#define CS_DONE 2
__device__ __forceinline__ int* collideFlag(double* ct) { return reinterpret_cast<int*>(ct + H_COLLIDE); }
__device__ __forceinline__ void collidePost(double* ct, int state, int lane) {
  if (lane == 0) __hip_atomic_store(collideFlag(ct), state, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// false when the deadlock guard expired (see helperWait)
__device__ __forceinline__ bool collideWait(double* ct, int want, int site) {
  if (guardForced(ct, site)) {
    protocolFail(ct);
    return false;
  }
  const long long t0 = spinClock();
  for (int it = 0;; it++) {
    if (uni(__hip_atomic_load(collideFlag(ct), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) == want) return true;
    if (protocolFailed(ct) || spinExpired(t0, it)) {
      protocolFail(ct);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Early rows (one-row kernel): the helper wave is idle from the end of the
// collision detection until A is built, while wave 0 is still in the
// composites, the mass matrix, its Cholesky factor and the unconstrained
// solve.  So, once the contacts are final, the helper builds the LCP rows and
// J^T in the LDS pool -- their slots come first in the pool (carveFwd) and
// the one-row kernel's layout puts the dynamics buffers at the far end of the
// pool area (capi.cpp makeLayout, Layout::early), so they are clear of
// everything wave 0 still uses.  Once wave 0's dynamics are done (HF_DYN in
// helperFlags(ct)[1], which the board's mode overwrites later) the helper
// forms Y = L^-1 J^T into M1 (+ M2, free until the cascade) and A = Y^T Y;
// wave 0 forms b = -J v1 from J^T meanwhile and posts HF_B, after which the
// helper moves Y into J^T's place; wave 0, through the penetration terms,
// meets a built A.  Same
// operations in the same order on the same operands as wave 0's own path,
// so the same bits.  The helper's progress is the second int of H_COLLIDE
// (written by the helper only; EA_NONE is stored before its CS_DONE):
#define EA_PENDING 0  // contacts final, rows in progress
#define EA_NONE 1     // not taken: wave 0 builds the rows itself
#define EA_ROWS 2     // rows + J^T in the pool
#define EA_A 3        // Y and A formed
#define HF_DYN 2      // helperFlags(ct)[1] before the board: wave 0's dynamics are done (Cholesky final)
#define HF_B 3        // ... and b formed: J^T read
__device__ __forceinline__ void dynDonePost(double* ct, int lane) {
  if (lane == 0) __hip_atomic_store(helperFlags(ct) + 1, HF_DYN, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int* earlyFlag(double* ct) { return reinterpret_cast<int*>(ct + H_COLLIDE) + 1; }
__device__ __forceinline__ void earlyPost(double* ct, int state, int lane) {
  if (lane == 0) __hip_atomic_store(earlyFlag(ct), state, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int earlyState(double* ct) {
  return uni(__hip_atomic_load(earlyFlag(ct), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
// spin until pred() (the early hand-off's waits, both waves); false when the
// deadlock guard expired (or was forced at `site`, or the partner failed)
template <class Pred>
__device__ __forceinline__ bool earlyWait(double* ct, Pred pred, int site) {
  if (guardForced(ct, site)) {
    protocolFail(ct);
    return false;
  }
  const long long t0 = spinClock();
  for (int it = 0;; it++) {
    if (pred()) return true;
    if (protocolFailed(ct) || spinExpired(t0, it)) {
      protocolFail(ct);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// the one-row kernel's deferred worlds, bucketed by LCP rows for the wide
// kernel's launch order (largest first; DEFER_BUCKETS in pool_sizes.h)
__device__ __forceinline__ int deferBucket(int m) { return m > 88 ? 0 : (m > 80 ? 1 : (m > 64 ? 2 : 3)); }
// The lists are kept in memory the call owns (the launch's snapshot rows):
// DEFER_BUCKETS counters in the first world's header (SN_DEFERCNT, zeroed by
// the host before the launch), and entry g = q * grid + i (world index) in
// header slot SN_DEFER of world g / 4 -- so concurrent forwards of one world
// handle on different streams never share them.  No header write of a step
// touches these slots.
__device__ __forceinline__ int* deferCount(double* snapBase) {
  return reinterpret_cast<int*>(snapBase + SN_DEFERCNT);
}
__device__ __forceinline__ int* deferEntry(double* snapBase, int snapDoubles, int g) {
  return reinterpret_cast<int*>(snapBase + (size_t)(g >> 2) * snapDoubles + SN_DEFER) + (g & 3);
}

// status bits
#define ST_CONTACT_OVERFLOW 1
#define ST_UNSUPPORTED_SHAPE 2
#define ST_DROPPED_OVERFLOW 4
#define ST_DUPLICATE_COLUMNS 8  // LCPUtils::reduce merged columns (reference behaviour)
#define ST_LCP_TOO_LARGE 16     // more LCP rows than the wave solves (NIMBLE_MAX_SOLVED_LCP)
#define ST_DEFERRED 32          // (internal) the world's LCP has more rows than the one-row-per-lane
                                // kernel takes: the two-rows-per-lane kernel steps it
#define ST_PROTOCOL 64          // a wait between the world's two waves hit the deadlock guard (helperWait)

// wave 0 after a protocol failure (see helperWait): the world's contact step
// is abandoned without reading or writing anything the helper may still
// touch -- the snapshot says no contacts and no rows (the backward and the
// Jacobians see a contact-free step), the warm start is dropped, the status
// raises (ST_PROTOCOL) and the velocity stays the unconstrained v1
__device__ __forceinline__ void protocolAbort(double* snap, double* cache, int lane) {
  if (lane == 0) {
    for (int i = 0; i < SN_DEFER; i++) snap[i] = 0.0;
    snap[SN_STATUS] = ST_PROTOCOL;
    cache[0] = -1.0;
  }
  WSYNC();
}

// row record fields
#define RR_CONTACT 0
#define RR_DIR 1
#define RR_D 2
#define RR_B 5
#define RR_X 6
#define RR_MAP 7
#define RR_CIDX 8
#define RR_UIDX 9
#define RR_EVAL 10
#define RR_BOUNCE 11

// ---------------------------------------------------------------------------
// Narrow phase over the candidate pairs + postProcess dedup + the
// ConstraintSolver::updateConstraints filter.  Kept contacts land at
// ct + CT_CONTACTS in detector order.
// ---------------------------------------------------------------------------
// snapEdge: the world's snapshot slots for the kept contacts' EDGE_EDGE
// metadata (global memory)
// kMeshInline: the mesh-box narrow phase inlined (the helper wave's pass,
// the one that runs on the hot path; the other call sites keep the out-of-
// line instance, so the kernel carries one inlined copy)
template <bool kMeshInline = false>
__device__ __forceinline__ void collideWorld(const ModelDev& md, double* s, const Layout& L, int lane,
                                             double* snapEdge, double* g_stamp = nullptr) {
  (void)g_stamp;
  double* ct = s + L.ct;
  double* dropped = s + L.cscr;                         // clear of the dynamics buffers
  double* pairbuf = dropped + CT_MAX_DROPPED * DROP_REC;
  if (lane == 0) { ct[H_NCON] = 0; ct[H_NDROP] = 0; ct[H_STATUS] = 0; }
  WSYNC();
  const int PC = md.pairChunk;
  for (int p0 = 0; p0 < md.numPairs; p0 += PC) {
    TACC_BEGIN(tNP);
    const int p = p0 + lane;
    if (lane < PC && p < md.numPairs) {
      const int si = md.pairA[p], sj = md.pairB[p];
      const int bi = md.shapeBody[si], bj = md.shapeBody[sj];
      int cnt = 0;
      if (md.shapeType[si] == NIMBLE_SHAPE_BOX && md.shapeType[sj] == NIMBLE_SHAPE_BOX) {
        double T1[12], T2[12];
        tmul(s + L.Tw + 12 * bi, md.shapeT[si], T1);
        tmul(s + L.Tw + 12 * bj, md.shapeT[sj], T2);
        const double R1[9] = {T1[0], T1[1], T1[2], T1[4], T1[5], T1[6], T1[8], T1[9], T1[10]};
        const double R2[9] = {T2[0], T2[1], T2[2], T2[4], T2[5], T2[6], T2[8], T2[9], T2[10]};
        const double p1[3] = {T1[3], T1[7], T1[11]}, p2[3] = {T2[3], T2[7], T2[11]};
        const double A[3] = {0.5 * md.shapeSize[si][0], 0.5 * md.shapeSize[si][1], 0.5 * md.shapeSize[si][2]};
        const double B[3] = {0.5 * md.shapeSize[sj][0], 0.5 * md.shapeSize[sj][1], 0.5 * md.shapeSize[sj][2]};
        cnt = deviceBoxBox(p1, R1, A, p2, R2, B, md.clipDepth, bi, bj, pairbuf + lane * 8 * PBREC);
      } else if ((md.shapeType[si] == NIMBLE_SHAPE_BOX && md.shapeType[sj] == NIMBLE_SHAPE_CAPSULE) ||
                 (md.shapeType[si] == NIMBLE_SHAPE_CAPSULE && md.shapeType[sj] == NIMBLE_SHAPE_BOX)) {
        // collideBoxCapsule / collideCapsuleBox (DARTCollide.cpp:4422, :4533)
        const bool boxFirst = md.shapeType[si] == NIMBLE_SHAPE_BOX;
        const int sb = boxFirst ? si : sj, sc = boxFirst ? sj : si;
        double Tb[12], Tc[12];
        tmul(s + L.Tw + 12 * md.shapeBody[sb], md.shapeT[sb], Tb);
        tmul(s + L.Tw + 12 * md.shapeBody[sc], md.shapeT[sc], Tc);
        int unsup = 0;
        cnt = deviceCapsuleBox(Tb, md.shapeSize[sb], Tc, md.shapeSize[sc][0], md.shapeSize[sc][1], boxFirst,
                               md.clipDepth, bi, bj, sb, pairbuf + lane * 8 * PBREC, &unsup);
        if (unsup) cnt = -1 - cnt;  // flagged; the contacts found are still kept
      } else if (md.shapeType[si] == NIMBLE_SHAPE_CAPSULE && md.shapeType[sj] == NIMBLE_SHAPE_CAPSULE) {
        double T1[12], T2[12];
        tmul(s + L.Tw + 12 * bi, md.shapeT[si], T1);
        tmul(s + L.Tw + 12 * bj, md.shapeT[sj], T2);
        cnt = deviceCapsuleCapsule(T1, md.shapeSize[si][0], md.shapeSize[si][1], T2, md.shapeSize[sj][0],
                                   md.shapeSize[sj][1], md.clipDepth, bi, bj, pairbuf + lane * 8 * PBREC);
      } else if (md.shapeType[si] == NIMBLE_SHAPE_MESH || md.shapeType[sj] == NIMBLE_SHAPE_MESH) {
        cnt = 0;  // narrow-phased by the whole wave below
      } else if (md.shapeType[si] == NIMBLE_SHAPE_SPHERE || md.shapeType[sj] == NIMBLE_SHAPE_SPHERE) {
        const int ti = md.shapeType[si], tj = md.shapeType[sj];
        double T1[12], T2[12];
        tmul(s + L.Tw + 12 * bi, md.shapeT[si], T1);
        tmul(s + L.Tw + 12 * bj, md.shapeT[sj], T2);
        const double c1[3] = {T1[3], T1[7], T1[11]}, c2[3] = {T2[3], T2[7], T2[11]};
        double* out = pairbuf + lane * 8 * PBREC;
        if (ti == NIMBLE_SHAPE_SPHERE && tj == NIMBLE_SHAPE_SPHERE)
          cnt = deviceSphereSphere(c1, md.shapeSize[si][0], c2, md.shapeSize[sj][0], md.clipDepth, bi, bj, out);
        else if (ti == NIMBLE_SHAPE_SPHERE && tj == NIMBLE_SHAPE_BOX)
          cnt = deviceSphereBox(T2, md.shapeSize[sj], c1, md.shapeSize[si][0], false, md.clipDepth, bi, bj, sj, out);
        else if (ti == NIMBLE_SHAPE_BOX && tj == NIMBLE_SHAPE_SPHERE)
          cnt = deviceSphereBox(T1, md.shapeSize[si], c2, md.shapeSize[sj][0], true, md.clipDepth, bi, bj, si, out);
        else if (ti == NIMBLE_SHAPE_SPHERE && tj == NIMBLE_SHAPE_CAPSULE)
          cnt = deviceSphereCapsule(c1, md.shapeSize[si][0], T2, md.shapeSize[sj][0], md.shapeSize[sj][1], true,
                                    md.clipDepth, bi, bj, out);
        else if (ti == NIMBLE_SHAPE_CAPSULE && tj == NIMBLE_SHAPE_SPHERE)
          cnt = deviceSphereCapsule(c2, md.shapeSize[sj][0], T1, md.shapeSize[si][0], md.shapeSize[si][1], false,
                                    md.clipDepth, bi, bj, out);
        else
          cnt = -1;
      } else {
        cnt = -1;
      }
      ct[H_PAIRCNT + lane] = cnt;
    }
    if (md.hasMesh) {
      // a model with mesh pairs takes one pair per chunk; a mesh pair is
      // collided by the whole wave (collideMeshBox / collideBoxMesh)
      WSYNC();
      const int si = md.pairA[p0], sj = md.pairB[p0];
      const int ti = md.shapeType[si], tj = md.shapeType[sj];
      if (ti == NIMBLE_SHAPE_MESH || tj == NIMBLE_SHAPE_MESH) {
        int cnt = -1;  // mesh-sphere / mesh-capsule / mesh-mesh: no collider on this path
        if ((ti == NIMBLE_SHAPE_MESH && tj == NIMBLE_SHAPE_BOX) || (ti == NIMBLE_SHAPE_BOX && tj == NIMBLE_SHAPE_MESH)) {
          const bool meshFirst = ti == NIMBLE_SHAPE_MESH;
          const int sm = meshFirst ? si : sj, sb = meshFirst ? sj : si;
          double Tm[12], Tb[12];
          tmul(s + L.Tw + 12 * md.shapeBody[sm], md.shapeT[sm], Tm);
          tmul(s + L.Tw + 12 * md.shapeBody[sb], md.shapeT[sb], Tb);
          // the mesh's bounding sphere more than 1 mm clear of the box: the
          // convex hull and the box are separated, MPR reports no contact
          double gap2 = 0.0;
          for (int i = 0; i < 3; i++) {
            const double c = (Tm[3] - Tb[3]) * Tb[i] + (Tm[7] - Tb[7]) * Tb[4 + i] + (Tm[11] - Tb[11]) * Tb[8 + i];
            const double h = 0.5 * md.shapeSize[sb][i];
            const double e = c > h ? c - h : (c < -h ? -h - c : 0.0);
            gap2 += e * e;
          }
          const double reach = md.meshRadius[sm] + 1e-3;
          if (gap2 > reach * reach) {
            cnt = 0;
          } else {
            lds_double* mscr = (lds_double*)(pairbuf + pairBufRecs(PC, true) * PBREC);
            if (kMeshInline)
              cnt = meshBoxPair(Tm, md.meshVerts + 3 * md.meshFirst[sm], md.meshCount[sm], md.shapeSize[sm], Tb,
                                md.shapeSize[sb], meshFirst, md.clipDepth, md.shapeBody[si], md.shapeBody[sj],
                                pairbuf, mscr, lane, g_stamp);
            else
              cnt = deviceMeshBox(Tm, md.meshVerts + 3 * md.meshFirst[sm], md.meshCount[sm], md.shapeSize[sm], Tb,
                                  md.shapeSize[sb], meshFirst, md.clipDepth, md.shapeBody[si], md.shapeBody[sj],
                                  pairbuf, mscr, lane);
          }
        }
        if (lane == 0) ct[H_PAIRCNT] = cnt;
      }
    }
    WSYNC();
    TACC_END(76, tNP);
    TACC_BEGIN(tPP);
    // postProcess dedup + filter, lane-parallel over this chunk's candidate
    // points (lane = candidate, detector order) when none of them lies
    // within the dedup distance of an earlier candidate of the chunk; then a
    // candidate is dropped exactly when it is close to an already listed
    // contact, and its kept / dropped list slot is its rank among its kind.
    // Otherwise (or > 64 candidates) the sequential loop below runs.
    bool serial = true;
    {
      const int npc = md.numPairs - p0 < PC ? md.numPairs - p0 : PC;
      int cq = lane < npc ? (int)ct[H_PAIRCNT + lane] : 0;
      const bool unsup = cq < 0;
      if (unsup) cq = -1 - cq;
      const unsigned long long um = __ballot(unsup);
      int incl = cq;
      for (int d = 1; d < 16; d <<= 1) {
        const int t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
      }
      const int total = uni(__shfl(incl, npc > 0 ? npc - 1 : 0));
      const int excl = incl - cq;
      if (total == 0) {
        // no candidate point in this chunk (most pairs of a mesh model, one
        // per chunk): nothing to list; only an unsupported pair's flag
        serial = false;
        if (um && lane == 0) ct[H_STATUS] = (double)((int)ct[H_STATUS] | ST_UNSUPPORTED_SHAPE);
      } else if (npc > 0 && total <= WAVE) {
        serial = false;
        // candidate -> (pair, point)
        int q = 0, exq = 0;
        for (int k = 0; k < npc; k++) {
          const int e0 = rdli(excl, k), e1 = rdli(incl, k);
          if (lane >= e0 && lane < e1) { q = k; exq = e0; }
        }
        const bool live = lane < total;
        const int c = live ? lane - exq : 0;
        const double* rec = pairbuf + (q * 8 + c) * PBREC;
        const double px = live ? rec[0] : 0.0, py = live ? rec[1] : 0.0, pz = live ? rec[2] : 0.0;
        bool dupCand = false;
        for (int j = 0; j < total; j++) {
          const double dx = px - rdl(px, j), dy = py - rdl(py, j), dz = pz - rdl(pz, j);
          double dd = 0;
          dd += dx * dx;
          dd += dy * dy;
          dd += dz * dz;
          if (j < lane && live && sqrt(dd) < 3.0e-12) dupCand = true;
        }
        if (__ballot(dupCand)) {
          serial = true;
        } else {
          const int nk0 = uni((int)ct[H_NCON]), nd0 = uni((int)ct[H_NDROP]);
          bool close = false;
          for (int t = 0; t < nk0 + nd0; t++) {
            const double* o = t < nk0 ? ct + CT_CONTACTS + t * CREC : dropped + (t - nk0) * DROP_REC;
            double dd = 0;
            dd += (px - o[0]) * (px - o[0]);
            dd += (py - o[1]) * (py - o[1]);
            dd += (pz - o[2]) * (pz - o[2]);
            if (sqrt(dd) < 3.0e-12) close = true;
          }
          bool keep = false;
          if (live && !close) {
            const double nn = rec[3] * rec[3] + rec[4] * rec[4] + rec[5] * rec[5];
            const int ba = (int)rec[8], bb = (int)rec[9];
            keep = !(nn < 1e-12) && !(rec[6] < 0.0) && !(rec[6] > md.clipDepth) && (md.reactive[ba] || md.reactive[bb]);
          }
          const bool drop = live && !close && !keep;
          const unsigned long long km = __ballot(keep), dm = __ballot(drop);
          const unsigned long long below = (1ull << lane) - 1ull;
          double* dst = nullptr;
          int len = CREC;
          if (keep) {
            const int idx = nk0 + __popcll(km & below);
            if (idx < md.maxContacts) {
              dst = ct + CT_CONTACTS + idx * CREC;
              if (((int)rec[7] & 15) == CT_EDGE_EDGE || ((int)rec[7] & 15) >= CT_SPHERE_SPHERE)
                for (int i = 0; i < EDGE_REC; i++) snapEdge[idx * EDGE_REC + i] = rec[CREC + i];
            }
          } else if (drop) {
            const int idx = nd0 + __popcll(dm & below);
            if (idx < CT_MAX_DROPPED) dst = dropped + idx * DROP_REC;
            len = DROP_REC;
          }
          if (dst)
            for (int i = 0; i < len; i++) dst[i] = rec[i];
          if (lane == 0) {
            const int nk = nk0 + __popcll(km), nd = nd0 + __popcll(dm);
            int st = (int)ct[H_STATUS];
            if (um) st |= ST_UNSUPPORTED_SHAPE;
            if (nk > md.maxContacts) st |= ST_CONTACT_OVERFLOW;
            if (nd > CT_MAX_DROPPED) st |= ST_DROPPED_OVERFLOW;
            ct[H_NCON] = nk < md.maxContacts ? nk : md.maxContacts;
            ct[H_NDROP] = nd < CT_MAX_DROPPED ? nd : CT_MAX_DROPPED;
            ct[H_STATUS] = st;
          }
        }
      }
    }
    WSYNC();
    if (serial && lane == 0) {
      int nk = (int)ct[H_NCON], nd = (int)ct[H_NDROP], st = (int)ct[H_STATUS];
      for (int q = 0; q < PC && p0 + q < md.numPairs; q++) {
        int cnt = (int)ct[H_PAIRCNT + q];
        if (cnt < 0) { st |= ST_UNSUPPORTED_SHAPE; cnt = -1 - cnt; }
        for (int c = 0; c < cnt; c++) {
          const double* rec = pairbuf + (q * 8 + c) * PBREC;
          bool close = false;
          for (int t = 0; t < nk + nd && !close; t++) {
            const double* o = t < nk ? ct + CT_CONTACTS + t * CREC : dropped + (t - nk) * DROP_REC;
            double dd = 0;
            for (int i = 0; i < 3; i++) dd += (rec[i] - o[i]) * (rec[i] - o[i]);
            if (sqrt(dd) < 3.0e-12) close = true;
          }
          if (close) continue;
          const double nn = rec[3] * rec[3] + rec[4] * rec[4] + rec[5] * rec[5];
          const int ba = (int)rec[8], bb = (int)rec[9];
          const bool keep = !(nn < 1e-12) && !(rec[6] < 0.0) && !(rec[6] > md.clipDepth) &&
                            (md.reactive[ba] || md.reactive[bb]);
          double* dst = nullptr;
          int len = CREC;
          if (keep) {
            if (nk < md.maxContacts) {
              if (((int)rec[7] & 15) == CT_EDGE_EDGE || ((int)rec[7] & 15) >= CT_SPHERE_SPHERE)
                for (int i = 0; i < EDGE_REC; i++) snapEdge[nk * EDGE_REC + i] = rec[CREC + i];
              dst = ct + CT_CONTACTS + (nk++) * CREC;
            } else {
              st |= ST_CONTACT_OVERFLOW;
            }
          } else {
            if (nd < CT_MAX_DROPPED) {
              // keep kept contacts contiguous: the dropped list (positions) is separate
              dst = dropped + (nd++) * DROP_REC;
              len = DROP_REC;
            } else {
              st |= ST_DROPPED_OVERFLOW;
            }
          }
          if (dst)
            for (int i = 0; i < len; i++) dst[i] = rec[i];
        }
      }
      ct[H_NCON] = nk; ct[H_NDROP] = nd; ct[H_STATUS] = st;
    }
    WSYNC();
    TACC_END(77, tPP);
  }
}

// generalized force of a unit impulse along d at contact c (J^T e column entry
// for dof i): sum over the reactive contact bodies of +-S_i . [p x d; d]
__device__ inline double rowForceEntry(const ModelDev& md, const double* s, const Layout& L, const double* rec,
                                       const double* d, int dof) {
  const int body = md.dofBody[dof];
  double wr[6];
  cross3(rec, d, wr);
  wr[3] = d[0]; wr[4] = d[1]; wr[5] = d[2];
  const double sdot = dot6(s + L.Sw + 6 * dof, wr);
  double val = 0.0;
  const int ba = (int)rec[8], bb = (int)rec[9];
  if (md.reactive[ba] && ((md.anc[ba] >> body) & 1ull)) val += sdot;
  if (md.reactive[bb] && ((md.anc[bb] >> body) & 1ull)) val -= sdot;
  return val;
}

// the LCP rows' per-row data and J^T (n x m, row i = dof i): the pool's
struct RowsOut {
  double *cols, *dvec, *lo, *hi, *rest;
  int *fi, *rowC, *rowDir;
};
// rows (ContactConstraint: normal + 2 tangents with friction), lane =
// contact; a contact's first row is its rank among the rows of the contacts
// before it (popcount of the frictional ones).  Then J^T: lane = dof, loop
// over the rows; the row's contact data are wave-uniform (rowForceEntry's
// arithmetic, without a division-based (dof, row) unranking per element).
// `rest` receives the row's restitution coefficient.
__device__ __forceinline__ void buildRows(const ModelDev& md, const double* s, const Layout& L, const double* ct,
                                          int nCon, int m, const RowsOut& O, int lane) {
  const int n = md.n;
  {
    const int c = lane;
    const bool live = c < nCon;
    const double* rec = ct + CT_CONTACTS + (live ? c : 0) * CREC;
    const int ba = (int)rec[8], bb = (int)rec[9];
    const double mu = fmin(md.friction[ba], md.friction[bb]);
    const double restC = md.restitution[ba] * md.restitution[bb];
    const bool fr = live && mu > 1e-3;
    const unsigned long long frm = __ballot(fr);  // (the whole wave: cross-lane ops stay out of divergent code)
    if (live) {
      int r = c + 2 * __popcll(frm & ((1ull << c) - 1ull));
      const int base = r;
      O.rowC[r] = c; O.rowDir[r] = 0;
      for (int i = 0; i < 3; i++) O.dvec[3 * r + i] = rec[3 + i];
      O.lo[r] = 0.0; O.hi[r] = __builtin_inf(); O.fi[r] = -1;
      O.rest[r] = restC > 1e-3 ? restC : 0.0;
      r++;
      if (fr) {
        double t1[3], t2[3];
        tangentBasisODE(rec + 3, t1, t2);
        for (int k = 0; k < 2; k++) {
          O.rowC[r] = c; O.rowDir[r] = 1 + k;
          for (int i = 0; i < 3; i++) O.dvec[3 * r + i] = k == 0 ? t1[i] : t2[i];
          O.lo[r] = -mu; O.hi[r] = mu; O.fi[r] = base; O.rest[r] = 0.0;
          r++;
        }
      }
    }
  }
  WSYNC();
  for (int i = lane; i < n; i += WAVE) {
    const int body = md.dofBody[i];
    double S[6];
    for (int q = 0; q < 6; q++) S[q] = s[L.Sw + 6 * i + q];
    for (int j = 0; j < m; j++) {
      const double* rec = ct + CT_CONTACTS + uni(O.rowC[j]) * CREC;
      const double* d = O.dvec + 3 * j;
      double wr[6];
      cross3(rec, d, wr);
      wr[3] = d[0]; wr[4] = d[1]; wr[5] = d[2];
      const double sdot = dot6(S, wr);
      const int ba = uni((int)rec[8]), bb = uni((int)rec[9]);
      double val = 0.0;
      if (md.reactive[ba] && ((md.anc[ba] >> body) & 1ull)) val += sdot;
      if (md.reactive[bb] && ((md.anc[bb] >> body) & 1ull)) val -= sdot;
      O.cols[i * m + j] = val;
    }
  }
  WSYNC();
}

// b = -J v1 (lane = row; J^T in `cols`)
__device__ __forceinline__ void rowsRhs(const double* cols, const double* v1, double* b, int n, int m, int lane) {
  for (int r = lane; r < m; r += WAVE) {
    double acc = 0;
#pragma unroll 8
    for (int i = 0; i < n; i++) acc += cols[i * m + r] * v1[i];
    b[r] = -acc;
  }
  WSYNC();
}

// Y = L^-1 J^T in place (J^T in Y) by columns (lane = column j): element
// (i, j) receives -L_ik Y_kj for k = 0 .. i-1 in order and is then scaled by
// 1/L_ii -- the same operation sequence as the row-by-row elimination.  Rows
// in blocks of eight with their accumulators in registers: each earlier row
// k (its Y_kj final, loaded once) updates the eight accumulators at once --
// eight independent multiply-adds instead of one dependent chain per row --
// then the block's own triangle in order, its Y values kept in registers.
// Every element still sees its k terms in ascending order, so the same bits
// as the row-at-a-time loop (which waited on each row's stored Y before the
// next row's loads: ~33k clocks for the Atlas LCP's 33 x 24).
// (Jt: J^T, n x m; Y: the result, in place when Y == Jt)
__device__ __forceinline__ void formYWide(double* Y, const double* Jt, const double* Lm, const double* dinv, int n,
                                          int m, int lane) {
  for (int j = lane; j < m; j += WAVE) {
    for (int i0 = 0; i0 < n; i0 += 8) {
      double acc[8], yb[8];
      // (rows past n: clamped to row n - 1, their results unused)
      int ro[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int i = i0 + u < n ? i0 + u : n - 1;
        ro[u] = tri(i, 0);
        acc[u] = Jt[i * m + j];
      }
      // (four rows k per pass: their 36 loads issued before the 32
      // multiply-adds, so the LDS latency is paid once per pass; i0 is a
      // multiple of 8)
      for (int k = 0; k < i0; k += 4) {
        double yv[4], lv[4][8];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          yv[q] = Y[(k + q) * m + j];
#pragma unroll
          for (int u = 0; u < 8; u++) lv[q][u] = Lm[ro[u] + k + q];
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
          asm volatile("" : "+v"(yv[q]));
#pragma unroll
          for (int u = 0; u < 8; u++) asm volatile("" : "+v"(lv[q][u]));
        }
#pragma unroll
        for (int q = 0; q < 4; q++)
#pragma unroll
          for (int u = 0; u < 8; u++) acc[u] -= lv[q][u] * yv[q];
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        if (i0 + u < n) {
#pragma unroll
          for (int v = 0; v < u; v++) acc[u] -= Lm[ro[u] + i0 + v] * yb[v];
          yb[u] = acc[u] * dinv[i0 + u];
          Y[(i0 + u) * m + j] = yb[u];
        }
      }
    }
  }
  WSYNC();
}

// Up to 32 columns: the wave's two halves share each 8-row block, lane = 32 h
// + column, half h holding rows i0 + 4 h .. i0 + 4 h + 3 -- half the
// accumulators and L loads per earlier row.  The block's triangle: half 0's
// four rows, then half 1's (their terms from half 0's rows first, through
// LDS), each element's terms still in ascending k.
__device__ __forceinline__ void formY(double* Y, const double* Jt, const double* Lm, const double* dinv, int n, int m,
                                      int lane) {
  if (m > 32) {
    formYWide(Y, Jt, Lm, dinv, n, m, lane);
    return;
  }
  const int h = lane >> 5, j = lane & 31;
  const bool live = j < m;
  const int jc = live ? j : 0;
  for (int i0 = 0; i0 < n; i0 += 8) {
    double acc[4], yb[4];
    int ro[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int r = i0 + 4 * h + u;
      const int i = r < n ? r : n - 1;  // (rows past n: clamped, results unused)
      ro[u] = tri(i, 0);
      acc[u] = Jt[i * m + jc];
    }
    // rows before the block, four per pass (i0 is a multiple of 8)
    for (int k = 0; k < i0; k += 4) {
      double yv[4], lv[4][4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        yv[q] = Y[(k + q) * m + jc];
#pragma unroll
        for (int u = 0; u < 4; u++) lv[q][u] = Lm[ro[u] + k + q];
      }
#pragma unroll
      for (int q = 0; q < 4; q++) {
        asm volatile("" : "+v"(yv[q]));
#pragma unroll
        for (int u = 0; u < 4; u++) asm volatile("" : "+v"(lv[q][u]));
      }
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int u = 0; u < 4; u++) acc[u] -= lv[q][u] * yv[q];
    }
    // half 0's rows
    if (h == 0) {
#pragma unroll
      for (int u = 0; u < 4; u++) {
        if (i0 + u < n) {
#pragma unroll
          for (int v = 0; v < u; v++) acc[u] -= Lm[ro[u] + i0 + v] * yb[v];
          yb[u] = acc[u] * dinv[i0 + u];
          if (live) Y[(i0 + u) * m + j] = yb[u];
        }
      }
    }
    WSYNC();
    // half 1's rows: half 0's four rows' terms, then their own triangle
    if (h == 1 && i0 + 4 < n) {
      double y0[4];
#pragma unroll
      for (int q = 0; q < 4; q++) y0[q] = Y[(i0 + q) * m + jc];
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int u = 0; u < 4; u++) acc[u] -= Lm[ro[u] + i0 + q] * y0[q];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        if (i0 + 4 + u < n) {
#pragma unroll
          for (int v = 0; v < u; v++) acc[u] -= Lm[ro[u] + i0 + 4 + v] * yb[v];
          yb[u] = acc[u] * dinv[i0 + 4 + u];
          if (live) Y[(i0 + 4 + u) * m + j] = yb[u];
        }
      }
    }
    WSYNC();
  }
}

// ---------------------------------------------------------------------------
// ConstrainedGroupGradientMatrices::constructMatrices (:482) followed by
// opportunisticallyStandardizeResults (:218), iterated while the
// standardisation makes rows newly not-clamping (the reference recurses).
// Q = A_cc + A_cu E + cfm I  (== A_c^T Minv A_c_ub_E + cfm I).
// Returns the standardized flag (wave-uniform).
// ---------------------------------------------------------------------------
// COD factorisation of a matrix in the HBM workspace (worlds whose LCP pool
// is off chip: the wide kernels, > 64 rows) staged through the workgroup's
// LDS when the launch provides a stage (Layout::stage / stageCap, see capi.cpp:
// the pool area, idle in those kernels, extended for the model's largest
// clamping set): the matrix and the COD workspace are copied in, factorised by
// the LDS code (the same arithmetic, so the same factor bit for bit) and
// copied back.  Each step of the factorisation reads its trailing columns
// from LDS instead of L2 / HBM (~5M -> well under 1M clocks at 96 x 96).
template <bool kLds, int R>
__device__ __forceinline__ void codFactorAny(typename Space<kLds>::dptr A, typename Space<kLds>::dptr ws, int m, int n,
                                             int ld, typename Space<kLds>::dptr v, int lane, lds_double* stage,
                                             int stageCap, double* prof = nullptr) {
  m = uni(m);
  n = uni(n);
  ld = uni(ld);
  const int mx = m > n ? m : n;
  const int wsd = 4 * mx + (mx + 1) / 2 + 3;  // carveCod: vd vn zd zn perm rank
  if (kLds || stage == nullptr || m * ld + wsd + mx > stageCap) {
    codFactorR<kLds, R>(A, ws, m, n, ld, v, lane, prof);
    return;
  }
  double* gA = (double*)A;
  double* gW = (double*)ws;
  double* sA = (double*)stage;
  double* sW = sA + m * ld;
  double* sV = sW + wsd;
  for (int t = lane; t < m * ld; t += WAVE) sA[t] = gA[t];
  for (int t = lane; t < wsd; t += WAVE) sW[t] = gW[t];
  WSYNC();
  codFactorR<true, R>(sp<true>(sA), sp<true>(sW), m, n, ld, sp<true>(sV), lane, prof);
  WSYNC();
  for (int t = lane; t < m * ld; t += WAVE) gA[t] = sA[t];
  for (int t = lane; t < wsd; t += WAVE) gW[t] = sW[t];
  WSYNC();
}

// postDz > 0 (the wide kernel's first classification, task not yet posted):
// once the classification's size n_c is known, the task board's Dantzig task
// goes out here if the factor of this n_c still fits the stage after
// Dantzig's postDz doubles at its head (the helper then runs Dantzig beside
// this classification); whether it went out: helperState(ct) != HS_IDLE.
// kK: which forward kernel calls (0 the one-row kernel, 1 the wide one): a
// separate instance per kernel -- one instance reached from both kernels was
// compiled with callee-saved register spills on entry (16 -> 464 B/lane of
// scratch per call, forward writes ~25 -> ~85 KB/world measured)
template <bool kLds, int R = 1, int kK = 0>
__device__ bool devConstruct(typename Space<kLds>::dptr poolIn, int m, int n, double cfm, bool ignoreFriction,
                             lds_double* ctIn, int lane, double* g_stamp = nullptr, lds_double* stage = nullptr,
                             int stageCap = 0, int postDz = 0) {
  (void)g_stamp;
  FwdPool P;
  carveFwd((double*)poolIn, m, n, P);
  double* ct = (double*)ctIn;
  for (int guard = 0; guard <= m + 1; guard++) {
    TACC_BEGIN(tCls);
#ifdef NIMBLE_STAGE_TIMING
    if (lane == 0 && g_stamp) g_stamp[60] += 1;
#endif
    // Row-parallel classification (row j < m on lane j & 63, slot j >> 6).
    // Whether a row clamps depends on its own data and X[findex] only; a
    // row bounded by its friction parent additionally needs the parent's
    // clamping flag (ballot bit), and the clamping / upper-bound indices are
    // the rows' ranks among their kind (popcounts), which is the sequential
    // loop's numbering.
    {
      const double TH = 1e-6, tie = 1e-5;
      bool clampR[R], ubCand[R], live[R];
      double f[R], hiJ[R], loJ[R], up[R], low[R];
      int fp[R];
      unsigned long long cm[R], um[R];
#pragma unroll
      for (int s = 0; s < R; s++) {
        const int j = rowAt(s, lane);
        live[s] = j < m;
        f[s] = live[s] ? P.X[j] : 0.0;
        hiJ[s] = live[s] ? P.hi[j] : 0.0;
        loJ[s] = live[s] ? P.lo[j] : 0.0;
        fp[s] = live[s] ? P.fi[j] : -1;
        const bool colOk = live[s] && P.aCol[j] >= 1e-9;
        const double xfp = (live[s] && fp[s] != -1) ? P.X[fp[s]] : 1.0;
        up[s] = hiJ[s] * xfp;
        low[s] = loJ[s] * xfp;
        clampR[s] = false;
        ubCand[s] = false;
        if (colOk) {
          if (fabs(f[s]) < TH) {
            clampR[s] = fp[s] != -1 && !(fabs(xfp) < TH) && !ignoreFriction;
          } else if ((f[s] > low[s] + tie && f[s] < up[s] - tie) || (low[s] - f[s] > 1e-2 || f[s] - up[s] > 1e-2)) {
            clampR[s] = true;
          } else if (fp[s] != -1 && fabs(xfp) > 1e-9 && P.aCol[fp[s]] > 1e-9) {
            ubCand[s] = true;
          }
        }
        cm[s] = __ballot(clampR[s]);
      }
      bool ubR[R];
#pragma unroll
      for (int s = 0; s < R; s++) {
        ubR[s] = ubCand[s] && (fp[s] > rowAt(s, lane) || bitR(cm, fp[s] >= 0 ? fp[s] : 0));
        um[s] = __ballot(ubR[s]);
      }
#pragma unroll
      for (int s = 0; s < R; s++) {
        const int j = rowAt(s, lane);
        const int cIdx = clampR[s] ? rankR(cm, j) : -1;
        const int uIdx = ubR[s] ? rankR(um, j) : -1;
        if (live[s]) {
          P.mapping[j] = clampR[s] ? CM_CLAMPING : (ubR[s] ? fp[s] : CM_NOT_CLAMPING);
          P.clampIdx[j] = cIdx;
          P.ubIdx[j] = uIdx;
          P.Eval[j] = ubR[s] ? (fabs(f[s] - up[s]) < fabs(f[s] - low[s]) ? hiJ[s] : loJ[s]) : 0.0;
          if (clampR[s]) {
            P.fc[cIdx] = f[s];
            P.relVel[cIdx] = P.b[j];
            P.clampRow[cIdx] = j;
          }
        }
      }
      if (lane == 0) { ct[H_NC] = popR(cm); ct[H_NU] = popR(um); }
    }
    WSYNC();
    TACC_END(61, tCls);
    const int nc = uni((int)ct[H_NC]);
    if (postDz > 0 && guard == 0 && nc > 0 && nc * nc + 4 * nc + (nc + 1) / 2 + 3 + nc + postDz <= stageCap) {
      boardPost(ct, HB_WIDE, true, lane);
      stage += postDz;
      stageCap -= postDz;
    }
    double bR[R], hiR[R], loR[R];
    int fiR[R];
#pragma unroll
    for (int s = 0; s < R; s++) {
      const int j = rowAt(s, lane);
      bR[s] = j < m ? P.b[j] : 0.0;
      hiR[s] = j < m ? P.hi[j] : 0.0;
      loR[s] = j < m ? P.lo[j] : 0.0;
      fiR[s] = j < m ? P.fi[j] : -1;
    }
    if (nc == 0) {
      double zero[R];
#pragma unroll
      for (int s = 0; s < R; s++) zero[s] = 0.0;
      const bool ok = waveLcpValidR<kLds, R>(m, spc<kLds>(P.A), cfm, zero, bR, hiR, loR, fiR, ignoreFriction, lane);
      if (ok)
#pragma unroll
        for (int s = 0; s < R; s++)
          if (rowAt(s, lane) < m) P.X[rowAt(s, lane)] = 0.0;
      WSYNC();
      return ok;
    }
    STAMP(40);
    TACC_BEGIN(tQ);
    // Q (nc x nc) into M1
    double* Q = P.M1;
    for (int t = lane; t < nc * nc; t += WAVE) {
      const int cr = t / nc, cc = t % nc;
      const int rr = P.clampRow[cr], rc = P.clampRow[cc];
      double v = P.A[rr * m + rc];
      // upper-bound rows feeding clamping column cc are the friction rows of
      // its contact (rows rc+1, rc+2) whose findex is rc
      for (int u = rc + 1; u <= rc + 2 && u < m; u++)
        if (P.mapping[u] == rc) v += P.Eval[u] * P.A[rr * m + u];
      if (cr == cc) v += cfm;
      Q[t] = v;
    }
    WSYNC();
    Cod cod;
    double* w = carveCod(P.scr, Q, nc, nc, nc, cod);
    double* cn = w; w += m;
    double* vv = w; w += m;
    double* rhs = w; w += m;
    double* z = w; w += m;
    (void)cn;
    STAMP(41);
    TACC_END(62, tQ);
    TACC_BEGIN(tF);
#ifdef NIMBLE_STAGE_TIMING
    codFactorAny<kLds, R>(sp<kLds>(Q), sp<kLds>(P.scr), nc, nc, nc, sp<kLds>(vv), lane, stage, stageCap,
                          g_stamp ? g_stamp + SLOT_COD : nullptr);
#else
    codFactorAny<kLds, R>(sp<kLds>(Q), sp<kLds>(P.scr), nc, nc, nc, sp<kLds>(vv), lane, stage, stageCap);
#endif
    if (lane == 0) ct[H_CODOK] = 1;
    STAMP(42);
    TACC_END(63, tF);
    TACC_BEGIN(tS);
    {
      double rv[R], fs[R];
#pragma unroll
      for (int s = 0; s < R; s++) rv[s] = rowAt(s, lane) < nc ? P.relVel[rowAt(s, lane)] : 0.0;
      codSolveWaveR<kLds, R>(sp<kLds>(Q), sp<kLds>(P.scr), nc, nc, nc, rv, sp<kLds>(z), lane, fs);
#pragma unroll
      for (int s = 0; s < R; s++)
        if (rowAt(s, lane) < nc) P.fsol[rowAt(s, lane)] = fs[s];
    }
    STAMP(43);
    TACC_END(64, tS);
    TACC_BEGIN(tN);
    (void)rhs;
    WSYNC();
    double nxR[R];
    {
      // row-parallel: new x from the clamping solution
      bool newlyNot = false;
#pragma unroll
      for (int s = 0; s < R; s++) {
        const int j = rowAt(s, lane);
        nxR[s] = 0.0;
        if (j < m) {
          double v = 0.0;
          const int ci = P.clampIdx[j];
          if (ci != -1) {
            v = P.fsol[ci];
            newlyNot = newlyNot || (fabs(v) < 1e-6 && fabs(P.X[j]) > 1e-6 && P.fi[j] == -1);
          }
          if (P.ubIdx[j] != -1) {
            const int pc = P.clampIdx[P.fi[j]];
            const double hiJ = P.hi[j], loJ = P.lo[j];
            const double om = P.fc[pc] / P.X[j];
            v = P.fsol[pc] * (fabs(om - hiJ) < fabs(om - loJ) ? hiJ : loJ);
          }
          P.nx[j] = v;
          nxR[s] = v;
        }
      }
      const bool anyNewlyNot = __ballot(newlyNot) != 0ull;
      if (lane == 0) ct[H_FLAG] = anyNewlyNot ? 1 : 0;
    }
    WSYNC();
    TACC_END(65, tN);
    TACC_BEGIN(tV);
    const bool ok = waveLcpValidR<kLds, R>(m, spc<kLds>(P.A), cfm, nxR, bR, hiR, loR, fiR, ignoreFriction, lane);
    const int res = ok ? (uni((int)ct[H_FLAG]) ? 2 : 1) : 0;
    STAMP(44);
    TACC_END(66, tV);
    if (ok) {
#pragma unroll
      for (int s = 0; s < R; s++) {
        const int j = rowAt(s, lane);
        if (j < m) P.X[j] = P.nx[j];
        if (j < nc) P.fc[j] = P.fsol[j];
      }
    }
    WSYNC();
    if (res != 2) return res != 0;
  }
  return false;
}

// guessSolution (LCPUtils.cpp:69): COD solve on {normal rows with b > 0} U
// {friction rows}; result into x.
template <bool kLds, int R = 1, int kK = 0>  // (kK: as devConstruct)
__device__ void devGuess(typename Space<kLds>::dptr poolIn, int m, int n, lds_double* ctIn, int lane,
                         lds_double* stage = nullptr, int stageCap = 0) {
  FwdPool P;
  carveFwd((double*)poolIn, m, n, P);
  double* ct = (double*)ctIn;
  double* x = P.X;
  if (lane == 0) {
    int k = 0;
    for (int i = 0; i < m; i++) {
      if (P.fi[i] == -1) { if (P.b[i] > 0) P.cl[k++] = i; }
      else P.cl[k++] = i;
    }
    ct[H_K] = k;
  }
  WSYNC();
  const int k = uni((int)ct[H_K]);
  for (int i = lane; i < m; i += WAVE) x[i] = 0.0;
  if (k == 0) { WSYNC(); return; }
  double* Ar = P.M1;
  for (int t = lane; t < k * k; t += WAVE) Ar[t] = P.A[P.cl[t / k] * m + P.cl[t % k]];
  WSYNC();
  Cod cod;
  double* w = carveCod(P.scr, Ar, k, k, k, cod);
  double* cn = w; w += m;
  double* vv = w; w += m;
  double* rhs = w; w += m;
  double* z = w; w += m;
  double* xr = w; w += m;
  (void)cn;
  codFactorAny<kLds, R>(sp<kLds>(Ar), sp<kLds>(P.scr), k, k, k, sp<kLds>(vv), lane, stage, stageCap);
  {
    double rv[R], xo[R];
#pragma unroll
    for (int s = 0; s < R; s++) rv[s] = rowAt(s, lane) < k ? P.b[P.cl[rowAt(s, lane)]] : 0.0;
    codSolveWaveR<kLds, R>(sp<kLds>(Ar), sp<kLds>(P.scr), k, k, k, rv, sp<kLds>(z), lane, xo);
#pragma unroll
    for (int s = 0; s < R; s++)
      if (rowAt(s, lane) < k) x[P.cl[rowAt(s, lane)]] = xo[s];
  }
  (void)rhs; (void)xr;
  WSYNC();
}

// pinv(Q) from its COD factor `c` (factor, workspace and Z in LDS: the wide
// kernels' stage), 64 columns per pass, lane = column: Z[i * 65 + lane] is
// the column's right-hand side (row stride 65: the transposed write-back
// below reads it conflict-free).  Per column the same operations in the same
// order as the per-lane solve of backwardPrecompute's off-stage path (Q^T
// reflectors, back substitution on T, Z^T reflectors), so the results are
// bit for bit those.  Writes pinv(Q)^T rows to PTG (row col = column col of
// pinv(Q), permuted) and the solves z_c to Zs (row c, for the imprecision
// map), both in HBM.
__device__ __forceinline__ void pinvColumnsStaged(const lds_double* F, const lds_double* W, lds_double* Z, int nc,
                                                  double* PTG, double* Zs, int lane) {
  // the COD workspace as carveCod lays it out (vd vn zd zn perm rank), typed
  // as LDS so that every access below is an LDS instruction
  const lds_double* vdA = W;
  const lds_double* vnA = W + nc;
  const lds_double* zdA = W + 2 * nc;
  const lds_double* znA = W + 3 * nc;
  const lds_int* perm = (const lds_int*)(W + 4 * nc);
  const lds_int* rankP = (const lds_int*)(W + 4 * nc + (nc + 1) / 2 + 1);
  const int kmax = nc;
  const int r = uni(*rankP);
  for (int c0 = 0; c0 < nc; c0 += WAVE) {
    const int col = c0 + lane;
    const int cnt = nc - c0 < WAVE ? nc - c0 : WAVE;
    for (int i = 0; i < nc; i++) Z[i * 65 + lane] = i == col ? 1.0 : 0.0;
    WSYNC();
    lds_double* z = Z + lane;
    for (int k = 0; k < kmax; k++) {
      const double vnorm = unid(vnA[k]);
      if (!(vnorm > 0)) continue;
      const double vd = unid(vdA[k]);
      double sc = vd * z[k * 65];
      int i = k + 1;
      for (; i + 8 <= nc; i += 8) {
        double fv[8], zv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) { fv[u] = F[(i + u) * nc + k]; zv[u] = z[(i + u) * 65]; }
#pragma unroll
        for (int u = 0; u < 8; u++) asm volatile("" : "+v"(fv[u]), "+v"(zv[u]));
#pragma unroll
        for (int u = 0; u < 8; u++) sc += fv[u] * zv[u];
      }
      for (; i < nc; i++) sc += F[i * nc + k] * z[i * 65];
      sc = 2 * sc / vnorm;
      z[k * 65] -= sc * vd;
      // (eight elements' loads issued before their stores: the compiler cannot
      // tell Z from F, and would otherwise order every load after the
      // previous element's store -- one LDS round trip per element)
      for (i = k + 1; i + 8 <= nc; i += 8) {
        double fv[8], zv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) { fv[u] = F[(i + u) * nc + k]; zv[u] = z[(i + u) * 65]; }
#pragma unroll
        for (int u = 0; u < 8; u++) asm volatile("" : "+v"(fv[u]), "+v"(zv[u]));
#pragma unroll
        for (int u = 0; u < 8; u++) z[(i + u) * 65] = zv[u] - sc * fv[u];
      }
      for (; i < nc; i++) z[i * 65] -= sc * F[i * nc + k];
    }
    for (int i = r - 1; i >= 0; i--) {
      double sc = z[i * 65];
      for (int j = i + 1; j < r; j++) sc -= F[i * nc + j] * z[j * 65];
      z[i * 65] = sc / F[i * nc + i];
    }
    for (int j = r; j < nc; j++) z[j * 65] = 0.0;
    for (int i = 0; i < r && r < nc; i++) {
      const double vn = unid(znA[i]);
      if (vn == 0) continue;
      const double zd = unid(zdA[i]);
      double sc = z[i * 65] * zd;
      for (int j = r; j < nc; j++) sc += z[j * 65] * F[i * nc + j];
      sc = 2 * sc / vn;
      z[i * 65] -= sc * zd;
      for (int j = r; j < nc; j++) z[j * 65] -= sc * F[i * nc + j];
    }
    WSYNC();
    // write-back, lane-contiguous in HBM: element t of the chunk is column
    // c0 + t / nc, row t % nc
    for (int t = lane; t < cnt * nc; t += WAVE) {
      const int j = t / nc, i = t - j * nc;
      const double v = Z[i * 65 + j];
      Zs[(size_t)c0 * nc + t] = v;
      PTG[(size_t)(c0 + j) * nc + perm[i]] = v;
    }
    WSYNC();
  }
}

// pinv(Q) from its COD factor as blocked products on the matrix cores, 64
// right-hand-side columns per pass (the stage layout of pinvColumnsStaged,
// plus 512 doubles at Tb for a block's 16 x 16 Gram matrix and triangular
// factor) -- the same three steps as the per-column solves, reorganised:
//   X = Q_h^T [e_c0 .. e_c0+63]: the QR reflectors sixteen at a time as one
//     block reflector I - V T V^T (T from the Gram matrix V^T V by LAPACK
//     dlarft's columnwise recurrence), applied as X -= V (T^T (V^T X)):
//     three v_mfma_f64_16x16x4f64 products;
//   Y = T^-1 X on the leading r rows (r = rank; the rows below are 0): block
//     back substitution, the 16 x 16 diagonal blocks solved lane-per-column,
//     the blocks above updated by MFMA products;
//   for r < n_c the RZ reflectors Z^T (reflector i over {i} U {r .. n_c-1})
//     as block reflectors in the same way.
// The results equal the per-column solves' up to the rounding of the
// reordered sums.  The per-column form is lane-serial over n_c^2 steps
// (~1.5M clocks at n_c = 93 on the mesh Atlas' flat-foot worlds).
// MFMA operand layout (as gramMfma): A / B lane l = row / column l % 16 of
// the tile, k = l / 16; result element e of lane l = row l / 16 + 4 e,
// column l % 16 -- so a product's result feeds the next product's B operand
// directly (its element s is B's k-step s).  All 64 lanes active.
template <class VFn, class TauFn>
__device__ __forceinline__ void blockReflect(VFn Vfn, TauFn tau, int k0, int kRow0, int nc, lds_double* Z,
                                             lds_double* G, lds_double* T, lds_double* Pn, int lane) {
  // applies H_{k0+15} .. H_{k0} (H_k = I - tau_k v_k v_k^T, v_k = V(., k),
  // zero outside rows >= kRow0) to the nc x 64 block Z (row stride 65).
  // Pn (optional): a 16 * NB x 17 LDS panel the block's sixteen reflectors
  // are first expanded into (zeros included), so that every MFMA operand is
  // one LDS read instead of the masked element function
  const int i16 = lane & 15, kq = lane >> 4;
  const int NB = (nc + 15) >> 4;
  const int kStart = kRow0 & ~3;
  if (Pn != nullptr) {
    for (int t = kStart * 16 + lane; t < NB * 256; t += WAVE) {
      const int i = t >> 4, j = t & 15;
      Pn[i * 17 + j] = Vfn(i, k0 + j);
    }
    WSYNC();
  }
  auto V = [&](int i, int k) -> double { return Pn != nullptr ? Pn[i * 17 + (k - k0)] : Vfn(i, k); };
  // (independent accumulator chains throughout: a chain of dependent MFMAs
  // runs at the instruction's latency, independent ones at its issue rate)
  {
    nimble_double4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
    int k = kStart;
    for (; k + 4 < nc; k += 8) {
      const double a0 = V(k + kq, k0 + i16), a1 = V(k + 4 + kq, k0 + i16);
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, a0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, a1, acc1, 0, 0, 0);
    }
    if (k < nc) {
      const double a0 = V(k + kq, k0 + i16);
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, a0, acc0, 0, 0, 0);
    }
#pragma unroll
    for (int e = 0; e < 4; e++) G[(kq + 4 * e) * 16 + i16] = acc0[e] + acc1[e];
  }
  WSYNC();
  // T: lane i < 16 computes row i: T_ii = tau_i, T_ij = -tau_j sum_{k=i}^{j-1} T_ik G_kj
  if (lane < 16) {
    double t[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const double tj = tau(k0 + j);
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < j; k++) acc += (k >= lane ? t[k] : 0.0) * G[k * 16 + j];
      t[j] = j < lane ? 0.0 : (j == lane ? tj : -tj * acc);
    }
#pragma unroll
    for (int j = 0; j < 16; j++) T[lane * 16 + j] = t[j];
  }
  WSYNC();
  // W = V^T Z (16 x 64, four column tiles), W2 = T^T W, Z -= V W2
  nimble_double4 w[4], w2[4];
#pragma unroll
  for (int ct = 0; ct < 4; ct++) w[ct] = nimble_double4{0.0, 0.0, 0.0, 0.0};
  for (int k = kStart; k < nc; k += 4) {
    const int row = k + kq;
    const double a = V(row, k0 + i16);
    double bv[4];
#pragma unroll
    for (int ct = 0; ct < 4; ct++) {
      const double zv = Z[(row < nc ? row : nc - 1) * 65 + ct * 16 + i16];
      bv[ct] = row < nc ? zv : 0.0;
    }
#pragma unroll
    for (int ct = 0; ct < 4; ct++) w[ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bv[ct], w[ct], 0, 0, 0);
  }
#pragma unroll
  for (int ct = 0; ct < 4; ct++) w2[ct] = nimble_double4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s2 = 0; s2 < 4; s2++) {
    const double ta = T[(kq + 4 * s2) * 16 + i16];
#pragma unroll
    for (int ct = 0; ct < 4; ct++) w2[ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(ta, w[ct][s2], w2[ct], 0, 0, 0);
  }
  for (int rt = kRow0 >> 4; rt < NB; rt++) {
    const int r0 = rt * 16;
    double vrow[4];
#pragma unroll
    for (int s2 = 0; s2 < 4; s2++) vrow[s2] = -V(r0 + i16, k0 + kq + 4 * s2);
    nimble_double4 acc[4];
#pragma unroll
    for (int ct = 0; ct < 4; ct++)
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int row = r0 + kq + 4 * e;
        const double zv = Z[(row < nc ? row : nc - 1) * 65 + ct * 16 + i16];
        acc[ct][e] = row < nc ? zv : 0.0;
      }
#pragma unroll
    for (int s2 = 0; s2 < 4; s2++)
#pragma unroll
      for (int ct = 0; ct < 4; ct++)
        acc[ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(vrow[s2], w2[ct][s2], acc[ct], 0, 0, 0);
#pragma unroll
    for (int ct = 0; ct < 4; ct++)
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int row = r0 + kq + 4 * e;
        if (row < nc) Z[row * 65 + ct * 16 + i16] = acc[ct][e];
      }
  }
  WSYNC();
}

__device__ __forceinline__ void pinvColumnsMfma(const lds_double* F, const lds_double* W, lds_double* Z,
                                                lds_double* Tb, lds_double* Pn, int nc, double* PTG, double* Zs,
                                                int lane) {
  const lds_double* vdA = W;
  const lds_double* vnA = W + nc;
  const lds_double* zdA = W + 2 * nc;
  const lds_double* znA = W + 3 * nc;
  const lds_int* perm = (const lds_int*)(W + 4 * nc);
  const lds_int* rankP = (const lds_int*)(W + 4 * nc + (nc + 1) / 2 + 1);
  const int r = uni(*rankP);
  const int i16 = lane & 15, kq = lane >> 4;
  const int NB = (nc + 15) >> 4, NBr = (r + 15) >> 4;
  lds_double* G = Tb;        // 16 x 16 Gram matrix of a block's reflectors
  lds_double* T = Tb + 256;  // 16 x 16 upper-triangular block factor
  // QR reflector k's element i (0 above its head; skipped reflectors: 0)
  auto Vq = [&](int i, int k) -> double {
    if (k >= nc || i >= nc || i < k) return 0.0;
    if (!(vnA[k] > 0)) return 0.0;
    return i == k ? vdA[k] : F[i * nc + k];
  };
  auto tauQ = [&](int k) -> double {
    const double vn = k < nc ? vnA[k] : 0.0;
    return vn > 0 ? 2.0 / vn : 0.0;
  };
  // RZ reflector k (k < r): head zd_k at row k, tail F[k][r ..] at rows r ..
  auto Vz = [&](int i, int k) -> double {
    if (k >= r || i >= nc) return 0.0;
    if (znA[k] == 0) return 0.0;
    return i == k ? zdA[k] : (i >= r ? F[k * nc + i] : 0.0);
  };
  auto tauZ = [&](int k) -> double {
    const double vn = k < r ? znA[k] : 0.0;
    return vn != 0 ? 2.0 / vn : 0.0;
  };
  for (int c0 = 0; c0 < nc; c0 += WAVE) {
    const int cnt = nc - c0 < WAVE ? nc - c0 : WAVE;
    for (int i = 0; i < nc; i++) Z[i * 65 + lane] = i == c0 + lane ? 1.0 : 0.0;
    WSYNC();
    // ---- X = Q_h^T X
    for (int b = 0; b < NB; b++) blockReflect(Vq, tauQ, b * 16, b * 16, nc, Z, G, T, Pn, lane);
    // ---- rows r .. n_c - 1 are 0; Y = T^-1 X on rows 0 .. r - 1, from the bottom
    for (int i = r; i < nc; i++) Z[i * 65 + lane] = 0.0;
    WSYNC();
    for (int rb = NBr - 1; rb >= 0; rb--) {
      const int r0 = rb * 16;
      const int r1 = (r0 + 16 < r ? r0 + 16 : r) - 1;
      {
        double y[16];
#pragma unroll
        for (int u = 15; u >= 0; u--) {
          const int i = r0 + u;
          double acc = i <= r1 ? Z[i * 65 + lane] : 0.0;
#pragma unroll
          for (int v2 = u + 1; v2 < 16; v2++)
            if (r0 + v2 <= r1) acc -= F[i * nc + r0 + v2] * y[v2];
          y[u] = i <= r1 ? acc / F[i * nc + i] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 16; u++)
          if (r0 + u <= r1) Z[(r0 + u) * 65 + lane] = y[u];
      }
      WSYNC();
      // the blocks above: X_rt -= T[rt, rb] Y_rb
      for (int rt = 0; rt < rb; rt++) {
        const int q0 = rt * 16;
        double rrow[4];
#pragma unroll
        for (int s2 = 0; s2 < 4; s2++) {
          const int col = r0 + kq + 4 * s2;
          const double fv = F[(q0 + i16) * nc + (col <= r1 ? col : r1)];
          rrow[s2] = col <= r1 ? -fv : 0.0;
        }
        nimble_double4 acc[4];
#pragma unroll
        for (int ct = 0; ct < 4; ct++)
#pragma unroll
          for (int e = 0; e < 4; e++) acc[ct][e] = Z[(q0 + kq + 4 * e) * 65 + ct * 16 + i16];
#pragma unroll
        for (int s2 = 0; s2 < 4; s2++) {
          const int row = r0 + kq + 4 * s2;
#pragma unroll
          for (int ct = 0; ct < 4; ct++) {
            const double yz = Z[(row <= r1 ? row : r1) * 65 + ct * 16 + i16];
            acc[ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(rrow[s2], row <= r1 ? yz : 0.0, acc[ct], 0, 0, 0);
          }
        }
#pragma unroll
        for (int ct = 0; ct < 4; ct++)
#pragma unroll
          for (int e = 0; e < 4; e++) Z[(q0 + kq + 4 * e) * 65 + ct * 16 + i16] = acc[ct][e];
      }
      WSYNC();
    }
    // ---- Z^T (the RZ reflectors, reflector 0 first)
    if (r < nc)
      for (int b = 0; b < NBr; b++) blockReflect(Vz, tauZ, b * 16, b * 16, nc, Z, G, T, Pn, lane);
    // write-back, lane-contiguous in HBM (as pinvColumnsStaged)
    for (int t = lane; t < cnt * nc; t += WAVE) {
      const int j = t / nc, i = t - j * nc;
      const double v = Z[i * 65 + j];
      Zs[(size_t)c0 * nc + t] = v;
      PTG[(size_t)(c0 + j) * nc + perm[i]] = v;
    }
    WSYNC();
  }
}

// The upstream-gradient-independent pieces of the constrained backward
// (BackpropSnapshot.cpp:2723 getJacobianOfConstraintForce and the clamping
// matrices it uses), computed here where A = J Minv J^T is on chip:
// A_c, A_c_ub_E, Q = A_c^T Minv A_c_ub_E + cfm I, pinv(Q) (COD) and the
// rank-deficiency flag ||I - Q Q^+||^2 >= 1e-18.
// A_c and A_c_ub_E of the clamping rows into the snapshot (n x n_c each):
// J^T columns re-evaluated from the rows' contacts and directions
__device__ __forceinline__ void snapshotAc(const ModelDev& md, const double* s, const Layout& L, const FwdPool& P,
                                          const double* cts, double* AcG, double* AcubEG, int m, int nc, int n,
                                          int lane) {
  for (int t = lane; t < n * nc; t += WAVE) {
    const int i = t / nc, c = t % nc;
    const int r = P.clampRow[c];
    const double a = rowForceEntry(md, s, L, cts + P.rowC[r] * CREC, P.dvec + 3 * r, i);
    double ae = a;
    for (int u = r + 1; u <= r + 2 && u < m; u++)
      if (P.mapping[u] == r) ae += P.Eval[u] * rowForceEntry(md, s, L, cts + P.rowC[u] * CREC, P.dvec + 3 * u, i);
    AcG[t] = a;
    AcubEG[t] = ae;
  }
}

template <bool kLds, int R = 1, int kK = 0>  // (kK: as devConstruct)
__device__ void backwardPrecompute(const ModelDev& md, lds_double* sIn, const Layout& L, int lane,
                                   typename Space<kLds>::dptr poolIn, int m, double cfm, double* snap, lds_double* ctIn,
                                   lds_double* stage = nullptr, int stageCap = 0, bool acByHelper = false) {
  const int n = md.n;
  double* s = (double*)sIn;
  double* ct = (double*)ctIn;
  snap = gbl(snap);
  FwdPool P;
  carveFwd(kLds ? (double*)poolIn : gbl((double*)poolIn), m, n, P);
#ifdef NIMBLE_STAGE_TIMING
  double* g_stamp = snap + snStamps(n);
#endif
  STAMP(45);
  const int nc = uni((int)ct[H_NC]);
  if (lane == 0) snap[SN_IMP] = 0.0;
  if (nc == 0) { WSYNC(); return; }
  double* AcG = snap + snAc(n);
  double* AcubEG = snap + snAcubE(n);
  double* PTG = snap + snPT(n);
  double* QG = snap + snQ(n);
  const double* cts = s + L.ct + CT_CONTACTS;
  // A_c, A_c_ub_E (global): J^T columns re-evaluated (the on-chip copy of J^T
  // was overwritten by Y); the helper's post-answer share in the one-row
  // kernel (acByHelper)
  if (!acByHelper) snapshotAc(md, s, L, P, cts, AcG, AcubEG, m, nc, n, lane);
  STAMP(46);
  STAMP(47);
  // Q into M1 (kept) and M2 (factored)
  for (int t = lane; t < nc * nc; t += WAVE) {
    const int cr = t / nc, cc = t % nc;
    const int rr = P.clampRow[cr], rc = P.clampRow[cc];
    double v = P.A[rr * m + rc];
    for (int u = rc + 1; u <= rc + 2 && u < m; u++)
      if (P.mapping[u] == rc) v += P.Eval[u] * P.A[rr * m + u];
    if (cr == cc) v += cfm;
    P.M2[t] = v;
    QG[t] = v;
  }
  // the final classification's COD of this Q is normally still on chip (M1 +
  // scr, devConstruct); refactor only if a fallback solver clobbered it
  const bool reuse = uni(ct[H_CODOK] != 0 ? 1 : 0) != 0;
  WSYNC();
  if (!reuse)
    for (int t = lane; t < nc * nc; t += WAVE) P.M1[t] = P.M2[t];
  WSYNC();
  Cod cod;
  double* w = carveCod(P.scr, P.M1, nc, nc, nc, cod);
  double* cn = w; w += m;
  double* vv = w; w += m;
  double* Zs = P.A;
  // off-chip pools (the wide kernels): the factor and the right-hand sides
  // on chip when the launch's LDS stage holds them (F n_c x n_c, the COD
  // workspace, 64 right-hand sides n_c x 65): every access of the column
  // solves below is then an LDS broadcast (F) or lane-contiguous (Z) instead
  // of a dependent HBM / L2 load with a 64-line gather (~8.7M clocks at
  // n_c = 96 on the mesh Atlas)
  const int wsdS = 4 * nc + (nc + 1) / 2 + 3;
  const bool staged = !kLds && stage != nullptr && nc * nc + wsdS + 65 * nc <= stageCap;
  // (+512: the MFMA solve's block Gram matrix and triangular factor; + the
  // reflector panel when it fits too)
  const bool stagedMfma = staged && nc * nc + wsdS + 65 * nc + 512 <= stageCap && md.pinvMfma;
  const int panelD = ((nc + 15) >> 4) * 16 * 17;
  const bool panel = stagedMfma && nc * nc + wsdS + 65 * nc + 512 + panelD <= stageCap;
  STAMP(48);
  if (staged) {
    double* sF = (double*)stage;
    double* sW = sF + nc * nc;
    double* sZ = sW + wsdS;
    if (reuse) {
      for (int t = lane; t < nc * nc; t += WAVE) sF[t] = P.M1[t];
      for (int t = lane; t < wsdS; t += WAVE) sW[t] = P.scr[t];
      WSYNC();
    } else {
      for (int t = lane; t < nc * nc; t += WAVE) sF[t] = P.M2[t];
      WSYNC();
      codFactorR<true, R>(sp<true>(sF), sp<true>(sW), nc, nc, nc, sp<true>(sZ), lane);
    }
    carveCod(sW, sF, nc, nc, nc, cod);
    STAMP(49);
    if (stagedMfma)
      pinvColumnsMfma((const lds_double*)sF, (const lds_double*)sW, (lds_double*)sZ, (lds_double*)(sZ + 65 * nc),
                      panel ? (lds_double*)(sZ + 65 * nc + 512) : nullptr, nc, PTG, Zs, lane);
    else
      pinvColumnsStaged((const lds_double*)sF, (const lds_double*)sW, (lds_double*)sZ, nc, PTG, Zs, lane);
  } else {
  if (!reuse) codFactorAny<kLds, R>(sp<kLds>(P.M1), sp<kLds>(P.scr), nc, nc, nc, sp<kLds>(vv), lane, stage, stageCap);
  STAMP(49);
  // pinv(Q): lane c solves Q x = e_c in place in row c of the (now free) A
  // region (columns c, c + 64, .. when n_c > 64)
  for (int col = lane; col < nc; col += WAVE) {
    double* rhs = Zs + col * nc;
    for (int i = 0; i < nc; i++) rhs[i] = i == col ? 1.0 : 0.0;
    const double* F = cod.A;
    for (int k = 0; k < cod.kmax; k++) {
      const double vnorm = cod.vn[k];
      if (!(vnorm > 0)) continue;
      double sc = cod.vd[k] * rhs[k];
      for (int i = k + 1; i < nc; i++) sc += F[i * nc + k] * rhs[i];
      sc = 2 * sc / vnorm;
      rhs[k] -= sc * cod.vd[k];
      for (int i = k + 1; i < nc; i++) rhs[i] -= sc * F[i * nc + k];
    }
    const int r = *cod.rank;
    for (int i = r - 1; i >= 0; i--) {
      double sc = rhs[i];
      for (int j = i + 1; j < r; j++) sc -= F[i * nc + j] * rhs[j];
      rhs[i] = sc / F[i * nc + i];
    }
    for (int j = r; j < nc; j++) rhs[j] = 0.0;
    for (int i = 0; i < r && r < nc; i++) {
      const double vn = cod.zn[i];
      if (vn == 0) continue;
      double sc = rhs[i] * cod.zd[i];
      for (int j = r; j < nc; j++) sc += rhs[j] * F[i * nc + j];
      sc = 2 * sc / vn;
      rhs[i] -= sc * cod.zd[i];
      for (int j = r; j < nc; j++) rhs[j] -= sc * F[i * nc + j];
    }
    // column `col` of pinv(Q) = row `col` of pinv(Q)^T
    for (int j = 0; j < nc; j++) PTG[col * nc + cod.perm[j]] = rhs[j];
  }
  }
  WSYNC();
  STAMP(50);
  // ||I - Q Q^+||^2 with (Q Q^+)[r][c] = sum_j Q[r][perm_j] z_c[j] on the
  // matrix cores: one v_mfma_f64_16x16x4f64 chain per 16 x 16 tile (A
  // operand lane l: row l % 16 of Q with columns permuted, k = l / 16; B
  // operand: the tile's columns of Q^+, i.e. the rows z_c of Zs; result
  // element e of lane l = row l / 16 + 4 e, column l % 16).  The reference's
  // GEMM (BackpropSnapshot.cpp:2964 imprecisionMap = I - Q * Qinv): O(n_c^3)
  // multiply-adds, which the lane-per-entry dot products took ~7M clocks
  // for at n_c = 96 (stage timing, mesh Atlas).
  // A rank-deficient factor (rank r < n_c) needs no product: Q Q^+ is then
  // the orthogonal projector onto Q's r-dimensional range (exactly so for
  // the COD pseudo-inverse, up to rounding), so ||I - Q Q^+||_F^2 = n_c - r
  // >= 1, far above the reference's 1e-18 test -- the outcome is the rank's.
  const int rankQ = uni(*cod.rank);
  double part = 0.0;
  if (rankQ == nc && staged) {
    // the stage is free again: Q with its columns permuted (row stride n_c |
    // 1: the A operand's sixteen rows in distinct banks) and 64 pinv columns
    // at a time from Zs, every MFMA operand an LDS read (from HBM with the
    // permutation gathered per element this took ~0.44M clocks at n_c = 93)
    lds_double* sQ = (lds_double*)stage;
    const int ldq = nc | 1;
    lds_double* sZt = sQ + nc * ldq;
    const lds_int* permS = (const lds_int*)cod.perm;
    for (int t = lane; t < nc * nc; t += WAVE) {
      const int r = t / nc, k = t - r * nc;
      sQ[r * ldq + k] = P.M2[r * nc + permS[k]];
    }
    const int i16 = lane & 15, kq = lane >> 4;
    const int T = (nc + 15) >> 4;
    for (int c0 = 0; c0 < nc; c0 += WAVE) {
      const int cnt = nc - c0 < WAVE ? nc - c0 : WAVE;
      WSYNC();
      // Zt[k][c] = z_{c0+c}[k]: lane-contiguous HBM reads of the rows z_c
      for (int t = lane; t < cnt * nc; t += WAVE) {
        const int c = t / nc, k = t - c * nc;
        sZt[k * 65 + c] = Zs[(size_t)(c0 + c) * nc + k];
      }
      WSYNC();
      for (int ti = 0; ti < T; ti++) {
        const int r = ti * 16 + i16;
        const int rc = r < nc ? r : nc - 1;
        nimble_double4 acc[4];
#pragma unroll
        for (int tj = 0; tj < 4; tj++) acc[tj] = nimble_double4{0.0, 0.0, 0.0, 0.0};
        for (int k0 = 0; k0 < nc; k0 += 4) {
          const int k = k0 + kq;
          const int kc = k < nc ? k : nc - 1;
          const double qa = sQ[rc * ldq + kc];
          const double a = (k < nc && r < nc) ? qa : 0.0;
#pragma unroll
          for (int tj = 0; tj < 4; tj++) {
            const int cl = tj * 16 + i16;
            const double zb = sZt[kc * 65 + (cl < cnt ? cl : 0)];
            acc[tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, (k < nc && cl < cnt) ? zb : 0.0, acc[tj], 0, 0, 0);
          }
        }
#pragma unroll
        for (int tj = 0; tj < 4; tj++)
#pragma unroll
          for (int e = 0; e < 4; e++) {
            const int rr = ti * 16 + kq + 4 * e;
            const int cl = tj * 16 + i16;
            const double d = (rr == c0 + cl ? 1.0 : 0.0) - acc[tj][e];
            if (rr < nc && cl < cnt) part += d * d;
          }
      }
    }
    WSYNC();
  } else if (rankQ == nc) {
    const int i16 = lane & 15, kq = lane >> 4;
    const int T = (nc + 15) >> 4;
    const double* Qm = P.M2;
    for (int ti = 0; ti < T; ti++) {
      const int r = ti * 16 + i16;
      for (int tj = 0; tj < T; tj++) {
        const int c = tj * 16 + i16;
        nimble_double4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
        for (int k0 = 0; k0 < nc; k0 += 4) {
          const int k = k0 + kq;
          const bool kin = k < nc;
          const int pk = cod.perm[kin ? k : 0];
          const double a = (kin && r < nc) ? Qm[(r < nc ? r : 0) * nc + pk] : 0.0;
          const double b = (kin && c < nc) ? Zs[(c < nc ? c : 0) * nc + (kin ? k : 0)] : 0.0;
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
        }
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const int rr = ti * 16 + kq + 4 * e;
          const double d = (rr == c ? 1.0 : 0.0) - acc[e];
          if (rr < nc && c < nc) part += d * d;
        }
      }
    }
  }
  const double tot = rankQ < nc ? (double)(nc - rankQ) : waveSum(part);
  if (lane == 0) snap[SN_IMP] = tot >= 1e-18 ? 1.0 : 0.0;
  WSYNC();
  STAMP(51);
}

// ---------------------------------------------------------------------------
// The LCP fallbacks of BoxedLcpConstraintSolver::solve, as functions of the
// problem (A, b, lo, hi, findex, warm start in the pool) so that either wave
// of the forward workgroup can run them (see the task board above).
// ---------------------------------------------------------------------------
template <int R>
__device__ __forceinline__ bool allRowsAlive(int m, const unsigned long long (&alive)[R]) {
  bool eq = true;
#pragma unroll
  for (int q = 0; q < R; q++) {
    const int lo64 = 64 * q;
    const unsigned long long full = m >= lo64 + 64 ? ~0ull : (m > lo64 ? ((1ull << (m - lo64)) - 1ull) : 0ull);
    eq = eq && alive[q] == full;
  }
  return eq;
}

// PGS on the reduced A + cfm I (BoxedLcpConstraintSolver.cpp:550-597) from
// the warm start x_c: LCPUtils::reduce at shift cfm; when it merges columns
// the reduced matrix goes to `Mred` (M1 or M2: whichever the running wave
// owns) and the solution is mapped out (x_i = x_r[rank(rep_i)]).  Returns
// success and validity on the full problem; `dup`: reduce merged columns.
// (The pool's A and warm start come as plain pointers: a FwdPool passed by
// reference to a function that is not inlined is materialised in per-lane
// scratch, 16 KB of stores per wave.)
template <bool kLds, int R>
__device__ bool pgsFallbackR(const double* PA, const double* Pxc, int m, double cf, const double (&bR)[R],
                             const double (&loR)[R], const double (&hiR)[R], const int (&fiR)[R],
                             typename Space<kLds>::dptr Mred, int lane, double (&xd)[R], bool& dup, const int* cancel,
                             double* dbg, int* tally) {
  struct { const double *A, *xc; } P{PA, Pxc};
  double scl[R];
  int rep[R];
  unsigned long long alive[R];
  waveReduceR<kLds, R>(m, spc<kLds>(P.A), cf, bR, loR, hiR, fiR, lane, scl, rep, alive);
  WSYNC();
  dup = !allRowsAlive<R>(m, alive);
  bool ok;
  if (dup) {
    double br[R], lr[R], hr[R], xc[R], xr[R];
    int fr[R], act[R];
#pragma unroll
    for (int q = 0; q < R; q++) {
      br[q] = bR[q]; lr[q] = loR[q]; hr[q] = hiR[q]; fr[q] = fiR[q];
      xc[q] = rowAt(q, lane) < m ? P.xc[rowAt(q, lane)] : 0.0;
    }
    const int mr = reducedVectorsR<R>(alive, rep, lane, br, lr, hr, fr, act);
    reducedMatrixR<kLds, R>(m, spc<kLds>(P.A), cf, alive, act, scl, Mred, true, lane);
#pragma unroll
    for (int q = 0; q < R; q++) {
      xr[q] = gatherR(xc, rowAt(q, lane) < mr ? act[q] : 0);
      if (rowAt(q, lane) >= mr) xr[q] = 0.0;
    }
    ok = wavePgsR<kLds, false, R>(mr, (typename Space<kLds>::cdptr)Mred, xr, br, lr, hr, fr, lane, nullptr, 0.0, cancel,
                                  -1, nullptr, tally);
#pragma unroll
    for (int q = 0; q < R; q++) xd[q] = gatherR(xr, rankR(alive, rep[q]));
  } else {
#pragma unroll
    for (int q = 0; q < R; q++) xd[q] = rowAt(q, lane) < m ? P.xc[rowAt(q, lane)] : 0.0;
    ok = wavePgsR<kLds, false, R>(m, spc<kLds>(P.A), xd, bR, loR, hiR, fiR, lane, dbg, cf, cancel, -1, nullptr, tally);
  }
  if (ok) ok = waveLcpValidR<kLds, R>(m, spc<kLds>(P.A), cf, xd, bR, hiR, loR, fiR, false, lane);
  return ok;
}

// LCPUtils::removeFriction + PGS on the normal rows only (the principal
// submatrix of A + cfm I over them, read in place), from zero; the answer
// per row (friction rows 0).
template <bool kLds, int R>
__device__ void frictionlessPgsR(const double* PA, const double* Pb, const double* Plo, const double* Phi, int m,
                                 double cf, const int (&fiR)[R], int lane, double (&X)[R], const int* cancel,
                                 int* tally) {
  struct { const double *A, *b, *lo, *hi; } P{PA, Pb, Plo, Phi};
  bool keepMe[R];
  unsigned long long km[R];
#pragma unroll
  for (int q = 0; q < R; q++) {
    keepMe[q] = rowAt(q, lane) < m && fiR[q] == -1;
    km[q] = __ballot(keepMe[q]);
  }
  const int k2 = popR(km);
  int myRow[R];
#pragma unroll
  for (int q = 0; q < R; q++) myRow[q] = 0;
  for (int t = 0, c = 0; t < m; t++)
    if (bitR(km, t)) { setRi(myRow, c, lane, t); c++; }
  double xr[R], br[R], lr[R], hr[R];
  int fr[R];
#pragma unroll
  for (int q = 0; q < R; q++) {
    const bool in = rowAt(q, lane) < k2;
    xr[q] = 0.0;
    br[q] = in ? P.b[myRow[q]] : 0.0;
    lr[q] = in ? P.lo[myRow[q]] : 0.0;
    hr[q] = in ? P.hi[myRow[q]] : 0.0;
    fr[q] = -1;
  }
  wavePgsR<kLds, true, R>(k2, spc<kLds>(P.A), xr, br, lr, hr, fr, lane, nullptr, cf, cancel, m, myRow, tally);
#pragma unroll
  for (int q = 0; q < R; q++) {
    const double v = gatherR(xr, keepMe[q] ? rankR(km, rowAt(q, lane)) : 0);
    X[q] = keepMe[q] ? v : 0.0;
  }
}

// impulses (applyConstraintImpulses + computeImpulseForwardDynamics): the
// velocity change u = Minv J^T x = L^-T (Y x) on lane i < n (and the
// pre-impulse velocity into the snapshot)
__device__ __forceinline__ double impulseDelta(const double* Y, const double* Xf, const double* Lm, const double* dinv,
                                               const double* v1, double* snap, int n, int m, int lane) {
  double u = 0.0;
  if (lane < n) {
#pragma unroll 4
    for (int j = 0; j < m; j++) u += Y[lane * m + j] * Xf[j];
    snap[SN_VF + lane] = v1[lane];
  }
  for (int k = n - 1; k >= 0; k--) {
    const double uk = rdl(u, k) * dinv[k];
    if (lane == k) u = uk;
    else if (lane < k) u -= Lm[tri(k, lane)] * uk;
  }
  return u;
}

// the snapshot's contacts, rows, clamping impulses and unconstrained
// acceleration
__device__ __forceinline__ void snapshotRows(const FwdPool& P, const double* ct, const double* ddq, double* snap,
                                             int nCon, int m, int nc, int n, int lane) {
  for (int t = lane; t < nCon * CREC; t += WAVE) snap[SN_CONTACTS + t] = ct[CT_CONTACTS + t];
  for (int j = lane; j < m; j += WAVE) {
    double* rr = snap + SN_ROWS + j * SN_ROWREC;
    rr[RR_CONTACT] = P.rowC[j];
    rr[RR_DIR] = P.rowDir[j];
    for (int i = 0; i < 3; i++) rr[RR_D + i] = P.dvec[3 * j + i];
    rr[RR_B] = P.b[j];
    rr[RR_X] = P.X[j];
    rr[RR_MAP] = P.mapping[j];
    rr[RR_CIDX] = P.clampIdx[j];
    rr[RR_UIDX] = P.ubIdx[j];
    rr[RR_EVAL] = P.Eval[j];
    rr[RR_BOUNCE] = 1.0 + P.rest[j];
  }
  for (int i = lane; i < nc; i += WAVE) snap[SN_FC + i] = P.fc[i];
  for (int i = lane; i < n; i += WAVE) snap[snYf(n) + i] = ddq[i];
}

// ---------------------------------------------------------------------------
// The whole constraint stage of one world (World.cpp:254 runConstraintEngine
// on the hot path): rows, A = J Minv J^T, b, LCP with the short-circuit,
// fallbacks, impulses (v1 += Minv J^T x), warm-start cache and snapshot.
// `Lm` is the Cholesky factor of M (lower triangle, n x n).
// ---------------------------------------------------------------------------
template <bool kLds, int R, int kK = 0>
__device__ __forceinline__ void contactLcp(const ModelDev& md, lds_double* sIn, const Layout& L, int lane,
                                           lds_double* v1In, const lds_double* ddqIn, double* cache, double* snap,
                                           typename Space<kLds>::dptr poolIn, int nCon, int m, bool helperOn);

// inlined into the forward kernel: the model, layout and LDS base keep their
// kernel-argument provenance (scalar loads, LDS instructions).  R row slots
// per lane (R = 1: <= 64 LCP rows).  A world with more than `deferRows` rows
// is left to the R = 2 kernel (status ST_DEFERRED, nothing else of the step
// written, the warm-start cache untouched): returns true then.
template <int R>
__device__ __forceinline__ bool contactStage(const ModelDev& md, double* s, const Layout& L, int lane, double* v1,
                                             const double* ddq, double* cache, double* snap, double* overflowWs,
                                             bool helperOn, bool collided, int deferRows, bool handedOff = false,
                                             double* deferSnap = nullptr, int snapDoubles = 0, int env = 0) {
  const int n = md.n;
  s = lds<true>(s);
  snap = gbl(snap);
  cache = gbl(cache);
  overflowWs = gbl(overflowWs);
#ifdef NIMBLE_STAGE_TIMING
  double* g_stamp = snap + snStamps(n);
#endif
  STAMP(0);
  double* ct = s + L.ct;
  if (handedOff) {
    // the one-row kernel's contact header and kept contacts (written to the
    // workspace when it deferred this world; read before the LCP pool,
    // which starts there, overwrites them)
    // (only the header fields of the step, not the helper / collision flags
    // or the board, which this kernel's helper is already polling)
    // (a protocol failure of the one-row kernel's turn, flagged in the
    // snapshot status after the hand-off, stays in the world's status)
    const int nk = uni((int)overflowWs[H_NCON]);
    if (lane < H_HELPER) {
      double v = overflowWs[lane];
      if (lane == H_STATUS) v = (double)((int)v | ((int)snap[SN_STATUS] & ST_PROTOCOL));
      ct[lane] = v;
    }
    for (int t = lane; t < nk * CREC; t += WAVE) ct[CT_CONTACTS + t] = overflowWs[CT_CONTACTS + t];
    WSYNC();
  } else if (collided) {
    // the helper wave ran the collision detection during the dynamics (the
    // deadlock guard expired: the helper may still be writing the contacts,
    // the world's contact step is abandoned)
    if (collideWait(ct, CS_DONE, GW_COLLIDE_DONE)) {
      collidePost(ct, CS_IDLE, lane);
    } else {
      protocolAbort(snap, cache, lane);
      return false;
    }
  } else {
#ifdef NIMBLE_STAGE_TIMING
    collideWorld(md, s, L, lane, snap + snEdge(n), g_stamp);
#else
    collideWorld(md, s, L, lane, snap + snEdge(n));
#endif
  }
  STAMP(1);
  const int nCon = uni((int)ct[H_NCON]);
  if (nCon == 0) {
    if (lane == 0) {
      for (int i = 0; i < SN_DEFER; i++) snap[i] = 0.0;
      snap[SN_STATUS] = ct[H_STATUS];
    }
    WSYNC();
    return false;
  }
  // row count: 3 rows per frictional contact, 1 otherwise (lane = contact)
  bool fr = false;
  if (lane < nCon) {
    const double* rec = ct + CT_CONTACTS + lane * CREC;
    fr = fmin(md.friction[(int)rec[8]], md.friction[(int)rec[9]]) > 1e-3;
  }
  const int m = nCon + 2 * __popcll(__ballot(fr));
  if (m > deferRows) {
    // hand the contacts to the wide kernel (the snapshot's workspace, its
    // LCP pool later); the dynamics are in the snapshot's dynamics cache
    for (int t = lane; t < CT_CONTACTS + nCon * CREC; t += WAVE) overflowWs[t] = ct[t];
    if (lane == 0) snap[SN_STATUS] = (double)((int)ct[H_STATUS] | ST_DEFERRED);
    if (deferSnap != nullptr && lane == 0) {
      // the wide kernel's order: largest LCPs first (deferBucket); the lists
      // live in the call's own snapshot headers (deferCount / deferEntry)
      const int q = deferBucket(m);
      const int i = __hip_atomic_fetch_add(deferCount(deferSnap) + q, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *deferEntry(deferSnap, snapDoubles, q * gridDim.x + i) = env;
    }
    WSYNC();
    return true;
  }
  if (m > 64 * R) {
    // more rows than one wave's lanes: the contacts are recorded, the solve
    // is not taken (flagged; the snapshot says no rows, so the backward and
    // the Jacobians see a contact-free step)
    for (int t = lane; t < nCon * CREC; t += WAVE) snap[SN_CONTACTS + t] = ct[CT_CONTACTS + t];
    if (lane == 0) {
      for (int i = 0; i < SN_DEFER; i++) snap[i] = 0.0;
      snap[SN_NCON] = nCon;
      snap[SN_STATUS] = (double)((int)ct[H_STATUS] | ST_LCP_TOO_LARGE);
      ct[H_M] = 0;
      cache[0] = -1.0;
    }
    WSYNC();
    return false;
  }
  if (lane == 0) ct[H_M] = m;  // read by the helper wave
  // the LCP workspace is in LDS when it fits the pool (the common case, LDS
  // instructions throughout), else in the world's HBM snapshot tail (always
  // for the wide problems of R = 2)
  if ((R == 1 && fwdPoolDoubles(m, n) <= L.poolCap) ||
      (R > 1 && m <= 64 && L.stageCap > 0 && fwdPoolDoubles(m, n) <= L.stageCap))
    // the pool on chip: the one-row kernel's own pool, or the wide kernel's
    // LDS stage (which starts at the pool) for the worlds the one-row kernel
    // deferred because its pool could not hold them
    contactLcp<true, 1, (R > 1 ? 1 : 0)>(md, sp<true>(s), L, lane, sp<true>(v1), spc<true>(ddq), cache, snap, sp<true>(s + L.pool),
                        nCon, m, helperOn);
  else
    // (the helper joins through the LDS stage: contactLcp's task board)
    contactLcp<false, R>(md, sp<true>(s), L, lane, sp<true>(v1), spc<true>(ddq), cache, snap, overflowWs, nCon, m,
                         helperOn);
  return false;
}

template <bool kLds, int R, int kK>
__device__ __forceinline__ void contactLcp(const ModelDev& md, lds_double* sIn, const Layout& L, int lane,
                                           lds_double* v1In, const lds_double* ddqIn, double* cache, double* snap,
                                           typename Space<kLds>::dptr poolIn, int nCon, int m, bool helperOn) {
  const int n = md.n;
  double* s = (double*)sIn;
  double* v1 = (double*)v1In;
  const double* ddq = (const double*)ddqIn;
  double* pool = kLds ? (double*)poolIn : gbl((double*)poolIn);
  snap = gbl(snap);
  cache = gbl(cache);
#ifdef NIMBLE_STAGE_TIMING
  double* g_stamp = snap + snStamps(n);
#endif
  double* ct = s + L.ct;
  const double* Lm = s + L.M;
  FwdPool P;
  carveFwd(pool, m, n, P);
  // (the pair counts are dead: the solvers' tally starts here, before any
  // task goes out to the helper)
  if (lane < 4) tallyOf(ct)[lane] = 0;
  // the helper builds the rows and A (early rows, see EA_*): EA_NONE when it
  // does not (stored before its CS_DONE, which wave 0 has taken)
  const bool early = kLds && R == 1 && kK == 0 && helperOn && earlyState(ct) != EA_NONE;
  if (early) {
    if (!earlyWait(ct, [&]() { return earlyState(ct) >= EA_ROWS; }, GW_EARLY_ROWS)) {
      protocolAbort(snap, cache, lane);
      return;
    }
  } else {
    buildRows(md, s, L, ct, nCon, m, RowsOut{P.cols, P.dvec, P.lo, P.hi, P.rest, P.fi, P.rowC, P.rowDir}, lane);
  }
  STAMP(2);
  // b = -J v1 first: Y = L^-1 J^T is formed in place of J^T, so that
  // A = J Minv J^T = Y^T Y and Minv J^T x = L^-T (Y x)
  rowsRhs(P.cols, v1, P.b, n, m, lane);
  if (early && lane == 0)  // (J^T read: the helper may overwrite it with Y)
    __hip_atomic_store(helperFlags(ct) + 1, HF_B, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  STAMP(86);
  // penetration correction / restitution bounce of the normal rows (lane = row)
  for (int r = lane; r < m; r += WAVE) {
    P.pen[r] = 0.0;
    if (P.rowDir[r] != 0) continue;
    const double* rec = ct + CT_CONTACTS + P.rowC[r] * CREC;
    double bv = rec[6];
    if (bv < 0.0) bv = 0.0;
    else { bv *= 0.01 / md.dt; if (bv > 1e-3) bv = 1e-3; }
    if (!md.penCorr) bv = 0;
    P.pen[r] = bv;
    if (P.rest[r] > 0) {
      const double rv = P.b[r] * P.rest[r];
      if (rv > 1e-1 && rv > bv) { bv = rv > 1e2 ? 1e2 : rv; P.pen[r] = 0.0; }
      else P.rest[r] = 0.0;
    }
    P.b[r] += bv;
  }
  WSYNC();
  if (early) {
    if (!earlyWait(ct, [&]() { return earlyState(ct) == EA_A; }, GW_EARLY_A)) {
      protocolAbort(snap, cache, lane);
      return;
    }
    STAMP(87);
  } else {
    formY(P.massed, P.cols, Lm, s + L.dinv, n, m, lane);
    STAMP(87);
    // A = Y^T Y on the matrix cores (the LCP matrix J Minv J^T)
    gramMfma(P.massed, P.A, n, m, lane);
    WSYNC();
  }
  STAMP(88);
  for (int j = lane; j < m; j += WAVE) {
    double acc = 0;
#pragma unroll 8
    for (int i = 0; i < m; i++) acc += P.A[i * m + j] * P.A[i * m + j];
    P.aCol[j] = acc;
  }
  WSYNC();
  STAMP(3);
  // the helper wave starts Dantzig on A now (the task board, see helperWave):
  // A, b, lo, hi and findex are final; the warm start follows
  // off-chip pools (wide kernels) factorise through the launch's LDS stage
  lds_double* stage = (!kLds && L.stageCap > 0) ? sp<true>(s + L.stage) : nullptr;
  int stageCap = L.stageCap;
  // the wide kernel's worlds with an off-chip pool share the cascade on the
  // task board too when Dantzig's LDL^T factor and scatter vector fit the
  // start of the stage: the helper keeps them there for the whole cascade,
  // wave 0's factorisations use the rest until the helper is out
  // (posted at once when the rest of the stage still holds the first
  // classification's largest COD; otherwise only once that classification
  // has failed, so that it factorises with the whole stage, and Dantzig then
  // overlaps the PGS fallbacks only)
  // (the factor packed: dantzigLDoubles, 37 KB instead of 74 KB at 96 rows)
  const int dzStage = (dantzigLDoubles(m, true) + m + 1) & ~1;
  const int codNeed = m * m + 4 * m + (m + 1) / 2 + 3 + m;  // codFactorAny's stage check at n_c = m
  const bool taskable = helperOn && (kLds ? R == 1 : (stage != nullptr && dzStage < stageCap));
  const bool earlyPost = taskable && (kLds || codNeed + dzStage <= stageCap);
  bool tasked = taskable;
  lds_double* const stageAll = stage;
  const int stageCapAll = stageCap;
  auto postTask = [&](bool warmFinal) {
    if (!kLds) {
      stage += dzStage;
      stageCap -= dzStage;
    }
    boardPost(ct, kLds ? HB_LDS_POOL : HB_WIDE, warmFinal, lane);
  };
  if (earlyPost) postTask(false);
  // a settled answer makes every solve still running moot
  auto stopAll = [&]() {
    boardSet(ct, BD_STOPD, 1, lane);
    boardSet(ct, BD_STOPP, 1, lane);
    boardSet(ct, BD_STOPF, 1, lane);
  };
  // warm start (BoxedLcpConstraintSolver::mX) or guessSolution
  const bool cached = uni((int)cache[0]) == m;
  if (cached) {
    for (int i = lane; i < m; i += WAVE) { P.X[i] = cache[1 + i]; P.xc[i] = cache[1 + i]; }
    WSYNC();
  } else {
    devGuess<kLds, R, kK>(poolIn, m, n, sp<true>(ct), lane, stage, stageCap);
    for (int i = lane; i < m; i += WAVE) P.xc[i] = P.X[i];
    WSYNC();
  }
  if (earlyPost) boardSet(ct, BD_G, 1, lane);
  if (lane == 0) ct[H_CODOK] = 0;
  STAMP(4);
  // (not posted at once: the classification posts the task itself as soon as
  // its n_c shows that its factor fits beside Dantzig's)
  const int postDz = taskable && !earlyPost ? dzStage : 0;
#ifdef NIMBLE_STAGE_TIMING
  bool success = devConstruct<kLds, R, kK>(poolIn, m, n, 0.0, false, sp<true>(ct), lane, g_stamp, stage, stageCap, postDz);
  double* dbgPgs = g_stamp ? g_stamp + SLOT_PGS : nullptr;
#else
  bool success = devConstruct<kLds, R, kK>(poolIn, m, n, 0.0, false, sp<true>(ct), lane, nullptr, stage, stageCap, postDz);
  double* dbgPgs = nullptr;
#endif
  bool posted = earlyPost;
  if (postDz > 0 && helperState(ct) != HS_IDLE) {
    posted = true;
    stage += dzStage;
    stageCap -= dzStage;
  }
  if (posted && success) stopAll();
  if (taskable && !posted) {
    if (success) tasked = false;  // (no task went out; helperRetire posts SKIP)
    else postTask(true);
  }
  STAMP(5);
  const bool shortCircuit = success;
  double cfm = 0.0;
  bool ignoredFriction = false;
  // the problem's row-held vectors (row j on lane j & 63, slot j >> 6)
  double bR[R], hiR[R], loR[R];
  int fiR[R];
#pragma unroll
  for (int q = 0; q < R; q++) {
    const int j = rowAt(q, lane);
    bR[q] = j < m ? P.b[j] : 0.0;
    hiR[q] = j < m ? P.hi[j] : 0.0;
    loR[q] = j < m ? P.lo[j] : 0.0;
    fiR[q] = j < m ? P.fi[j] : -1;
  }
  // the board's answer when Dantzig failed: 1 the PGS fallback, 2 the
  // frictionless PGS (-1: Dantzig's, or no board)
  int boardSrc = -1;
  if (!success) {
    // Dantzig on the reduced problem (BoxedLcpConstraintSolver.cpp:466-521):
    // LCPUtils::reduce merges near-duplicate columns; when it merges any, the
    // reduced matrix (in M1, free here) goes to Dantzig and the solution is
    // mapped out (x_i = x_r[rank(rep_i)]); validity on the full problem
    if (lane == 0) ct[H_CODOK] = 0;
    double scl[R];
    int rep[R];
    unsigned long long alive[R];
    waveReduceR<kLds, R>(m, spc<kLds>(P.A), 0.0, bR, loR, hiR, fiR, lane, scl, rep, alive);
    WSYNC();
    double xd[R];
#pragma unroll
    for (int q = 0; q < R; q++) xd[q] = 0.0;
    bool ok;
    bool validated = false;
    const bool merged = !allRowsAlive<R>(m, alive);
    if (merged && lane == 0) ct[H_STATUS] = (double)((int)ct[H_STATUS] | ST_DUPLICATE_COLUMNS);
    if (merged && (kLds || !tasked)) {
      // (on chip the helper sees the same merge and solves nothing: wait
      // until it is out of the pool; the wide kernel's helper solves the
      // reduced problem on the board below)
      if (tasked && helperWait(ct, [](int v) { return v == HS_DONE; }, GW_MERGED) < 0) {
        stopAll();
        protocolAbort(snap, cache, lane);
        return;
      }
      double br[R], lr[R], hr[R], xr[R];
      int fr[R], act[R];
#pragma unroll
      for (int q = 0; q < R; q++) { br[q] = bR[q]; lr[q] = loR[q]; hr[q] = hiR[q]; fr[q] = fiR[q]; }
      const int mr = reducedVectorsR<R>(alive, rep, lane, br, lr, hr, fr, act);
      reducedMatrixR<kLds, R>(m, spc<kLds>(P.A), 0.0, alive, act, scl, sp<kLds>(P.M1), false, lane);
      ok = waveDantzigR<kLds, R>(mr, spc<kLds>(P.M1), sp<kLds>(P.M2), sp<kLds>(P.scr), xr, br, lr, hr, fr, lane,
                                 nullptr, nullptr, tallyOf(ct));
#pragma unroll
      for (int q = 0; q < R; q++) xd[q] = gatherR(xr, rankR(alive, rep[q]));
    } else if (tasked) {
      // the helper runs Dantzig; meanwhile this wave claims the PGS fallback,
      // then the frictionless PGS, until the reference's order decides:
      // Dantzig's answer if it succeeds, else the PGS fallback's, else the
      // frictionless one
      bool expired = guardForced(ct, GW_BOARD);
      const long long t0 = spinClock();
      for (int it = 0; !expired; it++) {
        const int d = boardGet(ct, BD_D);
        if (d == 1) break;
        const int pst = boardGet(ct, BD_P);
        if (d >= 2 && pst == 1) { boardSrc = 1; break; }
        if (d >= 2 && pst == 2 && boardGet(ct, BD_F) == 1) { boardSrc = 2; break; }
        if (pst == 0 && boardClaim(ct, BD_PCLAIM, 1, lane)) {
#ifdef NIMBLE_STAGE_TIMING
          if (lane == 0 && g_stamp) { g_stamp[97] = 1; g_stamp[100] = (double)__builtin_amdgcn_s_memtime(); }
#endif
          bool dup;
          double xp[R];
          const bool okp = pgsFallbackR<kLds, R>(P.A, P.xc, m, md.fallbackCfm, bR, loR, hiR, fiR, sp<kLds>(P.M1), lane, xp,
                                                 dup, board(ct) + BD_STOPP, dbgPgs, tallyOf(ct));
#pragma unroll
          for (int q = 0; q < R; q++)
            if (rowAt(q, lane) < m) P.xp[rowAt(q, lane)] = xp[q];
          boardSet(ct, BD_PDUP, dup ? 1 : 0, lane);
          if (okp) boardSet(ct, BD_STOPF, 1, lane);
          boardSet(ct, BD_P, okp ? 1 : 2, lane);
#ifdef NIMBLE_STAGE_TIMING
          if (lane == 0 && g_stamp) g_stamp[101] = (double)__builtin_amdgcn_s_memtime();
#endif
          continue;
        }
        if (pst != 1 && boardGet(ct, BD_F) == 0 && boardClaim(ct, BD_FCLAIM, 1, lane)) {
#ifdef NIMBLE_STAGE_TIMING
          if (lane == 0 && g_stamp) { g_stamp[98] = 1; g_stamp[102] = (double)__builtin_amdgcn_s_memtime(); }
#endif
          double xf[R];
          frictionlessPgsR<kLds, R>(P.A, P.b, P.lo, P.hi, m, md.fallbackCfm, fiR, lane, xf, board(ct) + BD_STOPF,
                                    tallyOf(ct));
#pragma unroll
          for (int q = 0; q < R; q++)
            if (rowAt(q, lane) < m) P.xf[rowAt(q, lane)] = xf[q];
          boardSet(ct, BD_F, 1, lane);
#ifdef NIMBLE_STAGE_TIMING
          if (lane == 0 && g_stamp) g_stamp[103] = (double)__builtin_amdgcn_s_memtime();
#endif
          continue;
        }
        if (protocolFailed(ct) || spinExpired(t0, it)) {
          expired = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (expired) {
        // the deadlock guard: the helper may still be in the pool (its
        // Dantzig factor, the board's vectors); the world's contact step is
        // abandoned
        protocolFail(ct);
        stopAll();
        protocolAbort(snap, cache, lane);
        return;
      }
      // Dantzig's answer (checked valid by the helper)
      ok = boardSrc < 0;
      validated = true;
#pragma unroll
      for (int q = 0; q < R; q++) xd[q] = ok && rowAt(q, lane) < m ? P.xh[rowAt(q, lane)] : 0.0;
    } else {
      // off-chip pools: the LDL^T factor in the launch's LDS stage when it
      // fits (every pivot's triangular solves and its row / column shifts
      // read and write it; A is read a row at a time and stays in HBM)
#ifdef NIMBLE_STAGE_TIMING
      double* dbgDz = g_stamp ? g_stamp + SLOT_DANTZIG : nullptr;
#else
      double* dbgDz = nullptr;
#endif
      const int ldL = m | 1, nPk = m * (m + 1) / 2, nL = dantzigLDoubles(m, true);
      if (stage != nullptr && nL + nPk + m <= stageCap) {
        // L and A's packed lower triangles and the scatter vector all in the
        // stage: every Dantzig access an LDS instruction
        lds_double* sL = stage;
        lds_double* sA = stage + nL;
        lds_double* sS = sA + nPk;
        for (int i = 0; i < m; i++)
          for (int j = lane; j <= i; j += WAVE) sA[i * (i + 1) / 2 + j] = P.A[i * m + j];
        WSYNC();
        ok = waveDantzigR<true, R, true, true, true>(m, sA, sL, sS, xd, bR, loR, hiR, fiR, lane, dbgDz, nullptr,
                                                     tallyOf(ct));
      } else {
        double* Ld = (stage != nullptr && m * ldL <= stageCap) ? (double*)stage : (double*)P.M2;
        ok = waveDantzigR<kLds, R>(m, spc<kLds>(P.A), sp<kLds>(Ld), sp<kLds>(P.scr), xd, bR, loR, hiR, fiR, lane, dbgDz,
                                   nullptr, tallyOf(ct));
      }
    }
    if (ok) {
#pragma unroll
      for (int q = 0; q < R; q++)
        if (rowAt(q, lane) < m) P.X[rowAt(q, lane)] = xd[q];
      WSYNC();
      if (!validated) ok = waveLcpValidR<kLds, R>(m, spc<kLds>(P.A), 0.0, xd, bR, hiR, loR, fiR, false, lane);
    }
    success = ok;
  }
  STAMP(6);
  {
    bool ok = success;
    bool ign = false;
    double cf = 0.0;
    double X[R];
    if (boardSrc > 0) {
      // a fallback the board ran (validated by the wave that ran it)
      cf = md.fallbackCfm;
      ign = boardSrc == 2;
      if (boardGet(ct, BD_PDUP) && lane == 0) ct[H_STATUS] = (double)((int)ct[H_STATUS] | ST_DUPLICATE_COLUMNS);
#pragma unroll
      for (int q = 0; q < R; q++) {
        const int j = rowAt(q, lane);
        X[q] = j < m ? (boardSrc == 1 ? P.xp[j] : P.xf[j]) : 0.0;
      }
    } else {
      bool nan = false;
#pragma unroll
      for (int q = 0; q < R; q++) {
        X[q] = rowAt(q, lane) < m ? P.X[rowAt(q, lane)] : 0.0;
        nan = nan || (rowAt(q, lane) < m && isnan(X[q]));
      }
      if (__ballot(nan)) {
        ok = false;
#pragma unroll
        for (int q = 0; q < R; q++) X[q] = 0.0;
      }
      if (!ok) {
        // (reached with a board only when the classification's answer holds
        // a NaN: the helper has been stopped; wait until it is out of the pool)
        if (tasked) {
          stopAll();
          if (helperWait(ct, [](int v) { return v == HS_DONE; }, GW_NAN) < 0) {
            protocolAbort(snap, cache, lane);
            return;
          }
        }
        cf = md.fallbackCfm;
        if (lane == 0) ct[H_CODOK] = 0;
        bool dup;
        double xd[R];
        // off-chip pools: the PGS sweeps read A from the LDS stage when it
        // fits (a row per row step: LDS instead of L2 latency)
        const double* As = P.A;
        if (stage != nullptr && m * m <= stageCap) {
          double* sA = (double*)stage;
          for (int t = lane; t < m * m; t += WAVE) sA[t] = P.A[t];
          WSYNC();
          As = sA;
        }
        ok = pgsFallbackR<kLds, R>(As, P.xc, m, cf, bR, loR, hiR, fiR, sp<kLds>(P.M1), lane, xd, dup, nullptr, dbgPgs,
                                   tallyOf(ct));
        if (dup && lane == 0) ct[H_STATUS] = (double)((int)ct[H_STATUS] | ST_DUPLICATE_COLUMNS);
        if (ok)
#pragma unroll
          for (int q = 0; q < R; q++) X[q] = xd[q];
      }
      if (!ok) {
        ign = true;
        const double* As = P.A;
        if (stage != nullptr && m * m <= stageCap) {
          // (the stage holds A already when the PGS fallback ran from it)
          double* sA = (double*)stage;
          for (int t = lane; t < m * m; t += WAVE) sA[t] = P.A[t];
          WSYNC();
          As = sA;
        }
        frictionlessPgsR<kLds, R>(As, P.b, P.lo, P.hi, m, cf, fiR, lane, X, nullptr, tallyOf(ct));
      }
    }
    bool nan2 = false;
#pragma unroll
    for (int q = 0; q < R; q++) nan2 = nan2 || (rowAt(q, lane) < m && isnan(X[q]));
    if (__ballot(nan2))
#pragma unroll
      for (int q = 0; q < R; q++) X[q] = 0.0;
#pragma unroll
    for (int q = 0; q < R; q++)
      if (rowAt(q, lane) < m) P.X[rowAt(q, lane)] = X[q];
    if (lane == 0) { ct[H_CFM] = cf; ct[H_IGN] = ign ? 1 : 0; }
    WSYNC();
  }
  // the helper out of the pool before construct 2 and the backward
  // precompute overwrite it (M1, M2, A); the whole stage is wave 0's again
  if (tasked) {
    stopAll();
    if (helperWait(ct, [](int v) { return v == HS_DONE; }, GW_COLLECT) < 0) {
      protocolAbort(snap, cache, lane);
      return;
    }
    stage = stageAll;
    stageCap = stageCapAll;
  }
  cfm = unid(ct[H_CFM]);
  ignoredFriction = uni(ct[H_IGN] != 0 ? 1 : 0) != 0;
  STAMP(7);
  // the step keeps the solver's x unless the re-standardisation succeeds
  // (BoxedLcpConstraintSolver: `if (gm.standardized) x = gm.X`)
  bool std2 = true;
  if (!shortCircuit) {
    for (int i = lane; i < m; i += WAVE) P.xc[i] = P.X[i];
    WSYNC();
    std2 = devConstruct<kLds, R, kK>(poolIn, m, n, cfm, ignoredFriction, sp<true>(ct), lane, nullptr, stage, stageCap);
  }
  const double* Xf = std2 ? P.X : P.xc;
  STAMP(8);
  const int nc = uni((int)ct[H_NC]);
  // The post-answer work in two shares (one-row kernel): the helper forms
  // the impulse's velocity change into s + L.rhs (dead since the dynamics)
  // and writes the snapshot's contacts and rows and the clamping rows' J^T
  // columns A_c, A_c_ub_E (HS_POST; the flag tells it
  // which x the step keeps) while wave 0 runs the backward precompute --
  // disjoint pool slots -- then wave 0 adds the change to v1.  Nothing of
  // the state, the cache or the snapshot header is the helper's, so a
  // protocol failure still leaves the contact-free step.
  const bool postSplit = kLds && R == 1 && kK == 0 && helperOn && md.postSplit;
  if (postSplit) {
    if (lane == 0) helperFlags(ct)[1] = std2 ? 1 : 0;
    helperPost(ct, HS_POST, lane);
  } else {
    const double u = impulseDelta(P.massed, Xf, Lm, s + L.dinv, v1, snap, n, m, lane);
    WSYNC();
    if (lane < n) v1[lane] += u;
    snapshotRows(P, ct, ddq, snap, nCon, m, nc, n, lane);
  }
  if (lane == 0) cache[0] = m;
  for (int i = lane; i < m; i += WAVE) cache[1 + i] = Xf[i];
  backwardPrecompute<kLds, R, kK>(md, sIn, md.lay[0], lane, poolIn, m, cfm, snap, sp<true>(ct), stage, stageCap,
                                  postSplit);  // (not inlined)
  if (postSplit) {
    if (helperWait(ct, [](int v) { return v == HS_POSTDONE; }, GW_POST) < 0) {
      protocolAbort(snap, cache, lane);
      return;
    }
    if (lane < n) v1[lane] += s[L.rhs + lane];
    WSYNC();
  }
  if (lane == 0) {
    snap[SN_NCON] = nCon;
    snap[SN_M] = m;
    snap[SN_NC] = nc;
    snap[SN_NU] = ct[H_NU];
    snap[SN_CFM] = cfm;
    snap[SN_STATUS] = ct[H_STATUS];
    snap[SN_SC] = shortCircuit ? 1 : 0;
    snap[SN_IGN] = ignoredFriction ? 1 : 0;
    // (the helper's share is in: it answered DONE before construct 2)
    const int* ty = tallyOf(ct);
    snap[SN_PIVOTS] = ty[0];
    snap[SN_SWEEPS] = ty[1];
    snap[SN_SOLVER_FLOPS] = (double)(unsigned)ty[2];
  }
  WSYNC();
  STAMP(9);
}

// One world's turn of the helper wave (wave 1 of the forward workgroup):
// wait for wave 0's TASK or SKIP; for a task, run Dantzig on A (unless
// LCPUtils::reduce merges columns: wave 0 then solves the reduced problem
// itself), then claim whichever fallbacks are still open (the task board,
// see above); answer DONE, then wait until wave 0 has taken the answer.
// `g_stamp`: the stage-timing build's stamps (else null).
// The helper's share of the cascade for one world (see helperWave): R row
// slots per lane, the pool P on chip (kLds) or in HBM; Dantzig's LDL^T factor
// and scatter vector at Ldz / scrDz (LDS: the pool's M2 / xh2, or the wide
// kernel's stage), the PGS fallback's reduced matrix at Mred.
// The helper's end of the collision hand-off in the one-row kernel (see
// EA_*): posts CS_DONE, then, when the world's LCP will run in the LDS pool
// (wave 0 takes the same decision from the same contacts), builds the rows
// and J^T there, and once wave 0 has formed b from them forms Y and A.
// (deferRows: the kernel's threshold -- a world wave 0 defers to the wide
// kernel never reaches the b hand-off, so the helper does not take it)
__device__ __forceinline__ void helperEarly(const ModelDev& md, double* s, const Layout& L, int lane, int deferRows) {
  double* ct = s + L.ct;
  const int n = md.n;
  const int nCon = uni((int)ct[H_NCON]);
  bool fr = false;
  if (lane < nCon) {
    const double* rec = ct + CT_CONTACTS + lane * CREC;
    fr = fmin(md.friction[(int)rec[8]], md.friction[(int)rec[9]]) > 1e-3;
  }
  const int m = nCon + 2 * __popcll(__ballot(fr));
  const bool take = L.early > 0 && nCon > 0 && m <= WAVE && m <= deferRows && fwdPoolDoubles(m, n) <= L.poolCap;
  if (!take) {
    if (lane == 0) *earlyFlag(ct) = EA_NONE;  // (published by the release of CS_DONE)
    collidePost(ct, CS_DONE, lane);
    return;
  }
  collidePost(ct, CS_DONE, lane);
  // (the world's critical path until A is built)
  __builtin_amdgcn_s_setprio(2);
  FwdPool P;
  carveFwd(s + L.pool, m, n, P);
  buildRows(md, s, L, ct, nCon, m, RowsOut{P.cols, P.dvec, P.lo, P.hi, P.rest, P.fi, P.rowC, P.rowDir}, lane);
  earlyPost(ct, EA_ROWS, lane);
  // Y into M1 (+ M2, free until the cascade; when they hold n x m) while
  // wave 0 still needs J^T for b, A = Y^T Y from there, and Y moves into
  // J^T's place once wave 0 has b; otherwise Y in place after b
  double* Yt = P.M1;
  const bool aside = n * m <= m * m + m * (m | 1);
  auto flagAtLeast = [&](int v) {
    return uni(__hip_atomic_load(helperFlags(ct) + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) >= v;
  };
  if (earlyWait(ct, [&]() { return flagAtLeast(HF_DYN); }, GW_EARLY_DYN)) {
    if (aside) {
      formY(Yt, P.cols, s + L.M, s + L.dinv, n, m, lane);
      gramMfma(Yt, P.A, n, m, lane);
      WSYNC();
    }
    if (earlyWait(ct, [&]() { return flagAtLeast(HF_B); }, GW_EARLY_B)) {
      if (aside) {
        for (int t = lane; t < n * m; t += WAVE) P.massed[t] = Yt[t];
        WSYNC();
      } else {
        formY(P.massed, P.cols, s + L.M, s + L.dinv, n, m, lane);
        gramMfma(P.massed, P.A, n, m, lane);
        WSYNC();
      }
      earlyPost(ct, EA_A, lane);
    }
  }
  __builtin_amdgcn_s_setprio(0);
}

template <bool kLds, int R, bool kPL = false>
__device__ __forceinline__ void helperTask(const ModelDev& md, double* ct, const FwdPool& Pin, int m, int lane,
                                           lds_double* Ldz, lds_double* scrDz, typename Space<kLds>::dptr Mred,
                                           double* g_stamp) {
  (void)g_stamp;
  // (pointers copied out: a pool struct taken by reference into the
  // non-inlined solvers would be materialised in scratch)
  const double* PA = Pin.A;
  const double *Pb = Pin.b, *Plo = Pin.lo, *Phi = Pin.hi, *Pxc = Pin.xc;
  double *Pxh = Pin.xh, *Pxp = Pin.xp, *Pxf = Pin.xf;
  const int* Pfi = Pin.fi;
  double bR[R], hiR[R], loR[R];
  int fiR[R];
#pragma unroll
  for (int q = 0; q < R; q++) {
    const int j = rowAt(q, lane);
    bR[q] = j < m ? Pb[j] : 0.0;
    hiR[q] = j < m ? Phi[j] : 0.0;
    loR[q] = j < m ? Plo[j] : 0.0;
    fiR[q] = j < m ? Pfi[j] : -1;
  }
  double scl[R];
  int rep[R];
  unsigned long long alive[R];
  // LCPUtils::reduce (BoxedLcpConstraintSolver.cpp:466-521).  On chip
  // (kLds) there is no room for a reduced matrix beside wave 0's fallbacks:
  // a merge hands Dantzig back to wave 0 (only whether reduce merges anything
  // is needed, the first merge settles it).  The wide kernel's HBM pool has
  // one: Dantzig runs on the reduced problem here (matrix in Mred, which this
  // wave's own PGS fallback reuses only after it), mapped out as wave 0 would
  // (x_i = x_r[rank(rep_i)]), and is validated on the full problem.
  waveReduceR<kLds, R>(m, spc<kLds>(PA), 0.0, bR, loR, hiR, fiR, lane, scl, rep, alive, kLds ? 1 : 128);
  const bool merged = !allRowsAlive<R>(m, alive);
  if (kLds && merged) {
    boardSet(ct, BD_D, 3, lane);
    return;
  }
#ifdef NIMBLE_STAGE_TIMING
  if (lane == 0 && g_stamp) g_stamp[94] = (double)__builtin_amdgcn_s_memtime();
  double* dbgD = g_stamp ? g_stamp + SLOT_DANTZIG : nullptr;
#else
  double* dbgD = nullptr;
#endif
  double xd[R];
#pragma unroll
  for (int q = 0; q < R; q++) xd[q] = 0.0;
  bool ok;
  if (!kLds && merged) {
    double br[R], lr[R], hr[R], xr[R];
    int fr[R], act[R];
#pragma unroll
    for (int q = 0; q < R; q++) { br[q] = bR[q]; lr[q] = loR[q]; hr[q] = hiR[q]; fr[q] = fiR[q]; }
    const int mr = reducedVectorsR<R>(alive, rep, lane, br, lr, hr, fr, act);
    reducedMatrixR<kLds, R>(m, spc<kLds>(PA), 0.0, alive, act, scl, Mred, false, lane);
    WSYNC();
    ok = waveDantzigR<kLds, R, false, true, kPL>(mr, Mred, Ldz, scrDz, xr, br, lr, hr, fr, lane, dbgD,
                                                 board(ct) + BD_STOPD, tallyOf(ct));
#pragma unroll
    for (int q = 0; q < R; q++) xd[q] = gatherR(xr, rankR(alive, rep[q]));
  } else {
    ok = waveDantzigR<kLds, R, false, true, kPL>(m, spc<kLds>(PA), Ldz, scrDz, xd, bR, loR, hiR, fiR, lane, dbgD,
                                                 board(ct) + BD_STOPD, tallyOf(ct));
  }
  bool nan = false;
#pragma unroll
  for (int q = 0; q < R; q++) nan = nan || (rowAt(q, lane) < m && isnan(xd[q]));
  ok = ok && !__ballot(nan);
  if (ok) ok = waveLcpValidR<kLds, R>(m, spc<kLds>(PA), 0.0, xd, bR, hiR, loR, fiR, false, lane);
#pragma unroll
  for (int q = 0; q < R; q++)
    if (rowAt(q, lane) < m) Pxh[rowAt(q, lane)] = xd[q];
  if (ok) {
    boardSet(ct, BD_STOPP, 1, lane);
    boardSet(ct, BD_STOPF, 1, lane);
  }
  boardSet(ct, BD_D, ok ? 1 : 2, lane);
#ifdef NIMBLE_STAGE_TIMING
  if (lane == 0 && g_stamp) { g_stamp[95] = (double)__builtin_amdgcn_s_memtime(); g_stamp[96] = ok ? 1 : 2; }
#endif
  // the fallbacks still open: the PGS fallback once the warm start is
  // final, the frictionless PGS unless the PGS fallback has succeeded
  const double cf = md.fallbackCfm;
  const long long t0 = spinClock();
  for (int it = 0; !ok; it++) {
    const bool pOpen = boardGet(ct, BD_PCLAIM) == 0 && !boardGet(ct, BD_STOPP);
    const bool fOpen = boardGet(ct, BD_FCLAIM) == 0 && !boardGet(ct, BD_STOPF) && boardGet(ct, BD_P) != 1;
    if (pOpen && boardGet(ct, BD_G) == 1) {
      if (boardClaim(ct, BD_PCLAIM, 2, lane)) {
#ifdef NIMBLE_STAGE_TIMING
        if (lane == 0 && g_stamp) { g_stamp[97] = 2; g_stamp[100] = (double)__builtin_amdgcn_s_memtime(); }
#endif
        bool dup;
        double xp[R];
        const bool okp = pgsFallbackR<kLds, R>(PA, Pxc, m, cf, bR, loR, hiR, fiR, Mred, lane, xp, dup,
                                               board(ct) + BD_STOPP, nullptr, tallyOf(ct));
#pragma unroll
        for (int q = 0; q < R; q++)
          if (rowAt(q, lane) < m) Pxp[rowAt(q, lane)] = xp[q];
        boardSet(ct, BD_PDUP, dup ? 1 : 0, lane);
        if (okp) boardSet(ct, BD_STOPF, 1, lane);
        boardSet(ct, BD_P, okp ? 1 : 2, lane);
#ifdef NIMBLE_STAGE_TIMING
        if (lane == 0 && g_stamp) g_stamp[101] = (double)__builtin_amdgcn_s_memtime();
#endif
      }
      continue;
    }
    if (fOpen) {
      if (boardClaim(ct, BD_FCLAIM, 2, lane)) {
#ifdef NIMBLE_STAGE_TIMING
        if (lane == 0 && g_stamp) { g_stamp[98] = 2; g_stamp[102] = (double)__builtin_amdgcn_s_memtime(); }
#endif
        double xf[R];
        frictionlessPgsR<kLds, R>(PA, Pb, Plo, Phi, m, cf, fiR, lane, xf, board(ct) + BD_STOPF, tallyOf(ct));
#pragma unroll
        for (int q = 0; q < R; q++)
          if (rowAt(q, lane) < m) Pxf[rowAt(q, lane)] = xf[q];
        boardSet(ct, BD_F, 1, lane);
#ifdef NIMBLE_STAGE_TIMING
        if (lane == 0 && g_stamp) g_stamp[103] = (double)__builtin_amdgcn_s_memtime();
#endif
      }
      continue;
    }
    if (!pOpen) break;
    // only the PGS fallback is open, waiting for the warm start
    if (guardForced(ct, GW_HELPER_WARM) || protocolFailed(ct) || spinExpired(t0, it)) {
      protocolFail(ct);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// the helper's post-answer share (HS_POST, see contactLcp), then its end of
// the world: POSTDONE, and wait until wave 0 has taken it
__device__ __forceinline__ void helperPostShare(const ModelDev& md, double* s, const Layout& L, double* ct, double* snap,
                                                int lane) {
  const int n = md.n;
  const int m = uni((int)ct[H_M]), nCon = uni((int)ct[H_NCON]), nc = uni((int)ct[H_NC]);
  const bool std2 = uni(helperFlags(ct)[1]) != 0;
  FwdPool P;
  carveFwd(s + L.pool, m, n, P);
  snap = gbl(snap);
  const double u = impulseDelta(P.massed, std2 ? P.X : P.xc, s + L.M, s + L.dinv, s + L.v1, snap, n, m, lane);
  if (lane < n) s[L.rhs + lane] = u;
  snapshotRows(P, ct, s + L.x, snap, nCon, m, nc, n, lane);
  if (nc > 0) snapshotAc(md, s, L, P, s + L.ct + CT_CONTACTS, snap + snAc(n), snap + snAcubE(n), m, nc, n, lane);
  helperPost(ct, HS_POSTDONE, lane);
  helperWait(ct, [](int v) { return v != HS_POSTDONE; }, GW_HELPER_IDLE);
}

// kWide: the wide kernel's helper (both board modes); the one-row kernel's
// only ever sees HB_LDS_POOL (a separate, smaller function: the wide mode's
// registers made every call save ~160 callee-saved VGPRs to scratch)
// (snap: the world's snapshot, for the one-row kernel's post-answer share)
template <bool kWide>
__device__ void helperWave(const ModelDev& md, double* s, const Layout& L, int lane, double* g_stamp, double* hbmPool,
                           double* snap) {
  (void)g_stamp;
  s = lds<true>(s);
  double* ct = s + L.ct;
  int st = helperWait(ct, [](int v) { return v == HS_TASK || v == HS_SKIP || (!kWide && v == HS_POST); },
                      GW_HELPER_TASK);
  if (st < 0) return;  // (the deadlock guard expired: wave 0 goes on alone)
  if (!kWide && st == HS_POST) {  // (no task went out)
    helperPostShare(md, s, L, ct, snap, lane);
    return;
  }
  if (st == HS_TASK) {
    // the cascade's Dantzig is on the world's critical path: the helper
    // competes for issue with the other world's step wave on its SIMD
    const int prio = md.helperPrio;
    if (prio == 1) __builtin_amdgcn_s_setprio(1);
    else if (prio == 2) __builtin_amdgcn_s_setprio(2);
    else if (prio == 3) __builtin_amdgcn_s_setprio(3);
    const int m = uni((int)ct[H_M]);
    const int mode = uni(helperFlags(ct)[1]);
    FwdPool P;
    if (kWide && mode == HB_WIDE) {
      carveFwd(gbl(hbmPool), m, md.n, P);
      lds_double* Ldz = (lds_double*)(s + L.pool);
      helperTask<false, 2, true>(md, ct, P, m, lane, Ldz, Ldz + dantzigLDoubles(m, true), sp<false>(P.M2), g_stamp);
    } else {
      carveFwd(s + L.pool, m, md.n, P);
      helperTask<true, 1>(md, ct, P, m, lane, sp<true>(P.M2), sp<true>(P.xh2), sp<true>(P.M2), g_stamp);
    }
  }
  __builtin_amdgcn_s_setprio(0);
  helperPost(ct, HS_DONE, lane);
  st = helperWait(ct, [](int v) { return v != HS_DONE; }, GW_HELPER_IDLE);
  if (!kWide && st == HS_POST) helperPostShare(md, s, L, ct, snap, lane);
}

// wave 0's end of a world's protocol: post SKIP if no task went out, collect
// DONE (a task has been stopped and collected in contactLcp already) and
// reset to IDLE
__device__ __forceinline__ void helperRetire(double* s, const Layout& L, int lane) {
  double* ct = lds<true>(s) + L.ct;
  if (helperState(ct) == HS_IDLE) helperPost(ct, HS_SKIP, lane);
  // (POSTDONE: a post-answer share taken, the helper has answered already)
  helperWait(ct, [](int v) { return v == HS_DONE || v == HS_POSTDONE; }, GW_RETIRE);
  helperPost(ct, HS_IDLE, lane);
}

// ===========================================================================
// Backward: the constraint terms of BackpropSnapshot::backprop as
// vector-Jacobian products.  With w = Minv gv, u = A_cubE^T w,
// lambda = (Q^+)^T u, beta = bounce .* lambda, mu = A_c beta, nu = Minv mu:
//   grad_tau = dt (w - nu)
//   grad_v   = gv - mu - dt (dC/dv + D + dt K)^T (w - nu)
//   grad_q   = -dt (dID(a*)/dq)^T (w - nu) - dt K (w - nu) - dt m(delta, nu)
//              + m(sigma, kappa) - [imprecise] (m(MA1, MArho) + m(MA2, MApi))
//              + sum_j G_j^T g_j
// where m(a, c) = (d(M a)/dq)^T c, G_j = d(J^T e_j)/dq
// (DifferentiableContactConstraint.cpp:1654) and g_j collects, per clamping /
// upper-bound row, the vectors multiplying G_j in
//   dA_c f  (BackpropSnapshot.cpp:1046), dB (getJacobianOfLCPOffsetClampingSubset
//   :3181), -Q^+ dQ(Q^+ b) and the pseudo-inverse gradient branch
//   (getJacobianOfConstraintForce :2723, :2960).
// ===========================================================================
enum { NV_DELTA = 0, NV_NU, NV_SIGMA, NV_KAPPA, NV_MA1, NV_MARHO, NV_MA2, NV_MAPI, NV_YF, NV_W, NV_W2, NV_MU, NV_T0 };


struct BwdPool {
  double *gRows, *TAB, *NV;
  double *fc, *bc, *bounce, *u, *lam, *beta, *xq, *rho, *piv, *zeta, *r1;
  int* rowOf;
};

__device__ inline void carveBwd(double* base, int m, int n, BwdPool& P) {
  double* p = base;
  P.gRows = p; p += n * m;
  P.TAB = p; p += 12 * m;
  P.NV = p; p += NV_COLS * n;
  P.fc = p; p += m;
  P.bc = p; p += m;
  P.bounce = p; p += m;
  P.u = p; p += m;
  P.lam = p; p += m;
  P.beta = p; p += m;
  P.xq = p; p += m;
  P.rho = p; p += m;
  P.piv = p; p += m;
  P.zeta = p; p += m;
  P.r1 = p; p += m;
  P.rowOf = reinterpret_cast<int*>(p);
}

// the dofs (bit r) whose joint moves body b: wave-uniform 64-bit mask
// (n <= NIMBLE_MAX_DOFS = 64), so loops over them skip the unrelated dofs
__device__ __forceinline__ unsigned long long ancestorDofMask(const ModelDev& md, unsigned long long bodies, int lane) {
  const bool in = lane < md.n && ((bodies >> md.dofBody[lane < md.n ? lane : 0]) & 1ull);
  return __ballot(in);
}

// twist of body `b` for joint velocity vector g (column `col` of X, ld):
// sum over ancestor dofs r of S_r g_r.  b < 0 -> 0.
__device__ inline void bodyTwist(const ModelDev& md, const double* Sw, int b, const double* g, int ld, double* T) {
  for (int i = 0; i < 6; i++) T[i] = 0.0;
  if (b < 0) return;
  const unsigned long long a = md.anc[b];
  // unpredicated: skipped dofs contribute fma(S, 0, T) = T
#pragma unroll 4
  for (int r = 0; r < md.n; r++) {
    const double gr = ((a >> md.dofBody[r]) & 1ull) ? g[r * ld] : 0.0;
    for (int i = 0; i < 6; i++) T[i] = fma(Sw[6 * r + i], gr, T[i]);
  }
}

// ContactConstraint::getTangentBasisMatrixODEGradient (ContactConstraint.cpp:772)
__device__ void tangentBasisGradient(const double* nrm, const double* g, double* T0, double* T1) {
  const double ez[3] = {0, 0, 1}, ex[3] = {1, 0, 0}, ey[3] = {0, 1, 0};
  const double* cr = ez;
  double t[3];
  cross3(cr, nrm, t);
  if (dot3(t, t) < 1e-12) {
    cr = ex; cross3(cr, nrm, t);
    if (dot3(t, t) < 1e-12) {
      cr = ey; cross3(cr, nrm, t);
      if (dot3(t, t) < 1e-12) { cr = ez; cross3(cr, nrm, t); }
    }
  }
  const double tn = sqrt(dot3(t, t));
  for (int i = 0; i < 3; i++) t[i] /= tn;
  double gc[3];
  cross3(cr, g, gc);
  for (int i = 0; i < 3; i++) gc[i] /= tn;
  double gt[3];
  if (fabs(tn - 1.0) > 1e-6) {
    const double dd = dot3(gc, t);
    for (int i = 0; i < 3; i++) gt[i] = gc[i] - dd * t[i];
  } else {
    for (int i = 0; i < 3; i++) gt[i] = gc[i];
  }
  double a[3], b[3];
  cross3(g, t, a);
  cross3(nrm, gt, b);
  for (int i = 0; i < 3; i++) { T0[i] = gt[i]; T1[i] = a[i] + b[i]; }
}

// Contact preparation of the backward from the snapshot's precomputed
// clamping data (backwardPrecompute).  The nine Minv products it needs are
// two batched register Cholesky solves:
//   batch 1: gv, A_cubE f_c, A_cubE x, A_c r1, A_c zeta -> w, dt*delta, sigma, MA1, MA2
//   batch 2: A_c beta, A_c lambda, A_cubE rho, A_cubE pi -> nu, kappa, MArho, MApi
// On return (all lanes): s[L.x] = a*, s[L.w] = w - nu, NV columns hold the
// M-derivative pairs and mu; P.gRows / P.TAB the per-row vectors of the
// G_j terms.  Returns the imprecise flag.
template <int R = 1>
__device__ int contactBackwardPrep(const ModelDev& md, double* s, const Layout& L, int lane, const double* sn,
                                   BwdPool& P, int m, int nc, double* ct, int fcRow) {
  const int n = md.n;
  const double dt = md.dt;
  const double* rows = sn + SN_ROWS;
  const double* Ac = sn + snAc(n);
  const double* AcubE = sn + snAcubE(n);
  const double* PT = sn + snPT(n);
  const double* Q = sn + snQ(n);
  const double* Lm = s + L.M;
  const double* dinv = s + L.dinv;
  const int imp = uni((int)sn[SN_IMP]);
#ifdef NIMBLE_STAGE_TIMING
  double* g_stamp = (double*)sn + snStamps(n);
#endif
  STAMP(30);
  (void)ct;
  for (int j = lane; j < m; j += WAVE)
    if ((int)rows[j * SN_ROWREC + RR_MAP] == CM_CLAMPING) P.rowOf[(int)rows[j * SN_ROWREC + RR_CIDX]] = j;
  WSYNC();
  for (int c = lane; c < nc; c += WAVE) {
    const int r = P.rowOf[c];
    P.fc[c] = sn[SN_FC + c];
    P.bc[c] = rows[r * SN_ROWREC + RR_B];
    P.bounce[c] = rows[r * SN_ROWREC + RR_BOUNCE];
  }
  WSYNC();
  // x = P b ; r1 = b - Q x ; zeta = P^T x
  for (int c = lane; c < nc; c += WAVE) {
    double xx = 0;
#pragma unroll 8
    for (int r = 0; r < nc; r++) xx += PT[r * nc + c] * P.bc[r];
    P.xq[c] = xx;
  }
  WSYNC();
  for (int c = lane; c < nc; c += WAVE) {
    double qx = 0, ze = 0;
    if (imp)
#pragma unroll 8
      for (int k = 0; k < nc; k++) {
        qx += Q[c * nc + k] * P.xq[k];
        ze += PT[c * nc + k] * P.xq[k];
      }
    P.r1[c] = imp ? P.bc[c] - qx : 0.0;
    P.zeta[c] = imp ? ze : 0.0;
  }
  WSYNC();
  STAMP(31);
  // batch 1
  {
    double X[5] = {0, 0, 0, 0, 0};
    if (lane < n) {
      X[0] = s[L.gv + lane];
      double a1 = 0, a2 = 0, a3 = 0, a4 = 0;
#pragma unroll 8
      for (int c = 0; c < nc; c++) {
        const double ae = AcubE[lane * nc + c], ac = Ac[lane * nc + c];
        a1 += ae * P.fc[c];
        a2 += ae * P.xq[c];
        a3 += ac * P.r1[c];
        a4 += ac * P.zeta[c];
      }
      X[1] = a1; X[2] = a2; X[3] = a3; X[4] = a4;
    }
    cholSolveReg<5>(Lm, dinv, X, n, lane);
    if (lane < n) {
      double* nv = P.NV + lane * NV_COLS;
      const double d = X[1] / dt;
      nv[NV_W] = X[0];
      nv[NV_DELTA] = d;
      nv[NV_SIGMA] = X[2];
      nv[NV_MA1] = X[3];
      nv[NV_MA2] = X[4];
      s[L.w + lane] = X[0];
      s[L.x + lane] = sn[snYf(n) + lane] + d;
    }
  }
  WSYNC();
  // u = A_c_ub_E^T w (the adjoint of f_c; e_fcRow for getJacobianOfConstraintForce
  // rows) ; lambda = P^T u ; beta ; rho = P lambda ; pi = u - Q^T lambda
  for (int c = lane; c < nc; c += WAVE) {
    double acc = 0;
#pragma unroll 8
    for (int i = 0; i < n; i++) acc += AcubE[i * nc + c] * s[L.w + i];
    P.u[c] = fcRow >= 0 ? (c == fcRow ? 1.0 : 0.0) : acc;
  }
  WSYNC();
  for (int c = lane; c < nc; c += WAVE) {
    double l = 0;
#pragma unroll 8
    for (int r = 0; r < nc; r++) l += PT[c * nc + r] * P.u[r];
    P.lam[c] = l;
    P.beta[c] = P.bounce[c] * l;
  }
  WSYNC();
  for (int c = lane; c < nc; c += WAVE) {
    double qtl = 0, rh = 0;
    if (imp)
#pragma unroll 8
      for (int k = 0; k < nc; k++) {
        qtl += Q[k * nc + c] * P.lam[k];
        rh += PT[k * nc + c] * P.lam[k];
      }
    P.piv[c] = imp ? P.u[c] - qtl : 0.0;
    P.rho[c] = imp ? rh : 0.0;
  }
  WSYNC();
  STAMP(35);
  // batch 2
  {
    double X[4] = {0, 0, 0, 0};
    double mu = 0;
    if (lane < n) {
      double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
#pragma unroll 8
      for (int c = 0; c < nc; c++) {
        const double ae = AcubE[lane * nc + c], ac = Ac[lane * nc + c];
        a0 += ac * P.beta[c];
        a1 += ac * P.lam[c];
        a2 += ae * P.rho[c];
        a3 += ae * P.piv[c];
      }
      X[0] = a0; X[1] = a1; X[2] = a2; X[3] = a3;
      mu = a0;
    }
    cholSolveReg<4>(Lm, dinv, X, n, lane);
    if (lane < n) {
      double* nv = P.NV + lane * NV_COLS;
      nv[NV_MU] = mu;
      nv[NV_NU] = X[0];
      nv[NV_KAPPA] = X[1];
      nv[NV_MARHO] = X[2];
      nv[NV_MAPI] = X[3];
      const double w2 = nv[NV_W] - X[0];
      nv[NV_W2] = w2;
      s[L.w + lane] = w2;
    }
  }
  WSYNC();
  STAMP(37);
  // per-row vectors g_j (lane = dof i, rows wave-uniform).  Each row's map,
  // clamping index and E value are loaded once, lane = row, and read back
  // with readlane: no dependent snapshot loads inside the row loop.
  int rMap[R], rC[R];
  double rE[R];
#pragma unroll
  for (int q = 0; q < R; q++) {
    const int j = rowAt(q, lane);
    rMap[q] = CM_NOT_CLAMPING;
    rC[q] = 0;
    rE[q] = 0.0;
    if (j < m) {
      const double* rr = rows + j * SN_ROWREC;
      rMap[q] = (int)rr[RR_MAP];
      if (rMap[q] == CM_CLAMPING) rC[q] = (int)rr[RR_CIDX];
      else if (rMap[q] >= 0) { rC[q] = (int)rows[rMap[q] * SN_ROWREC + RR_CIDX]; rE[q] = rr[RR_EVAL]; }
    }
  }
  // (lane = dof i: n <= NIMBLE_MAX_DOFS = 64, one dof per lane; the row
  // reads stay outside the lane-divergent part)
  {
    const int i = lane;
    const bool live = i < n;
    const double* nv = P.NV + (live ? i : 0) * NV_COLS;
    const double w = nv[NV_W], sg = nv[NV_SIGMA], ka = nv[NV_KAPPA], ma1 = nv[NV_MA1], mar = nv[NV_MARHO];
    const double ma2 = nv[NV_MA2], map = nv[NV_MAPI], vf = sn[SN_VF + (live ? i : 0)];
    for (int j = 0; j < m; j++) {
      const int mp = rdliR(rMap, j);
      const int c = rdliR(rC, j);
      const double e = rdlR(rE, j);
      double g = 0.0;
      if (mp == CM_CLAMPING) {
        g = P.fc[c] * w - P.beta[c] * vf - P.lam[c] * sg - P.xq[c] * ka;
        if (imp) g += P.rho[c] * ma1 + P.r1[c] * mar + P.piv[c] * ma2 + P.zeta[c] * map;
      } else if (mp >= 0) {
        double inner = P.fc[c] * w - P.xq[c] * ka;
        if (imp) inner += P.rho[c] * ma1 + P.piv[c] * ma2;
        g = e * inner;
      }
      if (live) P.gRows[j * n + i] = g;
    }
  }
  WSYNC();
  // T_A(g_j), T_B(g_j): lane = (row, side) -- 2m of them, in passes of 64 --
  // summed over the dofs that move any contact body (the others have weight
  // 0 for every lane)
  {
    auto bodyOf = [&](int t) {
      if (t >= 2 * m) return -1;
      const double* rec = sn + SN_CONTACTS + (int)rows[(t >> 1) * SN_ROWREC + RR_CONTACT] * CREC;
      return (int)rec[8 + (t & 1)];
    };
    // union over all rows of the ancestor sets
    unsigned long long anAll = 0ull;
    for (int t = lane; t < 2 * m; t += WAVE) {
      const int body = bodyOf(t);
      if (body >= 0) anAll |= md.anc[body];
    }
    unsigned lo = (unsigned)anAll, hi = (unsigned)(anAll >> 32);
    for (int o = 32; o >= 1; o >>= 1) {
      lo |= __shfl_xor(lo, o);
      hi |= __shfl_xor(hi, o);
    }
    const unsigned long long all = ((unsigned long long)uni((int)hi) << 32) | (unsigned)uni((int)lo);
    const unsigned long long dmAll = ancestorDofMask(md, all, lane);
    for (int t0 = 0; t0 < 2 * m; t0 += WAVE) {
      const int t = t0 + lane;
      const int body = bodyOf(t);
      const unsigned long long an = body >= 0 ? md.anc[body] : 0ull;
      unsigned long long dm = dmAll;
      double T[6] = {0, 0, 0, 0, 0, 0};
      const double* g = P.gRows + (t < 2 * m ? (t >> 1) : 0) * n;
      while (dm) {
        const int r = __ffsll((long long)dm) - 1;
        dm &= dm - 1ull;
        // bodyTwist's arithmetic: fma(S_r, g_r, T) for the ancestor dofs
        const double gr = ((an >> md.dofBody[r]) & 1ull) ? g[r] : 0.0;
        for (int i = 0; i < 6; i++) T[i] = fma(s[L.Sw + 6 * r + i], gr, T[i]);
      }
      if (t < 2 * m)
        for (int i = 0; i < 6; i++) P.TAB[(t >> 1) * 12 + (t & 1) * 6 + i] = T[i];
    }
  }
  WSYNC();
  STAMP(38);
  return imp;
}

// Sphere-box contact rows (SPHERE_BOX / BOX_SPHERE): the full derivative
// (T_A - T_B) . [p x dd + dp x d; dd] for dof k, with the contact position
// and normal gradients of DifferentiableContactConstraint.cpp:353 (SPHERE_TO_BOX:
// the sphere centre's motion with the locked box-face components removed),
// :376 (BOX_TO_SPHERE), :640/:672 (normal gradients) and :1092 (friction
// directions).  Locked face normals are the box's world axes (type field:
// mask << 4, box shape << 8).
__device__ double sphereRowTerm(const ModelDev& md, const double* s, const Layout& L, const BwdPool& P, int j,
                                const double* rec, const double* rr, const double* Z, int bk) {
  const int A = (int)rec[8], B = (int)rec[9], typ = (int)rec[7], type = typ & 15;
  const bool pa = (md.anc[A] >> bk) & 1ull, pb = (md.anc[B] >> bk) & 1ull;
  if (pa == pb) return 0.0;  // unrelated dof (self-collision is off by default)
  const bool sphereToBox = type == CT_SPHERE_BOX ? pa : pb;
  const int mask = (typ >> 4) & 7, shape = typ >> 8;
  const double* p = rec;
  const double* nrm = rec + 3;
  const double* c = rec + 10;
  const double wv[3] = {Z[0], Z[1], Z[2]};
  const bool rotates = sqrt(Z[0] * Z[0] + Z[1] * Z[1] + Z[2] * Z[2]) > 1e-6;
  // gradientWrtTheta(Z, x, 0) (dart/math/Geometry.cpp:968)
  auto gwt = [&](const double* x, double* o) {
    if (rotates) { cross3(wv, x, o); for (int i = 0; i < 3; i++) o[i] += Z[3 + i]; }
    else { for (int i = 0; i < 3; i++) o[i] = Z[3 + i]; }
  };
  auto lockProject = [&](double* x) {
    if (!mask) return;
    const double* Tw = s + L.Tw + 12 * md.shapeBody[shape];
    const double* Ts = md.shapeT[shape];
    for (int f = 0; f < 3; f++) {
      if (!((mask >> f) & 1)) continue;
      double fn[3];
      for (int r = 0; r < 3; r++) fn[r] = Tw[4 * r] * Ts[f] + Tw[4 * r + 1] * Ts[4 + f] + Tw[4 * r + 2] * Ts[8 + f];
      const double d0 = dot3(fn, x);
      for (int i = 0; i < 3; i++) x[i] -= fn[i] * d0;
    }
  };
  double sg[3], dp[3], dn[3];
  gwt(c, sg);
  double dist2 = 0.0;
  for (int i = 0; i < 3; i++) dist2 += (c[i] - p[i]) * (c[i] - p[i]);
  const double norm = sqrt(dist2);
  const double inv = norm > 1e-5 ? 1.0 / norm : 1.0;
  if (sphereToBox) {
    for (int i = 0; i < 3; i++) dp[i] = sg[i];
    lockProject(dp);
    for (int i = 0; i < 3; i++) {
      const double cpg = dp[i] * inv, spg = sg[i] * inv;
      dn[i] = type == CT_BOX_SPHERE ? cpg - spg : spg - cpg;
    }
  } else {
    double neg[3], pg[3];
    for (int i = 0; i < 3; i++) neg[i] = -sg[i];
    lockProject(neg);
    gwt(p, pg);
    for (int i = 0; i < 3; i++) {
      dp[i] = pg[i] + neg[i];
      dn[i] = type == CT_BOX_SPHERE ? dp[i] * inv : -dp[i] * inv;
    }
  }
  const double dnn = dot3(dn, nrm);
  for (int i = 0; i < 3; i++) dn[i] -= dnn * nrm[i];
  double dd[3];
  const int dirIdx = (int)rr[RR_DIR];
  if (dirIdx == 0 || dot3(dn, dn) <= 1e-12) {
    for (int i = 0; i < 3; i++) dd[i] = dn[i];
  } else {
    double T0[3], T1[3];
    tangentBasisGradient(nrm, dn, T0, T1);
    for (int i = 0; i < 3; i++) dd[i] = dirIdx == 1 ? T0[i] : T1[i];
  }
  const double* d = rr + RR_D;
  double pxdd[3], dpxd[3];
  cross3(p, dd, pxdd);
  cross3(dp, d, dpxd);
  double v = 0.0;
  for (int i = 0; i < 3; i++)
    v += (P.TAB[j * 12 + i] - P.TAB[j * 12 + 6 + i]) * (pxdd[i] + dpxd[i]) +
         (P.TAB[j * 12 + 3 + i] - P.TAB[j * 12 + 9 + i]) * dd[i];
  return v;
}

// SPHERE_SPHERE rows (SPHERE_A / SPHERE_B of DifferentiableContactConstraint.cpp
// :343 / :348 and :625 / :634): the contact point moves with the dof's
// sphere centre weighted by the other radius, the normal with that centre
// over the centre distance, projected off the normal.  E = centre B,
// radius A, radius B (centre A is the record's sphere centre).
__device__ double sphereSphereRowTerm(const ModelDev& md, const BwdPool& P, int j, const double* rec,
                                      const double* rr, const double* E, const double* Z, int bk, int A, int B) {
  const bool pa = (md.anc[A] >> bk) & 1ull, pb = (md.anc[B] >> bk) & 1ull;
  if (pa == pb) return 0.0;
  const double* nrm = rec + 3;
  const double* cA = rec + 10;
  const double* cen = pa ? cA : E;
  const double wt = (pa ? E[4] : E[3]) / (E[3] + E[4]);
  const double wv[3] = {Z[0], Z[1], Z[2]};
  double g[3];
  if (sqrt(Z[0] * Z[0] + Z[1] * Z[1] + Z[2] * Z[2]) > 1e-6) {  // gradientWrtTheta (Geometry.cpp:968)
    cross3(wv, cen, g);
    for (int i = 0; i < 3; i++) g[i] += Z[3 + i];
  } else {
    for (int i = 0; i < 3; i++) g[i] = Z[3 + i];
  }
  double dp[3], dn[3], dist2 = 0.0;
  for (int i = 0; i < 3; i++) { dp[i] = wt * g[i]; dist2 += (cA[i] - E[i]) * (cA[i] - E[i]); }
  const double norm = sqrt(dist2);
  for (int i = 0; i < 3; i++) dn[i] = g[i] / norm;
  const double dnn = dot3(dn, nrm);
  for (int i = 0; i < 3; i++) dn[i] = (pa ? 1.0 : -1.0) * (dn[i] - dnn * nrm[i]);
  double dd[3];
  const int dirIdx = (int)rr[RR_DIR];
  if (dirIdx == 0 || dot3(dn, dn) <= 1e-12) {
    for (int i = 0; i < 3; i++) dd[i] = dn[i];
  } else {
    double T0[3], T1[3];
    tangentBasisGradient(nrm, dn, T0, T1);
    for (int i = 0; i < 3; i++) dd[i] = dirIdx == 1 ? T0[i] : T1[i];
  }
  const double* d = rr + RR_D;
  const double* p = rec;
  double pxdd[3], dpxd[3];
  cross3(p, dd, pxdd);
  cross3(dp, d, dpxd);
  double v = 0.0;
  for (int i = 0; i < 3; i++)
    v += (P.TAB[j * 12 + i] - P.TAB[j * 12 + 6 + i]) * (pxdd[i] + dpxd[i]) +
         (P.TAB[j * 12 + 3 + i] - P.TAB[j * 12 + 9 + i]) * dd[i];
  return v;
}

// SPHERE_PIPE / PIPE_SPHERE rows: SPHERE_TO_PIPE (DifferentiableContactConstraint.cpp
// :484 point, :819 normal) moves the point with the sphere centre, its
// off-axis part weighted by the pipe radius; PIPE_TO_SPHERE (:496, :837) with
// the axis point closest to the sphere centre (math::closestPointOnLineGradient,
// Geometry.cpp:4427) weighted by the sphere radius.  E = pipe closest point,
// pipe fixed point, pipe direction, sphere radius, pipe radius.
__device__ double spherePipeRowTerm(const ModelDev& md, const BwdPool& P, int j, const double* rec,
                                    const double* rr, const double* E, const double* Z, int bk, int A, int B,
                                    int type) {
  const bool pa = (md.anc[A] >> bk) & 1ull, pb = (md.anc[B] >> bk) & 1ull;
  if (pa == pb) return 0.0;
  const bool sphereSide = type == CT_SPHERE_PIPE ? pa : pb;
  const double* nrm = rec + 3;
  const double* sc = rec + 10;
  const double* cl = E;
  const double* fx = E + 3;
  const double* dir = E + 6;
  const double sR = E[9], pR = E[10];
  const double wv[3] = {Z[0], Z[1], Z[2]};
  const bool rotates = sqrt(Z[0] * Z[0] + Z[1] * Z[1] + Z[2] * Z[2]) > 1e-6;
  auto gwt = [&](const double* x, double* o) {
    if (rotates) { cross3(wv, x, o); for (int i = 0; i < 3; i++) o[i] += Z[3 + i]; }
    else { for (int i = 0; i < 3; i++) o[i] = Z[3 + i]; }
  };
  double g[3], dp[3], dn[3];
  if (sphereSide) {
    gwt(sc, g);
    const double par = dot3(dir, g);
    const double wt = pR / (sR + pR);
    for (int i = 0; i < 3; i++) { dp[i] = par * dir[i] + wt * (g[i] - par * dir[i]); dn[i] = g[i] - par * dir[i]; }
  } else {
    double fg[3], dg[3];
    gwt(fx, fg);
    cross3(wv, dir, dg);
    double off = 0, dOff = 0, gOff = 0, dGOff = 0;
    for (int i = 0; i < 3; i++) {
      off += dir[i] * fx[i];
      dOff += dg[i] * fx[i] + dir[i] * fg[i];
      gOff += dir[i] * sc[i];
      dGOff += dg[i] * sc[i];
    }
    const double rel = gOff - off, dRel = dGOff - dOff;
    for (int i = 0; i < 3; i++) g[i] = fg[i] + rel * dg[i] + dRel * dir[i];
    const double wt = sR / (sR + pR);
    for (int i = 0; i < 3; i++) { dp[i] = wt * g[i]; dn[i] = g[i]; }
  }
  double dist2 = 0.0;
  for (int i = 0; i < 3; i++) dist2 += (cl[i] - sc[i]) * (cl[i] - sc[i]);
  const double norm = sqrt(dist2);
  for (int i = 0; i < 3; i++) dn[i] /= norm;
  const double dnn = dot3(dn, nrm);
  const bool plus = sphereSide ? type == CT_SPHERE_PIPE : type == CT_PIPE_SPHERE;
  for (int i = 0; i < 3; i++) dn[i] = (plus ? 1.0 : -1.0) * (dn[i] - dnn * nrm[i]);
  double dd[3];
  const int dirIdx = (int)rr[RR_DIR];
  if (dirIdx == 0 || dot3(dn, dn) <= 1e-12) {
    for (int i = 0; i < 3; i++) dd[i] = dn[i];
  } else {
    double T0[3], T1[3];
    tangentBasisGradient(nrm, dn, T0, T1);
    for (int i = 0; i < 3; i++) dd[i] = dirIdx == 1 ? T0[i] : T1[i];
  }
  const double* d = rr + RR_D;
  const double* p = rec;
  double pxdd[3], dpxd[3];
  cross3(p, dd, pxdd);
  cross3(dp, d, dpxd);
  double v = 0.0;
  for (int i = 0; i < 3; i++)
    v += (P.TAB[j * 12 + i] - P.TAB[j * 12 + 6 + i]) * (pxdd[i] + dpxd[i]) +
         (P.TAB[j * 12 + 3 + i] - P.TAB[j * 12 + 9 + i]) * dd[i];
  return v;
}

// math::getContactPointGradient (dart/math/Geometry.cpp:1129), radii 1: the
// derivative of the midpoint of the two edges' closest approach
__device__ inline void edgeContactPointGradient(const double* pA, const double* dpA, const double* uA,
                                                const double* duA, const double* pB, const double* dpB,
                                                const double* uB, const double* duB, double* out, double rA = 1.0, double rB = 1.0) {
  double p[3], d_p[3];
  for (int i = 0; i < 3; i++) { p[i] = pB[i] - pA[i]; d_p[i] = dpB[i] - dpA[i]; }
  const double uaub = dot3(uA, uB);
  const double d_uaub = dot3(duA, uB) + dot3(uA, duB);
  const double q1 = dot3(uA, p);
  const double d_q1 = dot3(duA, p) + dot3(uA, d_p);
  const double q2 = -dot3(uB, p);
  const double d_q2 = -dot3(duB, p) - dot3(uB, d_p);
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

// PIPE_PIPE rows (PIPE_A / PIPE_B of DifferentiableContactConstraint.cpp:510 /
// :529 and :862 / :901): getContactPointGradient of the moving axis with the
// contact's normalised radii for the point, and the two closest points'
// gradients (radii 0/1, 1/0) over their distance for the normal.
// E = edge A fixed point, edge A dir, edge B fixed point, edge B dir; the
// record holds radius A / rsum, the distance, radius B / rsum at [10..12].
__device__ double pipePipeRowTerm(const ModelDev& md, const BwdPool& P, int j, const double* rec, const double* rr,
                                  const double* E, const double* Z, int bk, int A, int B) {
  const bool pa = (md.anc[A] >> bk) & 1ull, pb = (md.anc[B] >> bk) & 1ull;
  if (pa == pb) return 0.0;
  const double* nrm = rec + 3;
  const double* aF = E;
  const double* aD = E + 3;
  const double* bF = E + 6;
  const double* bD = E + 9;
  const double wv[3] = {Z[0], Z[1], Z[2]};
  double fg[3], dg[3];
  const double* x = pa ? aF : bF;
  if (sqrt(Z[0] * Z[0] + Z[1] * Z[1] + Z[2] * Z[2]) > 1e-6) {
    cross3(wv, x, fg);
    for (int i = 0; i < 3; i++) fg[i] += Z[3 + i];
  } else {
    for (int i = 0; i < 3; i++) fg[i] = Z[3 + i];
  }
  cross3(wv, pa ? aD : bD, dg);
  const double zero[3] = {0, 0, 0};
  const double* dpA = pa ? fg : zero;
  const double* duA = pa ? dg : zero;
  const double* dpB = pa ? zero : fg;
  const double* duB = pa ? zero : dg;
  double dp[3], ca[3], cb[3], dn[3];
  edgeContactPointGradient(aF, dpA, aD, duA, bF, dpB, bD, duB, dp, rec[10], rec[12]);
  edgeContactPointGradient(aF, dpA, aD, duA, bF, dpB, bD, duB, ca, 0.0, 1.0);
  edgeContactPointGradient(aF, dpA, aD, duA, bF, dpB, bD, duB, cb, 1.0, 0.0);
  for (int i = 0; i < 3; i++) dn[i] = (ca[i] - cb[i]) / rec[11];
  const double dnn = dot3(dn, nrm);
  for (int i = 0; i < 3; i++) dn[i] -= dnn * nrm[i];
  double dd[3];
  const int dirIdx = (int)rr[RR_DIR];
  if (dirIdx == 0 || dot3(dn, dn) <= 1e-12) {
    for (int i = 0; i < 3; i++) dd[i] = dn[i];
  } else {
    double T0[3], T1[3];
    tangentBasisGradient(nrm, dn, T0, T1);
    for (int i = 0; i < 3; i++) dd[i] = dirIdx == 1 ? T0[i] : T1[i];
  }
  const double* d = rr + RR_D;
  const double* p = rec;
  double pxdd[3], dpxd[3];
  cross3(p, dd, pxdd);
  cross3(dp, d, dpxd);
  double v = 0.0;
  for (int i = 0; i < 3; i++)
    v += (P.TAB[j * 12 + i] - P.TAB[j * 12 + 6 + i]) * (pxdd[i] + dpxd[i]) +
         (P.TAB[j * 12 + 3 + i] - P.TAB[j * 12 + 9 + i]) * dd[i];
  return v;
}

// PIPE_VERTEX / VERTEX_PIPE and PIPE_EDGE / EDGE_PIPE rows (the capsule-box
// vertex-pipe, edge-pipe and face-edge contacts).  getDofContactType (:166,
// :213): a dof moving the pipe side gives PIPE_TO_VERTEX (point fixed, :334;
// normal :967 -- math::closestPointOnLineGradient of the axis point nearest
// the vertex) / PIPE_TO_EDGE (:538, :1029); moving the mesh side
// VERTEX_TO_PIPE (the vertex moves, :408; normal :940) / EDGE_TO_PIPE (:555,
// :1075).  The edge cases go through math::getContactPointGradient with
// radii (0, 1) -- the contact point -- and (1, 0).  Record: [10..12] pipe
// closest point; E = pipe fixed point, pipe dir (vertex types) or edge A
// fixed point, edge A dir, pipe fixed point, pipe dir (edge types).
__device__ double pipeMeshRowTerm(const ModelDev& md, const BwdPool& P, int j, const double* rec, const double* rr,
                                  const double* E, const double* Z, int bk, int A, int B, int type) {
  const bool pa = (md.anc[A] >> bk) & 1ull, pb = (md.anc[B] >> bk) & 1ull;
  if (pa == pb) return 0.0;
  const bool vertexType = type == CT_PIPE_VERTEX || type == CT_VERTEX_PIPE;
  const bool pipeFirst = type == CT_PIPE_VERTEX || type == CT_PIPE_EDGE;
  const bool pipeMoves = pa == pipeFirst;
  const double* nrm = rec + 3;
  const double* p = rec;
  const double* pcl = rec + 10;
  const double wv[3] = {Z[0], Z[1], Z[2]};
  const bool rotates = sqrt(Z[0] * Z[0] + Z[1] * Z[1] + Z[2] * Z[2]) > 1e-6;
  auto gwt = [&](const double* x, double* o) {
    if (rotates) { cross3(wv, x, o); for (int i = 0; i < 3; i++) o[i] += Z[3 + i]; }
    else { for (int i = 0; i < 3; i++) o[i] = Z[3 + i]; }
  };
  double dp[3], dn[3];
  if (vertexType) {
    const double* pf = E;
    const double* dir = E + 3;
    double g[3] = {0, 0, 0}, fg[3] = {0, 0, 0}, dg[3] = {0, 0, 0};
    if (pipeMoves) { gwt(pf, fg); cross3(wv, dir, dg); }
    else gwt(p, g);
    double off = 0, dOff = 0, gOff = 0, dGOff = 0;
    for (int i = 0; i < 3; i++) {
      off += dir[i] * pf[i];
      dOff += dg[i] * pf[i] + dir[i] * fg[i];
      gOff += dir[i] * p[i];
      dGOff += dg[i] * p[i] + dir[i] * g[i];
    }
    const double rel = gOff - off, dRel = dGOff - dOff;
    double dist2 = 0.0;
    for (int i = 0; i < 3; i++) dist2 += (pcl[i] - p[i]) * (pcl[i] - p[i]);
    const double inv = 1.0 / sqrt(dist2);
    for (int i = 0; i < 3; i++) {
      dp[i] = g[i];
      dn[i] = (fg[i] + rel * dg[i] + dRel * dir[i] - g[i]) * inv;
    }
  } else {
    const double *ef = E, *ed = E + 3, *pf = E + 6, *pd = E + 9;
    double fg[3], dg[3], other[3];
    const double zero[3] = {0, 0, 0};
    gwt(pipeMoves ? pf : ef, fg);
    cross3(wv, pipeMoves ? pd : ed, dg);
    const double* dpE = pipeMoves ? zero : fg;
    const double* duE = pipeMoves ? zero : dg;
    const double* dpP = pipeMoves ? fg : zero;
    const double* duP = pipeMoves ? dg : zero;
    edgeContactPointGradient(ef, dpE, ed, duE, pf, dpP, pd, duP, dp, 0.0, 1.0);
    edgeContactPointGradient(ef, dpE, ed, duE, pf, dpP, pd, duP, other, 1.0, 0.0);
    double dist2 = 0.0;
    for (int i = 0; i < 3; i++) dist2 += (p[i] - pcl[i]) * (p[i] - pcl[i]);
    const double inv = 1.0 / sqrt(dist2);
    for (int i = 0; i < 3; i++) dn[i] = (other[i] - dp[i]) * inv;
  }
  const double dnn = dot3(dn, nrm);
  const double sg = pipeFirst ? 1.0 : -1.0;
  for (int i = 0; i < 3; i++) dn[i] = sg * (dn[i] - dnn * nrm[i]);
  double dd[3];
  const int dirIdx = (int)rr[RR_DIR];
  if (dirIdx == 0 || dot3(dn, dn) <= 1e-12) {
    for (int i = 0; i < 3; i++) dd[i] = dn[i];
  } else {
    double T0[3], T1[3];
    tangentBasisGradient(nrm, dn, T0, T1);
    for (int i = 0; i < 3; i++) dd[i] = dirIdx == 1 ? T0[i] : T1[i];
  }
  const double* d = rr + RR_D;
  double pxdd[3], dpxd[3];
  cross3(p, dd, pxdd);
  cross3(dp, d, dpxd);
  double v = 0.0;
  for (int i = 0; i < 3; i++)
    v += (P.TAB[j * 12 + i] - P.TAB[j * 12 + 6 + i]) * (pxdd[i] + dpxd[i]) +
         (P.TAB[j * 12 + 3 + i] - P.TAB[j * 12 + 9 + i]) * dd[i];
  return v;
}

// G-term of an EDGE_EDGE row for direction k (position generator Z) when
// k's joint moves exactly one of the two bodies: EDGE_A / EDGE_B contact
// position gradient (DifferentiableContactConstraint.cpp:412 / :429) and
// normal gradient (:708 / :722, not renormalised, as in the reference), the
// tangent directions following through the tangent-basis gradient (:1092).
// E: edgeAFixedPoint, edgeADir, edgeBFixedPoint, edgeBDir of the contact.
__device__ double edgeRowTerm(const ModelDev& md, const BwdPool& P, int j, const double* rec, const double* rr,
                              const double* E, const double* Z, int bk, int A, int B) {
  const bool inA = (md.anc[A] >> bk) & 1ull, inB = (md.anc[B] >> bk) & 1ull;
  if (inA == inB) return 0.0;  // neither body moves (self-collision pairs are not generated)
  const double* eaF = E;
  const double* eaD = E + 3;
  const double* ebF = E + 6;
  const double* ebD = E + 9;
  const double wv[3] = {Z[0], Z[1], Z[2]}, vv[3] = {Z[3], Z[4], Z[5]};
  double fg[3], dg[3];
  const double* fx = inA ? eaF : ebF;
  if (sqrt(dot3(wv, wv)) > 1e-6) {  // math::gradientWrtTheta
    cross3(wv, fx, fg);
    for (int i = 0; i < 3; i++) fg[i] += vv[i];
  } else {
    for (int i = 0; i < 3; i++) fg[i] = vv[i];
  }
  cross3(wv, inA ? eaD : ebD, dg);  // math::gradientWrtThetaPureRotation
  const double zero[3] = {0, 0, 0};
  double dp[3];
  edgeContactPointGradient(eaF, inA ? fg : zero, eaD, inA ? dg : zero, ebF, inA ? zero : fg, ebD, inA ? zero : dg,
                           dp);
  const double* nrm = rec + 3;
  double nb[3];
  cross3(ebD, eaD, nb);
  const double sign = dot3(nb, nrm) < 0 ? -1.0 : 1.0;
  double dn[3];
  if (inA) cross3(ebD, dg, dn);
  else cross3(dg, eaD, dn);
  for (int i = 0; i < 3; i++) dn[i] *= sign;
  const int dirIdx = (int)rr[RR_DIR];
  double dd[3];
  if (dirIdx == 0 || dot3(dn, dn) <= 1e-12) {
    for (int i = 0; i < 3; i++) dd[i] = dn[i];
  } else {
    double T0[3], T1[3];
    tangentBasisGradient(nrm, dn, T0, T1);
    for (int i = 0; i < 3; i++) dd[i] = dirIdx == 1 ? T0[i] : T1[i];
  }
  const double* p = rec;
  const double* d = rr + RR_D;
  double t1[3], t2[3];
  cross3(dp, d, t1);
  cross3(p, dd, t2);
  double v = 0.0;
  for (int i = 0; i < 3; i++)
    v += (P.TAB[j * 12 + i] - P.TAB[j * 12 + 6 + i]) * (t1[i] + t2[i]) +
         (P.TAB[j * 12 + 3 + i] - P.TAB[j * 12 + 9 + i]) * dd[i];
  return v;
}

// sum_j (G_j^T g_j)[k] for every direction k (lane k, position generator Z),
// G_j = d(J^T e_j)/dq (DifferentiableContactConstraint.cpp:1654), grouped by
// contact body c instead of by row:
//   screw-axis part  (Z x Y_j).wr_j = Z.(Y_j x* wr_j) summed over the rows of
//     c gives Z.(P^c_c - P^c_lambda(k)) with P^c_b = sum over the ancestor
//     dofs r of b of S_r x* omega^c_r, omega^c_r = sum_j s_j g_j[r] wr_j
//     (s_j = +1 when c is the row's body A, -1 for body B);
//   vertex side      (T_A - T_B).[dp x d; 0] with dp = Z_w x p + Z_v gives
//     Z_w.V^c + Z_v.U^c, U^c = sum_j d_j x Tw_j, V^c = sum_j p_j x (d_j x Tw_j)
//     (the Z_w term only when |Z_w| > 1e-6, DifferentiableContactConstraint.cpp:328);
//   face side        per row (tangent-basis gradient, ContactConstraint.cpp:772).
// `ws` is workspace of 6 n + 6 nb + 16 doubles.  Returns the lane's sum.
template <int R = 1>
__device__ double contactGTermsAll(const ModelDev& md, double* s, const Layout& L, const double* sn,
                                   const BwdPool& P, int m, const double* Z, double* ws, int lane,
                                   double* g_stamp = nullptr) {
  (void)g_stamp;
  const int n = md.n, nb = md.nb;
  const double* rows = sn + SN_ROWS;
  double* omega = ws;            // n x 6
  double* Pc = ws + 6 * n;       // nb x 6
  double* UV = Pc + 6 * nb;      // 6 (+ group body)
  const int k = lane;
  const int bk = k < n ? md.dofBody[k] : 0;
  const int lam = k < n ? md.parent[bk] : -1;
  double acc = 0.0;
  unsigned long long done = 0ull;  // bodies already processed
  // bodies carrying a dof; a contact body with none of them among its
  // ancestors (the static ground) contributes to no direction k: skipped
  unsigned lo = 0u, hi = 0u;
  if (k < n) {
    if (bk < 32) lo = 1u << bk;
    else hi = 1u << (bk - 32);
  }
  for (int o = 32; o >= 1; o >>= 1) {
    lo |= __shfl_xor(lo, o);
    hi |= __shfl_xor(hi, o);
  }
  const unsigned long long dofBodies = ((unsigned long long)uni((int)hi) << 32) | (unsigned)uni((int)lo);
  // row data, row j < m on lane j & 63 (slot j >> 6), loaded once from the
  // snapshot; the loops below read them by readlane instead of chains of
  // dependent memory loads
  int rMap[R], rA[R], rB[R], rTyp[R], rDir[R], rCon[R];
  double rp[3][R], rd[3][R], rn[3][R];
  unsigned long long liveRows[R];
#pragma unroll
  for (int q = 0; q < R; q++) {
    const int j = rowAt(q, lane);
    rMap[q] = CM_NOT_CLAMPING; rA[q] = 0; rB[q] = 0; rTyp[q] = 0; rDir[q] = 0; rCon[q] = 0;
    for (int i = 0; i < 3; i++) { rp[i][q] = 0.0; rd[i][q] = 0.0; rn[i][q] = 0.0; }
    if (j < m) {
      const double* rr = rows + j * SN_ROWREC;
      rMap[q] = (int)rr[RR_MAP];
      rDir[q] = (int)rr[RR_DIR];
      rCon[q] = (int)rr[RR_CONTACT];
      const double* rec = sn + SN_CONTACTS + rCon[q] * CREC;
      rA[q] = (int)rec[8]; rB[q] = (int)rec[9]; rTyp[q] = (int)rec[7];
      for (int i = 0; i < 3; i++) { rp[i][q] = rec[i]; rn[i][q] = rec[3 + i]; rd[i][q] = rr[RR_D + i]; }
    }
    liveRows[q] = __ballot(j < m && rMap[q] != CM_NOT_CLAMPING);
  }
  for (int j0 = 0; j0 < m; j0++) {
    if (!bitR(liveRows, j0)) continue;
    for (int side = 0; side < 2; side++) {
      const int c = side ? rdliR(rB, j0) : rdliR(rA, j0);
      if ((done >> c) & 1ull) continue;
      done |= 1ull << c;
      if (!(md.anc[c] & dofBodies)) continue;
      // omega^c_r (lane r), vertex sums (lanes over rows), all for body c
      TACC_BEGIN(tO);
      double om[6] = {0, 0, 0, 0, 0, 0};
      unsigned long long rowsC[R];
#pragma unroll
      for (int q = 0; q < R; q++) rowsC[q] = __ballot(((liveRows[q] >> lane) & 1ull) && (rA[q] == c || rB[q] == c));
#pragma unroll
      for (int q = 0; q < R; q++)
      for (unsigned long long bits = rowsC[q]; bits; bits &= bits - 1ull) {
        const int j = 64 * q + __ffsll((long long)bits) - 1;
        const double sg = rdliR(rA, j) == c ? 1.0 : -1.0;
        double p[3], d[3];
        for (int i = 0; i < 3; i++) { p[i] = rdlR(rp[i], j); d[i] = rdlR(rd[i], j); }
        double wr[6];
        cross3(p, d, wr);
        wr[3] = d[0]; wr[4] = d[1]; wr[5] = d[2];
        if (lane < n) {
          const double gr = sg * P.gRows[j * n + lane];
#pragma unroll
          for (int i = 0; i < 6; i++) om[i] = fma(gr, wr[i], om[i]);
        }
      }
      // vertex sides of c's rows (lane = row), summed over the wave
      {
        double uvl[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < R; q++) {
          const int type = rTyp[q] & 15;
          const bool vertexSide = ((rowsC[q] >> lane) & 1ull) && ((type == CT_VERTEX_FACE && rA[q] == c) ||
                                                                   (type == CT_FACE_VERTEX && rB[q] == c));
          if (vertexSide) {
            const int j = rowAt(q, lane);
            double tw[3], dxt[3], pxd[3], dj[3], pj[3];
            for (int i = 0; i < 3; i++) {
              tw[i] = P.TAB[j * 12 + i] - P.TAB[j * 12 + 6 + i];
              dj[i] = rd[i][q];
              pj[i] = rp[i][q];
            }
            cross3(dj, tw, dxt);
            cross3(pj, dxt, pxd);
            for (int i = 0; i < 3; i++) { uvl[i] += dxt[i]; uvl[3 + i] += pxd[i]; }
          }
        }
        double uvs[6];
        for (int i = 0; i < 6; i++) uvs[i] = waveSum(uvl[i]);
        if (lane == 0)
          for (int i = 0; i < 6; i++) UV[i] = uvs[i];
      }
      if (lane < n)
        for (int i = 0; i < 6; i++) omega[lane * 6 + i] = om[i];
      WSYNC();
      TACC_END(82, tO);
      TACC_BEGIN(tP);
      // P^c_b = sum over ancestor dofs r of b of S_r x* omega_r
      // (terms S_r x* omega_r formed once per dof, in place of omega_r;
      // lane b adds them with 0 / 1 ancestor weights)
      if (lane < n) {
        double t[6];
        crf(s + L.Sw + 6 * lane, omega + 6 * lane, t);
        for (int i = 0; i < 6; i++) omega[lane * 6 + i] = t[i];
      }
      WSYNC();
      {
        // omega is non-zero only on the dofs that move body c (its rows'
        // bodies are c), so the sums run over those
        unsigned long long dm = ancestorDofMask(md, md.anc[c], lane);
        if (lane < nb) {
          double pb[6] = {0, 0, 0, 0, 0, 0};
          const unsigned long long an = md.anc[lane];
          while (dm) {
            const int r = __ffsll((long long)dm) - 1;
            dm &= dm - 1ull;
            const double w = ((an >> md.dofBody[r]) & 1ull) ? 1.0 : 0.0;
#pragma unroll
            for (int i = 0; i < 6; i++) pb[i] = fma(w, omega[6 * r + i], pb[i]);
          }
          for (int i = 0; i < 6; i++) Pc[lane * 6 + i] = pb[i];
        }
      }
      WSYNC();
      if (k < n && ((md.anc[c] >> bk) & 1ull)) {
        double y[6];
        for (int i = 0; i < 6; i++) y[i] = Pc[c * 6 + i] - (lam >= 0 ? Pc[lam * 6 + i] : 0.0);
        acc += dot6(Z, y);
        const double zw = sqrt(Z[0] * Z[0] + Z[1] * Z[1] + Z[2] * Z[2]);
        if (zw > 1e-6) acc += Z[0] * UV[3] + Z[1] * UV[4] + Z[2] * UV[5];
        acc += Z[3] * UV[0] + Z[4] * UV[1] + Z[5] * UV[2];
      }
      WSYNC();
      TACC_END(83, tP);
      if (lane == 0 && g_stamp) g_stamp[85] += 1;
    }
  }
  // face side: per row
  TACC_BEGIN(tF);
  {
    // (the rows' readlanes for every lane; the terms for the lanes k < n)
#pragma unroll
    for (int q = 0; q < R; q++)
    for (unsigned long long bits = liveRows[q]; bits; bits &= bits - 1ull) {
      const int j = 64 * q + __ffsll((long long)bits) - 1;
      const int A = rdliR(rA, j), B = rdliR(rB, j), type = rdliR(rTyp, j) & 15;
      const int con = rdliR(rCon, j), dirIdx = rdliR(rDir, j);
      double p[3], nrm[3];
      for (int i = 0; i < 3; i++) { p[i] = rdlR(rp[i], j); nrm[i] = rdlR(rn[i], j); }
      if (k >= n) continue;
      if (type >= CT_EDGE_EDGE) {
        const double* rr = rows + j * SN_ROWREC;
        const double* rec = sn + SN_CONTACTS + con * CREC;
        if (type == CT_EDGE_EDGE) acc += edgeRowTerm(md, P, j, rec, rr, sn + snEdge(n) + con * EDGE_REC, Z, bk, A, B);
        else if (type == CT_SPHERE_SPHERE)
          acc += sphereSphereRowTerm(md, P, j, rec, rr, sn + snEdge(n) + con * EDGE_REC, Z, bk, A, B);
        else if (type == CT_PIPE_PIPE)
          acc += pipePipeRowTerm(md, P, j, rec, rr, sn + snEdge(n) + con * EDGE_REC, Z, bk, A, B);
        else if (type == CT_SPHERE_PIPE || type == CT_PIPE_SPHERE)
          acc += spherePipeRowTerm(md, P, j, rec, rr, sn + snEdge(n) + con * EDGE_REC, Z, bk, A, B, type);
        else if (type >= CT_PIPE_VERTEX && type <= CT_EDGE_PIPE)
          acc += pipeMeshRowTerm(md, P, j, rec, rr, sn + snEdge(n) + con * EDGE_REC, Z, bk, A, B, type);
        else acc += sphereRowTerm(md, s, L, P, j, rec, rr, Z, bk);
        continue;
      }
      int faceBody = -1;
      if (type == CT_VERTEX_FACE) faceBody = B;
      else if (type == CT_FACE_VERTEX) faceBody = A;
      if (faceBody < 0 || !((md.anc[faceBody] >> bk) & 1ull)) continue;
      double dn[3];
      const double wv[3] = {Z[0], Z[1], Z[2]};
      cross3(wv, nrm, dn);
      double dd[3];
      if (dirIdx == 0 || dot3(dn, dn) <= 1e-12) {
        for (int i = 0; i < 3; i++) dd[i] = dn[i];
      } else {
        double T0[3], T1[3];
        tangentBasisGradient(nrm, dn, T0, T1);
        for (int i = 0; i < 3; i++) dd[i] = dirIdx == 1 ? T0[i] : T1[i];
      }
      double pxdd[3];
      cross3(p, dd, pxdd);
      double v = 0.0;
      for (int i = 0; i < 3; i++)
        v += (P.TAB[j * 12 + i] - P.TAB[j * 12 + 6 + i]) * pxdd[i] +
             (P.TAB[j * 12 + 3 + i] - P.TAB[j * 12 + 9 + i]) * dd[i];
      acc += v;
    }
  }
  TACC_END(84, tF);
  return acc;
}

// M-derivative pairs m(a, c) = (d(M a)/dq)^T c evaluated for all directions:
//   d(c^T M a)/dq_k = -(Z_k x V_c,lam) . H_a(k) - (Z_k x V_a,lam) . H_c(k)
// with V_x,b the world twist of body b under joint rates x and H_x(k) the
// subtree momentum sum_{b in sub(k)} I_b V_x,b.  For each of the four (a, c)
// column pairs of NV, lane b builds both fields' twists and momenta I_b V
// (world inertias are formed once, kept as their 3x3 rotational block, world
// COM and mass: 13 doubles per body after the 2 x nb x 12 field doubles in
// `buf`), then the momenta are summed over each subtree level by level.
__device__ double mFieldsTerm(const ModelDev& md, double* s, const Layout& L, const double* NV, double* buf, int lane,
                              int k, const double* Z, double coefDelta, double imp) {
  const int nb = md.nb;
  const double coef[4] = {coefDelta, 1.0, -imp, -imp};
  double* wI = buf + 24 * nb;
  if (lane < nb) {
    // worldInertia's arithmetic, stored compactly
    const int b = lane;
    const double* Tw = s + L.Tw + 12 * b;
    const double m = md.mass[b];
    double cw[3], Rc[9], tmp[9];
    for (int r = 0; r < 3; r++)
      cw[r] = Tw[r * 4] * md.com[b][0] + Tw[r * 4 + 1] * md.com[b][1] + Tw[r * 4 + 2] * md.com[b][2] + Tw[r * 4 + 3];
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++)
        tmp[r * 3 + c] = Tw[r * 4] * md.Ic[b][c] + Tw[r * 4 + 1] * md.Ic[b][3 + c] + Tw[r * 4 + 2] * md.Ic[b][6 + c];
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++)
        Rc[r * 3 + c] = tmp[r * 3] * Tw[c * 4] + tmp[r * 3 + 1] * Tw[c * 4 + 1] + tmp[r * 3 + 2] * Tw[c * 4 + 2];
    const double C[9] = {0, -cw[2], cw[1], cw[2], 0, -cw[0], -cw[1], cw[0], 0};
    double* w = wI + 13 * b;
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        const double cct = C[r * 3] * C[c * 3] + C[r * 3 + 1] * C[c * 3 + 1] + C[r * 3 + 2] * C[c * 3 + 2];
        w[r * 3 + c] = Rc[r * 3 + c] + m * cct;
      }
    w[9] = cw[0]; w[10] = cw[1]; w[11] = cw[2]; w[12] = m;
  }
  WSYNC();
  double total = 0.0;
  // the pseudo-inverse branch's two pairs carry the factor -imp: skipped
  // when Q has full rank
  const int npairs = imp != 0.0 ? 4 : 2;
  for (int pr = 0; pr < npairs; pr++) {
    if (lane < nb) {
      const int b = lane;
      double Va[6] = {0, 0, 0, 0, 0, 0}, Vc[6] = {0, 0, 0, 0, 0, 0};
      const unsigned long long an = md.anc[b];
      const double* ga = NV + 2 * pr;
      const double* gc = NV + 2 * pr + 1;
#pragma unroll 4
      for (int r = 0; r < md.n; r++) {
        const bool in = (an >> md.dofBody[r]) & 1ull;
        const double xa = in ? ga[r * NV_COLS] : 0.0, xc = in ? gc[r * NV_COLS] : 0.0;
        const double* S = s + L.Sw + 6 * r;
        for (int i = 0; i < 6; i++) {
          Va[i] = fma(S[i], xa, Va[i]);
          Vc[i] = fma(S[i], xc, Vc[i]);
        }
      }
      const double* w = wI + 13 * b;
      const double m = w[12];
      const double C[9] = {0, -w[11], w[10], w[11], 0, -w[9], -w[10], w[9], 0};
      double I[36];
      for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
          I[r * 6 + c] = w[r * 3 + c];
          I[r * 6 + c + 3] = m * C[r * 3 + c];
          I[(r + 3) * 6 + c] = m * C[c * 3 + r];
          I[(r + 3) * 6 + c + 3] = (r == c) ? m : 0.0;
        }
      double* Fa = buf + b * 12;
      double* Fc = buf + (nb + b) * 12;
      double ha[6], hc[6];
      mv6(I, Va, ha);
      mv6(I, Vc, hc);
      for (int i = 0; i < 6; i++) { Fa[i] = Va[i]; Fa[6 + i] = ha[i]; Fc[i] = Vc[i]; Fc[6 + i] = hc[i]; }
    }
    WSYNC();
    // subtree momenta in place over the deepest-child-first edge list (lane =
    // field x component; see composites) -- instead of every lane reading all
    // nb bodies' 12 momenta (the four worlds of a CU share the LDS bandwidth)
    if (lane < 12) {
      double* base = buf + (lane < 6 ? 0 : nb * 12) + 6 + (lane % 6);
#pragma unroll 4
      for (int k = 0; k < md.numAcc; k++) {
        const int p = md.accEdge[k][0], c = md.accEdge[k][1];
        base[p * 12] += base[c * 12];
      }
    }
    WSYNC();
    // dof k reads its body's subtree momenta
    const int bk = k < md.n ? md.dofBody[k] : 0;
    double ha[6], hc[6];
    for (int i = 0; i < 6; i++) { ha[i] = buf[bk * 12 + 6 + i]; hc[i] = buf[(nb + bk) * 12 + 6 + i]; }
    if (k < md.n) {
      const int lam = md.parent[bk];
      double val = 0.0;
      if (lam >= 0) {
        double t[6];
        crm(Z, buf + (nb + lam) * 12, t);
        val -= dot6(t, ha);
        crm(Z, buf + lam * 12, t);
        val -= dot6(t, hc);
      }
      total += coef[pr] * val;
    }
    WSYNC();
  }
  return total;
}
