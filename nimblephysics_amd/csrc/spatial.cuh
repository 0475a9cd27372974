// World-frame spatial algebra on doubles for the gfx950 kernels.
// Motion vectors m = [w; v], force vectors f = [t; f] (reference convention,
// dart/math/Geometry.cpp).  All quantities here are expressed at the WORLD
// origin in world axes, which turns the reference's per-body frame changes
// (AdInvT / dAdInvT / transformInertia in the recursions) into plain sums --
// the layout the composite-body and derivative kernels are built on.
#pragma once
#include <hip/hip_runtime.h>

#define DEV __device__ __forceinline__

DEV void cross3(const double* a, const double* b, double* o) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
// packed lower-triangular index (row i, column k <= i)
DEV int tri(int i, int k) { return ((i * (i + 1)) >> 1) + k; }
DEV double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
DEV double dot6(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}

// m x m'  (ad, dart/math/Geometry.cpp:1469)
DEV void crm(const double* m, const double* x, double* o) {
  double a[3], b[3], c[3];
  cross3(m, x, a);
  cross3(m, x + 3, b);
  cross3(m + 3, x, c);
  o[0] = a[0]; o[1] = a[1]; o[2] = a[2];
  o[3] = b[0] + c[0]; o[4] = b[1] + c[1]; o[5] = b[2] + c[2];
}
// m x* f  (= -dad(m, f), Geometry.cpp:3506)
DEV void crf(const double* m, const double* f, double* o) {
  double a[3], b[3], c[3];
  cross3(m, f, a);
  cross3(m + 3, f + 3, b);
  cross3(m, f + 3, c);
  o[0] = a[0] + b[0]; o[1] = a[1] + b[1]; o[2] = a[2] + b[2];
  o[3] = c[0]; o[4] = c[1]; o[5] = c[2];
}
DEV void mv6(const double* M, const double* x, double* o) {
#pragma unroll
  for (int r = 0; r < 6; r++) {
    double s = 0;
#pragma unroll
    for (int c = 0; c < 6; c++) s = fma(M[r * 6 + c], x[c], s);
    o[r] = s;
  }
}

// Transform [R|p] (row-major 3x4) helpers
DEV void tmul(const double* A, const double* B, double* O) {
  double t[12];
#pragma unroll
  for (int r = 0; r < 3; r++) {
#pragma unroll
    for (int c = 0; c < 3; c++)
      t[r * 4 + c] = A[r * 4 + 0] * B[0 * 4 + c] + A[r * 4 + 1] * B[1 * 4 + c] + A[r * 4 + 2] * B[2 * 4 + c];
    t[r * 4 + 3] = A[r * 4 + 0] * B[3] + A[r * 4 + 1] * B[7] + A[r * 4 + 2] * B[11] + A[r * 4 + 3];
  }
#pragma unroll
  for (int i = 0; i < 12; i++) O[i] = t[i];
}
// Ad_T applied to a motion vector
DEV void adT(const double* T, const double* m, double* o) {
  double w[3], v[3], pxw[3];
#pragma unroll
  for (int r = 0; r < 3; r++) {
    w[r] = T[r * 4] * m[0] + T[r * 4 + 1] * m[1] + T[r * 4 + 2] * m[2];
    v[r] = T[r * 4] * m[3] + T[r * 4 + 1] * m[4] + T[r * 4 + 2] * m[5];
  }
  double p[3] = {T[3], T[7], T[11]};
  cross3(p, w, pxw);
  o[0] = w[0]; o[1] = w[1]; o[2] = w[2];
  o[3] = v[0] + pxw[0]; o[4] = v[1] + pxw[1]; o[5] = v[2] + pxw[2];
}

// expMapRot (dart/math/Geometry.cpp:539)
DEV void expMapRot(const double* q, double* R /*3x3 row-major*/) {
  double t2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2];
  double th = sqrt(t2);
  double K[9] = {0, -q[2], q[1], q[2], 0, -q[0], -q[1], q[0], 0};
  double K2[9];
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) K2[r * 3 + c] = K[r * 3] * K[c] + K[r * 3 + 1] * K[3 + c] + K[r * 3 + 2] * K[6 + c];
  double a, b;
  if (th < 1.0e-3) {
    a = 1.0;
    b = 0.5;
  } else {
    a = sin(th) / th;
    b = (1.0 - cos(th)) / t2;
  }
#pragma unroll
  for (int i = 0; i < 9; i++) R[i] = ((i % 4) == 0 ? 1.0 : 0.0) + a * K[i] + b * K2[i];
}

// logMap (dart/math/Geometry.cpp:720)
DEV void logMap(const double* R, double* o) {
  const double pi = 3.14159265358979323846;
  const double eps = 1e-6;
  double c = 0.5 * (R[0] + R[4] + R[8] - 1.0);
  c = fmin(fmax(c, -1.0), 1.0);
  double th = acos(c);
  if (th > pi - eps) {
    double delta = 0.5 + 0.125 * (pi - th) * (pi - th);
    double s0 = th * sqrt(1.0 + (R[0] - 1.0) * delta);
    double s1 = th * sqrt(1.0 + (R[4] - 1.0) * delta);
    double s2 = th * sqrt(1.0 + (R[8] - 1.0) * delta);
    o[0] = R[7] > R[5] ? s0 : -s0;
    o[1] = R[2] > R[6] ? s1 : -s1;
    o[2] = R[3] > R[1] ? s2 : -s2;
    return;
  }
  double alpha = th > eps ? 0.5 * th / sin(th) : 0.5 + (1.0 / 12.0) * th * th;
  o[0] = alpha * (R[7] - R[5]);
  o[1] = alpha * (R[2] - R[6]);
  o[2] = alpha * (R[3] - R[1]);
}

// FreeJoint::integratePositionsExplicit (dart/dynamics/FreeJoint.cpp:920) with
// DART_USE_IDENTITY_JACOBIAN: convertToPositions(Q(q) * convertToTransform(v dt))
DEV void freeIntegrate(const double* q, const double* v, double dt, double* out) {
  double R[9], Rd[9], wd[3] = {v[0] * dt, v[1] * dt, v[2] * dt};
  expMapRot(q, R);
  expMapRot(wd, Rd);
  double Rn[9];
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) Rn[r * 3 + c] = R[r * 3] * Rd[c] + R[r * 3 + 1] * Rd[3 + c] + R[r * 3 + 2] * Rd[6 + c];
  double l[3] = {v[3] * dt, v[4] * dt, v[5] * dt};
  logMap(Rn, out);
#pragma unroll
  for (int r = 0; r < 3; r++) out[3 + r] = R[r * 3] * l[0] + R[r * 3 + 1] * l[1] + R[r * 3 + 2] * l[2] + q[3 + r];
}
