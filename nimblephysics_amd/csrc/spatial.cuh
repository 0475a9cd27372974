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

// BallJoint::integratePositionsExplicit (dart/dynamics/BallJoint.cpp:333) with
// DART_USE_IDENTITY_JACOBIAN: convertToPositions(R(q) * R(dq dt)) -- the
// rotational half of freeIntegrate, the same operations
DEV void ballIntegrate(const double* q, const double* v, double dt, double* out) {
  double R[9], Rd[9], wd[3] = {v[0] * dt, v[1] * dt, v[2] * dt};
  expMapRot(q, R);
  expMapRot(wd, Rd);
  double Rn[9];
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) Rn[r * 3 + c] = R[r * 3] * Rd[c] + R[r * 3 + 1] * Rd[3 + c] + R[r * 3 + 2] * Rd[6 + c];
  logMap(Rn, out);
}

// ---------------------------------------------------------------------------
// The FreeJoint finite-difference blocks (FreeJoint.cpp:965 eps 1e-6, :987
// eps 1e-7) difference two position integrations 2 eps apart, so the last
// bits of each integration become the block's leading digits.  Their
// integrations run here as one fixed sequence of IEEE operations: the
// elementary functions below use only +, -, *, / and sqrt (quadrant reduction
// by a three-part pi/2, Taylor series of sin / cos on |r| <= pi/4, the
// arcsine series on |x| <= 1/2), nothing is contracted into a fused multiply-
// add, and the integration keeps the reference's operation order
// (Geometry.cpp:539 expMapRot, :720 logMap).  The oracle evaluates the same
// sequence (oracle/nimble_oracle.cpp, the fd* functions), so the device's
// blocks equal the oracle's bit for bit instead of differing by the rounding
// noise of two libms amplified by 1 / (2 eps).
// ---------------------------------------------------------------------------
constexpr double kFdPi = 0x1.921fb54442d18p+1, kFdPio2 = 0x1.921fb54442d18p+0, kFdTwoOverPi = 0x1.45f306dc9c883p-1;
// pi / 2 = kFdP1 + kFdP2 + kFdP3, kFdP1 with 33 significant bits (k * kFdP1 exact)
constexpr double kFdP1 = 0x1.921fb54400000p+0, kFdP2 = 0x1.0b4611a626331p-34, kFdP3 = 0x1.1701b839a2520p-88;
DEV double fdSinK(double r) {  // |r| <= pi / 4
#pragma clang fp contract(off)
  const double z = r * r;
  // (-1)^k / (2k + 1)!, k = 1 .. 10
  double p = 0x1.71b8ef6dcf572p-66;
  p = -0x1.2f49b46814157p-57 + z * p;
  p = 0x1.952c77030ad4ap-49 + z * p;
  p = -0x1.ae7f3e733b81fp-41 + z * p;
  p = 0x1.6124613a86d09p-33 + z * p;
  p = -0x1.ae64567f544e4p-26 + z * p;
  p = 0x1.71de3a556c734p-19 + z * p;
  p = -0x1.a01a01a01a01ap-13 + z * p;
  p = 0x1.1111111111111p-7 + z * p;
  p = -0x1.5555555555555p-3 + z * p;
  return r + r * (z * p);
}
DEV double fdCosK(double r) {
#pragma clang fp contract(off)
  const double z = r * r;
  // (-1)^k / (2k)!, k = 1 .. 10
  double p = 0x1.e542ba4020225p-62;
  p = -0x1.6827863b97d97p-53 + z * p;
  p = 0x1.ae7f3e733b81fp-45 + z * p;
  p = -0x1.93974a8c07c9dp-37 + z * p;
  p = 0x1.1eed8eff8d898p-29 + z * p;
  p = -0x1.27e4fb7789f5cp-22 + z * p;
  p = 0x1.a01a01a01a01ap-16 + z * p;
  p = -0x1.6c16c16c16c17p-10 + z * p;
  p = 0x1.5555555555555p-5 + z * p;
  p = -0x1.0000000000000p-1 + z * p;
  return 1.0 + z * p;
}
DEV int fdReduce(double x, double& r) {
#pragma clang fp contract(off)
  const double k = floor(x * kFdTwoOverPi + 0.5);
  r = ((x - k * kFdP1) - k * kFdP2) - k * kFdP3;
  return ((int)k) & 3;
}
DEV double fdSin(double x) {
  double r;
  const int q = fdReduce(x, r);
  return q == 0 ? fdSinK(r) : (q == 1 ? fdCosK(r) : (q == 2 ? -fdSinK(r) : -fdCosK(r)));
}
DEV double fdCos(double x) {
  double r;
  const int q = fdReduce(x, r);
  return q == 0 ? fdCosK(r) : (q == 1 ? -fdSinK(r) : (q == 2 ? -fdCosK(r) : fdSinK(r)));
}
DEV double fdAsinK(double x) {  // |x| <= 1 / 2
#pragma clang fp contract(off)
  const double z = x * x;
  // (2n)! / (4^n (n!)^2 (2n + 1)), n = 1 .. 30
  double p = 0x1.b8d2e5667ce6cp-10;
  p = 0x1.cf7dea5b6e830p-10 + z * p;
  p = 0x1.e82be60d9127ep-10 + z * p;
  p = 0x1.018f963c229bfp-9 + z * p;
  p = 0x1.1052bc5fa960ap-9 + z * p;
  p = 0x1.208d3570ae5a6p-9 + z * p;
  p = 0x1.3275586c5f2f0p-9 + z * p;
  p = 0x1.464c0950f7d47p-9 + z * p;
  p = 0x1.5c5f56efaaaabp-9 + z * p;
  p = 0x1.750de64d7d05fp-9 + z * p;
  p = 0x1.90cb77f60c7cep-9 + z * p;
  p = 0x1.b026f57b13b14p-9 + z * p;
  p = 0x1.d3d2a8e0dd67dp-9 + z * p;
  p = 0x1.fcaf8fb6db6dbp-9 + z * p;
  p = 0x1.15ee9d45d1746p-8 + z * p;
  p = 0x1.31683bdef7bdfp-8 + z * p;
  p = 0x1.51ba308d3dcb1p-8 + z * p;
  p = 0x1.782dda12f684cp-8 + z * p;
  p = 0x1.a6863d70a3d71p-8 + z * p;
  p = 0x1.df3bd37a6f4dfp-8 + z * p;
  p = 0x1.12ef3cf3cf3cfp-7 + z * p;
  p = 0x1.3fde50d79435ep-7 + z * p;
  p = 0x1.7a87878787878p-7 + z * p;
  p = 0x1.c99999999999ap-7 + z * p;
  p = 0x1.1c4ec4ec4ec4fp-6 + z * p;
  p = 0x1.6e8ba2e8ba2e9p-6 + z * p;
  p = 0x1.f1c71c71c71c7p-6 + z * p;
  p = 0x1.6db6db6db6db7p-5 + z * p;
  p = 0x1.3333333333333p-4 + z * p;
  p = 0x1.5555555555555p-3 + z * p;
  return x + x * (z * p);
}
DEV double fdAcos(double c) {
#pragma clang fp contract(off)
  if (c > 0.5) return 2.0 * fdAsinK(sqrt((1.0 - c) * 0.5));
  if (c < -0.5) return kFdPi - 2.0 * fdAsinK(sqrt((1.0 + c) * 0.5));
  return kFdPio2 - fdAsinK(c);
}
// expMapRot (Geometry.cpp:539) in the reference's order
DEV void fdExpMapRot(const double* q, double* R) {
#pragma clang fp contract(off)
  const double th = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
  const double K[9] = {0.0, -q[2], q[1], q[2], 0.0, -q[0], -q[1], q[0], 0.0};
  double K2[9];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) K2[r * 3 + c] = K[r * 3] * K[c] + K[r * 3 + 1] * K[3 + c] + K[r * 3 + 2] * K[6 + c];
  if (th < 1.0e-3) {
    for (int i = 0; i < 9; i++) R[i] = ((i % 4) == 0 ? 1.0 : 0.0) + K[i] + 0.5 * K2[i];
  } else {
    const double a = fdSin(th) / th, b = (1.0 - fdCos(th)) / (th * th);
    for (int i = 0; i < 9; i++) R[i] = ((i % 4) == 0 ? 1.0 : 0.0) + a * K[i] + b * K2[i];
  }
}
// logMap (Geometry.cpp:720)
DEV void fdLogMap(const double* R, double* o) {
#pragma clang fp contract(off)
  const double eps = 1e-6;
  const double th = fdAcos(fmax(fmin(0.5 * (R[0] + R[4] + R[8] - 1.0), 1.0), -1.0));
  if (th > kFdPi - eps) {
    const double delta = 0.5 + 0.125 * (kFdPi - th) * (kFdPi - th);
    const double s0 = th * sqrt(1.0 + (R[0] - 1.0) * delta);
    const double s1 = th * sqrt(1.0 + (R[4] - 1.0) * delta);
    const double s2 = th * sqrt(1.0 + (R[8] - 1.0) * delta);
    o[0] = R[7] > R[5] ? s0 : -s0;
    o[1] = R[2] > R[6] ? s1 : -s1;
    o[2] = R[3] > R[1] ? s2 : -s2;
    return;
  }
  const double alpha = th > eps ? 0.5 * th / fdSin(th) : 0.5 + (1.0 / 12.0) * th * th;
  o[0] = alpha * (R[7] - R[5]);
  o[1] = alpha * (R[2] - R[6]);
  o[2] = alpha * (R[3] - R[1]);
}
// FreeJoint::integratePositionsExplicit (FreeJoint.cpp:920) for the finite-
// difference blocks: convertToPositions(Q(q) * convertToTransform(v dt))
DEV void fdFreeIntegrate(const double* q, const double* v, double dt, double* out) {
#pragma clang fp contract(off)
  double R[9], Rd[9], Rn[9];
  const double wd[3] = {v[0] * dt, v[1] * dt, v[2] * dt};
  fdExpMapRot(q, R);
  fdExpMapRot(wd, Rd);
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) Rn[r * 3 + c] = R[r * 3] * Rd[c] + R[r * 3 + 1] * Rd[3 + c] + R[r * 3 + 2] * Rd[6 + c];
  const double l[3] = {v[3] * dt, v[4] * dt, v[5] * dt};
  fdLogMap(Rn, out);
  for (int r = 0; r < 3; r++) out[3 + r] = R[r * 3] * l[0] + R[r * 3 + 1] * l[1] + R[r * 3 + 2] * l[2] + q[3 + r];
}
