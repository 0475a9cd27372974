// ORACLE / TEST INFRASTRUCTURE ONLY -- never linked into the product path.
//
// Small dense + spatial-algebra helpers for the CPU restatement of the
// reference's timestep.  Templated on the scalar so the same recursions run on
// double (values) and on Dual (forward-mode derivatives used for the analytic
// Jacobians, which the reference computes in closed form in
// dart/dynamics/Skeleton.cpp:1779 getJacobianOfC and :2024 getJacobianOfMinv).
//
// Conventions follow dart/math/Geometry.cpp: spatial vectors are [angular;
// linear], ad() at Geometry.cpp:1469, dad() at :3506, AdInvT() at :1437,
// dAdInvT() at :1530, AdT() at :1300, expMapRot() at :539, logMap() at :720.
#pragma once
#include <cmath>
#include <algorithm>

namespace oracle {

using std::sin;
using std::cos;
using std::sqrt;

struct Dual {
  double v, d;
  Dual() : v(0), d(0) {}
  Dual(double x) : v(x), d(0) {}
  Dual(double x, double dx) : v(x), d(dx) {}
};
inline Dual operator+(Dual a, Dual b) { return Dual(a.v + b.v, a.d + b.d); }
inline Dual operator-(Dual a, Dual b) { return Dual(a.v - b.v, a.d - b.d); }
inline Dual operator-(Dual a) { return Dual(-a.v, -a.d); }
inline Dual operator*(Dual a, Dual b) { return Dual(a.v * b.v, a.d * b.v + a.v * b.d); }
inline Dual operator/(Dual a, Dual b) { return Dual(a.v / b.v, (a.d * b.v - a.v * b.d) / (b.v * b.v)); }
inline Dual& operator+=(Dual& a, Dual b) { a = a + b; return a; }
inline Dual& operator-=(Dual& a, Dual b) { a = a - b; return a; }
inline Dual& operator*=(Dual& a, Dual b) { a = a * b; return a; }
inline Dual sin(Dual a) { return Dual(std::sin(a.v), a.d * std::cos(a.v)); }
inline Dual cos(Dual a) { return Dual(std::cos(a.v), -a.d * std::sin(a.v)); }
inline Dual sqrt(Dual a) { double s = std::sqrt(a.v); return Dual(s, s > 0 ? a.d / (2 * s) : 0.0); }
inline double val(double x) { return x; }
inline double val(Dual x) { return x.v; }

template <class S> struct V3 { S x[3]; S& operator[](int i) { return x[i]; } const S& operator[](int i) const { return x[i]; } };
template <class S> struct V6 { S x[6]; S& operator[](int i) { return x[i]; } const S& operator[](int i) const { return x[i]; } };
template <class S> struct M3 { S m[9]; S& operator()(int r, int c) { return m[r * 3 + c]; } const S& operator()(int r, int c) const { return m[r * 3 + c]; } };
template <class S> struct M6 { S m[36]; S& operator()(int r, int c) { return m[r * 6 + c]; } const S& operator()(int r, int c) const { return m[r * 6 + c]; } };
// Isometry: x -> R x + p
template <class S> struct Iso { M3<S> R; V3<S> p; };

template <class S> V3<S> zero3() { V3<S> r; for (int i = 0; i < 3; i++) r[i] = S(0.0); return r; }
template <class S> V6<S> zero6() { V6<S> r; for (int i = 0; i < 6; i++) r[i] = S(0.0); return r; }
template <class S> M6<S> zero66() { M6<S> r; for (int i = 0; i < 36; i++) r.m[i] = S(0.0); return r; }
template <class S> M3<S> eye3() { M3<S> r; for (int i = 0; i < 9; i++) r.m[i] = S((i % 4 == 0) ? 1.0 : 0.0); return r; }
template <class S> Iso<S> identityIso() { Iso<S> t; t.R = eye3<S>(); t.p = zero3<S>(); return t; }

template <class S> V3<S> cross(const V3<S>& a, const V3<S>& b) {
  V3<S> r;
  r[0] = a[1] * b[2] - a[2] * b[1];
  r[1] = a[2] * b[0] - a[0] * b[2];
  r[2] = a[0] * b[1] - a[1] * b[0];
  return r;
}
template <class S> V3<S> add(const V3<S>& a, const V3<S>& b) { V3<S> r; for (int i = 0; i < 3; i++) r[i] = a[i] + b[i]; return r; }
template <class S> V3<S> sub(const V3<S>& a, const V3<S>& b) { V3<S> r; for (int i = 0; i < 3; i++) r[i] = a[i] - b[i]; return r; }
template <class S> V3<S> scale(const V3<S>& a, S s) { V3<S> r; for (int i = 0; i < 3; i++) r[i] = a[i] * s; return r; }
template <class S> S dot(const V3<S>& a, const V3<S>& b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
template <class S> V3<S> mul(const M3<S>& m, const V3<S>& v) {
  V3<S> r;
  for (int i = 0; i < 3; i++) r[i] = m(i, 0) * v[0] + m(i, 1) * v[1] + m(i, 2) * v[2];
  return r;
}
template <class S> V3<S> mulT(const M3<S>& m, const V3<S>& v) {
  V3<S> r;
  for (int i = 0; i < 3; i++) r[i] = m(0, i) * v[0] + m(1, i) * v[1] + m(2, i) * v[2];
  return r;
}
template <class S> M3<S> mul(const M3<S>& a, const M3<S>& b) {
  M3<S> r;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) r(i, j) = a(i, 0) * b(0, j) + a(i, 1) * b(1, j) + a(i, 2) * b(2, j);
  return r;
}
template <class S> M3<S> transpose(const M3<S>& a) { M3<S> r; for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) r(i, j) = a(j, i); return r; }
template <class S> M3<S> skew(const V3<S>& v) {
  M3<S> r;
  r(0, 0) = S(0.0); r(0, 1) = -v[2]; r(0, 2) = v[1];
  r(1, 0) = v[2]; r(1, 1) = S(0.0); r(1, 2) = -v[0];
  r(2, 0) = -v[1]; r(2, 1) = v[0]; r(2, 2) = S(0.0);
  return r;
}

template <class S> Iso<S> compose(const Iso<S>& a, const Iso<S>& b) {
  Iso<S> r; r.R = mul(a.R, b.R); r.p = add(mul(a.R, b.p), a.p); return r;
}
template <class S> Iso<S> inverse(const Iso<S>& a) {
  Iso<S> r; r.R = transpose(a.R); r.p = scale(mulT(a.R, a.p), S(-1.0)); return r;
}
template <class S> V3<S> apply(const Iso<S>& t, const V3<S>& x) { return add(mul(t.R, x), t.p); }

// Geometry.cpp:1300 AdT
template <class S> V6<S> AdT(const Iso<S>& T, const V6<S>& V) {
  V3<S> w{{V[0], V[1], V[2]}}, v{{V[3], V[4], V[5]}};
  V3<S> rw = mul(T.R, w);
  V3<S> rv = add(mul(T.R, v), cross(T.p, rw));
  V6<S> r; for (int i = 0; i < 3; i++) { r[i] = rw[i]; r[i + 3] = rv[i]; } return r;
}
// Geometry.cpp:1437 AdInvT
template <class S> V6<S> AdInvT(const Iso<S>& T, const V6<S>& V) {
  V3<S> w{{V[0], V[1], V[2]}}, v{{V[3], V[4], V[5]}};
  V3<S> rw = mulT(T.R, w);
  V3<S> rv = mulT(T.R, add(v, cross(w, T.p)));
  V6<S> r; for (int i = 0; i < 3; i++) { r[i] = rw[i]; r[i + 3] = rv[i]; } return r;
}
// Geometry.cpp:1530 dAdInvT  (= Ad_{T^-1}^T F)
template <class S> V6<S> dAdInvT(const Iso<S>& T, const V6<S>& F) {
  V3<S> a{{F[0], F[1], F[2]}}, l{{F[3], F[4], F[5]}};
  V3<S> rl = mul(T.R, l);
  V3<S> ra = add(mul(T.R, a), cross(T.p, rl));
  V6<S> r; for (int i = 0; i < 3; i++) { r[i] = ra[i]; r[i + 3] = rl[i]; } return r;
}
// Geometry.cpp:1469 ad
template <class S> V6<S> ad(const V6<S>& X, const V6<S>& Y) {
  V3<S> xw{{X[0], X[1], X[2]}}, xv{{X[3], X[4], X[5]}}, yw{{Y[0], Y[1], Y[2]}}, yv{{Y[3], Y[4], Y[5]}};
  V3<S> a = cross(xw, yw);
  V3<S> b = add(cross(xw, yv), cross(xv, yw));
  V6<S> r; for (int i = 0; i < 3; i++) { r[i] = a[i]; r[i + 3] = b[i]; } return r;
}
// Geometry.cpp:3506 dad
template <class S> V6<S> dad(const V6<S>& s, const V6<S>& t) {
  V3<S> sw{{s[0], s[1], s[2]}}, sv{{s[3], s[4], s[5]}}, tw{{t[0], t[1], t[2]}}, tv{{t[3], t[4], t[5]}};
  V3<S> a = add(cross(tw, sw), cross(tv, sv));
  V3<S> b = cross(tv, sw);
  V6<S> r; for (int i = 0; i < 3; i++) { r[i] = a[i]; r[i + 3] = b[i]; } return r;
}
template <class S> M6<S> AdMatrix(const Iso<S>& T) {  // Geometry.cpp:1314 getAdTMatrix
  M6<S> r = zero66<S>();
  M3<S> pR = mul(skew(T.p), T.R);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      r(i, j) = T.R(i, j);
      r(i + 3, j + 3) = T.R(i, j);
      r(i + 3, j) = pR(i, j);
    }
  return r;
}
template <class S> V6<S> mul(const M6<S>& m, const V6<S>& v) {
  V6<S> r;
  for (int i = 0; i < 6; i++) { S s(0.0); for (int j = 0; j < 6; j++) s += m(i, j) * v[j]; r[i] = s; }
  return r;
}
template <class S> M6<S> mul(const M6<S>& a, const M6<S>& b) {
  M6<S> r;
  for (int i = 0; i < 6; i++)
    for (int j = 0; j < 6; j++) { S s(0.0); for (int k = 0; k < 6; k++) s += a(i, k) * b(k, j); r(i, j) = s; }
  return r;
}
template <class S> M6<S> transpose(const M6<S>& a) { M6<S> r; for (int i = 0; i < 6; i++) for (int j = 0; j < 6; j++) r(i, j) = a(j, i); return r; }
template <class S> V6<S> add(const V6<S>& a, const V6<S>& b) { V6<S> r; for (int i = 0; i < 6; i++) r[i] = a[i] + b[i]; return r; }
template <class S> V6<S> sub(const V6<S>& a, const V6<S>& b) { V6<S> r; for (int i = 0; i < 6; i++) r[i] = a[i] - b[i]; return r; }
template <class S> V6<S> scale(const V6<S>& a, S s) { V6<S> r; for (int i = 0; i < 6; i++) r[i] = a[i] * s; return r; }
template <class S> S dot(const V6<S>& a, const V6<S>& b) { S s(0.0); for (int i = 0; i < 6; i++) s += a[i] * b[i]; return s; }

// Geometry.cpp:3515 transformInertia(T, I) = Ad_T^T I Ad_T
template <class S> M6<S> transformInertia(const Iso<S>& T, const M6<S>& I) {
  M6<S> A = AdMatrix(T);
  return mul(transpose(A), mul(I, A));
}

// Geometry.cpp:539 expMapRot
template <class S> M3<S> expMapRot(const V3<S>& q) {
  S theta = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
  M3<S> qss = skew(q);
  M3<S> qss2 = mul(qss, qss);
  M3<S> R = eye3<S>();
  const double EPSILON_EXPMAP_THETA = 1.0e-3;  // dart/math/Geometry.cpp
  if (val(theta) < EPSILON_EXPMAP_THETA) {
    for (int i = 0; i < 9; i++) R.m[i] = R.m[i] + qss.m[i] + S(0.5) * qss2.m[i];
  } else {
    S a = sin(theta) / theta;
    S b = (S(1.0) - cos(theta)) / (theta * theta);
    for (int i = 0; i < 9; i++) R.m[i] = R.m[i] + a * qss.m[i] + b * qss2.m[i];
  }
  return R;
}

// Geometry.cpp:720 logMap (double only; used on the position integrator)
inline V3<double> logMap(const M3<double>& R) {
  const double pi = 3.14159265358979323846;
  const double DART_EPSILON = 1e-6;
  double theta = std::acos(std::max(std::min(0.5 * (R(0, 0) + R(1, 1) + R(2, 2) - 1.0), 1.0), -1.0));
  V3<double> r;
  if (theta > pi - DART_EPSILON) {
    double delta = 0.5 + 0.125 * (pi - theta) * (pi - theta);
    r[0] = R(2, 1) > R(1, 2) ? theta * std::sqrt(1.0 + (R(0, 0) - 1.0) * delta) : -theta * std::sqrt(1.0 + (R(0, 0) - 1.0) * delta);
    r[1] = R(0, 2) > R(2, 0) ? theta * std::sqrt(1.0 + (R(1, 1) - 1.0) * delta) : -theta * std::sqrt(1.0 + (R(1, 1) - 1.0) * delta);
    r[2] = R(1, 0) > R(0, 1) ? theta * std::sqrt(1.0 + (R(2, 2) - 1.0) * delta) : -theta * std::sqrt(1.0 + (R(2, 2) - 1.0) * delta);
    return r;
  }
  double alpha = theta > DART_EPSILON ? 0.5 * theta / std::sin(theta) : 0.5 + (1.0 / 12.0) * theta * theta;
  r[0] = alpha * (R(2, 1) - R(1, 2));
  r[1] = alpha * (R(0, 2) - R(2, 0));
  r[2] = alpha * (R(1, 0) - R(0, 1));
  return r;
}

}  // namespace oracle
