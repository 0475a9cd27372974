// ORACLE / TEST INFRASTRUCTURE ONLY -- see nimble_oracle.cpp header.
//
// Capsule-box narrow phase of the half-cheetah world (data/skel/half_cheetah.skel:
// capsule colliders on a ground box), restating
//  * libccd's Minkowski Portal Refinement, ccdMPRPenetration (libccd 2.x
//    src/mpr.c: discoverPortal, refinePortal, findPenetr, findPenetrTouch,
//    findPenetrSegment, findPos; src/vec3.c ccdVec3PointTriDist2).  libccd is a
//    third-party dependency of the reference (cmake/DARTFindccd.cmake:
//    find_package(ccd 2.0)) that is not vendored under /root/reference; the
//    published algorithm is restated and parity is anchored on the
//    reference's capsule-box known-answer tests
//    (unittests/unit/test_DARTCollide.cpp:2572, :2738) -- tests/test_oracle_pins.py;
//  * the reference's ccd callbacks and settings: ccdSupportBox
//    (DARTCollide.cpp:1885), ccdSupportCapsule (:1983), ccdCenterBox (:2023),
//    ccdCenterCapsule (:2051), setCcdDefaultSettings (:3698);
//  * collideBoxCapsule (:4422) / collideCapsuleBox (:4533), collideBoxSphere
//    (:1482, with the TOP/BOTTOM half-space clip) / collideSphereBox (:1655),
//    ccdPointsAtWitnessBox (:2060), the face branch of createCapsuleMeshContact
//    (:3366) with createFaceFaceContacts (:2203), keepOnlyConvex2DHull (:3545),
//    math::prepareConvex2DShape / pointInPlane (dart/math/Geometry.cpp:3813,
//    :3843), convex2DShapeContains (:3756), get2DLineIntersection (:3790).
// and createCapsuleMeshContact's vertex-pipe (one box witness point),
// edge-pipe (two; :3071, :3225, the parallel case :3122) branches and the
// EDGE_EDGE contacts of its face branch, converted to PIPE_EDGE / EDGE_PIPE
// (:3320, :3494) -- with createFaceFaceContacts' edge intersections (:2403,
// get2DLineIntersection :3790, math::getContactPoint Geometry.cpp:1075).
// Flagged `unsupported`: the parallel case's SPHERE_EDGE contacts (kept; the
// reference carries a NaN sphere centre into their gradients) and the
// 8-point witness set of a zero penetration direction (dropped).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <vector>

#include "oracle.hpp"

namespace oracle {

namespace {

const double kEps = std::numeric_limits<double>::epsilon();  // CCD_EPS (double build)

inline bool isZero(double v) { return std::fabs(v) < kEps; }
inline bool ccdEq(double a, double b) {
  double ab = std::fabs(a - b);
  if (std::fabs(ab) < kEps) return true;
  a = std::fabs(a);
  b = std::fabs(b);
  return b > a ? ab < kEps * b : ab < kEps * a;
}
inline int ccdSign(double v) { return isZero(v) ? 0 : (v < 0 ? -1 : 1); }

struct V { double x[3]; };
inline V mk(double a, double b, double c) { V r; r.x[0] = a; r.x[1] = b; r.x[2] = c; return r; }
inline V operator-(const V& a, const V& b) { return mk(a.x[0] - b.x[0], a.x[1] - b.x[1], a.x[2] - b.x[2]); }
inline V operator+(const V& a, const V& b) { return mk(a.x[0] + b.x[0], a.x[1] + b.x[1], a.x[2] + b.x[2]); }
inline V operator*(const V& a, double s) { return mk(a.x[0] * s, a.x[1] * s, a.x[2] * s); }
inline double dot(const V& a, const V& b) { return a.x[0] * b.x[0] + a.x[1] * b.x[1] + a.x[2] * b.x[2]; }
inline V cross(const V& a, const V& b) {
  return mk(a.x[1] * b.x[2] - a.x[2] * b.x[1], a.x[2] * b.x[0] - a.x[0] * b.x[2], a.x[0] * b.x[1] - a.x[1] * b.x[0]);
}
inline double len2(const V& a) { return dot(a, a); }
// ccdVec3Normalize: scale by 1/sqrt(len2)
inline V ccdNormalize(const V& a) { return a * (1.0 / std::sqrt(len2(a))); }
// Eigen normalized(): divide by the norm (when positive)
inline V eigNormalized(const V& a) {
  double z = len2(a);
  if (z > 0) { double s = std::sqrt(z); return mk(a.x[0] / s, a.x[1] / s, a.x[2] / s); }
  return a;
}

// rigid transform, R row-major
struct Xf { double R[9]; V p; };
inline V rot(const Xf& T, const V& v) {
  return mk(T.R[0] * v.x[0] + T.R[1] * v.x[1] + T.R[2] * v.x[2], T.R[3] * v.x[0] + T.R[4] * v.x[1] + T.R[5] * v.x[2],
            T.R[6] * v.x[0] + T.R[7] * v.x[1] + T.R[8] * v.x[2]);
}
inline V rotT(const Xf& T, const V& v) {
  return mk(T.R[0] * v.x[0] + T.R[3] * v.x[1] + T.R[6] * v.x[2], T.R[1] * v.x[0] + T.R[4] * v.x[1] + T.R[7] * v.x[2],
            T.R[2] * v.x[0] + T.R[5] * v.x[1] + T.R[8] * v.x[2]);
}
inline V xf(const Xf& T, const V& v) { return rot(T, v) + T.p; }
// Eigen's Isometry inverse applied to v: R^T v + (-(R^T p))
inline V xfInv(const Xf& T, const V& v) { return rotT(T, v) - rotT(T, T.p); }
inline V col(const Xf& T, int c) { return mk(T.R[c], T.R[3 + c], T.R[6 + c]); }

// ccd objects: box (size), capsule (radius, height) or mesh (vertex list,
// scale in size)
struct Obj {
  bool capsule;
  Xf T;
  double size[3];
  double r, h;
  const std::vector<double>* mesh = nullptr;
};

// ccdSupportMesh (DARTCollide.cpp:1935): the first vertex of largest
// v . (R^T dir / scale), scaled and transformed
V meshSupport(const Obj& o, const V& dir) {
  V ld = rotT(o.T, dir);
  ld.x[0] /= o.size[0];
  ld.x[1] /= o.size[1];
  ld.x[2] /= o.size[2];
  double maxDot = -std::numeric_limits<double>::infinity();
  V best = mk(0, 0, 0);
  const std::vector<double>& v = *o.mesh;
  for (size_t k = 0; k + 2 < v.size(); k += 3) {
    const double d = v[k] * ld.x[0] + v[k + 1] * ld.x[1] + v[k + 2] * ld.x[2];
    if (d > maxDot) { maxDot = d; best = mk(v[k], v[k + 1], v[k + 2]); }
  }
  best.x[0] *= o.size[0];
  best.x[1] *= o.size[1];
  best.x[2] *= o.size[2];
  return xf(o.T, best);
}

void support(const Obj& o, const V& dir, V& out) {
  if (o.mesh) { out = meshSupport(o, dir); return; }
  V ld = rotT(o.T, dir);
  if (!o.capsule) {  // ccdSupportBox (DARTCollide.cpp:1885)
    V c = mk(ccdSign(ld.x[0]) * o.size[0] * 0.5, ccdSign(ld.x[1]) * o.size[1] * 0.5, ccdSign(ld.x[2]) * o.size[2] * 0.5);
    out = xf(o.T, c);
  } else {  // ccdSupportCapsule (:1983)
    ld = eigNormalized(ld) * o.r;
    if (std::fabs(ld.x[2]) < 1e-10) out = xf(o.T, ld);
    else if (ld.x[2] > 0) out = xf(o.T, ld + mk(0, 0, o.h / 2));
    else out = xf(o.T, ld + mk(0, 0, -o.h / 2));
  }
}

struct Supp { V v, v1, v2; };

void ccdSupport(const Obj& a, const Obj& b, const V& dir, Supp& s) {
  support(a, dir, s.v1);
  support(b, dir * -1.0, s.v2);
  s.v = s.v1 - s.v2;
}

struct Portal { Supp p[4]; int size = 0; };

void portalDir(const Portal& P, V& dir) {
  V v2v1 = P.p[2].v - P.p[1].v, v3v1 = P.p[3].v - P.p[1].v;
  dir = ccdNormalize(cross(v2v1, v3v1));
}
bool portalEncapsulesOrigin(const Portal& P, const V& dir) {
  double d = dot(dir, P.p[1].v);
  return isZero(d) || d > 0;
}
bool portalReachTolerance(const Portal& P, const Supp& v4, const V& dir, double tol) {
  double dv1 = dot(P.p[1].v, dir), dv2 = dot(P.p[2].v, dir), dv3 = dot(P.p[3].v, dir), dv4 = dot(v4.v, dir);
  double d1 = dv4 - dv1, d2 = dv4 - dv2, d3 = dv4 - dv3;
  d1 = std::fmin(d1, d2);
  d1 = std::fmin(d1, d3);
  return ccdEq(d1, tol) || d1 < tol;
}
bool portalCanEncapsuleOrigin(const Supp& v4, const V& dir) {
  double d = dot(v4.v, dir);
  return isZero(d) || d > 0;
}
void expandPortal(Portal& P, const Supp& v4) {
  V v4v0 = cross(v4.v, P.p[0].v);
  if (dot(P.p[1].v, v4v0) > 0) {
    if (dot(P.p[2].v, v4v0) > 0) P.p[1] = v4;
    else P.p[3] = v4;
  } else {
    if (dot(P.p[3].v, v4v0) > 0) P.p[2] = v4;
    else P.p[1] = v4;
  }
}

// returns -1 no intersection, 0 portal found, 1 touching on v1, 2 origin on v0-v1
int discoverPortal(const Obj& a, const Obj& b, Portal& P) {
  // findOrigin: center1 - center2
  P.p[0].v1 = a.T.p;
  P.p[0].v2 = b.T.p;
  P.p[0].v = P.p[0].v1 - P.p[0].v2;
  P.size = 1;
  const V& c0 = P.p[0].v;
  if (isZero(c0.x[0]) && isZero(c0.x[1]) && isZero(c0.x[2])) P.p[0].v.x[0] += kEps * 10.0;
  V dir = ccdNormalize(P.p[0].v * -1.0);
  ccdSupport(a, b, dir, P.p[1]);
  P.size = 2;
  double d = dot(P.p[1].v, dir);
  if (isZero(d) || d < 0) return -1;
  dir = cross(P.p[0].v, P.p[1].v);
  if (isZero(len2(dir))) {
    const V& v1 = P.p[1].v;
    if (isZero(v1.x[0]) && isZero(v1.x[1]) && isZero(v1.x[2])) return 1;
    return 2;
  }
  dir = ccdNormalize(dir);
  ccdSupport(a, b, dir, P.p[2]);
  d = dot(P.p[2].v, dir);
  if (isZero(d) || d < 0) return -1;
  P.size = 3;
  V va = P.p[1].v - P.p[0].v, vb = P.p[2].v - P.p[0].v;
  dir = ccdNormalize(cross(va, vb));
  if (dot(dir, P.p[0].v) > 0) {
    std::swap(P.p[1], P.p[2]);
    dir = dir * -1.0;
  }
  while (P.size < 4) {
    ccdSupport(a, b, dir, P.p[3]);
    d = dot(P.p[3].v, dir);
    if (isZero(d) || d < 0) return -1;
    bool cont = false;
    va = cross(P.p[1].v, P.p[3].v);
    d = dot(va, P.p[0].v);
    if (d < 0 && !isZero(d)) { P.p[2] = P.p[3]; cont = true; }
    if (!cont) {
      va = cross(P.p[3].v, P.p[2].v);
      d = dot(va, P.p[0].v);
      if (d < 0 && !isZero(d)) { P.p[1] = P.p[3]; cont = true; }
    }
    if (cont) {
      va = P.p[1].v - P.p[0].v;
      vb = P.p[2].v - P.p[0].v;
      dir = ccdNormalize(cross(va, vb));
    } else {
      P.size = 4;
    }
  }
  return 0;
}

int refinePortal(const Obj& a, const Obj& b, Portal& P, double tol) {
  V dir;
  Supp v4;
  for (;;) {
    portalDir(P, dir);
    if (portalEncapsulesOrigin(P, dir)) return 0;
    ccdSupport(a, b, dir, v4);
    if (!portalCanEncapsuleOrigin(v4, dir) || portalReachTolerance(P, v4, dir, tol)) return -1;
    expandPortal(P, v4);
  }
}

// __ccdVec3PointSegmentDist2
double pointSegmentDist2(const V& P, const V& x0, const V& b, V* witness) {
  V d = b - x0, a = x0 - P;
  double t = -1.0 * dot(a, d);
  t /= len2(d);
  if (t < 0 || isZero(t)) {
    if (witness) *witness = x0;
    return len2(x0 - P);
  } else if (t > 1.0 || ccdEq(t, 1.0)) {
    if (witness) *witness = b;
    return len2(b - P);
  }
  V w = d * t + x0;
  if (witness) *witness = w;
  return len2(w - P);
}

// ccdVec3PointTriDist2 with a witness
double pointTriDist2(const V& P, const V& x0, const V& B, const V& C, V& witness) {
  V d1 = B - x0, d2 = C - x0, a = x0 - P;
  double u = dot(a, a), v = dot(d1, d1), w = dot(d2, d2), p = dot(a, d1), q = dot(a, d2), r = dot(d1, d2);
  (void)u;
  double d = w * v - r * r, s, t;
  if (isZero(d)) {
    s = t = -1.0;
  } else {
    s = (q * r - w * p) / d;
    t = (-s * r - q) / w;
  }
  if ((isZero(s) || s > 0) && (ccdEq(s, 1.0) || s < 1.0) && (isZero(t) || t > 0) && (ccdEq(t, 1.0) || t < 1.0) &&
      (ccdEq(t + s, 1.0) || t + s < 1.0)) {
    witness = x0 + d1 * s + d2 * t;
    return len2(witness - P);
  }
  V w2;
  double dist = pointSegmentDist2(P, x0, B, &witness);
  double dist2 = pointSegmentDist2(P, x0, C, &w2);
  if (dist2 < dist) { dist = dist2; witness = w2; }
  dist2 = pointSegmentDist2(P, B, C, &w2);
  if (dist2 < dist) { dist = dist2; witness = w2; }
  return dist;
}

void findPos(const Portal& P, V& pos) {
  V dir;
  portalDir(P, dir);
  double b[4];
  b[0] = dot(cross(P.p[1].v, P.p[2].v), P.p[3].v);
  b[1] = dot(cross(P.p[3].v, P.p[2].v), P.p[0].v);
  b[2] = dot(cross(P.p[0].v, P.p[1].v), P.p[3].v);
  b[3] = dot(cross(P.p[2].v, P.p[1].v), P.p[0].v);
  double sum = b[0] + b[1] + b[2] + b[3];
  if (isZero(sum) || sum < 0) {
    b[0] = 0.0;
    b[1] = dot(cross(P.p[2].v, P.p[3].v), dir);
    b[2] = dot(cross(P.p[3].v, P.p[1].v), dir);
    b[3] = dot(cross(P.p[1].v, P.p[2].v), dir);
    sum = b[1] + b[2] + b[3];
  }
  double inv = 1.0 / sum;
  V p1 = mk(0, 0, 0), p2 = mk(0, 0, 0);
  for (int i = 0; i < 4; i++) {
    p1 = p1 + P.p[i].v1 * b[i];
    p2 = p2 + P.p[i].v2 * b[i];
  }
  p1 = p1 * inv;
  p2 = p2 * inv;
  pos = (p1 + p2) * 0.5;
}

void findPenetr(const Obj& a, const Obj& b, Portal& P, double tol, unsigned long maxIt, double& depth, V& pdir,
                V& pos) {
  V dir;
  Supp v4;
  unsigned long it = 0;
  for (;;) {
    portalDir(P, dir);
    ccdSupport(a, b, dir, v4);
    if (portalReachTolerance(P, v4, dir, tol) || it > maxIt) {
      depth = std::sqrt(pointTriDist2(mk(0, 0, 0), P.p[1].v, P.p[2].v, P.p[3].v, pdir));
      if (isZero(depth)) pdir = mk(0, 0, 0);
      else pdir = ccdNormalize(pdir);
      findPos(P, pos);
      return;
    }
    expandPortal(P, v4);
    it++;
  }
}

// ccdMPRPenetration: 0 = intersecting (depth/dir/pos set), -1 = separated
int mprPenetration(const Obj& a, const Obj& b, double& depth, V& dir, V& pos) {
  const double tol = 0.0001;          // setCcdDefaultSettings: mpr_tolerance
  const unsigned long maxIt = 10000;  //                        max_iterations
  Portal P;
  int res = discoverPortal(a, b, P);
  if (res < 0) return -1;
  if (res == 1) {  // findPenetrTouch
    depth = 0.0;
    dir = mk(0, 0, 0);
    pos = (P.p[1].v1 + P.p[1].v2) * 0.5;
  } else if (res == 2) {  // findPenetrSegment
    pos = (P.p[1].v1 + P.p[1].v2) * 0.5;
    dir = P.p[1].v;
    depth = std::sqrt(len2(dir));
    dir = ccdNormalize(dir);
  } else {
    if (refinePortal(a, b, P, tol) < 0) return -1;
    findPenetr(a, b, P, tol, maxIt, depth, dir, pos);
  }
  return 0;
}

// ccdPointsAtWitnessBox (DARTCollide.cpp:2060)
std::vector<V> witnessBox(const Obj& box, const V& dir, bool neg) {
  const double kPlane = 0.01;  // DART_COLLISION_WITNESS_PLANE_DEPTH
  V ld = rotT(box.T, dir);
  std::vector<V> local;
  const double bx[2] = {box.size[0] * 0.5, box.size[0] * -0.5};
  const double by[2] = {box.size[1] * 0.5, box.size[1] * -0.5};
  const double bz[2] = {box.size[2] * 0.5, box.size[2] * -0.5};
  for (double x : bx)
    for (double y : by)
      for (double z : bz) local.push_back(mk(x, y, z));
  const double nm = neg ? -1.0 : 1.0;
  double maxDot = -std::numeric_limits<double>::infinity();
  for (const V& l : local) maxDot = std::max(maxDot, nm * dot(l, ld));
  std::vector<V> pts;
  for (const V& l : local)
    if (maxDot - nm * dot(l, ld) < kPlane) pts.push_back(xf(box.T, l));
  return pts;
}

// sphere-box contact (collideBoxSphere :1482 when boxFirst, collideSphereBox
// :1655 otherwise); halfspace 0 BOTH, 1 TOP, 2 BOTTOM (BOX_SPHERE only, the
// sphere-box variant ignores it).  sphereT = capsule transform (for the
// half-space test) and its centre c0.
int sphereBox(const Obj& box, const V& c0, const Xf* sphereT, double r, bool boxFirst, int halfspace, double clip,
              Contact& out) {
  const double kEpsCol = 1e-6;  // DART_COLLISION_EPS
  V half = mk(0.5 * box.size[0], 0.5 * box.size[1], 0.5 * box.size[2]);
  bool inside = true;
  V p = xfInv(box.T, c0);
  Contact c{};
  for (int i = 0; i < 3; i++) c.sphereCenter[i] = c0.x[i];
  for (int a = 0; a < 3; a++) {
    if (p.x[a] < -half.x[a]) {
      c.faceLocked[a] = 1;
      V n = col(box.T, a);
      for (int i = 0; i < 3; i++) c.faceNormal[3 * a + i] = n.x[i];
      p.x[a] = -half.x[a];
      inside = false;
    }
    if (p.x[a] > half.x[a]) {
      c.faceLocked[a] = 1;
      V n = col(box.T, a);
      for (int i = 0; i < 3; i++) c.faceNormal[3 * a + i] = n.x[i];
      p.x[a] = half.x[a];
      inside = false;
    }
  }
  auto nearestFace = [&](int& idx) {
    double mn = half.x[0] - std::fabs(p.x[0]);
    double t = half.x[1] - std::fabs(p.x[1]);
    idx = 0;
    if (t < mn) { mn = t; idx = 1; }
    t = half.x[2] - std::fabs(p.x[2]);
    if (t < mn) { mn = t; idx = 2; }
    return mn;
  };
  const double sgnIn = boxFirst ? -1.0 : 1.0;  // box-first variants flip the face normal
  if (inside) {
    int idx;
    double mn = nearestFace(idx);
    V nl = mk(0, 0, 0);
    nl.x[idx] = p.x[idx] > 0.0 ? sgnIn : -sgnIn;
    V n = rot(box.T, nl);
    double pen = mn + r;
    if (pen > clip) return 0;
    c.type = boxFirst ? 1 /*CT_FACE_VERTEX*/ : 2 /*CT_VERTEX_FACE*/;
    for (int i = 0; i < 3; i++) { c.point[i] = c0.x[i]; c.normal[i] = n.x[i]; }
    c.depth = pen;
    out = c;
    return 1;
  }
  V cp = xf(box.T, p);
  V n = boxFirst ? cp - c0 : c0 - cp;
  double mag = std::sqrt(len2(n));
  double pen = r - mag;
  if (pen > clip) return 0;
  if (boxFirst && sphereT) {
    // (T1.inverse() * contactpt)(2) with T1 = capsule transform * translation(0, 0, +-h/2)
    V loc = xfInv(*sphereT, cp);
    if (halfspace == 2 && loc.x[2] >= 0) return 0;
    if (halfspace == 1 && loc.x[2] <= 0) return 0;
  }
  if (pen < 0.0) return 0;
  if (mag > kEpsCol) {
    n = n * (1.0 / mag);
  } else {
    int idx;
    nearestFace(idx);
    V nl = mk(0, 0, 0);
    nl.x[idx] = p.x[idx] > 0.0 ? sgnIn : -sgnIn;
    n = rot(box.T, nl);
  }
  c.type = boxFirst ? 5 /*BOX_SPHERE*/ : 4 /*SPHERE_BOX*/;
  for (int i = 0; i < 3; i++) { c.point[i] = cp.x[i]; c.normal[i] = n.x[i]; }
  c.depth = pen;
  out = c;
  return 1;
}

inline double cross2(double ax, double ay, double bx, double by) { return ax * by - ay * bx; }

struct P2 { double x, y; };
inline P2 inPlane(const V& pt, const V& o, const V& bx, const V& by) { V d = pt - o; return {dot(d, bx), dot(d, by)}; }

void keepOnlyConvexHull(std::vector<V>& shape, const V& o, const V& bx, const V& by) {
  while (!shape.empty()) {
    bool removed = false;
    for (size_t i = 0; i < shape.size(); i++) {
      bool boundary = false;
      P2 si = inPlane(shape[i], o, bx, by);
      for (size_t j = 0; j < shape.size() && !boundary; j++) {
        if (i == j) continue;
        P2 sj = inPlane(shape[j], o, bx, by);
        double px = si.y - sj.y, py = sj.x - si.x;
        double nrm2 = px * px + py * py;
        if (nrm2 > 0) { double s = std::sqrt(nrm2); px /= s; py /= s; }
        double b = -(px * si.x + py * si.y);
        bool isB = true;
        int side = 0;
        for (size_t k = 0; k < shape.size(); k++) {
          P2 sk = inPlane(shape[k], o, bx, by);
          double meas = px * sk.x + py * sk.y + b;
          int ks = ccdSign(meas);
          if (std::fabs(meas) < 1e-3) {
          } else if (side == 0) {
            side = ks;
          } else if (side != ks) {
            isB = false;
            break;
          }
        }
        if (isB) boundary = true;
      }
      if (!boundary) {
        shape.erase(shape.begin() + i);
        removed = true;
        break;
      }
    }
    if (!removed) break;
  }
}

void prepareConvex(std::vector<V>& shape, const V& o, const V& bx, const V& by) {
  double ax = 0, ay = 0;
  for (const V& pt : shape) { P2 q = inPlane(pt, o, bx, by); ax += q.x; ay += q.y; }
  ax /= (double)shape.size();
  ay /= (double)shape.size();
  std::stable_sort(shape.begin(), shape.end(), [&](const V& a, const V& b) {
    P2 qa = inPlane(a, o, bx, by), qb = inPlane(b, o, bx, by);
    return std::atan2(qa.y - ay, qa.x - ax) < std::atan2(qb.y - ay, qb.x - ax);
  });
}

bool convexContains(const V& pt, const std::vector<V>& shape, const V& o, const V& bx, const V& by) {
  P2 q = inPlane(pt, o, bx, by);
  int side = 0;
  for (size_t i = 0; i < shape.size(); i++) {
    P2 a = inPlane(shape[i], o, bx, by), b = inPlane(shape[(i + 1) % shape.size()], o, bx, by);
    int ts = ccdSign(cross2(q.x - a.x, q.y - a.y, b.x - a.x, b.y - a.y));
    if (i == 0) side = ts;
    else if (ts == 0) continue;
    else if (side == 0 && ts != 0) side = ts;
    else if (side != ts && side != 0) return false;
  }
  return true;
}

// get2DLineIntersection (:3790), including its collinear branch's
// out = p + s t (sic)
bool lineIntersect2D(P2 p, P2 p1, P2 q, P2 q1, P2* out = nullptr) {
  double rx = p1.x - p.x, ry = p1.y - p.y, sx = q1.x - q.x, sy = q1.y - q.y;
  double rs = cross2(rx, ry, sx, sy);
  if (rs == 0 && cross2(q.x - p.x, q.y - p.y, rx, ry) == 0) {
    double rr = rx * rx + ry * ry;
    double t0 = ((q.x - p.x) * rx + (q.y - p.y) * ry) / rr;
    double t1 = ((q.x + sx - p.x) * rx + (q.y + sy - p.y) * ry) / rr;
    if (t0 >= 0 && t0 <= 1) { if (out) *out = {p.x + sx * t0, p.y + sy * t0}; return true; }
    if (t1 >= 0 && t1 <= 1) { if (out) *out = {p.x + sx * t1, p.y + sy * t1}; return true; }
    return false;
  } else if (rs == 0) {
    return false;
  }
  double t = cross2(q.x - p.x, q.y - p.y, sx, sy) / rs;
  double u = cross2(p.x - q.x, p.y - q.y, rx, ry) / cross2(sx, sy, rx, ry);
  if (t >= 0 && t <= 1 && u >= 0 && u <= 1) {
    if (out) *out = {p.x + t * rx, p.y + t * ry};
    return true;
  }
  return false;
}

// dSegmentsClosestApproach (DARTCollide.cpp:301): segment pa -> pb against
// ua -> ub, parameters not clamped beyond the routine's own edge cases
void segmentsClosestApproach(const double* pa, const double* ua, const double* pb, const double* ub, double* alpha,
                             double* beta) {
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
  *alpha = std::fabs(sN) < 1e-15 ? 0.0 : sN / sD;
  *beta = std::fabs(tN) < 1e-15 ? 0.0 : tN / tD;
}

// math::getContactPoint (Geometry.cpp:1075) via dLineClosestApproach (:1042)
V contactPoint(const V& pA, const V& uA, const V& pB, const V& uB, double rA, double rB) {
  V p = pB - pA;
  const double uaub = dot(uA, uB), q1 = dot(uA, p), q2 = -dot(uB, p);
  double d = 1 - uaub * uaub, alpha = 0, beta = 0;
  if (d > 0) {
    d = 1.0 / d;
    alpha = (q1 + uaub * q2) * d;
    beta = (uaub * q1 + q2) * d;
  }
  V ca = pA + uA * alpha, cb = pB + uB * beta;
  return (ca * rB + cb * rA) * (1.0 / (rA + rB));
}

// createFaceFaceContacts (:2203) restricted to its vertex-in-hull contacts
// (VERTEX_FACE for A's vertices, FACE_VERTEX for B's); the edge-edge
// intersections it would also emit are counted in *edgeEdge.
// type 1 VERTEX_FACE, 2 FACE_VERTEX, 3 EDGE_EDGE (edge A / B fixed point,
// direction and closest point)
struct FFContact {
  V point, normal;
  double depth;
  int type;
  V aFixed, aDir, aClosest, bFixed, bDir, bClosest;
};
void faceFaceVertices(const V& dir, const std::vector<V>& A, const std::vector<V>& B, int pin,
                      std::vector<FFContact>& outv, int* edgeEdge) {
  auto faceNormal = [&](const std::vector<V>& P) {
    return eigNormalized(cross(P[0] - P[1], P[1] - (P.size() > 2 ? P[2] : dir)));
  };
  V nA = faceNormal(A), nB = faceNormal(B);
  auto broken = [&](const V& n) {
    return std::fabs(len2(n) - 1) > 1e-10 || std::min(len2(n - dir), len2(n * -1.0 - dir)) > 0.2;
  };
  bool aB = broken(nA), bB = broken(nB);
  if (aB && !bB) nA = nB;
  else if (!aB && bB) nB = nA;
  else if (aB && bB) { nA = dir * -1.0; nB = nA; }
  if (nA.x[0] * dir.x[0] + nA.x[1] * dir.x[1] + nA.x[2] * dir.x[2] > 0) nA = nA * -1.0;
  if (nB.x[0] * dir.x[0] + nB.x[1] * dir.x[1] + nB.x[2] * dir.x[2] > 0) nB = nB * -1.0;
  V normal = eigNormalized((nA + nB) * 0.5);
  V oA = normal * dot(A[0], normal);
  V oB = normal * dot(B[0], normal);
  V origin = (oA + oB) * 0.5;
  if (pin == 1) { origin = oA; normal = nA; }
  else if (pin == 2) { origin = oB; normal = nB; }
  V tmp = cross(normal, mk(0, 0, 1));
  if (len2(tmp) < 1e-4) tmp = cross(normal, mk(1, 0, 0));
  V bx = cross(nA, tmp);
  V by = cross(nA, bx);
  std::vector<V> Ah = A, Bh = B;
  keepOnlyConvexHull(Ah, origin, bx, by);
  std::vector<V> As = Ah;
  prepareConvex(As, origin, bx, by);
  keepOnlyConvexHull(Bh, origin, bx, by);
  std::vector<V> Bs = Bh;
  prepareConvex(Bs, origin, bx, by);
  for (const V& va : Ah) {
    if (!convexContains(va, Bs, origin, bx, by)) continue;
    FFContact c;
    c.point = va;
    if (pin == 2) c.point = oB + bx * dot(bx, c.point) + by * dot(by, c.point);
    double distA = dot(va, nB), distB = dot(B[0], nB);
    c.normal = pin == 2 ? nA : nB;
    c.depth = distB - distA;
    c.type = 1;
    outv.push_back(c);
  }
  for (const V& vb : Bh) {
    if (!convexContains(vb, As, origin, bx, by)) continue;
    FFContact c;
    c.point = vb;
    if (pin == 1) c.point = oA + bx * dot(bx, c.point) + by * dot(by, c.point);
    double distA = dot(A[0], nA), distB = dot(vb, nA);
    c.normal = pin == 1 ? nB : nA;
    c.depth = distB - distA;
    c.type = 2;
    outv.push_back(c);
  }
  int ee = 0;
  for (size_t i = 0; i < As.size(); i++) {
    if (i == As.size() - 1 && As.size() == 2) continue;
    const V& a1w = As[i];
    const V& a2w = As[i == As.size() - 1 ? 0 : i + 1];
    P2 a1 = inPlane(a1w, origin, bx, by), a2 = inPlane(a2w, origin, bx, by);
    for (size_t j = 0; j < Bs.size(); j++) {
      if (j == Bs.size() - 1 && Bs.size() == 2) continue;
      const V& b1w = Bs[j];
      const V& b2w = Bs[j == Bs.size() - 1 ? 0 : j + 1];
      P2 b1 = inPlane(b1w, origin, bx, by), b2 = inPlane(b2w, origin, bx, by);
      P2 o;
      if (!lineIntersect2D(a1, a2, b1, b2, &o)) continue;
      ee++;
      // createFaceFaceContacts' EDGE_EDGE contact (:2441)
      FFContact c;
      c.type = 3;
      c.aClosest = oA + bx * o.x + by * o.y;
      c.bClosest = oB + bx * o.x + by * o.y;
      c.aFixed = a1w;
      c.aDir = eigNormalized(a2w - a1w);
      c.bFixed = b1w;
      c.bDir = eigNormalized(b2w - b1w);
      c.normal = cross(c.aDir, c.bDir);
      if (dot(c.normal, nA) < 0) c.normal = c.normal * -1.0;
      c.depth = dot(c.bClosest, c.normal) - dot(c.aClosest, c.normal);
      if (c.depth < 0) { c.normal = c.normal * -1.0; c.depth = -c.depth; }
      const double rA = pin == 1 ? 0.0 : 1.0, rB = pin == 2 ? 0.0 : 1.0;
      c.point = contactPoint(c.aFixed, c.aDir, c.bFixed, c.bDir, rA, rB);
      outv.push_back(c);
    }
  }
  *edgeEdge = ee;
}

// ccdPointsAtWitnessMesh (DARTCollide.cpp:2119): the vertices within the
// witness plane depth of the extreme one along dir (the least when neg),
// scaled and transformed, dropping any within 1e-3 m of one already taken
std::vector<V> witnessMesh(const Obj& o, const V& dir, bool neg) {
  const double kPlane = 0.01;  // DART_COLLISION_WITNESS_PLANE_DEPTH
  V ld = rotT(o.T, dir);
  ld.x[0] /= o.size[0];
  ld.x[1] /= o.size[1];
  ld.x[2] /= o.size[2];
  const std::vector<double>& v = *o.mesh;
  auto dotOf = [&](size_t k) {
    return v[k] * ld.x[0] * o.size[0] * o.size[0] + v[k + 1] * ld.x[1] * o.size[1] * o.size[1] +
           v[k + 2] * ld.x[2] * o.size[2] * o.size[2];
  };
  double maxDot = (neg ? 1.0 : -1.0) * std::numeric_limits<double>::infinity();
  for (size_t k = 0; k + 2 < v.size(); k += 3) {
    const double d = dotOf(k);
    if ((d > maxDot && !neg) || (d < maxDot && neg)) maxDot = d;
  }
  std::vector<V> pts;
  for (size_t k = 0; k + 2 < v.size(); k += 3) {
    const double d = dotOf(k);
    if (std::fabs(d - maxDot) < kPlane) {
      const V p = xf(o.T, mk(v[k] * o.size[0], v[k + 1] * o.size[1], v[k + 2] * o.size[2]));
      bool dup = false;
      for (const V& q : pts)
        if (len2(q - p) < 1e-6) { dup = true; break; }
      if (!dup) pts.push_back(p);
    }
  }
  return pts;
}

// createMeshMeshContacts (DARTCollide.cpp:2508) on the witness sets A (object
// 1) and B (object 2); contacts in the reference's order.  Returns false for
// an empty witness set (the reference asserts).
bool meshMeshContacts(const V& dir, const std::vector<V>& A, const std::vector<V>& B, std::vector<Contact>& outc) {
  auto setV = [](double* o, const V& x) { for (int i = 0; i < 3; i++) o[i] = x.x[i]; };
  auto dirDot = [&](const V& n) { return n.x[0] * dir.x[0] + n.x[1] * dir.x[1] + n.x[2] * dir.x[2]; };
  if (A.empty() || B.empty()) return false;
  const size_t na = A.size(), nb = B.size();
  if (std::getenv("ORACLE_MESH_DEBUG")) std::fprintf(stderr, "mmc na=%zu nb=%zu dir=%.6f %.6f %.6f\n", na, nb, dir.x[0], dir.x[1], dir.x[2]);
  if ((na == 1 && nb > 2) || (na > 2 && nb == 1)) {
    // single vertex-face (:2551) / face-vertex (:2586)
    const bool vf = na == 1;
    const std::vector<V>& F = vf ? B : A;
    V normal = eigNormalized(cross(F[0] - F[1], F[1] - F[2]));
    if (dirDot(normal) > 0) normal = normal * -1.0;
    Contact c{};
    setV(c.point, vf ? A[0] : B[0]);
    setV(c.normal, normal);
    const double distA = dot(vf ? A[0] : A[0], normal), distB = dot(vf ? B[0] : B[0], normal);
    c.depth = std::fabs(distA - distB);
    c.type = vf ? 2 /*CT_VERTEX_FACE*/ : 1 /*CT_FACE_VERTEX*/;
    outc.push_back(c);
    return true;
  }
  if (na == 2 && nb == 2) {
    // single edge-edge (:2621), dLineClosestApproach (:270)
    const V ua = eigNormalized(A[0] - A[1]), ub = eigNormalized(B[0] - B[1]);
    V pa = A[0], pb = B[0];
    const V pp = pb - pa;
    const double uaub = dot(ua, ub), q1 = dot(ua, pp), q2 = -dot(ub, pp);
    double d = 1 - uaub * uaub, alpha = 0, beta = 0;
    if (d > 0) {
      d = 1.0 / d;
      alpha = (q1 + uaub * q2) * d;
      beta = (uaub * q1 + q2) * d;
    }
    for (int i = 0; i < 3; i++) pa.x[i] += ua.x[i] * alpha;
    for (int i = 0; i < 3; i++) pb.x[i] += ub.x[i] * beta;
    V normal = cross(ua, ub);
    if (dirDot(normal) > 0) normal = normal * -1.0;
    Contact c{};
    setV(c.point, mk(0.5 * (pa.x[0] + pb.x[0]), 0.5 * (pa.x[1] + pb.x[1]), 0.5 * (pa.x[2] + pb.x[2])));
    c.type = 3;  // CT_EDGE_EDGE
    setV(c.edgeAFixed, A[0]); setV(c.edgeADir, ua);
    setV(c.edgeBFixed, B[0]); setV(c.edgeBDir, ub);
    setV(c.normal, normal);
    c.depth = std::fabs(dot(pb, normal) - dot(pa, normal));
    outc.push_back(c);
    return true;
  }
  if ((na == 1 && nb == 2) || (na == 2 && nb == 1)) {
    // vertex-edge (:2702) / edge-vertex (:2736): the normal is dir made
    // orthogonal to the edge -- the edge-vertex branch reads
    // (pointsAWitness[1] - pointsAWitness[1]).normalized() (sic): a zero
    // vector (Eigen leaves it zero), so the normal stays dir
    const bool ve = na == 1;
    V normal = dir;
    if (ve) {
      const V edgeB = eigNormalized(B[0] - B[1]);
      normal = normal - edgeB * dot(normal, edgeB);
    }
    if (dirDot(normal) > 0) normal = normal * -1.0;
    Contact c{};
    setV(c.point, ve ? A[0] : B[0]);
    setV(c.normal, normal);
    c.depth = std::fabs(dot(A[0], normal) - dot(B[0], normal));
    c.type = ve ? 2 /*CT_VERTEX_FACE*/ : 1 /*CT_FACE_VERTEX*/;
    outc.push_back(c);
    return true;
  }
  if (na == 1 && nb == 1) {
    // vertex-vertex (:2771): FACE_VERTEX at B's point, normal -dir
    const V normal = dir * -1.0;
    Contact c{};
    setV(c.point, B[0]);
    setV(c.normal, normal);
    c.depth = std::fabs(dot(B[0], normal) - dot(A[0], normal));
    c.type = 1;  // CT_FACE_VERTEX
    outc.push_back(c);
    return true;
  }
  // edge-face (:2672), face-edge (:2686) and face-face (:2804):
  // createFaceFaceContacts with PinToFace::AVERAGE
  std::vector<FFContact> fc;
  int ee = 0;
  faceFaceVertices(dir, A, B, 0, fc, &ee);
  for (const FFContact& f : fc) {
    Contact c{};
    setV(c.point, f.point);
    setV(c.normal, f.normal);
    c.depth = f.depth;
    if (f.type == 3) {
      c.type = 3;  // CT_EDGE_EDGE
      setV(c.edgeAFixed, f.aFixed); setV(c.edgeADir, f.aDir);
      setV(c.edgeBFixed, f.bFixed); setV(c.edgeBDir, f.bDir);
    } else {
      c.type = f.type == 1 ? 2 /*CT_VERTEX_FACE*/ : 1 /*CT_FACE_VERTEX*/;
    }
    outc.push_back(c);
  }
  return true;
}

}  // namespace

int meshBox(const Iso<double>& Tm, const Shape& mesh, const Iso<double>& Tb, const double* size, bool meshFirst,
            double clip, int shape1, int shape2, int body1, int body2, std::vector<Contact>& out, int* unsupported) {
  Obj box{}, msh{};
  box.capsule = msh.capsule = false;
  for (int i = 0; i < 9; i++) { box.T.R[i] = Tb.R.m[i]; msh.T.R[i] = Tm.R.m[i]; }
  for (int i = 0; i < 3; i++) {
    box.T.p.x[i] = Tb.p[i]; msh.T.p.x[i] = Tm.p[i];
    box.size[i] = size[i]; msh.size[i] = mesh.size[i];
  }
  msh.mesh = &mesh.verts;
  double depth;
  V dir, pos;
  const int intersect = meshFirst ? mprPenetration(msh, box, depth, dir, pos) : mprPenetration(box, msh, depth, dir, pos);
  if (intersect != 0) return 0;
  if (depth > clip) return 0;
  const std::vector<V> A = meshFirst ? witnessMesh(msh, dir, false) : witnessBox(box, dir, false);
  const std::vector<V> B = meshFirst ? witnessBox(box, dir, true) : witnessMesh(msh, dir, true);
  std::vector<Contact> cs;
  if (!meshMeshContacts(dir, A, B, cs)) { *unsupported = 1; return 0; }
  for (Contact& c : cs) {
    c.shapeA = shape1; c.shapeB = shape2; c.bodyA = body1; c.bodyB = body2;
    out.push_back(c);
  }
  return (int)cs.size();
}

// Capsule (radius r, height h along local z, transform Tc) vs box (size, Tb);
// boxFirst selects collideBoxCapsule (box is collision object 1) over
// collideCapsuleBox.  Appends contacts (shape/body indices of object 1 / 2);
// returns the number added, sets *unsupported when a branch that is not
// restated was taken (its contacts are dropped).
int capsuleBox(const Iso<double>& Tb, const double* size, const Iso<double>& Tc, double r, double h, bool boxFirst,
               double clip, int shape1, int shape2, int body1, int body2, std::vector<Contact>& out,
               int* unsupported) {
  Obj box{}, cap{};
  box.capsule = false;
  cap.capsule = true;
  for (int i = 0; i < 9; i++) { box.T.R[i] = Tb.R.m[i]; cap.T.R[i] = Tc.R.m[i]; }
  for (int i = 0; i < 3; i++) { box.T.p.x[i] = Tb.p[i]; cap.T.p.x[i] = Tc.p[i]; box.size[i] = size[i]; }
  cap.r = r;
  cap.h = h;
  double depth;
  V dir, pos;
  int intersect = boxFirst ? mprPenetration(box, cap, depth, dir, pos) : mprPenetration(cap, box, depth, dir, pos);
  if (intersect != 0) return 0;
  if (depth > clip) return 0;
  auto emit = [&](Contact c) {
    c.shapeA = shape1; c.shapeB = shape2; c.bodyA = body1; c.bodyB = body2;
    out.push_back(c);
  };
  V local = xfInv(cap.T, pos);
  if (local.x[2] > h / 2 || local.x[2] < -h / 2) {
    const double zc = local.x[2] > h / 2 ? h / 2 : -h / 2;
    V c0 = xf(cap.T, mk(0, 0, zc));
    Xf ST = cap.T;
    ST.p = c0;  // T1 * translation(0, 0, +-h/2)
    Contact c;
    int k = sphereBox(box, c0, &ST, r, boxFirst, local.x[2] > h / 2 ? 1 : 2, clip, c);
    if (k) emit(c);
    return k;
  }
  // pipe branch: box witness points, createCapsuleMeshContact (:3050) with
  // capsuleA / capsuleB the top / bottom axis points and flipObjectOrder =
  // boxFirst
  std::vector<V> W = witnessBox(box, dir, !boxFirst ? true : false);
  V capA = xf(cap.T, mk(0, 0, h / 2)), capB = xf(cap.T, mk(0, 0, -h / 2));
  const V axis = capB - capA;
  auto setPipe = [&](Contact& c, const V& closest, const V& fixed, const V& pdir) {
    for (int i = 0; i < 3; i++) { c.pipeClosest[i] = closest.x[i]; c.pipeFixed[i] = fixed.x[i]; c.pipeDir[i] = pdir.x[i]; }
    c.pipeRadius = r;
  };
  auto setV = [](double* o, const V& v) { for (int i = 0; i < 3; i++) o[i] = v.x[i]; };
  if (W.size() == 1) {
    // vertex-pipe (:3071): dDistPointToSegment from the vertex to the axis
    const V w = W[0] - capA;
    const double c1 = dot(w, axis), c2 = dot(axis, axis);
    const double alpha = c1 <= 0 ? 0.0 : (c2 <= c1 ? 1.0 : c1 / c2);
    const V nearest = capA + axis * alpha;
    V normal = eigNormalized(nearest - W[0]);
    Contact c{};
    setV(c.point, W[0]);
    if (boxFirst) normal = normal * -1.0;
    setV(c.normal, normal);
    c.type = boxFirst ? CT_VERTEX_PIPE : CT_PIPE_VERTEX;
    setPipe(c, nearest, capA, eigNormalized(axis));
    c.depth = r - std::sqrt(len2(W[0] - nearest));
    if (c.depth > clip) return 0;
    emit(c);
    return 1;
  }
  if (W.size() == 2) {
    const V pipeDir = eigNormalized(axis), edgeDir = eigNormalized(W[1] - W[0]);
    if (std::fabs(1.0 - std::fabs(dot(pipeDir, edgeDir))) < 1e-5) {
      // the edge is parallel to the pipe (:3122-:3300): a contact at each end
      // of the overlap, PIPE_VERTEX (VERTEX_PIPE) at an edge end the capsule
      // passes, else SPHERE_EDGE (EDGE_SPHERE) at the capsule end.  Those
      // leave Contact::sphereCenter NaN (Contact.cpp:59), which their
      // gradients read (DifferentiableContactConstraint.cpp:770): flagged
      // unsupported, the contacts kept.
      const double eA = dot(edgeDir, W[0]), eB = dot(edgeDir, W[1]);
      const double cA = dot(edgeDir, capA), cB = dot(edgeDir, capB);
      const double edgeMin = eA < eB ? eA : eB, edgeMax = eA < eB ? eB : eA;
      const V edgeMinP = eA < eB ? W[0] : W[1], edgeMaxP = eA < eB ? W[1] : W[0];
      const double capMin = cA < cB ? cA : cB, capMax = cA < cB ? cB : cA;
      const V capMinP = cA < cB ? capA : capB, capMaxP = cA < cB ? capB : capA;
      V normal = capA - W[0];
      normal = normal - edgeDir * dot(normal, edgeDir);
      const double dist = std::sqrt(len2(normal));
      normal = eigNormalized(normal);
      const double depth = r - dist;
      int added = 0;
      for (int end = 0; end < 2; end++) {
        const bool low = end == 0;
        Contact c{};
        setV(c.normal, boxFirst ? normal * -1.0 : normal);
        c.depth = depth;
        if (low ? capMin < edgeMin : capMax > edgeMax) {
          const V vp = low ? edgeMinP : edgeMaxP;
          setV(c.point, vp);
          c.type = boxFirst ? CT_VERTEX_PIPE : CT_PIPE_VERTEX;
          // collideCapsuleBox's low end keeps pipeFixedPoint = capsuleB and the
          // unnormalised axis (:3177-:3178); the other three use capsuleA
          const bool asIs = low && !boxFirst;
          setPipe(c, vp + normal * r, asIs ? capB : capA, asIs ? axis : pipeDir);
        } else {
          const V pt = (low ? capMinP : capMaxP) - normal * r;
          setV(c.point, pt);
          c.type = boxFirst ? CT_EDGE_SPHERE : CT_SPHERE_EDGE;
          setV(c.edgeAClosest, pt);
          setV(c.edgeAFixed, W[0]);
          setV(c.edgeADir, edgeDir);
          *unsupported = 1;
        }
        if (c.depth > 0 && c.depth < clip) { emit(c); added++; }
      }
      return added;
    }
    // edge-pipe (:3225): dSegmentsClosestApproach(W0, capA, W1, capB)
    double alpha, beta;
    segmentsClosestApproach(W[0].x, capA.x, W[1].x, capB.x, &alpha, &beta);
    const V edgeClosest = W[0] + (W[1] - W[0]) * alpha;
    const V pipeClosest = capA + axis * beta;
    const V normal = eigNormalized(edgeClosest - pipeClosest);
    Contact c{};
    setV(c.point, edgeClosest);
    setV(c.normal, boxFirst ? normal : normal * -1.0);
    c.type = boxFirst ? CT_EDGE_PIPE : CT_PIPE_EDGE;
    setV(c.edgeAClosest, edgeClosest);
    setV(c.edgeAFixed, W[0]);
    setV(c.edgeADir, edgeDir);
    setPipe(c, pipeClosest, capA, pipeDir);
    c.depth = r - std::sqrt(len2(edgeClosest - pipeClosest));
    if (c.depth > clip) return 0;
    emit(c);
    return 1;
  }
  // > 4 points: a zero penetration direction
  if (W.size() > 4) { *unsupported = 1; return 0; }
  V normal = eigNormalized(cross(W[0] - W[1], W[1] - W[2]));
  if (normal.x[0] * dir.x[0] + normal.x[1] * dir.x[1] + normal.x[2] * dir.x[2] > 0) normal = normal * -1.0;
  std::vector<FFContact> fc;
  int ee = 0;
  if (boxFirst) {
    std::vector<V> cw{capA + normal * r, capB + normal * r};
    faceFaceVertices(dir, W, cw, 1, fc, &ee);
  } else {
    std::vector<V> cw{capA - normal * r, capB - normal * r};
    faceFaceVertices(dir, cw, W, 2, fc, &ee);
  }
  int added = 0;
  for (const FFContact& f : fc) {
    if (f.type == 3) {
      // EDGE_EDGE -> EDGE_PIPE (flipped, :3320) / PIPE_EDGE (:3494)
      if (!(f.depth >= 0 && f.depth < clip)) continue;
      Contact c{};
      setV(c.normal, f.normal);
      c.depth = f.depth;
      if (boxFirst) {
        c.type = CT_EDGE_PIPE;
        setPipe(c, f.bClosest - normal * r, f.bFixed - normal * r, f.bDir);
        setV(c.edgeAFixed, f.aFixed); setV(c.edgeADir, f.aDir); setV(c.edgeAClosest, f.aClosest);
        setV(c.point, f.aClosest);
      } else {
        c.type = CT_PIPE_EDGE;
        setPipe(c, f.aClosest + normal * r, f.aFixed + normal * r, f.aDir);
        setV(c.edgeAFixed, f.bFixed); setV(c.edgeADir, f.bDir); setV(c.edgeAClosest, f.bClosest);
        setV(c.point, f.bClosest);
      }
      emit(c);
      added++;
      continue;
    }
    // flipped: FACE_VERTEX -> FACE_SPHERE; else VERTEX_FACE -> SPHERE_FACE
    if (f.type != (boxFirst ? 2 : 1)) continue;
    V sc = len2(f.point - capA) < len2(f.point - capB) ? capA : capB;
    if (!(f.depth >= 0 && f.depth < clip)) continue;
    Contact c;
    int k = sphereBox(box, sc, nullptr, r, boxFirst, 0, clip, c);
    if (k) { emit(c); added++; }
  }
  return added;
}

// A standalone sphere shape against a box: collideSphereBox (sphere is
// collision object 1) / collideBoxSphere with the default BOTH half-space.
int sphereBoxPair(const Iso<double>& Tb, const double* size, const double* c0, double r, bool boxFirst, double clip,
                  int shape1, int shape2, int body1, int body2, std::vector<Contact>& out) {
  Obj box{};
  box.capsule = false;
  for (int i = 0; i < 9; i++) box.T.R[i] = Tb.R.m[i];
  for (int i = 0; i < 3; i++) { box.T.p.x[i] = Tb.p[i]; box.size[i] = size[i]; }
  Contact c;
  if (!sphereBox(box, mk(c0[0], c0[1], c0[2]), nullptr, r, boxFirst, 0, clip, c)) return 0;
  c.shapeA = shape1; c.shapeB = shape2; c.bodyA = body1; c.bodyB = body2;
  out.push_back(c);
  return 1;
}

}  // namespace oracle

// Raw capsule-box entry for the reference's known-answer tests
// (collideCapsuleBox / collideBoxCapsule signatures: box full size + 3x4
// row-major world transforms).  Output per contact: point3, normal3, depth,
// type (reference ContactType numbering for SPHERE_BOX 4 / BOX_SPHERE 5).
extern "C" int oracle_capsule_box(const double* size, const double* Tbox, double height, double radius,
                                  const double* Tcap, int boxFirst, double clip, double* out) {
  oracle::Iso<double> Tb, Tc;
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) { Tb.R(r, c) = Tbox[r * 4 + c]; Tc.R(r, c) = Tcap[r * 4 + c]; }
    Tb.p[r] = Tbox[r * 4 + 3];
    Tc.p[r] = Tcap[r * 4 + 3];
  }
  std::vector<oracle::Contact> cs;
  int unsup = 0;
  oracle::capsuleBox(Tb, size, Tc, radius, height, boxFirst != 0, clip, 0, 1, 0, 1, cs, &unsup);
  for (size_t k = 0; k < cs.size(); k++) {
    for (int i = 0; i < 3; i++) { out[8 * k + i] = cs[k].point[i]; out[8 * k + 3 + i] = cs[k].normal[i]; }
    out[8 * k + 6] = cs[k].depth;
    out[8 * k + 7] = cs[k].type;
  }
  return unsup ? -1 - (int)cs.size() : (int)cs.size();
}

// Raw mesh-box entry (collideMeshBox / collideBoxMesh with the mesh's vertex
// list, scale and 3x4 transform; box full size + transform).  Output per
// contact: point3, normal3, depth, type (this oracle's CT numbering), edge A
// fixed3 / dir3, edge B fixed3 / dir3 (20 doubles).  Returns the count, or
// -1 - count when the witness sets were empty.
extern "C" int oracle_mesh_box(const double* verts, int nverts, const double* scale, const double* Tmesh,
                               const double* size, const double* Tbox, int meshFirst, double clip, double* out) {
  oracle::Iso<double> Tm, Tb;
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) { Tm.R(r, c) = Tmesh[r * 4 + c]; Tb.R(r, c) = Tbox[r * 4 + c]; }
    Tm.p[r] = Tmesh[r * 4 + 3];
    Tb.p[r] = Tbox[r * 4 + 3];
  }
  oracle::Shape m{};
  m.type = NIMBLE_SHAPE_MESH;
  for (int i = 0; i < 3; i++) m.size[i] = scale[i];
  m.verts.assign(verts, verts + 3 * nverts);
  std::vector<oracle::Contact> cs;
  int unsup = 0;
  oracle::meshBox(Tm, m, Tb, size, meshFirst != 0, clip, 0, 1, 0, 1, cs, &unsup);
  for (size_t k = 0; k < cs.size(); k++) {
    double* o = out + 20 * k;
    for (int i = 0; i < 3; i++) {
      o[i] = cs[k].point[i]; o[3 + i] = cs[k].normal[i];
      o[8 + i] = cs[k].edgeAFixed[i]; o[11 + i] = cs[k].edgeADir[i];
      o[14 + i] = cs[k].edgeBFixed[i]; o[17 + i] = cs[k].edgeBDir[i];
    }
    o[6] = cs[k].depth;
    o[7] = cs[k].type;
  }
  return unsup ? -1 - (int)cs.size() : (int)cs.size();
}

// collideBoxBoxAsMesh (DARTCollide.cpp:3889): MPR with ccdSupportBox on both,
// box witness sets, createMeshMeshContacts -- what the reference's
// verifyBoxMeshResultsIdenticalToAnalytical (test_DARTCollide.cpp:146)
// compares with dBoxBox.  Output rows as oracle_mesh_box.
extern "C" int oracle_box_box_as_mesh(const double* size0, const double* T0, const double* size1, const double* T1,
                                      double* out) {
  using namespace oracle;
  Obj a{}, b{};
  a.capsule = b.capsule = false;
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) { a.T.R[r * 3 + c] = T0[r * 4 + c]; b.T.R[r * 3 + c] = T1[r * 4 + c]; }
    a.T.p.x[r] = T0[r * 4 + 3];
    b.T.p.x[r] = T1[r * 4 + 3];
    a.size[r] = size0[r];
    b.size[r] = size1[r];
  }
  double depth;
  V dir, pos;
  if (mprPenetration(a, b, depth, dir, pos) != 0) return 0;
  std::vector<Contact> cs;
  if (!meshMeshContacts(dir, witnessBox(a, dir, false), witnessBox(b, dir, true), cs)) return -1;
  for (size_t k = 0; k < cs.size(); k++) {
    double* o = out + 20 * k;
    for (int i = 0; i < 3; i++) {
      o[i] = cs[k].point[i]; o[3 + i] = cs[k].normal[i];
      o[8 + i] = cs[k].edgeAFixed[i]; o[11 + i] = cs[k].edgeADir[i];
      o[14 + i] = cs[k].edgeBFixed[i]; o[17 + i] = cs[k].edgeBDir[i];
    }
    o[6] = cs[k].depth;
    o[7] = cs[k].type;
  }
  return (int)cs.size();
}
