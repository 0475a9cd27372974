// Capsule-box narrow phase for gfx950 (the half-cheetah's capsule colliders
// on its ground box), one candidate pair per lane.
//
// Reference behaviour (CPU restatement and pins: oracle/oracle_capsule.cpp,
// tests/test_oracle_pins.py::test_capsule_box_known_answers):
//   libccd 2.x ccdMPRPenetration (third-party, src/mpr.c) driven by
//   dart/collision/dart/DARTCollide.cpp ccdSupportBox :1885,
//   ccdSupportCapsule :1983, setCcdDefaultSettings :3698;
//   collideBoxCapsule :4422 / collideCapsuleBox :4533 -> collideBoxSphere
//   :1482 (TOP/BOTTOM half-space clip) / collideSphereBox :1655, or the
//   pipe-face branch: ccdPointsAtWitnessBox :2060, createCapsuleMeshContact
//   :3366, createFaceFaceContacts :2203.
// createCapsuleMeshContact's vertex-pipe (:3071) and non-parallel edge-pipe
// (:3225) branches and its face branch's edge intersections (EDGE_PIPE /
// PIPE_EDGE, :3320 / :3494) are restated; an edge parallel to the pipe
// (:3118) and a zero penetration direction (8 witness points) are flagged
// (ST_UNSUPPORTED_SHAPE) and dropped, as in the oracle.
//
// Output record (CREC doubles): point3 normal3 depth type bodyA bodyB
// sphereCentre3.  Sphere contacts encode type = base (4 SPHERE_BOX, 5
// BOX_SPHERE) + 16 * (locked-face mask) + 256 * (box shape index) so the
// backward can rebuild the locked face normals from the box's world
// rotation.
#pragma once
#include "model.h"
#include "spatial.cuh"

#define CT_SPHERE_BOX 4
#define CT_BOX_SPHERE 5
#define CT_SPHERE_SPHERE 6
#define CT_SPHERE_PIPE 7
#define CT_PIPE_SPHERE 8
#define CT_PIPE_PIPE 9
#define CT_PIPE_VERTEX 10
#define CT_VERTEX_PIPE 11
#define CT_PIPE_EDGE 12
#define CT_EDGE_PIPE 13
// a capsule end against a parallel box edge (SPHERE_EDGE / EDGE_SPHERE,
// the reference's 8 / 11); geometry only, its gradients are NaN there
#define CT_SPHERE_EDGE 14
#define CT_EDGE_SPHERE 15

namespace cap {

struct V { double x, y, z; };
DEV V mk(double a, double b, double c) { V r; r.x = a; r.y = b; r.z = c; return r; }
DEV V add(V a, V b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
DEV V sub(V a, V b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
DEV V scl(V a, double s) { return mk(a.x * s, a.y * s, a.z * s); }
DEV double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
DEV V crs(V a, V b) { return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
DEV double len2(V a) { return dot(a, a); }
DEV V ccdNormalize(V a) { return scl(a, 1.0 / sqrt(len2(a))); }
DEV V eigNormalized(V a) {
  const double z = len2(a);
  if (z > 0) { const double s = sqrt(z); return mk(a.x / s, a.y / s, a.z / s); }
  return a;
}
DEV double comp(V a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
DEV void setc(V& a, int i, double v) { if (i == 0) a.x = v; else if (i == 1) a.y = v; else a.z = v; }

constexpr double kEps = 2.220446049250313e-16;  // CCD_EPS (double)
DEV bool isZero(double v) { return fabs(v) < kEps; }
DEV bool ccdEq(double a, double b) {
  const double ab = fabs(a - b);
  if (ab < kEps) return true;
  a = fabs(a);
  b = fabs(b);
  return b > a ? ab < kEps * b : ab < kEps * a;
}
DEV int ccdSign(double v) { return isZero(v) ? 0 : (v < 0 ? -1 : 1); }

// [R|p] row-major 3x4
struct Xf { double m[12]; };
DEV V rot(const Xf& T, V v) {
  return mk(T.m[0] * v.x + T.m[1] * v.y + T.m[2] * v.z, T.m[4] * v.x + T.m[5] * v.y + T.m[6] * v.z,
            T.m[8] * v.x + T.m[9] * v.y + T.m[10] * v.z);
}
DEV V rotT(const Xf& T, V v) {
  return mk(T.m[0] * v.x + T.m[4] * v.y + T.m[8] * v.z, T.m[1] * v.x + T.m[5] * v.y + T.m[9] * v.z,
            T.m[2] * v.x + T.m[6] * v.y + T.m[10] * v.z);
}
DEV V pos(const Xf& T) { return mk(T.m[3], T.m[7], T.m[11]); }
DEV V xf(const Xf& T, V v) { return add(rot(T, v), pos(T)); }
// Eigen Isometry inverse applied to v: R^T v - R^T p
DEV V xfInv(const Xf& T, V v) { return sub(rotT(T, v), rotT(T, pos(T))); }
DEV V col(const Xf& T, int c) { return mk(T.m[c], T.m[4 + c], T.m[8 + c]); }

struct Obj {
  Xf T;
  double s0, s1, s2;  // box size, or (radius, height, -)
  bool capsule;
};

DEV V support(const Obj& o, V dir) {
  V ld = rotT(o.T, dir);
  if (!o.capsule) {
    return xf(o.T, mk(ccdSign(ld.x) * o.s0 * 0.5, ccdSign(ld.y) * o.s1 * 0.5, ccdSign(ld.z) * o.s2 * 0.5));
  }
  ld = scl(eigNormalized(ld), o.s0);
  if (fabs(ld.z) < 1e-10) return xf(o.T, ld);
  if (ld.z > 0) return xf(o.T, add(ld, mk(0, 0, o.s1 / 2)));
  return xf(o.T, add(ld, mk(0, 0, -o.s1 / 2)));
}

// ccd callbacks of an object type: supportOf (ccd.support) and centerOf
// (ccd.center); the mesh collider (mesh.cuh) adds its own object type
DEV V supportOf(const Obj& o, V dir) { return support(o, dir); }
DEV V centerOf(const Obj& o) { return pos(o.T); }

struct Supp { V v, v1, v2; };
template <class OA, class OB>
DEV void ccdSupport(const OA& a, const OB& b, V dir, Supp& s) {
  s.v1 = supportOf(a, dir);
  s.v2 = supportOf(b, scl(dir, -1.0));
  s.v = sub(s.v1, s.v2);
}

DEV V portalDir(const Supp* P) { return ccdNormalize(crs(sub(P[2].v, P[1].v), sub(P[3].v, P[1].v))); }
DEV bool reachTolerance(const Supp* P, const Supp& v4, V dir) {
  const double tol = 0.0001;  // setCcdDefaultSettings: mpr_tolerance
  const double dv4 = dot(v4.v, dir);
  double d1 = dv4 - dot(P[1].v, dir), d2 = dv4 - dot(P[2].v, dir), d3 = dv4 - dot(P[3].v, dir);
  d1 = fmin(d1, d2);
  d1 = fmin(d1, d3);
  return ccdEq(d1, tol) || d1 < tol;
}
DEV void expandPortal(Supp* P, const Supp& v4) {
  const V v4v0 = crs(v4.v, P[0].v);
  if (dot(P[1].v, v4v0) > 0) {
    if (dot(P[2].v, v4v0) > 0) P[1] = v4;
    else P[3] = v4;
  } else {
    if (dot(P[3].v, v4v0) > 0) P[2] = v4;
    else P[1] = v4;
  }
}

DEV double segDist2(V P, V x0, V b, V& w) {
  const V d = sub(b, x0), a = sub(x0, P);
  double t = -1.0 * dot(a, d);
  t /= len2(d);
  if (t < 0 || isZero(t)) { w = x0; return len2(sub(x0, P)); }
  if (t > 1.0 || ccdEq(t, 1.0)) { w = b; return len2(sub(b, P)); }
  w = add(scl(d, t), x0);
  return len2(sub(w, P));
}
DEV double triDist2(V P, V x0, V B, V C, V& w) {
  const V d1 = sub(B, x0), d2 = sub(C, x0), a = sub(x0, P);
  const double v = dot(d1, d1), ww = dot(d2, d2), p = dot(a, d1), q = dot(a, d2), r = dot(d1, d2);
  const double d = ww * v - r * r;
  double s, t;
  if (isZero(d)) { s = t = -1.0; }
  else { s = (q * r - ww * p) / d; t = (-s * r - q) / ww; }
  if ((isZero(s) || s > 0) && (ccdEq(s, 1.0) || s < 1.0) && (isZero(t) || t > 0) && (ccdEq(t, 1.0) || t < 1.0) &&
      (ccdEq(t + s, 1.0) || t + s < 1.0)) {
    w = add(add(x0, scl(d1, s)), scl(d2, t));
    return len2(sub(w, P));
  }
  V w2;
  double dist = segDist2(P, x0, B, w);
  double dist2 = segDist2(P, x0, C, w2);
  if (dist2 < dist) { dist = dist2; w = w2; }
  dist2 = segDist2(P, B, C, w2);
  if (dist2 < dist) { dist = dist2; w = w2; }
  return dist;
}

DEV V findPos(const Supp* P) {
  const V dir = portalDir(P);
  double b[4];
  b[0] = dot(crs(P[1].v, P[2].v), P[3].v);
  b[1] = dot(crs(P[3].v, P[2].v), P[0].v);
  b[2] = dot(crs(P[0].v, P[1].v), P[3].v);
  b[3] = dot(crs(P[2].v, P[1].v), P[0].v);
  double sum = b[0] + b[1] + b[2] + b[3];
  if (isZero(sum) || sum < 0) {
    b[0] = 0.0;
    b[1] = dot(crs(P[2].v, P[3].v), dir);
    b[2] = dot(crs(P[3].v, P[1].v), dir);
    b[3] = dot(crs(P[1].v, P[2].v), dir);
    sum = b[1] + b[2] + b[3];
  }
  const double inv = 1.0 / sum;
  V p1 = mk(0, 0, 0), p2 = mk(0, 0, 0);
  for (int i = 0; i < 4; i++) {
    p1 = add(p1, scl(P[i].v1, b[i]));
    p2 = add(p2, scl(P[i].v2, b[i]));
  }
  return scl(add(scl(p1, inv), scl(p2, inv)), 0.5);
}

// ccdMPRPenetration: 0 intersecting (depth, dir, pos), -1 separated
template <class OA, class OB>
DEV int mpr(const OA& a, const OB& b, double& depth, V& pdir, V& ppos) {
  Supp P[4];
  P[0].v1 = centerOf(a);
  P[0].v2 = centerOf(b);
  P[0].v = sub(P[0].v1, P[0].v2);
  if (isZero(P[0].v.x) && isZero(P[0].v.y) && isZero(P[0].v.z)) P[0].v.x += kEps * 10.0;
  V dir = ccdNormalize(scl(P[0].v, -1.0));
  ccdSupport(a, b, dir, P[1]);
  double d = dot(P[1].v, dir);
  if (isZero(d) || d < 0) return -1;
  dir = crs(P[0].v, P[1].v);
  if (isZero(len2(dir))) {
    ppos = scl(add(P[1].v1, P[1].v2), 0.5);
    if (isZero(P[1].v.x) && isZero(P[1].v.y) && isZero(P[1].v.z)) {  // findPenetrTouch
      depth = 0.0;
      pdir = mk(0, 0, 0);
    } else {  // findPenetrSegment
      pdir = P[1].v;
      depth = sqrt(len2(pdir));
      pdir = ccdNormalize(pdir);
    }
    return 0;
  }
  dir = ccdNormalize(dir);
  ccdSupport(a, b, dir, P[2]);
  d = dot(P[2].v, dir);
  if (isZero(d) || d < 0) return -1;
  dir = ccdNormalize(crs(sub(P[1].v, P[0].v), sub(P[2].v, P[0].v)));
  if (dot(dir, P[0].v) > 0) {
    const Supp t = P[1];
    P[1] = P[2];
    P[2] = t;
    dir = scl(dir, -1.0);
  }
  for (;;) {  // discoverPortal: vertex 3
    ccdSupport(a, b, dir, P[3]);
    d = dot(P[3].v, dir);
    if (isZero(d) || d < 0) return -1;
    bool cont = false;
    d = dot(crs(P[1].v, P[3].v), P[0].v);
    if (d < 0 && !isZero(d)) { P[2] = P[3]; cont = true; }
    if (!cont) {
      d = dot(crs(P[3].v, P[2].v), P[0].v);
      if (d < 0 && !isZero(d)) { P[1] = P[3]; cont = true; }
    }
    if (!cont) break;
    dir = ccdNormalize(crs(sub(P[1].v, P[0].v), sub(P[2].v, P[0].v)));
  }
  Supp v4;
  for (;;) {  // refinePortal
    dir = portalDir(P);
    d = dot(dir, P[1].v);
    if (isZero(d) || d > 0) break;
    ccdSupport(a, b, dir, v4);
    d = dot(v4.v, dir);
    if (!(isZero(d) || d > 0) || reachTolerance(P, v4, dir)) return -1;
    expandPortal(P, v4);
  }
  for (unsigned long it = 0;; it++) {  // findPenetr
    dir = portalDir(P);
    ccdSupport(a, b, dir, v4);
    if (reachTolerance(P, v4, dir) || it > 10000ul) {
      V w;
      depth = sqrt(triDist2(mk(0, 0, 0), P[1].v, P[2].v, P[3].v, w));
      pdir = isZero(depth) ? mk(0, 0, 0) : ccdNormalize(w);
      ppos = findPos(P);
      return 0;
    }
    expandPortal(P, v4);
  }
}

// collideBoxSphere (boxFirst) / collideSphereBox; halfspace 0 BOTH 1 TOP 2
// BOTTOM with sphereT the capsule transform moved to the cap centre.
// Writes one record (without bodies) and returns 1, or returns 0.
DEV int sphereBox(const Obj& box, V c0, const Xf* sphereT, double r, bool boxFirst, int halfspace, double clip,
                  int boxShape, double* o) {
  const V half = mk(0.5 * box.s0, 0.5 * box.s1, 0.5 * box.s2);
  bool inside = true;
  int lock = 0;
  V p = xfInv(box.T, c0);
#pragma unroll
  for (int ax = 0; ax < 3; ax++) {
    const double h = comp(half, ax);
    if (comp(p, ax) < -h) { lock |= 1 << ax; setc(p, ax, -h); inside = false; }
    if (comp(p, ax) > h) { lock |= 1 << ax; setc(p, ax, h); inside = false; }
  }
  const double sgnIn = boxFirst ? -1.0 : 1.0;
  auto nearestFace = [&](int& idx) {
    double mn = half.x - fabs(p.x), t = half.y - fabs(p.y);
    idx = 0;
    if (t < mn) { mn = t; idx = 1; }
    t = half.z - fabs(p.z);
    if (t < mn) { mn = t; idx = 2; }
    return mn;
  };
  V n, cp;
  double pen;
  int type;
  if (inside) {
    int idx;
    const double mn = nearestFace(idx);
    V nl = mk(0, 0, 0);
    setc(nl, idx, comp(p, idx) > 0.0 ? sgnIn : -sgnIn);
    n = rot(box.T, nl);
    pen = mn + r;
    if (pen > clip) return 0;
    cp = c0;
    type = boxFirst ? 1 /*CT_FACE_VERTEX*/ : 2 /*CT_VERTEX_FACE*/;
  } else {
    cp = xf(box.T, p);
    n = boxFirst ? sub(cp, c0) : sub(c0, cp);
    const double mag = sqrt(len2(n));
    pen = r - mag;
    if (pen > clip) return 0;
    if (boxFirst && sphereT) {
      const V loc = xfInv(*sphereT, cp);
      if (halfspace == 2 && loc.z >= 0) return 0;
      if (halfspace == 1 && loc.z <= 0) return 0;
    }
    if (pen < 0.0) return 0;
    if (mag > 1e-6) {  // DART_COLLISION_EPS
      n = scl(n, 1.0 / mag);
    } else {
      int idx;
      nearestFace(idx);
      V nl = mk(0, 0, 0);
      setc(nl, idx, comp(p, idx) > 0.0 ? sgnIn : -sgnIn);
      n = rot(box.T, nl);
    }
    type = (boxFirst ? CT_BOX_SPHERE : CT_SPHERE_BOX) + 16 * lock + 256 * boxShape;
  }
  o[0] = cp.x; o[1] = cp.y; o[2] = cp.z;
  o[3] = n.x; o[4] = n.y; o[5] = n.z;
  o[6] = pen;
  o[7] = type;
  o[10] = c0.x; o[11] = c0.y; o[12] = c0.z;
  return 1;
}

struct P2 { double x, y; };
DEV P2 inPlane(V pt, V o, V bx, V by) { const V d = sub(pt, o); P2 r; r.x = dot(d, bx); r.y = dot(d, by); return r; }
DEV double cross2(double ax, double ay, double bx, double by) { return ax * by - ay * bx; }

// keepOnlyConvex2DHull for <= 4 points; returns the kept count (order kept)
DEV int keepHull(V* s, int n, V o, V bx, V by) {
  for (;;) {
    bool removed = false;
    for (int i = 0; i < n && !removed; i++) {
      bool boundary = false;
      const P2 si = inPlane(s[i], o, bx, by);
      for (int j = 0; j < n && !boundary; j++) {
        if (i == j) continue;
        const P2 sj = inPlane(s[j], o, bx, by);
        double px = si.y - sj.y, py = sj.x - si.x;
        const double nn = px * px + py * py;
        if (nn > 0) { const double q = sqrt(nn); px /= q; py /= q; }
        const double b = -(px * si.x + py * si.y);
        bool isB = true;
        int side = 0;
        for (int k = 0; k < n; k++) {
          const P2 sk = inPlane(s[k], o, bx, by);
          const double meas = px * sk.x + py * sk.y + b;
          const int ks = ccdSign(meas);
          if (fabs(meas) < 1e-3) {
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
        for (int k = i; k + 1 < n; k++) s[k] = s[k + 1];
        n--;
        removed = true;
      }
    }
    if (!removed || n == 0) break;
  }
  return n;
}
// prepareConvex2DShape: stable sort by angle around the 2-D average
DEV void sortByAngle(V* s, int n, V o, V bx, V by) {
  double ax = 0, ay = 0;
  for (int i = 0; i < n; i++) { const P2 q = inPlane(s[i], o, bx, by); ax += q.x; ay += q.y; }
  ax /= (double)n;
  ay /= (double)n;
  double ang[4];
  for (int i = 0; i < n; i++) { const P2 q = inPlane(s[i], o, bx, by); ang[i] = atan2(q.y - ay, q.x - ax); }
  for (int i = 1; i < n; i++) {  // insertion sort (stable)
    const V sv = s[i];
    const double a = ang[i];
    int j = i - 1;
    while (j >= 0 && a < ang[j]) { s[j + 1] = s[j]; ang[j + 1] = ang[j]; j--; }
    s[j + 1] = sv;
    ang[j + 1] = a;
  }
}
DEV bool contains(V pt, const V* s, int n, V o, V bx, V by) {
  const P2 q = inPlane(pt, o, bx, by);
  int side = 0;
  for (int i = 0; i < n; i++) {
    const P2 a = inPlane(s[i], o, bx, by), b = inPlane(s[(i + 1) % n], o, bx, by);
    const int ts = ccdSign(cross2(q.x - a.x, q.y - a.y, b.x - a.x, b.y - a.y));
    if (i == 0) side = ts;
    else if (ts == 0) continue;
    else if (side == 0 && ts != 0) side = ts;
    else if (side != ts && side != 0) return false;
  }
  return true;
}
// get2DLineIntersection (DARTCollide.cpp:3790), with its intersection point
// (the collinear branch's out = p + s t, as written there)
DEV bool lineIntersect(P2 p, P2 p1, P2 q, P2 q1, P2& out) {
  const double rx = p1.x - p.x, ry = p1.y - p.y, sx = q1.x - q.x, sy = q1.y - q.y;
  const double rs = cross2(rx, ry, sx, sy);
  if (rs == 0 && cross2(q.x - p.x, q.y - p.y, rx, ry) == 0) {
    const double rr = rx * rx + ry * ry;
    const double t0 = ((q.x - p.x) * rx + (q.y - p.y) * ry) / rr;
    const double t1 = ((q.x + sx - p.x) * rx + (q.y + sy - p.y) * ry) / rr;
    if (t0 >= 0 && t0 <= 1) { out = {p.x + sx * t0, p.y + sy * t0}; return true; }
    if (t1 >= 0 && t1 <= 1) { out = {p.x + sx * t1, p.y + sy * t1}; return true; }
    return false;
  } else if (rs == 0) {
    return false;
  }
  const double t = cross2(q.x - p.x, q.y - p.y, sx, sy) / rs;
  const double u = cross2(p.x - q.x, p.y - q.y, rx, ry) / cross2(sx, sy, rx, ry);
  if (t >= 0 && t <= 1 && u >= 0 && u <= 1) { out = {p.x + t * rx, p.y + t * ry}; return true; }
  return false;
}
// math::getContactPoint (Geometry.cpp:1075) via dLineClosestApproach (:1042)
DEV V lineContactPoint(V pA, V uA, V pB, V uB, double rA, double rB) {
  const V p = sub(pB, pA);
  const double uaub = dot(uA, uB), q1 = dot(uA, p), q2 = -dot(uB, p);
  double d = 1 - uaub * uaub, alpha = 0, beta = 0;
  if (d > 0) {
    d = 1.0 / d;
    alpha = (q1 + uaub * q2) * d;
    beta = (uaub * q1 + q2) * d;
  }
  return scl(add(scl(add(pA, scl(uA, alpha)), rB), scl(add(pB, scl(uB, beta)), rA)), 1.0 / (rA + rB));
}
// dSegmentsClosestApproach (DARTCollide.cpp:301): segment pa -> pb against ua -> ub
DEV void segClosest(V pa, V ua, V pb, V ub, double& alpha, double& beta) {
  const V u = sub(pb, pa), v = sub(ub, ua), w = sub(pa, ua);
  const double a = dot(u, u), b = dot(u, v), c = dot(v, v), d = dot(u, w), e = dot(v, w);
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
  alpha = fabs(sN) < 1e-15 ? 0.0 : sN / sD;
  beta = fabs(tN) < 1e-15 ? 0.0 : tN / tD;
}
// pipe-mesh contact record: point, normal, depth, type; [10..12] pipe closest
// point; tail: PIPE_VERTEX / VERTEX_PIPE pipe fixed point, pipe direction;
// PIPE_EDGE / EDGE_PIPE edge A fixed point, edge A direction, pipe fixed
// point, pipe direction (the edge's closest point is the contact point)
DEV void pipeRecord(double* out, V point, V normal, double depth, int type, V pipeClosest) {
  out[0] = point.x; out[1] = point.y; out[2] = point.z;
  out[3] = normal.x; out[4] = normal.y; out[5] = normal.z;
  out[6] = depth; out[7] = type;
  out[10] = pipeClosest.x; out[11] = pipeClosest.y; out[12] = pipeClosest.z;
}
DEV void put3(double* o, V v) { o[0] = v.x; o[1] = v.y; o[2] = v.z; }

}  // namespace cap

// A standalone sphere shape (centre c0, radius r) against a box (size bs,
// transform Tb 3x4): collideSphereBox (DARTCollide.cpp:1655) or, boxFirst,
// collideBoxSphere (:1482) with the default BOTH half-space.  One record.
__device__ __noinline__ int deviceSphereBox(const double* Tb, const double* bs, const double* c0, double r,
                                            bool boxFirst, double clip, int body1, int body2, int boxShape,
                                            double* out) {
  using namespace cap;
  Obj box;
  for (int i = 0; i < 12; i++) box.T.m[i] = Tb[i];
  box.s0 = bs[0]; box.s1 = bs[1]; box.s2 = bs[2]; box.capsule = false;
  const int cnt = sphereBox(box, mk(c0[0], c0[1], c0[2]), nullptr, r, boxFirst, 0, clip, boxShape, out);
  if (cnt) { out[8] = body1; out[9] = body2; }
  return cnt;
}

// collideSphereSphere (DARTCollide.cpp:1812): one SPHERE_SPHERE record at the
// radius-weighted point between the centres, normal from centre 1 to centre
// 0 (zero for coincident centres); centre 0 at [10..12], and after the
// record (the EDGE_REC tail) centre 1, radius 0, radius 1.
__device__ __noinline__ int deviceSphereSphere(const double* c0, double r0, const double* c1, double r1, double clip,
                                               int body1, int body2, double* out) {
  const double rsum = r0 + r1;
  double nv[3] = {c0[0] - c1[0], c0[1] - c1[1], c0[2] - c1[2]};
  double nsq = nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2];
  if (nsq > rsum * rsum) return 0;
  const double w0 = r0 / rsum, w1 = r1 / rsum;
  double depth;
  if (nsq < 1e-6) {  // DART_COLLISION_EPS
    nv[0] = nv[1] = nv[2] = 0.0;
    depth = rsum;
  } else {
    nsq = sqrt(nsq);
    for (int i = 0; i < 3; i++) nv[i] *= 1.0 / nsq;
    depth = rsum - nsq;
  }
  if (depth > clip) return 0;
  for (int i = 0; i < 3; i++) {
    out[i] = w1 * c0[i] + w0 * c1[i];
    out[3 + i] = nv[i];
    out[10 + i] = c0[i];
    out[CREC + i] = c1[i];
  }
  out[6] = depth; out[7] = CT_SPHERE_SPHERE; out[8] = body1; out[9] = body2;
  out[CREC + 3] = w0 * rsum;
  out[CREC + 4] = w1 * rsum;
  return 1;
}

// collideSphereCapsule (DARTCollide.cpp:4286) / collideCapsuleSphere (:4354,
// capsule first): sphere centre c0 (radius rs) against the capsule's axis
// segment (dDistPointToSegment :384; Tc 3x4, radius rc, height h).  One
// record: SPHERE_SPHERE on a cap (tail: centre B, radius A, radius B; centre
// A at [10..12]) or SPHERE_PIPE / PIPE_SPHERE (sphere centre at [10..12];
// tail: pipe closest point, pipe fixed point, pipe direction, sphere radius,
// pipe radius).
__device__ __noinline__ int deviceSphereCapsule(const double* c0, double rs, const double* Tc, double rc, double h,
                                                bool sphereFirst, double clip, int body1, int body2, double* out) {
  double ua[3], ub[3], v[3], d[3];
  for (int i = 0; i < 3; i++) {
    ua[i] = Tc[4 * i + 2] * (-(h / 2)) + Tc[4 * i + 3];
    ub[i] = Tc[4 * i + 2] * (h / 2) + Tc[4 * i + 3];
    v[i] = ub[i] - ua[i];
  }
  const double c1 = (c0[0] - ua[0]) * v[0] + (c0[1] - ua[1]) * v[1] + (c0[2] - ua[2]) * v[2];
  const double c2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
  double alpha;
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
  const double dist = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  const double r0 = sphereFirst ? rs : rc, r1 = sphereFirst ? rc : rs;
  if (!(dist < r0 + r1)) return 0;
  const double rsum = r0 + r1, w0 = r0 / rsum, w1 = r1 / rsum;
  const double depth = rsum - dist;
  if (depth > clip) return 0;
  double cl[3], n[3];
  for (int i = 0; i < 3; i++) cl[i] = ua[i] + v[i] * alpha;
  const double* p1 = sphereFirst ? c0 : cl;
  const double* p2 = sphereFirst ? cl : c0;
  for (int i = 0; i < 3; i++) { out[i] = p1[i] * w1 + p2[i] * w0; n[i] = p1[i] - p2[i]; }
  const double nn = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
  for (int i = 0; i < 3; i++) out[3 + i] = nn > 0 ? n[i] / nn : n[i];
  out[6] = depth; out[8] = body1; out[9] = body2;
  const double rA = w0 * rsum, rB = w1 * rsum;
  if (fabs(alpha) < 1e-8 || fabs(1 - alpha) < 1e-8) {
    out[7] = CT_SPHERE_SPHERE;
    for (int i = 0; i < 3; i++) { out[10 + i] = p1[i]; out[CREC + i] = p2[i]; }
    out[CREC + 3] = rA;
    out[CREC + 4] = rB;
  } else {
    out[7] = sphereFirst ? CT_SPHERE_PIPE : CT_PIPE_SPHERE;
    const double vn = sqrt(c2);
    for (int i = 0; i < 3; i++) {
      out[10 + i] = c0[i];
      out[CREC + i] = cl[i];
      out[CREC + 3 + i] = ua[i];
      out[CREC + 6 + i] = vn > 0 ? v[i] / vn : v[i];
    }
    out[CREC + 9] = sphereFirst ? rA : rB;   // sphere radius
    out[CREC + 10] = sphereFirst ? rB : rA;  // pipe radius
  }
  return 1;
}

// collideCapsuleCapsule (DARTCollide.cpp:4183), T0 / T1 3x4.  One record:
// SPHERE_SPHERE / SPHERE_PIPE / PIPE_SPHERE tails as deviceSphereCapsule, or
// PIPE_PIPE: [10] radius A / rsum, [11] closest-point distance, [12] radius
// B / rsum; tail: edge A fixed point, edge A dir, edge B fixed point, edge B
// dir.
__device__ __noinline__ int deviceCapsuleCapsule(const double* T0, double r0, double h0, const double* T1, double r1,
                                                 double h1, double clip, int body1, int body2, double* out) {
  double pa[3], pb[3], ua[3], ub[3];
  for (int i = 0; i < 3; i++) {
    pa[i] = T0[4 * i + 2] * (-(h0 / 2)) + T0[4 * i + 3];
    pb[i] = T0[4 * i + 2] * (h0 / 2) + T0[4 * i + 3];
    ua[i] = T1[4 * i + 2] * (-(h1 / 2)) + T1[4 * i + 3];
    ub[i] = T1[4 * i + 2] * (h1 / 2) + T1[4 * i + 3];
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
  for (int i = 0; i < 3; i++) { out[i] = point[i]; out[3 + i] = nrm[i]; }
  out[6] = depth; out[8] = body1; out[9] = body2;
  if (s0 && s1) {
    out[7] = CT_SPHERE_SPHERE;
    for (int i = 0; i < 3; i++) { out[10 + i] = c0[i]; out[CREC + i] = c1[i]; }
    out[CREC + 3] = w0 * rsum;
    out[CREC + 4] = w1 * rsum;
  } else if (s0 || s1) {
    out[7] = s0 ? CT_SPHERE_PIPE : CT_PIPE_SPHERE;
    for (int i = 0; i < 3; i++) {
      out[10 + i] = s0 ? c0[i] : c1[i];
      out[CREC + i] = s0 ? c1[i] : c0[i];
      out[CREC + 3 + i] = s0 ? ua[i] : pa[i];
      out[CREC + 6 + i] = s0 ? dirB[i] : dirA[i];
    }
    out[CREC + 9] = s0 ? w0 * rsum : w1 * rsum;
    out[CREC + 10] = s0 ? w1 * rsum : w0 * rsum;
  } else {
    out[7] = CT_PIPE_PIPE;
    out[10] = w0; out[11] = dist; out[12] = w1;
    for (int i = 0; i < 3; i++) {
      out[CREC + i] = pa[i]; out[CREC + 3 + i] = dirA[i];
      out[CREC + 6 + i] = ua[i]; out[CREC + 9 + i] = dirB[i];
    }
  }
  return 1;
}

// One capsule-box pair (box size `bs`, transforms Tb / Tc 3x4, capsule
// radius r / height h).  Writes up to 2 records at `out`; returns the count
// and sets *unsup when a branch that is not restated was taken.
__device__ __noinline__ int deviceCapsuleBox(const double* Tb, const double* bs, const double* Tc, double r, double h,
                                             bool boxFirst, double clip, int body1, int body2, int boxShape,
                                             double* out, int* unsup) {
  using namespace cap;
  Obj box, capo;
  for (int i = 0; i < 12; i++) { box.T.m[i] = Tb[i]; capo.T.m[i] = Tc[i]; }
  box.s0 = bs[0]; box.s1 = bs[1]; box.s2 = bs[2]; box.capsule = false;
  capo.s0 = r; capo.s1 = h; capo.s2 = 0; capo.capsule = true;
  double depth;
  V dir, ppos;
  const int hit = boxFirst ? mpr(box, capo, depth, dir, ppos) : mpr(capo, box, depth, dir, ppos);
  if (hit != 0 || depth > clip) return 0;
  int cnt = 0;
  const V local = xfInv(capo.T, ppos);
  if (local.z > h / 2 || local.z < -h / 2) {
    const double zc = local.z > h / 2 ? h / 2 : -h / 2;
    const V c0 = xf(capo.T, mk(0, 0, zc));
    Xf ST = capo.T;
    ST.m[3] = c0.x; ST.m[7] = c0.y; ST.m[11] = c0.z;
    cnt = sphereBox(box, c0, &ST, r, boxFirst, local.z > h / 2 ? 1 : 2, clip, boxShape, out);
  } else {
    // ccdPointsAtWitnessBox
    const V ld = rotT(box.T, dir);
    const double nm = boxFirst ? 1.0 : -1.0;
    double maxDot = -__builtin_inf();
    V W[8];
    int nw = 0;
    for (int k = 0; k < 8; k++) {
      const V l = mk((k & 4) ? box.s0 * -0.5 : box.s0 * 0.5, (k & 2) ? box.s1 * -0.5 : box.s1 * 0.5,
                     (k & 1) ? box.s2 * -0.5 : box.s2 * 0.5);
      maxDot = fmax(maxDot, nm * dot(l, ld));
    }
    for (int k = 0; k < 8; k++) {
      const V l = mk((k & 4) ? box.s0 * -0.5 : box.s0 * 0.5, (k & 2) ? box.s1 * -0.5 : box.s1 * 0.5,
                     (k & 1) ? box.s2 * -0.5 : box.s2 * 0.5);
      if (maxDot - nm * dot(l, ld) < 0.01) W[nw++] = xf(box.T, l);  // DART_COLLISION_WITNESS_PLANE_DEPTH
    }
    const V capA = xf(capo.T, mk(0, 0, h / 2)), capB = xf(capo.T, mk(0, 0, -h / 2));
    const V axis = sub(capB, capA);
    if (nw == 1) {
      // vertex-pipe (createCapsuleMeshContact :3071): dDistPointToSegment
      const double c1 = dot(sub(W[0], capA), axis), c2 = dot(axis, axis);
      const double alpha = c1 <= 0 ? 0.0 : (c2 <= c1 ? 1.0 : c1 / c2);
      const V nearest = add(capA, scl(axis, alpha));
      V nv = eigNormalized(sub(nearest, W[0]));
      if (boxFirst) nv = scl(nv, -1.0);
      const double dep = r - sqrt(len2(sub(W[0], nearest)));
      if (dep > clip) return 0;
      pipeRecord(out, W[0], nv, dep, boxFirst ? CT_VERTEX_PIPE : CT_PIPE_VERTEX, nearest);
      put3(out + CREC, capA);
      put3(out + CREC + 3, eigNormalized(axis));
      out[8] = body1; out[9] = body2;
      return 1;
    }
    if (nw == 2) {
      const V pipeDir = eigNormalized(axis), edgeDir = eigNormalized(sub(W[1], W[0]));
      if (fabs(1.0 - fabs(dot(pipeDir, edgeDir))) < 1e-5) {
        // an edge parallel to the pipe (:3122): one contact at each end of
        // the overlap -- PIPE_VERTEX at an edge end the capsule passes, else
        // SPHERE_EDGE at the capsule end (the reference leaves that
        // contact's sphereCenter NaN, Contact.cpp:59, so its gradient is NaN:
        // flagged unsupported, the contact kept)
        const double eA = dot(edgeDir, W[0]), eB = dot(edgeDir, W[1]);
        const double cA = dot(edgeDir, capA), cB = dot(edgeDir, capB);
        V nv = sub(capA, W[0]);
        nv = sub(nv, scl(edgeDir, dot(nv, edgeDir)));
        const double dep = r - sqrt(len2(nv));
        nv = eigNormalized(nv);
        if (!(dep > 0 && dep < clip)) return 0;
        const V onrm = boxFirst ? scl(nv, -1.0) : nv;
        for (int end = 0; end < 2; end++) {
          double* o = out + PBREC * end;
          const bool lowEnd = end == 0;
          const bool vertex = lowEnd ? fmin(cA, cB) < fmin(eA, eB) : fmax(cA, cB) > fmax(eA, eB);
          if (vertex) {
            const V vp = lowEnd ? (eA < eB ? W[0] : W[1]) : (eA < eB ? W[1] : W[0]);
            pipeRecord(o, vp, onrm, dep, boxFirst ? CT_VERTEX_PIPE : CT_PIPE_VERTEX, add(vp, scl(nv, r)));
            // the low end of collideCapsuleBox keeps pipeFixedPoint = capsuleB
            // and the unnormalised axis as pipeDir (:3177-:3178)
            const bool asIs = lowEnd && !boxFirst;
            put3(o + CREC, asIs ? capB : capA);
            put3(o + CREC + 3, asIs ? axis : pipeDir);
          } else {
            const V cp = lowEnd ? (cA < cB ? capA : capB) : (cA < cB ? capB : capA);
            const V pt = sub(cp, scl(nv, r));
            pipeRecord(o, pt, onrm, dep, boxFirst ? CT_EDGE_SPHERE : CT_SPHERE_EDGE, pt);
            put3(o + CREC, W[0]);
            put3(o + CREC + 3, edgeDir);
            *unsup = 1;
          }
          o[8] = body1; o[9] = body2;
        }
        return 2;
      }
      // edge-pipe (:3225)
      double alpha, beta;
      segClosest(W[0], capA, W[1], capB, alpha, beta);
      const V ec = add(W[0], scl(sub(W[1], W[0]), alpha)), pc = add(capA, scl(axis, beta));
      const V nv = eigNormalized(sub(ec, pc));
      const double dep = r - sqrt(len2(sub(ec, pc)));
      if (dep > clip) return 0;
      pipeRecord(out, ec, boxFirst ? nv : scl(nv, -1.0), dep, boxFirst ? CT_EDGE_PIPE : CT_PIPE_EDGE, pc);
      put3(out + CREC, W[0]);
      put3(out + CREC + 3, edgeDir);
      put3(out + CREC + 6, capA);
      put3(out + CREC + 9, pipeDir);
      out[8] = body1; out[9] = body2;
      return 1;
    }
    if (nw > 4) { *unsup = 1; return 0; }
    V normal = eigNormalized(crs(sub(W[0], W[1]), sub(W[1], W[2])));
    if (dot(normal, dir) > 0) normal = scl(normal, -1.0);
    // createFaceFaceContacts: A = (box face | capsule segment), B = the other
    V A[4], B[4];
    int na, nb;
    if (boxFirst) {
      for (int i = 0; i < nw; i++) A[i] = W[i];
      na = nw;
      B[0] = add(capA, scl(normal, r)); B[1] = add(capB, scl(normal, r));
      nb = 2;
    } else {
      A[0] = sub(capA, scl(normal, r)); A[1] = sub(capB, scl(normal, r));
      na = 2;
      for (int i = 0; i < nw; i++) B[i] = W[i];
      nb = nw;
    }
    const int pin = boxFirst ? 1 : 2;
    auto faceNormal = [&](const V* P, int np) {
      return eigNormalized(crs(sub(P[0], P[1]), sub(P[1], np > 2 ? P[2] : dir)));
    };
    auto broken = [&](V nv) {
      return fabs(len2(nv) - 1) > 1e-10 || fmin(len2(sub(nv, dir)), len2(sub(scl(nv, -1.0), dir))) > 0.2;
    };
    V nA = faceNormal(A, na), nB = faceNormal(B, nb);
    const bool aB = broken(nA), bB = broken(nB);
    if (aB && !bB) nA = nB;
    else if (!aB && bB) nB = nA;
    else if (aB && bB) { nA = scl(dir, -1.0); nB = nA; }
    if (dot(nA, dir) > 0) nA = scl(nA, -1.0);
    if (dot(nB, dir) > 0) nB = scl(nB, -1.0);
    V nrm = eigNormalized(scl(add(nA, nB), 0.5));
    const V oA = scl(nrm, dot(A[0], nrm)), oB = scl(nrm, dot(B[0], nrm));
    V origin = scl(add(oA, oB), 0.5);
    if (pin == 1) { origin = oA; nrm = nA; }
    else { origin = oB; nrm = nB; }
    V tmp = crs(nrm, mk(0, 0, 1));
    if (len2(tmp) < 1e-4) tmp = crs(nrm, mk(1, 0, 0));
    const V bx = crs(nA, tmp), by = crs(nA, bx);
    V Ah[4], Bh[4], As[4], Bs[4];
    for (int i = 0; i < na; i++) Ah[i] = A[i];
    for (int i = 0; i < nb; i++) Bh[i] = B[i];
    const int nah = keepHull(Ah, na, origin, bx, by);
    const int nbh = keepHull(Bh, nb, origin, bx, by);
    for (int i = 0; i < nah; i++) As[i] = Ah[i];
    for (int i = 0; i < nbh; i++) Bs[i] = Bh[i];
    sortByAngle(As, nah, origin, bx, by);
    sortByAngle(Bs, nbh, origin, bx, by);
    // vertex-in-face contacts of the capsule's segment (FACE_VERTEX of B when
    // box first, VERTEX_FACE of A otherwise) -> sphere-box at the nearer end
    const V* seg = boxFirst ? Bh : Ah;
    const int nseg = boxFirst ? nbh : nah;
    for (int i = 0; i < nseg; i++) {
      const V vtx = seg[i];
      double dep;
      V pt;
      if (boxFirst) {
        if (!contains(vtx, As, nah, origin, bx, by)) continue;
        pt = add(add(oA, scl(bx, dot(bx, vtx))), scl(by, dot(by, vtx)));
        dep = dot(vtx, nA) - dot(A[0], nA);
      } else {
        if (!contains(vtx, Bs, nbh, origin, bx, by)) continue;
        pt = add(add(oB, scl(bx, dot(bx, vtx))), scl(by, dot(by, vtx)));
        dep = dot(B[0], nB) - dot(vtx, nB);
      }
      const V sc = len2(sub(pt, capA)) < len2(sub(pt, capB)) ? capA : capB;
      if (!(dep >= 0 && dep < clip)) continue;
      cnt += sphereBox(box, sc, nullptr, r, boxFirst, 0, clip, boxShape, out + PBREC * cnt);
    }
    // then createFaceFaceContacts' edge-edge intersections (:2403), as
    // EDGE_PIPE (box first, :3320) / PIPE_EDGE (:3494) contacts
    for (int i = 0; i < nah; i++) {
      if (i == nah - 1 && nah == 2) continue;
      const V a1w = As[i], a2w = As[i == nah - 1 ? 0 : i + 1];
      const P2 a1 = inPlane(a1w, origin, bx, by), a2 = inPlane(a2w, origin, bx, by);
      for (int j = 0; j < nbh; j++) {
        if (j == nbh - 1 && nbh == 2) continue;
        const V b1w = Bs[j], b2w = Bs[j == nbh - 1 ? 0 : j + 1];
        const P2 b1 = inPlane(b1w, origin, bx, by), b2 = inPlane(b2w, origin, bx, by);
        P2 o;
        if (!lineIntersect(a1, a2, b1, b2, o) || cnt >= 8) continue;
        const V aCl = add(add(oA, scl(bx, o.x)), scl(by, o.y)), bCl = add(add(oB, scl(bx, o.x)), scl(by, o.y));
        const V aDir = eigNormalized(sub(a2w, a1w)), bDir = eigNormalized(sub(b2w, b1w));
        V cn = crs(aDir, bDir);
        if (dot(cn, nA) < 0) cn = scl(cn, -1.0);
        double dep = dot(bCl, cn) - dot(aCl, cn);
        if (dep < 0) { cn = scl(cn, -1.0); dep = -dep; }
        if (!(dep >= 0 && dep < clip)) continue;
        double* rec = out + PBREC * cnt;
        if (boxFirst) {
          // edge A = the box edge, the pipe = edge B shifted back by r
          pipeRecord(rec, aCl, cn, dep, CT_EDGE_PIPE, sub(bCl, scl(normal, r)));
          put3(rec + CREC, a1w);
          put3(rec + CREC + 3, aDir);
          put3(rec + CREC + 6, sub(b1w, scl(normal, r)));
          put3(rec + CREC + 9, bDir);
        } else {
          pipeRecord(rec, bCl, cn, dep, CT_PIPE_EDGE, add(aCl, scl(normal, r)));
          put3(rec + CREC, b1w);
          put3(rec + CREC + 3, bDir);
          put3(rec + CREC + 6, add(a1w, scl(normal, r)));
          put3(rec + CREC + 9, aDir);
        }
        cnt++;
      }
    }
  }
  for (int c = 0; c < cnt; c++) { out[PBREC * c + 8] = body1; out[PBREC * c + 9] = body2; }
  return cnt;
}
