// Mesh-box narrow phase for gfx950 (the reference atlas_bench's STL foot and
// limb colliders on its ground box), one candidate pair per WAVE: the mesh's
// vertices are scanned lane-parallel, everything else runs wave-uniform.
//
// Reference behaviour (CPU restatement and pins: oracle/oracle_capsule.cpp
// meshBox / meshMeshContacts, tests/test_mesh_collide.py):
//   collideMeshBox (DARTCollide.cpp:3935) / collideBoxMesh (:3983): libccd
//   ccdMPRPenetration with ccdSupportMesh (:1935, the FIRST vertex of largest
//   dot product) / ccdSupportBox, ccdCenterMesh (:2042); the witness sets
//   ccdPointsAtWitnessMesh (:2119) / ccdPointsAtWitnessBox (:2060);
//   createMeshMeshContacts (:2508) with createFaceFaceContacts (:2203),
//   keepOnlyConvex2DHull (:3545), math::prepareConvex2DShape / pointInPlane
//   (Geometry.cpp:3813, :3843), convex2DShapeContains (:3756),
//   get2DLineIntersection (:3790), math::getContactPoint (Geometry.cpp:1075).
//
// The vertex list is the model's candidate vertices (mesh.py: the vertices
// within the witness depth of the hull boundary -- the only ones that can be
// a support or witness point) in their original order, so first-index
// tie-breaking and the witness order are the full list's.
//
// Records (PBREC doubles): point3 normal3 depth type bodyA bodyB -3, then the
// EDGE_EDGE tail edgeAFixed3 edgeADir3 edgeBFixed3 edgeBDir3 (CREC + 0..11).
#pragma once
#include "capsule.cuh"
#include "stamp.cuh"
#include "pool_sizes.h"
#include "wave.cuh"

#define MESH_WMAX 64               // witness points per side (more: flagged unsupported)
#define MESH_MAXC MESH_PAIR_RECS   // contact records of one mesh pair
// LDS scratch of one mesh pair (doubles): the 2-D coordinates of both
// witness sets (4 W), their angle-sorted hulls (6 W), the witness sets (6 W)
#define MESH_SCRATCH (16 * MESH_WMAX)
static_assert(MESH_SCRATCH == MESH_PAIR_SCRATCH, "pool_sizes.h mesh scratch");

namespace msh {
using namespace cap;

// a mesh as a ccd object: world transform, scale, candidate vertex list
struct MeshObj {
  Xf T;
  double sc[3];
  const double* v;
  int nv;
  int lane;
};

// argmax over the wave: larger value, then lower index (the first of equals).
// Two DPP reductions (the maximum, then the lowest index among the lanes
// holding it -- each lane's index is the first of its own maxima, and lanes'
// indices differ) instead of six rounds of cross-lane shuffles, each an LDS
// permute waited on in turn.  `best` is never NaN (only d > best updates it).
DEV int imin(int a, int b) { return a < b ? a : b; }
DEV int waveMinIdx(int v) {
  v = imin(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
  v = imin(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
  v = imin(v, __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, false));  // row_ror:4
  v = imin(v, __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false));  // row_ror:8
  return imin(imin(rdli(v, 0), rdli(v, 16)), imin(rdli(v, 32), rdli(v, 48)));
}
DEV void waveArgMax(double& best, int& bi) {
  const double mx = -waveMin(-best);
  bi = waveMinIdx(best == mx ? bi : 0x7fffffff);
  best = mx;
}

// ccdSupportMesh (DARTCollide.cpp:1935).  The lane's vertices are read four
// at a time (their loads issued together, then compared in index order: the
// same first-of-equals scan), so a candidate list of a few hundred vertices
// costs one memory latency per four of the lane's vertices, not per vertex
DEV V meshSupport(const MeshObj& o, V dir) {
#pragma clang fp contract(off)
  V ld = rotT(o.T, dir);
  ld.x /= o.sc[0];
  ld.y /= o.sc[1];
  ld.z /= o.sc[2];
  double best = -__builtin_inf();
  int bi = 0x7fffffff;
  int k = o.lane;
  for (; k + 192 < o.nv; k += 256) {
    double q[4][3];
#pragma unroll
    for (int u = 0; u < 4; u++)
#pragma unroll
      for (int c = 0; c < 3; c++) q[u][c] = o.v[3 * (k + 64 * u) + c];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const double d = q[u][0] * ld.x + q[u][1] * ld.y + q[u][2] * ld.z;
      if (d > best) { best = d; bi = k + 64 * u; }
    }
  }
  for (; k < o.nv; k += 64) {
    const double* p = o.v + 3 * k;
    const double d = p[0] * ld.x + p[1] * ld.y + p[2] * ld.z;
    if (d > best) { best = d; bi = k; }
  }
  waveArgMax(best, bi);
  // no vertex beat -inf (a NaN direction from a non-finite state, or an empty
  // list): the reference keeps maxDotPoint = 0, i.e. the mesh origin
  if (bi == 0x7fffffff) return pos(o.T);
  const double* p = o.v + 3 * bi;
  return xf(o.T, mk(p[0] * o.sc[0], p[1] * o.sc[1], p[2] * o.sc[2]));
}
DEV V supportOf(const MeshObj& o, V dir) { return meshSupport(o, dir); }
DEV V centerOf(const MeshObj& o) { return pos(o.T); }

// ccdPointsAtWitnessMesh (:2119) into W (LDS, x/y/z planes of MESH_WMAX);
// returns the count, -1 on overflow
DEV int meshWitness(const MeshObj& o, V dir, bool neg, lds_double* W) {
#pragma clang fp contract(off)
  V ld = rotT(o.T, dir);
  ld.x /= o.sc[0];
  ld.y /= o.sc[1];
  ld.z /= o.sc[2];
  const double s0 = o.sc[0], s1 = o.sc[1], s2 = o.sc[2];
  double ext = neg ? __builtin_inf() : -__builtin_inf();
  for (int k = o.lane; k < o.nv; k += 64) {
    const double* p = o.v + 3 * k;
    const double d = p[0] * ld.x * s0 * s0 + p[1] * ld.y * s1 * s1 + p[2] * ld.z * s2 * s2;
    ext = neg ? fmin(ext, d) : fmax(ext, d);
  }
  ext = neg ? waveMin(ext) : -waveMin(-ext);
  int cnt = 0;
  for (int k0 = 0; k0 < o.nv; k0 += 64) {
    const int k = k0 + o.lane;
    bool cand = false;
    V pt = mk(0, 0, 0);
    if (k < o.nv) {
      const double* p = o.v + 3 * k;
      const double d = p[0] * ld.x * s0 * s0 + p[1] * ld.y * s1 * s1 + p[2] * ld.z * s2 * s2;
      cand = fabs(d - ext) < 0.01;  // DART_COLLISION_WITNESS_PLANE_DEPTH
      pt = xf(o.T, mk(p[0] * s0, p[1] * s1, p[2] * s2));
    }
    unsigned long long m = __ballot(cand);
    while (m) {
      const int j = __ffsll((long long)m) - 1;
      m &= m - 1;
      const V q = mk(rdl(pt.x, j), rdl(pt.y, j), rdl(pt.z, j));
      // duplicate of an accepted point (squared distance < 1e-6)?
      bool dup = false;
      if (o.lane < cnt) {
        const double dx = W[o.lane] - q.x, dy = W[MESH_WMAX + o.lane] - q.y, dz = W[2 * MESH_WMAX + o.lane] - q.z;
        dup = dx * dx + dy * dy + dz * dz < 1e-6;
      }
      if (__ballot(dup)) continue;
      if (cnt >= MESH_WMAX) return -1;
      if (o.lane == 0) { W[cnt] = q.x; W[MESH_WMAX + cnt] = q.y; W[2 * MESH_WMAX + cnt] = q.z; }
      cnt++;
      WSYNC();
    }
  }
  return cnt;
}

// ccdPointsAtWitnessBox (:2060): the box corners (x, y, z over {+h, -h}, in
// the reference's loop order) within the witness depth of the extreme one
DEV int boxWitness(const Obj& box, V dir, bool neg, lds_double* W, int lane) {
#pragma clang fp contract(off)
  const V ld = rotT(box.T, dir);
  const double nm = neg ? -1.0 : 1.0;
  double maxDot = -__builtin_inf();
  for (int k = 0; k < 8; k++) {
    const V l = mk((k & 4) ? box.s0 * -0.5 : box.s0 * 0.5, (k & 2) ? box.s1 * -0.5 : box.s1 * 0.5,
                   (k & 1) ? box.s2 * -0.5 : box.s2 * 0.5);
    const double d = nm * (l.x * ld.x + l.y * ld.y + l.z * ld.z);
    if (d > maxDot) maxDot = d;
  }
  int cnt = 0;
  for (int k = 0; k < 8; k++) {
    const V l = mk((k & 4) ? box.s0 * -0.5 : box.s0 * 0.5, (k & 2) ? box.s1 * -0.5 : box.s1 * 0.5,
                   (k & 1) ? box.s2 * -0.5 : box.s2 * 0.5);
    const double d = nm * (l.x * ld.x + l.y * ld.y + l.z * ld.z);
    if (maxDot - d < 0.01) {
      const V q = xf(box.T, l);
      if (lane == 0) { W[cnt] = q.x; W[MESH_WMAX + cnt] = q.y; W[2 * MESH_WMAX + cnt] = q.z; }
      cnt++;
    }
  }
  WSYNC();
  return cnt;
}

DEV V wpt(const lds_double* W, int i) { return mk(W[i], W[MESH_WMAX + i], W[2 * MESH_WMAX + i]); }

DEV void putRec(double* o, V point, V normal, double depth, int type) {
  o[0] = point.x; o[1] = point.y; o[2] = point.z;
  o[3] = normal.x; o[4] = normal.y; o[5] = normal.z;
  o[6] = depth;
  o[7] = type;
  o[10] = o[11] = o[12] = 0.0;
}

// keepOnlyConvex2DHull (:3545) over the points of `alive` (2-D coordinates
// px/py in LDS): the first non-boundary point (in order) is removed and the
// scan resumes there -- earlier points stay boundary points, as a removed
// point never carries another point's supporting line.  Returns the
// surviving mask.
DEV unsigned long long hull2D(const lds_double* px, const lds_double* py, unsigned long long alive, int lane) {
#pragma clang fp contract(off)
  // Lane j tests the line through point i and its own point j against every
  // alive point k.  The reference's scan (the first clear sign, then the
  // first opposite one ends it) keeps j exactly when no two measured points
  // (|meas| >= 1e-3) lie on opposite sides, which does not depend on the
  // order of k: so every lane runs the same k sequence to the end, reading
  // the points by readlane from registers (each lane holds its own) instead
  // of an LDS load waited on per step under a divergent early exit.
  const bool have = (alive >> lane) & 1ull;
  const double myx = have ? (double)px[lane] : 0.0, myy = have ? (double)py[lane] : 0.0;
  // Deep points, settled without the scan.  The extreme points of the set
  // in sixteen directions lie on its hull boundary, so each has a supporting
  // line through another point: the scan keeps them, whatever it removed
  // before (removals never take a supporting line's points away).  A point
  // more than 1.5e-3 inside their polygon then has, for every line through
  // it and another point, polygon vertices (alive) farther than 1e-3 on both
  // sides: the scan removes it at its turn.  Unless another point projects
  // onto it exactly (a zero-length line the reference normalises by no-op,
  // keeping the point) -- such points take the scan.  The rest take the
  // scan at their turn, against the set as the reference has it then (the
  // deep points before them already gone, those after still there).
  unsigned long long deep = 0ull;
  if (__popcll(alive) > 8) {
    // (16 directions, k pi / 8, counter-clockwise: their extreme points
    // come in the hull's counter-clockwise order)
    const double dx[16] = {1, 0.92387953251128674, 0.70710678118654757, 0.38268343236508984, 6.123233995736766e-17, -0.38268343236508973, -0.70710678118654746, -0.92387953251128674, -1, -0.92387953251128685, -0.70710678118654768, -0.38268343236509034, -1.8369701987210297e-16, 0.38268343236509, 0.70710678118654735, 0.92387953251128652};
    const double dy[16] = {0, 0.38268343236508978, 0.70710678118654746, 0.92387953251128674, 1, 0.92387953251128674, 0.70710678118654757, 0.38268343236508989, 1.2246467991473532e-16, -0.38268343236508967, -0.70710678118654746, -0.92387953251128652, -1, -0.92387953251128663, -0.70710678118654768, -0.38268343236509039};
    double ox[16], oy[16];
#pragma unroll
    for (int e = 0; e < 16; e++) {
      const double pr = have ? myx * dx[e] + myy * dy[e] : -__builtin_inf();
      const double mx = -waveMin(-pr);
      const int w = waveFirst(have && pr == mx);
      ox[e] = rdl(myx, w);
      oy[e] = rdl(myy, w);
    }
    double dmin = __builtin_inf();
    bool degen = true;
#pragma unroll
    for (int e = 0; e < 16; e++) {
      const double ex = ox[(e + 1) & 15] - ox[e], ey = oy[(e + 1) & 15] - oy[e];
      const double L = sqrt(ex * ex + ey * ey);
      if (L > 1e-9) {
        degen = false;
        const double d = ((myx - ox[e]) * -ey + (myy - oy[e]) * ex) / L;  // inside: positive (CCW)
        dmin = fmin(dmin, d);
      }
    }
    bool twin = false;
    for (unsigned long long m = alive; m; m &= m - 1) {
      const int k = __ffsll((long long)m) - 1;
      const double tx = myy - rdl(myy, k), ty = rdl(myx, k) - myx;  // the reference's line terms
      twin = twin || (k != lane && tx * tx + ty * ty == 0.0);
    }
    deep = __ballot(have && !degen && dmin > 1.5e-3 && !twin);
  }
  // Partner candidates: a boundary point's supporting line usually runs to
  // a neighbour on the set's hull, so the hull is wrapped first (gift
  // wrapping, one lane reduction per vertex) and each point names two
  // candidates -- its hull neighbours, or the ends of the hull edge nearest
  // to it.  A candidate's line is checked exactly as the reference's lane j
  // checks it (the same operations, over every alive point, one per lane);
  // only when neither candidate holds does the point take the full scan
  // below.  (The wrap only steers the search: its result never decides a
  // point.  Small sets skip it: the scan is cheaper there.)
  int candA = -1, candB = -1;
  if (__popcll(alive & ~deep) > 8) {
    const double kx = have ? myx : __builtin_inf();
    const double mnx = waveMin(kx);
    const double ky = have && myx == mnx ? myy : __builtin_inf();
    const double mny = waveMin(ky);
    const int start = waveFirst(have && myx == mnx && myy == mny);
    unsigned long long hullMask = 0ull;
    int nxtH = -1, prvH = -1;
    int c = start;
    for (int step = 0; step < 64 && c >= 0; step++) {
      hullMask |= 1ull << c;
      const double cx = rdl(myx, c), cy = rdl(myy, c);
      double qx = myx, qy = myy;
      int qi = (have && lane != c && !(myx == cx && myy == cy)) ? lane : -1;
      auto better = [&](double bx, double by, int bi) {
        if (bi < 0) return false;
        if (qi < 0) return true;
        const double cr = (qx - cx) * (by - cy) - (qy - cy) * (bx - cx);
        if (cr != 0.0) return cr < 0.0;  // b clockwise of the current winner
        const double da = (qx - cx) * (qx - cx) + (qy - cy) * (qy - cy);
        const double db = (bx - cx) * (bx - cx) + (by - cy) * (by - cy);
        return db != da ? db > da : bi < qi;
      };
      auto combine = [&](double bx, double by, int bi) {
        if (better(bx, by, bi)) { qx = bx; qy = by; qi = bi; }
      };
      combine(dppd<0xB1>(qx), dppd<0xB1>(qy), __builtin_amdgcn_update_dpp(-1, qi, 0xB1, 0xF, 0xF, false));
      combine(dppd<0x4E>(qx), dppd<0x4E>(qy), __builtin_amdgcn_update_dpp(-1, qi, 0x4E, 0xF, 0xF, false));
      combine(dppd<0x124>(qx), dppd<0x124>(qy), __builtin_amdgcn_update_dpp(-1, qi, 0x124, 0xF, 0xF, false));
      combine(dppd<0x128>(qx), dppd<0x128>(qy), __builtin_amdgcn_update_dpp(-1, qi, 0x128, 0xF, 0xF, false));
      const double rx[4] = {rdl(qx, 0), rdl(qx, 16), rdl(qx, 32), rdl(qx, 48)};
      const double ry[4] = {rdl(qy, 0), rdl(qy, 16), rdl(qy, 32), rdl(qy, 48)};
      const int ri[4] = {rdli(qi, 0), rdli(qi, 16), rdli(qi, 32), rdli(qi, 48)};
      qx = rx[0]; qy = ry[0]; qi = ri[0];
#pragma unroll
      for (int r = 1; r < 4; r++) combine(rx[r], ry[r], ri[r]);
      const int nx = uni(qi);
      if (lane == c) nxtH = nx;
      if (nx >= 0 && lane == nx) prvH = c;
      if (nx < 0 || nx == start || ((hullMask >> nx) & 1ull)) break;
      c = nx;
    }
    // (every lane runs the edge loop: its readlanes need the whole wave)
    double best = __builtin_inf();
    for (unsigned long long m = hullMask; m; m &= m - 1) {
      const int v = __ffsll((long long)m) - 1;
      const int w = rdli(nxtH, v);
      if (w < 0) continue;
      const double vx = rdl(myx, v), vy = rdl(myy, v), wx = rdl(myx, w), wy = rdl(myy, w);
      const double ex = wx - vx, ey = wy - vy;
      const double L2 = ex * ex + ey * ey;
      const double cr = (myx - vx) * ey - (myy - vy) * ex;
      const double d2 = L2 > 0.0 ? cr * cr / L2 : (myx - vx) * (myx - vx) + (myy - vy) * (myy - vy);
      if (d2 < best) { best = d2; candA = v; candB = w; }
    }
    if ((hullMask >> lane) & 1ull) {
      candA = prvH;
      candB = nxtH;
    }
  }
  unsigned long long todo = alive & ~deep;
  while (todo) {
    const int i = __ffsll((long long)todo) - 1;
    todo &= todo - 1;
    alive &= ~(deep & ((1ull << i) - 1ull));
    const double six = rdl(myx, i), siy = rdl(myy, i);
    {
      // the candidates' lines, one alive point per lane
      const bool liveK = (alive >> lane) & 1ull;
      const int cA = rdli(candA, i), cB = rdli(candB, i);
      bool found = false;
#pragma unroll
      for (int t = 0; t < 2; t++) {
        const int j = t == 0 ? cA : cB;
        if (found || j < 0 || j == i || !((alive >> j) & 1ull)) continue;
        const double sjx = rdl(myx, j), sjy = rdl(myy, j);
        double ax = siy - sjy, ay = sjx - six;
        const double nn = ax * ax + ay * ay;
        if (nn > 0) { const double q = sqrt(nn); ax /= q; ay /= q; }
        const double b = -(ax * six + ay * siy);
        const double meas = ax * myx + ay * myy + b;
        const bool counted = liveK && !(fabs(meas) < 1e-3);
        const int ks = ccdSign(meas);
        const bool anyPos = __ballot(counted && ks > 0) != 0ull, anyNeg = __ballot(counted && ks < 0) != 0ull;
        found = !(anyPos && anyNeg);
      }
      if (found) continue;  // kept
    }
    const bool mine = ((alive >> lane) & 1ull) && lane != i;
    double ax = siy - myy, ay = myx - six;
    const double nn = ax * ax + ay * ay;
    if (nn > 0) { const double q = sqrt(nn); ax /= q; ay /= q; }
    const double b = -(ax * six + ay * siy);
    bool pos = false, neg = false;
    int seen = 0;
    for (unsigned long long m = alive; m; m &= m - 1) {
      const int k = __ffsll((long long)m) - 1;
      const double meas = ax * rdl(myx, k) + ay * rdl(myy, k) + b;
      if (!(fabs(meas) < 1e-3)) {
        const int ks = ccdSign(meas);
        pos = pos || ks > 0;
        neg = neg || ks < 0;
      }
      // every partner already has points on both sides: i is not a
      // boundary point, whatever the rest of the points say
      if ((++seen & 7) == 0 && !__ballot(mine && !(pos && neg))) break;
    }
    const bool isB = mine && !(pos && neg);
    if (!__ballot(isB)) alive &= ~(1ull << i);
  }
  return alive & ~deep;
}

// prepareConvex2DShape (Geometry.cpp:3813): the points of `mask` sorted by
// atan2 around their 2-D average (ties in order); writes the sorted 3-D
// points to S and returns the count
DEV int sortByAngle(const lds_double* W, const lds_double* px, const lds_double* py, unsigned long long mask,
                    lds_double* S, int lane) {
  const int n = __popcll(mask);
  double ax = 0, ay = 0;
  for (unsigned long long m = mask; m; m &= m - 1) {
    const int k = __ffsll((long long)m) - 1;
    ax += px[k];
    ay += py[k];
  }
  ax /= (double)n;
  ay /= (double)n;
  const bool mine = (mask >> lane) & 1ull;
  const double ang = mine ? atan2(py[lane] - ay, px[lane] - ax) : 0.0;
  int rank = 0;
  for (unsigned long long m = mask; m; m &= m - 1) {
    const int k = __ffsll((long long)m) - 1;
    const double ak = rdl(ang, k);
    if (ak < ang || (ak == ang && k < lane)) rank++;
  }
  if (mine) {
    S[rank] = W[lane];
    S[MESH_WMAX + rank] = W[MESH_WMAX + lane];
    S[2 * MESH_WMAX + rank] = W[2 * MESH_WMAX + lane];
  }
  WSYNC();
  return n;
}

DEV P2 plane2(V p, V o, V bx, V by) {
#pragma clang fp contract(off)
  const V d = sub(p, o);
  P2 r;
  r.x = d.x * bx.x + d.y * bx.y + d.z * bx.z;
  r.y = d.x * by.x + d.y * by.y + d.z * by.z;
  return r;
}

// convex2DShapeContains (:3756) of point q against the sorted polygon S (n)
DEV bool containsSorted(P2 q, const lds_double* S, int n, V o, V bx, V by) {
#pragma clang fp contract(off)
  int side = 0;
  for (int i = 0; i < n; i++) {
    const int i1 = (i + 1) % n;
    const P2 a = plane2(wpt(S, i), o, bx, by), b = plane2(wpt(S, i1), o, bx, by);
    const int ts = ccdSign((q.x - a.x) * (b.y - a.y) - (q.y - a.y) * (b.x - a.x));
    if (i == 0) side = ts;
    else if (ts == 0) continue;
    else if (side == 0 && ts != 0) side = ts;
    else if (side != ts && side != 0) return false;
  }
  return true;
}

// createFaceFaceContacts (:2203) with PinToFace::AVERAGE; A / B witness sets
// in LDS (na, nb <= MESH_WMAX), scratch for 2-D coordinates and sorted hulls.
// Appends records at out[PBREC * cnt]; returns the new count, -1 on overflow.
DEV int faceFace(V dir, const lds_double* A, int na, const lds_double* B, int nb, lds_double* scr, double* out,
                 int cnt, int lane, double* g_stamp = nullptr) {
#pragma clang fp contract(off)
  (void)g_stamp;
  // (stage timing: 124 hulls, 125 angle sort, 126 containment, 127 edge pairs)
  TACC_BEGIN(tH);
  lds_double* pxA = scr;
  lds_double* pyA = scr + MESH_WMAX;
  lds_double* pxB = scr + 2 * MESH_WMAX;
  lds_double* pyB = scr + 3 * MESH_WMAX;
  lds_double* SA = scr + 4 * MESH_WMAX;
  lds_double* SB = scr + 7 * MESH_WMAX;
  auto faceNormal = [&](const lds_double* P, int np) {
    const V p0 = wpt(P, 0), p1 = wpt(P, 1);
    const V p2 = np > 2 ? wpt(P, 2) : dir;
    return eigNormalized(crs(sub(p0, p1), sub(p1, p2)));
  };
  V nA = faceNormal(A, na), nB = faceNormal(B, nb);
  auto broken = [&](V n) {
    return fabs(len2(n) - 1) > 1e-10 || fmin(len2(sub(n, dir)), len2(sub(scl(n, -1.0), dir))) > 0.2;
  };
  const bool aB = broken(nA), bB = broken(nB);
  if (aB && !bB) nA = nB;
  else if (!aB && bB) nB = nA;
  else if (aB && bB) { nA = scl(dir, -1.0); nB = nA; }
  if (nA.x * dir.x + nA.y * dir.y + nA.z * dir.z > 0) nA = scl(nA, -1.0);
  if (nB.x * dir.x + nB.y * dir.y + nB.z * dir.z > 0) nB = scl(nB, -1.0);
  const V normal = eigNormalized(scl(add(nA, nB), 0.5));
  const V a0 = wpt(A, 0), b0 = wpt(B, 0);
  const V oA = scl(normal, dot(a0, normal)), oB = scl(normal, dot(b0, normal));
  const V origin = scl(add(oA, oB), 0.5);
  V tmp = crs(normal, mk(0, 0, 1));
  if (len2(tmp) < 1e-4) tmp = crs(normal, mk(1, 0, 0));
  const V bx = crs(nA, tmp);
  const V by = crs(nA, bx);
  if (lane < na) { const P2 q = plane2(wpt(A, lane), origin, bx, by); pxA[lane] = q.x; pyA[lane] = q.y; }
  if (lane < nb) { const P2 q = plane2(wpt(B, lane), origin, bx, by); pxB[lane] = q.x; pyB[lane] = q.y; }
  WSYNC();
  const unsigned long long fullA = na >= 64 ? ~0ull : ((1ull << na) - 1ull);
  const unsigned long long fullB = nb >= 64 ? ~0ull : ((1ull << nb) - 1ull);
  const unsigned long long hA = hull2D(pxA, pyA, fullA, lane);
  const unsigned long long hB = hull2D(pxB, pyB, fullB, lane);
  TACC_END(124, tH);
  TACC_BEGIN(tS);
  const int nsA = sortByAngle(A, pxA, pyA, hA, SA, lane);
  const int nsB = sortByAngle(B, pxB, pyB, hB, SB, lane);
  TACC_END(125, tS);
  TACC_BEGIN(tI);
  // vertices of A's hull inside B's (VERTEX_FACE), in hull order
  {
    bool in = false;
    V va = mk(0, 0, 0);
    if ((hA >> lane) & 1ull) {
      va = wpt(A, lane);
      in = containsSorted(P2{pxA[lane], pyA[lane]}, SB, nsB, origin, bx, by);
    }
    const unsigned long long m = __ballot(in);
    if (cnt + __popcll(m) > MESH_MAXC) return -1;
    if (in) {
      const int r = cnt + __popcll(m & ((1ull << lane) - 1ull));
      const double distA = dot(va, nB), distB = dot(b0, nB);
      putRec(out + PBREC * r, va, nB, distB - distA, 2 /*CT_VERTEX_FACE*/);
    }
    cnt += __popcll(m);
  }
  // vertices of B's hull inside A's (FACE_VERTEX)
  {
    bool in = false;
    V vb = mk(0, 0, 0);
    if ((hB >> lane) & 1ull) {
      vb = wpt(B, lane);
      in = containsSorted(P2{pxB[lane], pyB[lane]}, SA, nsA, origin, bx, by);
    }
    const unsigned long long m = __ballot(in);
    if (cnt + __popcll(m) > MESH_MAXC) return -1;
    if (in) {
      const int r = cnt + __popcll(m & ((1ull << lane) - 1ull));
      const double distA = dot(a0, nA), distB = dot(vb, nA);
      putRec(out + PBREC * r, vb, nA, distB - distA, 1 /*CT_FACE_VERTEX*/);
    }
    cnt += __popcll(m);
  }
  TACC_END(126, tI);
  TACC_BEGIN(tE);
  // edge pairs (i over A's sorted hull, j over B's), i-major: EDGE_EDGE
  const int ea = (nsA == 2) ? 1 : nsA, eb = (nsB == 2) ? 1 : nsB;
  for (int t0 = 0; t0 < ea * eb; t0 += 64) {
    const int t = t0 + lane;
    bool hit = false;
    P2 o2;
    int i = 0, j = 0;
    if (t < ea * eb) {
      i = t / eb;
      j = t - i * eb;
      const V a1w = wpt(SA, i), a2w = wpt(SA, i == nsA - 1 ? 0 : i + 1);
      const V b1w = wpt(SB, j), b2w = wpt(SB, j == nsB - 1 ? 0 : j + 1);
      hit = lineIntersect(plane2(a1w, origin, bx, by), plane2(a2w, origin, bx, by), plane2(b1w, origin, bx, by),
                          plane2(b2w, origin, bx, by), o2);
    }
    const unsigned long long m = __ballot(hit);
    if (cnt + __popcll(m) > MESH_MAXC) return -1;
    if (hit) {
      const int r = cnt + __popcll(m & ((1ull << lane) - 1ull));
      const V a1w = wpt(SA, i), a2w = wpt(SA, i == nsA - 1 ? 0 : i + 1);
      const V b1w = wpt(SB, j), b2w = wpt(SB, j == nsB - 1 ? 0 : j + 1);
      const V aC = add(add(oA, scl(bx, o2.x)), scl(by, o2.y));
      const V bC = add(add(oB, scl(bx, o2.x)), scl(by, o2.y));
      const V aD = eigNormalized(sub(a2w, a1w)), bD = eigNormalized(sub(b2w, b1w));
      V nrm = crs(aD, bD);
      if (dot(nrm, nA) < 0) nrm = scl(nrm, -1.0);
      double depth = dot(bC, nrm) - dot(aC, nrm);
      if (depth < 0) { nrm = scl(nrm, -1.0); depth = -depth; }
      double* o = out + PBREC * r;
      putRec(o, lineContactPoint(a1w, aD, b1w, bD, 1.0, 1.0), nrm, depth, 3 /*CT_EDGE_EDGE*/);
      put3(o + CREC, a1w);
      put3(o + CREC + 3, aD);
      put3(o + CREC + 6, b1w);
      put3(o + CREC + 9, bD);
    }
    cnt += __popcll(m);
  }
  TACC_END(127, tE);
  return cnt;
}

// createMeshMeshContacts (:2508) on witness sets A (object 1) / B (object 2);
// returns the record count, -1 when unsupported (empty set / overflow)
DEV int meshMeshContacts(V dir, const lds_double* A, int na, const lds_double* B, int nb, lds_double* scr, double* out,
                         int lane, double* g_stamp = nullptr) {
#pragma clang fp contract(off)
  if (na <= 0 || nb <= 0) return -1;
  auto dirDot = [&](V n) { return n.x * dir.x + n.y * dir.y + n.z * dir.z; };
  if ((na == 1 && nb > 2) || (na > 2 && nb == 1)) {
    const bool vf = na == 1;
    const lds_double* F = vf ? B : A;
    V n = eigNormalized(crs(sub(wpt(F, 0), wpt(F, 1)), sub(wpt(F, 1), wpt(F, 2))));
    if (dirDot(n) > 0) n = scl(n, -1.0);
    const V a0 = wpt(A, 0), b0 = wpt(B, 0);
    if (lane == 0) putRec(out, vf ? a0 : b0, n, fabs(dot(a0, n) - dot(b0, n)), vf ? 2 : 1);
    return 1;
  }
  if (na == 2 && nb == 2) {
    const V ua = eigNormalized(sub(wpt(A, 0), wpt(A, 1))), ub = eigNormalized(sub(wpt(B, 0), wpt(B, 1)));
    V pa = wpt(A, 0), pb = wpt(B, 0);
    const V pp = sub(pb, pa);
    const double uaub = dot(ua, ub), q1 = dot(ua, pp), q2 = -dot(ub, pp);
    double d = 1 - uaub * uaub, alpha = 0, beta = 0;
    if (d > 0) {
      d = 1.0 / d;
      alpha = (q1 + uaub * q2) * d;
      beta = (uaub * q1 + q2) * d;
    }
    pa = add(pa, scl(ua, alpha));
    pb = add(pb, scl(ub, beta));
    V n = crs(ua, ub);
    if (dirDot(n) > 0) n = scl(n, -1.0);
    if (lane == 0) {
      putRec(out, mk(0.5 * (pa.x + pb.x), 0.5 * (pa.y + pb.y), 0.5 * (pa.z + pb.z)), n,
             fabs(dot(pb, n) - dot(pa, n)), 3);
      put3(out + CREC, wpt(A, 0));
      put3(out + CREC + 3, ua);
      put3(out + CREC + 6, wpt(B, 0));
      put3(out + CREC + 9, ub);
    }
    return 1;
  }
  if ((na == 1 && nb == 2) || (na == 2 && nb == 1)) {
    // vertex-edge (:2702) / edge-vertex (:2736, whose edge is a zero vector:
    // the normal stays dir)
    const bool ve = na == 1;
    V n = dir;
    if (ve) {
      const V e = eigNormalized(sub(wpt(B, 0), wpt(B, 1)));
      n = sub(n, scl(e, dot(n, e)));
    }
    if (dirDot(n) > 0) n = scl(n, -1.0);
    const V a0 = wpt(A, 0), b0 = wpt(B, 0);
    if (lane == 0) putRec(out, ve ? a0 : b0, n, fabs(dot(a0, n) - dot(b0, n)), ve ? 2 : 1);
    return 1;
  }
  if (na == 1 && nb == 1) {
    const V n = scl(dir, -1.0);
    const V a0 = wpt(A, 0), b0 = wpt(B, 0);
    if (lane == 0) putRec(out, b0, n, fabs(dot(b0, n) - dot(a0, n)), 1);
    return 1;
  }
  return faceFace(dir, A, na, B, nb, scr, out, 0, lane, g_stamp);
}

}  // namespace msh

// collideMeshBox (meshFirst) / collideBoxMesh, one pair per wave (all lanes
// enter).  Tm / Tb world transforms (3x4), vertex list v[nv][3], scale sc,
// box size bs.  Writes up to MESH_MAXC records (PBREC stride) to `out`
// (wave-uniform pointer); returns the count, or -1 - count when unsupported.
// `scr` is MESH_SCRATCH doubles of LDS.
// meshBoxPair is the body; deviceMeshBox its out-of-line instance.  (The
// helper wave's collision pass inlines the body: as a called function its
// prologue saved ~92 callee-saved VGPRs per lane to scratch on every call,
// ~23 KB of writes per mesh pair near contact, the bulk of the mesh Atlas
// forward's HBM writes.)
__device__ __forceinline__ int meshBoxPair(const double* Tm, const double* v, int nv, const double* sc,
                                           const double* Tb, const double* bs, bool meshFirst, double clip, int body1,
                                           int body2, double* out, lds_double* scr, int lane,
                                           double* g_stamp = nullptr) {
  using namespace cap;
  (void)g_stamp;
  TACC_BEGIN(tM);
  msh::MeshObj mo;
  Obj box;
  for (int i = 0; i < 12; i++) { mo.T.m[i] = Tm[i]; box.T.m[i] = Tb[i]; }
  mo.sc[0] = sc[0]; mo.sc[1] = sc[1]; mo.sc[2] = sc[2];
  mo.v = v;
  mo.nv = nv;
  mo.lane = lane;
  box.s0 = bs[0]; box.s1 = bs[1]; box.s2 = bs[2]; box.capsule = false;
  double depth;
  V dir, ppos;
  const int hit = meshFirst ? mpr(mo, box, depth, dir, ppos) : mpr(box, mo, depth, dir, ppos);
  // (stage timing: 120 pairs through MPR, 121 MPR, 122 witness sets, 123 contacts)
  TACC_END(121, tM);
#ifdef NIMBLE_STAGE_TIMING
  if (lane == 0 && g_stamp) g_stamp[120] += 1;
#endif
  if (hit != 0 || depth > clip) return 0;
  TACC_BEGIN(tW);
  lds_double* wa = scr + 10 * MESH_WMAX;  // witness sets past the face-face scratch
  lds_double* wb = scr + 13 * MESH_WMAX;
  const int na = meshFirst ? msh::meshWitness(mo, dir, false, wa) : msh::boxWitness(box, dir, false, wa, lane);
  const int nb = meshFirst ? msh::boxWitness(box, dir, true, wb, lane) : msh::meshWitness(mo, dir, true, wb);
  if (na < 0 || nb < 0) return -1;
  TACC_END(122, tW);
  TACC_BEGIN(tC);
  const int cnt = msh::meshMeshContacts(dir, wa, na, wb, nb, scr, out, lane, g_stamp);
  TACC_END(123, tC);
  if (cnt < 0) return -1;
  WSYNC();
  for (int c = lane; c < cnt; c += 64) { out[PBREC * c + 8] = body1; out[PBREC * c + 9] = body2; }
  WSYNC();
  return cnt;
}
__device__ __noinline__ int deviceMeshBox(const double* Tm, const double* v, int nv, const double* sc,
                                          const double* Tb, const double* bs, bool meshFirst, double clip, int body1,
                                          int body2, double* out, lds_double* scr, int lane) {
  return meshBoxPair(Tm, v, nv, sc, Tb, bs, meshFirst, clip, body1, body2, out, scr, lane);
}
