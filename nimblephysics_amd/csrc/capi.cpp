// C-ABI implementation (include/nimble_amd.h): model upload and kernel
// launches.  Host-side C++ calling HIP; no torch types cross this boundary.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "model.h"
#include "pool_sizes.h"

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                        \
  do {                                                                       \
    hipError_t _e = (expr);                                                  \
    if (_e != hipSuccess) return fail(NIMBLE_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

struct nimble_world {
  ModelDev host;
  ModelDev* dev = nullptr;
  Layout fwd, bwd;
  int snapDoubles = 8;
  int poolRows = 0, maxRows = 0;
  // LCPs with more rows than this run in the two-rows-per-lane kernels
  // (nimble_forward_wide_kernel / nimble_backward_wide_kernel)
  int deferRows = 64;
  // the forward's own threshold: worlds whose LCP pool does not fit the
  // one-row kernel's LDS (more rows than fwdDeferRows <= deferRows) go to
  // the big-LDS wide kernel, which takes up to 64 rows with the pool in its
  // LDS stage (the one-row code and task board) and more with two rows per
  // lane; the backward keeps deferRows
  int fwdDeferRows = 64;
  Layout fwdWide{};     // the wide forward kernel's layout (LDS stage, see nimble_world_create)
  size_t wideLds = 0;   // its LDS bytes
  int jacWsDoubles = 0;  // per-workgroup LCP workspace of the Jacobian launch
  int cacheDoubles = NIMBLE_MAX_LCP + 1;
  hipFunction_t dummy = nullptr;
  double* meshDev = nullptr;  // ModelDev::meshVerts
};

extern "C" __global__ void nimble_forward_kernel(const ModelDev*, Layout, const double*, const double*, double*,
                                                 double*, double*, int, int, int, int);
extern "C" __global__ void nimble_forward_mesh_kernel(const ModelDev*, Layout, const double*, const double*, double*,
                                                      double*, double*, int, int, int, int);
extern "C" __global__ void nimble_forward_wide_kernel(const ModelDev*, Layout, const double*, const double*, double*,
                                                      double*, double*, int, int, int);
extern "C" __global__ void nimble_backward_kernel(const ModelDev*, int, const double*, const double*,
                                                  double*, int, const double*, double*, double*, int, double*, int,
                                                  double*, int, int, int);
extern "C" __global__ void nimble_backward_wide_kernel(const ModelDev*, int, const double*, const double*,
                                                       double*, int, const double*, double*, double*, int, double*,
                                                       int, double*, int, int, int);

static void isoInverse(const double* T, double* O) {
  // [R|p]^-1 = [R^T | -R^T p]
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) O[r * 4 + c] = T[c * 4 + r];
  for (int r = 0; r < 3; r++) O[r * 4 + 3] = -(O[r * 4] * T[3] + O[r * 4 + 1] * T[7] + O[r * 4 + 2] * T[11]);
}

// LCP rows the LDS pool is sized for; worlds with more rows in a step use the
// HBM workspace at the tail of their snapshot instead (same code path).
static int ldsPoolRows(const ModelDev& m, int mcap) {
  int r = 24;
  if (const char* e = getenv("NIMBLE_AMD_LDS_ROWS")) r = atoi(e);
  if (r < 0) r = 0;
  return r < mcap ? r : mcap;
}

static Layout makeLayout(const ModelDev& m, bool backward, int poolRows) {
  Layout L{};
  L.early = -1;
  int o = 0;
  auto take = [&](int count) { int r = o; o += (count + 1) & ~1; return r; };
  const int n = m.n, nb = m.nb;
  L.q = take(n); L.v = take(n); L.tau = take(n);
  L.Tw = take(12 * nb); L.Sw = take(6 * n);
  L.M = take(n * (n + 1) / 2);  // packed lower triangle (M, then its Cholesky factor)
  L.dinv = take(n);             // 1 / L_kk
  L.rhs = take(n); L.x = take(n);
  L.v1 = take(n);
  L.ct = take(!backward && m.numPairs > 0 ? ctDoubles(m.maxContacts) : 16);
  if (backward) {
    // adjoint vectors (alpha..kappa per body); afterwards the workspace of
    // the contact-geometry terms, the M-derivative field pairs and the free
    // joint finite differences
    L.adj = take(42 * nb > 24 * 6 ? 42 * nb : 24 * 6); L.Wt = take(6 * nb);
    L.scratch = L.adj;
    L.w = take(n); L.gp = take(n); L.gv = take(n);
    L.poolCap = 0;
    if (m.numPairs > 0 && poolRows > 0) L.poolCap = bwdPoolDoublesHost(poolRows, n);
    L.pool = take(L.poolCap);
    L.V = take(6 * nb); L.A = take(6 * nb); L.F = take(6 * nb);
    L.IC = -1;  // composite inertias are not needed by the adjoint backward
  } else {
    // V, A, IC, F in one area with the contact stage (narrow-phase buffers,
    // then the LCP pool): after the dynamics they are dead and the pool
    // reuses the space.  The dynamics buffers sit at the area's far end and
    // the narrow-phase buffers at its start, so that the helper wave can run
    // the collision detection, and then build the LCP rows in the pool's
    // leading rows slots (contact.cuh EA_*), while wave 0 is still in the
    // dynamics.
    const int dyn = 54 * nb;
    L.poolCap = 0;
    int area = dyn;
    if (m.numPairs > 0) {
      const int cs = collideScratchDoubles(m.pairChunk, m.hasMesh != 0);
      if (dyn + cs > area) area = dyn + cs;
      if (poolRows > 0) {
        L.poolCap = fwdPoolDoublesHost(poolRows, n);
        if (L.poolCap > area) area = L.poolCap;
      }
    }
    area = (area + 1) & ~1;
    L.pool = o;
    L.cscr = o;
    const int dynOff = area - dyn;
    L.V = o + dynOff; L.A = L.V + 6 * nb; L.IC = L.V + 12 * nb; L.F = L.V + 48 * nb;
    // the helper's early rows: when the pool's rows slots for its largest
    // on-chip LCP end before the dynamics buffers (NIMBLE_AMD_EARLY_ROWS=0:
    // off, for measurements)
    L.early = -1;
    const char* ee = getenv("NIMBLE_AMD_EARLY_ROWS");
    if (m.numPairs > 0 && poolRows > 0 && fwdPoolRowsDoubles(poolRows, n) <= dynOff && !(ee && atoi(ee) == 0))
      L.early = 1;
    take(area);
  }
  L.total = o;
  return L;
}

extern "C" {

const char* nimble_last_error(void) { return g_err.c_str(); }

int nimble_world_create(const nimble_world_desc* d, nimble_world_t* out) {
  if (!d || !out) return fail(NIMBLE_ERR_INVALID, "null argument");
  if (d->num_bodies <= 0 || d->num_bodies > NB_MAX) return fail(NIMBLE_ERR_INVALID, "num_bodies out of range");
  if (d->num_dofs < 0 || d->num_dofs > ND_MAX || d->num_dofs > 64)
    return fail(NIMBLE_ERR_INVALID, "num_dofs out of range");
  if (d->num_shapes < 0 || d->num_shapes > NS_MAX) return fail(NIMBLE_ERR_INVALID, "num_shapes out of range");
  auto* w = new nimble_world();
  ModelDev& m = w->host;
  std::memset(&m, 0, sizeof(m));
  m.nb = d->num_bodies;
  m.n = d->num_dofs;
  m.ns = d->num_shapes;
  m.dt = d->dt;
  for (int i = 0; i < 3; i++) m.g[i] = d->gravity[i];
  m.clipDepth = d->contact_clipping_depth;
  m.fallbackCfm = d->fallback_cfm;
  m.penCorr = d->penetration_correction;
  m.parallelPosVel = d->parallel_pos_vel;
  int dofCount = 0;
  for (int b = 0; b < m.nb; b++) {
    int p = d->parent[b];
    if (p >= b) { delete w; return fail(NIMBLE_ERR_INVALID, "bodies must be in topological order"); }
    m.parent[b] = p;
    m.jtype[b] = d->joint_type[b];
    m.dof0[b] = d->dof_offset[b];
    m.ndof[b] = jointDofs(m.jtype[b]);
    if (m.ndof[b] < 0) { delete w; return fail(NIMBLE_ERR_INVALID, "unknown joint type"); }
    m.depth[b] = p >= 0 ? m.depth[p] + 1 : 0;
    if (m.depth[b] > m.maxDepth) m.maxDepth = m.depth[b];
    m.anc[b] = (p >= 0 ? m.anc[p] : 0ull) | (1ull << b);
    m.skel[b] = d->skeleton[b];
    std::memcpy(m.Tpj[b], d->T_parent_joint + 12 * b, 12 * sizeof(double));
    std::memcpy(m.Tcj[b], d->T_child_joint + 12 * b, 12 * sizeof(double));
    isoInverse(m.Tcj[b], m.TcjInv[b]);
    for (int i = 0; i < 3; i++) m.axis[b][i] = d->axis[3 * b + i];
    m.mass[b] = d->mass[b];
    for (int i = 0; i < 3; i++) m.com[b][i] = d->com[3 * b + i];
    const double* mo = d->moment + 6 * b;
    double I[9] = {mo[0], mo[3], mo[4], mo[3], mo[1], mo[5], mo[4], mo[5], mo[2]};
    std::memcpy(m.Ic[b], I, sizeof(I));
    m.friction[b] = d->friction[b];
    m.restitution[b] = d->restitution[b];
    for (int k = 0; k < m.ndof[b]; k++) m.dofBody[m.dof0[b] + k] = b;
    dofCount += m.ndof[b];
    // the joints whose posPos / velPos blocks are central differences of the
    // position integration (FreeJoint.cpp:965 / :987, BallJoint.cpp:368 / :390)
    if (m.jtype[b] == NIMBLE_JOINT_FREE || m.jtype[b] == NIMBLE_JOINT_BALL) {
      if (m.numFree >= 8) { delete w; return fail(NIMBLE_ERR_UNSUPPORTED, "more than 8 free / ball joints"); }
      m.freeBody[m.numFree++] = b;
    }
  }
  if (dofCount != m.n) { delete w; return fail(NIMBLE_ERR_INVALID, "dof count mismatch"); }
  {
    int k = 0;
    for (int lev = 0; lev <= m.maxDepth; lev++) {
      m.levelStart[lev] = k;
      for (int b = 0; b < m.nb; b++)
        if (m.depth[b] == lev) m.levelBodies[k++] = b;
    }
    m.levelStart[m.maxDepth + 1] = k;
    k = 0;
    for (int p = 0; p < m.nb; p++) {
      m.childStart[p] = k;
      for (int b = 0; b < m.nb; b++)
        if (m.parent[b] == p) m.childList[k++] = b;
    }
    m.childStart[m.nb] = k;
    // (parent, child) edges, deepest child first and children in ascending
    // order: IC[p] += IC[c] over this list is the level loop's sum, term
    // for term
    k = 0;
    for (int lev = m.maxDepth; lev >= 1; lev--)
      for (int b = 0; b < m.nb; b++)
        if (m.depth[b] == lev && m.parent[b] >= 0) { m.accEdge[k][0] = m.parent[b]; m.accEdge[k][1] = b; k++; }
    m.numAcc = k;
  }
  // BodyNode::isReactive (BodyNode.cpp:2384): mobile skeleton with dependent dofs
  for (int b = 0; b < m.nb; b++) {
    bool hasDof = false;
    for (int a = b; a >= 0; a = m.parent[a]) if (m.ndof[a] > 0) { hasDof = true; break; }
    m.reactive[b] = (d->skeleton_mobile[b] && hasDof) ? 1 : 0;
  }
  for (int i = 0; i < m.n; i++) {
    m.damping[i] = d->damping[i]; m.spring[i] = d->spring[i]; m.rest[i] = d->rest_position[i];
    m.posLo[i] = d->pos_lower[i]; m.posHi[i] = d->pos_upper[i];
    m.velLo[i] = d->vel_lower[i]; m.velHi[i] = d->vel_upper[i];
    m.forceLo[i] = d->force_lower[i]; m.forceHi[i] = d->force_upper[i];
  }
  for (int sIdx = 0; sIdx < m.ns; sIdx++) {
    m.shapeBody[sIdx] = d->shape_body[sIdx];
    m.shapeType[sIdx] = d->shape_type[sIdx];
    for (int i = 0; i < 3; i++) m.shapeSize[sIdx][i] = d->shape_size[3 * sIdx + i];
    std::memcpy(m.shapeT[sIdx], d->shape_T + 12 * sIdx, 12 * sizeof(double));
  }
  // Candidate pairs: DARTCollisionDetector::collide (DARTCollisionDetector.cpp:127)
  // object order i<j filtered by BodyNodeCollisionFilter (CollisionFilter.cpp:105)
  // NIMBLE_AMD_HELPER_PRIO (measurements): the helper's priority on the task board
  m.helperPrio = 0;
  if (const char* e = getenv("NIMBLE_AMD_HELPER_PRIO")) m.helperPrio = atoi(e) & 3;
  m.postSplit = 1;
  if (const char* e = getenv("NIMBLE_AMD_POST_SPLIT")) m.postSplit = atoi(e) != 0;
  m.pinvMfma = 1;
  if (const char* e = getenv("NIMBLE_AMD_PINV_MFMA")) m.pinvMfma = atoi(e) != 0 ? 1 : 0;
  // NIMBLE_AMD_GUARD_TEST="sites:stride:offset" (tests only): force the
  // deadlock guard to expire at the wait sites `sites` (contact.cuh GW_*
  // mask) in the worlds with index % stride == offset
  m.guardSites = 0;
  m.guardStride = 1;
  m.guardOffset = 0;
  if (const char* e = getenv("NIMBLE_AMD_GUARD_TEST")) {
    int sites = 0, stride = 1, offset = 0;
    if (sscanf(e, "%d:%d:%d", &sites, &stride, &offset) >= 1 && stride > 0 && offset >= 0 && offset < stride) {
      m.guardSites = sites;
      m.guardStride = stride;
      m.guardOffset = offset;
    }
  }
  m.numPairs = 0;
  m.pairChunk = 0;
  for (int i = 0; i < m.ns; i++)
    for (int j = i + 1; j < m.ns; j++) {
      int bi = m.shapeBody[i], bj = m.shapeBody[j];
      if (bi == bj) continue;
      int si = m.skel[bi], sj = m.skel[bj];
      if (!d->skeleton_mobile[bi] && !d->skeleton_mobile[bj]) continue;
      if (si == sj) continue;  // self-collision checking is off by default
      m.pairA[m.numPairs] = i;
      m.pairB[m.numPairs] = j;
      m.numPairs++;
    }
  m.pairChunk = m.numPairs < CT_PAIR_CHUNK_HOST ? m.numPairs : CT_PAIR_CHUNK_HOST;
  // mesh colliders: candidate vertices (all when the description has no
  // candidate mask), concatenated per shape; a mesh pair is narrow-phased by
  // the whole wave, so a model with mesh pairs takes its pairs one at a time
  {
    std::vector<double> mv;
    m.hasMesh = 0;
    for (int sIdx = 0; sIdx < m.ns; sIdx++) {
      m.meshFirst[sIdx] = 0; m.meshCount[sIdx] = 0; m.meshRadius[sIdx] = 0.0;
      if (m.shapeType[sIdx] != NIMBLE_SHAPE_MESH) continue;
      if (d->mesh_vertices == nullptr || d->shape_mesh_count == nullptr || d->shape_mesh_count[sIdx] <= 0) {
        delete w;
        return fail(NIMBLE_ERR_INVALID, "mesh shape without vertices");
      }
      const int f = d->shape_mesh_first[sIdx], c = d->shape_mesh_count[sIdx];
      if (f < 0 || f + c > d->num_mesh_vertices) { delete w; return fail(NIMBLE_ERR_INVALID, "mesh vertex range"); }
      m.meshFirst[sIdx] = (int)(mv.size() / 3);
      double r2 = 0.0;
      for (int k = 0; k < c; k++) {
        const double* v = d->mesh_vertices + 3 * (size_t)(f + k);
        double q = 0.0;
        for (int i = 0; i < 3; i++) q += (v[i] * m.shapeSize[sIdx][i]) * (v[i] * m.shapeSize[sIdx][i]);
        if (q > r2) r2 = q;
        if (d->mesh_vertex_candidate != nullptr && d->mesh_vertex_candidate[f + k] == 0) continue;
        mv.insert(mv.end(), v, v + 3);
      }
      m.meshCount[sIdx] = (int)(mv.size() / 3) - m.meshFirst[sIdx];
      m.meshRadius[sIdx] = std::sqrt(r2);
      if (m.meshCount[sIdx] <= 0) {
        delete w;
        return fail(NIMBLE_ERR_INVALID, "mesh_vertex_candidate filters out every vertex of a mesh shape");
      }
    }
    if (!mv.empty()) {
      hipError_t e = hipMalloc(&w->meshDev, mv.size() * sizeof(double));
      if (e == hipSuccess) e = hipMemcpy(w->meshDev, mv.data(), mv.size() * sizeof(double), hipMemcpyHostToDevice);
      if (e != hipSuccess) {
        if (w->meshDev) (void)hipFree(w->meshDev);
        delete w;
        return fail(NIMBLE_ERR_HIP, std::string("mesh upload: ") + hipGetErrorString(e));
      }
    }
    m.meshVerts = w->meshDev;
    for (int p = 0; p < m.numPairs; p++)
      if (m.shapeType[m.pairA[p]] == NIMBLE_SHAPE_MESH || m.shapeType[m.pairB[p]] == NIMBLE_SHAPE_MESH) m.hasMesh = 1;
    if (m.hasMesh) m.pairChunk = m.numPairs > 0 ? 1 : 0;
  }
  // max contacts: <= 8 box-box points per pair (a mesh pair: any number),
  // <= NIMBLE_MAX_CONTACTS; LCP rows: 3 per contact (> 64: the two-rows-per-
  // lane kernels)
  int maxContacts = m.hasMesh ? NIMBLE_MAX_CONTACTS : 8 * m.numPairs;
  if (maxContacts > NIMBLE_MAX_CONTACTS) maxContacts = NIMBLE_MAX_CONTACTS;
  m.maxContacts = maxContacts;
  const int mcap = 3 * maxContacts < NIMBLE_MAX_SOLVED_LCP ? 3 * maxContacts : NIMBLE_MAX_SOLVED_LCP;
  // NIMBLE_AMD_DEFER_ROWS (tests): a lower threshold sends smaller problems
  // through the two-rows-per-lane kernels as well
  if (const char* e = getenv("NIMBLE_AMD_DEFER_ROWS")) {
    const int d = atoi(e);
    if (d >= 0 && d < w->deferRows) w->deferRows = d;
  }
  int fwdRows = ldsPoolRows(m, mcap);
  for (;;) {
    w->fwd = makeLayout(m, false, fwdRows);
    if (w->fwd.total * 8 <= 160 * 1024) break;
    if (fwdRows == 0) {
      if (w->meshDev) (void)hipFree(w->meshDev);
      delete w;
      return fail(NIMBLE_ERR_UNSUPPORTED, "model too large for LDS");
    }
    fwdRows = fwdRows > 6 ? fwdRows - 6 : 0;
  }
  // The backward kernel is occupancy-bound: its pool gets the rows that keep
  // a world within a quarter of the CU's LDS (4 worlds per CU), worlds with
  // more rows use the HBM workspace; failing that, whatever fits at all.
  int bwdRows = -1;
  for (int r = fwdRows; r >= 0; r--)
    if (makeLayout(m, true, r).total * 8 <= 40 * 1024) { bwdRows = r; break; }
  if (bwdRows < 0)
    for (int r = fwdRows; r >= 0; r--)
      if (makeLayout(m, true, r).total * 8 <= 160 * 1024) { bwdRows = r; break; }
  if (bwdRows < 0) {
    if (w->meshDev) (void)hipFree(w->meshDev);
    delete w;
    return fail(NIMBLE_ERR_UNSUPPORTED, "model too large for LDS");
  }
  w->bwd = makeLayout(m, true, bwdRows);
  // the wide forward kernel's layout: the forward's, plus an LDS stage at the
  // pool (idle there: its pools are off chip) for the O(m^3) pieces of the
  // largest LCPs -- the COD factorisations, the pseudo-inverse columns (the
  // factor plus 64 right-hand sides), the Dantzig LDL^T factor -- as far as a
  // CU's 160 KB allow.  One wide world per CU then (most of the launch's
  // workgroups are not deferred worlds and exit at once); each phase checks
  // at run time whether its operands fit the stage and otherwise works in
  // HBM.  NIMBLE_AMD_WIDE_STAGE=0 turns the stage off (measurements).
  w->fwdWide = w->fwd;
  w->wideLds = (size_t)w->fwd.total * sizeof(double);
  {
    const int mc = 3 * maxContacts < NIMBLE_MAX_SOLVED_LCP ? 3 * maxContacts : NIMBLE_MAX_SOLVED_LCP;
    const int wsd = 4 * mc + (mc + 1) / 2 + 3;
    int need = mc * mc + wsd + 65 * mc + 512;                    // COD factor + workspace + pinv right-hand sides
                                                                 // (+ the MFMA pinv's 16 x 16 block matrices)
    const int needL = mc * (mc | 1) + 2 * mc;                    // Dantzig L (odd leading dimension) + scratch
    if (needL > need) need = needL;
    const int room = (int)(160 * 1024 / sizeof(double)) - w->fwd.pool;
    const char* ev = getenv("NIMBLE_AMD_WIDE_STAGE");
    const bool on = !(ev && atoi(ev) == 0);
    if (m.numPairs > 0 && mc > 64 && on && room > 0) {
      const int cap = need < room ? need : room;
      w->fwdWide.stage = w->fwd.pool;
      w->fwdWide.stageCap = cap;
      const size_t end = (size_t)(w->fwd.pool + cap) * sizeof(double);
      if (end > w->wideLds) w->wideLds = end;
    }
    // worlds of up to 64 rows whose pool fits the stage: the wide kernel
    // steps them with the pool on chip (contactStage), so the one-row kernel
    // defers every world its own pool does not hold
    w->fwdDeferRows = w->deferRows;
    if (w->fwdWide.stageCap > 0 && fwdPoolDoublesHost(64, m.n) <= w->fwdWide.stageCap && fwdRows < w->fwdDeferRows) {
      const char* ef = getenv("NIMBLE_AMD_WIDE_POOL");
      if (!(ef && atoi(ef) == 0)) w->fwdDeferRows = fwdRows;
    }
    // NIMBLE_AMD_FWD_DEFER_ROWS (tests): a lower forward threshold sends
    // smaller LCPs through the wide kernel's on-chip-pool path as well
    if (const char* e = getenv("NIMBLE_AMD_FWD_DEFER_ROWS")) {
      const int d = atoi(e);
      if (d >= 0 && d < w->fwdDeferRows && w->fwdWide.stageCap > 0) w->fwdDeferRows = d;
    }
    if (getenv("NIMBLE_AMD_VERBOSE"))
      fprintf(stderr, "nimble_amd: wide forward LDS %zu B (stage %d doubles of %d for %d rows), forward defers > %d rows\n",
              w->wideLds, w->fwdWide.stageCap, need, mc, w->fwdDeferRows);
  }
  if (getenv("NIMBLE_AMD_VERBOSE"))
    fprintf(stderr, "nimble_amd: LDS forward %d B (pool rows %d, early rows at %d), backward %d B (pool rows %d), max rows %d\n",
            w->fwd.total * 8, fwdRows, w->fwd.early, w->bwd.total * 8, bwdRows, mcap);
  const int poolRows = fwdRows < bwdRows ? fwdRows : bwdRows;
  w->poolRows = poolRows;
  w->maxRows = mcap;
  if (m.numPairs > 0) {
    int ws = 0;
    // (the two-rows-per-lane forward always works in HBM)
    if (mcap > poolRows || mcap > w->fwdDeferRows) {
      const int a = fwdPoolDoublesHost(mcap, m.n), b = bwdPoolDoublesHost(mcap, m.n);
      ws = a > b ? a : b;
    }
    w->snapDoubles = snapWorkspaceOffsetHost(m.n) + ws;
  } else {
    w->snapDoubles = 8;
  }
  // Jacobian launches run 2n items per world concurrently on one snapshot, so
  // their off-chip LCP workspace is per workgroup instead of the snapshot tail
  if (m.numPairs > 0 && bwdPoolDoublesHost(mcap, m.n) > w->bwd.poolCap) w->jacWsDoubles = bwdPoolDoublesHost(mcap, m.n);
  // dynamics cache at the tail of every snapshot
  // (the wide forward's layout copy too: it reloads the cache the one-row
  // kernel stored for a deferred world)
  w->fwd.snDyn = w->bwd.snDyn = w->fwdWide.snDyn = w->snapDoubles;
  w->snapDoubles += dynCacheDoubles(m.n, m.nb);
  m.lay[0] = w->fwd;
  m.lay[1] = w->bwd;
  hipError_t e = hipMalloc(&w->dev, sizeof(ModelDev));
  if (e != hipSuccess) {
    if (w->meshDev) (void)hipFree(w->meshDev);
    delete w;
    return fail(NIMBLE_ERR_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
  }
  e = hipMemcpy(w->dev, &m, sizeof(ModelDev), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(w->dev);
    if (w->meshDev) (void)hipFree(w->meshDev);
    delete w;
    return fail(NIMBLE_ERR_HIP, std::string("hipMemcpy: ") + hipGetErrorString(e));
  }
  *out = w;
  return NIMBLE_OK;
}

int nimble_world_destroy(nimble_world_t w) {
  if (!w) return NIMBLE_OK;
  if (w->dev) (void)hipFree(w->dev);
  if (w->meshDev) (void)hipFree(w->meshDev);
  delete w;
  return NIMBLE_OK;
}

int64_t nimble_snapshot_doubles(nimble_world_t w) { return w ? w->snapDoubles : -1; }
int64_t nimble_lcp_cache_doubles(nimble_world_t w) { return w ? w->cacheDoubles : -1; }
int32_t nimble_num_collision_pairs(nimble_world_t w) { return w ? w->host.numPairs : -1; }

// worlds per forward launch (one workgroup each); NIMBLE_AMD_FWD_CHUNK
// lowers it so tests exercise the chunked launches at small batches
static int fwdChunk() {
  int c = 1 << 22;
  if (const char* e = getenv("NIMBLE_AMD_FWD_CHUNK")) c = atoi(e);
  return c > 0 && c < (1 << 22) ? c : (1 << 22);
}

static int gridFor(int batch) {
  // one wave per world; cap the grid so every wave loops over several worlds
  // only when the batch exceeds 64k
  return batch < 65536 ? batch : 65536;
}

int nimble_forward(nimble_world_t w, int32_t batch, const double* state, const double* forces, double* lcp_cache,
                   double* next_state, double* snapshot, void* stream) {
  if (!w || batch < 0) return fail(NIMBLE_ERR_INVALID, "bad arguments");
  if (batch == 0) return NIMBLE_OK;
  if (!state || !forces || !next_state || !snapshot || !lcp_cache) return fail(NIMBLE_ERR_INVALID, "null buffer");
  hipStream_t st = (hipStream_t)stream;
  const size_t lds = (size_t)w->fwd.total * sizeof(double);
  // contact models: a second (helper) wave per world for the LCP fallback
  const int fwdThreads = w->host.numPairs > 0 ? 128 : 64;
  // one workgroup per world; batches beyond one launch's grid go in chunks
  const size_t n = (size_t)w->host.n;
  const int chunk = fwdChunk();
  const bool wide = w->host.numPairs > 0 && w->maxRows > w->fwdDeferRows;
  // the wide kernel's largest-LCP-first order (deferred-world lists; mesh
  // Atlas 217 k -> 279 k timesteps/s); NIMBLE_AMD_LARGEST_FIRST=0 dispatches
  // in world order instead (measurements)
  static const bool largestFirst = [] {
    const char* e = getenv("NIMBLE_AMD_LARGEST_FIRST");
    return !(e != nullptr && atoi(e) == 0);
  }();
  for (int32_t b0 = 0; b0 < batch; b0 += chunk) {
    const int cnt = batch - b0 < chunk ? batch - b0 : chunk;
    // the deferred-world lists live in this call's snapshot headers
    // (contact.cuh deferEntry): only their counters are reset here
    if (wide && largestFirst)
      HIP_TRY(hipMemsetAsync(snapshot + (size_t)b0 * w->snapDoubles + SN_DEFERCNT, 0, DEFER_BUCKETS * sizeof(int), st));
    // (models with mesh colliders: the instance with the mesh-box narrow
    // phase inlined on the helper)
    if (w->host.hasMesh)
      hipLaunchKernelGGL(nimble_forward_mesh_kernel, dim3(cnt), dim3(fwdThreads), lds, st, w->dev, w->fwd,
                         state + b0 * 2 * n, forces + b0 * n, lcp_cache + (size_t)b0 * w->cacheDoubles,
                         next_state + b0 * 2 * n, snapshot + (size_t)b0 * w->snapDoubles, w->snapDoubles,
                         w->cacheDoubles, w->fwdDeferRows, wide && largestFirst ? 1 : 0);
    else
      hipLaunchKernelGGL(nimble_forward_kernel, dim3(cnt), dim3(fwdThreads), lds, st, w->dev, w->fwd,
                         state + b0 * 2 * n, forces + b0 * n, lcp_cache + (size_t)b0 * w->cacheDoubles,
                         next_state + b0 * 2 * n, snapshot + (size_t)b0 * w->snapDoubles, w->snapDoubles,
                         w->cacheDoubles, w->fwdDeferRows, wide && largestFirst ? 1 : 0);
    HIP_TRY(hipGetLastError());
    // the worlds whose LCP pool the one-row kernel does not hold on chip (or
    // more rows than the test threshold): stepped by the big-LDS wide kernel
    // (two waves: the LCP task board for the worlds of up to 64 rows)
    if (wide) {
      hipLaunchKernelGGL(nimble_forward_wide_kernel, dim3(cnt), dim3(128), w->wideLds, st, w->dev, w->fwdWide,
                         state + b0 * 2 * n, forces + b0 * n, lcp_cache + (size_t)b0 * w->cacheDoubles,
                         next_state + b0 * 2 * n, snapshot + (size_t)b0 * w->snapDoubles, w->snapDoubles,
                         w->cacheDoubles, largestFirst ? 1 : 0);
      HIP_TRY(hipGetLastError());
    }
  }
  return NIMBLE_OK;
}

// the backward kernels: items of worlds with <= deferRows LCP rows, then (if
// any world can have more) the two-rows-per-lane kernel for the others
static hipError_t launchBackward(nimble_world_t w, int grid, hipStream_t st, int batch, const double* state,
                                 const double* forces, double* snapshot, const double* gradNext, double* gradState,
                                 double* gradForces, int rows, double* ws, int wsDoubles, double* gradMasses,
                                 int fcMode, int massParams) {
  const size_t lds = (size_t)w->bwd.total * sizeof(double);
  hipLaunchKernelGGL(nimble_backward_kernel, dim3(grid), dim3(64), lds, st, w->dev, batch, state, forces, snapshot,
                     w->snapDoubles, gradNext, gradState, gradForces, rows, ws, wsDoubles, gradMasses, fcMode,
                     massParams, w->deferRows);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || w->host.numPairs == 0 || w->maxRows <= w->deferRows) return e;
  hipLaunchKernelGGL(nimble_backward_wide_kernel, dim3(grid), dim3(64), lds, st, w->dev, batch, state, forces,
                     snapshot, w->snapDoubles, gradNext, gradState, gradForces, rows, ws, wsDoubles, gradMasses,
                     fcMode, massParams, w->deferRows);
  return hipGetLastError();
}

int nimble_backward(nimble_world_t w, int32_t batch, const double* state, const double* forces,
                    double* snapshot, const double* grad_next_state, double* grad_state,
                    double* grad_forces, void* stream) {
  if (!w || batch < 0) return fail(NIMBLE_ERR_INVALID, "bad arguments");
  if (batch == 0) return NIMBLE_OK;
  if (!state || !forces || !grad_next_state || !grad_state || !grad_forces || !snapshot)
    return fail(NIMBLE_ERR_INVALID, "null buffer");
  hipStream_t st = (hipStream_t)stream;
  HIP_TRY(launchBackward(w, gridFor(batch), st, batch, state, forces, snapshot, grad_next_state, grad_state,
                        grad_forces, 1, nullptr, 0, nullptr, 0, 1));
  return NIMBLE_OK;
}

int nimble_backward_masses(nimble_world_t w, int32_t batch, const double* state, const double* forces,
                           double* snapshot, const double* grad_next_state, double* grad_state,
                           double* grad_forces, double* grad_masses, void* stream) {
  if (!w || batch < 0) return fail(NIMBLE_ERR_INVALID, "bad arguments");
  if (batch == 0) return NIMBLE_OK;
  if (!state || !forces || !grad_next_state || !grad_state || !grad_forces || !snapshot || !grad_masses)
    return fail(NIMBLE_ERR_INVALID, "null buffer");
  hipStream_t st = (hipStream_t)stream;
  HIP_TRY(launchBackward(w, gridFor(batch), st, batch, state, forces, snapshot, grad_next_state, grad_state,
                        grad_forces, 1, nullptr, 0, grad_masses, 0, 1));
  return NIMBLE_OK;
}

int nimble_backward_inertia(nimble_world_t w, int32_t batch, const double* state, const double* forces,
                            double* snapshot, const double* grad_next_state, double* grad_state,
                            double* grad_forces, double* grad_inertia, void* stream) {
  if (!w || batch < 0) return fail(NIMBLE_ERR_INVALID, "bad arguments");
  if (batch == 0) return NIMBLE_OK;
  if (!state || !forces || !grad_next_state || !grad_state || !grad_forces || !snapshot || !grad_inertia)
    return fail(NIMBLE_ERR_INVALID, "null buffer");
  hipStream_t st = (hipStream_t)stream;
  HIP_TRY(launchBackward(w, gridFor(batch), st, batch, state, forces, snapshot, grad_next_state, grad_state,
                        grad_forces, 1, nullptr, 0, grad_inertia, 0, 10));
  return NIMBLE_OK;
}

// Workgroups of a Jacobian launch: enough to keep every SIMD of the chip
// busy (items loop grid-stride), bounded so the per-workgroup workspace stays
// small.
#define JAC_GRID 8192

int64_t nimble_jacobian_workspace_doubles(nimble_world_t w, int32_t batch) {
  if (!w || batch < 0) return -1;
  // enough for nimble_jacobians (2n items per world) and
  // nimble_constraint_force_jacobians (NIMBLE_MAX_LCP items per world)
  const int rows = 2 * w->host.n > NIMBLE_MAX_LCP ? 2 * w->host.n : NIMBLE_MAX_LCP;
  const long long items = (long long)batch * rows;
  const long long grid = items < JAC_GRID ? items : JAC_GRID;
  return (int64_t)(grid * w->jacWsDoubles);
}

int nimble_jacobians(nimble_world_t w, int32_t batch, const double* state, const double* forces,
                     const double* snapshot, double* state_jacobian, double* force_jacobian, double* workspace,
                     void* stream) {
  if (!w || batch < 0) return fail(NIMBLE_ERR_INVALID, "bad arguments");
  if (batch == 0 || w->host.n == 0) return NIMBLE_OK;
  if (!state || !forces || !snapshot || !state_jacobian || !force_jacobian)
    return fail(NIMBLE_ERR_INVALID, "null buffer");
  if (w->jacWsDoubles > 0 && !workspace)
    return fail(NIMBLE_ERR_INVALID, "this model needs a Jacobian workspace (nimble_jacobian_workspace_doubles)");
  const int rows = 2 * w->host.n;
  const long long items = (long long)batch * rows;
  const int grid = items < JAC_GRID ? (int)items : JAC_GRID;
  hipStream_t st = (hipStream_t)stream;
  HIP_TRY(launchBackward(w, grid, st, batch, state, forces, const_cast<double*>(snapshot), nullptr, state_jacobian,
                        force_jacobian, rows, w->jacWsDoubles > 0 ? workspace : nullptr, w->jacWsDoubles, nullptr, 0,
                        1));
  return NIMBLE_OK;
}

int nimble_constraint_force_jacobians(nimble_world_t w, int32_t batch, const double* state, const double* forces,
                                      const double* snapshot, double* dfc_dstate, double* dfc_dforces,
                                      double* workspace, void* stream) {
  if (!w || batch < 0) return fail(NIMBLE_ERR_INVALID, "bad arguments");
  if (batch == 0 || w->host.n == 0) return NIMBLE_OK;
  if (!state || !forces || !snapshot || !dfc_dstate || !dfc_dforces) return fail(NIMBLE_ERR_INVALID, "null buffer");
  if (w->jacWsDoubles > 0 && !workspace)
    return fail(NIMBLE_ERR_INVALID, "this model needs a Jacobian workspace (nimble_jacobian_workspace_doubles)");
  const int rows = NIMBLE_MAX_LCP;
  const long long items = (long long)batch * rows;
  const int grid = items < JAC_GRID ? (int)items : JAC_GRID;
  hipStream_t st = (hipStream_t)stream;
  HIP_TRY(launchBackward(w, grid, st, batch, state, forces, const_cast<double*>(snapshot), nullptr, dfc_dstate,
                        dfc_dforces, rows, w->jacWsDoubles > 0 ? workspace : nullptr, w->jacWsDoubles, nullptr, 1, 1));
  return NIMBLE_OK;
}

}  // extern "C"
