// Device-side model constants for the batched differentiable timestep.
// Built once on the host from nimble_world_desc (include/nimble_amd.h) and read
// by every world-instance wavefront through the scalar cache (all indices into
// it are wave-uniform).
#pragma once
#include <stdint.h>

#include "../../include/nimble_amd.h"

// generalized coordinates of a joint type (-1: unknown)
inline int jointDofs(int jt) {
  switch (jt) {
    case NIMBLE_JOINT_WELD: return 0;
    case NIMBLE_JOINT_REVOLUTE: case NIMBLE_JOINT_PRISMATIC: return 1;
    case NIMBLE_JOINT_BALL: case NIMBLE_JOINT_TRANSLATIONAL: return 3;
    case NIMBLE_JOINT_FREE: return 6;
    default: return -1;
  }
}

#define NB_MAX NIMBLE_MAX_BODIES
#define ND_MAX NIMBLE_MAX_DOFS
#define NS_MAX NIMBLE_MAX_SHAPES

// LDS layout (in doubles) for one world instance; offsets computed on host.
struct Layout {
  int q, v, tau, Tw, Sw, V, A, IC, F, M, rhs, x, scratch;
  // backward extras: per-body adjoint vectors (7 x 6) and W, dof vectors
  int adj, Wt, w, gp, gv;
  // contacts: stage header/lists, post-dynamics velocity, LCP workspace pool
  int ct, v1, pool, poolCap, dinv;
  // offset (doubles) of the dynamics cache inside each world's snapshot
  int snDyn;
  // forward: narrow-phase scratch (dropped list + pair buffers), at the
  // start of the area whose far end holds the dynamics buffers V/A/IC/F, so
  // the helper wave can run the collision detection while wave 0 is still in
  // the dynamics
  int cscr;
  // forward, wide kernels only: an LDS stage (offset, capacity in doubles)
  // for the COD factorisations of off-chip LCP pools (0: none)
  int stage, stageCap;
  // forward, one-row kernel: 1 when the pool's rows slots
  // (fwdPoolRowsDoubles) lie clear of the dynamics buffers, so that the
  // helper may build the rows during the dynamics (contact.cuh EA_*); else -1
  int early;
  int total;
};

struct ModelDev {
  int nb, n, ns, maxDepth;
  int numFree;
  int freeBody[8];
  double dt, g[3], clipDepth, fallbackCfm;
  int penCorr, parallelPosVel;
  // per body
  int parent[NB_MAX], jtype[NB_MAX], dof0[NB_MAX], ndof[NB_MAX], depth[NB_MAX];
  int skel[NB_MAX], reactive[NB_MAX];
  unsigned long long anc[NB_MAX];  // bit a set <=> body a is an ancestor-or-self
  // tree structure for level-parallel sweeps: bodies grouped by depth and
  // children lists (both in ascending body order)
  int levelStart[NB_MAX + 1], levelBodies[NB_MAX];
  int childStart[NB_MAX + 1], childList[NB_MAX];
  // subtree-sum schedule: (parent, child) edges, deepest child first
  int numAcc;
  int accEdge[NB_MAX][2];
  double Tpj[NB_MAX][12];          // [R|p] row-major
  double Tcj[NB_MAX][12];
  double TcjInv[NB_MAX][12];
  double axis[NB_MAX][3];
  double mass[NB_MAX], com[NB_MAX][3], Ic[NB_MAX][9];
  double friction[NB_MAX], restitution[NB_MAX];
  // per dof
  int dofBody[ND_MAX];
  double damping[ND_MAX], spring[ND_MAX], rest[ND_MAX];
  double posLo[ND_MAX], posHi[ND_MAX], velLo[ND_MAX], velHi[ND_MAX], forceLo[ND_MAX], forceHi[ND_MAX];
  // collision shapes
  int shapeBody[NS_MAX], shapeType[NS_MAX];
  double shapeSize[NS_MAX][3];
  double shapeT[NS_MAX][12];
  // mesh shapes: their candidate vertices (mesh frame, unscaled; device
  // buffer), first / count per shape, and the bounding radius of the scaled
  // vertices about the mesh origin (pair culling)
  const double* meshVerts;
  int meshFirst[NS_MAX], meshCount[NS_MAX];
  double meshRadius[NS_MAX];
  int hasMesh;
  // issue priority (s_setprio) of the forward's helper wave while it runs
  // its share of the LCP cascade (the collision detection runs at 0)
  int helperPrio;
  // the forward's post-answer work in two shares (contact.cuh HS_POST; 0:
  // wave 0 alone, NIMBLE_AMD_POST_SPLIT=0, for tests and measurements)
  int postSplit;
  // backwardPrecompute's pinv(Q) of the wide worlds as blocked MFMA products
  // (contact.cuh pinvColumnsMfma) when the factor has full rank; 0: the
  // per-column solves (NIMBLE_AMD_PINV_MFMA=0, measurements)
  int pinvMfma;
  // the deadlock guard's test switch (contact.cuh GW_*): the waits at the
  // sites in guardSites expire at once in the worlds env with env %
  // guardStride == guardOffset (NIMBLE_AMD_GUARD_TEST="sites:stride:offset",
  // tests only; guardSites 0 in every other run)
  int guardSites, guardStride, guardOffset;
  // kept-contact capacity of the contact stage (<= NIMBLE_MAX_CONTACTS)
  int maxContacts;
  // candidate pairs (i < j) after BodyNodeCollisionFilter, in detector order
  int numPairs, pairChunk;
  int pairA[NS_MAX * (NS_MAX - 1) / 2], pairB[NS_MAX * (NS_MAX - 1) / 2];
  // the kernels' LDS layouts, [0] forward, [1] backward.  Functions that are
  // not inlined take them from here (through the scalar cache): a by-value
  // kernel argument passed to them by reference is copied into per-lane
  // scratch, ~7 KB of stores per wave
  Layout lay[2];
};

