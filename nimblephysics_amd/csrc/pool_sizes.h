// Sizes shared by the host launcher (capi.cpp) and the kernels: the contact
// stage's LDS regions, the per-world LCP workspace pools and the snapshot
// layout (doubles per world).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/nimble_amd.h"

// contact record: point3 normal3 depth type bodyA bodyB sphereCentre3
// (sphere-box types encode the locked-face mask and the box shape in `type`,
// see capsule.cuh)
#define CREC 13
// narrow-phase buffer records: the contact record + EDGE_EDGE metadata
// (edgeAFixedPoint, edgeADir, edgeBFixedPoint, edgeBDir: collision::Contact,
// set by dBoxBox), which the kept contacts carry into the snapshot
#define EDGE_REC 12
#define PBREC (CREC + EDGE_REC)

// contact-stage LDS region (Layout::ct): header, then the kept contacts
// (the model's contact capacity, ModelDev::maxContacts <= NIMBLE_MAX_CONTACTS)
#define CT_CONTACTS 32
// postProcess dedup points of the contacts the constraint filter drops
// (positions only: a later contact close to one is not kept either)
#define CT_MAX_DROPPED 64
#define DROP_REC 3
#define CT_PAIR_CHUNK 16
#define CT_PAIR_CHUNK_HOST CT_PAIR_CHUNK
// contact records one mesh pair may produce, and its LDS scratch (mesh.cuh)
// the one-row forward kernel's deferred worlds, in DEFER_BUCKETS lists by LCP
// rows (contact.cuh deferBucket) for the wide kernel's launch order
#define DEFER_BUCKETS 4
#define MESH_PAIR_RECS 64
#define MESH_PAIR_SCRATCH (16 * 64)
// the forward's header + kept contacts live in Layout::ct; the dropped list
// and the per-pair narrow-phase buffers (a mesh pair's records and scratch)
// live at the start of the alias area, clear of the dynamics buffers at its end
__host__ __device__ inline int ctDoubles(int maxContacts) { return CT_CONTACTS + maxContacts * CREC; }
__host__ __device__ inline int pairBufRecs(int pairChunk, bool mesh) {
  return mesh ? (MESH_PAIR_RECS > 8 * pairChunk ? MESH_PAIR_RECS : 8 * pairChunk) : 8 * pairChunk;
}
__host__ __device__ inline int collideScratchDoubles(int pairChunk, bool mesh) {
  return CT_MAX_DROPPED * DROP_REC + pairBufRecs(pairChunk, mesh) * PBREC + (mesh ? MESH_PAIR_SCRATCH : 0);
}

// snapshot layout
#define SN_NCON 0
#define SN_M 1
#define SN_NC 2
#define SN_NU 3
#define SN_CFM 4
#define SN_STATUS 5
#define SN_SC 6
#define SN_IGN 7
#define SN_IMP 8   // Q rank-deficient (pseudo-inverse gradient branch)
// the LCP solvers' executed work in this step (both waves): Dantzig pivots,
// PGS sweeps and their FLOPs (the roofline's frac_with_solvers)
#define SN_PIVOTS 9
#define SN_SWEEPS 10
#define SN_SOLVER_FLOPS 11
// the one-row forward kernel's deferred-world lists (contact.cuh deferEntry,
// deferCount): 2 doubles = 4 list entries per world, and in the first world
// of a launch 2 doubles = DEFER_BUCKETS counters
#define SN_DEFER 12
#define SN_DEFERCNT 14
#define SN_CONTACTS 16
#define SN_ROWS (SN_CONTACTS + NIMBLE_MAX_CONTACTS * CREC)
#define SN_ROWREC 12
#define SN_FC (SN_ROWS + NIMBLE_MAX_LCP * SN_ROWREC)
#define SN_VF (SN_FC + NIMBLE_MAX_LCP)
#define SN_MAXL NIMBLE_MAX_LCP
static_assert(SN_PIVOTS == NIMBLE_SNAPSHOT_PIVOTS && SN_SWEEPS == NIMBLE_SNAPSHOT_SWEEPS &&
                  SN_SOLVER_FLOPS == NIMBLE_SNAPSHOT_SOLVER_FLOPS && SN_DEFERCNT + 2 <= SN_CONTACTS,
              "include/nimble_amd.h snapshot offsets");
static_assert(SN_FC == NIMBLE_SNAPSHOT_FC && SN_NC == NIMBLE_SNAPSHOT_NUM_CLAMPING,
              "include/nimble_amd.h snapshot offsets");
__host__ __device__ inline int snAlign8(int x) { return ((x + 7) / 8) * 8; }
// unconstrained acceleration Minv (tau - C - D v - K ..) of the step
__host__ __device__ inline int snYf(int n) { return SN_VF + n; }
// gv-independent backward data, n x nc (leading dimension nc) / nc x nc
__host__ __device__ inline int snAc(int n) { return snAlign8(snYf(n) + n); }
__host__ __device__ inline int snAcubE(int n) { return snAc(n) + n * SN_MAXL; }
__host__ __device__ inline int snPT(int n) { return snAcubE(n) + n * SN_MAXL; }     // pinv(Q)^T
__host__ __device__ inline int snQ(int n) { return snPT(n) + SN_MAXL * SN_MAXL; }   // Q
// EDGE_EDGE metadata of the kept contacts (EDGE_REC doubles per contact slot)
__host__ __device__ inline int snEdge(int n) { return snQ(n) + SN_MAXL * SN_MAXL; }
// stage-timing builds (-DNIMBLE_STAGE_TIMING, tools/stage_timing*.py) keep
// SN_DEBUG_TAIL doubles of clock stamps at snStamps(n), ahead of the HBM
// workspace (which worlds with large LCPs use as their pool); product builds
// have none
#ifdef NIMBLE_STAGE_TIMING
#define SN_DEBUG_TAIL 128
#else
#define SN_DEBUG_TAIL 0
#endif
__host__ __device__ inline int snStamps(int n) { return snAlign8(snEdge(n) + NIMBLE_MAX_CONTACTS * EDGE_REC); }
__host__ __device__ inline int snapWorkspaceOffset(int n) { return snStamps(n) + SN_DEBUG_TAIL; }

// LCP workspace pools for m rows and n dofs
#define NV_COLS 16
// (+24: codFactor's register path stages a 24-double column in the scratch)
__host__ __device__ inline int fwdPoolDoubles(int m, int n) { return n * m + 3 * m * m + 33 * m + 2 * n + 72; }
__host__ __device__ inline int bwdPoolDoubles(int m, int n) { return n * m + 24 * m + NV_COLS * n + 64; }

// the rows' slots at the head of the forward pool (contact.cuh carveFwd: J^T,
// boxes, restitution, directions, the int vectors), which the helper's early
// rows write while wave 0 is still in the dynamics
__host__ __device__ inline int fwdPoolRowsDoubles(int m, int n) { return n * m + 10 * m; }

#define fwdPoolDoublesHost fwdPoolDoubles
#define bwdPoolDoublesHost bwdPoolDoubles
#define snapWorkspaceOffsetHost snapWorkspaceOffset

// Dynamics cache in every snapshot (forward -> backward): world transforms,
// world-frame motion subspace, body twists, the packed Cholesky factor of M,
// its reciprocal diagonal and the bias forces C.
__host__ __device__ inline int dynCacheDoubles(int n, int nb) {
  return 12 * nb + 6 * n + 6 * nb + n * (n + 1) / 2 + n + n;
}
