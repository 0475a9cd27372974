// Sizes shared by the host launcher (capi.cpp) and the kernels: the contact
// stage's LDS regions, the per-world LCP workspace pools and the snapshot
// layout (doubles per world).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/nimble_amd.h"

// contact record: point3 normal3 depth type bodyA bodyB
#define CREC 10

// contact-stage LDS region (Layout::ct)
#define CT_CONTACTS 32
#define CT_DROPPED (CT_CONTACTS + NIMBLE_MAX_CONTACTS * CREC)
#define CT_MAX_DROPPED 8
#define CT_PAIRBUF (CT_DROPPED + CT_MAX_DROPPED * CREC)
#define CT_PAIR_CHUNK 16
#define CT_PAIR_CHUNK_HOST CT_PAIR_CHUNK
__host__ __device__ inline int ctDoubles(int pairChunk) { return CT_PAIRBUF + pairChunk * 8 * CREC; }

// snapshot layout
#define SN_NCON 0
#define SN_M 1
#define SN_NC 2
#define SN_NU 3
#define SN_CFM 4
#define SN_STATUS 5
#define SN_SC 6
#define SN_IGN 7
#define SN_CONTACTS 16
#define SN_ROWS (SN_CONTACTS + NIMBLE_MAX_CONTACTS * CREC)
#define SN_ROWREC 12
#define SN_FC (SN_ROWS + NIMBLE_MAX_LCP * SN_ROWREC)
#define SN_VF (SN_FC + NIMBLE_MAX_LCP)
__host__ __device__ inline int snapWorkspaceOffset(int n) { return ((SN_VF + n + 7) / 8) * 8; }

// LCP workspace pools for m rows and n dofs
#define NV_COLS 16
__host__ __device__ inline int fwdPoolDoubles(int m, int n) { return 2 * n * m + 3 * m * m + 48 * m + 2 * n + 32; }
__host__ __device__ inline int bwdPoolDoubles(int m, int n) {
  return 4 * n * m + 5 * m * m + 48 * m + NV_COLS * n + 64;
}

#define fwdPoolDoublesHost fwdPoolDoubles
#define bwdPoolDoublesHost bwdPoolDoubles
#define snapWorkspaceOffsetHost snapWorkspaceOffset
