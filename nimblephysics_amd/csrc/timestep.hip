// Batched differentiable timestep for gfx950 (MI355X).
//
// One world instance per 64-lane wavefront (plus, for contact models, a
// second LCP helper wave in the forward's workgroup), all of its working set
// staged in LDS.  The reference advances one World at a time
// on the CPU (dart/simulation/World.cpp:221 World::step, with the
// articulated-body recursions of dart/dynamics/Skeleton.cpp:13034); here every
// quantity is kept in WORLD coordinates, which turns the per-body frame
// changes of the body-frame recursions into plain sums:
//   * forward kinematics / velocities / bias accelerations: one lane per body,
//     level-synchronous over tree depth;
//   * composite (subtree) inertias and forces: one lane per matrix element,
//     reverse body order;
//   * mass matrix M_jk = S_j^T I^C S_k: one lane per (j,k) pair (CRBA);
//   * M = L L^T and the solves: left-looking (Crout) Cholesky, lanes over rows;
//   * backward: one lane per input direction (q_k, v_k, tau_k), each lane
//     forming its column of dID/dq and dC/dv in closed form from the
//     world-frame composites and dotting it with Minv * dL/dv'.
#include <hip/hip_runtime.h>

#include "model.h"
#include "spatial.cuh"
#include "wave.cuh"
#include "stamp.cuh"
#include "chol_wave.cuh"

#define WAVE 64

// ---------------------------------------------------------------------------
// Forward kinematics + velocities + velocity-product (bias) accelerations.
//   Tw[b]  world transform of body b
//   Sw[k]  world-frame motion subspace column of dof k
//   V[b]   world-frame spatial velocity
//   A[b]   world-frame acceleration with ddq = `ddq` (nullptr => 0)
// Reference: BodyNode::updateTransform / updateVelocity /
// updatePartialAcceleration (dart/dynamics/BodyNode.cpp:1960-1983).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void ancestorAccelerations(const ModelDev& md, double* s, const Layout& L, int lane,
                                                      const double* ddq, double* X);
__device__ __forceinline__ void kinematics(const ModelDev& md, double* s, const Layout& L, int lane, const double* ddq,
                                           double* g_stamp = nullptr) {
  (void)g_stamp;
  STAMP(70);
  const double* q = s + L.q;
  const double* v = s + L.v;
  // 1. local transforms T_pj * Q(q) * T_cj^-1 (one lane per body), into Tw
  if (lane < md.nb) {
    const int b = lane;
    const int jt = md.jtype[b];
    const int o = md.dof0[b];
    double Q[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    const double* a = md.axis[b];
    if (jt == NIMBLE_JOINT_REVOLUTE) {
      // math::expAngular(axis * q) (Geometry.cpp:3414)
      double c = cos(q[o]), sn = sin(q[o]), t = 1.0 - c;
      Q[0] = c + t * a[0] * a[0];        Q[1] = t * a[0] * a[1] - sn * a[2]; Q[2] = t * a[0] * a[2] + sn * a[1];
      Q[4] = t * a[0] * a[1] + sn * a[2]; Q[5] = c + t * a[1] * a[1];        Q[6] = t * a[1] * a[2] - sn * a[0];
      Q[8] = t * a[0] * a[2] - sn * a[1]; Q[9] = t * a[1] * a[2] + sn * a[0]; Q[10] = c + t * a[2] * a[2];
    } else if (jt == NIMBLE_JOINT_PRISMATIC) {
      Q[3] = a[0] * q[o]; Q[7] = a[1] * q[o]; Q[11] = a[2] * q[o];
    } else if (jt == NIMBLE_JOINT_FREE || jt == NIMBLE_JOINT_BALL) {
      // FreeJoint::convertToTransform / BallJoint::convertToRotation
      // (FreeJoint.cpp:74, BallJoint.cpp:91): expMapRot of the exponential
      // coordinates (+ the translation for the free joint)
      double R[9];
      expMapRot(q + o, R);
      const bool fr = jt == NIMBLE_JOINT_FREE;
      Q[0] = R[0]; Q[1] = R[1]; Q[2] = R[2]; Q[3] = fr ? q[o + 3] : 0.0;
      Q[4] = R[3]; Q[5] = R[4]; Q[6] = R[5]; Q[7] = fr ? q[o + 4] : 0.0;
      Q[8] = R[6]; Q[9] = R[7]; Q[10] = R[8]; Q[11] = fr ? q[o + 5] : 0.0;
    } else if (jt == NIMBLE_JOINT_TRANSLATIONAL) {
      // TranslationalJoint::updateRelativeTransform (TranslationalJoint.cpp:127)
      Q[3] = q[o]; Q[7] = q[o + 1]; Q[11] = q[o + 2];
    }
    double T[12];
    tmul(md.Tpj[b], Q, T);
    tmul(T, md.TcjInv[b], s + L.Tw + 12 * b);
  }
  WSYNC();
  STAMP(71);
  // 2. compose down the tree, one level at a time
  for (int lev = 1; lev <= md.maxDepth; lev++) {
    const int b0 = md.levelStart[lev], cnt = md.levelStart[lev + 1] - b0;
    if (lane < cnt) {
      const int b = md.levelBodies[b0 + lane];
      double* Tw = s + L.Tw + 12 * b;
      tmul(s + L.Tw + 12 * md.parent[b], Tw, Tw);
    }
    WSYNC();
  }
  STAMP(72);
  // 3. world-frame motion subspace Ad_{Tw * Tcj} S_local (one lane per dof)
  if (lane < md.n) {
    const int k = lane, b = md.dofBody[k], jt = md.jtype[b];
    const double* a = md.axis[b];
    double loc[6] = {0, 0, 0, 0, 0, 0};
    if (jt == NIMBLE_JOINT_REVOLUTE) { loc[0] = a[0]; loc[1] = a[1]; loc[2] = a[2]; }
    else if (jt == NIMBLE_JOINT_PRISMATIC) { loc[3] = a[0]; loc[4] = a[1]; loc[5] = a[2]; }
    // TranslationalJoint.cpp:142: [0; e_k]; free / ball (identity Jacobian,
    // FreeJoint.cpp:536, BallJoint.cpp:446): e_k
    else if (jt == NIMBLE_JOINT_TRANSLATIONAL) loc[3 + k - md.dof0[b]] = 1.0;
    else loc[k - md.dof0[b]] = 1.0;
    double TwC[12];
    tmul(s + L.Tw + 12 * b, md.Tcj[b], TwC);
    adT(TwC, loc, s + L.Sw + 6 * k);
  }
  WSYNC();
  STAMP(73);
  // 4. V_b = sum over ancestor dofs of S_j qdot_j
  if (lane < md.nb) {
    const int b = lane;
    double V[6] = {0, 0, 0, 0, 0, 0};
    const unsigned long long an = md.anc[b];
    // unpredicated: a non-ancestor dof contributes fma(S, 0, V) = V
#pragma unroll 4
    for (int j = 0; j < md.n; j++) {
      const double vj = ((an >> md.dofBody[j]) & 1ull) ? v[j] : 0.0;
      const double* S = s + L.Sw + 6 * j;
#pragma unroll
      for (int i = 0; i < 6; i++) V[i] = fma(S[i], vj, V[i]);
    }
#pragma unroll
    for (int i = 0; i < 6; i++) s[L.V + 6 * b + i] = V[i];
  }
  WSYNC();
  STAMP(74);
  // 5. A_b = sum over ancestor dofs of S_j qddot_j + V_body(j) x (S_j qdot_j)
  //    (BodyNode::updatePartialAcceleration / updateAccelerationFD unrolled);
  //    the per-dof terms go through the (not yet used) IC region
  ancestorAccelerations(md, s, L, lane, ddq, s + L.IC);
  STAMP(75);
}

// A_b = sum over the ancestor dofs j of b of X_j, X_j = S_j qddot_j +
// V_body(j) x (S_j qdot_j): X_j is formed once per dof (lane = dof, into X,
// 6n doubles of LDS scratch), then lane b adds the X_j of every dof with a
// 0 / 1 weight (fma(1, X, A) = A + X; a non-ancestor adds nothing), the same
// sums as the per-body loop over its ancestors without divergent branches.
__device__ __forceinline__ void ancestorAccelerations(const ModelDev& md, double* s, const Layout& L, int lane,
                                                      const double* ddq, double* X) {
  const double* v = s + L.v;
  for (int j = lane; j < md.n; j += WAVE) {
    const int bj = md.dofBody[j];
    const double* S = s + L.Sw + 6 * j;
    double sv[6], cr[6];
#pragma unroll
    for (int i = 0; i < 6; i++) sv[i] = S[i] * v[j];
    crm(s + L.V + 6 * bj, sv, cr);
    const double qdd = ddq ? ddq[j] : 0.0;
#pragma unroll
    for (int i = 0; i < 6; i++) X[6 * j + i] = fma(S[i], qdd, cr[i]);
  }
  WSYNC();
  if (lane < md.nb) {
    const int b = lane;
    double A[6] = {0, 0, 0, 0, 0, 0};
    const unsigned long long an = md.anc[b];
#pragma unroll 4
    for (int j = 0; j < md.n; j++) {
      const double w = ((an >> md.dofBody[j]) & 1ull) ? 1.0 : 0.0;
#pragma unroll
      for (int i = 0; i < 6; i++) A[i] = fma(w, X[6 * j + i], A[i]);
    }
#pragma unroll
    for (int i = 0; i < 6; i++) s[L.A + 6 * b + i] = A[i];
  }
  WSYNC();
}

// World-frame spatial inertia of body b (6x6, row-major) at the world origin.
// dart/dynamics/Inertia.cpp:1368 computeSpatialTensor in world axes.
__device__ __forceinline__ void worldInertia(const ModelDev& md, const double* Tw, int b, double* I) {
  const double m = md.mass[b];
  double cw[3], Rc[9], tmp[9];
  for (int r = 0; r < 3; r++) cw[r] = Tw[r * 4] * md.com[b][0] + Tw[r * 4 + 1] * md.com[b][1] + Tw[r * 4 + 2] * md.com[b][2] + Tw[r * 4 + 3];
  // R Ic R^T
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++)
      tmp[r * 3 + c] = Tw[r * 4] * md.Ic[b][c] + Tw[r * 4 + 1] * md.Ic[b][3 + c] + Tw[r * 4 + 2] * md.Ic[b][6 + c];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++)
      Rc[r * 3 + c] = tmp[r * 3] * Tw[c * 4] + tmp[r * 3 + 1] * Tw[c * 4 + 1] + tmp[r * 3 + 2] * Tw[c * 4 + 2];
  const double C[9] = {0, -cw[2], cw[1], cw[2], 0, -cw[0], -cw[1], cw[0], 0};
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      // C C^T
      double cct = C[r * 3] * C[c * 3] + C[r * 3 + 1] * C[c * 3 + 1] + C[r * 3 + 2] * C[c * 3 + 2];
      I[r * 6 + c] = Rc[r * 3 + c] + m * cct;
      I[r * 6 + c + 3] = m * C[r * 3 + c];
      I[(r + 3) * 6 + c] = m * C[c * 3 + r];
      I[(r + 3) * 6 + c + 3] = (r == c) ? m : 0.0;
    }
}

// Composite inertias IC[b] (subtree sums) and bias forces F[b] = sum over the
// subtree of  I_i (A_i - a_g) + V_i x* (I_i V_i)  -- the world-frame
// restatement of BodyNode::updateTransmittedForceID (BodyNode.cpp:1994).
__device__ __forceinline__ void composites(const ModelDev& md, double* s, const Layout& L, int lane) {
  const double ag[6] = {0, 0, 0, md.g[0], md.g[1], md.g[2]};
  if (lane < md.nb) {
    const int b = lane;
    double* I = s + L.IC + 36 * b;
    worldInertia(md, s + L.Tw + 12 * b, b, I);
    double u[6], h[6], f[6], vxh[6];
    for (int i = 0; i < 6; i++) u[i] = s[L.A + 6 * b + i] - ag[i];
    mv6(I, u, f);
    mv6(I, s + L.V + 6 * b, h);
    crf(s + L.V + 6 * b, h, vxh);
    for (int i = 0; i < 6; i++) s[L.F + 6 * b + i] = f[i] + vxh[i];
  }
  WSYNC();
  // subtree sums: lane = one of the 42 entries (IC 36, F 6), walking the
  // model's deepest-child-first edge list (wave-uniform, scalar loads), so no
  // per-level barrier and no dependent per-lane tree-table loads
  if (lane < 42) {
    const int off = lane < 36 ? L.IC + lane : L.F + (lane - 36);
    const int stride = lane < 36 ? 36 : 6;
#pragma unroll 4
    for (int k = 0; k < md.numAcc; k++) {
      const int p = md.accEdge[k][0], c = md.accEdge[k][1];
      s[off + stride * p] += s[off + stride * c];
    }
  }
  WSYNC();
}

// M_jk = S_j^T IC_{deeper(j,k)} S_k (composite-rigid-body algorithm), and the
// generalized bias C_j = S_j . F_body(j).  M is stored full (n x n) at L.M.
__device__ __forceinline__ void massMatrixAndBias(const ModelDev& md, double* s, const Layout& L, int lane, double* C) {
  const int n = md.n;
  const int pairs = n * (n + 1) / 2;
  for (int t = lane; t < pairs; t += WAVE) {
    // unrank t -> (j >= k)
    int j = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while (j * (j + 1) / 2 > t) j--;
    while ((j + 1) * (j + 2) / 2 <= t) j++;
    const int k = t - j * (j + 1) / 2;
    const int bj = md.dofBody[j], bk = md.dofBody[k];
    int deep = -1;
    if ((md.anc[bj] >> bk) & 1ull) deep = bj;
    else if ((md.anc[bk] >> bj) & 1ull) deep = bk;
    double val = 0.0;
    if (deep >= 0) {
      double tmp[6];
      mv6(s + L.IC + 36 * deep, s + L.Sw + 6 * k, tmp);
      val = dot6(s + L.Sw + 6 * j, tmp);
    }
    s[L.M + tri(j, k)] = val;  // lower triangle, packed
  }
  for (int j = lane; j < n; j += WAVE) C[j] = dot6(s + L.Sw + 6 * j, s + L.F + 6 * md.dofBody[j]);
  WSYNC();
}

__device__ __forceinline__ void loadState(const ModelDev& md, double* s, const Layout& L, int lane, const double* state,
                          const double* tau) {
  const int n = md.n;
  for (int i = lane; i < n; i += WAVE) {
    s[L.q + i] = state[i];
    s[L.v + i] = state[n + i];
    s[L.tau + i] = tau[i];
  }
  WSYNC();
}

#include "contact.cuh"

// Dynamics cache <-> LDS (Layout regions Tw, Sw, V, M, dinv, rhs; the
// adjoint backward needs no composite inertias, so they are not stored).
__device__ __forceinline__ void dynCacheCopy(const ModelDev& md, double* s, const Layout& L, double* cache, bool store, int lane) {
  const int n = md.n, nb = md.nb;
  const int seg[6][2] = {{L.Tw, 12 * nb}, {L.Sw, 6 * n}, {L.V, 6 * nb},
                         {L.M, n * (n + 1) / 2}, {L.dinv, n}, {L.rhs, n}};
  if (store) {
    int o = 0;
    for (int k = 0; k < 6; k++) {
      const int base = seg[k][0], cnt = seg[k][1];
      if (base >= 0)  // (else: region not kept in this kernel's LDS)
        for (int t = lane; t < cnt; t += WAVE) cache[o + t] = s[base + t];
      o += cnt;
    }
  } else {
    // the load: eight elements per lane in flight (one HBM latency per 512
    // doubles instead of one per 64: the backward's load of the 1,455-double
    // Atlas cache took ~21k clocks one pass at a time), each element mapped
    // to its region by the segment ends (every region is kept on load)
    const int total = dynCacheDoubles(n, nb);
    const int e0 = 12 * nb, e1 = e0 + 6 * n, e2 = e1 + 6 * nb, e3 = e2 + n * (n + 1) / 2, e4 = e3 + n;
    for (int t0 = lane; t0 < total; t0 += 8 * WAVE) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int t = t0 + u * WAVE;
        v[u] = t < total ? cache[t] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int t = t0 + u * WAVE;
        if (t < total) {
          const int base = t < e0 ? L.Tw : t < e1 ? L.Sw - e0 : t < e2 ? L.V - e1 : t < e3 ? L.M - e2
                         : t < e4 ? L.dinv - e3 : L.rhs - e4;
          s[base + t] = v[u];
        }
      }
    }
  }
  WSYNC();
}

// Accelerations only (phase 5 of kinematics) for given ddq, with Tw, Sw, V
// already in LDS.
// (X: 6n doubles of LDS scratch)
__device__ __forceinline__ void accelerations(const ModelDev& md, double* s, const Layout& L, int lane, const double* ddq,
                                              double* X) {
  ancestorAccelerations(md, s, L, lane, ddq, X);
}

// Everything up to the factored mass matrix; leaves C in s[L.rhs].
__device__ __forceinline__ void coreDynamics(const ModelDev& md, double* s, const Layout& L, int lane) {
  kinematics(md, s, L, lane, nullptr);
  composites(md, s, L, lane);
  massMatrixAndBias(md, s, L, lane, s + L.rhs);
  cholesky(s + L.M, s + L.dinv, md.n, lane);
}

// ---------------------------------------------------------------------------
// Forward step.
// ---------------------------------------------------------------------------
// Two waves per world when the model has contact pairs (blockDim 128): wave
// 1 is the LCP helper (helperWave), all of the step runs on wave 0.  One
// world per workgroup and no world loop (the host splits batches larger than
// one launch): a loop lets the compiler hoist ~120 per-lane model / LDS
// addresses out of it, which stay live across the whole step and spilled
// ~150 VGPRs (~44 KB of scratch writes per world).
//
// R row slots per lane in the contact LCP (contactStage): the R = 1 kernel
// leaves a world whose LCP has more than `deferRows` rows (> 64: more than
// 21 frictional contacts) to the R = 2 kernel launched after it, which
// steps only those worlds, from the same inputs.
template <int R, bool kMesh = false>
__device__ __forceinline__ void forwardWorld(const ModelDev* __restrict__ mdp, const Layout& L,
                                             const double* __restrict__ state, const double* __restrict__ forces,
                                             double* __restrict__ lcpCache, double* __restrict__ nextState,
                                             double* __restrict__ snapshot, int snapDoubles, int cacheDoubles,
                                             int deferRows, int env, bool deferLists) {
  extern __shared__ double s[];
  const ModelDev& md = *mdp;
  const int lane = threadIdx.x & (WAVE - 1);
  const int n = md.n;
  const bool helperOn = blockDim.x > WAVE;
  if (helperOn) {
    if (threadIdx.x == 0) {
      int* hf = reinterpret_cast<int*>(s + L.ct + H_HELPER);
      // hf[2]: the deadlock guard's forced-expiry sites for this world (the
      // tests' NIMBLE_AMD_GUARD_TEST; 0 otherwise)
      const int gs = md.guardSites;
      hf[0] = HS_IDLE; hf[1] = 0; hf[3] = 0;
      hf[2] = (gs != 0 && (R == 1 || !(gs & GW_ONE_ROW_ONLY)) && env % md.guardStride == md.guardOffset) ? gs : 0;
      *collideFlag(s + L.ct) = CS_IDLE;
      *earlyFlag(s + L.ct) = EA_PENDING;
    }
    __syncthreads();  // the one barrier both waves take: flags initialised
    if (threadIdx.x >= WAVE) {
      // the helper's work is speculative: it only takes issue slots the
      // step's wave leaves idle (lower wave priority on the shared SIMD)
      __builtin_amdgcn_s_setprio(0);
      {
        double* ct = lds<true>(s) + L.ct;
#ifdef NIMBLE_STAGE_TIMING
        // where the helper runs: HW_ID (SIMD, CU, SE) and XCC_ID
        if (lane == 0 && md.numPairs > 0) {
          double* gs = snapshot + (size_t)env * snapDoubles + snStamps(n);
          gs[92] = (double)(unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));
          gs[93] = (double)(unsigned)__builtin_amdgcn_s_getreg(20 | (15 << 11));
        }
#endif
        if (R == 1) {
          // (the deadlock guard expired: wave 0 detects the contacts itself)
          if (collideWait(ct, CS_GO, GW_HELPER_GO)) {
#ifdef NIMBLE_STAGE_TIMING
            collideWorld<kMesh>(md, lds<true>(s), L, lane, snapshot + (size_t)env * snapDoubles + snEdge(n),
                                snapshot + (size_t)env * snapDoubles + snStamps(n));
#else
            collideWorld<kMesh>(md, lds<true>(s), L, lane, snapshot + (size_t)env * snapDoubles + snEdge(n));
#endif
            // CS_DONE, then the early rows, Y and A (EA_*)
            helperEarly(md, lds<true>(s), L, lane, deferRows);
          }
        }  // (the wide kernel's worlds come with the one-row kernel's contacts)
#ifdef NIMBLE_STAGE_TIMING
        double* hstamp = snapshot + (size_t)env * snapDoubles + snStamps(n);
#else
        double* hstamp = nullptr;
#endif
        // (the world's HBM LCP pool, the wide kernel's off-chip cascade)
        double* hbmPool = snapshot + (size_t)env * snapDoubles + snapWorkspaceOffset(n);
        helperWave<(R > 1)>(md, s, md.lay[0], lane, hstamp, hbmPool,
                            snapshot + (size_t)env * snapDoubles);  // not inlined: the model's copy of L, not the argument's
      }
      return;
    }
    __builtin_amdgcn_s_setprio(2);
  }
  {
    const double* st = state + (size_t)env * 2 * n;
#ifdef NIMBLE_STAGE_TIMING
    double* g_stamp = md.numPairs > 0 ? snapshot + (size_t)env * snapDoubles + snStamps(n) : nullptr;
#endif
    // (stage timing: a deferred world's stamps of the wide kernel's own
    // phases go to slots 104..107, so that every interval the tool forms is
    // between two stamps of one launch -- shader clocks of two launches are
    // not comparable)
    if (R > 1) STAMP(104);
    else STAMP(10);
#ifdef NIMBLE_STAGE_TIMING
    // where wave 0 runs: HW_ID (SIMD, CU, SE) and XCC_ID
    if (lane == 0 && g_stamp) {
      g_stamp[90] = (double)(unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));
      g_stamp[91] = (double)(unsigned)__builtin_amdgcn_s_getreg(20 | (15 << 11));
    }
#endif
    loadState(md, s, L, lane, st, forces + (size_t)env * n);
    if (R > 1) {
      // a world the one-row kernel deferred: its kinematics, Cholesky factor
      // and bias forces are in the snapshot's dynamics cache (stored before
      // it deferred), its contacts in the workspace hand-off (contactStage):
      // reloaded, not recomputed
      dynCacheCopy(md, s, L, snapshot + (size_t)env * snapDoubles + L.snDyn, false, lane);
      STAMP(105);
    } else {
#ifdef NIMBLE_STAGE_TIMING
    kinematics(md, s, L, lane, nullptr, g_stamp);
#else
    kinematics(md, s, L, lane, nullptr);
#endif
    // body transforms final: the helper wave detects the contacts meanwhile
    if (helperOn) collidePost(lds<true>(s) + L.ct, CS_GO, lane);
    STAMP(14);
    composites(md, s, L, lane);
    STAMP(15);
    massMatrixAndBias(md, s, L, lane, s + L.rhs);
    STAMP(16);
    cholesky(s + L.M, s + L.dinv, md.n, lane);
    STAMP(17);
    dynCacheCopy(md, s, L, snapshot + (size_t)env * snapDoubles + L.snDyn, true, lane);
    // V, A, IC, F dead, the Cholesky factor final: the helper's early rows
    // may turn into Y and A (contact.cuh EA_*)
    if (helperOn) dynDonePost(lds<true>(s) + L.ct, lane);
    STAMP(11);
    }
    // rhs = tau + spring + damping - C   (GenericJoint::updateTotalForceDynamic)
    double* x = s + L.x;
    for (int i = lane; i < n; i += WAVE) {
      const double qi = s[L.q + i], vi = s[L.v + i];
      const double springF = -md.spring[i] * (qi - md.rest[i] + vi * md.dt);
      const double dampF = -md.damping[i] * vi;
      x[i] = s[L.tau + i] + springF + dampF - s[L.rhs + i];
    }
    WSYNC();
    cholSolve(s + L.M, s + L.dinv, x, n, lane);  // x = ddq
    // integrateVelocities (Skeleton.cpp:9329): v1 = v + dt ddq
    double* v1 = s + L.v1;
    for (int i = lane; i < n; i += WAVE) v1[i] = s[L.v + i] + md.dt * x[i];
    WSYNC();
    if (R > 1) STAMP(106);
    else STAMP(12);
    // runConstraintEngine (World.cpp:254): collision, LCP, impulses
    bool deferred = false;
    if (md.numPairs > 0) {
      double* sn = snapshot + (size_t)env * snapDoubles;
      deferred = contactStage<R>(md, s, L, lane, v1, x, lcpCache + (size_t)env * cacheDoubles, sn,
                                 sn + snapWorkspaceOffset(n), helperOn, helperOn && R == 1, deferRows, R > 1,
                                 deferLists ? snapshot : nullptr, snapDoubles, env);
    } else if (lane < 8) {
      // a model without collision pairs still has a snapshot header (no
      // contacts, no rows, no clamping) for the getters to read
      snapshot[(size_t)env * snapDoubles + lane] = 0.0;
    }
    if (helperOn) {
      helperRetire(s, L, lane);
      // a wait between the two waves hit the deadlock guard: the step went on
      // without the helper; flagged so that it raises (ST_PROTOCOL)
      if (protocolFailed(lds<true>(s) + L.ct) && lane == 0) {
        double* stp = snapshot + (size_t)env * snapDoubles + SN_STATUS;
        *stp = (double)((int)*stp | ST_PROTOCOL);
      }
    }
    if (deferred) return;  // the R = 2 kernel writes this world's step
    double* out = nextState + (size_t)env * 2 * n;
    for (int i = lane; i < n; i += WAVE) out[n + i] = v1[i];
    // integratePositions (World.cpp:300): with the pre-step velocity when
    // position and velocity updates run in parallel (the default)
    const double* vint = md.parallelPosVel ? s + L.v : v1;
    if (lane < md.nb) {
      const int b = lane, o = md.dof0[b];
      const int jt = md.jtype[b];
      if (jt == NIMBLE_JOINT_REVOLUTE || jt == NIMBLE_JOINT_PRISMATIC) {
        out[o] = s[L.q + o] + vint[o] * md.dt;
      } else if (jt == NIMBLE_JOINT_TRANSLATIONAL) {
        // math::integratePosition<R3Space> (GenericJoint::integratePositions)
        for (int i = 0; i < 3; i++) out[o + i] = s[L.q + o + i] + vint[o + i] * md.dt;
      } else if (jt == NIMBLE_JOINT_FREE) {
        double r[6];
        freeIntegrate(s + L.q + o, vint + o, md.dt, r);
        for (int i = 0; i < 6; i++) out[o + i] = r[i];
      } else if (jt == NIMBLE_JOINT_BALL) {
        double r[3];
        ballIntegrate(s + L.q + o, vint + o, md.dt, r);
        for (int i = 0; i < 3; i++) out[o + i] = r[i];
      }
    }
    WSYNC();
    if (R > 1) STAMP(107);
    else STAMP(13);
  }
}

extern "C" __global__ void __launch_bounds__(2 * WAVE) __attribute__((amdgpu_waves_per_eu(2)))
nimble_forward_kernel(const ModelDev* __restrict__ mdp, Layout L, const double* __restrict__ state,
                      const double* __restrict__ forces, double* __restrict__ lcpCache,
                      double* __restrict__ nextState, double* __restrict__ snapshot, int snapDoubles,
                      int cacheDoubles, int deferRows, int deferLists) {
  forwardWorld<1>(mdp, L, state, forces, lcpCache, nextState, snapshot, snapDoubles, cacheDoubles, deferRows,
                  blockIdx.x, deferLists != 0);
}

// the same step for models with mesh colliders: the helper wave's collision
// pass with the mesh-box narrow phase inlined (out of line, its prologue
// saved ~92 callee-saved VGPRs per lane on every mesh pair near contact).  A
// separate instance because the inlined collider raises the kernel's
// register pressure everywhere: with it the mesh-free models' forward
// spilled 115 instead of 43 VGPRs (Scratch_Size 1,872 vs 1,504 B/lane)
extern "C" __global__ void __launch_bounds__(2 * WAVE) __attribute__((amdgpu_waves_per_eu(2)))
nimble_forward_mesh_kernel(const ModelDev* __restrict__ mdp, Layout L, const double* __restrict__ state,
                           const double* __restrict__ forces, double* __restrict__ lcpCache,
                           double* __restrict__ nextState, double* __restrict__ snapshot, int snapDoubles,
                           int cacheDoubles, int deferRows, int deferLists) {
  forwardWorld<1, true>(mdp, L, state, forces, lcpCache, nextState, snapshot, snapDoubles, cacheDoubles, deferRows,
                        blockIdx.x, deferLists != 0);
}

// the worlds nimble_forward_kernel deferred (snapshot status ST_DEFERRED),
// from the one-row kernel's dynamics and contacts: up to 64 LCP rows with the
// pool in the big LDS stage (the one-row code, the helper wave on the task
// board), more with two rows per lane and the pool in HBM (the stage holding
// the factorisations).  One wide world per CU (its LDS stage), so one wave
// per SIMD: the kernel takes the whole register file (256 VGPRs + AGPRs, no
// spills; at two waves per SIMD it spilled 117 VGPRs to scratch: mesh Atlas
// forward 2.54 -> 2.49 ms, r05 variant v1).  The non-inlined narrow-phase
// functions both forward kernels call are compiled once, for the tighter of
// the two register budgets.
extern "C" __global__ void __launch_bounds__(2 * WAVE) __attribute__((amdgpu_waves_per_eu(1)))
nimble_forward_wide_kernel(const ModelDev* __restrict__ mdp, Layout L, const double* __restrict__ state,
                           const double* __restrict__ forces, double* __restrict__ lcpCache,
                           double* __restrict__ nextState, double* __restrict__ snapshot, int snapDoubles,
                           int cacheDoubles, int deferLists) {
  // workgroup b steps the b-th deferred world in the one-row kernel's lists,
  // the largest LCPs first (DEFER_BUCKETS counters, then one list of
  // gridDim.x world indices per bucket, in the launch's snapshot headers):
  // the slowest worlds start at once instead of behind the others on a CU
  // (one wide world per CU)
  int env = blockIdx.x;
  if (deferLists) {
    int b = blockIdx.x, q = 0;
    for (; q < DEFER_BUCKETS; q++) {
      const int c = deferCount(snapshot)[q];
      if (b < c) break;
      b -= c;
    }
    if (q == DEFER_BUCKETS) return;  // (whole workgroup: past the deferred worlds)
    env = *deferEntry(snapshot, snapDoubles, q * gridDim.x + b);
  }
  const int st = uni((int)snapshot[(size_t)env * snapDoubles + SN_STATUS]);
  if (!(st & ST_DEFERRED)) return;  // (whole workgroup)
  forwardWorld<2>(mdp, L, state, forces, lcpCache, nextState, snapshot, snapDoubles, cacheDoubles, 1 << 30, env,
                  false);
}

// posPos^T gp and velPos^T gp of one free (ND = 6) or ball (ND = 3) joint at
// dof offset o, added to lane k's gq / gvOut: 4 ND lanes run one perturbed
// integration each into fd (spatial.cuh fdFreeIntegrate: the oracle's
// operation sequence; a ball joint's translation inputs are zero)
template <int ND>
__device__ __forceinline__ void fdBlocksVjp(const double* s, const Layout& L, int o, double dt, int lane, int k,
                                            double* fd, double& gq, double& gvOut) {
  if (lane < 4 * ND) {
    const int which = lane / (2 * ND);  // 0: wrt pos, 1: wrt vel
    const int i = (lane % (2 * ND)) / 2;
    const double sign = (lane % 2) ? -1.0 : 1.0;
    const double eps = which == 0 ? 1e-6 : 1e-7;
    double qq[6] = {0, 0, 0, 0, 0, 0}, vv[6] = {0, 0, 0, 0, 0, 0}, r[6];
    for (int j = 0; j < ND; j++) { qq[j] = s[L.q + o + j]; vv[j] = s[L.v + o + j]; }
    if (which == 0) qq[i] += sign * eps; else vv[i] += sign * eps;
    fdFreeIntegrate(qq, vv, dt, r);
    for (int j = 0; j < 6; j++) fd[lane * 6 + j] = r[j];
  }
  WSYNC();
  if (k >= o && k < o + ND) {
    const int i = k - o;
    double pp = 0.0, vp = 0.0;
    for (int r = 0; r < ND; r++) {
      const double jp = (fd[(i * 2) * 6 + r] - fd[(i * 2 + 1) * 6 + r]) / (2 * 1e-6);
      const double jv = (fd[(2 * ND + i * 2) * 6 + r] - fd[(2 * ND + i * 2 + 1) * 6 + r]) / (2 * 1e-7);
      pp += jp * s[L.gp + o + r];
      vp += jv * s[L.gp + o + r];
    }
    gq += pp;
    gvOut += vp;
  }
  WSYNC();
}

// ---------------------------------------------------------------------------
// Backward: BackpropSnapshot::backprop (dart/neural/BackpropSnapshot.cpp:121)
// as vector-Jacobian products, no full Jacobian is ever formed.
// ---------------------------------------------------------------------------

// Adjoint (vector-Jacobian) form of the world-frame RNEA derivatives.  The
// backward needs w^T dtau/dq and w^T dtau/dqdot at a* for the dynamics
// adjoint w = Minv gv.  With W_c = sum of w_i S_i over the dofs of c and its
// ancestors, per-body 6-vectors
//   alpha = W x* p,  beta = I W,  gamma = -V x* beta,  eps = W x* h,
//   delta = (V x W) x* h - V x* eps,  zeta = -I (V x W),
//   kappa = (W - W_parent) x* F
// (p = I (A - a_g), h = I V, F the composite force) and their subtree sums
// (A, B, Gam, D, E, Zt, K), a dof k on body b with parent l gives
//   w^T dtau/dq_k    = Z_k . [-A - u_l x* B + V_l x* (Gam + V_l x* B + E - Zt) + D + K]
//   w^T dtau/dqdot_k = S_k . [-(V_l + V_b) x* B - Gam - E + Zt]
// (Z_k the subtree's world twist per unit q_k, u_l = A_l - a_g).  This is the
// per-direction sum over subtree bodies of the reference's dID/dq columns
// (Skeleton::getJacobianOfID, DifferentiableContactConstraint / BackpropSnapshot
// use) contracted with w, collapsed to O(nb) 6-vector work; the identity is
// checked against central differences in tools/proto/adjoint_rnea.py.
__device__ __forceinline__ void adjointVectors(const ModelDev& md, double* s, const Layout& L, int lane) {
  const double ag[6] = {0, 0, 0, md.g[0], md.g[1], md.g[2]};
  const int nb = md.nb, n = md.n;
  if (lane < nb) {
    const int b = lane;
    double W[6] = {0, 0, 0, 0, 0, 0};
    for (int k = 0; k < n; k++)  // dofs in topological order: ancestors first
      if ((md.anc[b] >> md.dofBody[k]) & 1ull) {
        const double wk = s[L.w + k];
        for (int i = 0; i < 6; i++) W[i] += wk * s[L.Sw + 6 * k + i];
      }
    double I[36];
    worldInertia(md, s + L.Tw + 12 * b, b, I);
    const double* V = s + L.V + 6 * b;
    double u[6], p[6], h[6], t[6], t2[6], VxW[6];
    for (int i = 0; i < 6; i++) u[i] = s[L.A + 6 * b + i] - ag[i];
    mv6(I, u, p);
    mv6(I, V, h);
    crf(V, h, t);
    for (int i = 0; i < 6; i++) {
      s[L.F + 6 * b + i] = p[i] + t[i];  // f_b, summed over the subtree below
      s[L.Wt + 6 * b + i] = W[i];
    }
    double* a = s + L.adj + 42 * b;
    crf(W, p, a);           // alpha
    mv6(I, W, a + 6);       // beta
    crf(V, a + 6, t);
    for (int i = 0; i < 6; i++) a[12 + i] = -t[i];  // gamma
    crf(W, h, a + 24);      // eps
    crm(V, W, VxW);
    crf(VxW, h, t);
    crf(V, a + 24, t2);
    for (int i = 0; i < 6; i++) a[18 + i] = t[i] - t2[i];  // delta
    mv6(I, VxW, t);
    for (int i = 0; i < 6; i++) a[30 + i] = -t[i];  // zeta
  }
  WSYNC();
  // subtree sums of alpha..zeta and f (-> composite F) over the deepest-
  // child-first edge list (lane = entry; see composites)
  if (lane < 42) {
    const int off = lane < 36 ? L.adj + lane : L.F + (lane - 36);
    const int stride = lane < 36 ? 42 : 6;
#pragma unroll 4
    for (int k = 0; k < md.numAcc; k++) {
      const int p = md.accEdge[k][0], c = md.accEdge[k][1];
      s[off + stride * p] += s[off + stride * c];
    }
  }
  WSYNC();
  if (lane < nb) {
    const int b = lane, par = md.parent[b];
    double d[6];
    for (int i = 0; i < 6; i++) d[i] = s[L.Wt + 6 * b + i] - (par >= 0 ? s[L.Wt + 6 * par + i] : 0.0);
    crf(d, s + L.F + 6 * b, s + L.adj + 42 * b + 36);  // kappa
  }
  WSYNC();
  if (lane < 6) {
    const int off = L.adj + 36 + lane;
#pragma unroll 4
    for (int k = 0; k < md.numAcc; k++) {
      const int p = md.accEdge[k][0], c = md.accEdge[k][1];
      s[off + 42 * p] += s[off + 42 * c];
    }
  }
  WSYNC();
}

// Right Jacobian of SO(3) exp (J_r(th) = I - (1-cos)/t^2 [th] + (t-sin)/t^3 [th]^2)
__device__ void rightJacobianCol(const double* th, int k, double* o) {
  const double t2 = th[0] * th[0] + th[1] * th[1] + th[2] * th[2];
  const double t = sqrt(t2);
  double a, b;
  if (t < 1e-3) { a = 0.5; b = 1.0 / 6.0; }  // expMapJac small-angle branch (Geometry.cpp)
  else { a = (1.0 - cos(t)) / t2; b = (t - sin(t)) / (t2 * t); }
  const double K[9] = {0, -th[2], th[1], th[2], 0, -th[0], -th[1], th[0], 0};
  for (int r = 0; r < 3; r++) {
    double k2 = K[r * 3] * K[k] + K[r * 3 + 1] * K[3 + k] + K[r * 3 + 2] * K[6 + k];
    o[r] = (r == k ? 1.0 : 0.0) - a * K[r * 3 + k] + b * k2;
  }
}

// `rows` upstream gradients per world: rows == 1 is backpropState with the
// given gradNext [batch][2n]; rows == 2n (Jacobian mode) takes the unit
// vectors e_r as upstream gradients (gradNext unused) and skips the bound
// clipping, so item (world, r) of gradState / gradForces is row r of
// d(next state)/d(state) / d(next state)/d(forces) -- the reference's
// getStateJacobian / getControlForceVelJacobian (BackpropSnapshot.cpp:1230,
// :482).  Items of one world then share its snapshot, so each item that
// needs an off-chip LCP workspace uses its workgroup's slice of `ws`
// (wsDoubles per workgroup; a workgroup runs its items one after another).
// fcMode (rows == SN_MAXL): the upstream gradient sits on the clamping
// impulses f_c instead -- item (world, r) puts e_r on f_c (no gradient on the
// next state), so its outputs are row r of d f_c / d(q, v) and d f_c / d tau,
// getJacobianOfConstraintForce (BackpropSnapshot.cpp:2723) for POSITION,
// VELOCITY and FORCE; rows r >= n_c are zero.  The backward's contact terms
// already run through lambda = (Q^+)^T u with u the adjoint of f_c, so the
// mode only replaces u = A_c_ub_E^T Minv gv by e_r (and gv, gp by 0).
// R row slots per lane: the R = 1 kernel takes the items of worlds with at
// most `deferRows` LCP rows, the R = 2 kernel the others.
template <int R>
__device__ __forceinline__ void backwardItems(const ModelDev* __restrict__ mdp, int batch,
                                              const double* __restrict__ state, const double* __restrict__ forces,
                                              double* __restrict__ snapshot, int snapDoubles,
                                              const double* __restrict__ gradNext, double* __restrict__ gradState,
                                              double* __restrict__ gradForces, int rows, double* __restrict__ ws,
                                              int wsDoubles, double* __restrict__ gradMasses, int fcMode,
                                              int massParams, int deferRows) {
  extern __shared__ double s[];
  const ModelDev& md = *mdp;
  const Layout& L = md.lay[1];
  const int lane = threadIdx.x;
  const int n = md.n;
  const double dt = md.dt;
  const long long items = (long long)batch * rows;
  for (long long item = blockIdx.x; item < items; item += gridDim.x) {
    const int env = rows == 1 ? (int)item : (int)(item / rows);
    const int unitRow = rows == 1 ? -1 : (int)(item - (long long)env * rows);
    if (md.numPairs > 0) {
      const int mEnv = uni((int)snapshot[(size_t)env * snapDoubles + SN_M]);
      if ((mEnv > deferRows) != (R > 1)) continue;  // the other kernel's item
    }
#ifdef NIMBLE_STAGE_TIMING
    double* g_stamp = md.numPairs > 0 ? snapshot + (size_t)env * snapDoubles + snStamps(n) : nullptr;
#endif
    STAMP(20);
    if (fcMode && (md.numPairs == 0 || unitRow >= uni((int)snapshot[(size_t)env * snapDoubles + SN_NC]))) {
      for (int i = lane; i < 2 * n; i += WAVE) gradState[(size_t)item * 2 * n + i] = 0.0;
      for (int i = lane; i < n; i += WAVE) gradForces[(size_t)item * n + i] = 0.0;
      continue;
    }
    loadState(md, s, L, lane, state + (size_t)env * 2 * n, forces + (size_t)env * n);
    if (fcMode) {
      for (int i = lane; i < n; i += WAVE) { s[L.gp + i] = 0.0; s[L.gv + i] = 0.0; }
    } else if (unitRow < 0) {
      const double* gN = gradNext + (size_t)env * 2 * n;
      for (int i = lane; i < n; i += WAVE) {
        s[L.gp + i] = gN[i];
        s[L.gv + i] = gN[n + i];
      }
    } else {
      for (int i = lane; i < n; i += WAVE) {
        s[L.gp + i] = i == unitRow ? 1.0 : 0.0;
        s[L.gv + i] = n + i == unitRow ? 1.0 : 0.0;
      }
    }
    double* sn = snapshot + (size_t)env * snapDoubles;
    double* hbmWs = ws != nullptr ? ws + (size_t)blockIdx.x * wsDoubles : sn + snapWorkspaceOffset(n);
    dynCacheCopy(md, s, L, sn + L.snDyn, false, lane);  // the forward's kinematics, L, C
    STAMP(21);
    const int nc = md.numPairs > 0 ? uni((int)sn[SN_NC]) : 0;
    const int m = md.numPairs > 0 ? uni((int)sn[SN_M]) : 0;
    double* x = s + L.x;
    double* w = s + L.w;
    BwdPool P;
    int imp = 0;
    if (nc > 0) {
      // constrained: a* = Minv (z + A_c_ub_E f_c) / dt, w <- w - nu
      const int need = bwdPoolDoubles(m, n);
      carveBwd(need <= L.poolCap ? s + L.pool : hbmWs, m, n, P);
      imp = contactBackwardPrep<R>(md, s, L, lane, sn, P, m, nc, s + L.ct, fcMode ? unitRow : -1);
    } else {
      // z = dt (tau - C - D v - K (q - q0 + dt v))
      for (int i = lane; i < n; i += WAVE) {
        const double qi = s[L.q + i], vi = s[L.v + i];
        const double springF = md.spring[i] * (qi - md.rest[i] + dt * vi);
        const double dampF = md.damping[i] * vi;
        x[i] = dt * (s[L.tau + i] - s[L.rhs + i] - dampF - springF);
        w[i] = s[L.gv + i];
      }
      WSYNC();
      cholSolve(s + L.M, s + L.dinv, x, n, lane);  // x = y = Minv z  => a* = y / dt
      cholSolve(s + L.M, s + L.dinv, w, n, lane);  // w = Minv gv
      for (int i = lane; i < n; i += WAVE) x[i] /= dt;
      WSYNC();
    }
    STAMP(22);
    accelerations(md, s, L, lane, x, s + L.adj);  // A = accelerations at a* (adjoint area not yet in use)
    adjointVectors(md, s, L, lane);
    STAMP(23);

    // ---- per-direction columns -------------------------------------------
    double gq = 0.0, gvOut = 0.0, gt = 0.0;
    double Z[6] = {0, 0, 0, 0, 0, 0};
    const int k = lane;
    if (k < n) {
      const int b = md.dofBody[k];
      const int lam = md.parent[b];
      const double ag[6] = {0, 0, 0, md.g[0], md.g[1], md.g[2]};
      double Vl[6], ul[6];
      for (int i = 0; i < 6; i++) {
        Vl[i] = lam >= 0 ? s[L.V + 6 * lam + i] : 0.0;
        ul[i] = (lam >= 0 ? s[L.A + 6 * lam + i] : 0.0) - ag[i];
      }
      // position generator Z (world twist of the subtree per unit q_k)
      const double* Sk = s + L.Sw + 6 * k;
      // (ball joints: the free joint's rotational half, BallJoint.cpp:282)
      if (md.jtype[b] == NIMBLE_JOINT_FREE || md.jtype[b] == NIMBLE_JOINT_BALL) {
        const int o = md.dof0[b];
        const int c = k - o;
        double xi[6] = {0, 0, 0, 0, 0, 0};
        const double* th = s + L.q + o;
        if (c < 3) {
          rightJacobianCol(th, c, xi);
        } else {
          double Rm[9];
          expMapRot(th, Rm);
          for (int r = 0; r < 3; r++) xi[3 + r] = Rm[(c - 3) * 3 + r];  // R^T e_c
        }
        double TwC[12];
        tmul(s + L.Tw + 12 * b, md.Tcj[b], TwC);
        adT(TwC, xi, Z);
      } else {
        for (int i = 0; i < 6; i++) Z[i] = Sk[i];
      }
      // adjoint contraction at body b (subtree sums, see adjointVectors)
      const double* a = s + L.adj + 42 * b;
      double t[6], r[6], acc6[6];
      crf(Vl, a + 6, t);  // V_l x* B
      for (int i = 0; i < 6; i++) r[i] = a[12 + i] + t[i] + a[24 + i] - a[30 + i];
      crf(Vl, r, t);
      crf(ul, a + 6, r);  // u_l x* B
      for (int i = 0; i < 6; i++) acc6[i] = -a[i] - r[i] + t[i] + a[18 + i] + a[36 + i];
      const double accQ = dot6(Z, acc6);
      double vs[6];
      for (int i = 0; i < 6; i++) vs[i] = Vl[i] + s[L.V + 6 * b + i];
      crf(vs, a + 6, t);
      for (int i = 0; i < 6; i++) acc6[i] = -t[i] - a[12 + i] - a[24 + i] + a[30 + i];
      const double accV = dot6(Sk, acc6);
      const double wk = w[k];
      gq = -dt * accQ - dt * md.spring[k] * wk;
      gvOut = s[L.gv + k] - dt * accV - dt * md.damping[k] * wk - dt * dt * md.spring[k] * wk;
      gt = dt * wk;
      if (nc > 0) gvOut -= P.NV[k * NV_COLS + NV_MU];
      // posPos^T gp and velPos^T gp for the Euclidean joints (revolute,
      // prismatic, translational: GenericJoint::getPosPosJacobian /
      // getVelPosJacobian): identity / dt * identity
      if (md.jtype[b] != NIMBLE_JOINT_FREE && md.jtype[b] != NIMBLE_JOINT_BALL) {
        gq += s[L.gp + k];
        gvOut += dt * s[L.gp + k];
      }
    }
    WSYNC();
    STAMP(24);
    if (nc > 0) {
      // the adjoint vectors are dead now: workspace for the contact-geometry
      // terms (6n + 6nb <= 42nb), then for the M-derivative field pairs (24nb)
      double* buf = s + L.adj;
      TACC_BEGIN(tG);
#ifdef NIMBLE_STAGE_TIMING
      const double gterm = contactGTermsAll<R>(md, s, L, sn, P, m, Z, buf, lane, g_stamp);
#else
      const double gterm = contactGTermsAll<R>(md, s, L, sn, P, m, Z, buf, lane);
#endif
      WSYNC();
      TACC_END(80, tG);
      TACC_BEGIN(tM);
      const double mterm = mFieldsTerm(md, s, L, P.NV, buf, lane, k, Z, -dt, (double)imp);
      TACC_END(81, tM);
      if (k < n) {
        gq += gterm;
        gq += mterm;
      }
      WSYNC();
    }
    STAMP(25);
    if (gradMasses != nullptr) {
      // lossWrtMass = getMassVelJacobian^T gv (BackpropSnapshot.cpp:177, :580:
      // getVelJacobianWrt(WithRespectTo::MASS), :980) for every body's inertia
      // parameters (WithRespectToMass.cpp:35, INERTIA_FULL order: mass, local
      // COM x y z, moment about the COM Ixx Iyy Izz Ixy Ixz Iyz; massParams 1
      // = the mass only).  They enter M and C only (not A_c, springs or the
      // integration), so each takes the M / C terms of the position gradient
      // above with d/dq replaced by d/dtheta:  -dt (dID(q,v,a*)/dtheta)^T (w - nu)
      // plus the M-derivative pairs  sum coef * x_a^T (dG_b/dtheta) x_c.  With
      // twists x = [w; v] (world frame), the COM c (world), its velocity
      // u_x = v - c x w and the body-frame angular velocity wb = R^T w:
      //   x^T G y = wb_x^T I wb_y + m u_x . u_y,   G y = [R I wb_y + m c x u_y; m u_y]
      // so d/dm: u_x . u_y; d/dc_k (r_k = R e_k, du_y = w_y x r_k):
      // m (w_x x r_k . u_y + u_x . w_y x r_k); d/dI_ij: wb_x,i wb_y,j (+ sym).
      // y^T dID/dtheta = V_y^T [dG (A_b - a_g) + V_b x* (dG V_b)].
      if (lane < md.nb) {
        const int b = lane;
        const double* Tw = s + L.Tw + 12 * b;
        const double m = md.mass[b];
        double cw[3];
        for (int r = 0; r < 3; r++)
          cw[r] = Tw[r * 4] * md.com[b][0] + Tw[r * 4 + 1] * md.com[b][1] + Tw[r * 4 + 2] * md.com[b][2] + Tw[r * 4 + 3];
        auto comVel = [&](const double* y, double* u) {
          double cx[3];
          cross3(cw, y, cx);  // c x y_ang
          for (int i = 0; i < 3; i++) u[i] = y[3 + i] - cx[i];
        };
        auto bodyAng = [&](const double* y, double* wb) {  // R^T y_ang
          for (int i = 0; i < 3; i++) wb[i] = Tw[i] * y[0] + Tw[4 + i] * y[1] + Tw[8 + i] * y[2];
        };
        // x^T dG/dtheta y for every parameter p (out[p], accumulated with coef)
        auto pairTerms = [&](const double* x, const double* y, double coef, double* out) {
          double ux[3], uy[3];
          comVel(x, ux);
          comVel(y, uy);
          out[0] += coef * (ux[0] * uy[0] + ux[1] * uy[1] + ux[2] * uy[2]);
          if (massParams < 10) return;
          for (int k = 0; k < 3; k++) {
            const double rk[3] = {Tw[k], Tw[4 + k], Tw[8 + k]};
            double a[3], c[3];
            cross3(x, rk, a);  // w_x x r_k
            cross3(y, rk, c);  // w_y x r_k
            out[1 + k] += coef * m * (a[0] * uy[0] + a[1] * uy[1] + a[2] * uy[2] + ux[0] * c[0] + ux[1] * c[1] + ux[2] * c[2]);
          }
          double bx[3], by[3];
          bodyAng(x, bx);
          bodyAng(y, by);
          out[4] += coef * bx[0] * by[0];
          out[5] += coef * bx[1] * by[1];
          out[6] += coef * bx[2] * by[2];
          out[7] += coef * (bx[0] * by[1] + bx[1] * by[0]);
          out[8] += coef * (bx[0] * by[2] + bx[2] * by[0]);
          out[9] += coef * (bx[1] * by[2] + bx[2] * by[1]);
        };
        const double ag[6] = {0, 0, 0, md.g[0], md.g[1], md.g[2]};
        const double* Vb = s + L.V + 6 * b;
        double Ab[6], Vw[6], val[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int i = 0; i < 6; i++) Ab[i] = s[L.A + 6 * b + i] - ag[i];
        bodyTwist(md, s + L.Sw, b, s + L.w, 1, Vw);
        pairTerms(Vw, Ab, -dt, val);
        // Vw^T (V_b x* (dG V_b)) per parameter
        {
          double uV[3], h[6], fh[6];
          comVel(Vb, uV);
          cross3(cw, uV, h);
          for (int i = 0; i < 3; i++) h[3 + i] = uV[i];
          crf(Vb, h, fh);
          val[0] += -dt * dot6(Vw, fh);
          if (massParams >= 10) {
            double bv[3];
            bodyAng(Vb, bv);
            for (int k = 0; k < 3; k++) {
              const double rk[3] = {Tw[k], Tw[4 + k], Tw[8 + k]};
              double du[3], t1[3], t2[3];
              cross3(Vb, rk, du);  // dU/dc_k = w_V x r_k
              cross3(rk, uV, t1);
              cross3(cw, du, t2);
              for (int i = 0; i < 3; i++) { h[i] = m * (t1[i] + t2[i]); h[3 + i] = m * du[i]; }
              crf(Vb, h, fh);
              val[1 + k] += -dt * dot6(Vw, fh);
            }
            // dG/dI_ij V_b = [R E_ij R^T w_V; 0]
            const int pi[6] = {0, 1, 2, 0, 0, 1}, pj[6] = {0, 1, 2, 1, 2, 2};
            for (int q = 0; q < 6; q++) {
              double eb[3] = {0, 0, 0};
              eb[pi[q]] += bv[pj[q]];
              if (pi[q] != pj[q]) eb[pj[q]] += bv[pi[q]];
              for (int i = 0; i < 3; i++) { h[i] = Tw[i * 4] * eb[0] + Tw[i * 4 + 1] * eb[1] + Tw[i * 4 + 2] * eb[2]; h[3 + i] = 0.0; }
              crf(Vb, h, fh);
              val[4 + q] += -dt * dot6(Vw, fh);
            }
          }
        }
        if (nc > 0) {
          const double coef[4] = {-dt, 1.0, -(double)imp, -(double)imp};
          for (int pr = 0; pr < (imp ? 4 : 2); pr++) {
            double Va[6], Vc[6];
            bodyTwist(md, s + L.Sw, b, P.NV + 2 * pr, NV_COLS, Va);
            bodyTwist(md, s + L.Sw, b, P.NV + 2 * pr + 1, NV_COLS, Vc);
            pairTerms(Va, Vc, coef[pr], val);
          }
        }
        for (int q = 0; q < massParams; q++) gradMasses[((size_t)item * md.nb + b) * massParams + q] = val[q];
      }
      WSYNC();
    }
    // FreeJoint / BallJoint posPos / velPos blocks: central differences
    // exactly as FreeJoint::finiteDifferencePosPosJacobian / VelPosJacobian
    // (FreeJoint.cpp:965, :987) and BallJoint's (BallJoint.cpp:368, :390);
    // 4 ND lanes (ND = 6 / 3 coordinates), one perturbed integration each.  A
    // ball joint's integration is the free joint's rotational half (the same
    // operations; its translation inputs zero, outputs unused)
    double* fd = s + L.scratch;
    for (int f = 0; f < md.numFree; f++) {
      const int b = md.freeBody[f], o = md.dof0[b];
      if (md.jtype[b] == NIMBLE_JOINT_FREE)
        fdBlocksVjp<6>(s, L, o, dt, lane, k, fd, gq, gvOut);
      else
        fdBlocksVjp<3>(s, L, o, dt, lane, k, fd, gq, gvOut);
    }
    if (k < n) {
      if (unitRow < 0) {
        // clipLossGradientsToBounds (BackpropSnapshot.cpp:425); the
        // Jacobian getters do not clip
        const double qk = s[L.q + k], vk = s[L.v + k], tk = s[L.tau + k];
        if (qk == md.posLo[k] && gq > 0) gq = 0;
        if (qk == md.posHi[k] && gq < 0) gq = 0;
        if (vk == md.velLo[k] && gvOut > 0) gvOut = 0;
        if (vk == md.velHi[k] && gvOut < 0) gvOut = 0;
        if (tk == md.forceLo[k] && gt > 0) gt = 0;
        if (tk == md.forceHi[k] && gt < 0) gt = 0;
      }
      gradState[(size_t)item * 2 * n + k] = gq;
      gradState[(size_t)item * 2 * n + n + k] = gvOut;
      gradForces[(size_t)item * n + k] = gt;
    }
    WSYNC();
    STAMP(26);
  }
}

extern "C" __global__ void __launch_bounds__(WAVE)
nimble_backward_kernel(const ModelDev* __restrict__ mdp, int batch, const double* __restrict__ state,
                       const double* __restrict__ forces, double* __restrict__ snapshot, int snapDoubles,
                       const double* __restrict__ gradNext, double* __restrict__ gradState,
                       double* __restrict__ gradForces, int rows, double* __restrict__ ws, int wsDoubles,
                       double* __restrict__ gradMasses, int fcMode, int massParams, int deferRows) {
  backwardItems<1>(mdp, batch, state, forces, snapshot, snapDoubles, gradNext, gradState, gradForces, rows, ws,
                   wsDoubles, gradMasses, fcMode, massParams, deferRows);
}

extern "C" __global__ void __launch_bounds__(WAVE)
nimble_backward_wide_kernel(const ModelDev* __restrict__ mdp, int batch, const double* __restrict__ state,
                            const double* __restrict__ forces, double* __restrict__ snapshot, int snapDoubles,
                            const double* __restrict__ gradNext, double* __restrict__ gradState,
                            double* __restrict__ gradForces, int rows, double* __restrict__ ws, int wsDoubles,
                            double* __restrict__ gradMasses, int fcMode, int massParams, int deferRows) {
  backwardItems<2>(mdp, batch, state, forces, snapshot, snapDoubles, gradNext, gradState, gradForces, rows, ws,
                   wsDoubles, gradMasses, fcMode, massParams, deferRows);
}
