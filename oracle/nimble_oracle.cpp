// ORACLE / TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference's differentiable timestep, used by tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.  It
// is never linked into, called by, or shipped with the product path
// (nimblephysics_amd/csrc), which must fail loudly without its HIP library.
//
// Structure follows the reference call graph:
//   World::step                         dart/simulation/World.cpp:221
//     Skeleton::computeForwardDynamics  dart/dynamics/Skeleton.cpp:13034 (ABA,
//        BodyNode::updateBiasForce BodyNode.cpp:2067, updateAccelerationFD :2149,
//        GenericJoint::updateTotalForceDynamic detail/GenericJoint.hpp:2554,
//        updateAccelerationDynamic :2656, addChildArtInertiaToDynamic :2168,
//        addChildBiasForceToDynamic :2395)
//     Skeleton::integrateVelocities     Skeleton.cpp:9329
//     ConstraintSolver::solve (contacts) -- oracle_contact.cpp
//     World::integratePositions         World.cpp:300 (parallel pos/vel update)
//   BackpropSnapshot::backprop          dart/neural/BackpropSnapshot.cpp:121
//
// Analytic derivatives that the reference computes in closed form
// (Skeleton::getJacobianOfC Skeleton.cpp:1779, getJacobianOfMinv :2024) are
// obtained here by forward-mode dual numbers through the same body-frame
// recursions: exact to rounding, and independent of the product's
// world-frame closed-form derivative kernels.
#include "oracle.hpp"

#include <cmath>
#include <cstring>
#include <cstdio>
#include <vector>

namespace oracle {

//------------------------------------------------------------------------------
World::World(const nimble_world_desc* d) {
  nb = d->num_bodies;
  n = d->num_dofs;
  dt = d->dt;
  for (int i = 0; i < 3; i++) g[i] = d->gravity[i];
  clipDepth = d->contact_clipping_depth;
  fallbackCfm = d->fallback_cfm;
  penetrationCorrection = d->penetration_correction != 0;
  parallelPosVel = d->parallel_pos_vel != 0;
  bodies.resize(nb);
  for (int b = 0; b < nb; b++) {
    Body& B = bodies[b];
    B.parent = d->parent[b];
    B.skel = d->skeleton[b];
    B.jtype = d->joint_type[b];
    B.dof0 = d->dof_offset[b];
    B.mobile = d->skeleton_mobile[b] != 0;
    // (WeldJoint 0, Revolute / Prismatic 1, Ball / Translational 3, Free 6)
    B.ndof = B.jtype == NIMBLE_JOINT_WELD ? 0
             : B.jtype == NIMBLE_JOINT_FREE ? 6
             : (B.jtype == NIMBLE_JOINT_BALL || B.jtype == NIMBLE_JOINT_TRANSLATIONAL) ? 3 : 1;
    auto loadIso = [](const double* t, Iso<double>& T) {
      for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) T.R(r, c) = t[r * 4 + c];
        T.p[r] = t[r * 4 + 3];
      }
    };
    loadIso(d->T_parent_joint + 12 * b, B.Tpj);
    loadIso(d->T_child_joint + 12 * b, B.Tcj);
    for (int i = 0; i < 3; i++) B.axis[i] = d->axis[3 * b + i];
    // dart/dynamics/Inertia.cpp:1368 computeSpatialTensor
    double m = d->mass[b];
    V3<double> c{{d->com[3 * b], d->com[3 * b + 1], d->com[3 * b + 2]}};
    const double* mo = d->moment + 6 * b;
    M3<double> I;
    I(0, 0) = mo[0]; I(1, 1) = mo[1]; I(2, 2) = mo[2];
    I(0, 1) = I(1, 0) = mo[3]; I(0, 2) = I(2, 0) = mo[4]; I(1, 2) = I(2, 1) = mo[5];
    M3<double> C = skew(c);
    M3<double> CCt = mul(C, transpose(C));
    B.G = zero66<double>();
    for (int r = 0; r < 3; r++)
      for (int cc = 0; cc < 3; cc++) {
        B.G(r, cc) = I(r, cc) + m * CCt(r, cc);
        B.G(r, cc + 3) = m * C(r, cc);
        B.G(r + 3, cc) = m * C(cc, r);
        B.G(r + 3, cc + 3) = (r == cc) ? m : 0.0;
      }
    B.friction = d->friction[b];
    B.restitution = d->restitution[b];
  }
  damping.assign(d->damping, d->damping + n);
  spring.assign(d->spring, d->spring + n);
  restPos.assign(d->rest_position, d->rest_position + n);
  posLo.assign(d->pos_lower, d->pos_lower + n);
  posHi.assign(d->pos_upper, d->pos_upper + n);
  velLo.assign(d->vel_lower, d->vel_lower + n);
  velHi.assign(d->vel_upper, d->vel_upper + n);
  forceLo.assign(d->force_lower, d->force_lower + n);
  forceHi.assign(d->force_upper, d->force_upper + n);
  shapes.resize(d->num_shapes);
  for (int s = 0; s < d->num_shapes; s++) {
    Shape& S = shapes[s];
    S.body = d->shape_body[s];
    S.type = d->shape_type[s];
    for (int i = 0; i < 3; i++) S.size[i] = d->shape_size[3 * s + i];
    for (int r = 0; r < 3; r++) {
      for (int c = 0; c < 3; c++) S.T.R(r, c) = d->shape_T[12 * s + r * 4 + c];
      S.T.p[r] = d->shape_T[12 * s + r * 4 + 3];
    }
    if (S.type == NIMBLE_SHAPE_MESH && d->mesh_vertices != nullptr) {
      const int f = d->shape_mesh_first[s], c = d->shape_mesh_count[s];
      S.verts.assign(d->mesh_vertices + 3 * (size_t)f, d->mesh_vertices + 3 * (size_t)(f + c));
    }
  }
  // dof -> body map
  dofBody.assign(n, -1);
  for (int b = 0; b < nb; b++)
    for (int k = 0; k < bodies[b].ndof; k++) dofBody[bodies[b].dof0 + k] = b;
}

//------------------------------------------------------------------------------
// Joint relative transform and Jacobian (RevoluteJoint.cpp:203, :141;
// PrismaticJoint.cpp:188, :140; FreeJoint.cpp:1027, :1049 identity-Jacobian).
template <class S>
void jointTransform(const Body& B, const S* q, Iso<S>& T, M6<S>& Sj /* 6 x ndof, col-major in first ndof cols */) {
  Iso<S> Tpj, Tcj;
  for (int i = 0; i < 9; i++) { Tpj.R.m[i] = S(B.Tpj.R.m[i]); Tcj.R.m[i] = S(B.Tcj.R.m[i]); }
  for (int i = 0; i < 3; i++) { Tpj.p[i] = S(B.Tpj.p[i]); Tcj.p[i] = S(B.Tcj.p[i]); }
  Iso<S> Q = identityIso<S>();
  M6<S> local = zero66<S>();
  if (B.jtype == NIMBLE_JOINT_REVOLUTE) {
    // math::expAngular(axis * q): Rodrigues
    S c = cos(q[0]), s = sin(q[0]);
    S a[3] = {S(B.axis[0]), S(B.axis[1]), S(B.axis[2])};
    for (int r = 0; r < 3; r++)
      for (int cc = 0; cc < 3; cc++) Q.R(r, cc) = (S(1.0) - c) * a[r] * a[cc] + ((r == cc) ? c : S(0.0));
    Q.R(0, 1) = Q.R(0, 1) - s * a[2]; Q.R(0, 2) = Q.R(0, 2) + s * a[1];
    Q.R(1, 0) = Q.R(1, 0) + s * a[2]; Q.R(1, 2) = Q.R(1, 2) - s * a[0];
    Q.R(2, 0) = Q.R(2, 0) - s * a[1]; Q.R(2, 1) = Q.R(2, 1) + s * a[0];
    for (int i = 0; i < 3; i++) local(i, 0) = a[i];
  } else if (B.jtype == NIMBLE_JOINT_PRISMATIC) {
    for (int i = 0; i < 3; i++) { Q.p[i] = S(B.axis[i]) * q[0]; local(i + 3, 0) = S(B.axis[i]); }
  } else if (B.jtype == NIMBLE_JOINT_FREE) {
    V3<S> w{{q[0], q[1], q[2]}};
    Q.R = expMapRot(w);
    for (int i = 0; i < 3; i++) Q.p[i] = q[3 + i];
    for (int i = 0; i < 6; i++) local(i, i) = S(1.0);
  } else if (B.jtype == NIMBLE_JOINT_BALL) {
    // BallJoint::updateRelativeTransform (BallJoint.cpp:422, convertToRotation
    // = expMapRot :91) and, with DART_USE_IDENTITY_JACOBIAN, the Jacobian
    // getAdTMatrix(T_cj).leftCols<3>() (:446)
    V3<S> w{{q[0], q[1], q[2]}};
    Q.R = expMapRot(w);
    for (int i = 0; i < 3; i++) local(i, i) = S(1.0);
  } else if (B.jtype == NIMBLE_JOINT_TRANSLATIONAL) {
    // TranslationalJoint::updateRelativeTransform / updateRelativeJacobian
    // (TranslationalJoint.cpp:127, :138): Translation(q), [0; R_cj]
    for (int i = 0; i < 3; i++) { Q.p[i] = q[i]; local(3 + i, i) = S(1.0); }
  }
  T = compose(compose(Tpj, Q), inverse(Tcj));
  // S = Ad(T_cj) * local  (AdTAngular / AdTLinear / getAdTMatrix)
  Sj = zero66<S>();
  for (int k = 0; k < B.ndof; k++) {
    V6<S> col; for (int i = 0; i < 6; i++) col[i] = local(i, k);
    V6<S> r = AdT(Tcj, col);
    for (int i = 0; i < 6; i++) Sj(i, k) = r[i];
  }
}

//------------------------------------------------------------------------------
template <class S>
void Kin<S>::compute(const World& w, const S* q, const S* dq) {
  int nb = w.nb;
  T.resize(nb); Tw.resize(nb); Sj.resize(nb); V.resize(nb); eta.resize(nb);
  for (int b = 0; b < nb; b++) {
    const Body& B = w.bodies[b];
    jointTransform<S>(B, q + B.dof0, T[b], Sj[b]);
    Tw[b] = B.parent >= 0 ? compose(Tw[B.parent], T[b]) : T[b];
    V6<S> Sdq = zero6<S>();
    for (int k = 0; k < B.ndof; k++)
      for (int i = 0; i < 6; i++) Sdq[i] = Sdq[i] + Sj[b](i, k) * dq[B.dof0 + k];
    V[b] = B.parent >= 0 ? add(AdInvT(T[b], V[B.parent]), Sdq) : Sdq;
    // GenericJoint::setPartialAccelerationTo (detail/GenericJoint.hpp:1814), dS = 0
    eta[b] = ad(V[b], Sdq);
  }
}
template struct Kin<double>;
template struct Kin<Dual>;

//------------------------------------------------------------------------------
// Inverse dynamics (BodyNode::updateTransmittedForceID BodyNode.cpp:1994 +
// GenericJoint::updateForceID): tau = S^T F with
//   F_i = G A_i - Fgrav_i - dad(V_i, G V_i) + sum_c dAdInvT(T_c, F_c).
// Used for C(q,v)+g (Skeleton::updateCoriolisAndGravityForces :12652, i.e.
// ddq = 0) and for mass-matrix products (gravity off, v = 0).
template <class S>
void inverseDynamics(const World& w, const Kin<S>& k, const S* ddq, bool withGravity, bool withVel, S* tau) {
  int nb = w.nb;
  std::vector<V6<S>> A(nb), F(nb);
  for (int b = 0; b < nb; b++) {
    const Body& B = w.bodies[b];
    V6<S> Sddq = zero6<S>();
    for (int kk = 0; kk < B.ndof; kk++)
      for (int i = 0; i < 6; i++) Sddq[i] = Sddq[i] + k.Sj[b](i, kk) * ddq[B.dof0 + kk];
    V6<S> base = B.parent >= 0 ? AdInvT(k.T[b], A[B.parent]) : zero6<S>();
    A[b] = add(base, Sddq);
    if (withVel) A[b] = add(A[b], k.eta[b]);
  }
  for (int b = nb - 1; b >= 0; b--) {
    const Body& B = w.bodies[b];
    M6<S> G; for (int i = 0; i < 36; i++) G.m[i] = S(B.G.m[i]);
    V6<S> f = mul(G, A[b]);
    if (withGravity) {
      // AdInvRLinear(T_world, g)
      V3<S> gg{{S(w.g[0]), S(w.g[1]), S(w.g[2])}};
      V3<S> gl = mulT(k.Tw[b].R, gg);
      V6<S> ag = zero6<S>(); for (int i = 0; i < 3; i++) ag[3 + i] = gl[i];
      f = sub(f, mul(G, ag));
    }
    if (withVel) f = sub(f, dad(k.V[b], mul(G, k.V[b])));
    F[b] = add(F[b], f);
    if (B.parent >= 0) F[B.parent] = add(F[B.parent], dAdInvT(k.T[b], F[b]));
    for (int kk = 0; kk < B.ndof; kk++) {
      S s(0.0);
      for (int i = 0; i < 6; i++) s += k.Sj[b](i, kk) * F[b][i];
      tau[B.dof0 + kk] = s;
    }
  }
}
//------------------------------------------------------------------------------
// Articulated-body forward dynamics exactly as Skeleton::computeForwardDynamics
// (Skeleton.cpp:13034): backward pass updateArtInertia + updateBiasForce,
// forward pass updateAccelerationFD.  Returns ddq.
void forwardDynamicsABA(const World& w, const Kin<double>& k, const double* q, const double* dq,
                        const double* tauCtrl, double* ddq) {
  int nb = w.nb;
  std::vector<M6<double>> AI(nb);
  std::vector<V6<double>> Bias(nb), Acc(nb);
  std::vector<std::vector<double>> Psi(nb), totalForce(nb);
  for (int b = nb - 1; b >= 0; b--) {
    const Body& B = w.bodies[b];
    // updateArtInertia (BodyNode.cpp:2037)
    AI[b] = B.G;
    // updateBiasForce (BodyNode.cpp:2067)
    V3<double> gl = mulT(k.Tw[b].R, V3<double>{{w.g[0], w.g[1], w.g[2]}});
    V6<double> ag = zero6<double>(); for (int i = 0; i < 3; i++) ag[3 + i] = gl[i];
    V6<double> Fg = mul(B.G, ag);
    Bias[b] = sub(scale(dad(k.V[b], mul(B.G, k.V[b])), -1.0), Fg);
    // children were processed already (reverse order): they added themselves.
    (void)q;
  }
  // The reverse loop above initialised AI/Bias with the body's own terms;
  // now accumulate children contributions in a second reverse sweep so that a
  // child is complete before it is added to its parent.
  for (int b = nb - 1; b >= 0; b--) {
    const Body& B = w.bodies[b];
    int nd = B.ndof;
    // parent joint: updateInvProjArtInertia (detail/GenericJoint.hpp:2276)
    Psi[b].assign(nd * nd, 0.0);
    totalForce[b].assign(nd, 0.0);
    if (nd > 0) {
      std::vector<double> P(nd * nd);
      for (int r = 0; r < nd; r++)
        for (int c = 0; c < nd; c++) {
          double s = 0;
          for (int i = 0; i < 6; i++)
            for (int j = 0; j < 6; j++) s += k.Sj[b](i, r) * AI[b](i, j) * k.Sj[b](j, c);
          P[r * nd + c] = s;
        }
      invertSmall(P.data(), Psi[b].data(), nd);
      // updateTotalForceDynamic (detail/GenericJoint.hpp:2554)
      V6<double> bf = add(mul(AI[b], k.eta[b]), Bias[b]);
      for (int r = 0; r < nd; r++) {
        int dof = B.dof0 + r;
        double springF = -w.spring[dof] * (q[dof] - w.restPos[dof] + dq[dof] * w.dt);
        double dampF = -w.damping[dof] * dq[dof];
        double s = 0; for (int i = 0; i < 6; i++) s += k.Sj[b](i, r) * bf[i];
        totalForce[b][r] = tauCtrl[dof] + springF + dampF - s;
      }
    }
    if (B.parent >= 0) {
      // addChildArtInertiaToDynamic (detail/GenericJoint.hpp:2168)
      M6<double> PI = AI[b];
      if (nd > 0) {
        double AIS[6][6];
        for (int i = 0; i < 6; i++)
          for (int c = 0; c < nd; c++) {
            double s = 0; for (int j = 0; j < 6; j++) s += AI[b](i, j) * k.Sj[b](j, c);
            AIS[i][c] = s;
          }
        for (int i = 0; i < 6; i++)
          for (int j = 0; j < 6; j++) {
            double s = 0;
            for (int r = 0; r < nd; r++)
              for (int c = 0; c < nd; c++) s += AIS[i][r] * Psi[b][r * nd + c] * AIS[j][c];
            PI(i, j) -= s;
          }
      }
      M6<double> add6 = transformInertia(inverse(k.T[b]), PI);
      for (int i = 0; i < 36; i++) AI[B.parent].m[i] += add6.m[i];
      // addChildBiasForceToDynamic (detail/GenericJoint.hpp:2395)
      V6<double> SPsiTau = zero6<double>();
      for (int r = 0; r < nd; r++) {
        double t = 0; for (int c = 0; c < nd; c++) t += Psi[b][r * nd + c] * totalForce[b][c];
        for (int i = 0; i < 6; i++) SPsiTau[i] += k.Sj[b](i, r) * t;
      }
      V6<double> beta = add(Bias[b], mul(AI[b], add(k.eta[b], SPsiTau)));
      Bias[B.parent] = add(Bias[B.parent], dAdInvT(k.T[b], beta));
    }
  }
  // forward recursion: updateAccelerationFD / updateAccelerationDynamic
  for (int b = 0; b < nb; b++) {
    const Body& B = w.bodies[b];
    int nd = B.ndof;
    V6<double> pa = B.parent >= 0 ? AdInvT(k.T[b], Acc[B.parent]) : zero6<double>();
    V6<double> AIpa = mul(AI[b], pa);
    std::vector<double> rhs(nd);
    for (int r = 0; r < nd; r++) {
      double s = 0; for (int i = 0; i < 6; i++) s += k.Sj[b](i, r) * AIpa[i];
      rhs[r] = totalForce[b][r] - s;
    }
    V6<double> acc = add(pa, k.eta[b]);
    for (int r = 0; r < nd; r++) {
      double a = 0; for (int c = 0; c < nd; c++) a += Psi[b][r * nd + c] * rhs[c];
      ddq[B.dof0 + r] = a;
      for (int i = 0; i < 6; i++) acc[i] += k.Sj[b](i, r) * a;
    }
    Acc[b] = acc;
  }
}

//------------------------------------------------------------------------------
void invertSmall(const double* A, double* Ainv, int n) {
  // Gauss-Jordan with partial pivoting (math::inverse<ConfigSpaceT>)
  std::vector<double> M(A, A + n * n), I(n * n, 0.0);
  for (int i = 0; i < n; i++) I[i * n + i] = 1.0;
  for (int c = 0; c < n; c++) {
    int p = c;
    for (int r = c + 1; r < n; r++) if (std::fabs(M[r * n + c]) > std::fabs(M[p * n + c])) p = r;
    if (p != c) for (int j = 0; j < n; j++) { std::swap(M[c * n + j], M[p * n + j]); std::swap(I[c * n + j], I[p * n + j]); }
    double d = M[c * n + c];
    for (int j = 0; j < n; j++) { M[c * n + j] /= d; I[c * n + j] /= d; }
    for (int r = 0; r < n; r++) {
      if (r == c) continue;
      double f = M[r * n + c];
      if (f == 0) continue;
      for (int j = 0; j < n; j++) { M[r * n + j] -= f * M[c * n + j]; I[r * n + j] -= f * I[c * n + j]; }
    }
  }
  std::memcpy(Ainv, I.data(), sizeof(double) * n * n);
}

//------------------------------------------------------------------------------
void World::massMatrix(const Kin<double>& k, double* M) const {
  // Skeleton::updateMassMatrix (Skeleton.cpp:12110): column-wise inverse
  // dynamics with unit accelerations, no velocity or gravity terms.
  std::vector<double> e(n, 0.0), col(n);
  for (int c = 0; c < n; c++) {
    std::fill(e.begin(), e.end(), 0.0);
    e[c] = 1.0;
    inverseDynamics<double>(*this, k, e.data(), false, false, col.data());
    for (int r = 0; r < n; r++) M[r * n + c] = col[r];
  }
  // symmetrise exactly like the reference's lower-triangle fill
  for (int r = 0; r < n; r++)
    for (int c = r + 1; c < n; c++) M[c * n + r] = M[r * n + c];
}

void World::coriolisGravity(const Kin<double>& k, double* C) const {
  std::vector<double> z(n, 0.0);
  inverseDynamics<double>(*this, k, z.data(), true, true, C);
}

//------------------------------------------------------------------------------
// Position integration.  World::integratePositions (World.cpp:300) with
// mParallelVelocityAndPositionUpdates: p_{t+1} = integrate(p_t, v_t).
void World::integratePositionsExplicit(const double* q, const double* v, double dtt, double* out) const {
  for (int b = 0; b < nb; b++) {
    const Body& B = bodies[b];
    int o = B.dof0;
    if (B.jtype == NIMBLE_JOINT_REVOLUTE || B.jtype == NIMBLE_JOINT_PRISMATIC) {
      out[o] = q[o] + v[o] * dtt;  // math::integratePosition<R1Space>
    } else if (B.jtype == NIMBLE_JOINT_FREE) {
      // FreeJoint::integratePositionsExplicit (FreeJoint.cpp:920), identity-J:
      // convertToPositions(convertToTransform(q) * convertToTransform(v*dt))
      V3<double> w{{q[o], q[o + 1], q[o + 2]}};
      M3<double> R = expMapRot(w);
      V3<double> wd{{v[o] * dtt, v[o + 1] * dtt, v[o + 2] * dtt}};
      M3<double> Rd = expMapRot(wd);
      V3<double> ld{{v[o + 3] * dtt, v[o + 4] * dtt, v[o + 5] * dtt}};
      M3<double> Rn = mul(R, Rd);
      V3<double> pn = add(mul(R, ld), V3<double>{{q[o + 3], q[o + 4], q[o + 5]}});
      V3<double> lg = logMap(Rn);
      for (int i = 0; i < 3; i++) { out[o + i] = lg[i]; out[o + 3 + i] = pn[i]; }
    } else if (B.jtype == NIMBLE_JOINT_BALL) {
      // BallJoint::integratePositionsExplicit (BallJoint.cpp:333), identity-J:
      // convertToPositions(convertToRotation(q) * convertToRotation(dq * dt))
      V3<double> w{{q[o], q[o + 1], q[o + 2]}};
      V3<double> wd{{v[o] * dtt, v[o + 1] * dtt, v[o + 2] * dtt}};
      V3<double> lg = logMap(mul(expMapRot(w), expMapRot(wd)));
      for (int i = 0; i < 3; i++) out[o + i] = lg[i];
    } else if (B.jtype == NIMBLE_JOINT_TRANSLATIONAL) {
      for (int i = 0; i < 3; i++) out[o + i] = q[o + i] + v[o + i] * dtt;  // integratePosition<R3Space>
    }
  }
}

// Skeleton::getPosPosJac / getVelPosJac (Skeleton.cpp:9291, :9310):
// identity / dt*identity for the Euclidean joints (R1 / R3 spaces: revolute,
// prismatic, translational), central finite differences for the FreeJoint
// (FreeJoint.cpp:965 EPS=1e-6, :987 EPS=1e-7) and the BallJoint
// (BallJoint.cpp:368 EPS=1e-6, :390 EPS=1e-7).
void World::posPosJac(const double* q, const double* v, double* J) const {
  std::fill(J, J + n * n, 0.0);
  for (int b = 0; b < nb; b++) {
    const Body& B = bodies[b];
    int o = B.dof0;
    if (B.jtype == NIMBLE_JOINT_FREE) freeJointFD(q + o, v + o, true, J, o);
    else if (B.jtype == NIMBLE_JOINT_BALL) ballJointFD(q + o, v + o, true, J, o);
    else for (int i = 0; i < B.ndof; i++) J[(o + i) * n + o + i] = 1.0;
  }
}
void World::velPosJac(const double* q, const double* v, double* J) const {
  std::fill(J, J + n * n, 0.0);
  for (int b = 0; b < nb; b++) {
    const Body& B = bodies[b];
    int o = B.dof0;
    if (B.jtype == NIMBLE_JOINT_FREE) freeJointFD(q + o, v + o, false, J, o);
    else if (B.jtype == NIMBLE_JOINT_BALL) ballJointFD(q + o, v + o, false, J, o);
    else for (int i = 0; i < B.ndof; i++) J[(o + i) * n + o + i] = dt;
  }
}
//------------------------------------------------------------------------------
// The FreeJoint finite-difference blocks (FreeJoint.cpp:965 eps 1e-6, :987 eps
// 1e-7) difference two position integrations 2 eps apart, so their last bits
// are the block's leading digits.  Both restatements evaluate those
// integrations as the same fixed sequence of IEEE double operations (the
// device's fd* functions in nimblephysics_amd/csrc/spatial.cuh, compiled
// without contraction; this file is built for x86-64 SSE2, which has no fused
// multiply-add): elementary functions from +, -, *, / and sqrt only
// (three-part pi/2 reduction, Taylor series for sin / cos on |r| <= pi/4, the
// arcsine series on |x| <= 1/2) and the reference's operation order
// (Geometry.cpp:539 expMapRot, :720 logMap).  The blocks then agree bit for
// bit instead of differing by two libms' rounding amplified by 1 / (2 eps).
// The step's own position integration keeps std::sin / cos / acos.
constexpr double kFdPi = 0x1.921fb54442d18p+1, kFdPio2 = 0x1.921fb54442d18p+0, kFdTwoOverPi = 0x1.45f306dc9c883p-1;
// pi / 2 = kFdP1 + kFdP2 + kFdP3, kFdP1 with 33 significant bits (k * kFdP1 exact)
constexpr double kFdP1 = 0x1.921fb54400000p+0, kFdP2 = 0x1.0b4611a626331p-34, kFdP3 = 0x1.1701b839a2520p-88;
static double fdSinK(double r) {  // |r| <= pi / 4
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
static double fdCosK(double r) {
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
static int fdReduce(double x, double& r) {
  const double k = std::floor(x * kFdTwoOverPi + 0.5);
  r = ((x - k * kFdP1) - k * kFdP2) - k * kFdP3;
  return ((int)k) & 3;
}
static double fdSin(double x) {
  double r;
  const int q = fdReduce(x, r);
  return q == 0 ? fdSinK(r) : (q == 1 ? fdCosK(r) : (q == 2 ? -fdSinK(r) : -fdCosK(r)));
}
static double fdCos(double x) {
  double r;
  const int q = fdReduce(x, r);
  return q == 0 ? fdCosK(r) : (q == 1 ? -fdSinK(r) : (q == 2 ? -fdCosK(r) : fdSinK(r)));
}
static double fdAsinK(double x) {  // |x| <= 1 / 2
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
static double fdAcos(double c) {
  if (c > 0.5) return 2.0 * fdAsinK(std::sqrt((1.0 - c) * 0.5));
  if (c < -0.5) return kFdPi - 2.0 * fdAsinK(std::sqrt((1.0 + c) * 0.5));
  return kFdPio2 - fdAsinK(c);
}
// Test switch (oracle_set_fd_libm): evaluate the same integrations with
// std::sin / cos / acos, as the reference does (Geometry.cpp:539, :720), so a
// CPU test bounds how far the fixed sequence above sits from libm at the
// reference's FD steps (tests/test_oracle_pins.py).
static bool gFdLibm = false;
static double fdS(double x) { return gFdLibm ? std::sin(x) : fdSin(x); }
static double fdC(double x) { return gFdLibm ? std::cos(x) : fdCos(x); }
static double fdA(double x) { return gFdLibm ? std::acos(x) : fdAcos(x); }
// expMapRot (Geometry.cpp:539) in the reference's order
static void fdExpMapRot(const double* q, double* R) {
  const double th = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
  const double K[9] = {0.0, -q[2], q[1], q[2], 0.0, -q[0], -q[1], q[0], 0.0};
  double K2[9];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) K2[r * 3 + c] = K[r * 3] * K[c] + K[r * 3 + 1] * K[3 + c] + K[r * 3 + 2] * K[6 + c];
  if (th < 1.0e-3) {
    for (int i = 0; i < 9; i++) R[i] = ((i % 4) == 0 ? 1.0 : 0.0) + K[i] + 0.5 * K2[i];
  } else {
    const double a = fdS(th) / th, b = (1.0 - fdC(th)) / (th * th);
    for (int i = 0; i < 9; i++) R[i] = ((i % 4) == 0 ? 1.0 : 0.0) + a * K[i] + b * K2[i];
  }
}
// logMap (Geometry.cpp:720)
static void fdLogMap(const double* R, double* o) {
  const double eps = 1e-6;
  const double th = fdA(std::fmax(std::fmin(0.5 * (R[0] + R[4] + R[8] - 1.0), 1.0), -1.0));
  if (th > kFdPi - eps) {
    const double delta = 0.5 + 0.125 * (kFdPi - th) * (kFdPi - th);
    const double s0 = th * std::sqrt(1.0 + (R[0] - 1.0) * delta);
    const double s1 = th * std::sqrt(1.0 + (R[4] - 1.0) * delta);
    const double s2 = th * std::sqrt(1.0 + (R[8] - 1.0) * delta);
    o[0] = R[7] > R[5] ? s0 : -s0;
    o[1] = R[2] > R[6] ? s1 : -s1;
    o[2] = R[3] > R[1] ? s2 : -s2;
    return;
  }
  const double alpha = th > eps ? 0.5 * th / fdS(th) : 0.5 + (1.0 / 12.0) * th * th;
  o[0] = alpha * (R[7] - R[5]);
  o[1] = alpha * (R[2] - R[6]);
  o[2] = alpha * (R[3] - R[1]);
}
// FreeJoint::integratePositionsExplicit (FreeJoint.cpp:920) for the finite-
// difference blocks: convertToPositions(Q(q) * convertToTransform(v dt))
static void fdFreeIntegrate(const double* q, const double* v, double dt, double* out) {
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

// BallJoint::finiteDifferencePosPosJacobian / VelPosJacobian (BallJoint.cpp:368,
// :390): the same central differences of its integration, which is the free
// joint's rotational half (BallJoint.cpp:333 vs FreeJoint.cpp:920) -- evaluated
// by fdFreeIntegrate with zero translation inputs, whose rotation outputs do
// not depend on them
void World::ballJointFD(const double* q3, const double* v3, bool wrtPos, double* J, int o) const {
  const double EPS = wrtPos ? 1e-6 : 1e-7;
  for (int i = 0; i < 3; i++) {
    double pq[6], pv[6], plus[6], minus[6];
    for (int j = 0; j < 6; j++) { pq[j] = j < 3 ? q3[j] : 0.0; pv[j] = j < 3 ? v3[j] : 0.0; }
    if (wrtPos) pq[i] += EPS; else pv[i] += EPS;
    fdFreeIntegrate(pq, pv, dt, plus);
    for (int j = 0; j < 3; j++) { pq[j] = q3[j]; pv[j] = v3[j]; }
    if (wrtPos) pq[i] -= EPS; else pv[i] -= EPS;
    fdFreeIntegrate(pq, pv, dt, minus);
    for (int r = 0; r < 3; r++) J[(o + r) * n + (o + i)] = (plus[r] - minus[r]) / (2 * EPS);
  }
}

void World::freeJointFD(const double* q6, const double* v6, bool wrtPos, double* J, int o) const {
  const double EPS = wrtPos ? 1e-6 : 1e-7;
  auto integ = [&](const double* qq, const double* vv, double* out) { fdFreeIntegrate(qq, vv, dt, out); };
  for (int i = 0; i < 6; i++) {
    double pq[6], pv[6], plus[6], minus[6];
    for (int j = 0; j < 6; j++) { pq[j] = q6[j]; pv[j] = v6[j]; }
    if (wrtPos) pq[i] += EPS; else pv[i] += EPS;
    integ(pq, pv, plus);
    for (int j = 0; j < 6; j++) { pq[j] = q6[j]; pv[j] = v6[j]; }
    if (wrtPos) pq[i] -= EPS; else pv[i] -= EPS;
    integ(pq, pv, minus);
    for (int r = 0; r < 6; r++) J[(o + r) * n + (o + i)] = (plus[r] - minus[r]) / (2 * EPS);
  }
}

//------------------------------------------------------------------------------
// Jacobians of the unconstrained dynamics terms by forward-mode duals.
//   dC[r*n+c]  = d C_r / d x_c   (x = q if wrtPos else v)       (getJacobianOfC)
//   dMy[r*n+c] = d (M(q) y)_r / d q_c                           (getJacobianOfM)
void World::jacobianOfC(const double* q, const double* v, bool wrtPos, double* dC) const {
  std::vector<Dual> qd(n), vd(n), z(n, Dual(0.0)), tau(n);
  for (int c = 0; c < n; c++) {
    for (int i = 0; i < n; i++) { qd[i] = Dual(q[i]); vd[i] = Dual(v[i]); }
    if (wrtPos) qd[c].d = 1.0; else vd[c].d = 1.0;
    Kin<Dual> k; k.compute(*this, qd.data(), vd.data());
    inverseDynamics<Dual>(*this, k, z.data(), true, true, tau.data());
    for (int r = 0; r < n; r++) dC[r * n + c] = tau[r].d;
  }
}
void World::jacobianOfMy(const double* q, const double* y, double* dMy) const {
  std::vector<Dual> qd(n), vd(n, Dual(0.0)), yd(n), tau(n);
  for (int i = 0; i < n; i++) yd[i] = Dual(y[i]);
  for (int c = 0; c < n; c++) {
    for (int i = 0; i < n; i++) qd[i] = Dual(q[i]);
    qd[c].d = 1.0;
    Kin<Dual> k; k.compute(*this, qd.data(), vd.data());
    inverseDynamics<Dual>(*this, k, yd.data(), false, false, tau.data());
    for (int r = 0; r < n; r++) dMy[r * n + c] = tau[r].d;
  }
}

}  // namespace oracle

extern "C" void oracle_set_fd_libm(int on) { oracle::gFdLibm = on != 0; }
