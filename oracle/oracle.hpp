// ORACLE / TEST INFRASTRUCTURE ONLY -- see nimble_oracle.cpp header.
#pragma once
#include <vector>

#include "../include/nimble_amd.h"
#include "spatial.hpp"

namespace oracle {

struct Body {
  int parent, skel, jtype, dof0, ndof;
  bool mobile;
  Iso<double> Tpj, Tcj;
  double axis[3];
  M6<double> G;  // spatial inertia in body frame
  double friction, restitution;
};

struct Shape {
  int body, type;
  double size[3];
  Iso<double> T;
  // NIMBLE_SHAPE_MESH: the aiMesh vertex list (float values as the reference
  // reads them), mesh frame, unscaled (size = scale)
  std::vector<double> verts;  // [count][3]
};

struct World;

template <class S>
struct Kin {
  std::vector<Iso<S>> T, Tw;   // relative (parent->child) and world transforms
  std::vector<M6<S>> Sj;       // joint Jacobian columns (child frame)
  std::vector<V6<S>> V, eta;   // body velocity and partial acceleration
  void compute(const World& w, const S* q, const S* dq);
};

// One contact point as produced by the collision detector
// (dart/collision/Contact.hpp).  normal points from B into A.
// Sphere-box contacts (types 4 SPHERE_BOX / 5 BOX_SPHERE, the reference's
// ContactType numbering) also carry the sphere centre and the box faces the
// centre was clamped against (Contact::faceNLocked / faceNNormal).
// pipe-mesh contact types of the capsule-box branches (this package's
// numbering; the reference's PIPE_VERTEX 16 / VERTEX_PIPE 18 / PIPE_EDGE 17 /
// EDGE_PIPE 19, dart/collision/Contact.hpp:76)
enum { CT_PIPE_VERTEX = 10, CT_VERTEX_PIPE = 11, CT_PIPE_EDGE = 12, CT_EDGE_PIPE = 13, CT_SPHERE_EDGE = 14,
       CT_EDGE_SPHERE = 15 };

struct Contact {
  int shapeA, shapeB, bodyA, bodyB;
  double point[3], normal[3], depth;
  int type;
  double sphereCenter[3];
  int faceLocked[3];
  double faceNormal[9];
  // EDGE_EDGE metadata (collision::Contact::edgeAFixedPoint / edgeADir /
  // edgeBFixedPoint / edgeBDir, set by dBoxBox, DARTCollide.cpp:1046, :1334)
  double edgeAFixed[3], edgeADir[3], edgeBFixed[3], edgeBDir[3];
  // SPHERE_SPHERE metadata (collision::Contact::centerA / radiusA / centerB /
  // radiusB, DARTCollide.cpp:1866); centerA is sphereCenter
  double centerB[3], radiusA, radiusB;
  // SPHERE_PIPE / PIPE_SPHERE metadata (pipeClosestPoint / pipeFixedPoint /
  // pipeDir / sphereRadius / pipeRadius, DARTCollide.cpp:4330, :4398);
  // the sphere centre is sphereCenter
  double pipeClosest[3], pipeFixed[3], pipeDir[3], sphereRadius, pipeRadius;
  // PIPE_PIPE: edgeA/B fixed point and direction above, plus the closest
  // points (edgeAClosestPoint / edgeBClosestPoint, DARTCollide.cpp:4270);
  // radiusA / radiusB hold the normalised radii there, as in the reference
  double edgeAClosest[3], edgeBClosest[3];
};

// Everything BackpropSnapshot needs (dart/neural/BackpropSnapshot.hpp and
// ConstrainedGroupGradientMatrices.hpp).
struct Snapshot {
  std::vector<double> q, v, tau, preConstraintV, postQ, postV;
  // constraint data (empty when no contact)
  int numRows = 0;
  std::vector<Contact> contacts;
  std::vector<int> rowContact, rowDirIdx;  // per LCP row
  std::vector<double> rowDir;              // per LCP row, world direction for body A (3)
  std::vector<double> freeAcc;             // unconstrained ddq (Minv (tau - C - D v - K ..))
  std::vector<double> Aall;      // n x rows, column j = J^T e_j (getConstraintForces)
  std::vector<double> massedImpulse;  // n x rows, column j = Minv J^T e_j
  std::vector<double> lcpA, lcpB, lcpLo, lcpHi, lcpX;
  std::vector<int> lcpFIndex;
  std::vector<double> aColNorms;
  std::vector<int> mapping;      // per row: CLAMPING=-1 .. see ConstraintMapping
  std::vector<int> clampingIndex, upperBoundIndex;
  int numClamping = 0, numUpperBound = 0;
  std::vector<double> fc;        // clamping impulses
  std::vector<double> bounceDiag, restitutionDiag, penetrationVel;
  std::vector<double> E;         // numUpperBound x numClamping
  double cfm = 0.0;
  bool ignoredFriction = false;
  bool shortCircuit = false;
  bool lcpReduced = false;  // LCPUtils::reduce merged columns on a fallback solve
  int unsupportedContacts = 0;   // a narrow-phase branch not restated was hit
};

struct World {
  int nb = 0, n = 0;
  double dt = 0.001, g[3] = {0, 0, 0};
  double clipDepth = 0.03, fallbackCfm = 1e-4;
  bool penetrationCorrection = false, parallelPosVel = true;
  std::vector<Body> bodies;
  std::vector<Shape> shapes;
  std::vector<int> dofBody;
  std::vector<double> damping, spring, restPos, posLo, posHi, velLo, velHi, forceLo, forceHi;

  explicit World(const nimble_world_desc* d);

  void massMatrix(const Kin<double>& k, double* M) const;
  void coriolisGravity(const Kin<double>& k, double* C) const;
  void integratePositionsExplicit(const double* q, const double* v, double dtt, double* out) const;
  void posPosJac(const double* q, const double* v, double* J) const;
  void velPosJac(const double* q, const double* v, double* J) const;
  void freeJointFD(const double* q6, const double* v6, bool wrtPos, double* J, int o) const;
  void ballJointFD(const double* q3, const double* v3, bool wrtPos, double* J, int o) const;
  void jacobianOfC(const double* q, const double* v, bool wrtPos, double* dC) const;
  void jacobianOfMy(const double* q, const double* y, double* dMy) const;

  // ancestry helpers
  bool isAncestorOrSelf(int anc, int b) const {
    while (b >= 0) { if (b == anc) return true; b = bodies[b].parent; }
    return false;
  }
};

void forwardDynamicsABA(const World& w, const Kin<double>& k, const double* q, const double* dq,
                        const double* tauCtrl, double* ddq);
void invertSmall(const double* A, double* Ainv, int n);
template <class S>
void inverseDynamics(const World& w, const Kin<S>& k, const S* ddq, bool withGravity, bool withVel, S* tau);

// timestep (oracle_step.cpp)
void step(const World& w, const double* state, const double* tau, std::vector<double>& lcpCache,
          double* nextState, Snapshot& snap);
void backprop(const World& w, const Snapshot& snap, const double* gradNext, double* gradState, double* gradTau);
void stepJacobians(const World& w, const Snapshot& snap, double* posPos, double* posVel, double* velPos,
                   double* velVel, double* forceVel, std::vector<double>* dFcOut = nullptr);

// contacts (oracle_contact.cpp)
// *unsupported (optional) is set when a narrow-phase branch that is not
// restated was hit (its contacts are dropped).
void collide(const World& w, const Kin<double>& k, std::vector<Contact>& out, int* unsupported = nullptr);
int capsuleBox(const Iso<double>& Tb, const double* size, const Iso<double>& Tc, double r, double h, bool boxFirst,
               double clip, int shape1, int shape2, int body1, int body2, std::vector<Contact>& out,
               int* unsupported);

// mesh (vertices, scale, transform Tm) vs box (size, Tb): collideMeshBox
// (DARTCollide.cpp:3935) when meshFirst, else collideBoxMesh (:3983)
int meshBox(const Iso<double>& Tm, const Shape& mesh, const Iso<double>& Tb, const double* size, bool meshFirst,
            double clip, int shape1, int shape2, int body1, int body2, std::vector<Contact>& out, int* unsupported);

// standalone sphere shapes: collideSphereBox (DARTCollide.cpp:1655) /
// collideBoxSphere (:1482, halfspace BOTH) and collideSphereSphere (:1812)
int sphereBoxPair(const Iso<double>& Tb, const double* size, const double* c0, double r, bool boxFirst, double clip,
                  int shape1, int shape2, int body1, int body2, std::vector<Contact>& out);
int sphereSphere(const double* c0, double r0, const double* c1, double r1, double clip, int shape1, int shape2,
                 int body1, int body2, std::vector<Contact>& out);

// collideSphereCapsule (:4286) / collideCapsuleSphere (:4354, capsule first)
int sphereCapsule(const double* c0, double rs, const Iso<double>& Tc, double rc, double h, bool sphereFirst,
                  double clip, int shape1, int shape2, int body1, int body2, std::vector<Contact>& out);

// collideCapsuleCapsule (:4183)
int capsuleCapsule(const Iso<double>& T0, double r0, double h0, const Iso<double>& T1, double r1, double h1,
                   double clip, int shape1, int shape2, int body1, int body2, std::vector<Contact>& out);

// Replay of another solver path (test infrastructure): when set for the
// calling thread, solveContacts takes this final LCP solution and path (the
// gradient short-circuit flag, the fallback CFM, friction removed) instead of
// running the short-circuit classification and the Dantzig / PGS cascade, and
// then classifies, standardises, applies impulses and records the snapshot
// exactly as after its own solve.  Used to check a world whose ill-posed LCP
// the GPU solved along another (equally valid) path: every quantity after
// the solve is then compared on the GPU's path.
struct ForcedLcp {
  int m = -1;  // rows the forced x has (must equal the step's rows)
  const double* x = nullptr;
  bool shortCircuit = false, ignoredFriction = false;
  double cfm = 0.0;
  bool mismatch = false;  // set when the step's row count differed
};
extern thread_local ForcedLcp* tForcedLcp;

// dense helpers
void cholSolve(const double* A, const double* b, double* x, int n);
void pinvSolve(const double* A, const double* b, double* x, int n, double* pinvOut = nullptr);

}  // namespace oracle
