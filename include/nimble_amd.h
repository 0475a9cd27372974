/*
 * nimble_amd.h -- C-ABI boundary of the MI355X-native differentiable timestep.
 *
 * This is the drop-in boundary for the hot path that the reference exposes as
 *   python/nimblephysics/timestep.py:13  TimestepLayer (torch.autograd.Function)
 * whose forward calls
 *   dart/neural/NeuralUtils.cpp:26       neural::forwardPass(world)  -> World::step
 *   dart/simulation/World.cpp:221        World::step
 * and whose backward calls
 *   dart/neural/BackpropSnapshot.cpp:382 BackpropSnapshot::backpropState
 *   dart/neural/BackpropSnapshot.cpp:121 BackpropSnapshot::backprop
 *
 * The reference binds those through pybind11 on one World object at a time.
 * Here one call advances a whole batch of independent worlds (same model,
 * different state) that live in device memory (HBM).  All pointers passed to
 * nimble_forward / nimble_backward are DEVICE pointers; the stream is a
 * hipStream_t passed as void* so that this header needs no HIP/torch types.
 *
 * Scalar type: double everywhere (the reference's s_t is double,
 * dart/math/MathTypes.hpp:53).
 */
#ifndef NIMBLE_AMD_H_
#define NIMBLE_AMD_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Joint types (subset of the dart/dynamics Joint classes on the hot path). */
enum nimble_joint_type {
  NIMBLE_JOINT_WELD = 0,      /* dart/dynamics/WeldJoint.hpp      0 dof */
  NIMBLE_JOINT_REVOLUTE = 1,  /* dart/dynamics/RevoluteJoint.cpp  1 dof */
  NIMBLE_JOINT_PRISMATIC = 2, /* dart/dynamics/PrismaticJoint.cpp 1 dof */
  NIMBLE_JOINT_FREE = 3,      /* dart/dynamics/FreeJoint.cpp      6 dof
                                 (built with DART_USE_IDENTITY_JACOBIAN,
                                 dart/CMakeLists.txt:184) */
  NIMBLE_JOINT_BALL = 4,      /* dart/dynamics/BallJoint.cpp      3 dof: exponential
                                 coordinates, identity Jacobian (as FREE's
                                 rotational part) */
  NIMBLE_JOINT_TRANSLATIONAL = 5 /* dart/dynamics/TranslationalJoint.cpp 3 dof
                                 (R3 space: q is the joint frame's offset) */
};

/* Collision shape types (dart/collision/dart/DARTCollide.cpp:5030 collide()). */
enum nimble_shape_type {
  NIMBLE_SHAPE_BOX = 0,
  NIMBLE_SHAPE_SPHERE = 1,
  NIMBLE_SHAPE_CAPSULE = 2,   /* dart/dynamics/CapsuleShape.hpp: shape_size =
                                 (radius, height, 0), axis = local z */
  NIMBLE_SHAPE_MESH = 3       /* dart/dynamics/MeshShape.hpp: shape_size =
                                 scale; vertices in mesh_vertices (the
                                 aiScene's vertex list in order, collided as
                                 their convex hull by libccd MPR,
                                 DARTCollide.cpp:1935) */
};

#define NIMBLE_MAX_BODIES 64
#define NIMBLE_MAX_DOFS 64
#define NIMBLE_MAX_SHAPES 64
/* Max contact points per world per step and LCP rows (3 per frictional
 * contact, dart/constraint/ContactConstraint.cpp:147 mDim = 3): the layout of
 * the snapshot and the LCP cache.  The device solves LCPs of up to
 * NIMBLE_MAX_SOLVED_LCP rows: one row per lane of a 64-lane wavefront up to
 * 64 rows, two per lane above (a second kernel takes those worlds), so every
 * NIMBLE_MAX_LCP-row problem is solved; NIMBLE_STATUS_LCP_TOO_LARGE is kept
 * for the layout's sake. */
#define NIMBLE_MAX_CONTACTS 42
#define NIMBLE_MAX_LCP (3 * NIMBLE_MAX_CONTACTS)
#define NIMBLE_MAX_SOLVED_LCP 128

/*
 * Flat description of a World (all skeletons of the world concatenated in
 * World::addSkeleton order, bodies of each skeleton in DART tree order).
 * Transforms are 3x4 row-major [R | p] (12 doubles).
 */
typedef struct nimble_world_desc {
  int32_t num_bodies;
  int32_t num_dofs;
  int32_t num_shapes;
  int32_t reserved;
  double dt;                        /* World::mTimeStep (World.cpp:75)      */
  double gravity[3];                /* World::mGravity                     */
  double contact_clipping_depth;    /* World::mContactClippingDepth (0.03) */
  double fallback_cfm;              /* World::mFallbackConstraintForceMixingConstant (1e-4) */
  int32_t penetration_correction;   /* World::mPenetrationCorrectionEnabled (false) */
  int32_t parallel_pos_vel;         /* World::mParallelVelocityAndPositionUpdates (true) */

  /* per body [num_bodies] */
  const int32_t* parent;            /* parent body index, -1 for a root    */
  const int32_t* skeleton;          /* skeleton index                      */
  const int32_t* joint_type;        /* nimble_joint_type of parent joint   */
  const int32_t* dof_offset;        /* first world dof of the parent joint */
  const int32_t* skeleton_mobile;   /* 1 if the body's skeleton is mobile  */
  const double* T_parent_joint;     /* [12] Joint::mT_ParentBodyToJoint    */
  const double* T_child_joint;      /* [12] Joint::mT_ChildBodyToJoint     */
  const double* axis;               /* [3]  revolute / prismatic axis      */
  const double* mass;               /* Inertia::mMass                      */
  const double* com;                /* [3]  Inertia::mCenterOfMass         */
  const double* moment;             /* [6]  Ixx Iyy Izz Ixy Ixz Iyz        */
  const double* friction;           /* BodyNode friction coeff (1.0)       */
  const double* restitution;        /* BodyNode restitution coeff (0.0)    */

  /* per dof [num_dofs] */
  const double* damping;
  const double* spring;
  const double* rest_position;
  const double* pos_lower;
  const double* pos_upper;
  const double* vel_lower;
  const double* vel_upper;
  const double* force_lower;
  const double* force_upper;

  /* per collision shape [num_shapes] */
  const int32_t* shape_body;
  const int32_t* shape_type;        /* nimble_shape_type                   */
  const double* shape_size;         /* [3] box size; sphere (r); capsule (r, h) */
  const double* shape_T;            /* [12] ShapeNode relative transform   */

  /* mesh shapes: vertices of all meshes concatenated, shape s (type
   * NIMBLE_SHAPE_MESH) owns [shape_mesh_first[s], + shape_mesh_count[s]) */
  int32_t num_mesh_vertices;
  int32_t reserved2;
  const double* mesh_vertices;      /* [num_mesh_vertices][3], mesh frame, unscaled */
  const int32_t* shape_mesh_first;  /* [num_shapes] (unused for other types) */
  const int32_t* shape_mesh_count;  /* [num_shapes]                         */
  /* optional (NULL = all vertices): 1 for the vertices within the witness
   * plane depth (0.01, DARTCollide.cpp:58) of the mesh's convex hull
   * boundary -- the only ones that can be a support point or a witness
   * point; the device scans only these, in their original order */
  const int32_t* mesh_vertex_candidate;
} nimble_world_desc;

typedef struct nimble_world* nimble_world_t;

/* Error codes. */
#define NIMBLE_OK 0
#define NIMBLE_ERR_INVALID 1
#define NIMBLE_ERR_HIP 2
#define NIMBLE_ERR_UNSUPPORTED 3

/*
 * Upload a world description to the device.  Replaces the reference's
 * World construction + Skeleton loading (dart/simulation/World.cpp:70,
 * dart/utils/urdf/DartLoader.cpp:199) for the hot path.
 */
int nimble_world_create(const nimble_world_desc* desc, nimble_world_t* out);
int nimble_world_destroy(nimble_world_t world);

/* Number of doubles of per-world snapshot workspace (the batched
 * BackpropSnapshot, dart/neural/BackpropSnapshot.cpp:34) and of the per-world
 * LCP warm-start cache (BoxedLcpConstraintSolver::mX,
 * dart/constraint/BoxedLcpConstraintSolver.cpp:180). */
int64_t nimble_snapshot_doubles(nimble_world_t world);
int64_t nimble_lcp_cache_doubles(nimble_world_t world);

/* Candidate collision shape pairs of the model (DARTCollisionDetector::collide
 * object pairs after BodyNodeCollisionFilter, DARTCollisionDetector.cpp:127,
 * CollisionFilter.cpp:105).  0 means the model has no contact stage and its
 * snapshots carry no contact header. */
int32_t nimble_num_collision_pairs(nimble_world_t world);

/* Per-world status word, snapshot element NIMBLE_SNAPSHOT_STATUS after
 * nimble_forward (models with collision pairs).  The first three bits mean the
 * world's contact set did not fit this path and its step differs from the
 * reference's World::step; the host layer raises on them. */
#define NIMBLE_SNAPSHOT_STATUS 5
/* Number of clamping LCP rows (f_c entries) of the step, snapshot element
 * NIMBLE_SNAPSHOT_NUM_CLAMPING; the clamping impulses f_c follow at
 * NIMBLE_SNAPSHOT_FC (BackpropSnapshot::getClampingConstraintImpulses). */
#define NIMBLE_SNAPSHOT_NUM_CLAMPING 2
#define NIMBLE_SNAPSHOT_FC (16 + 13 * NIMBLE_MAX_CONTACTS + 12 * NIMBLE_MAX_LCP)
#define NIMBLE_STATUS_CONTACT_OVERFLOW 1  /* > NIMBLE_MAX_CONTACTS contacts     */
#define NIMBLE_STATUS_UNSUPPORTED_SHAPE 2 /* shape pair without a collider     */
#define NIMBLE_STATUS_DROPPED_OVERFLOW 4  /* dropped-contact dedup list full   */
#define NIMBLE_STATUS_LCP_REDUCED 8       /* LCPUtils::reduce merged duplicate
                                             columns (reference behaviour,
                                             LCPUtils.cpp:144; informational) */
#define NIMBLE_STATUS_LCP_TOO_LARGE 16    /* more than NIMBLE_MAX_SOLVED_LCP LCP
                                             rows: contacts recorded, the
                                             constraint solve not taken      */
#define NIMBLE_STATUS_PROTOCOL 64         /* a wait between the world's two
                                             waves hit the kernel's deadlock
                                             guard; the step finished on one
                                             wave (raised like the above)    */
/* The LCP solvers' executed work in the step (snapshot elements, doubles):
 * Dantzig pivots, PGS sweeps and their FLOPs, both waves of the world. */
#define NIMBLE_SNAPSHOT_PIVOTS 9
#define NIMBLE_SNAPSHOT_SWEEPS 10
#define NIMBLE_SNAPSHOT_SOLVER_FLOPS 11

/*
 * Batched differentiable forward step == neural::forwardPass + World::step
 * on each of `batch` worlds.
 *   state      [batch][2*num_dofs]  (positions | velocities), device
 *   forces     [batch][num_dofs]    control forces, device
 *   lcp_cache  [batch][lcp_cache_doubles] warm start, read + updated, device
 *   next_state [batch][2*num_dofs]  output, device
 *   snapshot   [batch][snapshot_doubles]  output, consumed by nimble_backward:
 *              contacts, LCP rows and classification (clamping / upper-bound
 *              / separating), clamping impulses f_c, pre-constraint velocity
 *              -- the per-world state of BackpropSnapshot.
 */
int nimble_forward(nimble_world_t world, int32_t batch, const double* state,
                   const double* forces, double* lcp_cache, double* next_state,
                   double* snapshot, void* stream);

/*
 * Batched analytic backward == BackpropSnapshot::backpropState on each world
 * (dart/neural/BackpropSnapshot.cpp:382), with the Jacobian-transpose products
 * of BackpropSnapshot::backprop (BackpropSnapshot.cpp:161-183) and
 * clipLossGradientsToBounds (BackpropSnapshot.cpp:425).
 *   grad_next_state [batch][2*num_dofs]  dL/d(next_state), device
 *   grad_state      [batch][2*num_dofs]  dL/d(state) output, device
 *   grad_forces     [batch][num_dofs]    dL/d(forces) output, device
 * The snapshot's contact records are read; its workspace tail (present only
 * for models whose worst-case LCP exceeds the on-chip pool) is scratch.
 */
int nimble_backward(nimble_world_t world, int32_t batch, const double* state,
                    const double* forces, double* snapshot,
                    const double* grad_next_state, double* grad_state,
                    double* grad_forces, void* stream);

/*
 * nimble_backward plus the gradient with respect to every body's mass:
 *   grad_masses [batch][num_bodies]  dL/d(mass of body b), device
 * == BackpropSnapshot::backpropState's lossWrtMass = getMassVelJacobian^T
 * dL/dv' (dart/neural/BackpropSnapshot.cpp:177, :580; getVelJacobianWrt with
 * WithRespectTo::MASS, :980) for a world whose getMassDims() entries are the
 * bodies' masses (World::tuneMass with INERTIA_MASS); the Python layer picks
 * the tuned bodies' columns (python/nimblephysics/timestep.py:34, :57
 * `mass` / lossWrtMass).
 */
int nimble_backward_masses(nimble_world_t world, int32_t batch, const double* state,
                           const double* forces, double* snapshot,
                           const double* grad_next_state, double* grad_state,
                           double* grad_forces, double* grad_masses, void* stream);

/*
 * nimble_backward plus the gradient with respect to every body's ten inertia
 * parameters, in WithRespectToMass's INERTIA_FULL order
 * (dart/neural/WithRespectToMass.cpp:35-181): mass, local COM x y z, moment
 * about the COM Ixx Iyy Izz Ixy Ixz Iyz:
 *   grad_inertia [batch][num_bodies][10]  device
 * The Python / C++ layers pick the tuned entries' components (INERTIA_MASS,
 * INERTIA_COM, INERTIA_COM_MU (beta-weighted COM), INERTIA_DIAGONAL,
 * INERTIA_OFF_DIAGONAL, INERTIA_FULL).
 */
int nimble_backward_inertia(nimble_world_t world, int32_t batch, const double* state,
                            const double* forces, double* snapshot,
                            const double* grad_next_state, double* grad_state,
                            double* grad_forces, double* grad_inertia, void* stream);

/*
 * Batched step Jacobians of a forward's snapshot, without bound clipping:
 *   state_jacobian [batch][2n][2n]  d(next_state)/d(state) ==
 *       BackpropSnapshot::getStateJacobian (dart/neural/BackpropSnapshot.cpp:1230):
 *       [[posPos, velPos], [posVel, velVel]] (:1263, :1338, :762, :643)
 *   force_jacobian [batch][2n][n]   d(next_state)/d(forces); its velocity rows
 *       are getControlForceVelJacobian (:482), the columns of the action
 *       space give getActionJacobian (:1245)
 * Both are formed as 2n vector-Jacobian products per world (unit upstream
 * gradients through the backward kernel), so they are exactly the matrices
 * whose transposed products nimble_backward applies.
 *   workspace  device buffer of nimble_jacobian_workspace_doubles(world,
 *              batch) doubles (NULL when that is 0)
 */
int64_t nimble_jacobian_workspace_doubles(nimble_world_t world, int32_t batch);
int nimble_jacobians(nimble_world_t world, int32_t batch, const double* state,
                     const double* forces, const double* snapshot,
                     double* state_jacobian, double* force_jacobian,
                     double* workspace, void* stream);

/*
 * Batched Jacobians of the clamping constraint impulses f_c (the snapshot's
 * clamping rows, in the LCP's clamping order) of a forward's snapshot ==
 * BackpropSnapshot::getJacobianOfConstraintForce (dart/neural/
 * BackpropSnapshot.cpp:2723) for WithRespectTo POSITION / VELOCITY / FORCE:
 *   dfc_dstate  [batch][NIMBLE_MAX_LCP][2n]  row r: d f_c[r] / d(q, v)
 *   dfc_dforces [batch][NIMBLE_MAX_LCP][n]   row r: d f_c[r] / d tau
 * rows r >= n_c (the world's clamping count, snapshot element
 * NIMBLE_SNAPSHOT_NUM_CLAMPING) are zero.  Formed as vector-Jacobian products
 * with unit upstream gradients on f_c through the backward kernel.
 *   workspace  as for nimble_jacobians (nimble_jacobian_workspace_doubles)
 */
int nimble_constraint_force_jacobians(nimble_world_t world, int32_t batch, const double* state,
                                      const double* forces, const double* snapshot,
                                      double* dfc_dstate, double* dfc_dforces,
                                      double* workspace, void* stream);

/* Last error message (thread-local). */
const char* nimble_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* NIMBLE_AMD_H_ */
