/*
 * nimble_world.hpp -- C++ World / Skeleton API surface over the C-ABI.
 *
 * The reference's C++ users build worlds with dart::dynamics::Skeleton /
 * BodyNode / Joint / Shape and step them with dart::simulation::World and
 * dart::neural::forwardPass + BackpropSnapshot.  This header keeps those class
 * and method names (namespace nimble_amd instead of dart) for the part of the
 * API the differentiable timestep reads, so reference C++ code that builds a
 * world and steps it ports by changing the namespace and the vector types:
 *
 *   reference                                   here
 *   dart/dynamics/Skeleton.hpp:178 create        dynamics::Skeleton::create
 *   Skeleton.hpp:453 createJointAndBodyNodePair  same template, same return
 *   BodyNode.hpp setMass / setLocalCOM / setMomentOfInertia /
 *     setFrictionCoeff / setRestitutionCoeff     same
 *   BodyNode.hpp createShapeNodeWith<Aspects>    same (CollisionAspect tag)
 *   Joint.hpp setTransformFromParentBodyNode /
 *     setTransformFromChildBodyNode, GenericJoint damping / spring / limits,
 *     RevoluteJoint / PrismaticJoint setAxis     same
 *   dart/simulation/World.hpp create / addSkeleton / setGravity /
 *     setTimeStep / getState / setState / setControlForces / step /
 *     setPenetrationCorrectionEnabled /
 *     setParallelVelocityAndPositionUpdates      same
 *   dart/neural/NeuralUtils.hpp forwardPass      neural::forwardPass
 *   dart/neural/BackpropSnapshot.hpp backpropState / getStateJacobian /
 *     getActionJacobian                          neural::BackpropSnapshot
 *
 * Eigen is not part of this toolchain: Eigen::VectorXs becomes
 * std::vector<double>, Eigen::Vector3s std::array<double, 3>, and
 * Eigen::Isometry3s the 3x4 row-major Isometry3 below.  Stepping runs on the
 * current HIP device through include/nimble_amd.h (batch of one world; use
 * the C-ABI directly for batches).
 */
#ifndef NIMBLE_WORLD_HPP_
#define NIMBLE_WORLD_HPP_

#include <array>
#include <cstddef>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "nimble_amd.h"

namespace nimble_amd {

using VectorXs = std::vector<double>;
using Vector3s = std::array<double, 3>;

/* Eigen::Isometry3s stand-in: rotation R (row-major) and translation p. */
struct Isometry3 {
  double m[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
  static Isometry3 Identity() { return Isometry3(); }
  void setTranslation(const Vector3s& p) { m[3] = p[0]; m[7] = p[1]; m[11] = p[2]; }
  void setRotation(const double R[9]) {
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) m[4 * r + c] = R[3 * r + c];
  }
  Vector3s translation() const { return {m[3], m[7], m[11]}; }
};

/* A step whose contact set does not fit the batched path (more contacts than
 * NIMBLE_MAX_CONTACTS, a shape pair without a collider): it would differ from
 * the reference's World::step, so it throws instead. */
struct ContactCapacityError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

namespace simulation { class World; }

namespace neural {
/* dart/neural/WithRespectToMass.hpp:25: the tunable entries of a body's
 * inertia (dims 1, 3, 1, 3, 3, 10; FULL = mass, COM, Ixx Iyy Izz Ixy Ixz Iyz) */
enum class WrtMassBodyNodeEntryType {
  INERTIA_MASS,
  INERTIA_COM,
  INERTIA_COM_MU,
  INERTIA_DIAGONAL,
  INERTIA_OFF_DIAGONAL,
  INERTIA_FULL
};
/* dart/neural/WithRespectTo.hpp (the state / control spaces) */
enum class WithRespectTo { POSITION, VELOCITY, FORCE };
}  // namespace neural
namespace neural {
class BackpropSnapshot;
std::shared_ptr<BackpropSnapshot> forwardPass(const std::shared_ptr<simulation::World>& world, bool idempotent);
}  // namespace neural

namespace dynamics {

class Skeleton;
class BodyNode;

/* dart/dynamics/Shape.hpp family */
class Shape {
 public:
  virtual ~Shape() = default;
  int kind() const { return mKind; }
  const Vector3s& size() const { return mSize; }
 protected:
  Shape(int kind, Vector3s size) : mKind(kind), mSize(size) {}
  int mKind;
  Vector3s mSize;
};
class BoxShape : public Shape {
 public:
  explicit BoxShape(const Vector3s& size) : Shape(NIMBLE_SHAPE_BOX, size) {}
  Vector3s getSize() const { return mSize; }
};
class SphereShape : public Shape {
 public:
  explicit SphereShape(double radius) : Shape(NIMBLE_SHAPE_SPHERE, {radius, 0, 0}) {}
  double getRadius() const { return mSize[0]; }
};
/* radius, height: cylinder along the local z axis, caps at z = +-height/2 */
class CapsuleShape : public Shape {
 public:
  CapsuleShape(double radius, double height) : Shape(NIMBLE_SHAPE_CAPSULE, {radius, height, 0}) {}
  double getRadius() const { return mSize[0]; }
  double getHeight() const { return mSize[1]; }
};
/* dart/dynamics/MeshShape.hpp: collided as the convex hull of its vertex list
 * (DARTCollide.cpp:1935); vertices [3k..3k+2] in the mesh frame, in the
 * aiMesh's order, scaled by `scale` */
class MeshShape : public Shape {
 public:
  MeshShape(const Vector3s& scale, std::vector<double> vertices)
      : Shape(NIMBLE_SHAPE_MESH, scale), mVertices(std::move(vertices)) {}
  Vector3s getScale() const { return mSize; }
  const std::vector<double>& getVertices() const { return mVertices; }
 private:
  std::vector<double> mVertices;
};
using ShapePtr = std::shared_ptr<Shape>;

/* Aspect tags of BodyNode::createShapeNodeWith<...> */
struct VisualAspect {};
struct CollisionAspect {};
struct DynamicsAspect {};

class ShapeNode {
 public:
  ShapeNode(BodyNode* body, ShapePtr shape, bool collision) : mBody(body), mShape(std::move(shape)), mCollision(collision) {}
  void setRelativeTransform(const Isometry3& T);
  const Isometry3& getRelativeTransform() const { return mT; }
  const ShapePtr& getShape() const { return mShape; }
  bool hasCollisionAspect() const { return mCollision; }
 private:
  friend class simulation::World;
  BodyNode* mBody;
  ShapePtr mShape;
  bool mCollision;
  Isometry3 mT;
};

/* Host-side joint kinds beyond the C-ABI's (nimble_joint_type): products of
 * elementary axis rotations / translations, which World::describe() hands to
 * the device as the equivalent chain of 1-dof joints through massless frames
 * (the same transform as a function of q, hence the same motion subspace,
 * dynamics, Euclidean integration and posPos / velPos blocks). */
enum { kJointUniversal = 6, kJointEuler = 7, kJointPlanar = 8 };

/* dart/dynamics/Joint.hpp + GenericJoint per-dof properties */
class Joint {
 public:
  struct Properties {
    std::string mName = "joint";
    Isometry3 mT_ParentBodyToJoint, mT_ChildBodyToJoint;
  };
  virtual ~Joint() = default;
  std::size_t getNumDofs() const { return mDamping.size(); }
  const std::string& getName() const { return mName; }
  void setName(const std::string& n) { mName = n; }
  void setTransformFromParentBodyNode(const Isometry3& T);
  void setTransformFromChildBodyNode(const Isometry3& T);
  const Isometry3& getTransformFromParentBodyNode() const { return mTp; }
  const Isometry3& getTransformFromChildBodyNode() const { return mTc; }
  void setDampingCoefficient(std::size_t i, double d);
  void setSpringStiffness(std::size_t i, double k);
  void setRestPosition(std::size_t i, double q0);
  void setPositionLowerLimit(std::size_t i, double v);
  void setPositionUpperLimit(std::size_t i, double v);
  void setVelocityLowerLimit(std::size_t i, double v);
  void setVelocityUpperLimit(std::size_t i, double v);
  void setControlForceLowerLimit(std::size_t i, double v);
  void setControlForceUpperLimit(std::size_t i, double v);
  int type() const { return mType; }

 protected:
  Joint(Skeleton* skel, int type, int dofs, const Properties& p);
  void changed();
  friend struct JointChainAccess;
  friend class simulation::World;
  friend class Skeleton;
  Skeleton* mSkel;
  int mType;
  std::string mName;
  Isometry3 mTp, mTc;
  Vector3s mAxis{{1, 0, 0}};
  /* UniversalJoint's second axis; EulerJoint's axis order (XYZ 0, ZYX 1, ZXY
   * 2, XZY 3) and flip map; PlanarJoint's translation and rotation axes */
  Vector3s mAxis2{{0, 1, 0}};
  int mOrder = 0;
  Vector3s mFlip{{1, 1, 1}};
  Vector3s mTrans1{{1, 0, 0}}, mTrans2{{0, 1, 0}}, mRot{{0, 0, 1}};
  VectorXs mDamping, mSpring, mRest, mPosLo, mPosHi, mVelLo, mVelHi, mForceLo, mForceHi;
  std::size_t mDofOffset = 0;
};
class WeldJoint : public Joint {
 public:
  using Properties = Joint::Properties;
  WeldJoint(Skeleton* s, const Properties& p) : Joint(s, NIMBLE_JOINT_WELD, 0, p) {}
};
class FreeJoint : public Joint {
 public:
  using Properties = Joint::Properties;
  FreeJoint(Skeleton* s, const Properties& p) : Joint(s, NIMBLE_JOINT_FREE, 6, p) {}
};
/* BallJoint (BallJoint.cpp: exponential coordinates, identity Jacobian) and
 * TranslationalJoint (TranslationalJoint.cpp: R3 offset), 3 dofs each */
class BallJoint : public Joint {
 public:
  using Properties = Joint::Properties;
  BallJoint(Skeleton* s, const Properties& p) : Joint(s, NIMBLE_JOINT_BALL, 3, p) {}
};
class TranslationalJoint : public Joint {
 public:
  using Properties = Joint::Properties;
  TranslationalJoint(Skeleton* s, const Properties& p) : Joint(s, NIMBLE_JOINT_TRANSLATIONAL, 3, p) {}
};
/* UniversalJoint.cpp:193 T_pj AngleAxis(q0, axis1) AngleAxis(q1, axis2)
 * T_cj^-1 (UniversalJointAspect defaults: axes x, y; normalised) */
class UniversalJoint : public Joint {
 public:
  using Properties = Joint::Properties;
  UniversalJoint(Skeleton* s, const Properties& p) : Joint(s, kJointUniversal, 2, p) {}
  void setAxis1(const Vector3s& axis);
  void setAxis2(const Vector3s& axis);
  Vector3s getAxis1() const { return mAxis; }
  Vector3s getAxis2() const { return mAxis2; }
};
/* EulerJoint.cpp:1333 T_pj euler_<order>(q .* flip) T_cj^-1 (Geometry.cpp
 * eulerXYZToMatrix = Rx Ry Rz, ZYX = Rz Ry Rx, ZXY = Rz Rx Ry, XZY = Rx Rz Ry) */
class EulerJoint : public Joint {
 public:
  using Properties = Joint::Properties;
  enum class AxisOrder { XYZ = 0, ZYX = 1, ZXY = 2, XZY = 3 };
  EulerJoint(Skeleton* s, const Properties& p) : Joint(s, kJointEuler, 3, p) {}
  void setAxisOrder(AxisOrder order);
  AxisOrder getAxisOrder() const { return static_cast<AxisOrder>(mOrder); }
  void setFlipAxisMap(const Vector3s& flip);
};
/* PlanarJoint.cpp:296 T_pj Trans(t1 q0) Trans(t2 q1) expAngular(r q2) T_cj^-1
 * (PlanarJointAspect.cpp:88: the XY plane by default) */
class PlanarJoint : public Joint {
 public:
  using Properties = Joint::Properties;
  PlanarJoint(Skeleton* s, const Properties& p) : Joint(s, kJointPlanar, 3, p) {}
  void setXYPlane();
  void setYZPlane();
  void setZXPlane();
  void setArbitraryPlane(const Vector3s& transAxis1, const Vector3s& transAxis2);
};
/* RevoluteJoint / PrismaticJoint::setAxis normalise the axis */
class RevoluteJoint : public Joint {
 public:
  using Properties = Joint::Properties;
  RevoluteJoint(Skeleton* s, const Properties& p) : Joint(s, NIMBLE_JOINT_REVOLUTE, 1, p) {}
  void setAxis(const Vector3s& axis);
  Vector3s getAxis() const { return mAxis; }
};
class PrismaticJoint : public Joint {
 public:
  using Properties = Joint::Properties;
  PrismaticJoint(Skeleton* s, const Properties& p) : Joint(s, NIMBLE_JOINT_PRISMATIC, 1, p) {}
  void setAxis(const Vector3s& axis);
  Vector3s getAxis() const { return mAxis; }
};

/* dart/dynamics/BodyNode.hpp; defaults: mass 1, COM 0, unit moment of
 * inertia (Inertia.hpp:68), friction 1, restitution 0 (BodyNodeAspect.hpp:47) */
class BodyNode {
 public:
  struct Properties {
    std::string mName = "body";
  };
  BodyNode(Skeleton* skel, BodyNode* parent, Joint* joint, const Properties& p)
      : mSkel(skel), mParent(parent), mJoint(joint), mName(p.mName) {}
  const std::string& getName() const { return mName; }
  Joint* getParentJoint() const { return mJoint; }
  BodyNode* getParentBodyNode() const { return mParent; }
  Skeleton* getSkeleton() const { return mSkel; }
  void setMass(double m);
  double getMass() const { return mMass; }
  void setLocalCOM(const Vector3s& c);
  Vector3s getLocalCOM() const { return mCom; }
  void setMomentOfInertia(double Ixx, double Iyy, double Izz, double Ixy = 0, double Ixz = 0, double Iyz = 0);
  /* Ixx Iyy Izz Ixy Ixz Iyz */
  std::array<double, 6> getMomentOfInertia() const { return mMoment; }
  /* BodyNode::setBeta (BodyNode.cpp:652): the COM direction INERTIA_COM_MU scales */
  void setBeta(const Vector3s& beta) { mBeta = beta; }
  Vector3s getBeta() const { return mBeta; }
  void setFrictionCoeff(double f);
  double getFrictionCoeff() const { return mFriction; }
  void setRestitutionCoeff(double r);
  double getRestitutionCoeff() const { return mRestitution; }
  template <class... Aspects>
  ShapeNode* createShapeNodeWith(const ShapePtr& shape) {
    const bool collision = (std::is_same<Aspects, CollisionAspect>::value || ...);
    return addShapeNode(shape, collision);
  }
  std::size_t getNumShapeNodes() const { return mShapes.size(); }
  ShapeNode* getShapeNode(std::size_t i) const { return mShapes.at(i).get(); }

 private:
  ShapeNode* addShapeNode(const ShapePtr& shape, bool collision);
  friend class simulation::World;
  friend class ShapeNode;
  Skeleton* mSkel;
  BodyNode* mParent;
  Joint* mJoint;
  std::string mName;
  double mMass = 1.0;
  Vector3s mCom{{0, 0, 0}};
  std::array<double, 6> mMoment{{1, 1, 1, 0, 0, 0}};  // Ixx Iyy Izz Ixy Ixz Iyz
  double mFriction = 1.0, mRestitution = 0.0;
  Vector3s mBeta{{1, 1, 1}};
  std::vector<std::unique_ptr<ShapeNode>> mShapes;
};

class Skeleton {
 public:
  static std::shared_ptr<Skeleton> create(const std::string& name = "Skeleton") {
    return std::shared_ptr<Skeleton>(new Skeleton(name));
  }
  /* Skeleton.hpp:453: bodies are appended in creation order; a parent must
   * exist before its children (DART tree order for a depth-first build) */
  template <class JointType, class NodeType = BodyNode>
  std::pair<JointType*, NodeType*> createJointAndBodyNodePair(
      BodyNode* parent = nullptr, const typename JointType::Properties& jointProperties = typename JointType::Properties(),
      const typename NodeType::Properties& bodyProperties = typename NodeType::Properties()) {
    auto* j = new JointType(this, jointProperties);
    auto* b = new NodeType(this, parent, j, bodyProperties);
    mJoints.emplace_back(j);
    mBodies.emplace_back(b);
    reindex();
    return {j, b};
  }
  const std::string& getName() const { return mName; }
  std::size_t getNumDofs() const { return mQ.size(); }
  std::size_t getNumBodyNodes() const { return mBodies.size(); }
  BodyNode* getBodyNode(std::size_t i) const { return mBodies.at(i).get(); }
  BodyNode* getBodyNode(const std::string& name) const;
  Joint* getJoint(std::size_t i) const { return mJoints.at(i).get(); }
  BodyNode* getRootBodyNode() const { return mBodies.empty() ? nullptr : mBodies[0].get(); }
  void setMobile(bool mobile);
  bool isMobile() const { return mMobile; }
  VectorXs getPositions() const { return mQ; }
  VectorXs getVelocities() const { return mV; }
  void setPositions(const VectorXs& q);
  void setVelocities(const VectorXs& v);
  void setPosition(std::size_t i, double q) { mQ.at(i) = q; }
  void setVelocity(std::size_t i, double v) { mV.at(i) = v; }
  double getPosition(std::size_t i) const { return mQ.at(i); }

 private:
  explicit Skeleton(std::string name) : mName(std::move(name)) {}
  void reindex();
  void changed();
  friend class Joint;
  friend class BodyNode;
  friend class ShapeNode;
  friend class simulation::World;
  std::string mName;
  std::vector<std::unique_ptr<Joint>> mJoints;
  std::vector<std::unique_ptr<BodyNode>> mBodies;
  VectorXs mQ, mV;
  bool mMobile = true;
  simulation::World* mWorld = nullptr;
};
using SkeletonPtr = std::shared_ptr<Skeleton>;

}  // namespace dynamics

namespace simulation {

/* dart/simulation/World.hpp; defaults as World.cpp:70-90: gravity
 * (0, 0, -9.81), dt 0.001, contact clipping depth 0.03, fallback CFM 1e-4,
 * penetration correction off, parallel position / velocity updates on */
class World {
 public:
  static std::shared_ptr<World> create(const std::string& name = "world") {
    return std::shared_ptr<World>(new World(name));
  }
  ~World();
  World(const World&) = delete;
  World& operator=(const World&) = delete;

  std::string addSkeleton(const dynamics::SkeletonPtr& skel);
  std::size_t getNumSkeletons() const { return mSkels.size(); }
  dynamics::SkeletonPtr getSkeleton(std::size_t i) const { return mSkels.at(i); }
  std::size_t getNumDofs() const;
  void setGravity(const Vector3s& g) { mGravity = g; touch(); }
  Vector3s getGravity() const { return mGravity; }
  void setTimeStep(double dt) { mDt = dt; touch(); }
  double getTimeStep() const { return mDt; }
  void setPenetrationCorrectionEnabled(bool e) { mPenCorr = e; touch(); }
  bool getPenetrationCorrectionEnabled() const { return mPenCorr; }
  void setParallelVelocityAndPositionUpdates(bool e) { mParallel = e; touch(); }
  bool getParallelVelocityAndPositionUpdates() const { return mParallel; }
  void setFallbackConstraintForceMixingConstant(double c) { mCfm = c; touch(); }
  void setContactClippingDepth(double d) { mClip = d; touch(); }

  VectorXs getPositions() const;
  VectorXs getVelocities() const;
  void setPositions(const VectorXs& q);
  void setVelocities(const VectorXs& v);
  VectorXs getState() const;            /* positions | velocities */
  void setState(const VectorXs& state);
  void setControlForces(const VectorXs& f);
  VectorXs getControlForces() const { return mForces; }

  /* World::step (World.cpp:221): one timestep of this world on the device;
   * the control forces are cleared afterwards when resetCommand (as
   * Skeleton::resetCommands).  Throws ContactCapacityError when the step
   * could not be the reference's. */
  void step(bool resetCommand = true);

  /* World::tuneMass / getMassDims / getMasses / setMasses (World.cpp,
   * WithRespectToMass.cpp:45 set / :136 get): the registered entries, in
   * order, form the mass vector whose gradient backpropState returns
   * (lossWrtMass); a body may carry several entry types, each once. */
  void tuneMass(dynamics::BodyNode* node, neural::WrtMassBodyNodeEntryType type, const VectorXs& upperBound,
                const VectorXs& lowerBound);
  std::size_t getMassDims() const { return mMassUpper.size(); }
  VectorXs getMasses() const;
  void setMasses(const VectorXs& masses);
  VectorXs getMassUpperBound() const { return mMassUpper; }
  VectorXs getMassLowerBound() const { return mMassLower; }
  /* global body index (device model order) of each tuned entry */
  std::vector<int> massBodyIndices() const;
  /* true when every entry is INERTIA_MASS (nimble_backward_masses suffices);
   * otherwise S [num_bodies * 10][getMassDims()] row-major takes
   * nimble_backward_inertia's per-body parameters to the mass vector */
  bool massSelection(std::vector<double>& S) const;

  /* The flat description handed to nimble_world_create (storage owned by the
   * World until the next call) and the uploaded handle (rebuilt after any
   * model change). */
  const nimble_world_desc& describe();
  nimble_world_t handle();
  void touch() { mVersion++; }

 private:
  explicit World(std::string name) : mName(std::move(name)) {}
  void release();
  void runForward(std::vector<double>* snapshotOut);
  std::string mName;
  std::vector<dynamics::SkeletonPtr> mSkels;
  Vector3s mGravity{{0, 0, -9.81}};
  double mDt = 0.001, mClip = 0.03, mCfm = 1e-4;
  bool mPenCorr = false, mParallel = true;
  VectorXs mForces;
  std::vector<std::pair<dynamics::BodyNode*, neural::WrtMassBodyNodeEntryType>> mTunedMass;
  VectorXs mMassUpper, mMassLower;
  long mVersion = 0, mBuiltVersion = -1;
  nimble_world_t mHandle = nullptr;
  // describe() storage
  std::vector<int32_t> mI32[6];
  std::vector<double> mF64[20];
  std::vector<int32_t> mShapeTypes;
  std::vector<int32_t> mMeshFirst, mMeshCount;
  std::vector<double> mMeshVertices;
  nimble_world_desc mDesc{};
  // batch-of-one device buffers (state, forces, LCP cache, next state, snapshot)
  double* mDev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  std::size_t mDevDoubles[5] = {0, 0, 0, 0, 0};
  std::vector<double> mLcpCache;  // BoxedLcpConstraintSolver::mX across steps
 public:
  /* the World's batch-of-one device buffer k (grown to `doubles`) */
  double* deviceBuffer(int k, std::size_t doubles);
 private:
  friend std::shared_ptr<neural::BackpropSnapshot> neural::forwardPass(const std::shared_ptr<World>&, bool);
  friend class neural::BackpropSnapshot;
};
using WorldPtr = std::shared_ptr<World>;

}  // namespace simulation

namespace neural {

struct LossGradient {
  VectorXs lossWrtPosition, lossWrtVelocity, lossWrtTorque;
};

/* dart/neural/BackpropSnapshot.hpp: the record of one step taken by
 * forwardPass, differentiated on the device */
class BackpropSnapshot {
 public:
  /* BackpropSnapshot::backpropState (BackpropSnapshot.cpp:382): upstream
   * gradient of the next state [2n] -> gradient of the state [2n] and of the
   * control forces [n] */
  void backpropState(const VectorXs& nextStateLossGrad, VectorXs& stateLossGrad, VectorXs& forceLossGrad) const;
  /* ... and lossWrtMass [getMassDims()] = getMassVelJacobian^T dL/dv'
   * (:177, :580) for the world's tuned body masses */
  void backpropState(const VectorXs& nextStateLossGrad, VectorXs& stateLossGrad, VectorXs& forceLossGrad,
                     VectorXs& massLossGrad) const;
  /* getClampingConstraintImpulses: f_c of the step's clamping LCP rows */
  VectorXs getClampingConstraintImpulses() const;
  /* getJacobianOfConstraintForce (:2723): d f_c / d wrt, [n_c x n] row-major */
  std::vector<double> getJacobianOfConstraintForce(WithRespectTo wrt) const;
  /* BackpropSnapshot::backprop (:121) with the reference's LossGradient */
  void backprop(const LossGradient& thisTimestepLoss, LossGradient& prevTimestepLoss) const;
  /* getStateJacobian (:1230) [2n x 2n] and getControlForceJacobian-style
   * d next_state / d forces [2n x n], row-major */
  std::vector<double> getStateJacobian() const;
  std::vector<double> getForceJacobian() const;
  const VectorXs& getPreStepState() const { return mState; }
  const VectorXs& getPostStepState() const { return mNext; }

 private:
  friend std::shared_ptr<BackpropSnapshot> forwardPass(const simulation::WorldPtr& world, bool idempotent);
  void checkModel(const char* what) const;
  int clampingCount() const;
  simulation::WorldPtr mWorld;
  nimble_world_t mHandle = nullptr;
  long mVersion = 0;
  int mNumPairs = 0;  // collision pairs of the model that took the step
  std::size_t mN = 0;
  VectorXs mState, mForces, mNext;
  std::vector<double> mSnapshot;  // host copy of the device snapshot
};

/* neural::forwardPass (NeuralUtils.cpp:26): step the world and return the
 * snapshot; with idempotent the world keeps its pre-step state */
inline std::shared_ptr<BackpropSnapshot> forwardPass(const simulation::WorldPtr& world) {
  return forwardPass(world, false);
}

}  // namespace neural

namespace utils {

/* dart/utils/urdf/DartLoader.hpp parseSkeleton (DartLoader.cpp:199): one
 * Skeleton from a URDF file; joints of a link in name order (urdfdom's
 * std::map), a FreeJoint "rootJoint" above a root link not named "world",
 * box / sphere / STL mesh collision geometry (paths resolved against the
 * file's directory, package:// and file:// prefixes dropped); throws
 * std::invalid_argument for what the timestep path does not model */
class DartLoader {
 public:
  dynamics::SkeletonPtr parseSkeleton(const std::string& path);
};

/* dart/utils/SkelParser.hpp readWorld (SkelParser.cpp:402): the <world> of a
 * .skel file (time step, gravity, skeletons with box / sphere / capsule
 * collision shapes and weld / revolute / prismatic / free joints) */
struct SkelParser {
  static simulation::WorldPtr readWorld(const std::string& path);
};

}  // namespace utils
}  // namespace nimble_amd

#endif /* NIMBLE_WORLD_HPP_ */
