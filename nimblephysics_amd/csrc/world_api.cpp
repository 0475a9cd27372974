// C++ World / Skeleton API surface (include/nimble_world.hpp) over the C-ABI.
// Host code only: it flattens the object model into a nimble_world_desc the
// way simulation.World.desc_arrays does on the Python side (same field
// order and defaults), uploads it through nimble_world_create, and steps a
// batch of one world through nimble_forward / nimble_backward /
// nimble_jacobians on the current HIP device.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <limits>
#include <string>

#include "../../include/nimble_world.hpp"

namespace nimble_amd {

static void check(int rc, const char* what) {
  if (rc != NIMBLE_OK) throw std::runtime_error(std::string(what) + ": " + nimble_last_error());
}
static void hipCheck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

namespace dynamics {

static const double kInf = std::numeric_limits<double>::infinity();

// --- model-change propagation: every setter re-uploads the World's model ---
void Skeleton::changed() {
  if (mWorld) mWorld->touch();
}
void Joint::changed() { mSkel->changed(); }

Joint::Joint(Skeleton* skel, int type, int dofs, const Properties& p)
    : mSkel(skel), mType(type), mName(p.mName), mTp(p.mT_ParentBodyToJoint), mTc(p.mT_ChildBodyToJoint) {
  mDamping.assign(dofs, 0.0);
  mSpring.assign(dofs, 0.0);
  mRest.assign(dofs, 0.0);
  mPosLo.assign(dofs, -kInf);
  mPosHi.assign(dofs, kInf);
  mVelLo.assign(dofs, -kInf);
  mVelHi.assign(dofs, kInf);
  mForceLo.assign(dofs, -kInf);
  mForceHi.assign(dofs, kInf);
}
void Joint::setTransformFromParentBodyNode(const Isometry3& T) { mTp = T; changed(); }
void Joint::setTransformFromChildBodyNode(const Isometry3& T) { mTc = T; changed(); }
void Joint::setDampingCoefficient(std::size_t i, double d) { mDamping.at(i) = d; changed(); }
void Joint::setSpringStiffness(std::size_t i, double k) { mSpring.at(i) = k; changed(); }
void Joint::setRestPosition(std::size_t i, double q0) { mRest.at(i) = q0; changed(); }
void Joint::setPositionLowerLimit(std::size_t i, double v) { mPosLo.at(i) = v; changed(); }
void Joint::setPositionUpperLimit(std::size_t i, double v) { mPosHi.at(i) = v; changed(); }
void Joint::setVelocityLowerLimit(std::size_t i, double v) { mVelLo.at(i) = v; changed(); }
void Joint::setVelocityUpperLimit(std::size_t i, double v) { mVelHi.at(i) = v; changed(); }
void Joint::setControlForceLowerLimit(std::size_t i, double v) { mForceLo.at(i) = v; changed(); }
void Joint::setControlForceUpperLimit(std::size_t i, double v) { mForceHi.at(i) = v; changed(); }

static Vector3s normalized(const Vector3s& a) {
  const double l = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
  if (!(l > 0)) throw std::invalid_argument("setAxis: zero axis");
  return {a[0] / l, a[1] / l, a[2] / l};
}
void UniversalJoint::setAxis1(const Vector3s& axis) { mAxis = normalized(axis); changed(); }
void UniversalJoint::setAxis2(const Vector3s& axis) { mAxis2 = normalized(axis); changed(); }
void EulerJoint::setAxisOrder(AxisOrder order) { mOrder = static_cast<int>(order); changed(); }
void EulerJoint::setFlipAxisMap(const Vector3s& flip) { mFlip = flip; changed(); }
void PlanarJoint::setXYPlane() { mTrans1 = {{1, 0, 0}}; mTrans2 = {{0, 1, 0}}; mRot = {{0, 0, 1}}; changed(); }
void PlanarJoint::setYZPlane() { mTrans1 = {{0, 1, 0}}; mTrans2 = {{0, 0, 1}}; mRot = {{1, 0, 0}}; changed(); }
void PlanarJoint::setZXPlane() { mTrans1 = {{0, 0, 1}}; mTrans2 = {{1, 0, 0}}; mRot = {{0, 1, 0}}; changed(); }
// PlanarJointUniqueProperties::setArbitraryPlane: normalised, the second axis
// orthogonalised against the first, rotation about their cross product
void PlanarJoint::setArbitraryPlane(const Vector3s& transAxis1, const Vector3s& transAxis2) {
  const Vector3s t1 = normalized(transAxis1);
  Vector3s t2 = normalized(transAxis2);
  const double d = t1[0] * t2[0] + t1[1] * t2[1] + t1[2] * t2[2];
  if (std::fabs(d) > 1e-6) t2 = normalized({{t2[0] - d * t1[0], t2[1] - d * t1[1], t2[2] - d * t1[2]}});
  mTrans1 = t1;
  mTrans2 = t2;
  mRot = normalized({{t1[1] * t2[2] - t1[2] * t2[1], t1[2] * t2[0] - t1[0] * t2[2], t1[0] * t2[1] - t1[1] * t2[0]}});
  changed();
}

// The device model's 1-dof elements of a joint (as dynamics.Joint.chain in
// the Python mirror): a compound joint's elementary transforms in series,
// the first with the joint's parent transform, the last with its child
// transform, identity frames between them
struct ChainElem {
  int type;
  Vector3s axis;
  Isometry3 tp, tc;
};
struct JointChainAccess {
  static std::vector<ChainElem> chain(const Joint& j);
};
std::vector<ChainElem> JointChainAccess::chain(const Joint& j) {
  std::vector<std::pair<int, Vector3s>> el;
  const Vector3s ex{{1, 0, 0}}, ey{{0, 1, 0}}, ez{{0, 0, 1}};
  const Vector3s unit[3] = {ex, ey, ez};
  if (j.type() == kJointUniversal) {
    el = {{NIMBLE_JOINT_REVOLUTE, j.mAxis}, {NIMBLE_JOINT_REVOLUTE, j.mAxis2}};
  } else if (j.type() == kJointEuler) {
    static const int order[4][3] = {{0, 1, 2}, {2, 1, 0}, {2, 0, 1}, {0, 2, 1}};  // XYZ ZYX ZXY XZY
    for (int i = 0; i < 3; i++) {
      const Vector3s& u = unit[order[j.mOrder][i]];
      el.push_back({NIMBLE_JOINT_REVOLUTE, {{u[0] * j.mFlip[i], u[1] * j.mFlip[i], u[2] * j.mFlip[i]}}});
    }
  } else if (j.type() == kJointPlanar) {
    el = {{NIMBLE_JOINT_PRISMATIC, j.mTrans1}, {NIMBLE_JOINT_PRISMATIC, j.mTrans2}, {NIMBLE_JOINT_REVOLUTE, j.mRot}};
  } else {
    return {ChainElem{j.type(), j.mAxis, j.mTp, j.mTc}};
  }
  std::vector<ChainElem> out;
  for (std::size_t i = 0; i < el.size(); i++)
    out.push_back(ChainElem{el[i].first, el[i].second, i == 0 ? j.mTp : Isometry3::Identity(),
                            i + 1 == el.size() ? j.mTc : Isometry3::Identity()});
  return out;
}
void RevoluteJoint::setAxis(const Vector3s& axis) { mAxis = normalized(axis); changed(); }
void PrismaticJoint::setAxis(const Vector3s& axis) { mAxis = normalized(axis); changed(); }

void ShapeNode::setRelativeTransform(const Isometry3& T) {
  mT = T;
  mBody->mSkel->changed();
}

void BodyNode::setMass(double m) { mMass = m; mSkel->changed(); }
void BodyNode::setLocalCOM(const Vector3s& c) { mCom = c; mSkel->changed(); }
void BodyNode::setMomentOfInertia(double Ixx, double Iyy, double Izz, double Ixy, double Ixz, double Iyz) {
  mMoment = {Ixx, Iyy, Izz, Ixy, Ixz, Iyz};
  mSkel->changed();
}
void BodyNode::setFrictionCoeff(double f) { mFriction = f; mSkel->changed(); }
void BodyNode::setRestitutionCoeff(double r) { mRestitution = r; mSkel->changed(); }
ShapeNode* BodyNode::addShapeNode(const ShapePtr& shape, bool collision) {
  mShapes.emplace_back(new ShapeNode(this, shape, collision));
  mSkel->changed();
  return mShapes.back().get();
}

BodyNode* Skeleton::getBodyNode(const std::string& name) const {
  for (const auto& b : mBodies)
    if (b->getName() == name) return b.get();
  return nullptr;
}
void Skeleton::setMobile(bool mobile) { mMobile = mobile; changed(); }
void Skeleton::setPositions(const VectorXs& q) {
  if (q.size() != mQ.size()) throw std::invalid_argument("Skeleton::setPositions: size mismatch");
  mQ = q;
}
void Skeleton::setVelocities(const VectorXs& v) {
  if (v.size() != mV.size()) throw std::invalid_argument("Skeleton::setVelocities: size mismatch");
  mV = v;
}
// dof offsets in body order; existing dofs keep their values, new ones start at 0
void Skeleton::reindex() {
  std::size_t off = 0;
  for (auto& j : mJoints) {
    j->mDofOffset = off;
    off += j->getNumDofs();
  }
  mQ.resize(off, 0.0);
  mV.resize(off, 0.0);
  changed();
}

}  // namespace dynamics

namespace simulation {

World::~World() { release(); }

void World::release() {
  if (mHandle) nimble_world_destroy(mHandle);
  mHandle = nullptr;
  for (int k = 0; k < 5; k++) {
    if (mDev[k]) (void)hipFree(mDev[k]);
    mDev[k] = nullptr;
    mDevDoubles[k] = 0;
  }
}

std::string World::addSkeleton(const dynamics::SkeletonPtr& skel) {
  if (skel->mWorld && skel->mWorld != this) throw std::invalid_argument("skeleton already belongs to a world");
  skel->mWorld = this;
  mSkels.push_back(skel);
  mForces.resize(getNumDofs(), 0.0);
  touch();
  return skel->getName();
}

std::size_t World::getNumDofs() const {
  std::size_t n = 0;
  for (const auto& s : mSkels) n += s->getNumDofs();
  return n;
}

VectorXs World::getPositions() const {
  VectorXs q;
  for (const auto& s : mSkels) q.insert(q.end(), s->mQ.begin(), s->mQ.end());
  return q;
}
VectorXs World::getVelocities() const {
  VectorXs v;
  for (const auto& s : mSkels) v.insert(v.end(), s->mV.begin(), s->mV.end());
  return v;
}
void World::setPositions(const VectorXs& q) {
  if (q.size() != getNumDofs()) throw std::invalid_argument("World::setPositions: size mismatch");
  std::size_t c = 0;
  for (auto& s : mSkels)
    for (auto& x : s->mQ) x = q[c++];
}
void World::setVelocities(const VectorXs& v) {
  if (v.size() != getNumDofs()) throw std::invalid_argument("World::setVelocities: size mismatch");
  std::size_t c = 0;
  for (auto& s : mSkels)
    for (auto& x : s->mV) x = v[c++];
}
VectorXs World::getState() const {
  VectorXs st = getPositions();
  const VectorXs v = getVelocities();
  st.insert(st.end(), v.begin(), v.end());
  return st;
}
void World::setState(const VectorXs& state) {
  const std::size_t n = getNumDofs();
  if (state.size() != 2 * n) throw std::invalid_argument("World::setState: size mismatch");
  setPositions(VectorXs(state.begin(), state.begin() + n));
  setVelocities(VectorXs(state.begin() + n, state.end()));
}
void World::setControlForces(const VectorXs& f) {
  if (f.size() != getNumDofs()) throw std::invalid_argument("World::setControlForces: size mismatch");
  mForces = f;
}

// simulation.World.desc_arrays, field by field
const nimble_world_desc& World::describe() {
  enum { PARENT, SKEL, JTYPE, DOFOFF, MOBILE, SHAPEBODY };
  enum { TP, TC, AXIS, MASS, COM, MOMENT, FRIC, REST, DAMP, SPRING, RESTPOS, PLO, PHI, VLO, VHI, FLO, FHI, SSHAPE, ST };
  for (auto& v : mI32) v.clear();
  for (auto& v : mF64) v.clear();
  std::vector<int32_t>& shapeType = mShapeTypes;
  shapeType.clear();
  mMeshFirst.clear();
  mMeshCount.clear();
  mMeshVertices.clear();
  int bodyBase = 0, dofBase = 0, nb = 0;
  for (std::size_t si = 0; si < mSkels.size(); si++) {
    const auto& s = *mSkels[si];
    // every body's 1-dof chain (compound joints: massless frames before the
    // body itself) and the model index of the body
    std::vector<std::vector<dynamics::ChainElem>> chains;
    std::vector<int> index;
    int next = bodyBase;
    for (const auto& bp : s.mBodies) {
      chains.push_back(dynamics::JointChainAccess::chain(*bp->mJoint));
      next += (int)chains.back().size();
      index.push_back(next - 1);
    }
    for (std::size_t k = 0; k < s.mBodies.size(); k++) {
      const auto& b = *s.mBodies[k];
      const auto& j = *b.mJoint;
      int parent = -1;
      for (std::size_t q = 0; q < s.mBodies.size(); q++)
        if (s.mBodies[q].get() == b.mParent) parent = index[q];
      if (b.mParent && parent < 0) throw std::invalid_argument("describe: parent body of another skeleton");
      const auto& ch = chains[k];
      for (std::size_t e = 0; e < ch.size(); e++) {
        const bool self = e + 1 == ch.size();  // (the others: massless frames)
        mI32[PARENT].push_back(e == 0 ? parent : nb - 1);
        mI32[SKEL].push_back((int32_t)si);
        mI32[JTYPE].push_back(ch[e].type);
        mI32[DOFOFF].push_back(dofBase + (int32_t)j.mDofOffset + (int32_t)e);
        mI32[MOBILE].push_back(s.mMobile ? 1 : 0);
        mF64[TP].insert(mF64[TP].end(), ch[e].tp.m, ch[e].tp.m + 12);
        mF64[TC].insert(mF64[TC].end(), ch[e].tc.m, ch[e].tc.m + 12);
        mF64[AXIS].insert(mF64[AXIS].end(), ch[e].axis.begin(), ch[e].axis.end());
        mF64[MASS].push_back(self ? b.mMass : 0.0);
        const Vector3s zero3{{0, 0, 0}};
        const Vector3s& com = self ? b.mCom : zero3;
        mF64[COM].insert(mF64[COM].end(), com.begin(), com.end());
        for (int t = 0; t < 6; t++) mF64[MOMENT].push_back(self ? b.mMoment[t] : 0.0);
        mF64[FRIC].push_back(b.mFriction);
        mF64[REST].push_back(b.mRestitution);
        if (!self) nb++;
      }
      auto app = [&](int key, const VectorXs& v) { mF64[key].insert(mF64[key].end(), v.begin(), v.end()); };
      app(DAMP, j.mDamping); app(SPRING, j.mSpring); app(RESTPOS, j.mRest);
      app(PLO, j.mPosLo); app(PHI, j.mPosHi); app(VLO, j.mVelLo); app(VHI, j.mVelHi);
      app(FLO, j.mForceLo); app(FHI, j.mForceHi);
      for (const auto& node : b.mShapes) {
        if (!node->mCollision) continue;
        mI32[SHAPEBODY].push_back((int32_t)index[k]);
        shapeType.push_back(node->mShape->kind());
        const Vector3s& sz = node->mShape->size();
        mF64[SSHAPE].insert(mF64[SSHAPE].end(), sz.begin(), sz.end());
        mF64[ST].insert(mF64[ST].end(), node->mT.m, node->mT.m + 12);
        const auto* mesh = dynamic_cast<const dynamics::MeshShape*>(node->mShape.get());
        mMeshFirst.push_back(mesh ? (int32_t)(mMeshVertices.size() / 3) : 0);
        mMeshCount.push_back(mesh ? (int32_t)(mesh->getVertices().size() / 3) : 0);
        if (mesh) mMeshVertices.insert(mMeshVertices.end(), mesh->getVertices().begin(), mesh->getVertices().end());
      }
      nb++;
    }
    bodyBase = next;
    dofBase += (int)s.getNumDofs();
  }
  if (nb > NIMBLE_MAX_BODIES || dofBase > NIMBLE_MAX_DOFS || (int)shapeType.size() > NIMBLE_MAX_SHAPES)
    throw std::invalid_argument("describe: model too large for this path");
  std::memset(&mDesc, 0, sizeof(mDesc));
  mDesc.num_bodies = nb;
  mDesc.num_dofs = dofBase;
  mDesc.num_shapes = (int32_t)shapeType.size();
  mDesc.dt = mDt;
  for (int i = 0; i < 3; i++) mDesc.gravity[i] = mGravity[i];
  mDesc.contact_clipping_depth = mClip;
  mDesc.fallback_cfm = mCfm;
  mDesc.penetration_correction = mPenCorr ? 1 : 0;
  mDesc.parallel_pos_vel = mParallel ? 1 : 0;
  mDesc.parent = mI32[PARENT].data();
  mDesc.skeleton = mI32[SKEL].data();
  mDesc.joint_type = mI32[JTYPE].data();
  mDesc.dof_offset = mI32[DOFOFF].data();
  mDesc.skeleton_mobile = mI32[MOBILE].data();
  mDesc.T_parent_joint = mF64[TP].data();
  mDesc.T_child_joint = mF64[TC].data();
  mDesc.axis = mF64[AXIS].data();
  mDesc.mass = mF64[MASS].data();
  mDesc.com = mF64[COM].data();
  mDesc.moment = mF64[MOMENT].data();
  mDesc.friction = mF64[FRIC].data();
  mDesc.restitution = mF64[REST].data();
  mDesc.damping = mF64[DAMP].data();
  mDesc.spring = mF64[SPRING].data();
  mDesc.rest_position = mF64[RESTPOS].data();
  mDesc.pos_lower = mF64[PLO].data();
  mDesc.pos_upper = mF64[PHI].data();
  mDesc.vel_lower = mF64[VLO].data();
  mDesc.vel_upper = mF64[VHI].data();
  mDesc.force_lower = mF64[FLO].data();
  mDesc.force_upper = mF64[FHI].data();
  mDesc.shape_body = mI32[SHAPEBODY].data();
  mDesc.shape_type = mShapeTypes.data();
  mDesc.shape_size = mF64[SSHAPE].data();
  mDesc.shape_T = mF64[ST].data();
  // mesh vertices; no candidate mask (the device scans every vertex)
  mDesc.num_mesh_vertices = (int32_t)(mMeshVertices.size() / 3);
  mDesc.mesh_vertices = mMeshVertices.data();
  mDesc.shape_mesh_first = mMeshFirst.data();
  mDesc.shape_mesh_count = mMeshCount.data();
  mDesc.mesh_vertex_candidate = nullptr;
  return mDesc;
}

nimble_world_t World::handle() {
  if (mHandle && mBuiltVersion == mVersion) return mHandle;
  if (mHandle) nimble_world_destroy(mHandle);
  mHandle = nullptr;
  const nimble_world_desc& d = describe();
  check(nimble_world_create(&d, &mHandle), "nimble_world_create");
  mBuiltVersion = mVersion;
  return mHandle;
}

namespace {
using Entry = neural::WrtMassBodyNodeEntryType;
std::size_t entryDims(Entry t) {
  switch (t) {
    case Entry::INERTIA_MASS: return 1;
    case Entry::INERTIA_COM: return 3;
    case Entry::INERTIA_COM_MU: return 1;
    case Entry::INERTIA_DIAGONAL: return 3;
    case Entry::INERTIA_OFF_DIAGONAL: return 3;
    case Entry::INERTIA_FULL: return 10;
  }
  throw std::invalid_argument("tuneMass: unknown WrtMassBodyNodeEntryType");
}
// WrtMassBodyNodyEntry::get (WithRespectToMass.cpp:136)
VectorXs entryGet(const dynamics::BodyNode* b, Entry t) {
  const Vector3s c = b->getLocalCOM();
  const std::array<double, 6> I = b->getMomentOfInertia();
  switch (t) {
    case Entry::INERTIA_MASS: return {b->getMass()};
    case Entry::INERTIA_COM: return {c[0], c[1], c[2]};
    case Entry::INERTIA_COM_MU: {
      const Vector3s beta = b->getBeta();
      const int k = beta[0] != 0 ? 0 : (beta[1] != 0 ? 1 : 2);
      return {c[k] / beta[k]};
    }
    case Entry::INERTIA_DIAGONAL: return {I[0], I[1], I[2]};
    case Entry::INERTIA_OFF_DIAGONAL: return {I[3], I[4], I[5]};
    case Entry::INERTIA_FULL: return {b->getMass(), c[0], c[1], c[2], I[0], I[1], I[2], I[3], I[4], I[5]};
  }
  return {};
}
}  // namespace

void World::tuneMass(dynamics::BodyNode* node, neural::WrtMassBodyNodeEntryType type, const VectorXs& upperBound,
                     const VectorXs& lowerBound) {
  const std::size_t dims = entryDims(type);
  bool found = false;
  for (const auto& sk : mSkels)
    for (const auto& b : sk->mBodies) found = found || b.get() == node;
  if (!found) throw std::invalid_argument("tuneMass: the body node is not in this world");
  for (const auto& e : mTunedMass)
    if (e.first == node && e.second == type) throw std::invalid_argument("tuneMass: entry already registered");
  // bounds: one value per dim, or one value broadcast
  auto bound = [&](const VectorXs& v, double dflt, std::size_t k) {
    if (v.empty()) return dflt;
    if (v.size() == 1) return v[0];
    if (v.size() != dims) throw std::invalid_argument("tuneMass: bound size does not match the entry's dims");
    return v[k];
  };
  const double lo = type == Entry::INERTIA_MASS ? 0.0 : -std::numeric_limits<double>::infinity();
  mTunedMass.push_back({node, type});
  for (std::size_t k = 0; k < dims; k++) {
    mMassUpper.push_back(bound(upperBound, std::numeric_limits<double>::infinity(), k));
    mMassLower.push_back(bound(lowerBound, lo, k));
  }
}

VectorXs World::getMasses() const {
  VectorXs m;
  for (const auto& e : mTunedMass) {
    const VectorXs v = entryGet(e.first, e.second);
    m.insert(m.end(), v.begin(), v.end());
  }
  return m;
}

// WrtMassBodyNodyEntry::set (WithRespectToMass.cpp:45); an unchanged entry
// keeps the device model
void World::setMasses(const VectorXs& masses) {
  if (masses.size() != getMassDims()) throw std::invalid_argument("setMasses: size mismatch");
  std::size_t o = 0;
  for (const auto& e : mTunedMass) {
    dynamics::BodyNode* b = e.first;
    const std::size_t d = entryDims(e.second);
    const VectorXs v(masses.begin() + o, masses.begin() + o + d);
    o += d;
    if (v == entryGet(b, e.second)) continue;
    const std::array<double, 6> I = b->getMomentOfInertia();
    switch (e.second) {
      case Entry::INERTIA_MASS: b->setMass(v[0]); break;
      case Entry::INERTIA_COM: b->setLocalCOM({v[0], v[1], v[2]}); break;
      case Entry::INERTIA_COM_MU: {
        const Vector3s beta = b->getBeta();
        b->setLocalCOM({beta[0] * v[0], beta[1] * v[0], beta[2] * v[0]});
        break;
      }
      case Entry::INERTIA_DIAGONAL: b->setMomentOfInertia(v[0], v[1], v[2], I[3], I[4], I[5]); break;
      case Entry::INERTIA_OFF_DIAGONAL: b->setMomentOfInertia(I[0], I[1], I[2], v[0], v[1], v[2]); break;
      case Entry::INERTIA_FULL:
        b->setMass(v[0]);
        b->setLocalCOM({v[1], v[2], v[3]});
        b->setMomentOfInertia(v[4], v[5], v[6], v[7], v[8], v[9]);
        break;
    }
  }
}

bool World::massSelection(std::vector<double>& S) const {
  bool massOnly = true;
  for (const auto& e : mTunedMass) massOnly = massOnly && e.second == Entry::INERTIA_MASS;
  if (massOnly) return true;
  const std::vector<int> idx = massBodyIndices();
  std::size_t nb = 0;  // the device model's bodies (compound joints' massless frames included)
  for (const auto& sk : mSkels)
    for (const auto& b : sk->mBodies) nb += dynamics::JointChainAccess::chain(*b->mJoint).size();
  const std::size_t dims = getMassDims();
  S.assign(nb * 10 * dims, 0.0);
  std::size_t col = 0;
  for (std::size_t i = 0; i < mTunedMass.size(); i++) {
    const std::size_t base = 10 * (std::size_t)idx[i];
    int first = 0, count = 0;
    switch (mTunedMass[i].second) {
      case Entry::INERTIA_MASS: first = 0; count = 1; break;
      case Entry::INERTIA_COM: first = 1; count = 3; break;
      case Entry::INERTIA_DIAGONAL: first = 4; count = 3; break;
      case Entry::INERTIA_OFF_DIAGONAL: first = 7; count = 3; break;
      case Entry::INERTIA_FULL: first = 0; count = 10; break;
      case Entry::INERTIA_COM_MU: {  // d com / d mu = beta
        const Vector3s beta = mTunedMass[i].first->getBeta();
        for (int k = 0; k < 3; k++) S[(base + 1 + k) * dims + col] = beta[k];
        col++;
        continue;
      }
    }
    for (int c = 0; c < count; c++) S[(base + first + c) * dims + col++] = 1.0;
  }
  return false;
}

std::vector<int> World::massBodyIndices() const {
  std::vector<int> idx;
  for (const auto& e : mTunedMass) {
    const dynamics::BodyNode* t = e.first;
    // (the device model's index: compound joints' massless frames come
    // before their body, see describe())
    int base = 0, found = -1;
    for (const auto& sk : mSkels) {
      for (std::size_t k = 0; k < sk->mBodies.size(); k++) {
        base += (int)dynamics::JointChainAccess::chain(*sk->mBodies[k]->mJoint).size();
        if (sk->mBodies[k].get() == t) found = base - 1;
      }
    }
    idx.push_back(found);
  }
  return idx;
}

double* World::deviceBuffer(int k, std::size_t doubles) {
  if (mDevDoubles[k] < doubles) {
    if (mDev[k]) (void)hipFree(mDev[k]);
    mDev[k] = nullptr;
    hipCheck(hipMalloc(&mDev[k], (doubles ? doubles : 1) * sizeof(double)), "hipMalloc");
    mDevDoubles[k] = doubles;
  }
  return mDev[k];
}

// one World::step on the device; the snapshot is copied out when asked for
void World::runForward(std::vector<double>* snapshotOut) {
  nimble_world_t h = handle();
  const std::size_t n = getNumDofs();
  const std::size_t snapD = (std::size_t)nimble_snapshot_doubles(h), cacheD = (std::size_t)nimble_lcp_cache_doubles(h);
  if (mForces.size() != n) mForces.assign(n, 0.0);
  if (mLcpCache.size() != cacheD) {
    mLcpCache.assign(cacheD, 0.0);
    mLcpCache[0] = -1;  // no warm start yet
  }
  const VectorXs st = getState();
  double* dSt = deviceBuffer(0, 2 * n);
  double* dF = deviceBuffer(1, n);
  double* dC = deviceBuffer(2, cacheD);
  double* dN = deviceBuffer(3, 2 * n);
  double* dS = deviceBuffer(4, snapD);
  hipCheck(hipMemcpy(dSt, st.data(), 2 * n * sizeof(double), hipMemcpyHostToDevice), "hipMemcpy");
  hipCheck(hipMemcpy(dF, mForces.data(), n * sizeof(double), hipMemcpyHostToDevice), "hipMemcpy");
  hipCheck(hipMemcpy(dC, mLcpCache.data(), cacheD * sizeof(double), hipMemcpyHostToDevice), "hipMemcpy");
  check(nimble_forward(h, 1, dSt, dF, dC, dN, dS, nullptr), "nimble_forward");
  hipCheck(hipDeviceSynchronize(), "nimble_forward");
  VectorXs next(2 * n);
  hipCheck(hipMemcpy(next.data(), dN, 2 * n * sizeof(double), hipMemcpyDeviceToHost), "hipMemcpy");
  if (nimble_num_collision_pairs(h) > 0) {
    double status = 0;
    hipCheck(hipMemcpy(&status, dS + NIMBLE_SNAPSHOT_STATUS, sizeof(double), hipMemcpyDeviceToHost), "hipMemcpy");
    const int bits = (int)status;
    if (bits & (NIMBLE_STATUS_CONTACT_OVERFLOW | NIMBLE_STATUS_UNSUPPORTED_SHAPE | NIMBLE_STATUS_DROPPED_OVERFLOW))
      throw ContactCapacityError("World::step: the contact set does not fit the batched path (status " +
                                 std::to_string(bits) + ")");
  }
  if (snapshotOut) {
    snapshotOut->resize(snapD);
    hipCheck(hipMemcpy(snapshotOut->data(), dS, snapD * sizeof(double), hipMemcpyDeviceToHost), "hipMemcpy");
  }
  hipCheck(hipMemcpy(mLcpCache.data(), dC, cacheD * sizeof(double), hipMemcpyDeviceToHost), "hipMemcpy");
  setState(next);
}

void World::step(bool resetCommand) {
  runForward(nullptr);
  if (resetCommand) mForces.assign(getNumDofs(), 0.0);
}

}  // namespace simulation

namespace neural {

std::shared_ptr<BackpropSnapshot> forwardPass(const simulation::WorldPtr& world, bool idempotent) {
  auto snap = std::shared_ptr<BackpropSnapshot>(new BackpropSnapshot());
  snap->mWorld = world;
  snap->mN = world->getNumDofs();
  snap->mState = world->getState();
  snap->mForces = world->getControlForces();
  if (snap->mForces.size() != snap->mN) snap->mForces.assign(snap->mN, 0.0);
  const std::vector<double> cache = world->mLcpCache;
  world->runForward(&snap->mSnapshot);
  snap->mHandle = world->mHandle;
  snap->mVersion = world->mVersion;
  snap->mNumPairs = nimble_num_collision_pairs(world->mHandle);
  snap->mNext = world->getState();
  if (idempotent) {
    // RestorableSnapshot::restore
    world->setState(snap->mState);
    world->mLcpCache = cache;
  } else {
    // world->step(!idempotent): the commands are reset
    world->mForces.assign(snap->mN, 0.0);
  }
  return snap;
}

// the snapshot belongs to the model it was taken on
void BackpropSnapshot::checkModel(const char* what) const {
  if (mWorld->mVersion != mVersion || mWorld->mHandle != mHandle)
    throw std::runtime_error(std::string(what) + ": the world's model changed since forwardPass");
}

// uploads the step's inputs and snapshot (the World's device buffers may have
// been reused by later steps)
static void uploadStep(simulation::World& w, const VectorXs& st, const VectorXs& f, const std::vector<double>& snap,
                       double*& dSt, double*& dF, double*& dS, std::size_t n) {
  dSt = w.deviceBuffer(0, 2 * n);
  dF = w.deviceBuffer(1, n);
  dS = w.deviceBuffer(4, snap.size());
  hipCheck(hipMemcpy(dSt, st.data(), 2 * n * sizeof(double), hipMemcpyHostToDevice), "hipMemcpy");
  hipCheck(hipMemcpy(dF, f.data(), n * sizeof(double), hipMemcpyHostToDevice), "hipMemcpy");
  hipCheck(hipMemcpy(dS, snap.data(), snap.size() * sizeof(double), hipMemcpyHostToDevice), "hipMemcpy");
}

void BackpropSnapshot::backpropState(const VectorXs& nextStateLossGrad, VectorXs& stateLossGrad,
                                     VectorXs& forceLossGrad) const {
  const std::size_t n = mN;
  if (nextStateLossGrad.size() != 2 * n) throw std::invalid_argument("backpropState: gradient size mismatch");
  checkModel("backpropState");
  double *dSt, *dF, *dS;
  uploadStep(*mWorld, mState, mForces, mSnapshot, dSt, dF, dS, n);
  double* dG = mWorld->deviceBuffer(3, 2 * n);  // the next-state buffer is free here
  double* dGs = mWorld->deviceBuffer(2, 2 * n > 1 ? 3 * n : 3 * n);
  hipCheck(hipMemcpy(dG, nextStateLossGrad.data(), 2 * n * sizeof(double), hipMemcpyHostToDevice), "hipMemcpy");
  double* dGf = dGs + 2 * n;
  check(nimble_backward(mHandle, 1, dSt, dF, dS, dG, dGs, dGf, nullptr), "nimble_backward");
  hipCheck(hipDeviceSynchronize(), "nimble_backward");
  stateLossGrad.resize(2 * n);
  forceLossGrad.resize(n);
  hipCheck(hipMemcpy(stateLossGrad.data(), dGs, 2 * n * sizeof(double), hipMemcpyDeviceToHost), "hipMemcpy");
  hipCheck(hipMemcpy(forceLossGrad.data(), dGf, n * sizeof(double), hipMemcpyDeviceToHost), "hipMemcpy");
}

void BackpropSnapshot::backpropState(const VectorXs& nextStateLossGrad, VectorXs& stateLossGrad,
                                     VectorXs& forceLossGrad, VectorXs& massLossGrad) const {
  const std::size_t n = mN;
  if (nextStateLossGrad.size() != 2 * n) throw std::invalid_argument("backpropState: gradient size mismatch");
  checkModel("backpropState");
  const std::vector<int> idx = mWorld->massBodyIndices();
  std::vector<double> S;
  const bool massOnly = mWorld->massSelection(S);
  const std::size_t nb = mWorld->describe().num_bodies, params = massOnly ? 1 : 10;
  double *dSt, *dF, *dS;
  uploadStep(*mWorld, mState, mForces, mSnapshot, dSt, dF, dS, n);
  double* dG = mWorld->deviceBuffer(3, 2 * n);
  double* dGs = mWorld->deviceBuffer(2, 3 * n + nb * params);
  hipCheck(hipMemcpy(dG, nextStateLossGrad.data(), 2 * n * sizeof(double), hipMemcpyHostToDevice), "hipMemcpy");
  double* dGf = dGs + 2 * n;
  double* dGm = dGs + 3 * n;
  if (massOnly)
    check(nimble_backward_masses(mHandle, 1, dSt, dF, dS, dG, dGs, dGf, dGm, nullptr), "nimble_backward_masses");
  else
    check(nimble_backward_inertia(mHandle, 1, dSt, dF, dS, dG, dGs, dGf, dGm, nullptr), "nimble_backward_inertia");
  hipCheck(hipDeviceSynchronize(), "nimble_backward_masses");
  stateLossGrad.resize(2 * n);
  forceLossGrad.resize(n);
  std::vector<double> gm(nb * params);
  hipCheck(hipMemcpy(stateLossGrad.data(), dGs, 2 * n * sizeof(double), hipMemcpyDeviceToHost), "hipMemcpy");
  hipCheck(hipMemcpy(forceLossGrad.data(), dGf, n * sizeof(double), hipMemcpyDeviceToHost), "hipMemcpy");
  hipCheck(hipMemcpy(gm.data(), dGm, gm.size() * sizeof(double), hipMemcpyDeviceToHost), "hipMemcpy");
  const std::size_t dims = mWorld->getMassDims();
  massLossGrad.assign(dims, 0.0);
  if (massOnly) {
    for (std::size_t i = 0; i < idx.size(); i++) massLossGrad[i] = gm[idx[i]];
  } else {
    for (std::size_t r = 0; r < nb * 10; r++)
      if (gm[r] != 0.0)
        for (std::size_t c = 0; c < dims; c++) massLossGrad[c] += S[r * dims + c] * gm[r];
  }
}

// Clamping rows of the step: 0 for a model without collision pairs (its
// snapshot has no contact region), and never past the snapshot's f_c block.
int BackpropSnapshot::clampingCount() const {
  if (mNumPairs <= 0) return 0;
  if (mSnapshot.size() < (std::size_t)(NIMBLE_SNAPSHOT_FC + NIMBLE_MAX_LCP)) return 0;
  const int nc = (int)mSnapshot[NIMBLE_SNAPSHOT_NUM_CLAMPING];
  return nc < 0 ? 0 : (nc > NIMBLE_MAX_LCP ? NIMBLE_MAX_LCP : nc);
}

VectorXs BackpropSnapshot::getClampingConstraintImpulses() const {
  const int nc = clampingCount();
  if (nc <= 0) return VectorXs();
  return VectorXs(mSnapshot.begin() + NIMBLE_SNAPSHOT_FC, mSnapshot.begin() + NIMBLE_SNAPSHOT_FC + nc);
}

std::vector<double> BackpropSnapshot::getJacobianOfConstraintForce(WithRespectTo wrt) const {
  checkModel("getJacobianOfConstraintForce");
  const std::size_t n = mN;
  const int nc = clampingCount();
  if (nc <= 0) return {};
  double *dSt, *dF, *dS;
  uploadStep(*mWorld, mState, mForces, mSnapshot, dSt, dF, dS, n);
  double *dJs = nullptr, *dJf = nullptr, *dWs = nullptr;
  hipCheck(hipMalloc(&dJs, (size_t)NIMBLE_MAX_LCP * 2 * n * sizeof(double)), "hipMalloc");
  hipCheck(hipMalloc(&dJf, (size_t)NIMBLE_MAX_LCP * n * sizeof(double)), "hipMalloc");
  const int64_t wsd = nimble_jacobian_workspace_doubles(mHandle, 1);
  if (wsd > 0) hipCheck(hipMalloc(&dWs, wsd * sizeof(double)), "hipMalloc");
  const int rc = nimble_constraint_force_jacobians(mHandle, 1, dSt, dF, dS, dJs, dJf, dWs, nullptr);
  hipError_t e = hipDeviceSynchronize();
  std::vector<double> Js((size_t)NIMBLE_MAX_LCP * 2 * n), Jf((size_t)NIMBLE_MAX_LCP * n);
  if (rc == NIMBLE_OK && e == hipSuccess) {
    e = hipMemcpy(Js.data(), dJs, Js.size() * sizeof(double), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(Jf.data(), dJf, Jf.size() * sizeof(double), hipMemcpyDeviceToHost);
  }
  (void)hipFree(dJs);
  (void)hipFree(dJf);
  if (dWs) (void)hipFree(dWs);
  check(rc, "nimble_constraint_force_jacobians");
  hipCheck(e, "nimble_constraint_force_jacobians");
  std::vector<double> out((size_t)nc * n);
  for (int r = 0; r < nc; r++)
    for (std::size_t c = 0; c < n; c++)
      out[r * n + c] = wrt == WithRespectTo::FORCE ? Jf[r * n + c]
                                                    : Js[r * 2 * n + (wrt == WithRespectTo::VELOCITY ? n : 0) + c];
  return out;
}

void BackpropSnapshot::backprop(const LossGradient& next, LossGradient& prev) const {
  const std::size_t n = mN;
  VectorXs g(2 * n, 0.0), gs, gf;
  for (std::size_t i = 0; i < n && i < next.lossWrtPosition.size(); i++) g[i] = next.lossWrtPosition[i];
  for (std::size_t i = 0; i < n && i < next.lossWrtVelocity.size(); i++) g[n + i] = next.lossWrtVelocity[i];
  backpropState(g, gs, gf);
  prev.lossWrtPosition.assign(gs.begin(), gs.begin() + n);
  prev.lossWrtVelocity.assign(gs.begin() + n, gs.end());
  prev.lossWrtTorque = gf;
}

static void jacobians(const BackpropSnapshot& s, simulation::World& w, nimble_world_t h, const VectorXs& st,
                      const VectorXs& f, const std::vector<double>& snap, std::size_t n, std::vector<double>& J,
                      std::vector<double>& F) {
  double *dSt, *dF, *dS;
  uploadStep(w, st, f, snap, dSt, dF, dS, n);
  (void)s;
  double *dJ = nullptr, *dFj = nullptr, *dWs = nullptr;
  hipCheck(hipMalloc(&dJ, 4 * n * n * sizeof(double)), "hipMalloc");
  hipCheck(hipMalloc(&dFj, 2 * n * n * sizeof(double)), "hipMalloc");
  const int64_t wsd = nimble_jacobian_workspace_doubles(h, 1);
  if (wsd > 0) hipCheck(hipMalloc(&dWs, wsd * sizeof(double)), "hipMalloc");
  const int rc = nimble_jacobians(h, 1, dSt, dF, dS, dJ, dFj, dWs, nullptr);
  hipError_t e = hipDeviceSynchronize();
  J.resize(4 * n * n);
  F.resize(2 * n * n);
  if (rc == NIMBLE_OK && e == hipSuccess) {
    e = hipMemcpy(J.data(), dJ, J.size() * sizeof(double), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(F.data(), dFj, F.size() * sizeof(double), hipMemcpyDeviceToHost);
  }
  (void)hipFree(dJ);
  (void)hipFree(dFj);
  if (dWs) (void)hipFree(dWs);
  check(rc, "nimble_jacobians");
  hipCheck(e, "nimble_jacobians");
}

std::vector<double> BackpropSnapshot::getStateJacobian() const {
  std::vector<double> J, F;
  checkModel("getStateJacobian");
  jacobians(*this, *mWorld, mHandle, mState, mForces, mSnapshot, mN, J, F);
  return J;
}

std::vector<double> BackpropSnapshot::getForceJacobian() const {
  std::vector<double> J, F;
  checkModel("getForceJacobian");
  jacobians(*this, *mWorld, mHandle, mState, mForces, mSnapshot, mN, J, F);
  return F;
}

}  // namespace neural
}  // namespace nimble_amd
