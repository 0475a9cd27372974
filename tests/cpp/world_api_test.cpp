// Driver for tests/test_world_api.py: builds worlds through the C++ World /
// Skeleton API (include/nimble_world.hpp) the way reference C++ code builds
// them with dart::dynamics / dart::simulation, then
//   world_api_test describe <box|pendulum>   prints the flattened
//       nimble_world_desc as JSON (no GPU needed)
//   world_api_test step <box|pendulum>       reads state [2n], forces [n] and an
//       upstream gradient [2n] from stdin, runs neural::forwardPass, then
//       BackpropSnapshot::backpropState and getStateJacobian / getForceJacobian,
//       then two World::step calls; prints JSON.
//   world_api_test describe-urdf|describe-skel <path>   loads the file with
//       utils::DartLoader::parseSkeleton / utils::SkelParser::readWorld and
//       prints {"positions": [...], "desc": {...}} (no GPU needed)
#include <cmath>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "nimble_world.hpp"

using namespace nimble_amd;

// tests/models.py box_world: a free box over a static ground box
static simulation::WorldPtr boxWorld() {
  auto world = simulation::World::create();
  world->setGravity({0, -9.81, 0});
  auto box = dynamics::Skeleton::create("box");
  auto pair = box->createJointAndBodyNodePair<dynamics::FreeJoint>();
  dynamics::BodyNode* b = pair.second;
  const double m = 1.0, sx = 0.4, sy = 0.3, sz = 0.2;
  b->setMass(m);
  b->setMomentOfInertia(m * (sy * sy + sz * sz) / 12, m * (sx * sx + sz * sz) / 12, m * (sx * sx + sy * sy) / 12);
  b->createShapeNodeWith<dynamics::VisualAspect, dynamics::CollisionAspect, dynamics::DynamicsAspect>(
      std::make_shared<dynamics::BoxShape>(Vector3s{sx, sy, sz}));
  b->setFrictionCoeff(1.0);
  world->addSkeleton(box);
  auto ground = dynamics::Skeleton::create("ground");
  auto gp = ground->createJointAndBodyNodePair<dynamics::WeldJoint>();
  Isometry3 T = Isometry3::Identity();
  T.setTranslation({0, -0.05, 0});
  gp.first->setTransformFromParentBodyNode(T);
  gp.second->createShapeNodeWith<dynamics::CollisionAspect>(std::make_shared<dynamics::BoxShape>(Vector3s{10.0, 0.1, 10.0}));
  ground->setMobile(false);
  world->addSkeleton(ground);
  return world;
}

// a damped, sprung two-link pendulum on a prismatic cart (revolute axes off
// the coordinate axes, joint offsets, COM offsets)
static simulation::WorldPtr pendulumWorld() {
  auto world = simulation::World::create();
  world->setGravity({0, -9.81, 0});
  world->setTimeStep(0.002);
  auto sk = dynamics::Skeleton::create("pendulum");
  auto cart = sk->createJointAndBodyNodePair<dynamics::PrismaticJoint>();
  cart.first->setAxis({1, 0, 0});
  cart.second->setMass(2.0);
  dynamics::BodyNode* parent = cart.second;
  for (int k = 0; k < 2; k++) {
    dynamics::RevoluteJoint::Properties jp;
    jp.mName = "hinge" + std::to_string(k);
    auto link = sk->createJointAndBodyNodePair<dynamics::RevoluteJoint>(parent, jp);
    link.first->setAxis({0.1 * k, 0.2, 1.0});
    Isometry3 Tp = Isometry3::Identity();
    Tp.setTranslation({0, k == 0 ? 0.0 : -0.5, 0});
    link.first->setTransformFromParentBodyNode(Tp);
    link.first->setDampingCoefficient(0, 0.05 * (k + 1));
    link.first->setSpringStiffness(0, 0.5);
    link.first->setRestPosition(0, 0.1);
    link.second->setMass(0.5 + k);
    link.second->setLocalCOM({0.01, -0.25, 0.0});
    link.second->setMomentOfInertia(0.02, 0.01, 0.02, 0.001, 0.0, 0.0);
    parent = link.second;
  }
  world->addSkeleton(sk);
  return world;
}

static Isometry3 tr(double x, double y, double z) {
  Isometry3 T = Isometry3::Identity();
  T.setTranslation({x, y, z});
  return T;
}
static void boxBody(dynamics::BodyNode* b, double m, double sx, double sy, double sz) {
  b->setMass(m);
  b->setMomentOfInertia(m * (sy * sy + sz * sz) / 12, m * (sx * sx + sz * sz) / 12, m * (sx * sx + sy * sy) / 12);
  b->createShapeNodeWith<dynamics::CollisionAspect>(std::make_shared<dynamics::BoxShape>(Vector3s{sx, sy, sz}));
}
static void addGround(simulation::WorldPtr& world) {
  auto ground = dynamics::Skeleton::create("ground");
  auto gp = ground->createJointAndBodyNodePair<dynamics::WeldJoint>();
  gp.first->setTransformFromParentBodyNode(tr(0, -0.05, 0));
  gp.second->createShapeNodeWith<dynamics::CollisionAspect>(std::make_shared<dynamics::BoxShape>(Vector3s{10.0, 0.1, 10.0}));
  ground->setMobile(false);
  world->addSkeleton(ground);
}

// tests/models.py ball_world: translational root, two ball joints, a revolute ankle
static simulation::WorldPtr ballWorld() {
  auto world = simulation::World::create();
  world->setGravity({0, -9.81, 0});
  auto rig = dynamics::Skeleton::create("rig");
  dynamics::Joint::Properties jp;
  dynamics::BodyNode::Properties bp;
  bp.mName = "base";
  auto base = rig->createJointAndBodyNodePair<dynamics::TranslationalJoint>(nullptr, jp, bp);
  boxBody(base.second, 2.0, 0.3, 0.2, 0.3);
  jp.mName = "hip";
  bp.mName = "leg";
  auto leg = rig->createJointAndBodyNodePair<dynamics::BallJoint>(base.second, jp, bp);
  leg.first->setTransformFromParentBodyNode(tr(0, -0.15, 0));
  leg.first->setTransformFromChildBodyNode(tr(0, 0.2, 0));
  boxBody(leg.second, 1.0, 0.1, 0.4, 0.1);
  jp.mName = "ankle";
  bp.mName = "foot";
  auto foot = rig->createJointAndBodyNodePair<dynamics::RevoluteJoint>(leg.second, jp, bp);
  foot.first->setAxis({0, 0, 1});
  foot.first->setTransformFromParentBodyNode(tr(0, -0.2, 0));
  foot.first->setTransformFromChildBodyNode(tr(0, 0.05, 0));
  boxBody(foot.second, 0.5, 0.2, 0.1, 0.3);
  jp.mName = "shoulder";
  bp.mName = "arm";
  auto arm = rig->createJointAndBodyNodePair<dynamics::BallJoint>(base.second, jp, bp);
  arm.first->setTransformFromParentBodyNode(tr(0.15, 0, 0));
  arm.first->setTransformFromChildBodyNode(tr(-0.12, 0, 0));
  boxBody(arm.second, 0.3, 0.24, 0.05, 0.05);
  world->addSkeleton(rig);
  addGround(world);
  return world;
}

// tests/models.py compound_world: planar root, universal shoulder, Euler (ZYX,
// flipped y) wrist
static simulation::WorldPtr compoundWorld() {
  auto world = simulation::World::create();
  world->setGravity({0, -9.81, 0});
  auto rig = dynamics::Skeleton::create("rig");
  dynamics::Joint::Properties jp;
  dynamics::BodyNode::Properties bp;
  bp.mName = "sled";
  auto sled = rig->createJointAndBodyNodePair<dynamics::PlanarJoint>(nullptr, jp, bp);
  sled.first->setXYPlane();
  boxBody(sled.second, 2.0, 0.4, 0.2, 0.4);
  jp.mName = "shoulder";
  bp.mName = "arm";
  auto arm = rig->createJointAndBodyNodePair<dynamics::UniversalJoint>(sled.second, jp, bp);
  arm.first->setAxis1({0, 0, 1});
  arm.first->setAxis2({1, 0, 0});
  arm.first->setTransformFromParentBodyNode(tr(0, -0.1, 0));
  arm.first->setTransformFromChildBodyNode(tr(0, 0.25, 0));
  boxBody(arm.second, 0.8, 0.1, 0.5, 0.1);
  jp.mName = "wrist";
  bp.mName = "hand";
  auto hand = rig->createJointAndBodyNodePair<dynamics::EulerJoint>(arm.second, jp, bp);
  hand.first->setAxisOrder(dynamics::EulerJoint::AxisOrder::ZYX);
  hand.first->setFlipAxisMap({1.0, -1.0, 1.0});
  hand.first->setTransformFromParentBodyNode(tr(0, -0.25, 0));
  hand.first->setTransformFromChildBodyNode(tr(0, 0.06, 0));
  boxBody(hand.second, 0.4, 0.2, 0.12, 0.2);
  world->addSkeleton(rig);
  addGround(world);
  return world;
}

static simulation::WorldPtr makeWorld(const std::string& name) {
  if (name == "box") return boxWorld();
  if (name == "pendulum") return pendulumWorld();
  if (name == "ballrig") return ballWorld();
  if (name == "compound") return compoundWorld();
  throw std::invalid_argument("unknown world " + name);
}

static void printArr(const char* key, const double* v, std::size_t n, bool comma = true) {
  std::printf("\"%s\": [", key);
  for (std::size_t i = 0; i < n; i++) std::printf("%s%.17g", i ? ", " : "", v[i]);
  std::printf("]%s", comma ? ", " : "");
}
static void printArrI(const char* key, const int32_t* v, std::size_t n, bool comma = true) {
  std::printf("\"%s\": [", key);
  for (std::size_t i = 0; i < n; i++) std::printf("%s%d", i ? ", " : "", v[i]);
  std::printf("]%s", comma ? ", " : "");
}
static void printVec(const char* key, const std::vector<double>& v, bool comma = true) {
  printArr(key, v.data(), v.size(), comma);
}

static void describe(simulation::World& w) {
  const nimble_world_desc& d = w.describe();
  const std::size_t nb = d.num_bodies, n = d.num_dofs, ns = d.num_shapes;
  std::printf("{\"num_bodies\": %d, \"num_dofs\": %d, \"num_shapes\": %d, \"dt\": %.17g, ", d.num_bodies, d.num_dofs,
              d.num_shapes, d.dt);
  printArr("gravity", d.gravity, 3);
  std::printf("\"contact_clipping_depth\": %.17g, \"fallback_cfm\": %.17g, \"penetration_correction\": %d, "
              "\"parallel_pos_vel\": %d, ", d.contact_clipping_depth, d.fallback_cfm, d.penetration_correction,
              d.parallel_pos_vel);
  printArrI("parent", d.parent, nb);
  printArrI("skeleton", d.skeleton, nb);
  printArrI("joint_type", d.joint_type, nb);
  printArrI("dof_offset", d.dof_offset, nb);
  printArrI("skeleton_mobile", d.skeleton_mobile, nb);
  printArr("T_parent_joint", d.T_parent_joint, 12 * nb);
  printArr("T_child_joint", d.T_child_joint, 12 * nb);
  printArr("axis", d.axis, 3 * nb);
  printArr("mass", d.mass, nb);
  printArr("com", d.com, 3 * nb);
  printArr("moment", d.moment, 6 * nb);
  printArr("friction", d.friction, nb);
  printArr("restitution", d.restitution, nb);
  printArr("damping", d.damping, n);
  printArr("spring", d.spring, n);
  printArr("rest_position", d.rest_position, n);
  printArr("pos_lower", d.pos_lower, n);
  printArr("pos_upper", d.pos_upper, n);
  printArr("vel_lower", d.vel_lower, n);
  printArr("vel_upper", d.vel_upper, n);
  printArr("force_lower", d.force_lower, n);
  printArr("force_upper", d.force_upper, n);
  printArrI("shape_body", d.shape_body, ns);
  printArrI("shape_type", d.shape_type, ns);
  printArr("shape_size", d.shape_size, 3 * ns);
  printArr("shape_T", d.shape_T, 12 * ns);
  printArrI("shape_mesh_first", d.shape_mesh_first, ns);
  printArrI("shape_mesh_count", d.shape_mesh_count, ns);
  printArr("mesh_vertices", d.mesh_vertices, 3 * (std::size_t)d.num_mesh_vertices);
  // no candidate mask from the C++ API (every vertex is scanned)
  printArrI("mesh_vertex_candidate", d.mesh_vertex_candidate, 0, false);
  std::printf("}\n");
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s describe|step box|pendulum | describe-urdf|describe-skel <path>\n", argv[0]);
    return 2;
  }
  try {
    const std::string mode = argv[1];
    if (mode == "describe-urdf" || mode == "describe-skel") {
      // utils::DartLoader / SkelParser: the loaded world's description plus
      // its initial positions
      simulation::WorldPtr w;
      if (mode == "describe-urdf") {
        w = simulation::World::create();
        utils::DartLoader loader;
        w->addSkeleton(loader.parseSkeleton(argv[2]));
      } else {
        w = utils::SkelParser::readWorld(argv[2]);
      }
      std::printf("{");
      printVec("positions", w->getPositions(), false);
      std::printf(", \"desc\": ");
      describe(*w);
      std::printf("}\n");
      return 0;
    }
    auto world = makeWorld(argv[2]);
    if (mode == "describe") {
      describe(*world);
      return 0;
    }
    const std::size_t n = world->getNumDofs();
    std::vector<double> st(2 * n), f(n), g(2 * n);
    for (auto& x : st) std::cin >> x;
    for (auto& x : f) std::cin >> x;
    for (auto& x : g) std::cin >> x;
    if (!std::cin) throw std::runtime_error("short input");
    world->setState(st);
    world->setControlForces(f);
    auto snap = neural::forwardPass(world, false);
    std::vector<double> gs, gf;
    snap->backpropState(g, gs, gf);
    neural::LossGradient next, prev;
    next.lossWrtPosition.assign(g.begin(), g.begin() + n);
    next.lossWrtVelocity.assign(g.begin() + n, g.end());
    snap->backprop(next, prev);
    const std::vector<double> J = snap->getStateJacobian(), F = snap->getForceJacobian();
    // lossWrtMass for the first mobile skeleton's root body (World::tuneMass)
    int tunedIndex = 0;
    for (std::size_t si = 0, base = 0; si < world->getNumSkeletons(); si++) {
      auto sk = world->getSkeleton(si);
      if (sk->isMobile()) {
        world->tuneMass(sk->getBodyNode(0), neural::WrtMassBodyNodeEntryType::INERTIA_MASS, {10.0}, {0.1});
        tunedIndex = (int)base;
        break;
      }
      base += sk->getNumBodyNodes();
    }
    std::vector<double> gs2, gf2, gm;
    snap->backpropState(g, gs2, gf2, gm);
    const std::size_t massDims = world->getMassDims();
    // then INERTIA_FULL and INERTIA_COM_MU (beta 0 1 2) on the same body:
    // lossWrtMass through nimble_backward_inertia and the entry selection
    dynamics::BodyNode* tunedBody = nullptr;
    for (std::size_t si = 0, base = 0; si < world->getNumSkeletons(); si++) {
      auto sk = world->getSkeleton(si);
      for (std::size_t k = 0; k < sk->getNumBodyNodes(); k++, base++)
        if ((int)base == tunedIndex) tunedBody = sk->getBodyNode(k);
    }
    tunedBody->setBeta({{0.0, 1.0, 2.0}});
    world->tuneMass(tunedBody, neural::WrtMassBodyNodeEntryType::INERTIA_FULL, {}, {});
    world->tuneMass(tunedBody, neural::WrtMassBodyNodeEntryType::INERTIA_COM_MU, {}, {});
    std::vector<double> gs4, gf4, gmFull;
    snap->backpropState(g, gs4, gf4, gmFull);
    const std::vector<double> massesFull = world->getMasses();
    world->setMasses(massesFull);  // unchanged values: the device model stays
    const std::vector<double> fc = snap->getClampingConstraintImpulses();
    const std::vector<double> dq = snap->getJacobianOfConstraintForce(neural::WithRespectTo::POSITION);
    const std::vector<double> dv = snap->getJacobianOfConstraintForce(neural::WithRespectTo::VELOCITY);
    const std::vector<double> dfo = snap->getJacobianOfConstraintForce(neural::WithRespectTo::FORCE);
    std::printf("{");
    printVec("grad_state_m", gs2);
    printVec("grad_mass", gm);
    printVec("grad_mass_full", gmFull);
    printVec("masses_full", massesFull);
    printVec("mass_bounds_full", world->getMassLowerBound());
    printVec("mass_dims", std::vector<double>{(double)massDims, (double)tunedIndex});
    printVec("fc", fc);
    printVec("dfc_q", dq);
    printVec("dfc_v", dv);
    printVec("dfc_f", dfo);
    printVec("next", snap->getPostStepState());
    printVec("world_state", world->getState());
    printVec("grad_state", gs);
    printVec("grad_forces", gf);
    printVec("prev_pos", prev.lossWrtPosition);
    printVec("prev_vel", prev.lossWrtVelocity);
    printVec("prev_torque", prev.lossWrtTorque);
    printVec("state_jacobian", J);
    printVec("force_jacobian", F);
    // two plain World::step calls continue the rollout (forces reset after
    // the first, as Skeleton::resetCommands)
    world->setControlForces(f);
    world->step();
    printVec("step2", world->getState());
    world->step();
    printVec("step3", world->getState());
    printVec("forces_after", world->getControlForces(), false);
    std::printf("}\n");
  } catch (const std::exception& e) {
    std::fprintf(stderr, "world_api_test: %s\n", e.what());
    return 1;
  }
  return 0;
}
