"""Host-side model description mirroring the reference's dart.dynamics API.

The reference builds skeletons through C++ classes bound with pybind11
(dart/dynamics/Skeleton.hpp, BodyNode.hpp, RevoluteJoint.hpp, ...; Python
bindings under python/_nimblephysics/dynamics/).  Only what the differentiable
timestep reads is mirrored here: the kinematic tree, joint transforms and axes,
inertia, joint damping/spring/limits, collision shapes and contact
coefficients.  The numbers are flattened into a ``nimble_world_desc``
(include/nimble_amd.h) by ``simulation.World``.

Defaults follow the reference:
  * Inertia: mass 1, COM 0, moment identity    (dart/dynamics/Inertia.hpp:68)
  * friction 1.0, restitution 0.0              (detail/BodyNodeAspect.hpp:47)
  * joint limits +-inf, damping/spring 0       (detail/GenericJointAspect.hpp)
"""
from __future__ import annotations

import math
from typing import List, Optional

import numpy as np

INF = float("inf")

JOINT_WELD = 0
JOINT_REVOLUTE = 1
JOINT_PRISMATIC = 2
JOINT_FREE = 3
JOINT_BALL = 4           # BallJoint.cpp: exponential coordinates, identity Jacobian
JOINT_TRANSLATIONAL = 5  # TranslationalJoint.cpp: R3 offset
# Multi-dof joints whose relative transform is a product of elementary axis
# rotations / translations with constant axes: the device model steps each as
# the equivalent chain of 1-dof joints through massless frames (Joint.chain),
# which has the same transform, motion subspace (velocities are the
# coordinate rates, GenericJoint), Euclidean integration and identity posPos /
# velPos blocks as the reference's joint
JOINT_UNIVERSAL = 6  # UniversalJoint.cpp:193: T_pj R(axis1, q0) R(axis2, q1) T_cj^-1
JOINT_EULER = 7      # EulerJoint.cpp:1333, :242: T_pj euler_<order>(q * flip) T_cj^-1
JOINT_PLANAR = 8     # PlanarJoint.cpp:296: T_pj Trans(t1 q0) Trans(t2 q1) R(r, q2) T_cj^-1
COMPOUND_JOINTS = (JOINT_UNIVERSAL, JOINT_EULER, JOINT_PLANAR)
_EULER_AXES = {"XYZ": (0, 1, 2), "ZYX": (2, 1, 0), "ZXY": (2, 0, 1), "XZY": (0, 2, 1)}  # Geometry.cpp:1767 ff.

SHAPE_BOX = 0
SHAPE_SPHERE = 1
SHAPE_CAPSULE = 2
SHAPE_MESH = 3


def _model_changed(skel: Optional["Skeleton"]) -> None:
    """A model parameter changed: the owning World re-uploads its device model
    before the next step (the reference's setters take effect on the next
    World::step, so the device copy must never go stale)."""
    if skel is not None and skel.world is not None:
        skel.world._touch()


def _iso(R=None, p=None) -> np.ndarray:
    T = np.eye(4)
    if R is not None:
        T[:3, :3] = np.asarray(R, dtype=np.float64)
    if p is not None:
        T[:3, 3] = np.asarray(p, dtype=np.float64)
    return T


class Isometry3:
    """Minimal stand-in for dart.math.Isometry3 (4x4 homogeneous transform)."""

    def __init__(self, matrix: Optional[np.ndarray] = None):
        self.m = np.eye(4) if matrix is None else np.array(matrix, dtype=np.float64)

    def set_translation(self, p):
        self.m[:3, 3] = np.asarray(p, dtype=np.float64)

    def set_rotation(self, R):
        self.m[:3, :3] = np.asarray(R, dtype=np.float64)

    def translation(self):
        return self.m[:3, 3].copy()

    def rotation(self):
        return self.m[:3, :3].copy()

    def matrix(self):
        return self.m.copy()


def _as_matrix(T) -> np.ndarray:
    if isinstance(T, Isometry3):
        return T.m.copy()
    return np.array(T, dtype=np.float64)


class Shape:
    def __init__(self, kind: int, size):
        self.kind = kind
        self.size = np.zeros(3)
        s = np.atleast_1d(np.asarray(size, dtype=np.float64))
        self.size[: len(s)] = s


class BoxShape(Shape):
    """dart/dynamics/BoxShape.hpp"""

    def __init__(self, size):
        super().__init__(SHAPE_BOX, size)

    def getSize(self):
        return self.size.copy()


class SphereShape(Shape):
    """dart/dynamics/SphereShape.hpp"""

    def __init__(self, radius: float):
        super().__init__(SHAPE_SPHERE, [radius, 0, 0])

    def getRadius(self):
        return float(self.size[0])


class CapsuleShape(Shape):
    """dart/dynamics/CapsuleShape.hpp: radius, height (cylinder length along
    the local z axis, hemispherical caps at z = +-height/2)."""

    def __init__(self, radius: float, height: float):
        super().__init__(SHAPE_CAPSULE, [radius, height, 0])

    def getRadius(self):
        return float(self.size[0])

    def getHeight(self):
        return float(self.size[1])


class MeshShape(Shape):
    """dart/dynamics/MeshShape.hpp: a triangle mesh collided as the convex
    hull of its vertex list (DARTCollide.cpp:1935).  ``vertices`` [N, 3] are
    the aiMesh vertices in order (see mesh.py), ``scale`` the per-axis scale
    (Shape size)."""

    def __init__(self, scale, vertices, path: str = ""):
        super().__init__(SHAPE_MESH, scale)
        self.vertices = np.ascontiguousarray(np.asarray(vertices, dtype=np.float64).reshape(-1, 3))
        self.path = path
        self._candidate = None

    def getScale(self):
        return self.size.copy()

    def getMeshPath(self):
        return self.path

    def candidate(self):
        """Per-vertex mask of possible support / witness points (mesh.py)."""
        # keyed on the scale: the mask depends on it (a stale one would drop
        # vertices that became support / witness points)
        size = np.asarray(self.size, dtype=np.float64)
        if self._candidate is None or not np.array_equal(getattr(self, "_candidate_size", None), size):
            from .mesh import candidate_mask
            self._candidate = candidate_mask(self.vertices, size)
            self._candidate_size = size.copy()
        return self._candidate


class ShapeNode:
    def __init__(self, body: "BodyNode", shape: Shape, collision: bool):
        self.body = body
        self.shape = shape
        self.T = np.eye(4)
        self.collision = collision
        self.visual = True

    def setRelativeTransform(self, T):
        self.T = _as_matrix(T)
        _model_changed(self.body.skel)

    def getShape(self):
        return self.shape

    def createCollisionAspect(self):
        self.collision = True
        _model_changed(self.body.skel)

    def createVisualAspect(self):
        self.visual = True
        return _VisualAspect()

    def getVisualAspect(self):
        return _VisualAspect()


class _VisualAspect:
    def setColor(self, *_):
        pass

    def setCastShadows(self, *_):
        pass


class Joint:
    def __init__(self, skel: "Skeleton", kind: int, name: str):
        self.skel = skel
        self.kind = kind
        self.name = name
        self.T_parent = np.eye(4)
        self.T_child = np.eye(4)
        self.axis = np.array([1.0, 0.0, 0.0]) if kind == JOINT_REVOLUTE else np.array([1.0, 0.0, 0.0])
        n = self.getNumDofs()
        self.damping = np.zeros(n)
        self.spring = np.zeros(n)
        self.rest = np.zeros(n)
        self.pos_lo = np.full(n, -INF)
        self.pos_hi = np.full(n, INF)
        self.vel_lo = np.full(n, -INF)
        self.vel_hi = np.full(n, INF)
        self.force_lo = np.full(n, -INF)
        self.force_hi = np.full(n, INF)
        self.initial_positions = np.zeros(n)
        self.dof_offset = 0
        self.axis1, self.axis2 = np.array([1.0, 0.0, 0.0]), np.array([0.0, 1.0, 0.0])
        self.axis_order, self.flip = "XYZ", np.ones(3)
        self.trans1, self.trans2, self.rot = np.array([1.0, 0, 0]), np.array([0, 1.0, 0]), np.array([0, 0, 1.0])

    def getNumDofs(self) -> int:
        return {JOINT_WELD: 0, JOINT_REVOLUTE: 1, JOINT_PRISMATIC: 1, JOINT_FREE: 6, JOINT_BALL: 3,
                JOINT_TRANSLATIONAL: 3, JOINT_UNIVERSAL: 2, JOINT_EULER: 3, JOINT_PLANAR: 3}[self.kind]

    # --- UniversalJoint / EulerJoint / PlanarJoint properties (defaults as
    # UniversalJointAspect: axes x, y; EulerJointAspect: XYZ, no flips;
    # PlanarJointAspect: the XY plane) and their 1-dof chains
    def setAxis1(self, axis):
        a = np.asarray(axis, dtype=np.float64)
        self.axis1 = a / np.linalg.norm(a)
        _model_changed(self.skel)

    def setAxis2(self, axis):
        a = np.asarray(axis, dtype=np.float64)
        self.axis2 = a / np.linalg.norm(a)
        _model_changed(self.skel)

    def getAxis1(self):
        return self.axis1.copy()

    def getAxis2(self):
        return self.axis2.copy()

    def setAxisOrder(self, order):
        order = getattr(order, "name", order)
        if order not in _EULER_AXES:
            raise ValueError(f"EulerJoint axis order {order!r}")
        self.axis_order = order
        _model_changed(self.skel)

    def getAxisOrder(self):
        return self.axis_order

    def setFlipAxisMap(self, flip):
        self.flip = np.asarray(flip, dtype=np.float64).reshape(3).copy()
        _model_changed(self.skel)

    def _set_plane(self, t1, t2, r):
        self.trans1, self.trans2, self.rot = (np.asarray(v, dtype=np.float64) for v in (t1, t2, r))
        _model_changed(self.skel)

    def setXYPlane(self):  # PlanarJointAspect.cpp:88
        self._set_plane([1, 0, 0], [0, 1, 0], [0, 0, 1])

    def setYZPlane(self):
        self._set_plane([0, 1, 0], [0, 0, 1], [1, 0, 0])

    def setZXPlane(self):
        self._set_plane([0, 0, 1], [1, 0, 0], [0, 1, 0])

    def setArbitraryPlane(self, transAxis1, transAxis2):
        """PlanarJointUniqueProperties::setArbitraryPlane: normalised, the
        second axis orthogonalised against the first, rotation about their
        cross product."""
        t1 = np.asarray(transAxis1, dtype=np.float64)
        t1 = t1 / np.linalg.norm(t1)
        t2 = np.asarray(transAxis2, dtype=np.float64)
        t2 = t2 / np.linalg.norm(t2)
        d = float(t1 @ t2)
        if abs(d) > 1e-6:
            t2 = t2 - d * t1
            t2 = t2 / np.linalg.norm(t2)
        r = np.cross(t1, t2)
        self._set_plane(t1, t2, r / np.linalg.norm(r))

    def chain(self):
        """The joint as 1-dof joints in series, [(kind, axis, T_parent,
        T_child)]: the first takes the joint's parent transform, the last its
        child transform, the frames between are the identity (the product of
        the elementary transforms is the reference's relative transform)."""
        if self.kind == JOINT_UNIVERSAL:
            elems = [(JOINT_REVOLUTE, self.axis1), (JOINT_REVOLUTE, self.axis2)]
        elif self.kind == JOINT_EULER:
            elems = [(JOINT_REVOLUTE, np.eye(3)[a] * self.flip[i]) for i, a in enumerate(_EULER_AXES[self.axis_order])]
        elif self.kind == JOINT_PLANAR:
            elems = [(JOINT_PRISMATIC, self.trans1), (JOINT_PRISMATIC, self.trans2), (JOINT_REVOLUTE, self.rot)]
        else:
            return [(self.kind, self.axis, self.T_parent, self.T_child)]
        out = []
        for i, (k, a) in enumerate(elems):
            out.append((k, np.asarray(a, dtype=np.float64), self.T_parent if i == 0 else np.eye(4),
                        self.T_child if i == len(elems) - 1 else np.eye(4)))
        return out

    def getName(self):
        return self.name

    def setName(self, name):
        self.name = name

    # RevoluteJoint::setAxis / PrismaticJoint::setAxis normalise the axis
    def setAxis(self, axis):
        a = np.asarray(axis, dtype=np.float64)
        self.axis = a / np.linalg.norm(a)
        _model_changed(self.skel)

    def getAxis(self):
        return self.axis.copy()

    def setTransformFromParentBodyNode(self, T):
        self.T_parent = _as_matrix(T)
        _model_changed(self.skel)

    def setTransformFromChildBodyNode(self, T):
        self.T_child = _as_matrix(T)
        _model_changed(self.skel)

    def setDampingCoefficient(self, i, d):
        self.damping[i] = d
        _model_changed(self.skel)

    def setSpringStiffness(self, i, k):
        self.spring[i] = k
        _model_changed(self.skel)

    def setRestPosition(self, i, q0):
        self.rest[i] = q0
        _model_changed(self.skel)

    def setPositionUpperLimit(self, i, v):
        self.pos_hi[i] = v
        _model_changed(self.skel)

    def setPositionLowerLimit(self, i, v):
        self.pos_lo[i] = v
        _model_changed(self.skel)

    def setVelocityUpperLimit(self, i, v):
        self.vel_hi[i] = v
        _model_changed(self.skel)

    def setVelocityLowerLimit(self, i, v):
        self.vel_lo[i] = v
        _model_changed(self.skel)

    def setControlForceUpperLimit(self, i, v):
        self.force_hi[i] = v
        _model_changed(self.skel)

    def setControlForceLowerLimit(self, i, v):
        self.force_lo[i] = v
        _model_changed(self.skel)


class BodyNode:
    def __init__(self, skel: "Skeleton", name: str, parent: Optional["BodyNode"], joint: Joint):
        self.skel = skel
        self.name = name
        self.parent = parent
        self.joint = joint
        self.mass = 1.0
        self.com = np.zeros(3)
        self.moment = np.array([1.0, 1.0, 1.0, 0.0, 0.0, 0.0])  # Ixx Iyy Izz Ixy Ixz Iyz
        self.friction = 1.0
        self.restitution = 0.0
        self.shape_nodes: List[ShapeNode] = []
        self.index = 0

    def getName(self):
        return self.name

    def getParentJoint(self):
        return self.joint

    def getParentBodyNode(self):
        return self.parent

    def setMass(self, m):
        self.mass = float(m)
        _model_changed(self.skel)

    def getMass(self):
        return self.mass

    def setBeta(self, beta):
        """BodyNode::setBeta (BodyNode.cpp:652): the COM direction that
        INERTIA_COM_MU scales."""
        self.beta = np.asarray(beta, dtype=np.float64).copy()
        _model_changed(self.skel)

    def getBeta(self):
        return getattr(self, "beta", np.ones(3)).copy()

    def getLocalCOM(self):
        return self.com.copy()

    def setLocalCOM(self, c):
        self.com = np.asarray(c, dtype=np.float64).copy()
        _model_changed(self.skel)

    def setMomentOfInertia(self, Ixx, Iyy, Izz, Ixy=0.0, Ixz=0.0, Iyz=0.0):
        self.moment = np.array([Ixx, Iyy, Izz, Ixy, Ixz, Iyz], dtype=np.float64)
        _model_changed(self.skel)

    def setFrictionCoeff(self, f):
        self.friction = float(f)
        _model_changed(self.skel)

    def setRestitutionCoeff(self, r):
        self.restitution = float(r)
        _model_changed(self.skel)

    def createShapeNode(self, shape: Shape, collision: bool = False):
        node = ShapeNode(self, shape, collision)
        self.shape_nodes.append(node)
        _model_changed(self.skel)
        return node

    def getShapeNode(self, i):
        return self.shape_nodes[i]

    def getNumShapeNodes(self):
        return len(self.shape_nodes)


class Skeleton:
    """Subset of dart/dynamics/Skeleton.hpp used by the timestep."""

    def __init__(self, name: str = "skeleton"):
        self.name = name
        self.bodies: List[BodyNode] = []
        self.mobile = True
        self.world = None
        self._q = np.zeros(0)
        self._v = np.zeros(0)

    # --- construction -------------------------------------------------------
    def _create(self, kind, parent, joint_name=None, body_name=None):
        j = Joint(self, kind, joint_name or f"joint_{len(self.bodies)}")
        b = BodyNode(self, body_name or f"body_{len(self.bodies)}", parent, j)
        b.index = len(self.bodies)
        self.bodies.append(b)
        self._reindex()
        _model_changed(self)
        return j, b

    def createRevoluteJointAndBodyNodePair(self, parent=None, joint_name=None, body_name=None):
        return self._create(JOINT_REVOLUTE, parent, joint_name, body_name)

    def createPrismaticJointAndBodyNodePair(self, parent=None, joint_name=None, body_name=None):
        return self._create(JOINT_PRISMATIC, parent, joint_name, body_name)

    def createFreeJointAndBodyNodePair(self, parent=None, joint_name=None, body_name=None):
        return self._create(JOINT_FREE, parent, joint_name, body_name)

    def createBallJointAndBodyNodePair(self, parent=None, joint_name=None, body_name=None):
        return self._create(JOINT_BALL, parent, joint_name, body_name)

    def createTranslationalJointAndBodyNodePair(self, parent=None, joint_name=None, body_name=None):
        return self._create(JOINT_TRANSLATIONAL, parent, joint_name, body_name)

    def createUniversalJointAndBodyNodePair(self, parent=None, joint_name=None, body_name=None):
        return self._create(JOINT_UNIVERSAL, parent, joint_name, body_name)

    def createEulerJointAndBodyNodePair(self, parent=None, joint_name=None, body_name=None):
        return self._create(JOINT_EULER, parent, joint_name, body_name)

    def createPlanarJointAndBodyNodePair(self, parent=None, joint_name=None, body_name=None):
        return self._create(JOINT_PLANAR, parent, joint_name, body_name)

    def createWeldJointAndBodyNodePair(self, parent=None, joint_name=None, body_name=None):
        return self._create(JOINT_WELD, parent, joint_name, body_name)

    def _reindex(self):
        off = 0
        for b in self.bodies:
            b.joint.dof_offset = off
            off += b.joint.getNumDofs()
        n = off
        q = np.zeros(n)
        v = np.zeros(n)
        m = min(n, len(self._q))
        q[:m] = self._q[:m]
        v[:m] = self._v[:m]
        # new dofs start at the joint's initial position
        for b in self.bodies:
            j = b.joint
            for k in range(j.getNumDofs()):
                if j.dof_offset + k >= m:
                    q[j.dof_offset + k] = j.initial_positions[k]
        self._q, self._v = q, v

    # --- queries --------------------------------------------------------------
    def getName(self):
        return self.name

    def getNumDofs(self) -> int:
        return sum(b.joint.getNumDofs() for b in self.bodies)

    def getNumBodyNodes(self):
        return len(self.bodies)

    def getBodyNode(self, key):
        if isinstance(key, int):
            return self.bodies[key]
        for b in self.bodies:
            if b.name == key:
                return b
        raise KeyError(key)

    def getJoint(self, key):
        if isinstance(key, int):
            return self.bodies[key].joint
        for b in self.bodies:
            if b.joint.name == key:
                return b.joint
        raise KeyError(key)

    def getRootBodyNode(self):
        return self.bodies[0]

    def setMobile(self, mobile: bool):
        self.mobile = bool(mobile)
        _model_changed(self)

    def isMobile(self):
        return self.mobile

    # --- state ------------------------------------------------------------------
    def getPositions(self):
        return self._q.copy()

    def setPositions(self, q):
        self._q = np.asarray(q, dtype=np.float64).copy()

    def getVelocities(self):
        return self._v.copy()

    def setVelocities(self, v):
        self._v = np.asarray(v, dtype=np.float64).copy()

    def setPosition(self, i, x):
        self._q[i] = x

    def getPosition(self, i):
        return float(self._q[i])

    def setVelocity(self, i, x):
        self._v[i] = x

    def _per_dof(self, attr):
        out = []
        for b in self.bodies:
            out.extend(list(getattr(b.joint, attr)))
        return np.array(out, dtype=np.float64)

    def getPositionLowerLimits(self):
        return self._per_dof("pos_lo")

    def getPositionUpperLimits(self):
        return self._per_dof("pos_hi")

    def _set_per_dof(self, attr, lim):
        lim = np.asarray(lim, dtype=np.float64)
        if lim.shape != (self.getNumDofs(),):
            raise ValueError(f"{attr}: expected {self.getNumDofs()} values, got shape {lim.shape}")
        for b in self.bodies:
            j = b.joint
            getattr(j, attr)[:] = lim[j.dof_offset:j.dof_offset + j.getNumDofs()]
        _model_changed(self)

    # Skeleton::setControlForceUpperLimits / ... (dart/dynamics/MetaSkeleton.cpp):
    # per-dof limits in the skeleton's dof order
    def setControlForceUpperLimits(self, lim):
        self._set_per_dof("force_hi", lim)

    def setControlForceLowerLimits(self, lim):
        self._set_per_dof("force_lo", lim)

    def setPositionUpperLimits(self, lim):
        self._set_per_dof("pos_hi", lim)

    def setPositionLowerLimits(self, lim):
        self._set_per_dof("pos_lo", lim)

    def setVelocityUpperLimits(self, lim):
        self._set_per_dof("vel_hi", lim)

    def setVelocityLowerLimits(self, lim):
        self._set_per_dof("vel_lo", lim)

    def getControlForceUpperLimits(self):
        return self._per_dof("force_hi")

    def getControlForceLowerLimits(self):
        return self._per_dof("force_lo")

    def getVelocityUpperLimits(self):
        return self._per_dof("vel_hi")

    def getVelocityLowerLimits(self):
        return self._per_dof("vel_lo")


def rpy_to_matrix(rpy) -> np.ndarray:
    """URDF fixed-axis roll/pitch/yaw -> rotation (Rz(yaw) Ry(pitch) Rx(roll))."""
    r, p, y = [float(x) for x in rpy]
    cr, sr, cp, sp, cy, sy = math.cos(r), math.sin(r), math.cos(p), math.sin(p), math.cos(y), math.sin(y)
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx
