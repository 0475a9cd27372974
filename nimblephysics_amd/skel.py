"""Minimal .skel reader (the subset the benchmark worlds use).

Mirrors dart/utils/SkelParser.cpp: ``readWorld`` (:402; <physics> time step and
gravity), ``readSkeleton`` (:940; skeleton frame, <mobile>, bodies keyed by
name, joints created in file order with parents first :1000-1050),
``readBodyNode`` (:1075; <transformation> as xyz + eulerXYZ angles composed
with the skeleton frame, <inertia> mass / moment_of_inertia / offset),
``readJoint`` (:1538; T_ParentBodyToJoint = parentWorld^-1 childWorld
childToJoint, T_ChildBodyToJoint = childToJoint), revolute / prismatic axes
and ``readJointDynamicsAndLimit`` (:1870; damping, spring stiffness, rest
position, position limits -- which the reference leaves un-enforced:
Joint::mIsPositionLimitEnforced defaults to false) and collision shapes
(box, sphere, capsule).  The collision detector named in <physics> is
ignored: the reference falls back to the DART detector when the requested one
is not built (:717-733), and only the DART detector is built.
"""
from __future__ import annotations

import math
import xml.etree.ElementTree as ET
from typing import Dict

import numpy as np

from . import dynamics as dyn


def _vec(text):
    return np.array([float(x) for x in text.split()], dtype=np.float64)


def euler_xyz_to_matrix(a) -> np.ndarray:
    """dart/math/Geometry.cpp:1767 eulerXYZToMatrix (R = Rx Ry Rz)."""
    cx, sx = math.cos(a[0]), math.sin(a[0])
    cy, sy = math.cos(a[1]), math.sin(a[1])
    cz, sz = math.cos(a[2]), math.sin(a[2])
    R = np.empty((3, 3))
    R[0, 0] = cy * cz
    R[1, 0] = cx * sz + cz * sx * sy
    R[2, 0] = sx * sz - cx * cz * sy
    R[0, 1] = -cy * sz
    R[1, 1] = cx * cz - sx * sy * sz
    R[2, 1] = cz * sx + cx * sy * sz
    R[0, 2] = sy
    R[1, 2] = -cy * sx
    R[2, 2] = cx * cy
    return R


def _iso(text) -> np.ndarray:
    """XmlHelpers.cpp toIsometry3s: "x y z rx ry rz" -> [eulerXYZ(r) | p]."""
    e = _vec(text)
    T = np.eye(4)
    T[:3, :3] = euler_xyz_to_matrix(e[3:6])
    T[:3, 3] = e[:3]
    return T


def _read_shape(el) -> dyn.Shape:
    geom = el.find("geometry")
    if geom.find("box") is not None:
        return dyn.BoxShape(_vec(geom.find("box/size").text))
    if geom.find("sphere") is not None:
        return dyn.SphereShape(float(geom.find("sphere/radius").text))
    if geom.find("capsule") is not None:
        c = geom.find("capsule")
        return dyn.CapsuleShape(float(c.find("radius").text), float(c.find("height").text))
    raise NotImplementedError(f"skel shape {[g.tag for g in geom]} is not on the timestep hot path")


def read_skeleton(sk_el) -> dyn.Skeleton:
    skel = dyn.Skeleton(sk_el.get("name", "skeleton"))
    frame = _iso(sk_el.find("transformation").text) if sk_el.find("transformation") is not None else np.eye(4)
    mob = sk_el.find("mobile")
    if mob is not None:
        skel.setMobile(mob.text.strip().lower() in ("true", "1"))
    bodies: Dict[str, dict] = {}
    for b in sk_el.findall("body"):
        name = b.get("name")
        T = frame @ _iso(b.find("transformation").text) if b.find("transformation") is not None else frame.copy()
        rec = {"init": T, "mass": 1.0, "com": np.zeros(3), "moment": None, "shapes": []}
        inert = b.find("inertia")
        if inert is not None:
            rec["mass"] = float(inert.find("mass").text)
            moi = inert.find("moment_of_inertia")
            if moi is not None:
                rec["moment"] = [float(moi.find(k).text) for k in ("ixx", "iyy", "izz", "ixy", "ixz", "iyz")]
            if inert.find("offset") is not None:
                rec["com"] = _vec(inert.find("offset").text)
        for cs in b.findall("collision_shape"):
            shape = _read_shape(cs)
            Ts = _iso(cs.find("transformation").text) if cs.find("transformation") is not None else np.eye(4)
            rec["shapes"].append((shape, Ts))
        bodies.setdefault(name, rec)
    joints = []
    for j in sk_el.findall("joint"):
        parent = j.find("parent").text.strip()
        child = j.find("child").text.strip()
        joints.append((j, None if parent == "world" else parent, child))
    created: Dict[str, dyn.BodyNode] = {}
    pending = list(joints)
    kinds = {"weld": dyn.JOINT_WELD, "revolute": dyn.JOINT_REVOLUTE, "prismatic": dyn.JOINT_PRISMATIC,
             "free": dyn.JOINT_FREE, "ball": dyn.JOINT_BALL, "translational": dyn.JOINT_TRANSLATIONAL}

    def create(jel, parent, child):
        jt = jel.get("type")
        if jt not in kinds:
            raise NotImplementedError(f"skel joint type {jt!r} is not on the timestep hot path")
        pnode = created[parent] if parent is not None else None
        joint, body = skel._create(kinds[jt], pnode, jel.get("name"), child)
        parent_world = bodies[parent]["init"] if parent is not None else np.eye(4)
        c2j = _iso(jel.find("transformation").text) if jel.find("transformation") is not None else np.eye(4)
        joint.setTransformFromParentBodyNode(np.linalg.inv(parent_world) @ bodies[child]["init"] @ c2j)
        joint.setTransformFromChildBodyNode(c2j)
        ax = jel.find("axis")
        if jt in ("revolute", "prismatic"):
            joint.setAxis(_vec(ax.find("xyz").text))
            dynel = ax.find("dynamics")
            if dynel is not None:
                if dynel.find("damping") is not None:
                    joint.setDampingCoefficient(0, float(dynel.find("damping").text))
                if dynel.find("spring_stiffness") is not None:
                    joint.setSpringStiffness(0, float(dynel.find("spring_stiffness").text))
                if dynel.find("spring_rest_position") is not None:
                    joint.setRestPosition(0, float(dynel.find("spring_rest_position").text))
            lim = ax.find("limit")
            if lim is not None:
                if lim.find("lower") is not None:
                    joint.setPositionLowerLimit(0, float(lim.find("lower").text))
                if lim.find("upper") is not None:
                    joint.setPositionUpperLimit(0, float(lim.find("upper").text))
            if jel.find("init_pos") is not None:
                joint.initial_positions[0] = float(jel.find("init_pos").text)
        rec = bodies[child]
        body.setMass(rec["mass"])
        body.setLocalCOM(rec["com"])
        if rec["moment"] is not None:
            body.setMomentOfInertia(*rec["moment"])
        for shape, Ts in rec["shapes"]:
            node = body.createShapeNode(shape, collision=True)
            node.setRelativeTransform(Ts)
        created[child] = body

    # getNextJointAndNodePair (:753): take the earliest remaining joint; if
    # its parent body does not exist yet, create the parent's joint first
    by_child = {child: item for item in joints for child in [item[2]]}
    while pending:
        item = pending[0]
        while item[1] is not None and item[1] not in created:
            if item[1] not in by_child:
                raise NotImplementedError("skel body without a parent joint (implicit free root)")
            item = by_child[item[1]]
        create(*item)
        pending.remove(item)
    skel._reindex()
    skel.setPositions(np.concatenate([b.joint.initial_positions for b in skel.bodies])
                      if skel.bodies else np.zeros(0))
    return skel


def read_world(path: str):
    """SkelParser::readWorld: a simulation.World with the file's skeletons,
    time step and gravity."""
    from .simulation import World
    root = ET.parse(path).getroot()
    wel = root.find("world")
    w = World(wel.get("name", "world"))
    phys = wel.find("physics")
    if phys is not None:
        if phys.find("time_step") is not None:
            w.setTimeStep(float(phys.find("time_step").text))
        if phys.find("gravity") is not None:
            w.setGravity(_vec(phys.find("gravity").text))
    for sk in wel.findall("skeleton"):
        w.addSkeleton(read_skeleton(sk))
    return w
