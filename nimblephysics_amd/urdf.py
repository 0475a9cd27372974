"""URDF -> Skeleton, following the reference's loader rules.

Mirrors dart/utils/urdf/DartLoader.cpp (modelInterfaceToSkeleton :199,
createSkeletonRecursive, createDartJoint :380-520, createDartNodeProperties
:524) on top of urdfdom's tree construction, whose ModelInterface::initTree
iterates joints in std::map (name-sorted) order -- so a link's children, and
therefore DART's depth-first BodyNode / DOF order, are sorted by joint name.

Supported collision geometry: box, sphere and STL meshes (MeshShape, read by
mesh.read_stl).  Visual geometry is ignored.  ``ignore_mesh_collisions=True``
drops mesh colliders.
"""
from __future__ import annotations

import math
import os
import xml.etree.ElementTree as ET
from typing import Dict, List, Optional

import numpy as np

from . import dynamics as dyn


def _vec(s: Optional[str], default=(0.0, 0.0, 0.0)) -> np.ndarray:
    if s is None:
        return np.array(default, dtype=np.float64)
    return np.array([float(x) for x in s.split()], dtype=np.float64)


def _origin(elem) -> np.ndarray:
    T = np.eye(4)
    if elem is None:
        return T
    o = elem.find("origin")
    if o is None:
        return T
    T[:3, :3] = dyn.rpy_to_matrix(_vec(o.get("rpy")))
    T[:3, 3] = _vec(o.get("xyz"))
    return T


class _Link:
    def __init__(self, e):
        self.e = e
        self.name = e.get("name")
        self.child_joints: List["_Joint"] = []


class _Joint:
    def __init__(self, e):
        self.e = e
        self.name = e.get("name")
        self.type = e.get("type")
        self.parent = e.find("parent").get("link")
        self.child = e.find("child").get("link")


def load_urdf(path: str, ignore_mesh_collisions: bool = False) -> dyn.Skeleton:
    root = ET.parse(path).getroot()
    links: Dict[str, _Link] = {l.get("name"): _Link(l) for l in root.findall("link")}
    joints = [_Joint(j) for j in root.findall("joint")]
    child_of = {}
    # urdfdom initTree: std::map<std::string, JointSharedPtr> => name order
    for j in sorted(joints, key=lambda j: j.name):
        links[j.parent].child_joints.append(j)
        child_of[j.child] = j
    roots = [l for name, l in links.items() if name not in child_of]
    if len(roots) != 1:
        raise ValueError(f"URDF {path}: expected one root link, found {[r.name for r in roots]}")
    root_link = roots[0]
    skel = dyn.Skeleton(root.get("name", "robot"))

    def make_body(link: _Link, joint_kind: int, joint_name: str, parent_body):
        j, b = skel._create(joint_kind, parent_body, joint_name, link.name)
        _node_properties(link, b)
        _shapes(link, b, ignore_mesh_collisions, os.path.dirname(os.path.abspath(path)))
        return j, b

    def recurse(link: _Link, parent_body):
        for jt in link.child_joints:
            child = links[jt.child]
            kind = {
                "revolute": dyn.JOINT_REVOLUTE,
                "continuous": dyn.JOINT_REVOLUTE,
                "prismatic": dyn.JOINT_PRISMATIC,
                "fixed": dyn.JOINT_WELD,
                "floating": dyn.JOINT_FREE,
            }.get(jt.type)
            if kind is None:
                raise NotImplementedError(f"URDF joint type {jt.type} not supported on the hot path")
            j, b = make_body(child, kind, jt.name, parent_body)
            j.T_parent = _origin(jt.e)
            if kind in (dyn.JOINT_REVOLUTE, dyn.JOINT_PRISMATIC):
                ax = jt.e.find("axis")
                j.setAxis(_vec(ax.get("xyz") if ax is not None else None, (1.0, 0.0, 0.0)))
                lim = jt.e.find("limit")
                if lim is not None and jt.type != "continuous":
                    lo = float(lim.get("lower", 0.0))
                    hi = float(lim.get("upper", 0.0))
                    j.pos_lo[0], j.pos_hi[0] = lo, hi
                if lim is not None:
                    vel = float(lim.get("velocity", 0.0))
                    eff = float(lim.get("effort", 0.0))
                    j.vel_lo[0], j.vel_hi[0] = -vel, vel
                    j.force_lo[0], j.force_hi[0] = -eff, eff
                    if jt.type != "continuous":
                        lo = float(lim.get("lower", 0.0))
                        hi = float(lim.get("upper", 0.0))
                        # DartLoader.cpp: zero outside the limits -> mid point
                        if lo > 0 or hi < 0:
                            if math.isfinite(lo) and math.isfinite(hi):
                                init = (lo + hi) / 2.0
                            elif math.isfinite(lo):
                                init = lo
                            else:
                                init = hi
                            j.initial_positions[0] = init
                            j.rest[0] = init
                dynm = jt.e.find("dynamics")
                if dynm is not None:
                    j.damping[0] = float(dynm.get("damping", 0.0))
            recurse(child, b)

    if root_link.name == "world":
        recurse(root_link, None)
    else:
        make_body(root_link, dyn.JOINT_FREE, "rootJoint", None)
        recurse(root_link, skel.bodies[0])
    # joint initial positions -> skeleton positions
    q = np.zeros(skel.getNumDofs())
    for b in skel.bodies:
        j = b.joint
        q[j.dof_offset:j.dof_offset + j.getNumDofs()] = j.initial_positions
    skel.setPositions(q)
    skel.setVelocities(np.zeros_like(q))
    return skel


def _node_properties(link: _Link, body: dyn.BodyNode):
    inertial = link.e.find("inertial")
    if inertial is None:
        return
    T = _origin(inertial)
    body.setLocalCOM(T[:3, 3])
    m = inertial.find("mass")
    body.setMass(float(m.get("value")))
    ie = inertial.find("inertia")
    g = lambda k: float(ie.get(k, 0.0))
    J = np.array([[g("ixx"), g("ixy"), g("ixz")], [g("ixy"), g("iyy"), g("iyz")], [g("ixz"), g("iyz"), g("izz")]])
    R = T[:3, :3]
    J = R @ J @ R.T
    body.setMomentOfInertia(J[0, 0], J[1, 1], J[2, 2], J[0, 1], J[0, 2], J[1, 2])


def _shapes(link: _Link, body: dyn.BodyNode, ignore_mesh: bool, base_dir: str = "."):
    for c in link.e.findall("collision"):
        geo = c.find("geometry")
        shape = None
        box = geo.find("box")
        sph = geo.find("sphere")
        msh = geo.find("mesh")
        if box is not None:
            shape = dyn.BoxShape(_vec(box.get("size")))
        elif sph is not None:
            shape = dyn.SphereShape(float(sph.get("radius")))
        elif msh is not None and not ignore_mesh:
            # DartLoader::createShape (DartLoader.cpp): a MeshShape of the
            # file (resolved against the URDF's directory) with its scale
            from .mesh import read_stl, unique_in_order
            fn = msh.get("filename")
            for pre in ("package://", "file://"):
                if fn.startswith(pre):
                    fn = fn[len(pre):]
            path = fn if os.path.isabs(fn) else os.path.join(base_dir, fn)
            if not path.lower().endswith(".stl"):
                raise NotImplementedError(f"mesh collision geometry {fn}: only STL files are read")
            shape = dyn.MeshShape(_vec(msh.get("scale"), (1.0, 1.0, 1.0)), unique_in_order(read_stl(path)), fn)
        else:
            if ignore_mesh:
                continue
            kinds = [x.tag for x in geo]
            raise NotImplementedError(f"collision geometry {kinds} on link {link.name} is not supported")
        node = body.createShapeNode(shape, collision=True)
        node.setRelativeTransform(_origin(c))


def resolve(path: str) -> str:
    return os.path.abspath(path)
