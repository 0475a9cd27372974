"""Model assets: skeletons serialised as JSON (kinematic tree + inertia +
joint parameters + box/sphere collision shapes).

The JSON files under nimblephysics_amd/assets/ were generated from the
reference's model data (data/sdf/atlas/*.urdf, data/urdf/KR5/*.urdf) by
tools/export_assets.py using this package's URDF loader (urdf.py), so the GPU
box -- which has no /root/reference -- can load the benchmark models.
Also home of the programmatic models the reference's examples build in code
(python/nimblephysics_examples/cartpole.py).
"""
from __future__ import annotations

import json
import os

import numpy as np

from . import dynamics as dyn

ASSET_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")


def _shape_dict(node) -> dict:
    d = {"kind": node.shape.kind, "size": node.shape.size.tolist(), "T": node.T.tolist()}
    if node.shape.kind == dyn.SHAPE_MESH:
        # float32 values (assimp's ai_real), exact in JSON as repr of the double
        d["mesh"] = node.shape.path
        d["vertices"] = node.shape.vertices.reshape(-1).tolist()
        d["candidate"] = node.shape.candidate().tolist()
    return d


def skeleton_to_dict(skel: dyn.Skeleton) -> dict:
    bodies = []
    for b in skel.bodies:
        j = b.joint
        bodies.append({
            "name": b.name,
            "parent": b.parent.index if b.parent is not None else -1,
            "joint": {
                "name": j.name, "type": j.kind,
                "T_parent": j.T_parent.tolist(), "T_child": j.T_child.tolist(), "axis": j.axis.tolist(),
                "damping": j.damping.tolist(), "spring": j.spring.tolist(), "rest": j.rest.tolist(),
                "pos_lo": j.pos_lo.tolist(), "pos_hi": j.pos_hi.tolist(),
                "vel_lo": j.vel_lo.tolist(), "vel_hi": j.vel_hi.tolist(),
                "force_lo": j.force_lo.tolist(), "force_hi": j.force_hi.tolist(),
                "initial": j.initial_positions.tolist(),
            },
            "mass": b.mass, "com": b.com.tolist(), "moment": b.moment.tolist(),
            "friction": b.friction, "restitution": b.restitution,
            "shapes": [_shape_dict(s) for s in b.shape_nodes if s.collision],
        })
    return {"name": skel.name, "mobile": skel.mobile, "bodies": bodies,
            "positions": skel.getPositions().tolist()}


def _fix(x):
    return [float("inf") if v == "inf" else float("-inf") if v == "-inf" else v for v in x]


def skeleton_from_dict(d: dict) -> dyn.Skeleton:
    skel = dyn.Skeleton(d["name"])
    for bd in d["bodies"]:
        jd = bd["joint"]
        parent = skel.bodies[bd["parent"]] if bd["parent"] >= 0 else None
        j, b = skel._create(jd["type"], parent, jd["name"], bd["name"])
        j.T_parent = np.array(jd["T_parent"])
        j.T_child = np.array(jd["T_child"])
        j.axis = np.array(jd["axis"])
        for k in ("damping", "spring", "rest", "pos_lo", "pos_hi", "vel_lo", "vel_hi", "force_lo", "force_hi"):
            setattr(j, k, np.array(_fix(jd[k]), dtype=np.float64))
        j.initial_positions = np.array(jd["initial"], dtype=np.float64)
        b.mass = bd["mass"]
        b.com = np.array(bd["com"])
        b.moment = np.array(bd["moment"])
        b.friction = bd["friction"]
        b.restitution = bd["restitution"]
        for sd in bd["shapes"]:
            if sd["kind"] == dyn.SHAPE_BOX:
                shape = dyn.BoxShape(sd["size"])
            elif sd["kind"] == dyn.SHAPE_CAPSULE:
                shape = dyn.CapsuleShape(sd["size"][0], sd["size"][1])
            elif sd["kind"] == dyn.SHAPE_MESH:
                shape = dyn.MeshShape(sd["size"], np.array(sd["vertices"]), sd.get("mesh", ""))
                if "candidate" in sd:
                    shape._candidate = np.asarray(sd["candidate"], dtype=np.int32)
                    shape._candidate_size = np.asarray(sd["size"], dtype=np.float64).copy()
            else:
                shape = dyn.SphereShape(sd["size"][0])
            node = b.createShapeNode(shape, collision=True)
            node.T = np.array(sd["T"])
    skel.mobile = d.get("mobile", True)
    skel.setPositions(np.array(d["positions"], dtype=np.float64))
    skel.setVelocities(np.zeros(skel.getNumDofs()))
    return skel


def _enc(o):
    if isinstance(o, float) and not np.isfinite(o):
        return "inf" if o > 0 else "-inf"
    if isinstance(o, dict):
        return {k: _enc(v) for k, v in o.items()}
    if isinstance(o, list):
        return [_enc(v) for v in o]
    return o


def save_skeleton(skel: dyn.Skeleton, path: str):
    with open(path, "w") as f:
        json.dump(_enc(skeleton_to_dict(skel)), f)


def load_skeleton(name_or_path: str) -> dyn.Skeleton:
    path = name_or_path
    if not os.path.exists(path):
        path = os.path.join(ASSET_DIR, name_or_path + ".json")
    with open(path) as f:
        return skeleton_from_dict(json.load(f))


def save_world(world, path: str):
    """A whole world (skeletons in World::addSkeleton order + time step and
    gravity) as JSON -- for .skel worlds, whose <physics> block is part of the
    model."""
    d = {"dt": world.getTimeStep(), "gravity": list(map(float, world.getGravity())),
         "skeletons": [skeleton_to_dict(s) for s in world.skeletons]}
    with open(path, "w") as f:
        json.dump(_enc(d), f)


def load_world(name_or_path: str):
    from .simulation import World
    path = name_or_path
    if not os.path.exists(path):
        path = os.path.join(ASSET_DIR, name_or_path + ".json")
    with open(path) as f:
        d = json.load(f)
    w = World()
    w.setTimeStep(d["dt"])
    w.setGravity(d["gravity"])
    for sd in d["skeletons"]:
        w.addSkeleton(skeleton_from_dict(sd))
    return w


def cartpole() -> dyn.Skeleton:
    """python/nimblephysics_examples/cartpole.py: prismatic cart + revolute
    pole, default inertias (mass 1, identity moment), visual-only shapes."""
    skel = dyn.Skeleton("cartpole")
    rail, cart = skel.createPrismaticJointAndBodyNodePair()
    rail.setAxis([1, 0, 0])
    cart.createShapeNode(dyn.BoxShape([0.5, 0.1, 0.1]))
    rail.setPositionUpperLimit(0, 10)
    rail.setPositionLowerLimit(0, -10)
    rail.setControlForceUpperLimit(0, 10)
    rail.setControlForceLowerLimit(0, -10)
    pole_joint, pole = skel.createRevoluteJointAndBodyNodePair(cart)
    pole_joint.setAxis([0, 0, 1])
    pole.createShapeNode(dyn.BoxShape([0.1, 1.0, 0.1]))
    pole_joint.setControlForceUpperLimit(0, 0)
    pole_joint.setControlForceLowerLimit(0, 0)
    off = dyn.Isometry3()
    off.set_translation([0, -0.5, 0])
    pole_joint.setTransformFromChildBodyNode(off)
    return skel
