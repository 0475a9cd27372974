"""ctypes mirror of ``nimble_world_desc`` (include/nimble_amd.h)."""
from __future__ import annotations

import ctypes as C

import numpy as np

P_I32 = C.POINTER(C.c_int32)
P_F64 = C.POINTER(C.c_double)

NIMBLE_MAX_BODIES = 64
NIMBLE_MAX_DOFS = 64
NIMBLE_MAX_SHAPES = 64
NIMBLE_MAX_CONTACTS = 42
NIMBLE_MAX_LCP = 3 * NIMBLE_MAX_CONTACTS


class NimbleWorldDesc(C.Structure):
    _fields_ = [
        ("num_bodies", C.c_int32),
        ("num_dofs", C.c_int32),
        ("num_shapes", C.c_int32),
        ("reserved", C.c_int32),
        ("dt", C.c_double),
        ("gravity", C.c_double * 3),
        ("contact_clipping_depth", C.c_double),
        ("fallback_cfm", C.c_double),
        ("penetration_correction", C.c_int32),
        ("parallel_pos_vel", C.c_int32),
        ("parent", P_I32),
        ("skeleton", P_I32),
        ("joint_type", P_I32),
        ("dof_offset", P_I32),
        ("skeleton_mobile", P_I32),
        ("T_parent_joint", P_F64),
        ("T_child_joint", P_F64),
        ("axis", P_F64),
        ("mass", P_F64),
        ("com", P_F64),
        ("moment", P_F64),
        ("friction", P_F64),
        ("restitution", P_F64),
        ("damping", P_F64),
        ("spring", P_F64),
        ("rest_position", P_F64),
        ("pos_lower", P_F64),
        ("pos_upper", P_F64),
        ("vel_lower", P_F64),
        ("vel_upper", P_F64),
        ("force_lower", P_F64),
        ("force_upper", P_F64),
        ("shape_body", P_I32),
        ("shape_type", P_I32),
        ("shape_size", P_F64),
        ("shape_T", P_F64),
        ("num_mesh_vertices", C.c_int32),
        ("reserved2", C.c_int32),
        ("mesh_vertices", P_F64),
        ("shape_mesh_first", P_I32),
        ("shape_mesh_count", P_I32),
        ("mesh_vertex_candidate", P_I32),
    ]


def _i32(a):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.int32))
    if a.size == 0:
        a = np.zeros(1, dtype=np.int32)
    return a, a.ctypes.data_as(P_I32)


def _f64(a):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    if a.size == 0:
        a = np.zeros(1, dtype=np.float64)
    return a, a.ctypes.data_as(P_F64)


def build_desc(arrays: dict):
    """Build a NimbleWorldDesc from a dict of numpy arrays.  Returns
    (desc, keepalive) -- keep ``keepalive`` referenced while desc is used."""
    d = NimbleWorldDesc()
    keep = []
    d.num_bodies = int(arrays["num_bodies"])
    d.num_dofs = int(arrays["num_dofs"])
    d.num_shapes = int(arrays["num_shapes"])
    d.dt = float(arrays["dt"])
    for i in range(3):
        d.gravity[i] = float(arrays["gravity"][i])
    d.contact_clipping_depth = float(arrays["contact_clipping_depth"])
    d.fallback_cfm = float(arrays["fallback_cfm"])
    d.penetration_correction = int(arrays["penetration_correction"])
    d.parallel_pos_vel = int(arrays["parallel_pos_vel"])
    for name in ("parent", "skeleton", "joint_type", "dof_offset", "skeleton_mobile", "shape_body", "shape_type"):
        a, p = _i32(arrays[name])
        keep.append(a)
        setattr(d, name, p)
    for name in ("T_parent_joint", "T_child_joint", "axis", "mass", "com", "moment", "friction", "restitution",
                 "damping", "spring", "rest_position", "pos_lower", "pos_upper", "vel_lower", "vel_upper",
                 "force_lower", "force_upper", "shape_size", "shape_T"):
        a, p = _f64(arrays[name])
        keep.append(a)
        setattr(d, name, p)
    mv = np.asarray(arrays.get("mesh_vertices", np.zeros((0, 3))), dtype=np.float64).reshape(-1, 3)
    d.num_mesh_vertices = int(mv.shape[0])
    a, p = _f64(mv)
    keep.append(a)
    d.mesh_vertices = p
    ns = int(arrays["num_shapes"])
    for name in ("shape_mesh_first", "shape_mesh_count"):
        a, p = _i32(arrays.get(name, np.zeros(ns, dtype=np.int32)))
        keep.append(a)
        setattr(d, name, p)
    cand = arrays.get("mesh_vertex_candidate")
    if cand is not None and mv.shape[0] > 0:
        a, p = _i32(cand)
        keep.append(a)
        d.mesh_vertex_candidate = p
    return d, keep
