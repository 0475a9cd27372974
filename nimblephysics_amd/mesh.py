"""Mesh collision geometry: STL reading and the per-vertex candidate mask.

The reference loads a MeshShape's file with assimp
(dart/dynamics/MeshShape.cpp:474, aiProcess_JoinIdenticalVertices among the
post-processing flags) and its DART collider treats the mesh as the convex
hull of the aiMesh vertex list, read in order (ccdSupportMesh,
DARTCollide.cpp:1935: the FIRST vertex of largest dot product;
ccdPointsAtWitnessMesh :2119: every vertex within the witness plane depth of
the extreme one, de-duplicated within 1e-3 m of an earlier one, in order).
Both depend only on the vertex positions and their first-occurrence order, so
the vertex list here is the STL's triangle corners with exact repeats of a
position removed, in order of first appearance (what JoinIdenticalVertices
keeps), as float32 values (assimp's ai_real) widened to double.

Candidate mask (device scan only): a vertex at distance > depth from every
face of the convex hull boundary (i.e. strictly inside by more than the
witness plane depth 0.01) can never be a support point or a witness point,
since for a unit direction d, v . d <= h(d) - dist(v, boundary).  The device
scans only candidates, in their original order, so its results are those of
the full list; the oracle scans the full list.
"""
from __future__ import annotations

import struct

import numpy as np

WITNESS_PLANE_DEPTH = 0.01  # DART_COLLISION_WITNESS_PLANE_DEPTH (DARTCollide.cpp:58)


def read_stl(path: str) -> np.ndarray:
    """Triangle corners of a binary or ASCII STL as float32 -> float64,
    [3 * triangles, 3] in file order."""
    with open(path, "rb") as fh:
        data = fh.read()
    if len(data) >= 84:
        ntri = struct.unpack_from("<I", data, 80)[0]
        if 84 + 50 * ntri == len(data):
            rec = np.frombuffer(data, dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]),
                                count=ntri, offset=84)
            return rec["v"].reshape(-1, 3).astype(np.float64)
    verts = []
    for line in data.decode("ascii", "replace").splitlines():
        t = line.split()
        if len(t) == 4 and t[0] == "vertex":
            verts.append([np.float32(float(x)) for x in t[1:]])
    return np.asarray(verts, dtype=np.float32).astype(np.float64).reshape(-1, 3)


def unique_in_order(corners: np.ndarray) -> np.ndarray:
    """Positions in order of first appearance, exact repeats removed."""
    _, first = np.unique(corners, axis=0, return_index=True)
    return corners[np.sort(first)]


def candidate_mask(verts: np.ndarray, scale=(1.0, 1.0, 1.0), depth: float = WITNESS_PLANE_DEPTH,
                   margin: float = 1e-4) -> np.ndarray:
    """1 for vertices within depth + margin of the convex hull boundary of the
    scaled vertex set (the only possible support / witness points), else 0."""
    v = np.asarray(verts, dtype=np.float64) * np.asarray(scale, dtype=np.float64)[None, :]
    if v.shape[0] < 5:
        return np.ones(v.shape[0], dtype=np.int32)
    try:
        from scipy.spatial import ConvexHull
        hull = ConvexHull(v)
    except Exception:
        return np.ones(v.shape[0], dtype=np.int32)
    # facet planes n . x + c <= 0 inside; distance to the boundary of an
    # interior point = min over facets of -(n . x + c)
    dist = -(v @ hull.equations[:, :3].T + hull.equations[:, 3][None, :])
    dmin = dist.min(axis=1)
    return (dmin <= depth + margin).astype(np.int32)
