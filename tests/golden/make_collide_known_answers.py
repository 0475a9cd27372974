"""Transcribes the reference's collider known-answer tests into
tests/golden/collide_known_answers.json (run from the repo root; the
reference is only read as text: every input and expected value below is
copied from the cited test body, as the formula it is written with).

  unittests/unit/test_DARTCollide.cpp
    :2167 CAPSULE_CAPSULE_T_SHAPED_COLLISION   collideCapsuleCapsule both orders
    :2248 CAPSULE_CAPSULE_X_SHAPED_COLLISION
    :2329 CAPSULE_CAPSULE_L_SHAPED_COLLISION
    :2424 CAPSULE_SPHERE_END_COLLISION         collideCapsuleSphere / collideSphereCapsule
    :2498 CAPSULE_SPHERE_SIDE_COLLISION
    :1639 VERTEX_SPHERE_COLLISION / :1903 SPHERE_VERTEX_COLLISION
    :1729 EDGE_SPHERE_COLLISION   / :1993 SPHERE_EDGE_COLLISION
    :1818 FACE_SPHERE_COLLISION   / :2082 SPHERE_FACE_COLLISION
    :3117 CAPSULE_BOX_PIPE_EDGE_COLLISION      collideCapsuleBox / collideBoxCapsule
    :3272 CAPSULE_BOX_PIPE_VERTEX_COLLISION
    :2936 CAPSULE_BOX_SPHERE_AND_PIPE_EDGE_COLLISION (capsule first; contacts
          in sortContacts(UnitZ) order)
    :3429 CAPSULE_BOX_PIPE_EDGE_PARALLEL_VERTEX_COLLISION
    :3662 CAPSULE_BOX_PIPE_EDGE_PARALLEL_SPHERE_COLLISION

The sphere tests collide a sphere with a unit box *mesh* (ccdMPRPenetration +
createMeshSphereContact).  The same geometry through the box collider
(collideSphereBox :1655 / collideBoxSphere :1482) must give the same contact
normal and depth, and at a vertex or an edge the same point (the box's
vertex / edge point); on a face the mesh path reports the sphere's deepest
point and the box path the box surface point, so the face cases check normal
and depth only ("check": ["normal", "depth"]).

Type numbering: this package's (csrc/capsule.cuh): SPHERE_BOX 4, BOX_SPHERE 5,
SPHERE_SPHERE 6, SPHERE_PIPE 7, PIPE_SPHERE 8, PIPE_PIPE 9, PIPE_VERTEX 10,
VERTEX_PIPE 11, PIPE_EDGE 12, EDGE_PIPE 13 (the reference's 16 / 18 / 17 / 19),
SPHERE_EDGE 14, EDGE_SPHERE 15 (the reference's 8 / 11); the reference's
VERTEX_SPHERE / EDGE_SPHERE / FACE_SPHERE (mesh first) correspond to the box
collider's BOX_SPHERE, SPHERE_VERTEX / SPHERE_EDGE / SPHERE_FACE to
SPHERE_BOX.
"""
import json
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "unittests/unit/test_DARTCollide.cpp"
SPHERE_BOX, BOX_SPHERE, SPHERE_SPHERE, SPHERE_PIPE, PIPE_SPHERE, PIPE_PIPE = 4, 5, 6, 7, 8, 9
PIPE_VERTEX, VERTEX_PIPE, PIPE_EDGE, EDGE_PIPE = 10, 11, 12, 13
SPHERE_EDGE, EDGE_SPHERE = 14, 15


def euler_xyz(a, b, c):
    """math::eulerXYZToMatrix (dart/math/Geometry.cpp): R = Rx(a) Ry(b) Rz(c)."""
    ca, sa, cb, sb, cc, sc = math.cos(a), math.sin(a), math.cos(b), math.sin(b), math.cos(c), math.sin(c)
    Rx = np.array([[1, 0, 0], [0, ca, -sa], [0, sa, ca]])
    Ry = np.array([[cb, 0, sb], [0, 1, 0], [-sb, 0, cb]])
    Rz = np.array([[cc, -sc, 0], [sc, cc, 0], [0, 0, 1]])
    return Rx @ Ry @ Rz


def iso(p=(0, 0, 0), R=None):
    T = np.eye(4)
    if R is not None:
        T[:3, :3] = R
    T[:3, 3] = p
    return T


def contact(point, normal, depth, typ):
    return {"point": [float(x) for x in point], "normal": [float(x) for x in normal], "depth": float(depth),
            "type": typ}


def main():
    cases = []
    h, r1, r2 = 1.0, 0.4, 0.3
    ex, ey, ez = np.eye(3)
    # :2167 T-shaped: capsule 2 (along x after Ry(pi/2)) ends on capsule 1's side
    T1 = iso()
    T2 = iso((r1 + r2 + h / 2 - 0.01, 0, 0), euler_xyz(0, math.pi / 2, 0))
    p = ex * (r1 - 0.01 * r1 / (r1 + r2))
    cases.append({"name": "capsule_capsule_T", "source": f"{SRC}:2167",
                  "a": [["capsule", [r1, h]], T1.tolist()], "b": [["capsule", [r2, h]], T2.tolist()],
                  "ab": [contact(p, -ex, 0.01, PIPE_SPHERE)], "ba": [contact(p, ex, 0.01, SPHERE_PIPE)]})
    # :2248 X-shaped: crossing pipes
    T2 = iso((0, r1 + r2 - 0.01, 0), euler_xyz(0, math.pi / 2, 0))
    p = ey * (r1 - 0.01 * r1 / (r1 + r2))
    cases.append({"name": "capsule_capsule_X", "source": f"{SRC}:2248",
                  "a": [["capsule", [r1, h]], T1.tolist()], "b": [["capsule", [r2, h]], T2.tolist()],
                  "ab": [contact(p, -ey, 0.01, PIPE_PIPE)], "ba": [contact(p, ey, 0.01, PIPE_PIPE)]})
    # :2329 L-shaped: end caps touching
    T2 = iso((math.sqrt(2) * h / 4, 0, h / 2 + (math.sqrt(2) * h / 4) + r1 + r2 - 0.01),
             euler_xyz(0, math.pi / 4, 0))
    p = ez * (h / 2 + r1 - (0.01 * r1 / (r1 + r2)))
    cases.append({"name": "capsule_capsule_L", "source": f"{SRC}:2329",
                  "a": [["capsule", [r1, h]], T1.tolist()], "b": [["capsule", [r2, h]], T2.tolist()],
                  "ab": [contact(p, -ez, 0.01, SPHERE_SPHERE)], "ba": [contact(p, ez, 0.01, SPHERE_SPHERE)]})
    # :2424 capsule end vs sphere
    T2 = iso((0, 0, h / 2 + r1 + r2 - 0.01))
    p = ez * (h / 2 + r1 - (0.01 * r1 / (r1 + r2)))
    cases.append({"name": "capsule_sphere_end", "source": f"{SRC}:2424",
                  "a": [["capsule", [r1, h]], T1.tolist()], "b": [["sphere", [r2]], T2.tolist()],
                  "ab": [contact(p, -ez, 0.01, SPHERE_SPHERE)], "ba": [contact(p, ez, 0.01, SPHERE_SPHERE)]})
    # :2498 capsule side vs sphere
    T2 = iso((r1 + r2 - 0.01, 0, 0))
    p = ex * (r1 - (0.01 * r1 / (r1 + r2)))
    cases.append({"name": "capsule_sphere_side", "source": f"{SRC}:2498",
                  "a": [["capsule", [r1, h]], T1.tolist()], "b": [["sphere", [r2]], T2.tolist()],
                  "ab": [contact(p, -ex, 0.01, PIPE_SPHERE)], "ba": [contact(p, ex, 0.01, SPHERE_PIPE)]})
    # sphere (radius 0.5) against the unit box at a vertex, an edge, a face
    rs = 0.5
    box = [["box", [1.0, 1.0, 1.0]], iso().tolist()]
    c = 0.5 + math.sqrt(0.25 / 3) - 0.01
    n = np.ones(3) / math.sqrt(3)
    cases.append({"name": "sphere_box_vertex", "source": f"{SRC}:1639, :1903",
                  "a": [["sphere", [rs]], iso((c, c, c)).tolist()], "b": box,
                  "ab": [contact([0.5, 0.5, 0.5], n, math.sqrt(3 * 0.01 * 0.01), SPHERE_BOX)],
                  "ba": [contact([0.5, 0.5, 0.5], -n, math.sqrt(3 * 0.01 * 0.01), BOX_SPHERE)]})
    c = 0.5 + math.sqrt(0.125) - 0.01
    n = np.array([1.0, 1.0, 0.0]) / math.sqrt(2)
    cases.append({"name": "sphere_box_edge", "source": f"{SRC}:1729, :1993",
                  "a": [["sphere", [rs]], iso((c, c, 0)).tolist()], "b": box,
                  "ab": [contact([0.5, 0.5, 0.0], n, math.sqrt(2 * 0.01 * 0.01), SPHERE_BOX)],
                  "ba": [contact([0.5, 0.5, 0.0], -n, math.sqrt(2 * 0.01 * 0.01), BOX_SPHERE)]})
    cases.append({"name": "sphere_box_face", "source": f"{SRC}:1818, :2082", "check": ["normal", "depth"],
                  "a": [["sphere", [rs]], iso((1.0 - 0.01, 0, 0)).tolist()], "b": box,
                  "ab": [contact([0.5 - 0.01, 0, 0], ex, 0.01, SPHERE_BOX)],
                  "ba": [contact([0.5 - 0.01, 0, 0], -ex, 0.01, BOX_SPHERE)]})
    # capsule (radius 0.5, height 1) against the unit box, crossing an edge /
    # a vertex of it (box witness sets of 2 / 1 points)
    r, h = 0.5, 1.0
    c = 0.5 + math.sqrt(r * r / 2) - math.sqrt(0.01 * 0.01 / 2)
    T2 = iso((0, c, c), euler_xyz(math.pi / 4, 0, 0))
    n = np.array([0.0, 1.0, 1.0]) / math.sqrt(2)
    cases.append({"name": "capsule_box_pipe_edge", "source": f"{SRC}:3117",
                  "a": [["capsule", [r, h]], T2.tolist()], "b": box,
                  "ab": [contact([0, 0.5, 0.5], n, 0.01, PIPE_EDGE)],
                  "ba": [contact([0, 0.5, 0.5], -n, 0.01, EDGE_PIPE)]})
    c = 0.5 + math.sqrt(r * r / 3) - math.sqrt(0.01 * 0.01 / 3)
    T2 = iso((c, c, c), euler_xyz(math.pi / 4, 0, 0))
    n = np.ones(3) / math.sqrt(3)
    cases.append({"name": "capsule_box_pipe_vertex", "source": f"{SRC}:3272",
                  "a": [["capsule", [r, h]], T2.tolist()], "b": box,
                  "ab": [contact([0.5, 0.5, 0.5], n, 0.01, PIPE_VERTEX)],
                  "ba": [contact([0.5, 0.5, 0.5], -n, 0.01, VERTEX_PIPE)]})
    # :2936 a capsule lying on a 2 x 1 x 2 box with one end past its edge
    cases.append({"name": "capsule_box_sphere_and_pipe_edge", "source": f"{SRC}:2936", "sort": "z",
                  "a": [["capsule", [r, h]], iso((0, 0.99, 1.0)).tolist()], "b": [["box", [2.0, 1.0, 2.0]], iso().tolist()],
                  "ab": [contact([0, 0.5, 0.5], ey, 0.01, SPHERE_BOX), contact([0, 0.5, 1.0], ey, 0.01, PIPE_EDGE)]})
    # :3429 a capsule (height 2) lying parallel to a box edge and past both
    # of its ends: a PIPE_VERTEX contact at each end of the edge
    s2 = math.sqrt(r * r / 2) - math.sqrt(0.01 * 0.01 / 2)
    T2 = iso((0.5 + s2, 0.5 + s2, 0))
    n = np.array([1.0, 1.0, 0.0]) / math.sqrt(2)
    cases.append({"name": "capsule_box_pipe_edge_parallel_vertex", "source": f"{SRC}:3429", "sort": "z",
                  "a": [["capsule", [r, 2.0]], T2.tolist()], "b": box,
                  "ab": [contact([0.5, 0.5, -0.5], n, 0.01, PIPE_VERTEX), contact([0.5, 0.5, 0.5], n, 0.01, PIPE_VERTEX)],
                  "ba": [contact([0.5, 0.5, -0.5], -n, 0.01, VERTEX_PIPE),
                         contact([0.5, 0.5, 0.5], -n, 0.01, VERTEX_PIPE)]})
    # :3662 the same against a 1 x 1 x 2 box, the capsule (height 1) inside
    # the edge's span: SPHERE_EDGE / EDGE_SPHERE at the capsule ends (geometry
    # only: the reference's gradients of these read a NaN sphere centre, so
    # the step flags them unsupported)
    q = 0.5 - math.sqrt(0.01 * 0.01 / 2)
    cases.append({"name": "capsule_box_pipe_edge_parallel_sphere", "source": f"{SRC}:3662", "sort": "z",
                  "unsupported": True,
                  "a": [["capsule", [r, 1.0]], T2.tolist()], "b": [["box", [1.0, 1.0, 2.0]], iso().tolist()],
                  "ab": [contact([q, q, -0.5], n, 0.01, SPHERE_EDGE), contact([q, q, 0.5], n, 0.01, SPHERE_EDGE)],
                  "ba": [contact([q, q, -0.5], -n, 0.01, EDGE_SPHERE), contact([q, q, 0.5], -n, 0.01, EDGE_SPHERE)]})
    out = {"source": SRC + " (reference), transcribed by tests/golden/make_collide_known_answers.py; "
                           "'ab' = collide(a, b), 'ba' = collide(b, a); tolerance 1e-10 as in the tests "
                           "(1e-8 depth for the mesh-sphere cases)",
           "cases": cases}
    with open(os.path.join(HERE, "collide_known_answers.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"{len(cases)} cases")


if __name__ == "__main__":
    main()
