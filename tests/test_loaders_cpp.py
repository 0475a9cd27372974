"""The C++ model loaders (nimblephysics_amd/csrc/loaders.cpp:
utils::DartLoader::parseSkeleton, DartLoader.cpp:199, and
utils::SkelParser::readWorld, SkelParser.cpp:402) against the Python loaders
(nimblephysics_amd/urdf.py, skel.py) that the parity tests already pin: the
same file gives the same nimble_world_desc field by field and the same initial
positions.

* self-contained fixtures written here: every URDF joint type the path models
  (revolute with limits that exclude 0 -> mid-point start, continuous,
  prismatic, fixed), rotated inertial frames, box / sphere / binary-STL mesh
  colliders with scale, a "world" root; a .skel world with a skeleton frame,
  eulerXYZ transforms, init_pos, joint dynamics and limits, joints listed
  child-before-parent (getNextJointAndNodePair order);
* the reference's own model files when /root/reference is present (this
  container only): Atlas with box and with STL mesh colliders, the cartpole
  URDF, the ground and half_cheetah.skel.

The C++ API scans every mesh vertex (no hull-candidate mask), so that one
field is not compared.  CPU only: loading needs no GPU.
"""
import json
import os
import struct
import subprocess

import numpy as np
import pytest

import nimblephysics_amd as nimble
from nimblephysics_amd import skel as _skel
from nimblephysics_amd import urdf as _urdf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "world_api_test")
REF = "/root/reference"


def _cpp(mode, path):
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} missing: run __graft_entry__.build()")
    r = subprocess.run([EXE, mode, path], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.replace("-inf", "-Infinity").replace("inf", "Infinity"))


def _compare(got, world):
    want = world.desc_arrays()
    desc = got["desc"]
    assert set(desc) == set(want), set(desc) ^ set(want)
    for k, v in want.items():
        if k == "mesh_vertex_candidate":
            continue
        a = np.asarray(desc[k], dtype=np.float64).reshape(-1)
        b = np.asarray(v, dtype=np.float64).reshape(-1)
        assert a.shape == b.shape, (k, a.shape, b.shape)
        fin = np.isfinite(b)
        assert np.array_equal(np.isfinite(a), fin) and np.array_equal(a[~fin], b[~fin]), k
        # rotations composed in a different operation order: last-bit slack
        assert np.abs(a[fin] - b[fin]).max(initial=0.0) <= 1e-14 * max(1.0, np.abs(b[fin]).max(initial=0.0)), k
    q = np.asarray(world.getPositions(), dtype=np.float64)
    assert np.allclose(np.asarray(got["positions"]), q, rtol=0, atol=1e-15), (got["positions"], q)


def _binary_stl(path, tris):
    with open(path, "wb") as fh:
        fh.write(b"\0" * 80)
        fh.write(struct.pack("<I", len(tris)))
        for t in tris:
            fh.write(struct.pack("<3f", 0, 0, 0))
            for v in t:
                fh.write(struct.pack("<3f", *v))
            fh.write(b"\0\0")


def _cube_tris(h=0.5):
    c = [(sx * h, sy * h, sz * h) for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)]
    faces = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    out = []
    for a, b, cc, d in faces:
        out += [(c[a], c[b], c[cc]), (c[a], c[cc], c[d])]
    return out


URDF = """<?xml version="1.0"?>
<!-- loader fixture -->
<robot name="fixture">
  <link name="base">
    <inertial><origin xyz="0.01 0.02 -0.03" rpy="0.3 -0.2 0.1"/><mass value="3.5"/>
      <inertia ixx="0.4" ixy="0.01" ixz="-0.02" iyy="0.5" iyz="0.03" izz="0.6"/></inertial>
    <collision><origin xyz="0 0 0.1" rpy="0 0.5 0"/><geometry><box size="0.3 0.2 0.1"/></geometry></collision>
  </link>
  <link name="arm_b"><inertial><mass value="1.25"/><inertia ixx="0.1" iyy="0.2" izz="0.3"/></inertial>
    <collision><geometry><sphere radius="0.07"/></geometry></collision></link>
  <link name="arm_a"><inertial><origin xyz="0 0 0.2"/><mass value="0.75"/>
      <inertia ixx="0.01" iyy="0.02" izz="0.03"/></inertial>
    <collision><origin xyz="0.1 0 0" rpy="0.1 0.2 0.3"/>
      <geometry><mesh filename="package://meshes/cube.stl" scale="0.5 1 2"/></geometry></collision></link>
  <link name="slider"><inertial><mass value="2"/><inertia ixx="1" iyy="1" izz="1"/></inertial></link>
  <link name="tip"><inertial><mass value="0.1"/><inertia ixx="0.001" iyy="0.001" izz="0.001"/></inertial></link>
  <joint name="z_continuous" type="continuous"><parent link="base"/><child link="arm_b"/>
    <origin xyz="0 0.3 0" rpy="0 0 1.0"/><axis xyz="0 0 2"/><limit effort="30" velocity="4"/>
    <dynamics damping="0.2"/></joint>
  <joint name="a_revolute" type="revolute"><parent link="base"/><child link="arm_a"/>
    <origin xyz="0.1 0 0.2" rpy="0.2 0 0"/><axis xyz="1 1 0"/>
    <limit lower="0.2" upper="1.4" effort="50" velocity="3"/></joint>
  <joint name="m_prismatic" type="prismatic"><parent link="arm_a"/><child link="slider"/>
    <axis xyz="0 1 0"/><limit lower="-0.9" upper="-0.1" effort="100" velocity="1"/></joint>
  <joint name="fixed_tip" type="fixed"><parent link="slider"/><child link="tip"/>
    <origin xyz="0 0 0.05"/></joint>
</robot>
"""

URDF_WORLD_ROOT = """<robot name="rooted">
  <link name="world"/>
  <link name="pole"><inertial><mass value="1"/><inertia ixx="0.1" iyy="0.1" izz="0.1"/></inertial>
    <collision><geometry><box size="0.1 0.1 1"/></geometry></collision></link>
  <joint name="hinge" type="revolute"><parent link="world"/><child link="pole"/>
    <axis xyz="0 1 0"/><limit lower="-3" upper="3" effort="1" velocity="1"/></joint>
</robot>
"""

SKEL = """<?xml version="1.0" ?>
<skel version="1.0">
  <world name="fixture world">
    <physics><time_step>0.002</time_step><gravity>0 -9.81 0</gravity>
      <collision_detector>fcl_mesh</collision_detector></physics>
    <skeleton name="ground"><mobile>false</mobile>
      <body name="ground"><transformation>0 -0.5 0 0 0 0</transformation>
        <collision_shape><geometry><box><size>5 0.1 5</size></box></geometry></collision_shape></body>
      <joint type="weld" name="joint 1"><parent>world</parent><child>ground</child></joint>
    </skeleton>
    <skeleton name="walker">
      <transformation>0 0.2 0 0 0.3 0</transformation>
      <body name="thigh"><transformation>0.1 -0.2 0 0.2 0 0.1</transformation>
        <inertia><mass>2.5</mass><offset>0 -0.1 0</offset>
          <moment_of_inertia><ixx>0.1</ixx><iyy>0.2</iyy><izz>0.3</izz><ixy>0.01</ixy><ixz>0</ixz><iyz>-0.02</iyz>
          </moment_of_inertia></inertia>
        <collision_shape><transformation>0 -0.1 0 1.5707963 0 0</transformation>
          <geometry><capsule><radius>0.05</radius><height>0.3</height></capsule></geometry></collision_shape>
      </body>
      <body name="torso"><transformation>0 0.1 0 0 0 0</transformation>
        <inertia><mass>6</mass></inertia>
        <collision_shape><geometry><sphere><radius>0.15</radius></sphere></geometry></collision_shape></body>
      <joint type="revolute" name="hip"><parent>torso</parent><child>thigh</child>
        <transformation>0 0.05 0 0 0 0.4</transformation>
        <axis><xyz>0 0 1</xyz><dynamics><damping>0.3</damping><spring_stiffness>2.0</spring_stiffness>
          <spring_rest_position>0.1</spring_rest_position></dynamics>
          <limit><lower>-1.0</lower><upper>0.7</upper></limit></axis>
        <init_pos>0.25</init_pos></joint>
      <joint type="prismatic" name="rootz"><parent>world</parent><child>torso</child>
        <axis><xyz>0 1 0</xyz></axis><init_pos>-0.05</init_pos></joint>
    </skeleton>
  </world>
</skel>
"""


def test_urdf_fixture(tmp_path):
    os.makedirs(tmp_path / "meshes")
    _binary_stl(str(tmp_path / "meshes" / "cube.stl"), _cube_tris())
    p = tmp_path / "fixture.urdf"
    p.write_text(URDF)
    w = nimble.World()
    w.addSkeleton(_urdf.load_urdf(str(p)))
    got = _cpp("describe-urdf", str(p))
    _compare(got, w)
    # bodies depth-first with children in joint-name order: base, arm_a,
    # slider, tip, arm_b
    assert got["desc"]["num_shapes"] == 3 and got["desc"]["shape_mesh_count"] == [0, 8, 0]
    assert got["positions"][6] == pytest.approx(0.8)  # a_revolute starts at the limits' mid point
    assert got["positions"][7] == pytest.approx(-0.5)  # m_prismatic likewise


def test_urdf_world_root(tmp_path):
    p = tmp_path / "rooted.urdf"
    p.write_text(URDF_WORLD_ROOT)
    w = nimble.World()
    w.addSkeleton(_urdf.load_urdf(str(p)))
    got = _cpp("describe-urdf", str(p))
    _compare(got, w)
    assert got["desc"]["num_dofs"] == 1


def test_skel_fixture(tmp_path):
    p = tmp_path / "fixture.skel"
    p.write_text(SKEL)
    got = _cpp("describe-skel", str(p))
    _compare(got, _skel.read_world(str(p)))
    assert got["desc"]["dt"] == 0.002 and got["positions"] == [-0.05, 0.25]


def test_loader_errors(tmp_path):
    p = tmp_path / "bad.urdf"
    p.write_text('<robot name="r"><link name="a"><collision><geometry><cylinder radius="1" length="1"/>'
                 '</geometry></collision></link></robot>')
    r = subprocess.run([EXE, "describe-urdf", str(p)], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "not on this path" in r.stderr
    r = subprocess.run([EXE, "describe-urdf", str(tmp_path / "missing.urdf")], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode != 0 and "cannot open" in r.stderr


REF_URDFS = ["data/sdf/atlas/atlas_v3_box_colliders.urdf", "data/sdf/atlas/atlas_v3_no_head.urdf",
             "data/sdf/atlas/ground.urdf", "data/urdf/cartpole.urdf"]


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference model files are only in the build container")
@pytest.mark.parametrize("rel", REF_URDFS)
def test_reference_urdf(rel):
    path = os.path.join(REF, rel)
    w = nimble.World()
    w.addSkeleton(_urdf.load_urdf(path))
    _compare(_cpp("describe-urdf", path), w)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference model files are only in the build container")
def test_reference_skel():
    path = os.path.join(REF, "data/skel/half_cheetah.skel")
    _compare(_cpp("describe-skel", path), _skel.read_world(path))
