"""Regenerate nimblephysics_amd/assets/*.json from the reference's model data
(run in the container that has /root/reference; the GPU box does not)."""
import os
import sys

import numpy as np  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nimblephysics_amd import assets, skel, urdf  # noqa: E402

REF = os.environ.get("NIMBLE_REFERENCE", "/root/reference")
MODELS = {
    "atlas": ("data/sdf/atlas/atlas_v3_box_colliders.urdf", False),
    # the reference atlas_bench's model (python/nimblephysics_benchmarks/
    # atlas_bench.py:18): STL mesh colliders
    "atlas_mesh": ("data/sdf/atlas/atlas_v3_no_head.urdf", False),
    "atlas_ground": ("data/sdf/atlas/ground.urdf", False),
    "kr5": ("data/urdf/KR5/KR5 sixx R650.urdf", True),
    "kr5_ground": ("data/urdf/KR5/ground.urdf", True),
    "cartpole_urdf": ("data/urdf/cartpole.urdf", False),
}

WORLDS = {
    "half_cheetah_world": "data/skel/half_cheetah.skel",
}

if __name__ == "__main__":
    for name, (rel, ignore_mesh) in MODELS.items():
        sk = urdf.load_urdf(os.path.join(REF, rel), ignore_mesh_collisions=ignore_mesh)
        out = os.path.join(assets.ASSET_DIR, name + ".json")
        assets.save_skeleton(sk, out)
        print(name, sk.getNumDofs(), "dofs", len(sk.bodies), "bodies ->", out)
    for name, rel in WORLDS.items():
        w = skel.read_world(os.path.join(REF, rel))
        out = os.path.join(assets.ASSET_DIR, name + ".json")
        assets.save_world(w, out)
        print(name, w.getNumDofs(), "dofs", [len(s.bodies) for s in w.skeletons], "bodies ->", out)
