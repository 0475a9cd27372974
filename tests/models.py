"""Benchmark / test worlds (BASELINE.json configs)."""
import numpy as np

import nimblephysics_amd as nimble
from nimblephysics_amd import assets


def cartpole_world():
    """configs[1]: cartpole (python/nimblephysics_examples/cartpole.py)."""
    w = nimble.World()
    w.setGravity([0, -9.81, 0])
    w.addSkeleton(assets.cartpole())
    w.setTimeStep(w.getTimeStep() * 10)
    return w


def kr5_world():
    """configs[0]: KR5 arm, no contact (data/urdf/KR5)."""
    w = nimble.World()
    w.setGravity([0, -9.81, 0])
    w.addSkeleton(assets.load_skeleton("kr5"))
    return w


def atlas_world(with_ground=True):
    """configs[3]: Atlas with box foot colliders on the ground box
    (python/nimblephysics_benchmarks/atlas_bench.py: gravity -y, root rotated
    by -pi/2 about x)."""
    w = nimble.World()
    w.setGravity([0, -9.81, 0])
    atlas = w.addSkeleton(assets.load_skeleton("atlas"))
    atlas.setPosition(0, -0.5 * 3.14159)
    if with_ground:
        w.addSkeleton(assets.load_skeleton("atlas_ground"))
    return w


def random_states(world, batch, seed=0, q_scale=0.3, v_scale=0.5, f_scale=1.0):
    rng = np.random.default_rng(seed)
    n = world.getNumDofs()
    q0 = world.getPositions()
    q = q0[None, :] + q_scale * rng.standard_normal((batch, n))
    v = v_scale * rng.standard_normal((batch, n))
    f = f_scale * rng.standard_normal((batch, n))
    return np.concatenate([q, v], axis=1), f
