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


def box_world(size=(0.4, 0.3, 0.2), friction=1.0, mass=1.0):
    """A free box over a static ground box (top face at y = 0) -- the small
    contact world the reference's own LCP / gradient tests use
    (unittests/comprehensive/test_Contacts.cpp style)."""
    from nimblephysics_amd import dynamics as D
    w = nimble.World()
    w.setGravity([0, -9.81, 0])
    box = D.Skeleton("box")
    _, b = box.createFreeJointAndBodyNodePair()
    b.setMass(mass)
    sx, sy, sz = size
    b.setMomentOfInertia(mass * (sy * sy + sz * sz) / 12, mass * (sx * sx + sz * sz) / 12,
                         mass * (sx * sx + sy * sy) / 12)
    b.createShapeNode(D.BoxShape(list(size)), collision=True)
    b.setFrictionCoeff(friction)
    w.addSkeleton(box)
    ground = D.Skeleton("ground")
    gj, gb = ground.createWeldJointAndBodyNodePair()
    T = np.eye(4)
    T[1, 3] = -0.05
    gj.setTransformFromParentBodyNode(T)
    gb.createShapeNode(D.BoxShape([10.0, 0.1, 10.0]), collision=True)
    ground.setMobile(False)
    w.addSkeleton(ground)
    return w


def box_states(kind, batch, seed=0, size=(0.4, 0.3, 0.2)):
    """Box states in distinct contact regimes: 'rest' (flat, ~1 mm
    penetration, small velocities: sticking), 'slide' (tangential speed:
    friction at the cone bound -> upper-bound rows), 'tilt' (rotated about z:
    two-point contact), 'lift' (separating velocity: nothing clamps)."""
    rng = np.random.default_rng(seed)
    q = np.zeros((batch, 6))
    v = np.zeros((batch, 6))
    h = 0.5 * size[1]
    q[:, 4] = h - 1e-3 + 2e-4 * rng.standard_normal(batch)
    q[:, 0:3] = 1e-3 * rng.standard_normal((batch, 3))
    v[:] = 0.01 * rng.standard_normal((batch, 6))
    if kind == "slide":
        v[:, 3] = 1.0 + 0.2 * rng.standard_normal(batch)
        v[:, 5] = 0.3 * rng.standard_normal(batch)
    elif kind == "tilt":
        ang = 0.3 + 0.05 * rng.standard_normal(batch)
        q[:, 2] = ang
        # lowest corner ~1 mm below the ground plane
        q[:, 4] = 0.5 * (size[0] * np.sin(np.abs(ang)) + size[1] * np.cos(ang)) - 1e-3
    elif kind == "lift":
        v[:, 4] = 0.5 + 0.1 * rng.standard_normal(batch)
    f = 0.5 * rng.standard_normal((batch, 6))
    return np.concatenate([q, v], axis=1), f
