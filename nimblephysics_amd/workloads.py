"""The benchmark workloads (BASELINE.json configs): world builders and the
synthetic state samplers bench.py times and the tests check.

configs[0] KR5 arm (no contact), configs[1] cartpole, configs[2] half-cheetah
on the ground box, configs[3] Atlas with ground + foot contact.
"""
import numpy as np

from . import assets
from .simulation import World


def cartpole_world():
    """configs[1]: cartpole (python/nimblephysics_examples/cartpole.py)."""
    w = World()
    w.setGravity([0, -9.81, 0])
    w.addSkeleton(assets.cartpole())
    w.setTimeStep(w.getTimeStep() * 10)
    return w


def kr5_world():
    """configs[0]: KR5 arm, no contact (data/urdf/KR5)."""
    w = World()
    w.setGravity([0, -9.81, 0])
    w.addSkeleton(assets.load_skeleton("kr5"))
    return w


def atlas_world(with_ground=True):
    """configs[3]: Atlas with box foot colliders on the ground box
    (python/nimblephysics_benchmarks/atlas_bench.py: gravity -y, root rotated
    by -pi/2 about x)."""
    w = World()
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


def half_cheetah_world():
    """configs[2]: data/skel/half_cheetah.skel (ground box 1500 x 0.05 x 5 +
    planar cheetah: prismatic x/y + revolute root, six revolute leg joints with
    damping and springs, capsule colliders), dt 0.002, gravity -y.  Loaded
    from the JSON export of SkelParser's result (tools/export_assets.py)."""
    return assets.load_world("half_cheetah_world")


def _fk_world(desc, q):
    """Body world transforms for revolute / prismatic / weld trees (host-side
    helper for placing synthetic states; the device computes its own)."""
    nb = int(desc["num_bodies"])
    Tw = np.zeros((nb, 4, 4))
    for b in range(nb):
        Tp = np.eye(4)
        Tp[:3, :4] = desc["T_parent_joint"][12 * b:12 * b + 12].reshape(3, 4)
        Tc = np.eye(4)
        Tc[:3, :4] = desc["T_child_joint"][12 * b:12 * b + 12].reshape(3, 4)
        J = np.eye(4)
        jt = int(desc["joint_type"][b])
        ax = desc["axis"][3 * b:3 * b + 3]
        if jt == 1:
            th = q[desc["dof_offset"][b]]
            K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
            J[:3, :3] = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
        elif jt == 2:
            J[:3, 3] = ax * q[desc["dof_offset"][b]]
        elif jt != 0:
            raise NotImplementedError("free joints: use the device kinematics")
        par = int(desc["parent"][b])
        base = Tw[par] if par >= 0 else np.eye(4)
        Tw[b] = base @ Tp @ J @ np.linalg.inv(Tc)
    return Tw


def lowest_capsule_point(world, q):
    """Lowest world y over the world's capsule colliders at configuration q."""
    d = world.desc_arrays()
    Tw = _fk_world(d, q)
    low = np.inf
    for s in range(int(d["num_shapes"])):
        if int(d["shape_type"][s]) != 2:
            continue
        T = np.eye(4)
        T[:3, :4] = d["shape_T"][12 * s:12 * s + 12].reshape(3, 4)
        T = Tw[int(d["shape_body"][s])] @ T
        r, h = d["shape_size"][3 * s], d["shape_size"][3 * s + 1]
        for z in (h / 2, -h / 2):
            low = min(low, (T @ np.array([0, 0, z, 1.0]))[1] - r)
    return low


def half_cheetah_states(world, batch, seed=0, angle_scale=0.25, v_scale=0.3, f_scale=5.0,
                        pen_range=(-4e-3, 2e-3)):
    """Synthetic half-cheetah states: random joint angles / velocities, the
    root lowered so the lowest capsule point sits `pen` below the ground top
    (negative = penetrating; contact for most worlds), random torques."""
    rng = np.random.default_rng(seed)
    n = world.getNumDofs()
    q = np.zeros((batch, n))
    q[:, 2] = 0.1 * rng.standard_normal(batch)
    q[:, 3:] = angle_scale * rng.standard_normal((batch, n - 3))
    q[:, 0] = 0.5 * rng.standard_normal(batch)
    for b in range(batch):
        pen = rng.uniform(*pen_range)
        q[b, 1] = pen - lowest_capsule_point(world, q[b])
    v = v_scale * rng.standard_normal((batch, n))
    f = f_scale * rng.standard_normal((batch, n))
    f[:, :3] = 0.0  # unactuated root (half_cheetah_bench.py force limits)
    return np.concatenate([q, v], axis=1), f


def atlas_states(world, batch, seed):
    """The Atlas bench sampler: perturbed standing poses near / in ground
    contact, small velocities, random torques."""
    return random_states(world, batch, seed=seed, q_scale=0.02, v_scale=0.05, f_scale=1.0)


def cheetah_states(world, batch, seed):
    """The half-cheetah bench sampler."""
    return half_cheetah_states(world, batch, seed=seed)


def atlas_mesh_world(with_ground=True):
    """The reference atlas_bench's own Atlas (python/nimblephysics_benchmarks/
    atlas_bench.py:18-19: atlas_v3_no_head.urdf, 29 STL mesh colliders) on the
    ground box, set up as atlas_world."""
    w = World()
    w.setGravity([0, -9.81, 0])
    atlas = w.addSkeleton(assets.load_skeleton("atlas_mesh"))
    atlas.setPosition(0, -0.5 * 3.14159)
    if with_ground:
        w.addSkeleton(assets.load_skeleton("atlas_ground"))
    return w
