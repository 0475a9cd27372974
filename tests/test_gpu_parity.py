"""Parity of the HIP path (through the C-ABI) against the CPU oracle.

Tolerance (BASELINE.json north_star): 1e-6 relative on positions, velocities
and gradients.  Dynamics-only paths (no contact) match to ~1e-10.
"""
import numpy as np
import pytest
import torch

import models
from oracle.oracle import OracleWorld

pytestmark = pytest.mark.gpu

RTOL = 1e-6


def _rel(a, b, floor=1e-6):
    """Largest per-element relative error, |a - b| / max(|b|, floor * max|b|)."""
    a, b = np.asarray(a), np.asarray(b)
    scale = np.maximum(np.abs(b), floor * max(np.abs(b).max(), 1e-300))
    return float((np.abs(a - b) / scale).max())


def _run_both(world, batch, seed):
    import nimblephysics_amd as nimble
    st, f = models.random_states(world, batch, seed=seed)
    o = OracleWorld(world)
    ref_next = o.forward(st, f)
    rng = np.random.default_rng(seed + 100)
    g = rng.standard_normal(st.shape)
    ref_gs, ref_gf = o.backward(g)

    dev = torch.device("cuda:0")
    tst = torch.tensor(st, device=dev, requires_grad=True)
    tf = torch.tensor(f, device=dev, requires_grad=True)
    nxt = nimble.timestep(world, tst, tf)
    nxt.backward(torch.tensor(g, device=dev))
    return (ref_next, ref_gs, ref_gf), (nxt.detach().cpu().numpy(), tst.grad.cpu().numpy(), tf.grad.cpu().numpy())


@pytest.mark.parametrize("name,batch", [("cartpole", 1024), ("kr5", 128), ("atlas_air", 64)])
def test_no_contact_parity(name, batch):
    world = {"cartpole": models.cartpole_world, "kr5": models.kr5_world,
             "atlas_air": lambda: models.atlas_world(with_ground=False)}[name]()
    (rn, rgs, rgf), (gn, ggs, ggf) = _run_both(world, batch, seed=3)
    n = world.getNumDofs()
    assert _rel(gn[:, :n], rn[:, :n]) < RTOL
    assert _rel(gn[:, n:], rn[:, n:]) < RTOL
    assert _rel(ggs, rgs) < RTOL
    assert _rel(ggf, rgf) < RTOL


def test_empty_mass_gradient():
    """The reference's mass argument with no tuned masses: an empty mass
    vector goes through and gets an empty gradient."""
    import nimblephysics_amd as nimble
    world = models.cartpole_world()
    st = torch.tensor(world.getState(), device="cuda:0", requires_grad=True)
    f = torch.tensor([1.0, 0.0], dtype=torch.float64, device="cuda:0", requires_grad=True)
    mass = torch.zeros(0, dtype=torch.float64, device="cuda:0", requires_grad=True)
    out = nimble.timestep(world, st, f, mass)
    out.sum().backward()
    assert mass.grad is not None and mass.grad.shape == (0,)
    assert st.grad.shape == (4,) and torch.isfinite(st.grad).all()


def test_single_world_api():
    import nimblephysics_amd as nimble
    world = models.cartpole_world()
    world.setPositions([0.2, 0.3])
    o = OracleWorld(world)
    st = world.getState()
    f = np.array([1.0, 0.0])
    ref = o.forward(st[None], f[None])[0]
    out = nimble.timestep(world, torch.tensor(st, device="cuda:0"), torch.tensor(f, device="cuda:0"))
    assert out.shape == (4,)
    assert _rel(out.cpu().numpy(), ref) < RTOL
    assert np.allclose(world.getState(), out.cpu().numpy())


def test_reference_example_half_cheetah_cpu_tensors():
    """python/new_examples/half_cheetah.py as written for the reference:
    nimble.loadWorld("half_cheetah.skel"), 1-D CPU tensors of
    getStateSize() / getActionSize(), chained nimble.timestep calls, then a
    backward through the chain -- checked step by step against the oracle."""
    import nimblephysics_amd as nimble
    world = nimble.loadWorld("half_cheetah.skel")
    o = OracleWorld(world)
    state = torch.zeros((world.getStateSize()), dtype=torch.float64, requires_grad=True)
    action = torch.zeros((world.getActionSize()), dtype=torch.float64)
    n = world.getNumDofs()
    cur = state
    ref = np.zeros(2 * n)
    forces = np.zeros(n)
    contact_steps = 0
    for _ in range(100):  # first ground contact at step 63
        cur = nimble.timestep(world, cur, action)
        assert cur.device.type == "cpu" and cur.shape == (2 * n,)
        ref = o.forward(ref[None], forces[None])[0]
        contact_steps += o.num_contacts(0) > 0
        assert _rel(cur.detach().numpy(), ref) < RTOL
    assert contact_steps > 10
    cur.sum().backward()
    assert state.grad is not None and state.grad.device.type == "cpu"
    assert np.isfinite(state.grad.numpy()).all()


def test_kr5_single_world_cpu_tensors():
    """configs[0]: the 6-DoF KR5 arm, one world, CPU tensors through
    nimble.timestep (forward + backward) vs the oracle."""
    import nimblephysics_amd as nimble
    world = models.kr5_world()
    st, f = models.random_states(world, 1, seed=17)
    o = OracleWorld(world)
    ref = o.forward(st, f)[0]
    g = np.random.default_rng(1).standard_normal(st.shape[1])
    rgs, rgf = o.backward(g[None])
    ts = torch.tensor(st[0], requires_grad=True)
    tf = torch.tensor(f[0], requires_grad=True)
    out = nimble.timestep(world, ts, tf)
    out.backward(torch.tensor(g))
    assert out.device.type == "cpu"
    assert _rel(out.detach().numpy(), ref) < RTOL
    assert _rel(ts.grad.numpy(), rgs[0]) < RTOL
    assert _rel(tf.grad.numpy(), rgf[0]) < RTOL
