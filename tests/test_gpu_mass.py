"""Mass gradients (lossWrtMass) on the GPU against central differences of the
oracle's step over the body masses.

The reference computes lossWrtMass = getMassVelJacobian^T dL/dv'
(dart/neural/BackpropSnapshot.cpp:177, :580 -> getVelJacobianWrt(MASS), :980)
and its python layer returns it from TimestepLayer.backward
(python/nimblephysics/timestep.py:34, :57).  The oracle restates the forward
step only, so these gradients are pinned to finite differences of that step
(the reference's own GradientTestUtils strategy), per world and per body:
nimble_backward_masses' [B, num_bodies] against (L(m_b + e) - L(m_b - e)) / 2e
with L = g . next_state.
"""
import numpy as np
import pytest
import torch

import models
from oracle import oracle as O
from test_gpu_contact_parity import _check_contacts, _device_step

pytestmark = pytest.mark.gpu


def _oracle_loss(world, st, f, g, body, mass):
    sk_b = [b for s in world.skeletons for b in s.bodies][body]
    m0 = sk_b.getMass()
    sk_b.setMass(mass)
    try:
        o = O.OracleWorld(world)
        nxt = o.forward(st, f)
    finally:
        sk_b.setMass(m0)
    return (nxt * g).sum(axis=1)


def _mass_parity(world, st, f, seed=5, bodies=None, tol=1e-6):
    n = world.getNumDofs()
    B = st.shape[0]
    ow = O.OracleWorld(world)
    ow.forward(st, f)
    nxt, snap, cache, ts, tf = _device_step(world, st, f)
    same = np.ones(B, dtype=bool)
    if world.native().num_pairs > 0:
        same = _check_contacts(ow, snap.cpu().numpy(), B, cache=cache.cpu().numpy())
    dev = world.native()
    g = np.random.default_rng(seed).standard_normal(st.shape)
    gt = torch.tensor(g, device=ts.device)
    gs, gf = torch.empty_like(ts), torch.empty_like(tf)
    gm = torch.empty((B, dev.nb), dtype=torch.float64, device=ts.device)
    stream = torch.cuda.current_stream().cuda_stream
    dev.backward_masses(ts, tf, snap, gt, gs, gf, gm, stream)
    gs2, gf2 = torch.empty_like(ts), torch.empty_like(tf)
    dev.backward(ts, tf, snap, gt, gs2, gf2, stream)
    torch.cuda.synchronize()
    # the mass term leaves the state / force gradients untouched
    assert torch.equal(gs, gs2) and torch.equal(gf, gf2)
    gm = gm.cpu().numpy()
    masses = np.asarray(world.desc_arrays()["mass"])
    bodies = range(dev.nb) if bodies is None else bodies
    got, ref, noise = [], [], []
    for b in bodies:
        if masses[b] <= 0:
            continue
        e = 1e-5 * masses[b]
        lp, lm = _oracle_loss(world, st, f, g, b, masses[b] + e), _oracle_loss(world, st, f, g, b, masses[b] - e)
        got.append(gm[same, b])
        ref.append(((lp - lm) / (2 * e))[same])
        # central-difference rounding of L through the step (~1e-14 |L|) / e
        noise.append(1e-14 * np.abs(lp).max() / e)
    assert got
    got, ref = np.stack(got, axis=1), np.stack(ref, axis=1)
    # 1e-6 relative to the largest mass gradient (per-element, with the
    # central differences' own rounding as the floor)
    err = np.abs(got - ref)
    bound = tol * np.abs(ref).max() + np.array(noise)[None, :]
    assert (err <= bound).all(), (err.max(axis=0), np.abs(ref).max(axis=0), noise)
    return gm


def test_mass_gradients_cartpole():
    """No contact: -dt (dID(q, v, a*)/dm_b)^T w only."""
    w = models.cartpole_world()
    st, f = models.random_states(w, 8, seed=2)
    _mass_parity(w, st, f)


def test_mass_gradients_atlas_air():
    """A floating base (FreeJoint) and a 35-body tree, no contact."""
    w = models.atlas_world(False)
    st, f = models.random_states(w, 4, seed=3, q_scale=0.2, v_scale=0.3)
    _mass_parity(w, st, f, bodies=[0, 1, 3, 5, 8, 20, 25, 30])


def test_mass_gradients_atlas_contact():
    """Feet on the ground: the LCP's M-dependence through Q and b (the
    M-derivative pairs of the position gradient, with d/dm_b)."""
    w = models.atlas_world(True)
    st, f = models.random_states(w, 8, seed=3, q_scale=0.01, v_scale=0.02)
    _mass_parity(w, st, f, bodies=[0, 2, 24, 27, 30, 33])


def test_mass_gradients_half_cheetah_contact():
    w = models.half_cheetah_world()
    st, f = models.half_cheetah_states(w, 16, seed=4)
    _mass_parity(w, st, f)


def test_timestep_layer_mass_argument():
    """nimble.timestep(world, state, action, mass) with tuned body masses:
    the forward uses them (next state = the oracle's with those masses) and
    mass.grad is the batch sum of the tuned bodies' lossWrtMass."""
    import nimblephysics_amd as nimble
    w = models.atlas_world(True)
    bodies = [b for s in w.skeletons for b in s.bodies]
    w.tuneMass(bodies[0], "INERTIA_MASS")
    w.tuneMass(bodies[27], "INERTIA_MASS")
    st, f = models.random_states(w, 6, seed=8, q_scale=0.01, v_scale=0.02)
    m0 = w.getMasses()
    mvals = m0 * np.array([1.1, 0.9])
    d = torch.device("cuda:0")
    mass = torch.tensor(mvals, device=d, requires_grad=True)
    ts = torch.tensor(st, device=d, requires_grad=True)
    tf = torch.tensor(f, device=d, requires_grad=True)
    out = nimble.timestep(w, ts, tf, mass)
    g = np.random.default_rng(1).standard_normal(st.shape)
    out.backward(torch.tensor(g, device=d))
    assert np.allclose(w.getMasses(), mvals)
    ow = O.OracleWorld(w)
    ref = ow.forward(st, f)
    assert np.abs(out.detach().cpu().numpy() - ref).max() <= 1e-9 * np.abs(ref).max()
    per = _mass_parity(w, st, f, seed=1, bodies=[0, 27])
    assert np.allclose(mass.grad.cpu().numpy(), per[:, [0, 27]].sum(0), rtol=1e-12, atol=0)


def test_backprop_snapshot_loss_wrt_mass():
    """neural.forwardPass(...).backpropState / backprop fill lossWrtMass
    [B, getMassDims()] (BackpropSnapshot.cpp:177, :418) with the same values
    as the batched mass gradient, and leave the state / action gradients as
    without tuned masses."""
    from nimblephysics_amd import neural
    w = models.atlas_world(True)
    bodies = [b for s in w.skeletons for b in s.bodies]
    w.tuneMass(bodies[27], "INERTIA_MASS")
    w.tuneMass(bodies[0], "INERTIA_MASS")
    st, f = models.random_states(w, 6, seed=9, q_scale=0.01, v_scale=0.02)
    d = torch.device("cuda:0")
    ts, tf = torch.tensor(st, device=d), torch.tensor(f, device=d)
    snap = neural.forwardPass(w, state=ts, action=tf)
    g = np.random.default_rng(3).standard_normal(st.shape)
    out = snap.backpropState(w, torch.tensor(g, device=d))
    assert tuple(out.lossWrtMass.shape) == (6, 2)
    per = _mass_parity(w, st, f, seed=3, bodies=[0, 27])
    assert np.allclose(out.lossWrtMass.cpu().numpy(), per[:, [27, 0]], rtol=1e-12, atol=0)
    this, nxt = neural.LossGradient(), neural.LossGradient()
    n = w.getNumDofs()
    nxt.lossWrtPosition = torch.tensor(g[:, :n], device=d)
    nxt.lossWrtVelocity = torch.tensor(g[:, n:], device=d)
    snap.backprop(w, this, nxt)
    assert torch.equal(this.lossWrtMass, out.lossWrtMass)
    assert torch.equal(torch.cat([this.lossWrtPosition, this.lossWrtVelocity], 1), out.lossWrtState)


def test_snapshot_state_is_copied():
    """The snapshot keeps its own copy of the step's state and forces: a
    caller reusing its buffers in place does not change later backprop."""
    from nimblephysics_amd import neural
    w = models.cartpole_world()
    st, f = models.random_states(w, 4, seed=2)
    d = torch.device("cuda:0")
    ts, tf = torch.tensor(st, device=d), torch.tensor(f, device=d)
    snap = neural.forwardPass(w, state=ts, action=tf)
    J0 = snap.getStateJacobian(w).clone()
    ts.add_(0.3)
    tf.mul_(2.0)
    snap2 = neural.forwardPass(w, state=torch.tensor(st, device=d), action=torch.tensor(f, device=d))
    assert torch.equal(snap2.getStateJacobian(w), J0)
    snap._jac = None
    assert torch.equal(snap.getStateJacobian(w), J0)


def test_constraint_force_getters_without_collision_pairs():
    """A contact-free model: no clamping rows, empty f_c and dF_c (the forward
    writes a zero snapshot header)."""
    from nimblephysics_amd import neural
    w = models.cartpole_world()
    st, f = models.random_states(w, 3, seed=1)
    d = torch.device("cuda:0")
    snap = neural.forwardPass(w, state=torch.tensor(st, device=d), action=torch.tensor(f, device=d))
    assert snap.getNumClamping().tolist() == [0, 0, 0]
    assert float(snap.getClampingConstraintImpulses().abs().sum()) == 0.0
    assert float(snap._snap[:, :8].abs().sum()) == 0.0
    w.setState(st[0])
    w.setControlForces(f[0])
    one = neural.forwardPass(w, idempotent=True)
    assert one.getClampingConstraintImpulses().shape == (0,)
    assert one.getJacobianOfConstraintForce(w, "POSITION").shape[0] == 0


def _set_param(body, p, val):
    """INERTIA_FULL component p of a body (WithRespectToMass.cpp:113)."""
    if p == 0:
        body.setMass(val)
    elif p < 4:
        c = body.com.copy()
        c[p - 1] = val
        body.setLocalCOM(c)
    else:
        I = body.moment.copy()
        I[p - 4] = val
        body.setMomentOfInertia(*I)


def _get_param(body, p):
    return body.mass if p == 0 else (body.com[p - 1] if p < 4 else body.moment[p - 4])


def _inertia_parity(world, st, f, bodies, seed=5, tol=1e-6):
    """nimble_backward_inertia's [B, nb, 10] against central differences of
    the oracle's step over each inertia parameter of `bodies`."""
    B = st.shape[0]
    ow = O.OracleWorld(world)
    ow.forward(st, f)
    nxt, snap, cache, ts, tf = _device_step(world, st, f)
    same = np.ones(B, dtype=bool)
    if world.native().num_pairs > 0:
        same = _check_contacts(ow, snap.cpu().numpy(), B, cache=cache.cpu().numpy())
    dev = world.native()
    g = np.random.default_rng(seed).standard_normal(st.shape)
    gt = torch.tensor(g, device=ts.device)
    gs, gf = torch.empty_like(ts), torch.empty_like(tf)
    gi = torch.empty((B, dev.nb, 10), dtype=torch.float64, device=ts.device)
    stream = torch.cuda.current_stream().cuda_stream
    dev.backward_inertia(ts, tf, snap, gt, gs, gf, gi, stream)
    gm = torch.empty((B, dev.nb), dtype=torch.float64, device=ts.device)
    gs2, gf2 = torch.empty_like(ts), torch.empty_like(tf)
    dev.backward_masses(ts, tf, snap, gt, gs2, gf2, gm, stream)
    torch.cuda.synchronize()
    assert torch.equal(gs, gs2) and torch.equal(gf, gf2)
    gi, gm = gi.cpu().numpy(), gm.cpu().numpy()
    assert np.allclose(gi[:, :, 0], gm, rtol=1e-12, atol=1e-14 * np.abs(gm).max())
    blist = [b for s in world.skeletons for b in s.bodies]
    got, ref, noise = [], [], []
    for bi in bodies:
        body = blist[bi]
        for p in range(10):
            v0 = _get_param(body, p)
            e = 1e-6 * max(abs(v0), 1e-2)
            try:
                _set_param(body, p, v0 + e)
                lp = (O.OracleWorld(world).forward(st, f) * g).sum(axis=1)
                _set_param(body, p, v0 - e)
                lm = (O.OracleWorld(world).forward(st, f) * g).sum(axis=1)
            finally:
                _set_param(body, p, v0)
            got.append(gi[same, bi, p])
            ref.append(((lp - lm) / (2 * e))[same])
            noise.append(1e-14 * np.abs(lp).max() / e)
    got, ref = np.stack(got, axis=1), np.stack(ref, axis=1)
    err = np.abs(got - ref)
    bound = tol * np.abs(ref).max() + 3 * np.array(noise)[None, :]
    assert (err <= bound).all(), (err.max(axis=0), np.abs(ref).max(axis=0), noise)


def test_inertia_gradients_cartpole():
    w = models.cartpole_world()
    st, f = models.random_states(w, 8, seed=2)
    _inertia_parity(w, st, f, bodies=[0, 1])


def test_inertia_gradients_atlas_air():
    w = models.atlas_world(False)
    st, f = models.random_states(w, 4, seed=3, q_scale=0.2, v_scale=0.3)
    _inertia_parity(w, st, f, bodies=[0, 5, 20, 30])


def test_inertia_gradients_atlas_contact():
    w = models.atlas_world(True)
    st, f = models.random_states(w, 8, seed=3, q_scale=0.01, v_scale=0.02)
    _inertia_parity(w, st, f, bodies=[0, 24, 33])


def test_inertia_gradients_half_cheetah_contact():
    w = models.half_cheetah_world()
    st, f = models.half_cheetah_states(w, 16, seed=4)
    _inertia_parity(w, st, f, bodies=[2, 4, 7])


def test_timestep_layer_inertia_entries():
    """timestep(world, state, action, mass) with COM / diagonal / COM_MU /
    FULL entries: mass.grad is the batch sum of the selected components."""
    import nimblephysics_amd as nimble
    w = models.atlas_world(True)
    bodies = [b for s in w.skeletons for b in s.bodies]
    bodies[27].setBeta([1.0, 0.5, 0.0])
    w.tuneMass(bodies[0], "INERTIA_COM")
    w.tuneMass(bodies[27], "INERTIA_DIAGONAL")
    w.tuneMass(bodies[27], "INERTIA_COM_MU")
    w.tuneMass(bodies[5], "INERTIA_FULL")
    st, f = models.random_states(w, 6, seed=8, q_scale=0.01, v_scale=0.02)
    d = torch.device("cuda:0")
    mass = torch.tensor(w.getMasses(), device=d, requires_grad=True)
    ts = torch.tensor(st, device=d, requires_grad=True)
    tf = torch.tensor(f, device=d, requires_grad=True)
    out = nimble.timestep(w, ts, tf, mass)
    g = np.random.default_rng(1).standard_normal(st.shape)
    out.backward(torch.tensor(g, device=d))
    dev = w.native()
    nxt, snap, cache, ts2, tf2 = _device_step(w, st, f)
    gi = torch.empty((6, dev.nb, 10), dtype=torch.float64, device=d)
    gs, gf = torch.empty_like(ts2), torch.empty_like(tf2)
    dev.backward_inertia(ts2, tf2, snap, torch.tensor(g, device=d), gs, gf, gi, torch.cuda.current_stream().cuda_stream)
    gi = gi.sum(0).cpu().numpy()
    want = np.concatenate([gi[0, 1:4], gi[27, 4:7], [gi[27, 1] * 1.0 + gi[27, 2] * 0.5], gi[5, :]])
    assert np.allclose(mass.grad.cpu().numpy(), want, rtol=1e-12, atol=1e-14 * np.abs(want).max())
