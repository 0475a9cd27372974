"""BackpropSnapshot Jacobian getters on the device (nimble_jacobians) against
the oracle's dense matrices (oracle_step.cpp stepJacobians: the reference's
getPosPosJacobian / getPosVelJacobian / getVelPosJacobian / getVelVelJacobian
/ getControlForceVelJacobian, BackpropSnapshot.cpp:1263/:762/:1338/:643/:482,
assembled as getStateJacobian :1230 and getActionJacobian :1245).

Tolerance: BASELINE.json's 1e-6 relative, per element, with an absolute
floor of 1e-3 x the matrix's largest entry (see test_gpu_contact_parity._rel).
"""
import numpy as np
import pytest
import torch

import models
import nimblephysics_amd as nimble
from oracle import oracle as O
from test_gpu_contact_parity import RTOL, _check_contacts, _rel

pytestmark = pytest.mark.gpu


# FreeJoint's posPos / velPos blocks are central differences in the
# reference itself (FreeJoint::finiteDifferencePosPosJacobian / VelPos,
# FreeJoint.cpp:965, :987, eps 1e-6 / 1e-7).  The device and the oracle
# evaluate their perturbed integrations as one fixed IEEE operation sequence
# (spatial.cuh fdFreeIntegrate / nimble_oracle.cpp), so those entries must be
# equal bit for bit; every other entry is compared at RTOL per element.


def _fd_mask(world):
    d = world.desc_arrays()
    n = world.getNumDofs()
    mask = np.zeros((2 * n, 2 * n), dtype=bool)
    for b, jt in enumerate(d["joint_type"]):
        if int(jt) in (3, 4):  # FreeJoint (6 coordinates), BallJoint (3: BallJoint.cpp:368, :390)
            o, k = int(d["dof_offset"][b]), 6 if int(jt) == 3 else 3
            mask[o:o + k, o:o + k] = True          # posPos
            mask[o:o + k, n + o:n + o + k] = True  # velPos
    return mask


def _jac_err(J, R, mask):
    """(per-element relative error off the FD blocks, max abs error on them:
    0 when they are bit-identical)."""
    Jm, Rm = np.where(mask, 0.0, J), np.where(mask, 0.0, R)
    return _rel(Jm, Rm), float(np.abs(J - R)[mask].max(initial=0.0))


def _batched(world, st, f, caches=None):
    d = torch.device("cuda:0")
    ts, tf = torch.tensor(st, device=d), torch.tensor(f, device=d)
    world._batch_state = None  # cold LCP caches, as the oracle's
    if caches is not None:
        world.setCachedLCPSolution(caches)
    snap = nimble.neural.forwardPass(world, state=ts, action=tf)
    torch.cuda.synchronize()
    return snap, ts, tf


@pytest.mark.parametrize("name", ["cartpole", "kr5", "atlas_air"])
def test_state_action_jacobians_no_contact(name):
    world = {"cartpole": models.cartpole_world, "kr5": models.kr5_world,
             "atlas_air": lambda: models.atlas_world(False)}[name]()
    st, f = models.random_states(world, 16, seed=4)
    ow = O.OracleWorld(world)
    ow.forward(st, f)
    RJ, RF = ow.jacobians()
    snap, ts, tf = _batched(world, st, f)
    J = snap.getStateJacobian(world).cpu().numpy()
    F = snap.getActionJacobian(world).cpu().numpy()
    assert J.shape == RJ.shape and F.shape == RF.shape
    mask = _fd_mask(world)
    for b in range(st.shape[0]):
        rel, fd = _jac_err(J[b], RJ[b], mask)
        assert rel < RTOL and fd == 0.0, (b, rel, fd)
        assert _rel(F[b], RF[b]) < RTOL, (b, _rel(F[b], RF[b]))
    n = world.getNumDofs()
    # the blocks are views of the same matrices
    np.testing.assert_array_equal(snap.getVelVelJacobian(world).cpu().numpy(), J[:, n:, n:])
    np.testing.assert_array_equal(snap.getPosVelJacobian(world).cpu().numpy(), J[:, n:, :n])
    np.testing.assert_array_equal(snap.getControlForceVelJacobian(world).cpu().numpy(), F[:, n:, :])


def test_state_action_jacobians_atlas_contact():
    """1024 Atlas worlds on the ground (the bench batch): 67,584 Jacobian rows
    in one launch, more than the 65,536-workgroup grid, so the kernel's
    grid-stride loop runs; compared with the oracle on every world on the
    oracle's LCP path."""
    world = models.atlas_world(True)
    B = 1024
    st, f = models.random_states(world, B, seed=1000, q_scale=0.02, v_scale=0.05)
    ow = O.OracleWorld(world)
    ow.forward(st, f)
    RJ, RF = ow.jacobians()
    snap, ts, tf = _batched(world, st, f)
    sn = world._last_snapshot.cpu().numpy()
    same = _check_contacts(ow, sn, B, cache=world._batch_state.cache.cpu().numpy())
    J = snap.getStateJacobian(world).cpu().numpy()
    F = snap.getActionJacobian(world).cpu().numpy()
    assert (sn[:, 0] > 0).mean() > 0.5
    mask = _fd_mask(world)
    errs = np.array([_jac_err(J[b], RJ[b], mask) for b in np.flatnonzero(same)])
    worstF = max(_rel(F[b], RF[b]) for b in np.flatnonzero(same))
    assert errs[:, 0].max() < RTOL and errs[:, 1].max() == 0.0 and worstF < RTOL, (errs.max(0), worstF)
    # the Jacobian is the matrix whose transposed product backpropState
    # applies (no clipping at these interior states)
    g = torch.tensor(np.random.default_rng(2).standard_normal(st.shape), device=ts.device)
    out = snap.backpropState(world, g)
    vjp = torch.einsum("bij,bi->bj", torch.tensor(J, device=ts.device), g)
    assert _rel(out.lossWrtState.cpu().numpy(), vjp.cpu().numpy()) < 1e-8


def test_world_jacobians_single():
    """World.getStateJacobian / getActionJacobian (World.cpp:2210 / :2227):
    idempotent at the world's current state, 2-D numpy like the reference."""
    world = models.kr5_world()
    n = world.getNumDofs()
    rng = np.random.default_rng(3)
    world.setPositions(rng.standard_normal(n) * 0.3)
    world.setVelocities(rng.standard_normal(n) * 0.3)
    world.setControlForces(rng.standard_normal(n))
    s0 = world.getState().copy()
    J = world.getStateJacobian()
    A = world.getActionJacobian()
    assert J.shape == (2 * n, 2 * n) and A.shape == (2 * n, world.getActionSize())
    np.testing.assert_array_equal(world.getState(), s0)  # idempotent
    ow = O.OracleWorld(world)
    ow.forward(s0[None], world.getControlForces()[None])
    RJ, RF = ow.jacobians()
    assert _rel(J, RJ[0]) < RTOL and _rel(A, RF[0]) < RTOL


@pytest.mark.parametrize("name", ["atlas", "half_cheetah", "capsule_edge", "atlas_broken", "atlas_mesh_broken"])
def test_constraint_force_jacobians(name):
    """getClampingConstraintImpulses and getJacobianOfConstraintForce for
    POSITION / VELOCITY / FORCE (BackpropSnapshot.cpp:2723;
    nimble_constraint_force_jacobians: unit upstream gradients on f_c through
    the backward kernel) against the oracle's dense dF_c (oracle_contact.cpp
    constrainedJacobians, itself checked against finite differences in
    test_oracle_pins), on every world of the oracle's LCP path."""
    if name == "atlas":
        world = models.atlas_world(True)
        st, f = models.random_states(world, 256, seed=7, q_scale=0.02, v_scale=0.05)
    elif name == "half_cheetah":
        world = models.half_cheetah_world()
        st, f = models.half_cheetah_states(world, 128, seed=4)
    elif name == "capsule_edge":
        world = models.capsule_edge_world()
        st, f = models.capsule_edge_states(64, seed=2)
    else:
        world, _, st, f, caches = models.broken_states("atlas_mesh" if name == "atlas_mesh_broken" else "atlas")
    n = world.getNumDofs()
    B = st.shape[0]
    ow = O.OracleWorld(world)
    if name == "atlas_mesh_broken":
        # the tests' 96-entry warm starts (World::setCachedLCPSolution)
        from test_oracle_pins import _seed_caches
        _seed_caches(ow, caches)
    ow.forward(st, f)
    RD = ow.constraint_force_jacobians()
    snap, ts, tf = _batched(world, st, f, caches if name == "atlas_mesh_broken" else None)
    sn = world._last_snapshot.cpu().numpy()
    same = _check_contacts(ow, sn, B, cache=world._batch_state.cache.cpu().numpy())
    fc = snap.getClampingConstraintImpulses().cpu().numpy()
    Jq = snap.getJacobianOfConstraintForce(world, "POSITION").cpu().numpy()
    Jv = snap.getJacobianOfConstraintForce(world, "VELOCITY").cpu().numpy()
    Jf = snap.getJacobianOfConstraintForce(world, "FORCE").cpu().numpy()
    checked = 0
    for b in np.flatnonzero(same):
        nc = int(sn[b, 2])
        assert not np.any(Jq[b, nc:]) and not np.any(Jf[b, nc:])
        if nc == 0:
            continue
        assert _rel(fc[b, :nc], O.lcp_fc(ow, b)[:nc]) < RTOL, b
        got = np.concatenate([Jq[b, :nc], Jv[b, :nc], Jf[b, :nc]], axis=1)
        assert _rel(got, RD[b, :nc]) < RTOL, (b, _rel(got, RD[b, :nc]))
        checked += 1
    assert checked >= 1
