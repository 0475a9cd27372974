"""The 3-dof joints on the device: BallJoint (dart/dynamics/BallJoint.cpp,
exponential coordinates with the identity Jacobian of the reference's build:
T = T_pj expMapRot(q) T_cj^-1, S = Ad(T_cj)[I; 0], integration log(exp(q)
exp(dq dt)), posPos / velPos blocks by central differences :368 / :390) and
TranslationalJoint (TranslationalJoint.cpp: Translation(q), S = [0; R_cj],
Euclidean integration and blocks), on a rig with a translational root, two
ball joints and a revolute ankle (tests/models.py ball_world), against the
oracle: contact sets bit-exact, LCP path, next state and gradients at
BASELINE's 1e-6 per element (test_gpu_contact_parity._parity), the step
Jacobians (the BallJoint FD blocks bit-identical, as the FreeJoint's), and
the C-ABI's rollout.  The oracle's own gradients for this rig are pinned
against central differences of its step (test_oracle_pins.py
test_ball_translational_gradients_vs_finite_differences)."""
import numpy as np
import pytest

import models
from oracle import oracle as O
from test_gpu_contact_parity import RTOL, _parity
from test_gpu_jacobians import _batched, _fd_mask, _jac_err

pytestmark = pytest.mark.gpu

# UniversalJoint / EulerJoint / PlanarJoint go to the device as their 1-dof
# chains through massless frames (dynamics.Joint.chain); the chains'
# transforms are pinned to the reference's formulas and the oracle's
# gradients to central differences in test_oracle_pins.py (compound_*)
RIGS = {"ball": (models.ball_world, models.ball_states), "compound": (models.compound_world, models.compound_states)}


@pytest.mark.parametrize("rig", sorted(RIGS))
@pytest.mark.parametrize("contact", [False, True])
def test_rig_parity(rig, contact):
    make, states = RIGS[rig]
    world = make(ground=contact)
    st, f = states(128, seed=21, contact=contact)
    ow, snap = _parity(world, st, f)
    if contact:
        assert (snap[:, 0] > 0).mean() > 0.9  # the foot on the ground


@pytest.mark.parametrize("rig", sorted(RIGS))
@pytest.mark.parametrize("contact", [False, True])
def test_rig_jacobians(rig, contact):
    make, states = RIGS[rig]
    world = make(ground=contact)
    st, f = states(32, seed=5, contact=contact)
    ow = O.OracleWorld(world)
    ow.forward(st, f)
    RJ, RF = ow.jacobians()
    snap, ts, tf = _batched(world, st, f)
    J = snap.getStateJacobian(world).cpu().numpy()
    F = snap.getActionJacobian(world).cpu().numpy()
    mask = _fd_mask(world)
    assert mask.sum() == (2 * 2 * 9 if rig == "ball" else 0)  # ball joints: 3 x 3 posPos and velPos blocks
    checked = 0
    for b in range(st.shape[0]):
        fl = O.lcp_flags(ow, b)
        sn = snap._snap[b].cpu().numpy() if hasattr(snap, "_snap") else None
        if sn is not None and (sn[6], sn[4]) != (fl[0], fl[2]):
            continue  # another LCP path (ambiguous problems are judged in test_ball_rig_parity)
        rel, fd = _jac_err(J[b], RJ[b], mask)
        assert rel < RTOL and fd == 0.0, (b, rel, fd)
        assert _jac_err(F[b], RF[b], np.zeros_like(F[b], dtype=bool))[0] < RTOL, b
        checked += 1
    assert checked >= st.shape[0] - 2
