"""nimble.neural on the batched device path: forwardPass and BackpropSnapshot.

Mirrors dart/neural/NeuralUtils.cpp:26 (``forwardPass(world, idempotent)``)
and dart/neural/BackpropSnapshot.hpp as bound in
python/_nimblephysics/simulation_and_neural/BackpropSnapshot.cpp: the
snapshot of a step answers ``backpropState``, ``backprop`` and the Jacobian
getters (``getStateJacobian`` :1230, ``getActionJacobian`` :1245,
``getPosPosJacobian`` :1263, ``getPosVelJacobian`` :762, ``getVelPosJacobian``
:1338, ``getVelVelJacobian`` :643, ``getControlForceVelJacobian`` :482).

Batched: ``forwardPass(world, state=[B, 2n], action=[B, |A|])`` steps B
independent worlds in one launch and returns one snapshot object for all of
them; its getters return [B, ...] device tensors.  ``forwardPass(world)``
(the reference's form) steps the world's own state and returns 2-D numpy
matrices, as the reference's Eigen matrices come back to Python.

The Jacobians are formed on the device as 2n vector-Jacobian products per
world (the backward kernel driven with unit upstream gradients, one launch
for all B*2n rows) -- the very matrices whose transposed products
``backpropState`` applies -- and cached on the snapshot.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from . import _native
from .simulation import World
from .timestep import _action_index, _compute_device, mass_gradient, step_batch


class LossGradient:
    """dart/neural/BackpropSnapshot.hpp LossGradient."""

    def __init__(self):
        self.lossWrtPosition = None
        self.lossWrtVelocity = None
        self.lossWrtTorque = None
        self.lossWrtMass = None


class LossGradientHighLevelAPI:
    """dart/neural/BackpropSnapshot.hpp LossGradientHighLevelAPI."""

    def __init__(self):
        self.lossWrtState = None
        self.lossWrtAction = None
        self.lossWrtMass = None


class BackpropSnapshot:
    """The batched BackpropSnapshot of one forward launch over B worlds."""

    def __init__(self, world: World, dev, state, forces, next_state, snapshot, single: bool):
        self._world = world
        self._dev = dev
        # copies: the caller may reuse or update its state / action buffers in
        # place before the lazily computed Jacobians and backprop read them
        self._state = state.clone()
        self._forces = forces.clone()
        self._next = next_state
        self._snap = snapshot
        self._single = single
        self._n = world.getNumDofs()
        self._jac = None
        self._fcjac = None

    # --- output shaping: [B, ...] device tensors, or 2-D numpy for forwardPass(world)
    def _out(self, t):
        if self._single:
            return t[0].detach().cpu().numpy()
        return t

    def _check_world(self, world):
        if world is not None and world is not self._world:
            raise ValueError("snapshot belongs to another world")
        if self._dev.h is None:
            raise RuntimeError("the world model that produced this snapshot was released")

    def _jacobians(self):
        if self._jac is None:
            with torch.cuda.device(self._state.device):
                stream = torch.cuda.current_stream(self._state.device).cuda_stream
                self._jac = self._dev.jacobians(self._state, self._forces, self._snap, stream)
        return self._jac

    # --- Jacobians (BackpropSnapshot.cpp) ---------------------------------------
    def getStateJacobian(self, world: Optional[World] = None):
        """d(next state)/d(state), [[posPos, velPos], [posVel, velVel]] (:1230)."""
        self._check_world(world)
        return self._out(self._jacobians()[0])

    def getActionJacobian(self, world: Optional[World] = None):
        """d(next state)/d(action) [2n, |A|]: forceVel columns of the action
        space under zero position rows (:1245)."""
        self._check_world(world)
        F = self._jacobians()[1]
        idx = _action_index(self._world, F.device)
        A = torch.zeros((F.shape[0], 2 * self._n, idx.shape[0]), dtype=F.dtype, device=F.device)
        A[:, self._n:, :] = F[:, self._n:, :].index_select(2, idx)
        return self._out(A)

    def getPosPosJacobian(self, world: Optional[World] = None):
        self._check_world(world)
        n = self._n
        return self._out(self._jacobians()[0][:, :n, :n])

    def getVelPosJacobian(self, world: Optional[World] = None):
        """d(next position)/d(velocity) (:1338)."""
        self._check_world(world)
        n = self._n
        return self._out(self._jacobians()[0][:, :n, n:])

    def getPosVelJacobian(self, world: Optional[World] = None):
        """d(next velocity)/d(position) (:762)."""
        self._check_world(world)
        n = self._n
        return self._out(self._jacobians()[0][:, n:, :n])

    def getVelVelJacobian(self, world: Optional[World] = None):
        self._check_world(world)
        n = self._n
        return self._out(self._jacobians()[0][:, n:, n:])

    def getControlForceVelJacobian(self, world: Optional[World] = None):
        """d(next velocity)/d(control forces) [n, n] (:482)."""
        self._check_world(world)
        n = self._n
        return self._out(self._jacobians()[1][:, n:, :])

    # --- constraint forces (BackpropSnapshot.cpp:2723) --------------------------
    def _clamping_counts(self):
        """Clamping rows per world, clamped to [0, MAX_LCP]; zeros for a model
        without collision pairs (whose snapshot has no contact region)."""
        from ._native import MAX_LCP, SN_NC
        if self._dev.num_pairs == 0:
            return torch.zeros(self._state.shape[0], dtype=torch.int64, device=self._state.device)
        return self._snap[:, SN_NC].to(torch.int64).clamp(0, MAX_LCP)

    def getClampingConstraintImpulses(self):
        """f_c, the clamping rows' impulses in the LCP's clamping order:
        [B, MAX_LCP] (zero past each world's count), or [n_c] for one world."""
        from ._native import MAX_LCP, SN_FC
        nc = self._clamping_counts()
        if self._dev.num_pairs == 0:
            fc = torch.zeros((self._state.shape[0], MAX_LCP), dtype=torch.float64, device=self._state.device)
        else:
            fc = self._snap[:, SN_FC:SN_FC + MAX_LCP].clone()
            fc[torch.arange(MAX_LCP, device=fc.device)[None, :] >= nc[:, None]] = 0.0
        if self._single:
            return fc[0, :int(nc[0])].detach().cpu().numpy()
        return fc

    def getJacobianOfConstraintForce(self, world: Optional[World] = None, wrt: str = "POSITION"):
        """d f_c / d wrt for wrt in POSITION / VELOCITY / FORCE (:2723):
        [B, MAX_LCP, n] device tensor (rows past each world's clamping count
        zero), or [n_c, n] for one world."""
        self._check_world(world)
        kind = getattr(wrt, "name", wrt)
        if self._fcjac is None:
            with torch.cuda.device(self._state.device):
                stream = torch.cuda.current_stream(self._state.device).cuda_stream
                self._fcjac = self._dev.constraint_force_jacobians(self._state, self._forces, self._snap, stream)
        Js, Jf = self._fcjac
        n = self._n
        J = {"POSITION": Js[:, :, :n], "VELOCITY": Js[:, :, n:], "FORCE": Jf}.get(kind)
        if J is None:
            raise ValueError(f"wrt must be POSITION, VELOCITY or FORCE, got {kind}")
        if self._single:
            return J[0, :int(self._clamping_counts()[0])].detach().cpu().numpy()
        return J

    # --- backprop (BackpropSnapshot.cpp:121, :382) ------------------------------
    def _vjp(self, grad_next):
        """(lossWrtState, lossWrtForces, lossWrtMass): the mass part is
        getMassVelJacobian^T dL/dv' (BackpropSnapshot.cpp:177, :418) for the
        world's tuned masses, [B, getMassDims()]."""
        g = grad_next.reshape(self._state.shape).to(self._state.device, torch.float64).contiguous()
        gs = torch.empty_like(self._state)
        gf = torch.empty_like(self._forces)
        B = self._state.shape[0]
        with torch.cuda.device(self._state.device):
            stream = torch.cuda.current_stream(self._state.device).cuda_stream
            if self._world.getMassDims() > 0:
                gm = mass_gradient(self._dev, self._world._mass_selection(), self._state, self._forces, self._snap, g,
                                   gs, gf, stream)
            else:
                self._dev.backward(self._state, self._forces, self._snap, g, gs, gf, stream)
                gm = torch.zeros((B, 0), dtype=torch.float64, device=self._state.device)
        return gs, gf, gm

    def backpropState(self, world: Optional[World], nextTimestepStateLossGrad) -> LossGradientHighLevelAPI:
        """lossWrtState [2n], lossWrtAction [|A|], lossWrtMass [getMassDims()]."""
        self._check_world(world)
        g = torch.as_tensor(np.asarray(nextTimestepStateLossGrad) if not torch.is_tensor(nextTimestepStateLossGrad)
                            else nextTimestepStateLossGrad, dtype=torch.float64)
        gs, gf, gm = self._vjp(g)
        idx = _action_index(self._world, gf.device)
        out = LossGradientHighLevelAPI()
        out.lossWrtState = self._out(gs)
        out.lossWrtAction = self._out(gf.index_select(1, idx))
        out.lossWrtMass = self._out(gm)
        return out

    def backprop(self, world: Optional[World], thisTimestepLoss: LossGradient, nextTimestepLoss: LossGradient):
        """Fills thisTimestepLoss from nextTimestepLoss (lossWrtPosition /
        lossWrtVelocity) as the reference's backprop does."""
        self._check_world(world)
        gp = torch.as_tensor(np.asarray(nextTimestepLoss.lossWrtPosition) if not torch.is_tensor(
            nextTimestepLoss.lossWrtPosition) else nextTimestepLoss.lossWrtPosition, dtype=torch.float64)
        gv = torch.as_tensor(np.asarray(nextTimestepLoss.lossWrtVelocity) if not torch.is_tensor(
            nextTimestepLoss.lossWrtVelocity) else nextTimestepLoss.lossWrtVelocity, dtype=torch.float64)
        B = self._state.shape[0]
        g = torch.cat([gp.reshape(B, -1), gv.reshape(B, -1)], dim=1)
        gs, gf, gm = self._vjp(g)
        n = self._n
        thisTimestepLoss.lossWrtPosition = self._out(gs[:, :n])
        thisTimestepLoss.lossWrtVelocity = self._out(gs[:, n:])
        thisTimestepLoss.lossWrtTorque = self._out(gf)
        thisTimestepLoss.lossWrtMass = self._out(gm)

    # --- recorded state (BackpropSnapshot.cpp:1403-1445, :1685-1702) -----------
    def getPreStepPosition(self):
        return self._out(self._state[:, :self._n])

    def getPreStepVelocity(self):
        return self._out(self._state[:, self._n:])

    def getPreStepTorques(self):
        return self._out(self._forces)

    def getPostStepPosition(self):
        return self._out(self._next[:, :self._n])

    def getPostStepVelocity(self):
        return self._out(self._next[:, self._n:])

    def getPostStepTorques(self):
        # the step's torques; the reference's world clears them afterwards
        return self._out(self._forces)

    def _header(self, k):
        if self._dev.num_pairs == 0:
            return self._out(torch.zeros(self._state.shape[0], dtype=torch.int64, device=self._state.device))
        return self._out(self._snap[:, k].to(torch.int64))

    def getNumContacts(self):
        return self._header(_native.SN_NCON)

    def getNumClamping(self):
        return self._header(_native.SN_NC)

    def getNumUpperBound(self):
        return self._header(_native.SN_NU)

    def getStatus(self):
        """Per-world status bits (see World.getLastStatus)."""
        return self._out(self._dev.status(self._snap))


def forwardPass(world: World, idempotent: bool = False, state=None, action=None) -> BackpropSnapshot:
    """neural::forwardPass (NeuralUtils.cpp:26).

    ``forwardPass(world)`` steps the world's own state and control forces (the
    reference's call: afterwards the world holds the next state and its
    control forces are cleared, unless ``idempotent``, which restores the
    pre-step state).  ``forwardPass(world, state=S, action=A)`` with device
    tensors [B, 2n] / [B, |A|] steps B worlds and leaves the world object
    untouched."""
    if state is None:
        single = True
        dev = _compute_device(torch.zeros(0))
        st = torch.tensor(world.getState(), dtype=torch.float64, device=dev).reshape(1, -1)
        act = torch.tensor(world.getAction(), dtype=torch.float64, device=dev).reshape(1, -1)
    else:
        single = False
        if action is None:
            raise ValueError("forwardPass with a batched state needs the batched action")
        st = state.detach().to(torch.float64)
        act = action.detach().to(torch.float64)
        if st.dim() == 1:
            st, act = st.reshape(1, -1), act.reshape(1, -1)
        if not st.is_cuda:
            raise RuntimeError("batched forwardPass takes device tensors")
        dev = st.device
        st, act = st.contiguous(), act.contiguous()
    prev = getattr(world, "_batch_state", None)
    saved = prev.cache.clone() if (idempotent and prev is not None) else None
    try:
        with torch.cuda.device(dev):
            devworld, forces, nxt, snap = step_batch(world, st, act)
    finally:
        if idempotent:
            # RestorableSnapshot: the LCP warm-start cache is part of the world
            # state the idempotent pass restores (NeuralUtils.cpp:26), also
            # when the step raised
            if saved is None:
                world._batch_state = prev
            else:
                prev.cache.copy_(saved)
                world._batch_state = prev
    if single and not idempotent:
        out = nxt[0].cpu().numpy()
        world.setState(out)
        world.setControlForces(np.zeros(world.getNumDofs()))
    snapshot = BackpropSnapshot(world, devworld, st, forces, nxt, snap, single)
    world._cached_snapshot = snapshot
    return snapshot
