"""nimble.timestep(world, state, action) as a torch.autograd.Function.

Mirrors python/nimblephysics/timestep.py:13 (TimestepLayer) and :59
(timestep): forward = neural::forwardPass(world) (World::step), backward =
BackpropSnapshot::backpropState.  The reference takes a 1-D state and round
trips through numpy on the CPU; here state/action are float64 device tensors,
either 1-D (one world) or 2-D [batch, ...] (independent worlds sharing the
model), and the whole batch is one kernel launch each way.

World-side effects match the reference for the 1-D case: the world's
positions/velocities are set to the returned state and the control forces are
cleared (World::step(resetCommand=true) via forwardPass(world)).

CPU tensors (what the reference's layer takes, timestep.py:31 calls
``state.detach().numpy()``) are accepted as a drop-in convenience: they are
staged to the current HIP device, stepped by the same kernels, and the
results / gradients come back on the CPU.  There is no CPU compute path --
without a HIP device the call raises.

Status: worlds whose contact set does not fit this path (more contacts than
NIMBLE_MAX_CONTACTS, a shape pair without a collider) would step differently
from the reference, so under the world's default status policy ('raise') the
call raises ContactCapacityError naming them; ``world.getLastStatus()`` holds
the per-world status bits of the last call either way.

``mass`` is the reference's tuned-mass vector (World::getMassDims entries,
registered with World::tuneMass(body, INERTIA_MASS), set with
World::setMasses before the step): 1-D, shared by every world of the batch
(the device model is rebuilt when it changes).  Its gradient is lossWrtMass
(BackpropSnapshot::getMassVelJacobian^T dL/dv', nimble_backward_masses),
summed over the batch for a batched state.
"""
from __future__ import annotations

from typing import Optional

import torch

from ._native import ContactCapacityError, ST_DIVERGES, status_message
from .simulation import World


class BatchState:
    """Per-world LCP warm-start caches (BoxedLcpConstraintSolver::mX) for a batch."""

    def __init__(self, batch: int, cache_doubles: int, device):
        self.batch = batch
        self.cache = torch.zeros((batch, cache_doubles), dtype=torch.float64, device=device)
        self.cache[:, 0] = -1.0  # empty cache


def _action_index(world: World, device) -> torch.Tensor:
    """Device copy of the action space's dof indices, made once per world and
    device (a pageable host->device copy per step would serialise the host
    with the stream)."""
    space = tuple(world.getActionSpace())
    cached = getattr(world, "_action_index", None)
    if cached is None or cached[0] != space or cached[1].device != device:
        cached = (space, torch.tensor(space, dtype=torch.long, device=device))
        world._action_index = cached
    return cached[1]


def _identity_action(world: World, n: int) -> bool:
    """True when the action space is every dof in order (the default), so
    actions are the control forces themselves."""
    space = world.getActionSpace()
    return len(space) == n and all(int(a) == k for k, a in enumerate(space))


def _batch_state(world: World, batch: int, dev, device) -> BatchState:
    bs = getattr(world, "_batch_state", None)
    if bs is None or bs.batch != batch or bs.cache.device != device or bs.cache.shape[1] != dev.cache_doubles:
        bs = BatchState(batch, dev.cache_doubles, device)
        world._batch_state = bs
    pending = getattr(world, "_pending_lcp_cache", None)
    if pending is not None:
        # World::setCachedLCPSolution: one vector for every world, or one per
        # world; every vector is checked before any cache row is written, and
        # a rejected value is dropped (it would fail every later step too)
        world._pending_lcp_cache = None
        if len(pending) not in (1, batch):
            raise ValueError(f"setCachedLCPSolution: {len(pending)} vectors for a batch of {batch}")
        cap = dev.cache_doubles - 1
        for r in pending:
            if r is not None and len(r) > cap:
                raise ValueError(f"cached LCP solution of {len(r)} rows; this model holds at most {cap}")
        for b in range(batch):
            r = pending[b if len(pending) > 1 else 0]
            bs.cache[b, 0] = -1.0 if r is None else float(len(r))
            if r is not None and len(r):
                bs.cache[b, 1:1 + len(r)] = torch.as_tensor(r, dtype=torch.float64, device=device)
    return bs


def _compute_device(t: torch.Tensor) -> torch.device:
    if t.device.type != "cpu":
        return t.device
    if not torch.cuda.is_available():
        raise RuntimeError("nimblephysics_amd.timestep runs on a HIP device (MI355X); no GPU is visible "
                           "and there is no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def _check_status(world: World, dev, snap: torch.Tensor) -> None:
    """Record the per-world status bits; under the 'raise' policy, fail loudly
    on worlds whose step cannot be the reference's (one host sync)."""
    status = dev.status(snap)
    world._last_status = status
    if dev.num_pairs == 0 or world.getStatusPolicy() != "raise":
        return
    bad = (status & ST_DIVERGES) != 0
    if bool(bad.any()):
        idx = torch.nonzero(bad).flatten().tolist()
        bits = 0
        for v in status[bad].tolist():
            bits |= int(v)
        raise ContactCapacityError(
            f"{len(idx)} world(s) {idx[:8]}{'...' if len(idx) > 8 else ''}: {status_message(bits)}; "
            f"their step would differ from the reference's (world.setStatusPolicy('record') to continue anyway)")


def step_batch(world: World, st: torch.Tensor, act: torch.Tensor):
    """One batched forward launch (neural::forwardPass on every row of the
    2-D device tensors `st` [B, 2n] / `act` [B, |action space|]).  Returns
    (device world, forces [B, n], next state [B, 2n], snapshot [B, S]); the
    world's LCP warm-start caches advance and its status word is checked."""
    B = st.shape[0]
    n = world.getNumDofs()
    if st.shape[1] != 2 * n:
        raise ValueError(f"state has {st.shape[1]} columns, world expects {2 * n}")
    idx = _action_index(world, st.device)
    if act.shape[1] != idx.shape[0]:
        raise ValueError(f"action has {act.shape[1]} columns, action space has {idx.shape[0]}")
    dev = world.native(st.device)
    if _identity_action(world, n):
        forces = act.contiguous()  # every dof actuated, in order: no scatter
    else:
        forces = torch.zeros((B, n), dtype=torch.float64, device=st.device)
        forces.index_copy_(1, idx, act.contiguous())
    bs = _batch_state(world, B, dev, st.device)
    nxt = torch.empty_like(st)
    snap = torch.empty((B, dev.snapshot_doubles), dtype=torch.float64, device=st.device)
    stream = torch.cuda.current_stream(st.device).cuda_stream
    dev.forward(st, forces, bs.cache, nxt, snap, stream)
    world._last_snapshot = snap  # the batched BackpropSnapshot of this step
    _check_status(world, dev, snap)
    return dev, forces, nxt, snap


def mass_gradient(dev, selection, st, forces, snap, g, gs, gf, stream):
    """lossWrtMass [B, getMassDims()] (with the state / force gradients into
    gs / gf): nimble_backward_masses when only body masses are tuned, else
    nimble_backward_inertia's ten parameters per body taken to the mass
    vector by World._mass_selection's matrix."""
    only_masses, sel = selection
    B = st.shape[0]
    if only_masses:
        gmb = torch.empty((B, dev.nb), dtype=torch.float64, device=st.device)
        dev.backward_masses(st, forces, snap, g, gs, gf, gmb, stream)
        return gmb.index_select(1, torch.tensor(sel, dtype=torch.long, device=st.device))
    gi = torch.empty((B, dev.nb, 10), dtype=torch.float64, device=st.device)
    dev.backward_inertia(st, forces, snap, g, gs, gf, gi, stream)
    return gi.reshape(B, dev.nb * 10) @ torch.as_tensor(sel, dtype=torch.float64, device=st.device)


class TimestepLayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, world: World, state: torch.Tensor, action: torch.Tensor, mass: Optional[torch.Tensor]):
        # `mass` follows the reference (timestep.py:34, world.setMasses): the
        # world's getMassDims() tuned body masses, one vector for the batch
        ctx.use_mass = mass is not None
        if ctx.use_mass:
            if mass.dim() != 1 or mass.shape[0] != world.getMassDims():
                raise ValueError(f"mass must be a vector of the world's {world.getMassDims()} tuned masses "
                                 f"(World::tuneMass), got shape {tuple(mass.shape)}")
            # one host round trip only when the masses may have changed: the
            # same tensor object (held here, so its id cannot be reused) at the
            # same in-place version on an unchanged world model is skipped
            last = getattr(world, "_last_mass", None)
            if last is None or last[0] is not mass or last[1] != mass._version or last[2] != world._version:
                world.setMasses(mass.detach().cpu().numpy())
                world._last_mass = (mass, mass._version, world._version)
            ctx.mass_shape = tuple(mass.shape)
            ctx.mass_device = mass.device
            ctx.mass_sel = world._mass_selection()
        ctx.out_device = state.device
        cdev = _compute_device(state)
        with torch.cuda.device(cdev):
            state = state.to(cdev, torch.float64)
            action = action.to(cdev, torch.float64)
            squeeze = state.dim() == 1
            st = state.detach().reshape(1, -1) if squeeze else state.detach()
            act = action.detach().reshape(1, -1) if squeeze else action.detach()
            st = st.contiguous()
            n = world.getNumDofs()
            dev, forces, nxt, snap = step_batch(world, st, act)
            idx = _action_index(world, st.device)
        ctx.world = world
        ctx.identity = _identity_action(world, world.getNumDofs())
        # the backward must run on the model (and snapshot layout) that
        # produced this snapshot, even if the world changes in between
        ctx.dev = dev
        ctx.squeeze = squeeze
        ctx.save_for_backward(st, forces, snap, idx)
        if squeeze:
            # World::step side effects on the single world
            out_cpu = nxt[0].cpu().numpy()
            world.setState(out_cpu)
            world.setControlForces(out_cpu[:n] * 0.0)
            return nxt[0].to(ctx.out_device)
        return nxt.to(ctx.out_device)

    @staticmethod
    def backward(ctx, grad_next):
        st, forces, snap, idx = ctx.saved_tensors
        dev = ctx.dev
        if dev.h is None:
            raise RuntimeError("the world model that produced this step was released before backward")
        if snap.shape[1] != dev.snapshot_doubles:
            raise RuntimeError("snapshot layout does not match the world model of the forward")
        with torch.cuda.device(st.device):
            g = grad_next.detach().reshape(st.shape).to(st.device, torch.float64).contiguous()
            gs = torch.empty_like(st)
            gf = torch.empty_like(forces)
            stream = torch.cuda.current_stream(st.device).cuda_stream
            gm = None
            if ctx.use_mass and ctx.mass_shape[0] > 0:
                gm = mass_gradient(dev, ctx.mass_sel, st, forces, snap, g, gs, gf, stream).sum(0).to(ctx.mass_device)
            else:
                dev.backward(st, forces, snap, g, gs, gf, stream)
            ga = gf if idx.shape[0] == gf.shape[1] and ctx.identity else gf.index_select(1, idx)
        od = ctx.out_device
        if ctx.use_mass and gm is None:
            gm = torch.zeros(ctx.mass_shape, dtype=torch.float64, device=ctx.mass_device)
        if ctx.squeeze:
            return None, gs[0].to(od), ga[0].to(od), gm
        return None, gs.to(od), ga.to(od), gm


def timestep(world: World, state: torch.Tensor, action: torch.Tensor,
             mass: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Differentiable step; see module docstring."""
    return TimestepLayer.apply(world, state, action, mass)
