"""Contact-path parity of the HIP timestep against the CPU oracle.

* contact index sets bit-exact: per world the same number of contacts and the
  same (bodyA, bodyB, type) sequence in detector order, points to 1e-9;
* LCP path: the same solver path (short-circuit / Dantzig / CFM+PGS /
  friction removed) and the same row classification (clamping / upper-bound /
  separating); then next state and gradients within BASELINE.json's 1e-6
  relative tolerance (observed ~1e-13);
* a world may take a different LCP path only when its LCP is numerically
  ill-posed for the reference algorithm itself: resting boxes give rank-
  deficient (e.g. rank 6 of 12) LCPs on which the reference's dSolveLCP
  succeeds or early-terminates depending on 1e-16-level rounding.  A split at
  Dantzig's outcome is checked against the reference's own compiled
  dSolveLCP (oracle/_ref: 1e-15-relative symmetric perturbations of A must
  give both outcomes), a split at the gradient short-circuit against the
  restated classification under the same perturbations; every split world
  is then replayed in the oracle with the GPU's path and final x forced
  (ForcedLcp) and its next state and gradients must match.  Such worlds must
  be rare (< 3 %);
* warm-started multi-step rollouts (the LCP cache, BoxedLcpConstraintSolver::mX).
"""
import numpy as np
import pytest
import torch

import models
from nimblephysics_amd import _native
from oracle import oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-6
SN_NCON, SN_M, SN_NC, SN_NU, SN_STATUS = 0, 1, 2, 3, 5
CREC = 13  # contact record doubles (csrc/pool_sizes.h)
SN_CONTACTS, SN_ROWREC, RR_MAP = 16, 12, 7
SN_ROWS = SN_CONTACTS + _native.MAX_CONTACTS * CREC
# Gradient floor.  The reference's FreeJoint posPos / velPos blocks are central
# differences (FreeJoint.cpp:965 eps 1e-6, :987 eps 1e-7), which the device
# and the oracle both restate: rounding in the perturbed integration gives
# ~eps_mach |q| / 1e-7 ~ 4e-9 absolute error per unit of upstream gradient in
# either one, independently.  Gradient elements below 1e-4 of the batch's
# largest are therefore compared absolutely, at 1e-10 of that largest.
GRAD_FLOOR = 1e-4


def _rel(a, b, floor=1e-5):
    """Largest per-element relative error |a - b| / max(|b|, floor * max|b|)
    (the absolute floor keeps components that are zero in exact arithmetic
    from dividing by rounding noise): with RTOL 1e-6, every element within
    1e-6 of itself, or within 1e-11 of the array's largest for elements
    below 1e-5 of it."""
    a, b = np.asarray(a), np.asarray(b)
    if b.size == 0:
        return 0.0
    scale = np.maximum(np.abs(b), floor * max(np.abs(b).max(), 1e-300))
    return float((np.abs(a - b) / scale).max())


def _device_step(world, st, f, cache=None):
    """One forward through the C-ABI with explicit buffers; returns
    (next_state, snapshot, cache) as numpy plus the device buffers."""
    dev = world.native()
    d = torch.device("cuda:0")
    B = st.shape[0]
    ts = torch.tensor(st, device=d)
    tf = torch.tensor(f, device=d)
    if cache is None:
        cache = torch.zeros((B, dev.cache_doubles), dtype=torch.float64, device=d)
        cache[:, 0] = -1
    nxt = torch.empty_like(ts)
    snap = torch.zeros((B, dev.snapshot_doubles), dtype=torch.float64, device=d)
    dev.forward(ts, tf, cache, nxt, snap, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return nxt, snap, cache, ts, tf


def _device_backward(world, ts, tf, snap, g):
    dev = world.native()
    gs = torch.empty_like(ts)
    gf = torch.empty_like(tf)
    dev.backward(ts, tf, snap, torch.tensor(g, device=ts.device), gs, gf, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return gs.cpu().numpy(), gf.cpu().numpy()


def _ref_dantzig_ambiguous(A, bb, lo, hi, fi, seed, trials=64):
    """The reference's compiled dSolveLCP (oracle/_ref) succeeds on some and
    early-terminates on other 1e-15-relative symmetric perturbations of A;
    None when oracle/_ref is not built."""
    rng = np.random.default_rng(seed)
    outs = set()
    for _ in range(trials):
        N = rng.standard_normal(A.shape)
        r = O.ref_dantzig(A * (1 + 1e-15 * (N + N.T) / 2), bb, lo, hi, fi, True)
        if r is None:
            return None
        outs.add(r[0])
        if len(outs) == 2:
            return True
    return False


def _split_kind(ow, b, sn):
    """Where world b's GPU path left the oracle's: at the gradient
    short-circuit, at Dantzig's outcome (the fallback CFM), at the friction
    removal, or in the final classification only."""
    of = O.lcp_flags(ow, b)
    return ("short-circuit" if of[0] != sn[6] else "cfm" if of[2] != sn[4] else
            "friction-removed" if of[1] != sn[7] else "classification")


def _split_ambiguous(ow, b, kind, warm, seed):
    """Whether a path split is ambiguous for the reference's algorithm, under
    1e-15-relative symmetric perturbations of A: a Dantzig-outcome split for
    the reference's own compiled dSolveLCP; a short-circuit split for the
    restated classification + standardisation (oracle classify, from the
    step's warm start: `warm`, or guessSolution when the step had no cache);
    a friction-removal or final-classification split for the restated whole
    LCP path (short-circuit, fallback cascade, final classification:
    oracle path_ambiguous).  Every kind is probed: a split on a problem whose
    outcome does not move under the perturbations fails the caller."""
    A, bb, lo, hi, fi = O.lcp_problem(ow, b)
    if kind == "cfm":
        amb = _ref_dantzig_ambiguous(A, bb, lo, hi, fi, seed)
        assert amb is not None, "oracle/_ref (the reference's compiled dSolveLCP) is not built"
        return amb
    if kind == "short-circuit":
        return O.classify_ambiguous(A, bb, lo, hi, fi, warm, seed)
    return O.path_ambiguous(A, bb, lo, hi, fi, warm, ow.desc.fallback_cfm, seed)


def _warm_start(cache, b, m):
    """The warm start world b's step read: its cache row when it holds m
    entries, else None (guessSolution)."""
    if cache is None or int(cache[b, 0]) != m:
        return None
    return cache[b, 1:1 + m].copy()


def _same_path(ow, sn, b):
    of = O.lcp_flags(ow, b)
    fl = np.concatenate([of[:5], [of[6]]])  # ... and whether LCPUtils::reduce merged columns
    gfl = np.array([sn[6], sn[7], sn[4], sn[2], sn[3], 1.0 if int(sn[5]) & 8 else 0.0])
    m = int(sn[SN_M])
    mapping, _ = O.lcp_debug(ow, b)
    gm = sn[SN_ROWS:SN_ROWS + SN_ROWREC * m].reshape(m, SN_ROWREC)[:, RR_MAP].astype(int)
    return np.array_equal(fl, gfl) and np.array_equal(gm, mapping)


def _check_lcp_solution(ow, sn, cache_row, b):
    """The GPU's final LCP solution of world b (its warm-start cache) solves
    the LCP its own path claims: A (+ the path's CFM) with the reference's
    isLCPSolutionValid, friction zero when friction was removed."""
    A, bb, lo, hi, fi = O.lcp_problem(ow, b)
    m = len(bb)
    assert int(cache_row[0]) == m, b
    x = cache_row[1:1 + m]
    if sn[7]:  # removeFriction: the reference does not check validity
        assert (x[fi >= 0] == 0).all(), b
        return
    assert O.lcp_valid(A + sn[4] * np.eye(m), x, bb, hi, lo, fi), f"world {b}: GPU LCP solution invalid"


def _check_contacts(ow, snap, B, max_diverge=0.03, cache=None, warm_cache=None, seed=0, kinds=None):
    """Contact sets bit-exact for every world; returns the mask of worlds on
    the same LCP path.  A world may leave the oracle's path only where the
    split is ambiguous for the reference's algorithm (`_split_ambiguous`:
    its compiled dSolveLCP for Dantzig-outcome splits); its GPU solution is
    then checked to solve the LCP of its own path (isLCPSolutionValid).
    `cache`: the GPU's cache after the step, `warm_cache`: the one the step
    read (None: no warm start); `kinds` collects the split kinds."""
    same = np.ones(B, dtype=bool)
    for b in range(B):
        ref = O.contacts(ow, b)
        sn = snap[b]
        nc = int(sn[SN_NCON])
        assert nc == len(ref), (b, nc, len(ref))
        got = sn[SN_CONTACTS:SN_CONTACTS + CREC * nc].reshape(nc, CREC)
        # bit-exact identity of the contact set: bodies and types in order
        # (sphere-box records carry the locked-face mask / box shape above bit 4)
        gtype = got[:, 7].astype(int) & 15
        assert np.array_equal(gtype, ref[:, 7].astype(int)), b
        assert np.array_equal(got[:, 8:10].astype(int), ref[:, 8:10].astype(int)), b
        assert np.abs(got[:, :7] - ref[:, :7]).max(initial=0) < 1e-9, b
        mapping, _ = O.lcp_debug(ow, b)
        assert int(sn[SN_M]) == len(mapping), b
        if not _same_path(ow, sn, b):
            kind = _split_kind(ow, b, sn)
            amb = _split_ambiguous(ow, b, kind, _warm_start(warm_cache, b, len(mapping)), seed * 100003 + b)
            assert amb, f"world {b}: LCP path split ({kind}) on a problem that is not ambiguous"
            if kinds is not None:
                kinds[kind] = kinds.get(kind, 0) + 1
            same[b] = False
            if cache is not None:
                _check_lcp_solution(ow, sn, cache[b], b)
    assert (~same).sum() <= max(1, int(max_diverge * B)), (~same).sum()
    return same


def _forced_replay(world, st, f, snap, gcache, div, warm_cache=None):
    """The oracle's step of `st` with the worlds `div` on the GPU's LCP path:
    their final x (the GPU's cache after the step) and path flags (gradient
    short-circuit, fallback CFM, friction removed) forced (ForcedLcp); the
    other worlds solve as usual.  Returns (oracle world, next state, number of
    forced worlds whose row count differed)."""
    ow = O.OracleWorld(world)
    B = st.shape[0]
    if warm_cache is not None:
        ow.reset_cache(B)
        ow.cache[:] = warm_cache
    fx = np.full((B, gcache.shape[1]), -1.0)
    fl = np.zeros((B, 3))
    fx[div] = gcache[div]
    fl[div, 0], fl[div, 1], fl[div, 2] = snap[div, 6], snap[div, 4], snap[div, 7]
    nxt, bad = ow.forward_forced(st, f, fx, fl)
    return ow, nxt, bad


def _parity(world, st, f, seed=11, check_grad=True, max_diverge=0.03, grad_floor=GRAD_FLOOR, kinds=None):
    """GPU vs oracle on one batch: contact sets bit-exact, same-path worlds'
    next state and gradients at 1e-6, and every split world (ambiguous for
    the reference's algorithm, `_check_contacts`) replayed with its GPU path
    forced, whose next state, classification and gradients must then match."""
    ow = O.OracleWorld(world)
    ref = ow.forward(st, f)
    nxt, snap, cache, ts, tf = _device_step(world, st, f)
    B = st.shape[0]
    snap_np, cache_np = snap.cpu().numpy(), cache.cpu().numpy()
    same = _check_contacts(ow, snap_np, B, max_diverge, cache_np, seed=seed, kinds=kinds)
    n = world.getNumDofs()
    got_all = nxt.cpu().numpy()
    got = got_all[same]
    refs = ref[same]
    assert _rel(got[:, :n], refs[:, :n]) < RTOL
    assert _rel(got[:, n:], refs[:, n:]) < RTOL
    g = np.random.default_rng(seed).standard_normal(st.shape)
    if check_grad:
        rgs, rgf = ow.backward(g)
        ggs_all, ggf_all = _device_backward(world, ts, tf, snap, g)
        ggs, ggf, rgs, rgf = ggs_all[same], ggf_all[same], rgs[same], rgf[same]
        fl = grad_floor
        assert _rel(ggs[:, :n], rgs[:, :n], fl) < RTOL, _rel(ggs[:, :n], rgs[:, :n], fl)
        assert _rel(ggs[:, n:], rgs[:, n:], fl) < RTOL, _rel(ggs[:, n:], rgs[:, n:], fl)
        assert _rel(ggf, rgf, fl) < RTOL, _rel(ggf, rgf, fl)
    div = np.flatnonzero(~same)
    if len(div):
        ow2, rep, bad = _forced_replay(world, st, f, snap_np, cache_np, div)
        assert bad == 0
        for b in div:
            assert _same_path(ow2, snap_np[b], b), f"world {b}: the forced replay classifies differently"
        assert _rel(got_all[div], rep[div]) < RTOL, _rel(got_all[div], rep[div])
        if check_grad:
            rgs2, rgf2 = ow2.backward(g)
            fl = grad_floor
            assert _rel(ggs_all[div], rgs2[div], fl) < RTOL, _rel(ggs_all[div], rgs2[div], fl)
            assert _rel(ggf_all[div], rgf2[div], fl) < RTOL, _rel(ggf_all[div], rgf2[div], fl)
    return ow, snap_np


@pytest.mark.parametrize("kind", ["rest", "slide", "tilt", "lift"])
def test_box_contact_parity(kind):
    world = models.box_world()
    st, f = models.box_states(kind, 64, seed=5)
    ow, snap = _parity(world, st, f)
    ncon = snap[:, SN_NCON]
    assert (ncon > 0).all()
    if kind == "slide":
        assert (snap[:, SN_NU] > 0).any()  # friction at the cone bound


def test_atlas_contact_parity():
    world = models.atlas_world(True)
    st, f = models.random_states(world, 64, seed=3, q_scale=0.01, v_scale=0.02)
    ow, snap = _parity(world, st, f)
    assert (snap[:, SN_NCON] > 0).mean() > 0.5


def test_atlas_rollout_warm_start():
    """Five chained steps: the LCP cache written by each step seeds the next."""
    world = models.atlas_world(True)
    st, f = models.random_states(world, 32, seed=9, q_scale=0.01, v_scale=0.02)
    ow = O.OracleWorld(world)
    cache = None
    cur = st
    n = world.getNumDofs()
    for k in range(5):
        ref = ow.forward(cur, f)
        warm = None if cache is None else cache.cpu().numpy().copy()
        nxt, snap, cache, ts, tf = _device_step(world, cur, f, cache)
        got = nxt.cpu().numpy()
        same = _check_contacts(ow, snap.cpu().numpy(), st.shape[0], cache=cache.cpu().numpy(), warm_cache=warm, seed=k)
        assert _rel(got[same], ref[same]) < RTOL, (k, _rel(got[same], ref[same]))
        g = np.random.default_rng(k).standard_normal(st.shape)
        rgs, rgf = ow.backward(g)
        ggs, ggf = _device_backward(world, ts, tf, snap, g)
        assert _rel(ggs[same], rgs[same], GRAD_FLOOR) < RTOL, (k, _rel(ggs[same], rgs[same], GRAD_FLOOR))
        assert _rel(ggf[same], rgf[same], GRAD_FLOOR) < RTOL
        cur = ref


def test_timestep_layer_with_contact():
    """The autograd.Function path (nimble.timestep) on the contact world."""
    import nimblephysics_amd as nimble
    world = models.atlas_world(True)
    st, f = models.random_states(world, 16, seed=21, q_scale=0.01, v_scale=0.02)
    ow = O.OracleWorld(world)
    ref = ow.forward(st, f)
    g = np.random.default_rng(4).standard_normal(st.shape)
    rgs, rgf = ow.backward(g)
    d = torch.device("cuda:0")
    ts = torch.tensor(st, device=d, requires_grad=True)
    tf = torch.tensor(f, device=d, requires_grad=True)
    out = nimble.timestep(world, ts, tf)
    out.backward(torch.tensor(g, device=d))
    assert _rel(out.detach().cpu().numpy(), ref) < RTOL
    assert _rel(ts.grad.cpu().numpy(), rgs) < RTOL
    assert _rel(tf.grad.cpu().numpy(), rgf) < RTOL


def test_half_cheetah_contact_parity():
    """configs[2]: half-cheetah capsules on the ground box (BOX_SPHERE
    contacts from collideBoxCapsule; the planar model's zero z-friction
    column sends most contact LCPs down the Dantzig / CFM+PGS fallback)."""
    world = models.half_cheetah_world()
    st, f = models.half_cheetah_states(world, 128, seed=4)
    ow, snap = _parity(world, st, f)
    assert (snap[:, SN_NCON] > 0).mean() > 0.4
    assert not any(O.lcp_flags(ow, b)[5] for b in range(st.shape[0]))


def test_half_cheetah_rollout():
    """Ten chained half-cheetah steps (contacts appear / vanish, warm starts)."""
    world = models.half_cheetah_world()
    st, f = models.half_cheetah_states(world, 64, seed=6)
    ow = O.OracleWorld(world)
    cache = None
    cur = st
    for k in range(10):
        ref = ow.forward(cur, f)
        warm = None if cache is None else cache.cpu().numpy().copy()
        nxt, snap, cache, ts, tf = _device_step(world, cur, f, cache)
        same = _check_contacts(ow, snap.cpu().numpy(), st.shape[0], cache=cache.cpu().numpy(), warm_cache=warm, seed=k)
        got = nxt.cpu().numpy()
        assert _rel(got[same], ref[same]) < RTOL, (k, _rel(got[same], ref[same]))
        g = np.random.default_rng(k).standard_normal(st.shape)
        rgs, rgf = ow.backward(g)
        ggs, ggf = _device_backward(world, ts, tf, snap, g)
        assert _rel(ggs[same], rgs[same], GRAD_FLOOR) < RTOL, (k, _rel(ggs[same], rgs[same], GRAD_FLOOR))
        assert _rel(ggf[same], rgf[same], GRAD_FLOOR) < RTOL
        cur = ref


def test_capsule_edge_contact_parity():
    """SPHERE_BOX contacts clamped on two box faces (non-zero normal and
    friction-direction gradients through the locked-face projection)."""
    world = models.capsule_edge_world()
    st, f = models.capsule_edge_states(64, seed=2)
    ow, snap = _parity(world, st, f)
    assert (snap[:, SN_NCON] > 0).all()
    types = snap[:, SN_CONTACTS + 7].astype(int)
    assert ((types & 15) == 4).all() and (((types >> 4) & 7) == 3).all()


@pytest.mark.parametrize("rows", [0, 6])
def test_hbm_workspace_path(rows, monkeypatch):
    """Worlds whose LCP exceeds the on-chip pool run the same code on the
    snapshot's HBM workspace; force that path (pool for 0 / 6 rows) and check
    parity on box and Atlas contact worlds."""
    monkeypatch.setenv("NIMBLE_AMD_LDS_ROWS", str(rows))
    world = models.box_world()
    st, f = models.box_states("slide", 32, seed=8)
    _parity(world, st, f)
    world = models.atlas_world(True)
    st, f = models.random_states(world, 32, seed=12, q_scale=0.01, v_scale=0.02)
    _parity(world, st, f)


@pytest.mark.parametrize("world_name", ["box", "atlas", "half_cheetah", "capsule_edge"])
def test_wide_kernels(world_name, monkeypatch):
    """The two-rows-per-lane kernels (nimble_forward_wide_kernel /
    nimble_backward_wide_kernel, which take worlds with more than 64 LCP
    rows) forced onto every contact world (NIMBLE_AMD_DEFER_ROWS=0): the
    same parity against the oracle as the one-row-per-lane kernels."""
    monkeypatch.setenv("NIMBLE_AMD_DEFER_ROWS", "0")
    if world_name == "box":
        world = models.box_world()
        st, f = models.box_states("slide", 32, seed=8)
    elif world_name == "atlas":
        world = models.atlas_world(True)
        st, f = models.random_states(world, 96, seed=12, q_scale=0.02, v_scale=0.05)
    elif world_name == "half_cheetah":
        world = models.half_cheetah_world()
        st, f = models.half_cheetah_states(world, 64, seed=5)
    else:
        world = models.capsule_edge_world()
        st, f = models.capsule_edge_states(32, seed=2)
    _parity(world, st, f)


@pytest.mark.parametrize("name", ["edge", "ledge"])
def test_edge_edge_contact_parity(name):
    """EDGE_EDGE contacts and their gradient terms: the reference's
    GRADIENTS.EDGE_EDGE_BOX_COLLISION setup (box-box separating-axis edge
    contact, box 2 driven into box 1) and a cube half over the edge of a
    static box (face-clipped contacts on the edge, the configuration of
    BOX_BOX_FACE_FACE_COLLISION_ANNOTATION); worlds perturbed around them."""
    if name == "edge":
        world, st0 = models.edge_world()
        st0 = st0.copy()
        st0[12 + 9], st0[12 + 10] = -0.3, 0.3
    else:
        world, st0 = models.ledge_world()
    B = 16
    rng = np.random.default_rng(21)
    st = st0[None, :] + 1e-4 * rng.standard_normal((B, st0.shape[0]))
    st[0] = st0
    f = 0.1 * rng.standard_normal((B, world.getNumDofs()))
    # the cube resting on the ledge has four contacts (12 rows, rank <= 6):
    # an ill-posed LCP on which the reference's Dantzig itself flips outcome
    # (each diverging world is checked to be such a case); the others must
    # match on path, state and gradients
    ow, snap = _parity(world, st, f, max_diverge=0.0 if name == "edge" else 0.25)
    types = []
    for b in range(B):
        nc = int(snap[b, SN_NCON])
        types += list((snap[b, SN_CONTACTS:SN_CONTACTS + CREC * nc].reshape(nc, CREC)[:, 7].astype(int) & 15))
    assert 3 in types  # EDGE_EDGE present
    assert (snap[:, SN_NC] > 0).any()  # and clamping


@pytest.mark.gpu
@pytest.mark.parametrize("ground_first", [True, False])
def test_sphere_contact_parity(ground_first):
    """Standalone sphere shapes: SPHERE_SPHERE contacts (collideSphereSphere)
    and sphere-ground contacts (BOX_SPHERE via collideBoxSphere when the
    ground is first in detector order, SPHERE_BOX via collideSphereBox
    otherwise, clamped on the ground's top face), forward and gradients."""
    world = models.sphere_world(ground_first)
    st, f = models.sphere_states(64, seed=5)
    ow, snap = _parity(world, st, f)
    assert (snap[:, SN_NCON] == 3).all()
    types = np.sort(snap[:, SN_CONTACTS + 7 + CREC * np.arange(3)].astype(int) & 15, axis=1)
    want = [5, 5, 6] if ground_first else [4, 4, 6]
    assert (types == want).all()


@pytest.mark.gpu
@pytest.mark.parametrize("sphere_first", [True, False])
def test_sphere_capsule_contact_parity(sphere_first):
    """collideSphereCapsule / collideCapsuleSphere: a ball pressed onto a
    free capsule bar, over its cylinder (SPHERE_PIPE / PIPE_SPHERE) and on
    its caps (SPHERE_SPHERE), forward and gradients."""
    world = models.sphere_capsule_world(sphere_first)
    sp, fp = models.sphere_capsule_states(48, seed=7, sphere_first=sphere_first)
    sc, fc = models.sphere_capsule_states(16, seed=8, sphere_first=sphere_first, cap=True)
    st, f = np.concatenate([sp, sc]), np.concatenate([fp, fc])
    ow, snap = _parity(world, st, f)
    assert (snap[:, SN_NCON] == 1).all()
    types = snap[:, SN_CONTACTS + 7].astype(int) & 15
    assert (types[:48] == (7 if sphere_first else 8)).all() and (types[48:] == 6).all()


@pytest.mark.gpu
def test_capsule_capsule_contact_parity():
    """collideCapsuleCapsule: crossing bars (PIPE_PIPE) and a bar standing on
    another (PIPE_SPHERE), forward and gradients."""
    world = models.capsule_pair_world()
    sx, fx = models.capsule_pair_states(40, seed=11, mode="cross")
    se, fe = models.capsule_pair_states(24, seed=12, mode="end")
    ow, snap = _parity(world, np.concatenate([sx, se]), np.concatenate([fx, fe]))
    ncon = snap[:, SN_NCON]
    assert (ncon <= 1).all() and (ncon[:40] == 1).sum() >= 30 and (ncon[40:] == 1).sum() >= 12
    types = snap[:, SN_CONTACTS + 7].astype(int) & 15
    assert (types[:40][ncon[:40] == 1] == 9).all() and (types[40:][ncon[40:] == 1] == 8).all()


@pytest.mark.parametrize("shape", ["sphere", "box"])
def test_lcp_reduce_duplicate_columns(shape):
    """LCPUtils::reduce on the hot path: a body with two shapes 1e-10 apart
    gives every contact twice, the fallback solves merge the duplicate
    columns (status bit 8 == the oracle's reduced flag, checked per world in
    _same_path), and state / gradients match."""
    world = models.twin_world(shape)
    st, f = models.twin_states(64, seed=3)
    # gradients run through the pseudo-inverse of a clamping matrix made
    # numerically rank deficient by construction (columns 1e-10 m apart), so
    # rounding is amplified: elements below 1e-4 of the largest are compared
    # absolutely at 1e-10 of it (~2e-12 x max observed), the rest at 1e-6
    ow, snap = _parity(world, st, f, max_diverge=0.1 if shape == "box" else 0.03)
    reduced = (snap[:, 5].astype(int) & 8) != 0
    assert reduced.mean() > 0.4, reduced.mean()


def test_contact_overflow_raises():
    """More contacts than NIMBLE_MAX_CONTACTS (MAX_CONTACTS // 4 + 1 boxes
    resting on the ground, four corner contacts each) cannot be the
    reference's step: timestep raises ContactCapacityError, and under the
    'record' policy the per-world status says why."""
    import nimblephysics_amd as nimble
    from nimblephysics_amd import dynamics as D
    from nimblephysics_amd._native import ContactCapacityError
    w = nimble.World()
    w.setGravity([0, -9.81, 0])
    g = D.Skeleton("ground")
    gj, gb = g.createWeldJointAndBodyNodePair()
    T = np.eye(4)
    T[1, 3] = -0.05
    gj.setTransformFromParentBodyNode(T)
    gb.createShapeNode(D.BoxShape([10.0, 0.1, 10.0]), collision=True)
    g.setMobile(False)
    w.addSkeleton(g)
    nbox = _native.MAX_CONTACTS // 4 + 1
    for k in range(nbox):
        # vertical sliders (the model allows at most 8 free joints)
        sk = D.Skeleton(f"box{k}")
        j, b = sk.createPrismaticJointAndBodyNodePair()
        j.setAxis([0, 1, 0])
        T = np.eye(4)
        T[0, 3] = 0.4 * k
        j.setTransformFromParentBodyNode(T)
        b.createShapeNode(D.BoxShape([0.2, 0.1, 0.2]), collision=True)
        w.addSkeleton(sk)
    st = np.zeros((4, 2 * nbox))
    st[:, :nbox] = 0.05 - 1e-3
    d = torch.device("cuda:0")
    ts = torch.tensor(st, device=d)
    act = torch.zeros((4, nbox), dtype=torch.float64, device=d)
    with pytest.raises(ContactCapacityError):
        nimble.timestep(w, ts, act)
    w.setStatusPolicy("record")
    nimble.timestep(w, ts, act)
    status = w.getLastStatus().cpu().numpy()
    assert ((status & 1) != 0).all()


def test_restitution_bounce_parity():
    """Restitution above DART_RESTITUTION_COEFF_THRESHOLD: a box dropped on
    the ground at ~1.5 m/s with coefficients 0.8 x 0.8 gets the bounce
    velocity in b (ContactConstraint.cpp:393 getInformation) and the
    bounce diagonal 1 + e in the backward (BackpropSnapshot's
    getBouncingConstraintMatrix); forward and gradients vs the oracle."""
    world = models.box_world()
    for s in range(2):
        world.getSkeleton(s).getBodyNode(0).setRestitutionCoeff(0.8)
    st, f = models.box_states("drop", 64, seed=7)
    ow, snap = _parity(world, st, f)
    bounced = 0
    for b in range(st.shape[0]):
        m = int(snap[b, SN_M])
        rr = snap[b, SN_ROWS:SN_ROWS + SN_ROWREC * m].reshape(m, SN_ROWREC)
        bounced += int((np.abs(rr[:, 11] - 1.64) < 1e-12).any())  # RR_BOUNCE = 1 + 0.8 * 0.8
    assert bounced > st.shape[0] // 2, bounced
    ref = ow.forward(st, f)
    assert (ref[:, 6 + 4] > 0.5).mean() > 0.5  # the box leaves the ground upwards


def test_penetration_correction_parity():
    """setPenetrationCorrectionEnabled(True): the normal rows' b gets the
    clamped penetration velocity min(depth * 0.01 / dt, 1e-3)
    (ContactConstraint.cpp getInformation); resting and tilted boxes ~1 mm
    into the ground, forward and gradients vs the oracle."""
    world = models.box_world()
    world.setPenetrationCorrectionEnabled(True)
    for kind in ("rest", "tilt"):
        st, f = models.box_states(kind, 48, seed=13)
        _parity(world, st, f)
    # and it changes the step: the same worlds without correction differ
    st, f = models.box_states("rest", 8, seed=13)
    on = O.OracleWorld(world).forward(st, f)
    world.setPenetrationCorrectionEnabled(False)
    off = O.OracleWorld(world).forward(st, f)
    assert np.abs(on - off).max() > 1e-6


def test_sequential_position_update_parity():
    """setParallelVelocityAndPositionUpdates(False): positions integrate with
    the post-constraint velocity (World.cpp:312 else-branch,
    skel->integratePositions), on Atlas with foot contact; the reference's
    BackpropSnapshot keeps its parallel-update Jacobians, as the oracle does."""
    world = models.atlas_world(True)
    world.setParallelVelocityAndPositionUpdates(False)
    st, f = models.random_states(world, 48, seed=17, q_scale=0.01, v_scale=0.02)
    _parity(world, st, f)
    world.setParallelVelocityAndPositionUpdates(True)
    par = O.OracleWorld(world).forward(st[:4], f[:4])
    world.setParallelVelocityAndPositionUpdates(False)
    seq = O.OracleWorld(world).forward(st[:4], f[:4])
    assert np.abs(par - seq).max() > 1e-9


def test_atlas_parity_bench_batch():
    """configs[3] at the bench's size: 1024 Atlas worlds (the bench sampler's
    perturbations), forward and gradients vs the oracle for every world."""
    world = models.atlas_world(True)
    st, f = models.random_states(world, 1024, seed=1000, q_scale=0.02, v_scale=0.05, f_scale=1.0)
    ow, snap = _parity(world, st, f, max_diverge=0.01)
    assert (snap[:, SN_NCON] > 0).mean() > 0.5


def test_half_cheetah_parity_bench_batch():
    """configs[2] at the bench's size: 4096 half-cheetah worlds, forward and
    gradients vs the oracle for every world."""
    world = models.half_cheetah_world()
    st, f = models.half_cheetah_states(world, 4096, seed=1000)
    ow, snap = _parity(world, st, f, max_diverge=0.01)
    assert (snap[:, SN_NCON] > 0).mean() > 0.4


def test_model_change_between_steps():
    """A body-mass change between two steps reaches the device model
    (dynamics setters invalidate the uploaded World): GPU == oracle on the
    new model, and differs from the old one."""
    import nimblephysics_amd as nimble
    world = models.atlas_world(True)
    st, f = models.random_states(world, 8, seed=5, q_scale=0.01, v_scale=0.02)
    d = torch.device("cuda:0")
    out1 = nimble.timestep(world, torch.tensor(st, device=d), torch.tensor(f, device=d)).cpu().numpy()
    body = world.getSkeleton(0).getBodyNode(3)
    body.setMass(body.getMass() * 3.0)
    world._batch_state = None  # fresh LCP warm start, as the oracle below
    out2 = nimble.timestep(world, torch.tensor(st, device=d), torch.tensor(f, device=d)).cpu().numpy()
    ref2 = O.OracleWorld(world).forward(st, f)
    assert np.abs(out2 - out1).max() > 1e-9
    assert _rel(out2, ref2) < RTOL


@pytest.mark.parametrize("order", ["ab", "ba"])
def test_collider_known_answers_on_device(order):
    """The device narrow phase on the reference's collider known answers
    (tests/golden/collide_known_answers.json: test_DARTCollide.cpp capsule-
    capsule T / X / L, capsule-sphere end / side, sphere-box vertex / edge /
    face), each pose one world, both detector orders: contact count, type,
    point, normal and depth as the reference's tests expect."""
    import json
    import os
    d = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                    "collide_known_answers.json")))
    for case in d["cases"]:
        if order not in case:
            continue
        check = case.get("check", ["point", "normal", "depth"])
        w, st = models.known_answer_world(case, order)
        _, snap, _, _, _ = _device_step(w, st[None], np.zeros((1, 6)))
        sn = snap.cpu().numpy()[0]
        exp = case[order]
        nc = int(sn[SN_NCON])
        assert nc == len(exp), (case["name"], nc)
        got = sn[SN_CONTACTS:SN_CONTACTS + CREC * nc].reshape(nc, CREC)
        if case.get("sort") == "z":  # the test's sortContacts(UnitZ)
            got = got[np.argsort(got[:, 2], kind="stable")]
        for c, e in zip(got, exp):
            if "point" in check:
                assert np.allclose(c[:3], e["point"], atol=1e-10), case["name"]
            assert np.allclose(c[3:6], e["normal"], atol=1e-10), case["name"]
            assert abs(c[6] - e["depth"]) < 1e-8, case["name"]
            assert (int(c[7]) & 15) == e["type"], case["name"]
        # ST_UNSUPPORTED_SHAPE (2) exactly where the reference's contacts have
        # undefined (NaN) gradients
        assert bool(int(sn[SN_STATUS]) & 2) == case.get("unsupported", False), case["name"]


@pytest.mark.parametrize("name", ["capsule_box_pipe_edge", "capsule_box_pipe_vertex", "capsule_box_sphere_and_pipe_edge",
                                  "capsule_box_pipe_edge_parallel_vertex"])
@pytest.mark.parametrize("order", ["ab", "ba"])
def test_pipe_box_contact_parity(name, order):
    """createCapsuleMeshContact's vertex-pipe, edge-pipe and face-edge
    contacts (PIPE_VERTEX / VERTEX_PIPE, PIPE_EDGE / EDGE_PIPE) around the
    reference's known-answer poses, both detector orders: contact sets,
    next state and gradients (PIPE_TO_VERTEX / VERTEX_TO_PIPE / PIPE_TO_EDGE
    / EDGE_TO_PIPE terms) vs the oracle."""
    import json
    import os
    d = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                    "collide_known_answers.json")))
    case = next(c for c in d["cases"] if c["name"] == name)
    if order not in case:
        pytest.skip("the reference's test has this detector order only")
    world, _ = models.known_answer_world(case, order)
    world.setGravity([0, -9.81, 0])
    st, f = models.pipe_box_states(case, order, 48, seed=4)
    ow, snap = _parity(world, st, f)
    types = snap[:, SN_CONTACTS + 7 + CREC * np.arange(2)].astype(int) & 15
    want = {c["type"] for c in case[order]} - {4, 5}
    assert any(((types[:, 0] == t) | (types[:, 1] == t)).any() for t in want)
    assert (snap[:, SN_NC] > 0).any()


def _seeded_cache(dev_doubles, caches, d):
    """Per-world LCP warm starts ([size, x...], -1 = empty) as the device's
    cache rows (World::setCachedLCPSolution)."""
    cache = torch.zeros((len(caches), dev_doubles), dtype=torch.float64, device=d)
    cache[:, 0] = -1
    for b, c in enumerate(caches):
        if c:
            cache[b, 0] = len(c)
            cache[b, 1:1 + len(c)] = torch.tensor(c, dtype=torch.float64)
    return cache


@pytest.mark.parametrize("kind", ["half_cheetah", "atlas", "atlas_mesh"])
def test_broken_state_parity(kind):
    """The reference's broken-state regressions (test_HalfCheetahTrajectory.cpp
    :126-330 with BROKEN_POINT's LCP cache, test_AtlasTrajectory.cpp :147-372
    on the box-foot Atlas and, with the tests' 96-entry LCP caches and
    createWorld's limits, on the STL-mesh Atlas they were written for;
    tests/golden/broken_states.json): contact sets and LCP path identical to
    the oracle's, the next state and the full Jacobians (getStateJacobian and
    d next / d tau, one device backward per basis vector over a replicated
    batch) within RTOL of the oracle's analytic ones, which
    tests/test_oracle_pins.py checks against finite differences at the same
    states."""
    from test_oracle_pins import _seed_caches
    w, names, st, f, caches = models.broken_states(kind)
    n = w.getNumDofs()
    B = len(names)
    d = torch.device("cuda:0")
    dev = w.native()
    ow = O.OracleWorld(w)
    _seed_caches(ow, caches)
    ref = ow.forward(st, f)
    J, F = ow.jacobians()
    seeded = _seeded_cache(dev.cache_doubles, caches, d)
    warm = seeded.cpu().numpy().copy()
    nxt, snap, cache, ts, tf = _device_step(w, st, f, seeded)
    same = _check_contacts(ow, snap.cpu().numpy(), B, cache=cache.cpu().numpy(), warm_cache=warm)
    assert same.all(), names
    assert (snap.cpu().numpy()[:, SN_NCON] > 0).all()
    assert _rel(nxt.cpu().numpy(), ref) < RTOL
    # full Jacobians: 2n copies of each world, backward of the i-th unit vector
    R = 2 * n
    st_r, f_r = np.repeat(st, R, axis=0), np.repeat(f, R, axis=0)
    _nx, snap_r, _c, ts_r, tf_r = _device_step(w, st_r, f_r,
                                               _seeded_cache(dev.cache_doubles, [c for c in caches for _ in range(R)], d))
    gs, gf = _device_backward(w, ts_r, tf_r, snap_r, np.tile(np.eye(R), (B, 1)))
    # the reference's "broken" (ill-conditioned) states: entries below 1e-4 of
    # the matrix's largest are held to 1e-10 of it absolutely (~1e-10 seen).
    # The backward is backprop's VJP, so its rows are the Jacobians' rows
    # after clipLossGradientsToBounds (BackpropSnapshot.cpp:425): with
    # createWorld's zero root force bounds (the mesh Atlas) every root-force
    # entry is clipped (tau = 0 = lower = upper)
    for b, name in enumerate(names):
        eJ, eF = _clip_rows(w, st[b], f[b], J[b].T.copy(), F[b].T.copy())
        eJ, eF = eJ.T, eF.T
        assert _rel(gs[b * R:(b + 1) * R], eJ, 1e-4) < RTOL, (name, _rel(gs[b * R:(b + 1) * R], eJ, 1e-4))
        assert _rel(gf[b * R:(b + 1) * R], eF, 1e-4) < RTOL, (name, _rel(gf[b * R:(b + 1) * R], eF, 1e-4))
    if kind == "atlas_mesh":
        # the Jacobian getters do not clip: getActionJacobian equals F
        from nimblephysics_amd import neural
        w.setCachedLCPSolution(caches)
        w._batch_state = None
        snap_j = neural.forwardPass(w, state=torch.tensor(st, device=d), action=torch.tensor(f, device=d))
        FJ = snap_j.getActionJacobian(w).cpu().numpy()
        for b, name in enumerate(names):
            assert _rel(FJ[b], F[b], 1e-4) < RTOL, (name, _rel(FJ[b], F[b], 1e-4))
        assert np.abs(F[0][:, :6]).max() > 0  # ... whose root columns the backward clips


def _clip_rows(w, s, f, Gs, Gf):
    """clipLossGradientsToBounds applied to each column of Gs [2n, k] / Gf
    [n, k] (a batch of loss gradients w.r.t. state / force) at state s and
    force f: a gradient that would push a dof past a bound it sits on is
    zeroed (BackpropSnapshot.cpp:425, oracle_step.cpp)."""
    d = w.desc_arrays()
    n = w.getNumDofs()
    q, v = s[:n], s[n:]
    for k in range(n):
        for col in range(Gs.shape[1]):
            if (q[k] == d["pos_lower"][k] and Gs[k, col] > 0) or (q[k] == d["pos_upper"][k] and Gs[k, col] < 0):
                Gs[k, col] = 0.0
            if (v[k] == d["vel_lower"][k] and Gs[n + k, col] > 0) or (v[k] == d["vel_upper"][k] and Gs[n + k, col] < 0):
                Gs[n + k, col] = 0.0
        for col in range(Gf.shape[1]):
            if (f[k] == d["force_lower"][k] and Gf[k, col] > 0) or (f[k] == d["force_upper"][k] and Gf[k, col] < 0):
                Gf[k, col] = 0.0
    return Gs, Gf


def test_forward_chunked_launches_match(monkeypatch):
    """The forward runs one workgroup per world; batches larger than one
    launch are split by the host (capi.cpp fwdChunk).  Chunks of 5 worlds
    over a 23-world batch give bit-identical next states, LCP caches,
    snapshot headers / contact records and backward results (the snapshot's
    scratch workspace may differ) to a single launch."""
    world = models.atlas_world(True)
    st, f = models.random_states(world, 23, seed=17, q_scale=0.01, v_scale=0.02)
    nxt1, snap1, cache1, ts, tf = _device_step(world, st, f)
    monkeypatch.setenv("NIMBLE_AMD_FWD_CHUNK", "5")
    nxt2, snap2, cache2, _, _ = _device_step(world, st, f)
    assert (snap1[:, SN_NCON] > 0).any()
    assert torch.equal(nxt1, nxt2)
    assert torch.equal(cache1, cache2)
    a, b = snap1.cpu().numpy(), snap2.cpu().numpy()
    for w in range(st.shape[0]):
        nc = int(a[w, SN_NCON])
        assert np.array_equal(a[w, :9], b[w, :9]), w
        ra = a[w, SN_CONTACTS:SN_CONTACTS + CREC * nc].reshape(nc, CREC)
        rb = b[w, SN_CONTACTS:SN_CONTACTS + CREC * nc].reshape(nc, CREC)
        assert np.array_equal(ra[:, :10], rb[:, :10]), w  # (sphere-centre slots unused for box contacts)
    g = np.random.default_rng(3).standard_normal(st.shape)
    gs2, gf2 = _device_backward(world, ts, tf, snap2, g)
    monkeypatch.delenv("NIMBLE_AMD_FWD_CHUNK")
    gs1, gf1 = _device_backward(world, ts, tf, snap1, g)
    assert np.array_equal(gs1, gs2) and np.array_equal(gf1, gf2)
