"""Pin the CPU oracle (CPU-only tests).

* box-box narrow phase vs the reference's known-answer test
  (unittests/unit/test_DARTCollide.cpp:554);
* the Dantzig restatement vs the reference's OWN solver outputs
  (tests/golden/lcp_fixtures.json, generated from oracle/_ref) and, when the
  reference build is present, live against oracle/_ref on fresh problems;
* COD solve == minimum-norm least squares;
* dynamics identities (ABA vs M ddq + C = tau, as unittests/comprehensive/
  test_Dynamics.cpp checks) and the analytic Jacobians vs central finite
  differences of the oracle's own forward step (the reference's
  GradientTestUtils.hpp strategy), with and without contact.
"""
import json
import os

import numpy as np
import pytest

import models
from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _dec(v):
    return [float("inf") if x == "inf" else float("-inf") if x == "-inf" else x for x in v]


def test_box_box_known_answer(oracle_built):
    d = json.load(open(os.path.join(GOLD, "box_box_annotation.json")))
    T1 = np.eye(4); T1[:3, 3] = d["T1_translation"]
    T2 = np.eye(4); T2[:3, 3] = d["T2_translation"]
    cs = O.box_box(d["size1"], T1, d["size2"], T2)
    assert len(cs) == len(d["expected"])
    names = {1: "FACE_VERTEX", 2: "VERTEX_FACE", 3: "EDGE_EDGE"}
    got = sorted([(tuple(np.round(c[:3], 9)), names[int(c[7])]) for c in cs])
    exp = sorted([(tuple(np.round(e["point"], 9)), e["type"]) for e in d["expected"]])
    assert got == exp
    # the reference's EDGE_EDGE metadata check (test_DARTCollide.cpp:578):
    # the contact at (0.25, 0.5, 0) has |edgeADir| = x, |edgeBDir| = y
    c1 = [c for c in cs if np.allclose(c[:3], [0.25, 0.5, 0.0])][0]
    assert np.allclose(np.abs(c1[11:14]), [1, 0, 0]) and np.allclose(np.abs(c1[17:20]), [0, 1, 0])


def test_edge_edge_gradients_vs_finite_differences(oracle_built):
    """EDGE_EDGE contact gradients (EDGE_A / EDGE_B position and normal
    terms) on the reference's GRADIENTS.EDGE_EDGE_BOX_COLLISION setup
    (test_CollideGradient.cpp:169), with box 2 driven into box 1 so that the
    edge contact clamps."""
    w, st = models.edge_world()
    st = st.copy()
    st[12 + 9], st[12 + 10] = -0.3, 0.3
    f = np.zeros(12)
    o = O.OracleWorld(w)
    o.forward(st[None], f[None])
    cs = O.contacts(o, 0)
    assert len(cs) > 0 and (cs[:, 7] == 3).all()
    assert O.lcp_flags(o, 0)[3] > 0  # clamping rows
    g = np.random.default_rng(2).standard_normal(24)
    gs, gf, fd_s, fd_f = _fd_check(w, st, f, g)
    assert np.abs(gs - fd_s).max() <= 1e-6 * np.abs(fd_s).max()
    assert np.abs(gf - fd_f).max() <= 1e-6 * np.abs(fd_f).max()


def test_dantzig_matches_reference_fixtures(oracle_built):
    d = json.load(open(os.path.join(GOLD, "lcp_fixtures.json")))
    for p in d["problems"]:
        A = np.array(p["A"]); b = np.array(p["b"])
        lo = np.array(_dec(p["lo"])); hi = np.array(_dec(p["hi"])); fi = np.array(p["findex"], dtype=np.int32)
        ok, x = O.dantzig(A, b, lo, hi, fi)
        assert ok == p["ref_success"], p["name"]
        ref = np.array(p["ref_x"])
        assert np.allclose(x, ref, rtol=1e-9, atol=1e-12), (p["name"], np.abs(x - ref).max())


def test_dantzig_live_vs_reference(oracle_built):
    if O.ref_lib() is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(7)
    for k in range(200):
        nc, nd = int(rng.integers(1, 13)), int(rng.integers(6, 40))
        J = rng.standard_normal((3 * nc, nd))
        L = rng.standard_normal((nd, nd))
        A = J @ (L @ L.T + 0.05 * np.eye(nd)) @ J.T
        b = rng.standard_normal(3 * nc) * 0.2
        lo = np.tile([0.0, -1.0, -1.0], nc); hi = np.tile([np.inf, 1.0, 1.0], nc)
        fi = np.array([v for c in range(nc) for v in (-1, 3 * c, 3 * c)], dtype=np.int32)
        for early in (False, True):
            ok1, x1 = O.dantzig(A, b, lo, hi, fi, early)
            ok2, x2 = O.ref_dantzig(A, b, lo, hi, fi, early)
            assert ok1 == ok2
            if ok1:
                assert np.allclose(x1, x2, rtol=1e-9, atol=1e-12), np.abs(x1 - x2).max()


def test_cod_is_min_norm_least_squares(oracle_built):
    rng = np.random.default_rng(3)
    for r in (1, 3, 5, 8):
        U = rng.standard_normal((8, r))
        A = U @ U.T  # rank r, symmetric PSD like Q
        b = rng.standard_normal(8)
        x = O.cod_solve(A, b)
        ref = np.linalg.pinv(A, rcond=1e-12) @ b
        assert np.allclose(x, ref, rtol=1e-8, atol=1e-10)
    A = rng.standard_normal((6, 6))
    b = rng.standard_normal(6)
    assert np.allclose(O.cod_solve(A, b), np.linalg.solve(A, b))


@pytest.mark.parametrize("name", ["cartpole", "kr5", "atlas_air"])
def test_aba_matches_mass_matrix(oracle_built, name):
    w = {"cartpole": models.cartpole_world, "kr5": models.kr5_world,
         "atlas_air": lambda: models.atlas_world(False)}[name]()
    o = O.OracleWorld(w)
    n = w.getNumDofs()
    st, f = models.random_states(w, 3, seed=5)
    d = w.desc_arrays()
    for b in range(3):
        q, v = st[b, :n], st[b, n:]
        M = o.mass_matrix(q)
        assert np.allclose(M, M.T)
        assert np.linalg.eigvalsh(M).min() > 0
        ddq = o.forward_dynamics(q, v, f[b])
        rhs = f[b] - d["spring"] * (q - d["rest_position"] + v * w.dt) - d["damping"] * v - o.coriolis_gravity(q, v)
        assert np.abs(M @ ddq - rhs).max() <= 1e-10 * max(1.0, np.abs(rhs).max())


def _fd_check(w, st, f, g, eps=1e-7):
    o = O.OracleWorld(w)
    n = w.getNumDofs()

    def fwd(s, ff):
        o.reset_cache(1)
        return o.forward(s[None], ff[None])[0]
    o.reset_cache(1)
    o.forward(st[None], f[None])
    gs, gf = o.backward(g[None])
    fd_s = np.array([(fwd(st + eps * e, f) - fwd(st - eps * e, f)) @ g / (2 * eps) for e in np.eye(2 * n)])
    fd_f = np.array([(fwd(st, f + eps * e) - fwd(st, f - eps * e)) @ g / (2 * eps) for e in np.eye(n)])
    return gs[0], gf[0], fd_s, fd_f


@pytest.mark.parametrize("name", ["cartpole", "kr5", "atlas_air", "atlas_contact"])
def test_analytic_gradients_vs_finite_differences(oracle_built, name):
    w = {"cartpole": models.cartpole_world, "kr5": models.kr5_world,
         "atlas_air": lambda: models.atlas_world(False), "atlas_contact": lambda: models.atlas_world(True)}[name]()
    small = name == "atlas_contact"
    st, f = models.random_states(w, 1, seed=3, q_scale=0.01 if small else 0.3, v_scale=0.02 if small else 0.5)
    g = np.random.default_rng(2).standard_normal(st.shape[1])
    gs, gf, fd_s, fd_f = _fd_check(w, st[0], f[0], g)
    if small:
        o = O.OracleWorld(w)
        o.forward(st, f)
        assert o.num_contacts(0) > 0
    assert np.abs(gs - fd_s).max() <= 1e-6 * np.abs(fd_s).max()
    assert np.abs(gf - fd_f).max() <= 1e-6 * np.abs(fd_f).max()


def test_capsule_box_known_answers(oracle_built):
    """Capsule-box narrow phase (libccd MPR + DARTCollide's capsule/sphere-box
    branches, createCapsuleMeshContact's face branch with its EDGE_EDGE ->
    PIPE_EDGE contacts) vs the reference's known-answer tests (reference
    type PIPE_EDGE 17 is this package's 12)."""
    ref_types = {17: 12, 19: 13, 16: 10, 18: 11}
    d = json.load(open(os.path.join(GOLD, "capsule_box_known_answers.json")))
    for case in d["cases"]:
        Tc = np.eye(4)
        Tc[:3, 3] = case["capsule_translation"]
        for order in ("capsule_first", "box_first"):
            if order not in case:
                continue
            cs, unsupported = O.capsule_box(case["box_size"], np.eye(4), case["height"], case["radius"], Tc,
                                            box_first=(order == "box_first"))
            exp = case[order]["contacts"]
            assert not unsupported, case["name"]
            cs = sorted(cs, key=lambda c: c[2])  # sortContacts(UnitZ)
            assert len(cs) == len(exp), (case["name"], order, cs)
            for c, e in zip(cs, exp):
                assert np.allclose(c[:3], e["point"], atol=1e-10), (case["name"], order)
                assert np.allclose(c[3:6], e["normal"], atol=1e-10), (case["name"], order)
                assert abs(c[6] - e["depth"]) < 1e-10, (case["name"], order)
                assert int(c[7]) == ref_types.get(e["type"], e["type"]), (case["name"], order)


@pytest.mark.parametrize("name", ["half_cheetah", "capsule_edge"])
def test_sphere_box_gradients_vs_finite_differences(oracle_built, name):
    """Analytic Jacobians through capsule-box contacts (BOX_SPHERE on the
    half-cheetah ground, SPHERE_BOX clamped on two faces at a block edge --
    the non-zero normal-gradient branch) vs central differences."""
    if name == "half_cheetah":
        w = models.half_cheetah_world()
        st, f = models.half_cheetah_states(w, 12, seed=1)
        picks = [1, 3, 4]
    else:
        w = models.capsule_edge_world()
        st, f = models.capsule_edge_states(8, seed=1)
        picks = [2, 6, 0]
    o = O.OracleWorld(w)
    o.forward(st, f)
    clamped = 0
    for b in picks:
        assert o.num_contacts(b) > 0 and O.lcp_flags(o, b)[5] == 0
        clamped += O.lcp_flags(o, b)[3] > 0
        g = np.random.default_rng(b).standard_normal(st.shape[1])
        gs, gf, fd_s, fd_f = _fd_check(w, st[b], f[b], g)
        assert np.abs(gs - fd_s).max() <= 1e-6 * np.abs(fd_s).max(), (name, b)
        assert np.abs(gf - fd_f).max() <= 1e-6 * np.abs(fd_f).max(), (name, b)
    assert clamped >= 2


@pytest.mark.parametrize("ground_first", [True, False])
def test_sphere_contact_gradients_vs_finite_differences(oracle_built, ground_first):
    """SPHERE_SPHERE (SPHERE_A / SPHERE_B terms) and sphere-ground
    (BOX_SPHERE or SPHERE_BOX with the locked top face) contacts: the
    collider's known geometry and the analytical gradients against central
    differences of the oracle's own step."""
    w = models.sphere_world(ground_first)
    st, f = models.sphere_states(1, seed=3)
    st, f = st[0], f[0]
    o = O.OracleWorld(w)
    o.forward(st[None], f[None])
    cs = O.contacts(o, 0)
    types = sorted(int(t) & 15 for t in cs[:, 7])
    assert types == ([5, 5, 6] if ground_first else [4, 4, 6]), types
    r0, r1 = models.SPHERE_RADII
    c0, c1 = st[3:6], st[9:12]
    ss = cs[(cs[:, 7].astype(int) & 15) == 6][0]
    d = np.linalg.norm(c0 - c1)
    assert np.allclose(ss[0:3], (r1 * c0 + r0 * c1) / (r0 + r1), atol=1e-12)
    assert np.allclose(ss[3:6], (c0 - c1) / d, atol=1e-12)
    assert abs(ss[6] - (r0 + r1 - d)) < 1e-12
    assert O.lcp_flags(o, 0)[3] > 0  # clamping rows
    g = np.random.default_rng(4).standard_normal(24)
    gs, gf, fd_s, fd_f = _fd_check(w, st, f, g)
    assert np.abs(gs - fd_s).max() <= 1e-6 * np.abs(fd_s).max()
    assert np.abs(gf - fd_f).max() <= 1e-6 * np.abs(fd_f).max()


@pytest.mark.parametrize("sphere_first", [True, False])
@pytest.mark.parametrize("cap", [False, True])
def test_sphere_capsule_gradients_vs_finite_differences(oracle_built, sphere_first, cap):
    """collideSphereCapsule / collideCapsuleSphere: the SPHERE_PIPE /
    PIPE_SPHERE contact (SPHERE_TO_PIPE and PIPE_TO_SPHERE terms) on the
    bar's cylinder and the SPHERE_SPHERE contact on its cap, against central
    differences of the oracle's step."""
    w = models.sphere_capsule_world(sphere_first)
    st, f = models.sphere_capsule_states(1, seed=6, sphere_first=sphere_first, cap=cap)
    st, f = st[0], f[0]
    o = O.OracleWorld(w)
    o.forward(st[None], f[None])
    cs = O.contacts(o, 0)
    assert len(cs) == 1
    assert int(cs[0, 7]) == (6 if cap else (7 if sphere_first else 8))
    assert O.lcp_flags(o, 0)[3] > 0  # clamping rows
    g = np.random.default_rng(8).standard_normal(24)
    gs, gf, fd_s, fd_f = _fd_check(w, st, f, g)
    assert np.abs(gs - fd_s).max() <= 1e-6 * np.abs(fd_s).max()
    assert np.abs(gf - fd_f).max() <= 1e-6 * np.abs(fd_f).max()


@pytest.mark.parametrize("mode", ["cross", "end"])
def test_capsule_capsule_gradients_vs_finite_differences(oracle_built, mode):
    """collideCapsuleCapsule: PIPE_PIPE (PIPE_A / PIPE_B terms through
    getContactPointGradient with the contact radii) for crossing bars and
    PIPE_SPHERE for a bar standing on another, against central differences
    of the oracle's step."""
    w = models.capsule_pair_world()
    for seed in range(9, 40):  # first deterministic case whose contact clamps
        st, f = models.capsule_pair_states(1, seed=seed, mode=mode)
        st, f = st[0], f[0]
        o = O.OracleWorld(w)
        o.forward(st[None], f[None])
        if O.lcp_flags(o, 0)[3] > 0:
            break
    cs = O.contacts(o, 0)
    assert len(cs) == 1 and int(cs[0, 7]) == (9 if mode == "cross" else 8)
    assert O.lcp_flags(o, 0)[3] > 0
    g = np.random.default_rng(10).standard_normal(24)
    gs, gf, fd_s, fd_f = _fd_check(w, st, f, g)
    assert np.abs(gs - fd_s).max() <= 1e-6 * np.abs(fd_s).max()
    assert np.abs(gf - fd_f).max() <= 1e-6 * np.abs(fd_f).max()


def _check_known(cs, exp, check, tag):
    assert len(cs) == len(exp), (tag, cs)
    for c, e in zip(cs, exp):
        if "point" in check:
            assert np.allclose(c[:3], e["point"], atol=1e-10), tag
        assert np.allclose(c[3:6], e["normal"], atol=1e-10), tag
        assert abs(c[6] - e["depth"]) < 1e-8, tag
        assert (int(c[7]) & 15) == e["type"], tag


def test_collider_known_answers(oracle_built):
    """collideCapsuleCapsule (T / X / L), collideCapsuleSphere /
    collideSphereCapsule (end / side) and the sphere-box collider on the
    reference's sphere vertex / edge / face geometry, both detector orders,
    vs the reference's known answers (tests/golden/collide_known_answers.json,
    made by make_collide_known_answers.py from test_DARTCollide.cpp)."""
    d = json.load(open(os.path.join(GOLD, "collide_known_answers.json")))
    for case in d["cases"]:
        check = case.get("check", ["point", "normal", "depth"])
        for order in ("ab", "ba"):
            if order not in case:
                continue
            first, second = (case["a"], case["b"]) if order == "ab" else (case["b"], case["a"])
            cs, unsupported = O.collide_pair(tuple(first[0]), np.array(first[1]), tuple(second[0]),
                                             np.array(second[1]))
            assert bool(unsupported) == case.get("unsupported", False), case["name"]
            if case.get("sort") == "z":  # the test's sortContacts(UnitZ)
                cs = cs[np.argsort(cs[:, 2], kind="stable")]
            _check_known(cs, case[order], check, (case["name"], order))
            # the same pose through a whole world (pair loop, postProcess)
            w, st = models.known_answer_world(case, order)
            o = O.OracleWorld(w)
            o.forward(st[None], np.zeros((1, 6)))
            got = O.contacts(o, 0)
            if case.get("sort") == "z":
                got = got[np.argsort(got[:, 2], kind="stable")]
            _check_known(got, case[order], check, (case["name"], order, "world"))


@pytest.mark.parametrize("name", ["capsule_box_pipe_edge", "capsule_box_pipe_vertex", "capsule_box_sphere_and_pipe_edge"])
@pytest.mark.parametrize("order", ["ab", "ba"])
def test_pipe_box_gradients_vs_finite_differences(oracle_built, name, order):
    """PIPE_EDGE / EDGE_PIPE (PIPE_TO_EDGE / EDGE_TO_PIPE through
    math::getContactPointGradient with radii (0, 1) / (1, 0)) and
    PIPE_VERTEX / VERTEX_PIPE (PIPE_TO_VERTEX / VERTEX_TO_PIPE through
    math::closestPointOnLineGradient) on the reference's known-answer poses
    (capsule across a box edge / vertex, and lying over a box edge), the free
    body pushed into the static one, vs central differences of the oracle's
    step."""
    d = json.load(open(os.path.join(GOLD, "collide_known_answers.json")))
    case = next(c for c in d["cases"] if c["name"] == name)
    if order not in case:
        pytest.skip("the reference's test has this detector order only")
    w, st0 = models.known_answer_world(case, order)
    w.setGravity([0, -9.81, 0])
    want = {c["type"] for c in case[order]} - {4, 5}
    rng = np.random.default_rng(3)
    for _ in range(40):  # a deterministic state whose pipe contact clamps
        st = st0.copy()
        st[6:] = 0.2 * rng.standard_normal(6)
        f = rng.standard_normal(6)
        o = O.OracleWorld(w)
        o.forward(st[None], f[None])
        types = {int(t) for t in O.contacts(o, 0)[:, 7]}
        if want <= types and O.lcp_flags(o, 0)[3] > 0:
            break
    assert want <= types and O.lcp_flags(o, 0)[3] > 0, types
    g = np.random.default_rng(10).standard_normal(12)
    gs, gf, fd_s, fd_f = _fd_check(w, st, f, g)
    assert np.abs(gs - fd_s).max() <= 1e-6 * np.abs(fd_s).max()
    assert np.abs(gf - fd_f).max() <= 1e-6 * np.abs(fd_f).max()


def _seed_caches(o, caches):
    """setCachedLCPSolution for each world (None = empty)."""
    o.reset_cache(len(caches))
    for b, c in enumerate(caches):
        if c:
            o.cache[b, 0] = len(c)
            o.cache[b, 1:1 + len(c)] = c


@pytest.mark.parametrize("kind", ["half_cheetah", "atlas", "atlas_mesh"])
def test_broken_state_jacobians_vs_finite_differences(oracle_built, kind):
    """The reference's broken-state regressions (test_HalfCheetahTrajectory.cpp
    :126-330, test_AtlasTrajectory.cpp :147-372, tests/golden/broken_states.json):
    at each state, with its LCP warm start, the full analytic Jacobians
    (getStateJacobian and d next / d tau, the blocks verifyAnalyticalJacobians
    / verifyVelGradients / verifyPosVelJacobian check) against central
    differences of the oracle's own step.  Each state is in contact:
    BOX_SPHERE capsule-ground contacts for the half-cheetah, eight
    VERTEX_FACE foot contacts on the CFM + PGS fallback for the box-foot
    Atlas; on the STL-mesh Atlas (the tests' own model, with createWorld's
    limits and the tests' 96-entry caches) 32 VERTEX_FACE sole contacts: the
    cache warm-starts BROKEN_2 onto the gradient short-circuit (68 clamping,
    16 upper-bound rows), BROKEN_1 / BROKEN_3 fall back to CFM + PGS and
    removeFriction."""
    w, names, st, f, caches = models.broken_states(kind)
    n = w.getNumDofs()
    o = O.OracleWorld(w)
    _seed_caches(o, caches)
    o.forward(st, f)
    J, F = o.jacobians()
    eps_s, eps_f = 1e-6, 1e-4  # forces enter through dt / M: a larger step keeps rounding out
    for b, name in enumerate(names):
        assert o.num_contacts(b) > 0, name
        if kind == "atlas":
            assert O.lcp_flags(o, b)[1] == 1, name  # Dantzig fails -> CFM + PGS
        if kind == "atlas_mesh":
            assert o.num_contacts(b) == 32 and int(caches[b] and len(caches[b])) == 96, name
            fl = O.lcp_flags(o, b)
            if name == "BROKEN_2":
                assert fl[0] == 1 and fl[3] == 68 and fl[4] == 16, fl  # warm start short-circuits
            else:
                assert fl[1] == 1 and fl[2] == 1e-4, fl  # CFM + PGS, friction removed
        fo = O.OracleWorld(w)

        def fwd(s, ff):
            _seed_caches(fo, [caches[b]])
            return fo.forward(s[None], ff[None])[0]
        fd_J = np.stack([(fwd(st[b] + eps_s * e, f[b]) - fwd(st[b] - eps_s * e, f[b])) / (2 * eps_s)
                         for e in np.eye(2 * n)], axis=1)
        fd_F = np.stack([(fwd(st[b], f[b] + eps_f * e) - fwd(st[b], f[b] - eps_f * e)) / (2 * eps_f)
                         for e in np.eye(n)], axis=1)
        # blockwise, as the reference's checks (pos-pos, pos-vel, vel-pos, vel-vel,
        # force-vel): 1e-6 relative to the block, or the reference's own absolute
        # 1e-8 (GradientTestUtils.hpp :1590 / :1686 equals(analytical, bruteForce, 1e-8))
        # where central-difference rounding on |q| ~ 1.6 dominates an O(dt) block
        for rows in (slice(0, n), slice(n, 2 * n)):
            for cols in (slice(0, n), slice(n, 2 * n)):
                blk, ref = J[b][rows, cols], fd_J[rows, cols]
                assert np.abs(blk - ref).max() <= max(1e-6 * np.abs(ref).max(), 1e-8), (name, rows, cols)
            assert np.abs(F[b][rows] - fd_F[rows]).max() <= 1e-6 * np.abs(fd_F[rows]).max(), (name, rows)


@pytest.mark.parametrize("name", ["half_cheetah", "capsule_edge", "atlas_broken", "atlas_mesh_broken"])
def test_constraint_force_jacobian_vs_finite_differences(oracle_built, name):
    """getJacobianOfConstraintForce (BackpropSnapshot.cpp:2723) for POSITION /
    VELOCITY / FORCE from the oracle (the matrix the GPU's
    nimble_constraint_force_jacobians is compared with) against central
    differences of the oracle's clamping impulses f_c."""
    if name == "half_cheetah":
        w = models.half_cheetah_world()
        st, f = models.half_cheetah_states(w, 12, seed=1)
        picks = [1, 3, 4]
    elif name == "capsule_edge":
        w = models.capsule_edge_world()
        st, f = models.capsule_edge_states(8, seed=1)
        picks = [2, 6]
    else:
        w, _, st, f, caches = models.broken_states("atlas_mesh" if name == "atlas_mesh_broken" else "atlas")
        picks = list(range(st.shape[0]))
    if name != "atlas_mesh_broken":
        caches = [None] * st.shape[0]
    n = w.getNumDofs()
    o = O.OracleWorld(w)
    _seed_caches(o, caches)
    o.forward(st, f)
    J = o.constraint_force_jacobians()
    for b in picks:
        nc = int(O.lcp_flags(o, b)[3])
        assert nc > 0, (name, b)
        assert not J[b, nc:].any()

        def fc(s, ff):
            oo = O.OracleWorld(w)
            _seed_caches(oo, [caches[b]])
            oo.forward(s[None], ff[None])
            return O.lcp_fc(oo, 0)[:nc]
        fd = np.zeros((nc, 3 * n))
        for i in range(2 * n):
            e = np.zeros(2 * n)
            e[i] = 1e-6
            fd[:, i] = (fc(st[b] + e, f[b]) - fc(st[b] - e, f[b])) / 2e-6
        for i in range(n):
            e = np.zeros(n)
            e[i] = 1e-4
            fd[:, 2 * n + i] = (fc(st[b], f[b] + e) - fc(st[b], f[b] - e)) / 2e-4
        assert np.abs(J[b, :nc] - fd).max() <= 1e-6 * np.abs(fd).max(), (name, b)


def test_forced_lcp_replay_reproduces_own_path(oracle_built):
    """The replay hook (ForcedLcp) fed a world's own final LCP solution and
    path gives that step back: next state, classification and gradients.
    (The GPU rollout test replays the GPU's path through it.)"""
    w = models.atlas_world(True)
    st, f = models.random_states(w, 24, seed=3, q_scale=0.01, v_scale=0.02)
    o = O.OracleWorld(w)
    ref = o.forward(st, f)
    B = st.shape[0]
    g = np.random.default_rng(2).standard_normal(st.shape)
    rgs, rgf = o.backward(g)
    fx = o.cache.copy()
    flags = np.array([[O.lcp_flags(o, b)[0], O.lcp_flags(o, b)[2], O.lcp_flags(o, b)[1]] for b in range(B)])
    maps = [O.lcp_debug(o, b)[0] for b in range(B)]
    o2 = O.OracleWorld(w)
    nxt, bad = o2.forward_forced(st, f, fx, flags)
    assert bad == 0
    assert np.abs(nxt - ref).max() <= 1e-12 * np.abs(ref).max()
    for b in range(B):
        assert np.array_equal(O.lcp_debug(o2, b)[0], maps[b])
    gs, gf = o2.backward(g)
    assert np.abs(gs - rgs).max() <= 1e-10 * np.abs(rgs).max()
    assert np.abs(gf - rgf).max() <= 1e-10 * np.abs(rgf).max()
    # a row-count mismatch is reported, not replayed
    fx2 = fx.copy()
    hit = [b for b in range(B) if fx[b, 0] > 0][0]
    fx2[hit, 0] += 3
    _, bad = O.OracleWorld(w).forward_forced(st, f, fx2, flags)
    assert bad == 1


def _jacobians(w, st, f, caches, libm):
    O.set_fd_libm(libm)
    try:
        o = O.OracleWorld(w)
        _seed_caches(o, caches)
        o.forward(st, f)
        return o.jacobians()
    finally:
        O.set_fd_libm(False)


@pytest.mark.parametrize("kind", ["atlas_broken", "atlas_mesh_broken", "atlas_bench", "atlas_mesh_bench"])
def test_fd_blocks_fixed_sequence_vs_libm(oracle_built, kind):
    """The FreeJoint FD blocks (FreeJoint.cpp:965 eps 1e-6, :987 eps 1e-7)
    that the device and the oracle evaluate with one fixed IEEE sequence
    (hand-written sin / cos / acos, nimble_oracle.cpp fd*) against the same
    blocks through libm's std::sin / cos / acos, as the reference evaluates
    them (Geometry.cpp:539 expMapRot, :720 logMap): at the reference's Atlas
    broken states (with their LCP caches) and at the bench sampler's states,
    the full getStateJacobian / d next / d tau differ only at the FD noise
    level, eps_mach |q| / (2 eps) ~ 1e-9, under the reference's own absolute
    1e-8 (GradientTestUtils.hpp :1590).  So the restatement of the FD blocks
    stays pinned to the reference's libm evaluation, not only to itself."""
    if kind.endswith("_broken"):
        w, _, st, f, caches = models.broken_states("atlas_mesh" if kind == "atlas_mesh_broken" else "atlas")
    else:
        from nimblephysics_amd import workloads
        w = workloads.atlas_mesh_world(True) if kind == "atlas_mesh_bench" else workloads.atlas_world(True)
        st, f = workloads.atlas_states(w, 48, 1000)
        caches = [None] * st.shape[0]
    J0, F0 = _jacobians(w, st, f, caches, False)
    J1, F1 = _jacobians(w, st, f, caches, True)
    dJ, dF = np.abs(J0 - J1), np.abs(F0 - F1)
    assert dJ.max() <= 1e-8 and dF.max() <= 1e-8, (dJ.max(), dF.max())
    # per element against the FD noise of each entry's scale
    n = w.getNumDofs()
    qmax = np.abs(st[:, :n]).max(axis=1)[:, None, None]
    assert (dJ <= 1e-8 * np.maximum(1.0, qmax)).all()
    # the switch really changes the evaluation (two libms' last bits differ)
    assert dJ.max() > 0


def test_lcp_path_reproduces_the_step(oracle_built):
    """oracle.lcp_path (the ambiguity probe of friction-removal and final-
    classification path splits in the GPU parity tests) restates the LCP part
    of the oracle's own step: on unperturbed problems it gives the step's
    path flags and per-row classification."""
    from nimblephysics_amd import workloads
    checked = 0
    for w in (workloads.atlas_world(True), workloads.atlas_mesh_world(True)):
        st, f = workloads.atlas_states(w, 32, 1000)
        o = O.OracleWorld(w)
        o.forward(st, f)
        for b in range(st.shape[0]):
            A, bb, lo, hi, fi = O.lcp_problem(o, b)
            if len(bb) == 0:
                continue
            got = O.lcp_path(A, bb, lo, hi, fi, None, o.desc.fallback_cfm)
            fl = O.lcp_flags(o, b)
            mapping, _ = O.lcp_debug(o, b)
            want = (fl[0], fl[1], fl[2], fl[3], fl[4], fl[6], tuple(int(v) for v in mapping))
            assert got == want, (b, got[:6], want[:6])
            checked += 1
    assert checked > 20


@pytest.mark.parametrize("contact", [False, True])
def test_ball_translational_gradients_vs_finite_differences(oracle_built, contact):
    """The 3-dof joints (BallJoint.cpp: exponential coordinates, identity
    Jacobian, finite-difference posPos / velPos blocks :368 / :390;
    TranslationalJoint.cpp: R3 offset, identity blocks): the oracle's
    analytic gradients of a rig with a translational root, two ball joints
    and a revolute ankle against central differences of its own step, in
    the air and with the foot on the ground (contact gradients through the
    ball joints' position screws and same-joint screw-axis terms)."""
    w = models.ball_world(ground=contact)
    st, f = models.ball_states(4, seed=3, contact=contact)
    assert w.getNumDofs() == 10
    o = O.OracleWorld(w)
    o.forward(st, f)
    if contact:
        assert all(o.num_contacts(b) > 0 for b in range(4))
    for b in range(2):
        g = np.random.default_rng(10 + b).standard_normal(st.shape[1])
        gs, gf, fd_s, fd_f = _fd_check(w, st[b], f[b], g)
        assert np.abs(gs - fd_s).max() <= 1e-6 * np.abs(fd_s).max(), (b, np.abs(gs - fd_s).max())
        assert np.abs(gf - fd_f).max() <= 1e-6 * np.abs(fd_f).max(), (b, np.abs(gf - fd_f).max())


def test_ball_joint_integration_matches_rotation_composition(oracle_built):
    """BallJoint::integratePositionsExplicit (BallJoint.cpp:333) in the
    oracle's contact-free step: the next exponential coordinates of a ball
    joint are log(exp(q) exp(v dt)) of the step's velocity (parallel
    position / velocity update: the pre-step velocity), and a translational
    joint's are q + v dt -- checked against scipy-free numpy Rodrigues."""
    w = models.ball_world(ground=False)
    st, f = models.ball_states(3, seed=9, contact=False)
    nxt = O.OracleWorld(w).forward(st, f)
    dt = w.getTimeStep() if hasattr(w, "getTimeStep") else w.dt

    def expm(r):
        th = np.linalg.norm(r)
        K = np.array([[0, -r[2], r[1]], [r[2], 0, -r[0]], [-r[1], r[0], 0]])
        if th < 1e-12:
            return np.eye(3) + K
        return np.eye(3) + np.sin(th) / th * K + (1 - np.cos(th)) / th ** 2 * K @ K

    def logm(R):
        c = np.clip((np.trace(R) - 1) / 2, -1, 1)
        th = np.arccos(c)
        return th / (2 * np.sin(th)) * np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    n = 10
    for b in range(3):
        q, v = st[b, :n], st[b, n:]
        assert np.allclose(nxt[b, 0:3], q[0:3] + v[0:3] * dt, rtol=0, atol=1e-15)
        for o in (3, 7):
            want = logm(expm(q[o:o + 3]) @ expm(v[o:o + 3] * dt))
            assert np.allclose(nxt[b, o:o + 3], want, rtol=0, atol=1e-12), (b, o)


def _rot(axis, a):
    axis = np.asarray(axis, dtype=np.float64)
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + np.sin(a) * K + (1 - np.cos(a)) * K @ K


def _iso(R=np.eye(3), p=(0, 0, 0)):
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = p
    return T


def test_compound_joint_transforms_match_reference_formulas(oracle_built):
    """The 1-dof chains the device model steps UniversalJoint, EulerJoint and
    PlanarJoint as (dynamics.Joint.chain) against the reference's relative
    transforms: PlanarJoint.cpp:296 T_pj Trans(t1 q0) Trans(t2 q1)
    expAngular(r q2) T_cj^-1, UniversalJoint.cpp:193 T_pj AngleAxis(q0, a1)
    AngleAxis(q1, a2) T_cj^-1, EulerJoint.cpp:1333 with eulerZYXToMatrix(q *
    flip) = Rz Ry Rx (Geometry.cpp) -- the world transforms of the rig's real
    bodies at random coordinates.  The transform as a function of q fixes the
    motion subspace (GenericJoint velocities are the coordinate rates), the
    mass matrix and the bias forces, so the chain is the reference's joint."""
    w = models.compound_world(ground=False)
    o = O.OracleWorld(w)
    rng = np.random.default_rng(4)
    for _ in range(5):
        q = rng.standard_normal(8)
        Tw = o.body_transforms(q)  # device-model bodies: sled chain 0-2, arm chain 3-4, hand chain 5-7
        sled = _iso(_rot([0, 0, 1], q[2]), [q[0], q[1], 0.0])
        arm = sled @ _iso(p=[0, -0.1, 0]) @ _iso(_rot([0, 0, 1], q[3]) @ _rot([1, 0, 0], q[4])) @ _iso(p=[0, -0.25, 0])
        a = q[5:8] * np.array([1.0, -1.0, 1.0])
        hand = arm @ _iso(p=[0, -0.25, 0]) @ _iso(_rot([0, 0, 1], a[0]) @ _rot([0, 1, 0], a[1]) @ _rot([1, 0, 0], a[2])) \
            @ _iso(p=[0, -0.06, 0])
        for k, T in ((2, sled), (4, arm), (7, hand)):
            assert np.abs(Tw[k] - T[:3, :4]).max() <= 1e-13, (k, np.abs(Tw[k] - T[:3, :4]).max())


@pytest.mark.parametrize("contact", [False, True])
def test_compound_gradients_vs_finite_differences(oracle_built, contact):
    """UniversalJoint / EulerJoint / PlanarJoint (as their 1-dof chains): the
    oracle's analytic gradients of the compound rig against central
    differences of its own step, in the air and with the hand on the ground."""
    w = models.compound_world(ground=contact)
    st, f = models.compound_states(4, seed=3, contact=contact)
    o = O.OracleWorld(w)
    o.forward(st, f)
    if contact:
        assert all(o.num_contacts(b) > 0 for b in range(4))
    for b in range(2):
        g = np.random.default_rng(20 + b).standard_normal(st.shape[1])
        gs, gf, fd_s, fd_f = _fd_check(w, st[b], f[b], g)
        assert np.abs(gs - fd_s).max() <= 1e-6 * np.abs(fd_s).max(), (b, np.abs(gs - fd_s).max())
        assert np.abs(gf - fd_f).max() <= 1e-6 * np.abs(fd_f).max(), (b, np.abs(gf - fd_f).max())
