"""The product kernels on the CPU: nimblephysics_amd/csrc compiled for the
host against an emulation of the HIP execution model (tests/cpp/wave_emu:
every lane a host thread, every cross-lane operation a rendezvous of the
wave, checked for lanes out of step), with AddressSanitizer.

* the wave LCP kernels (waveDantzigR, wavePgsR, waveLcpValidR, waveReduceR,
  the COD factor and solve) in their one-row-per-lane (R = 1) and
  two-rows-per-lane (R = 2) forms agree with each other bit for bit on
  problems up to 64 rows and Dantzig agrees with the oracle's dSolveLCP
  restatement up to 96 rows;
* a whole forward + backward step through the C-ABI (capi.cpp unchanged,
  kernels launched by the emulation), with the default split and with every
  contact world forced through the wide kernels (NIMBLE_AMD_DEFER_ROWS=0),
  and Atlas worlds through every answer of the LCP cascade (the two waves'
  task board), matches the oracle -- and any out-of-bounds access aborts the
  run.

No GPU needed; the emulation runs a few worlds in tens of seconds.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

import models
import wave_emu
from oracle import oracle as O

pytestmark = pytest.mark.skipif(not os.path.exists(wave_emu.CLANG) or shutil.which("true") is None,
                                reason="needs the ROCm clang for the host build")


def _problems(sizes, seed=3):
    rng = np.random.default_rng(seed)
    out = []
    for m in sizes:
        J = rng.standard_normal((m, 2 * m // 3 + 3))
        A = J @ J.T + 1e-3 * np.eye(m)
        b = rng.standard_normal(m)
        lo, hi, fi = np.zeros(m), np.full(m, np.inf), -np.ones(m, dtype=int)
        for c in range(m // 3):
            for k in (1, 2):
                lo[3 * c + k], hi[3 * c + k], fi[3 * c + k] = -0.8, 0.8, 3 * c
        out.append((m, A, b, lo, hi, fi))
    return out


def test_lcp_wave_kernels_r1_r2():
    exe = wave_emu.build("lcp_wave_emu")
    probs = _problems((12, 40, 63, 66, 96))
    txt = [str(len(probs))]
    for m, A, b, lo, hi, fi in probs:
        txt += [str(m), wave_emu._fmt(A), wave_emu._fmt(b), wave_emu._fmt(lo), wave_emu._fmt(hi),
                wave_emu._fmt(fi, True), wave_emu._fmt(np.zeros(m))]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([exe], input="\n".join(txt), capture_output=True, text=True, timeout=1800, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    res = {}
    for ln in r.stdout.splitlines():
        t = ln.split()
        R, m = int(t[0]), int(t[1])
        res[(R, m)] = t[2:]
    for m, A, b, lo, hi, fi in probs:
        t2 = res[(2, m)]
        if m <= 64:
            assert res[(1, m)] == t2, m  # bit for bit
        ok = bool(int(t2[0]))
        x = np.array(t2[1:1 + m], dtype=float)
        ok_ref, x_ref = O.dantzig(A, b, lo, hi, fi, True)
        assert ok == ok_ref, m
        if ok:
            assert np.abs(x - x_ref).max() <= 1e-9 * max(1.0, np.abs(x_ref).max()), m
        rank = int(t2[2 * m + 4])
        assert rank == m
        xc = np.array(t2[2 * m + 5:3 * m + 5], dtype=float)
        ref = np.linalg.solve(A, b)
        assert np.abs(xc - ref).max() <= 1e-8 * np.abs(ref).max(), m
        # the packed-factor Dantzig (the wide kernel's, R = 2) equals the square one
        assert t2[3 * m + 5] == "1", m


def test_dantzig_disagreement_fixture_emulated():
    """tests/golden/dantzig_disagreements.npz (tools/dantzig_reconcile.py: the
    bench Atlas LCPs on which the device, the oracle's restatement and the
    reference's compiled dSolveLCP do not all agree) through the host build
    of waveDantzigR (R = 1): the effective outcome (success AND
    isLCPSolutionValid) equals the reference's, with x within 1e-9 when
    valid, or the problem is ambiguous for the reference itself (1e-15
    perturbations).  A sample of 24 problems (the emulation runs ~1 s each)."""
    from test_gpu_lcp import FIXTURE, classify
    exe = wave_emu.build("lcp_wave_emu")
    d = np.load(FIXTURE)
    P = len(d["n"])
    pick = np.linspace(0, P - 1, min(P, 24)).astype(int)
    txt = [str(len(pick))]
    for k in pick:
        m = int(d["n"][k])
        txt += [str(m), wave_emu._fmt(d["A"][k, :m * m]), wave_emu._fmt(d["b"][k, :m]), wave_emu._fmt(d["lo"][k, :m]),
                wave_emu._fmt(d["hi"][k, :m]), wave_emu._fmt(d["fi"][k, :m], True), wave_emu._fmt(np.zeros(m))]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", LCP_EMU_DANTZIG_ONLY="1")
    r = subprocess.run([exe], input="\n".join(txt), capture_output=True, text=True, timeout=1800, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    kinds = {"agree": 0, "ambiguous": 0, "nonunique": 0}
    for k, ln in zip(pick, r.stdout.splitlines()):
        t = ln.split()
        m = int(d["n"][k])
        assert int(t[0]) == 1 and int(t[1]) == m
        ok, x = bool(int(t[2])), np.array(t[3:3 + m], dtype=float)
        A = d["A"][k, :m * m].reshape(m, m)
        kinds[classify(k, m, A, d["b"][k, :m], d["lo"][k, :m], d["hi"][k, :m], d["fi"][k, :m], ok, x, d)] += 1
    print(kinds)


def test_pgs_fast_clamp_matches_reference_chain():
    """The PGS fallback on contact-layout rows clamps with v_max / v_min
    (lcp_wave.cuh wavePgsR) and re-runs with the reference's
    compare-and-assign chain when a residual ends non-finite: against the
    oracle's PgsBoxedLcpSolver::solve restatement (A + 1e-4 I, x0 = 0) on
    contact-layout problems, one of them with a NaN in b."""
    exe = wave_emu.build("lcp_wave_emu")
    probs = _problems((12, 24, 40, 66), seed=5)
    m, A, b, lo, hi, fi = probs[1]
    b = b.copy()
    b[4] = np.nan
    probs.append((m, A, b, lo, hi, fi))
    txt = [str(len(probs))]
    for m, A, b, lo, hi, fi in probs:
        txt += [str(m), wave_emu._fmt(A), wave_emu._fmt(b), wave_emu._fmt(lo), wave_emu._fmt(hi),
                wave_emu._fmt(fi, True), wave_emu._fmt(np.zeros(m))]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([exe], input="\n".join(txt), capture_output=True, text=True, timeout=1800, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    out = iter(ln.split() for ln in r.stdout.splitlines())
    for k, (m, A, b, lo, hi, fi) in enumerate(probs):
        lines = [next(out)] + ([next(out)] if m <= 64 else [])  # R = 1 (m <= 64), then R = 2
        ok_ref, x_ref = O.pgs(A + 1e-4 * np.eye(m), np.zeros(m), b, lo, hi, fi)
        for t in lines:
            assert int(t[1]) == m
            okp = bool(int(t[3 + m]))
            xp = np.array(t[4 + m:4 + 2 * m], dtype=float)
            assert okp == ok_ref, (k, t[0], okp, ok_ref)
            assert np.array_equal(np.isnan(xp), np.isnan(x_ref)), (k, t[0])
            fin = ~np.isnan(x_ref)
            err = np.abs(xp[fin] - x_ref[fin]).max(initial=0.0)
            assert err <= 1e-9 * max(1.0, np.abs(x_ref[fin]).max(initial=0.0)), (k, t[0], err)


@pytest.mark.parametrize("defer", [None, "0"])
def test_box_step_emulated(defer):
    world = models.box_world()
    st, f = models.box_states("slide", 2, seed=8)
    g = np.random.default_rng(1).standard_normal(st.shape)
    env = {"NIMBLE_AMD_DEFER_ROWS": defer} if defer else {}
    nxt, gs, gf, head = wave_emu.step(world, st, f, g, env)
    ow = O.OracleWorld(world)
    ref = ow.forward(st, f)
    rgs, rgf = ow.backward(g)
    assert (head[:, 0] > 0).all()  # in contact
    assert np.abs(nxt - ref).max() <= 1e-12
    assert np.abs(gs - rgs).max() <= 1e-9 * np.abs(rgs).max()
    assert np.abs(gf - rgf).max() <= 1e-9 * np.abs(rgf).max()


@pytest.mark.parametrize("fwd_defer", [None, "0"])
def test_atlas_lcp_paths_emulated(fwd_defer):
    """Atlas bench-sampler worlds through each answer of the LCP cascade --
    the short-circuit (14), Dantzig (0), the PGS fallback (10, 35) and the
    frictionless PGS (1) -- with the forward's two waves sharing the cascade
    on the task board (contact.cuh: Dantzig on the helper, the fallbacks on
    whichever wave is free): the same answers as the oracle's sequential
    cascade, flags included.  With NIMBLE_AMD_FWD_DEFER_ROWS=0 every contact
    world is deferred to the wide kernel, which steps it from the one-row
    kernel's dynamics and contacts with the pool in its LDS stage (the path
    of the mesh Atlas' 25-64-row worlds)."""
    world = models.atlas_world(True)
    st, f = models.random_states(world, 1024, seed=1000, q_scale=0.02, v_scale=0.05)
    idx = [0, 1, 10, 14, 35]
    st, f = st[idx], f[idx]
    ow = O.OracleWorld(world)
    ref = ow.forward(st, f)
    g = np.random.default_rng(3).standard_normal(st.shape)
    rgs, rgf = ow.backward(g)
    nxt, gs, gf, head = wave_emu.step(world, st, f, g, {"NIMBLE_AMD_FWD_DEFER_ROWS": fwd_defer} if fwd_defer else None)
    paths = set()
    for i in range(len(idx)):
        fl = O.lcp_flags(ow, i)
        assert (head[i, 6], head[i, 7], head[i, 4]) == (fl[0], fl[1], fl[2]), idx[i]
        paths.add("C" if fl[0] else "F" if fl[1] else "P" if fl[2] > 0 else "D")
        assert np.abs(nxt[i] - ref[i]).max() <= 1e-12, idx[i]
        assert np.abs(gs[i] - rgs[i]).max() <= 1e-9 * np.abs(rgs[i]).max() * 10, idx[i]
        assert np.abs(gf[i] - rgf[i]).max() <= 1e-9 * np.abs(rgf[i]).max(), idx[i]
    assert paths == {"C", "D", "P", "F"}


def test_mesh_atlas_wide_step_emulated():
    """Atlas with the STL soles: a bench-sampler world whose LCP has more
    than 64 rows (81), stepped by the two-rows-per-lane kernels."""
    from nimblephysics_amd import workloads
    world = workloads.atlas_mesh_world(True)
    st, f = workloads.random_states(world, 5, seed=1000, q_scale=0.02, v_scale=0.05)
    st, f = st[4:5], f[4:5]
    ow = O.OracleWorld(world)
    ref = ow.forward(st, f)
    assert len(O.lcp_debug(ow, 0)[0]) > 64
    g = np.random.default_rng(3).standard_normal(st.shape)
    rgs, rgf = ow.backward(g)
    nxt, gs, gf, head = wave_emu.step(world, st, f, g)
    assert int(head[0, 1]) > 64
    assert np.abs(nxt - ref).max() <= 1e-11
    # velocity-gradient noise of the FreeJoint central differences (see
    # test_gpu_contact_parity.GRAD_FLOOR): 1e-9 of the largest element
    assert np.abs(gs - rgs).max() <= 1e-9 * np.abs(rgs).max() * 10
    assert np.abs(gf - rgf).max() <= 1e-9 * np.abs(rgf).max()


def test_mesh_atlas_wide_lds_pool_emulated():
    """Mesh-Atlas worlds whose LCP (39-45 rows) does not fit the one-row
    kernel's LDS pool: deferred to the wide kernel, which steps them from the
    one-row kernel's dynamics cache and contact hand-off with the pool in its
    LDS stage and the helper wave on the task board -- the short-circuit
    (22), Dantzig (20) and the fallback cascade (0) -- beside an 81-row world
    on the two-rows-per-lane path (4), all against the oracle."""
    from nimblephysics_amd import workloads
    world = workloads.atlas_mesh_world(True)
    st, f = workloads.random_states(world, 24, seed=1000, q_scale=0.02, v_scale=0.05)
    idx = [0, 4, 20, 22]
    st, f = st[idx], f[idx]
    ow = O.OracleWorld(world)
    ref = ow.forward(st, f)
    g = np.random.default_rng(5).standard_normal(st.shape)
    rgs, rgf = ow.backward(g)
    nxt, gs, gf, head = wave_emu.step(world, st, f, g, {"NIMBLE_AMD_VERBOSE": "1"})
    log = open(os.path.join("/tmp", f"nimble_wave_emu_{os.getuid()}.stderr")).read()
    assert "forward defers > 24 rows" in log, log[-400:]
    paths = set()
    for i in range(len(idx)):
        fl = O.lcp_flags(ow, i)
        m = len(O.lcp_debug(ow, i, max_rows=O.MAX_LCP)[0])
        assert int(head[i, 1]) == m, idx[i]
        assert (head[i, 6], head[i, 7], head[i, 4]) == (fl[0], fl[1], fl[2]), idx[i]
        paths.add("C" if fl[0] else "F" if fl[1] else "P" if fl[2] > 0 else "D")
        assert np.abs(nxt[i] - ref[i]).max() <= 1e-11, idx[i]
        assert np.abs(gs[i] - rgs[i]).max() <= 1e-9 * np.abs(rgs[i]).max() * 10, idx[i]
        assert np.abs(gf[i] - rgf[i]).max() <= 1e-9 * np.abs(rgf[i]).max(), idx[i]
    assert {"C", "D"} <= paths and ("F" in paths or "P" in paths)


def test_mesh_atlas_wide_board_emulated():
    """Mesh-Atlas worlds of 93 and 96 LCP rows (pool in HBM, two rows per
    lane) on the wide kernel's task board: Dantzig's factor at the head of
    the LDS stage on the helper wave.  At 93 rows the task goes out before
    the first classification, which short-circuits (18); at 96 rows the
    classification's COD needs the whole stage, so the task goes out only once
    it has failed, and the cascade ends at the frictionless PGS (14)."""
    from nimblephysics_amd import workloads
    world = workloads.atlas_mesh_world(True)
    st, f = workloads.random_states(world, 24, seed=1000, q_scale=0.02, v_scale=0.05)
    idx = [14, 18]
    st, f = st[idx], f[idx]
    ow = O.OracleWorld(world)
    ref = ow.forward(st, f)
    g = np.random.default_rng(6).standard_normal(st.shape)
    rgs, rgf = ow.backward(g)
    nxt, gs, gf, head = wave_emu.step(world, st, f, g)
    for i in range(len(idx)):
        fl = O.lcp_flags(ow, i)
        m = len(O.lcp_debug(ow, i, max_rows=O.MAX_LCP)[0])
        assert m in (93, 96) and int(head[i, 1]) == m, idx[i]
        assert (head[i, 6], head[i, 7], head[i, 4]) == (fl[0], fl[1], fl[2]), idx[i]
        assert np.abs(nxt[i] - ref[i]).max() <= 1e-11, idx[i]
        assert np.abs(gs[i] - rgs[i]).max() <= 1e-9 * np.abs(rgs[i]).max() * 10, idx[i]
        assert np.abs(gf[i] - rgf[i]).max() <= 1e-9 * np.abs(rgf[i]).max(), idx[i]
    assert head[0, 7] == 1 and head[1, 6] == 1


def test_snapshot_layout_matches_pool_sizes():
    """_native.snapshot_layout (tools, tests) against csrc/pool_sizes.h."""
    from nimblephysics_amd import _native
    exe = wave_emu.build("layout_emu")
    for n in (1, 6, 9, 33, 64):
        got = [int(x) for x in subprocess.check_output([exe, str(n)], text=True).split()]
        L = _native.snapshot_layout(n)
        want = [L[k] for k in ("contacts", "rows", "fc", "vf", "yf", "ac", "acube", "pt", "q", "edge", "workspace")]
        assert got == want, (n, got, want)


def test_bench_atlas_lds_fits_four_worlds_per_cu():
    """The bench's occupancy: the forward and backward workgroups of the
    Atlas bench world must each fit a quarter of a CU's 160 KB LDS, so that
    the 1024 worlds of the bench are all resident at once (4 per CU on 256
    CUs); one double over the budget leaves 256 worlds for a second round."""
    fwd, bwd = wave_emu.lds_bytes(models.atlas_world(True))
    assert fwd <= 40 * 1024, fwd
    assert bwd <= 40 * 1024, bwd


# contact.cuh GW_* wait sites, and what the forced expiry does to the world:
# "abort" -- wave 0 abandons the contact step (snapshot: no contacts, no rows;
# the contact-free step), "complete" -- the step is the oracle's but flagged,
# "either" -- which one depends on where wave 0 is when the helper gives up
GUARD_SITES = {"helper_go": (1, "abort"), "collide_done": (2, "abort"), "board": (8, "abort"),
               "collect": (32, "abort"), "helper_task": (64, "abort"), "helper_idle": (256, "either"),
               "retire": (512, "complete"), "early_b": (2048, "abort"), "early_dyn": (32768, "abort"), "early_rows": (4096, "abort"),
               "early_a": (8192, "abort"), "post": (16384, "abort")}


@pytest.mark.parametrize("site", sorted(GUARD_SITES))
def test_guard_forced_expiry_emulated(site):
    """The deadlock guard's failure paths, run on purpose (NIMBLE_AMD_GUARD_TEST:
    the wait at one site expires at once in the targeted worlds, contact.cuh
    GW_*): four box-on-ground worlds at rest on the PGS fallback, the
    frictionless PGS, the short-circuit and Dantzig, worlds 1 and 3 (the
    frictionless PGS and Dantzig, both with the helper on the task board)
    targeted.  The launch drains (the emulated waves all reach their exits,
    under ASan); exactly the targeted worlds carry NIMBLE_STATUS_PROTOCOL; a
    targeted world either abandons its contact step (no contacts and rows in
    the snapshot, the contact-free step -- nothing the helper may still write
    is read) or, for a late failure, completes it as the oracle does; every
    other world equals the oracle."""
    from nimblephysics_amd import _native
    bit, expect = GUARD_SITES[site]
    world = models.box_world()
    st, f = models.box_states("rest", 8, seed=8)
    st, f = st[:4], f[:4]
    ow = O.OracleWorld(world)
    ref = ow.forward(st, f)
    assert [O.lcp_flags(ow, b)[0] for b in range(4)] == [0, 0, 1, 0]  # (P, F, C, D)
    g = np.random.default_rng(3).standard_normal(st.shape)
    rgs, rgf = ow.backward(g)
    free = O.OracleWorld(models.box_world(ground=False)).forward(st, f)
    nxt, gs, gf, head = wave_emu.step(world, st, f, g, {"NIMBLE_AMD_GUARD_TEST": f"{bit}:2:1"}, timeout=600)
    for i in range(4):
        status = int(head[i, 5])
        if i % 2 == 0:
            assert not status & _native.ST_PROTOCOL, (site, i, status)
            assert np.abs(nxt[i] - ref[i]).max() <= 1e-12, (site, i)
            assert np.abs(gs[i] - rgs[i]).max() <= 1e-9 * np.abs(rgs[i]).max(), (site, i)
            continue
        assert status & _native.ST_PROTOCOL, (site, i, status)
        aborted = head[i, 0] == 0 and head[i, 1] == 0
        assert expect == "either" or aborted == (expect == "abort"), (site, i, head[i, :8])
        if aborted:
            assert status == _native.ST_PROTOCOL and not head[i, 2:5].any(), (site, i, head[i, :8])
            assert np.abs(nxt[i] - free[i]).max() <= 1e-12, (site, i)
        else:
            assert np.abs(nxt[i] - ref[i]).max() <= 1e-12, (site, i)
        assert np.isfinite(gs[i]).all() and np.isfinite(gf[i]).all()


@pytest.mark.parametrize("rig", ["ball", "compound"])
@pytest.mark.parametrize("contact", [False, True])
def test_rig_step_emulated(rig, contact):
    """The 3-dof joints through the emulated kernels (ball / translational
    local transforms, motion subspaces, integrations, position screws and the
    ball joints' FD blocks in the backward; universal / Euler / planar joints
    as 1-dof chains through massless frames) against the oracle."""
    make, states = {"ball": (models.ball_world, models.ball_states),
                    "compound": (models.compound_world, models.compound_states)}[rig]
    world = make(ground=contact)
    st, f = states(8, seed=21, contact=contact)
    st, f = st[:2], f[:2]
    g = np.random.default_rng(4).standard_normal(st.shape)
    ow = O.OracleWorld(world)
    ref = ow.forward(st, f)
    rgs, rgf = ow.backward(g)
    nxt, gs, gf, head = wave_emu.step(world, st, f, g, timeout=900)
    if contact:
        assert (head[:, 0] > 0).all()
    same = 0
    for i in range(2):
        fl = O.lcp_flags(ow, i)
        if (head[i, 6], head[i, 7], head[i, 4]) != (fl[0], fl[1], fl[2]):
            # a flat box sole: rank-deficient A, on which the reference's own
            # dSolveLCP flips outcome under 1e-15 perturbations
            A, bb, lo, hi, fi = O.lcp_problem(ow, i)
            assert head[i, 6] == fl[0] and O.ref_dantzig_ambiguous(A, bb, lo, hi, fi, seed=i), i
            continue
        same += 1
        assert np.abs(nxt[i] - ref[i]).max() <= 1e-12 * max(1.0, np.abs(ref[i]).max()), i
        assert np.abs(gs[i] - rgs[i]).max() <= 1e-9 * np.abs(rgs[i]).max(), i
        assert np.abs(gf[i] - rgf[i]).max() <= 1e-9 * np.abs(rgf[i]).max(), i
    assert same >= 1
