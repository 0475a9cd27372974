"""ORACLE / TEST INFRASTRUCTURE ONLY.

ctypes wrapper over oracle/liboracle.so -- the CPU restatement of the
reference's timestep -- for tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  Never imported by nimblephysics_amd.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_LIB = os.path.join(HERE, "_ref", "libodelcp.so")
MAX_LCP = 126  # include/nimble_amd.h NIMBLE_MAX_LCP (the LCP cache layout)

_lib = None
_ref = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE, "all"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        vp, ip, dp = C.c_void_p, C.c_int, C.POINTER(C.c_double)
        L.oracle_world_create.argtypes = [vp]
        L.oracle_world_create.restype = vp
        L.oracle_world_destroy.argtypes = [vp]
        L.oracle_snapshots_create.argtypes = [ip]
        L.oracle_snapshots_create.restype = vp
        L.oracle_snapshots_destroy.argtypes = [vp]
        L.oracle_forward.argtypes = [vp, ip, dp, dp, dp, dp, vp]
        L.oracle_forward_forced.argtypes = [vp, ip, dp, dp, dp, dp, vp, dp, dp]
        L.oracle_detect.argtypes = [vp, ip, dp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.oracle_backward.argtypes = [vp, ip, vp, dp, dp, dp]
        L.oracle_jacobians.argtypes = [vp, ip, vp, dp, dp]
        L.oracle_constraint_force_jacobians.argtypes = [vp, ip, vp, dp, ip]
        L.oracle_mass_matrix.argtypes = [vp, dp, dp]
        L.oracle_coriolis_gravity.argtypes = [vp, dp, dp, dp]
        L.oracle_forward_dynamics.argtypes = [vp, dp, dp, dp, dp]
        L.oracle_body_transforms.argtypes = [vp, dp, dp]
        L.oracle_jacobian_of_c.argtypes = [vp, dp, dp, ip, dp]
        L.oracle_num_contacts.argtypes = [vp, ip]
        L.oracle_num_contacts.restype = ip
        L.oracle_contacts.argtypes = [vp, ip, dp, ip]
        L.oracle_contacts.restype = ip
        L.oracle_lcp_debug.argtypes = [vp, ip, C.POINTER(ip), dp, ip]
        L.oracle_lcp_debug.restype = ip
        L.oracle_lcp_flags.argtypes = [vp, ip, dp]
        L.oracle_lcp_fc.argtypes = [vp, ip, dp, ip]
        L.oracle_lcp_fc.restype = ip
        L.oracle_lcp_cols.argtypes = [vp, ip, dp, ip]
        L.oracle_lcp_cols.restype = ip
        L.oracle_lcp_problem.argtypes = [vp, ip, dp, dp, dp, dp, C.POINTER(ip), ip]
        L.oracle_lcp_problem.restype = ip
        L.oracle_dantzig.argtypes = [ip, dp, dp, dp, dp, C.POINTER(ip), dp, ip]
        L.oracle_dantzig.restype = ip
        L.oracle_cod_solve.argtypes = [dp, ip, ip, dp, dp]
        L.oracle_box_box.argtypes = [dp, dp, dp, dp, dp]
        L.oracle_box_box.restype = ip
        L.oracle_collide_pair.argtypes = [ip, dp, dp, ip, dp, dp, C.c_double, dp, ip]
        L.oracle_collide_pair.restype = ip
        pi = C.POINTER(ip)
        L.oracle_lcp_reduce.argtypes = [ip, dp, dp, dp, dp, dp, pi, dp, dp, dp, dp, dp, pi, pi]
        L.oracle_lcp_reduce.restype = ip
        L.oracle_pgs.argtypes = [ip, dp, dp, dp, dp, dp, pi]
        L.oracle_pgs.restype = ip
        L.oracle_pgs_opt.argtypes = [ip, dp, dp, dp, dp, dp, pi, ip, C.c_double, C.c_double, C.c_double]
        L.oracle_pgs_opt.restype = ip
        L.oracle_lcp_valid.argtypes = [ip, dp, dp, dp, dp, dp, pi, ip]
        L.oracle_lcp_valid.restype = ip
        L.oracle_guess_solution.argtypes = [ip, dp, dp, pi, dp]
        L.oracle_lcp_cascade.argtypes = [ip, dp, dp, dp, dp, pi, dp, C.c_double, dp]
        L.oracle_classify.argtypes = [ip, dp, dp, dp, dp, pi, dp]
        L.oracle_classify.restype = ip
        L.oracle_lcp_path.argtypes = [ip, dp, dp, dp, dp, pi, dp, C.c_double, dp, pi]
        L.oracle_set_fd_libm.argtypes = [ip]
        _lib = L
    return _lib


def ref_lib():
    """The reference's own Dantzig solver compiled from /root/reference
    (oracle/_ref/libodelcp.so); None when it was not built."""
    global _ref
    if _ref is None and os.path.exists(REF_LIB):
        R = C.CDLL(REF_LIB)
        dp = C.POINTER(C.c_double)
        R.ref_dSolveLCP.argtypes = [C.c_int, dp, dp, dp, dp, C.c_int, dp, dp, C.POINTER(C.c_int), C.c_int]
        R.ref_dSolveLCP.restype = C.c_int
        _ref = R
    return _ref


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class OracleWorld:
    def __init__(self, world):
        self.desc, self._keep = world.desc()
        self.n = world.getNumDofs()
        self.nb = self.desc.num_bodies
        self.h = lib().oracle_world_create(C.byref(self.desc))
        self.snaps = None
        self.batch = 0
        self.cache = None

    def __del__(self):
        try:
            if self.snaps:
                lib().oracle_snapshots_destroy(self.snaps)
            lib().oracle_world_destroy(self.h)
        except Exception:
            pass

    def reset_cache(self, batch):
        self.cache = np.zeros((batch, MAX_LCP + 1))
        self.cache[:, 0] = -1

    def forward(self, state, forces):
        state = np.ascontiguousarray(np.atleast_2d(state), dtype=np.float64)
        forces = np.ascontiguousarray(np.atleast_2d(forces), dtype=np.float64)
        B = state.shape[0]
        if self.snaps is None or self.batch != B:
            if self.snaps:
                lib().oracle_snapshots_destroy(self.snaps)
            self.snaps = lib().oracle_snapshots_create(B)
            self.batch = B
        if self.cache is None or self.cache.shape[0] != B:
            self.reset_cache(B)
        nxt = np.zeros_like(state)
        lib().oracle_forward(self.h, B, _p(state), _p(forces), _p(self.cache), _p(nxt), self.snaps)
        return nxt

    def forward_forced(self, state, forces, forced_x, flags):
        """forward with the LCP path of selected worlds replayed (ForcedLcp,
        oracle.hpp): forced_x [B, MAX_LCP + 1] (column 0 = rows, < 0 = solve
        as usual, then the final x), flags [B, 3] = (gradient short-circuit,
        fallback cfm, friction removed).  Returns (next state, number of
        forced worlds whose row count did not match)."""
        state = np.ascontiguousarray(np.atleast_2d(state), dtype=np.float64)
        forces = np.ascontiguousarray(np.atleast_2d(forces), dtype=np.float64)
        fx = np.ascontiguousarray(forced_x, dtype=np.float64)
        fl = np.ascontiguousarray(flags, dtype=np.float64)
        B = state.shape[0]
        assert fx.shape == (B, MAX_LCP + 1) and fl.shape == (B, 3)
        if self.snaps is None or self.batch != B:
            if self.snaps:
                lib().oracle_snapshots_destroy(self.snaps)
            self.snaps = lib().oracle_snapshots_create(B)
            self.batch = B
        if self.cache is None or self.cache.shape[0] != B:
            self.reset_cache(B)
        nxt = np.zeros_like(state)
        bad = lib().oracle_forward_forced(self.h, B, _p(state), _p(forces), _p(self.cache), _p(nxt), self.snaps,
                                          _p(fx), _p(fl))
        return nxt, int(bad)

    def detect(self, state):
        """Contacts per world after the constraint filter (no step, no
        contact-count limit) and the unsupported-branch flags."""
        state = np.ascontiguousarray(np.atleast_2d(state), dtype=np.float64)
        B = state.shape[0]
        counts = np.zeros(B, dtype=np.int32)
        uns = np.zeros(B, dtype=np.int32)
        lib().oracle_detect(self.h, B, _p(state), _pi(counts), _pi(uns))
        return counts, uns

    def backward(self, grad_next):
        g = np.ascontiguousarray(np.atleast_2d(grad_next), dtype=np.float64)
        B = g.shape[0]
        gs = np.zeros_like(g)
        gf = np.zeros((B, self.n))
        lib().oracle_backward(self.h, B, self.snaps, _p(g), _p(gs), _p(gf))
        return gs, gf

    def jacobians(self):
        """getStateJacobian [B, 2n, 2n] and d(next state)/d(tau) [B, 2n, n]
        of the last forward (BackpropSnapshot.cpp:1230, :482)."""
        B, n = self.batch, self.n
        J = np.zeros((B, 2 * n, 2 * n))
        F = np.zeros((B, 2 * n, n))
        lib().oracle_jacobians(self.h, B, self.snaps, _p(J), _p(F))
        return J, F

    def constraint_force_jacobians(self, max_rows=MAX_LCP):
        """getJacobianOfConstraintForce of the last forward: [B, max_rows, 3n],
        row r = d f_c[r] / d(q, v, tau) (BackpropSnapshot.cpp:2723), zero past
        the world's clamping count."""
        out = np.zeros((self.batch, max_rows, 3 * self.n))
        lib().oracle_constraint_force_jacobians(self.h, self.batch, self.snaps, _p(out), max_rows)
        return out

    def mass_matrix(self, q):
        q = np.ascontiguousarray(q, dtype=np.float64)
        M = np.zeros((self.n, self.n))
        lib().oracle_mass_matrix(self.h, _p(q), _p(M))
        return M

    def coriolis_gravity(self, q, v):
        q = np.ascontiguousarray(q, dtype=np.float64)
        v = np.ascontiguousarray(v, dtype=np.float64)
        Cg = np.zeros(self.n)
        lib().oracle_coriolis_gravity(self.h, _p(q), _p(v), _p(Cg))
        return Cg

    def forward_dynamics(self, q, v, tau):
        q, v, tau = (np.ascontiguousarray(x, dtype=np.float64) for x in (q, v, tau))
        ddq = np.zeros(self.n)
        lib().oracle_forward_dynamics(self.h, _p(q), _p(v), _p(tau), _p(ddq))
        return ddq

    def body_transforms(self, q):
        q = np.ascontiguousarray(q, dtype=np.float64)
        T = np.zeros((self.nb, 12))
        lib().oracle_body_transforms(self.h, _p(q), _p(T))
        return T.reshape(self.nb, 3, 4)

    def jacobian_of_c(self, q, v, wrt_pos):
        q = np.ascontiguousarray(q, dtype=np.float64)
        v = np.ascontiguousarray(v, dtype=np.float64)
        J = np.zeros((self.n, self.n))
        lib().oracle_jacobian_of_c(self.h, _p(q), _p(v), 1 if wrt_pos else 0, _p(J))
        return J

    def num_contacts(self, b=0):
        return lib().oracle_num_contacts(self.snaps, b)


def set_fd_libm(on):
    """Test switch: the FreeJoint FD blocks' perturbed integrations through
    std::sin / cos / acos (the reference's, Geometry.cpp:539 / :720) instead
    of the fixed IEEE sequence the device shares (nimble_oracle.cpp fd*)."""
    lib().oracle_set_fd_libm(1 if on else 0)


def _pi(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


def contacts(ow: "OracleWorld", b=0, maxc=64):
    out = np.zeros((maxc, 10))
    k = lib().oracle_contacts(ow.snaps, b, _p(out), maxc)
    return out[:k]


def lcp_debug(ow: "OracleWorld", b=0, max_rows=MAX_LCP):
    mapping = np.zeros(max_rows, dtype=np.int32)
    x = np.zeros(max_rows)
    m = lib().oracle_lcp_debug(ow.snaps, b, _pi(mapping), _p(x), max_rows)
    return mapping[:m].copy(), x[:m].copy()


def lcp_flags(ow: "OracleWorld", b=0):
    """[shortCircuit, ignoredFriction, cfm, numClamping, numUpperBound, unsupportedContacts, lcpReduced]"""
    out = np.zeros(7)
    lib().oracle_lcp_flags(ow.snaps, b, _p(out))
    return out


def lcp_fc(ow: "OracleWorld", b=0, maxc=MAX_LCP):
    fc = np.zeros(maxc)
    k = lib().oracle_lcp_fc(ow.snaps, b, _p(fc), maxc)
    return fc[:k].copy()


def lcp_cols(ow: "OracleWorld", b=0):
    """J^T columns (n x m) of world b's LCP rows."""
    out = np.zeros(ow.n * MAX_LCP)
    m = lib().oracle_lcp_cols(ow.snaps, b, _p(out), out.size)
    return out[:ow.n * m].reshape(ow.n, m).copy()


def lcp_problem(ow: "OracleWorld", b=0, max_rows=MAX_LCP):
    """(A, b, lo, hi, findex) of world b's LCP (A without the fallback CFM)."""
    A = np.zeros(max_rows * max_rows)
    bb, lo, hi = np.zeros(max_rows), np.zeros(max_rows), np.zeros(max_rows)
    fi = np.zeros(max_rows, dtype=np.int32)
    m = lib().oracle_lcp_problem(ow.snaps, b, _p(A), _p(bb), _p(lo), _p(hi), _pi(fi), max_rows)
    return A[:m * m].reshape(m, m).copy(), bb[:m].copy(), lo[:m].copy(), hi[:m].copy(), fi[:m].copy()


def dantzig(A, b, lo, hi, findex, early=False):
    """The oracle's restatement of dSolveLCP."""
    A = np.ascontiguousarray(A, dtype=np.float64)
    n = A.shape[0]
    b, lo, hi = (np.ascontiguousarray(v, dtype=np.float64).copy() for v in (b, lo, hi))
    fi = np.ascontiguousarray(findex, dtype=np.int32).copy()
    x = np.zeros(n)
    ok = lib().oracle_dantzig(n, _p(A), _p(b), _p(lo), _p(hi), _pi(fi), _p(x), 1 if early else 0)
    return bool(ok), x


def ref_dantzig(A, b, lo, hi, findex, early=False):
    """The reference's own dSolveLCP (oracle/_ref/libodelcp.so); None if unbuilt."""
    R = ref_lib()
    if R is None:
        return None
    n = A.shape[0]
    nskip = n if n <= 1 else (((n - 1) | 3) + 1)
    Ap = np.zeros((n, nskip))
    Ap[:, :n] = A
    Ap = np.ascontiguousarray(Ap)
    b, lo, hi = (np.ascontiguousarray(v, dtype=np.float64).copy() for v in (b, lo, hi))
    fi = np.ascontiguousarray(findex, dtype=np.int32).copy()
    x = np.zeros(n)
    w = np.zeros(n)
    ok = R.ref_dSolveLCP(n, _p(Ap), _p(x), _p(b), _p(w), 0, _p(lo), _p(hi), _pi(fi), 1 if early else 0)
    return bool(ok), x


def ref_dantzig_ambiguous(A, b, lo, hi, findex, seed, trials=512, effective=True):
    """True when the reference's own dSolveLCP (oracle/_ref) gives both
    outcomes under 1e-15-relative symmetric perturbations of A; with
    `effective` the outcome is success AND isLCPSolutionValid (what the
    contact solver keeps), else the raw success flag.  None if unbuilt."""
    if ref_lib() is None:
        return None
    rng = np.random.default_rng(seed)
    outs = set()
    for _ in range(trials):
        N = rng.standard_normal(A.shape)
        Ap = A * (1 + 1e-15 * (N + N.T) / 2)
        ok, x = ref_dantzig(Ap, b, lo, hi, findex, True)
        outs.add(bool(ok and (not effective or lcp_valid(A, x, b, hi, lo, findex))))
        if len(outs) == 2:
            return True
    return False


def classify(A, b, lo, hi, findex, x):
    """The gradient short-circuit (constructMatrices + standardisation) on a
    raw problem from warm start x, Q from A's entries; (standardized, x)."""
    A = np.ascontiguousarray(A, dtype=np.float64)
    b, lo, hi = (np.ascontiguousarray(v, dtype=np.float64) for v in (b, lo, hi))
    fi = np.ascontiguousarray(findex, dtype=np.int32)
    xo = np.ascontiguousarray(x, dtype=np.float64).copy()
    ok = lib().oracle_classify(A.shape[0], _p(A), _p(b), _p(lo), _p(hi), _pi(fi), _p(xo))
    return bool(ok), xo


def classify_ambiguous(A, b, lo, hi, findex, warm, seed, trials=64):
    """True when the short-circuit outcome flips under 1e-15-relative
    symmetric perturbations of A (warm: the step's warm start, or None for
    guessSolution of the perturbed A, as the step without a cache)."""
    rng = np.random.default_rng(seed)
    outs = set()
    for _ in range(trials):
        N = rng.standard_normal(A.shape)
        Ap = A * (1 + 1e-15 * (N + N.T) / 2)
        x0 = guess_solution(Ap, b, findex) if warm is None else warm
        outs.add(classify(Ap, b, lo, hi, findex, x0)[0])
        if len(outs) == 2:
            return True
    return False


def lcp_path(A, b, lo, hi, findex, warm, fallback_cfm):
    """The LCP part of the oracle's step on a raw problem, Q from A's entries:
    the short-circuit classification from `warm` (None: guessSolution), else
    the fallback cascade, then the final classification.  Returns a hashable
    outcome (shortCircuit, ignoredFriction, cfm, numClamping, numUpperBound,
    lcpReduced, per-row mapping) -- the fields `_same_path` compares."""
    A = _f(A)
    m = A.shape[0]
    b, lo, hi, fi = _f(b), _f(lo), _f(hi), _i(findex)
    x0 = guess_solution(A, b, fi) if warm is None else _f(warm)
    flags = np.zeros(6)
    mapping = np.zeros(m, np.int32)
    lib().oracle_lcp_path(m, _p(A), _p(b), _p(lo), _p(hi), _pi(fi), _p(x0), float(fallback_cfm), _p(flags),
                          _pi(mapping))
    return tuple(float(v) for v in flags) + (tuple(int(v) for v in mapping),)


def path_ambiguous(A, b, lo, hi, findex, warm, fallback_cfm, seed, trials=64):
    """True when the whole LCP path (lcp_path: short-circuit, cascade, final
    classification) takes more than one outcome under 1e-15-relative
    symmetric perturbations of A: the probe of splits that are neither at the
    short-circuit nor at Dantzig's outcome (friction removal, final
    classification)."""
    rng = np.random.default_rng(seed)
    outs = {lcp_path(A, b, lo, hi, findex, warm, fallback_cfm)}
    for _ in range(trials):
        N = rng.standard_normal(A.shape)
        outs.add(lcp_path(A * (1 + 1e-15 * (N + N.T) / 2), b, lo, hi, findex, warm, fallback_cfm))
        if len(outs) >= 2:
            return True
    return False


def cod_solve(A, b):
    A = np.ascontiguousarray(A, dtype=np.float64)
    m, n = A.shape
    b = np.ascontiguousarray(b, dtype=np.float64)
    x = np.zeros(n)
    lib().oracle_cod_solve(_p(A), m, n, _p(b), _p(x))
    return x


def box_box(size1, T1, size2, T2):
    """dBoxBox restated; rows of (point3, normal3, depth, type, edgeAFixed3,
    edgeADir3, edgeBFixed3, edgeBDir3) -- the edge fields for EDGE_EDGE."""
    out = np.zeros((16, 20))
    s1, s2 = (np.ascontiguousarray(s, dtype=np.float64) for s in (size1, size2))
    t1, t2 = (np.ascontiguousarray(np.asarray(T, dtype=np.float64)[:3, :4]) for T in (T1, T2))
    k = lib().oracle_box_box(_p(s1), _p(t1), _p(s2), _p(t2), _p(out))
    return out[:k]


def capsule_box(size, T_box, height, radius, T_capsule, box_first=True, clip=0.03):
    """collideBoxCapsule (box_first) / collideCapsuleBox restated; rows of
    (point3, normal3, depth, type) and an `unsupported` flag."""
    out = np.zeros((16, 8))
    s = np.ascontiguousarray(size, dtype=np.float64)
    tb, tc = (np.ascontiguousarray(np.asarray(T, dtype=np.float64)[:3, :4]) for T in (T_box, T_capsule))
    k = lib().oracle_capsule_box(_p(s), _p(tb), C.c_double(height), C.c_double(radius), _p(tc),
                                 1 if box_first else 0, C.c_double(clip), _p(out))
    unsupported = k < 0
    if k < 0:
        k = -1 - k
    return out[:k], unsupported


def mesh_box(verts, scale, T_mesh, size, T_box, mesh_first=True, clip=0.03):
    """collideMeshBox (mesh_first) / collideBoxMesh restated; rows of
    (point3, normal3, depth, type, edgeAFixed3, edgeADir3, edgeBFixed3,
    edgeBDir3) and an `unsupported` flag (empty witness set)."""
    v = np.ascontiguousarray(np.asarray(verts, dtype=np.float64).reshape(-1, 3))
    out = np.zeros((256, 20))
    sc, sz = (np.ascontiguousarray(x, dtype=np.float64) for x in (scale, size))
    tm, tb = (np.ascontiguousarray(np.asarray(T, dtype=np.float64)[:3, :4]) for T in (T_mesh, T_box))
    k = lib().oracle_mesh_box(_p(v), v.shape[0], _p(sc), _p(tm), _p(sz), _p(tb), 1 if mesh_first else 0,
                              C.c_double(clip), _p(out))
    unsupported = k < 0
    if k < 0:
        k = -1 - k
    return out[:k], unsupported


def box_box_as_mesh(size1, T1, size2, T2):
    """collideBoxBoxAsMesh (DARTCollide.cpp:3889) restated; rows as mesh_box."""
    out = np.zeros((64, 20))
    s1, s2 = (np.ascontiguousarray(s, dtype=np.float64) for s in (size1, size2))
    t1, t2 = (np.ascontiguousarray(np.asarray(T, dtype=np.float64)[:3, :4]) for T in (T1, T2))
    k = lib().oracle_box_box_as_mesh(_p(s1), _p(t1), _p(s2), _p(t2), _p(out))
    assert k >= 0, "empty witness set"
    return out[:k]


SHAPE_TYPES = {"box": 0, "sphere": 1, "capsule": 2}


def collide_pair(shape1, T1, shape2, T2, clip=0.03):
    """One shape pair through the oracle's detector dispatch (the reference's
    collide<Shape1, Shape2> of DARTCollide.cpp).  shapeK = (kind, size) with
    kind box / sphere / capsule and size as in nimble_world_desc (box full
    size; sphere (r,); capsule (r, h)).  Rows of (point3, normal3, depth,
    type) in this package's type numbering, and an `unsupported` flag."""
    out = np.zeros((16, 8))
    sz = []
    for kind, size in (shape1, shape2):
        v = np.zeros(3)
        s_ = np.atleast_1d(np.asarray(size, dtype=np.float64))
        v[:len(s_)] = s_
        sz.append(v)
    t1, t2 = (np.ascontiguousarray(np.asarray(T, dtype=np.float64)[:3, :4]) for T in (T1, T2))
    k = lib().oracle_collide_pair(SHAPE_TYPES[shape1[0]], _p(sz[0]), _p(t1), SHAPE_TYPES[shape2[0]], _p(sz[1]),
                                  _p(t2), C.c_double(clip), _p(out), 16)
    unsupported = k < 0
    if k < 0:
        k = -1 - k
    return out[:k], unsupported


def _f(v):
    return np.ascontiguousarray(v, dtype=np.float64).copy()


def _i(v):
    return np.ascontiguousarray(v, dtype=np.int32).copy()


def lcp_reduce(A, x, b, hi, lo, fi):
    """LCPUtils::reduce restated: (A_r, x_r, b_r, hi_r, lo_r, fi_r, map) with
    x_full = x_r[map] (mapOut * x_r)."""
    A = _f(A)
    m = A.shape[0]
    x, b, hi, lo, fi = _f(x), _f(b), _f(hi), _f(lo), _i(fi)
    Ao, xo, bo, ho, lo_o = np.zeros(m * m), np.zeros(m), np.zeros(m), np.zeros(m), np.zeros(m)
    fo, mp = np.zeros(m, np.int32), np.zeros(m, np.int32)
    mr = lib().oracle_lcp_reduce(m, _p(A), _p(x), _p(b), _p(hi), _p(lo), _pi(fi), _p(Ao), _p(xo), _p(bo), _p(ho),
                                 _p(lo_o), _pi(fo), _pi(mp))
    return (Ao[:mr * mr].reshape(mr, mr), xo[:mr], bo[:mr], ho[:mr], lo_o[:mr], fo[:mr], mp)


def pgs(A, x, b, lo, hi, fi, options=None):
    """PgsBoxedLcpSolver::solve restated; options = (maxIter, deltaX, relTol,
    epsDiv) for PgsBoxedLcpSolver::Option, None for the default."""
    A, x, b, lo, hi, fi = _f(A), _f(x), _f(b), _f(lo), _f(hi), _i(fi)
    n = A.shape[0]
    if options is None:
        ok = lib().oracle_pgs(n, _p(A), _p(x), _p(b), _p(lo), _p(hi), _pi(fi))
    else:
        it, dx, rt, eps = options
        ok = lib().oracle_pgs_opt(n, _p(A), _p(x), _p(b), _p(lo), _p(hi), _pi(fi), int(it), dx, rt, eps)
    return bool(ok), x


def lcp_valid(A, x, b, hi, lo, fi, ignore_friction=False):
    """LCPUtils::isLCPSolutionValid restated."""
    A, x, b, hi, lo, fi = _f(A), _f(x), _f(b), _f(hi), _f(lo), _i(fi)
    return bool(lib().oracle_lcp_valid(A.shape[0], _p(A), _p(x), _p(b), _p(hi), _p(lo), _pi(fi),
                                       1 if ignore_friction else 0))


def guess_solution(A, b, fi):
    A, b, fi = _f(A), _f(b), _i(fi)
    x = np.zeros(A.shape[0])
    lib().oracle_guess_solution(A.shape[0], _p(A), _p(b), _pi(fi), _p(x))
    return x


def lcp_cascade(A, b, lo, hi, fi, warm, fallback_cfm=1e-4):
    """BoxedLcpConstraintSolver::solveLcp's fallbacks (reduce + Dantzig, CFM +
    reduce + PGS, removeFriction + PGS): (x, path, reduced, ignoredFriction, cfm)."""
    A, b, lo, hi, fi, x = _f(A), _f(b), _f(lo), _f(hi), _i(fi), _f(warm)
    info = np.zeros(4)
    lib().oracle_lcp_cascade(A.shape[0], _p(A), _p(b), _p(lo), _p(hi), _pi(fi), _p(x), fallback_cfm, _p(info))
    return x, int(info[0]), bool(info[1]), bool(info[2]), float(info[3])
