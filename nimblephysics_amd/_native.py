"""ctypes binding of the C-ABI in include/nimble_amd.h (libnimble_amd.so).

The product path has no CPU fallback: if the HIP library is missing or no
ROCm device is present, calls raise instead of silently computing elsewhere.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NIMBLE_AMD_LIB") or os.path.join(_HERE, "libnimble_amd.so")

_lib = None


class NativeLibraryMissing(ImportError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryMissing(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH)
        L.nimble_world_create.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
        L.nimble_world_create.restype = C.c_int
        L.nimble_world_destroy.argtypes = [C.c_void_p]
        L.nimble_world_destroy.restype = C.c_int
        L.nimble_snapshot_doubles.argtypes = [C.c_void_p]
        L.nimble_snapshot_doubles.restype = C.c_int64
        L.nimble_lcp_cache_doubles.argtypes = [C.c_void_p]
        L.nimble_lcp_cache_doubles.restype = C.c_int64
        L.nimble_forward.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 5 + [C.c_void_p]
        L.nimble_forward.restype = C.c_int
        L.nimble_backward.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 6 + [C.c_void_p]
        L.nimble_backward.restype = C.c_int
        L.nimble_last_error.argtypes = []
        L.nimble_last_error.restype = C.c_char_p
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise RuntimeError(f"nimble_amd error {rc}: {lib().nimble_last_error().decode()}")


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


def _require_device(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError("nimblephysics_amd runs on the ROCm device only; got a CPU tensor")
        if t is not None and t.dtype.is_floating_point and str(t.dtype) != "torch.float64":
            raise TypeError("nimblephysics_amd computes in float64 (the reference's s_t); got " + str(t.dtype))


class DeviceWorld:
    """A world model uploaded to the device (nimble_world_create)."""

    def __init__(self, world):
        L = lib()
        desc, keep = world.desc()
        self._keep = keep
        h = C.c_void_p()
        _check(L.nimble_world_create(C.byref(desc), C.byref(h)))
        self.h = h
        self.n = world.getNumDofs()
        self.snapshot_doubles = int(L.nimble_snapshot_doubles(h))
        self.cache_doubles = int(L.nimble_lcp_cache_doubles(h))

    def close(self):
        if self.h:
            lib().nimble_world_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def forward(self, state, forces, lcp_cache, next_state, snapshot, stream_ptr: int):
        _require_device(state, forces, lcp_cache, next_state, snapshot)
        B = state.shape[0]
        _check(lib().nimble_forward(self.h, B, _ptr(state), _ptr(forces), _ptr(lcp_cache), _ptr(next_state),
                                    _ptr(snapshot), C.c_void_p(stream_ptr)))

    def backward(self, state, forces, snapshot, grad_next, grad_state, grad_forces, stream_ptr: int):
        _require_device(state, forces, snapshot, grad_next, grad_state, grad_forces)
        B = state.shape[0]
        _check(lib().nimble_backward(self.h, B, _ptr(state), _ptr(forces), _ptr(snapshot), _ptr(grad_next),
                                     _ptr(grad_state), _ptr(grad_forces), C.c_void_p(stream_ptr)))


def contact_flop_estimate(world, rows: float, clamping: float) -> dict:
    """Algorithmic fp64 FLOPs per world of the contact stage for `rows` LCP
    rows of which `clamping` clamp (batch averages), FMA = 2.  Forward: J^T
    columns, Y = L^-1 J^T, A = Y^T Y, b, guess + standardisation COD solves,
    validity checks, impulses, and the backward precompute (A_c, A_c_ub_E, Q,
    COD + pinv(Q), rank check).  Backward: the nine Minv products (two batched
    Cholesky solves), the clamping-space vector chain, per-row G vectors,
    chain twists, grouped contact-geometry terms and the M-derivative fields.
    Iterative fallbacks (Dantzig pivots, PGS sweeps) are not counted."""
    d = world.desc_arrays()
    nb, n = int(d["num_bodies"]), int(d["num_dofs"])
    m, c = float(rows), float(clamping)
    if m <= 0:
        return {"forward": 0.0, "backward": 0.0}
    cod = lambda k: 4.0 / 3.0 * k ** 3 + 4.0 * k * k  # noqa: E731
    fwd = (14 * n * m + n * n * m + m * m * n + 2 * n * m + 2 * cod(m) + 4 * m * m + 2 * n * m + n * n
           + 2 * 14 * n * c + 2 * c * c + cod(c) + 4 * c ** 3 + 2 * c ** 3)
    groups = 2.0
    bwd = (18 * n * n + 12 * 2 * n * c + 6 * 2 * c * c + 12 * m * n + 24 * m * n
           + groups * (12 * m * n + 18 * nb * n) + 8 * nb * (12 * n + 100) + 20 * n)
    return {"forward": float(fwd), "backward": float(bwd)}


def flop_estimate(world, rows: float = 0.0, clamping: float = 0.0) -> dict:
    """Algorithmic fp64 FLOPs per world for one launch of each kernel, counted
    from the implemented algorithm's loop structure (FMA = 2 FLOPs): forward =
    kinematics, world-frame composites, CRBA mass matrix, Cholesky + solve
    (+ contact stage); backward = accelerations at a*, derivative composites,
    one closed-form dID/dq and dC/dv column per dof (only related body pairs)
    and two solves (+ contact terms)."""
    d = world.desc_arrays()
    nb, n = int(d["num_bodies"]), int(d["num_dofs"])
    parent = list(d["parent"])
    jt = list(d["joint_type"])
    ndof = [0 if t == 0 else (6 if t == 3 else 1) for t in jt]
    anc = []
    for b in range(nb):
        s = {b}
        p = parent[b]
        while p >= 0:
            s.add(p)
            p = parent[p]
        anc.append(s)
    dof_body = []
    for b in range(nb):
        dof_body += [b] * ndof[b]
    kin = sum(330 + 60 * ndof[b] for b in range(nb))
    comp = nb * 330 + nb * 42
    related_pairs = sum(1 for j in range(n) for k in range(j + 1)
                        if dof_body[k] in anc[dof_body[j]] or dof_body[j] in anc[dof_body[k]])
    mass = related_pairs * 84 + n * 12
    chol = n ** 3 / 3.0 + n ** 2
    solve = 2.0 * n * n
    fwd = kin + comp + mass + chol + solve + 10 * n
    dcomp = nb * 1800 + nb * 126
    lanes = 0.0
    for k in range(n):
        b = dof_body[k]
        lanes += 1020
        for c in range(nb):
            if ndof[c] == 0:
                continue
            if b in anc[c]:
                lanes += (1020 if c != b else 0) + 80 * ndof[c]
            elif c in anc[b]:
                lanes += 50 * ndof[c]
    # the backward reuses the forward's kinematics, composite inertias and
    # Cholesky factor (snapshot dynamics cache): accelerations + derivative
    # composites + the per-direction columns + two solves
    accel = nb * n * 30
    bwd = accel + dcomp + lanes + 2 * solve + 20 * n
    c = contact_flop_estimate(world, rows, clamping)
    return {"forward": float(fwd + c["forward"]), "backward": float(bwd + c["backward"])}
