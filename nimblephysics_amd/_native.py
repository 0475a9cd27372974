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
        L.nimble_backward_masses.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 7 + [C.c_void_p]
        L.nimble_backward_masses.restype = C.c_int
        L.nimble_backward_inertia.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 7 + [C.c_void_p]
        L.nimble_backward_inertia.restype = C.c_int
        L.nimble_last_error.argtypes = []
        L.nimble_last_error.restype = C.c_char_p
        L.nimble_jacobian_workspace_doubles.argtypes = [C.c_void_p, C.c_int32]
        L.nimble_jacobian_workspace_doubles.restype = C.c_int64
        L.nimble_jacobians.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 6 + [C.c_void_p]
        L.nimble_constraint_force_jacobians.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 6 + [C.c_void_p]
        L.nimble_constraint_force_jacobians.restype = C.c_int
        L.nimble_jacobians.restype = C.c_int
        L.nimble_num_collision_pairs.argtypes = [C.c_void_p]
        L.nimble_num_collision_pairs.restype = C.c_int32
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


# snapshot header (csrc/pool_sizes.h) and status bits (csrc/contact.cuh)
SN_NCON, SN_M, SN_NC, SN_NU, SN_CFM, SN_STATUS = 0, 1, 2, 3, 4, 5
MAX_CONTACTS = 42
MAX_LCP = 3 * MAX_CONTACTS  # include/nimble_amd.h NIMBLE_MAX_LCP
CREC, EDGE_REC, SN_ROWREC = 13, 12, 12  # csrc/pool_sizes.h


def snapshot_layout(n: int, timing: bool = False) -> dict:
    """Per-world snapshot offsets (doubles) of csrc/pool_sizes.h for a model
    with n dofs: header, contact records, row records, f_c, v_f, y_f, the
    backward blocks (A_c, A_c_ub_E, pinv(Q)^T, Q), EDGE metadata, the
    stage-timing build's stamps (`timing`: 128 doubles, ahead of the
    workspace) and the start of the HBM workspace.  tests/test_wave_emu.py
    checks it against the header."""
    a8 = lambda x: ((x + 7) // 8) * 8
    L = {"contacts": 16}
    L["rows"] = L["contacts"] + MAX_CONTACTS * CREC
    L["fc"] = L["rows"] + MAX_LCP * SN_ROWREC
    L["vf"] = L["fc"] + MAX_LCP
    L["yf"] = L["vf"] + n
    L["ac"] = a8(L["yf"] + n)
    L["acube"] = L["ac"] + n * MAX_LCP
    L["pt"] = L["acube"] + n * MAX_LCP
    L["q"] = L["pt"] + MAX_LCP * MAX_LCP
    L["edge"] = L["q"] + MAX_LCP * MAX_LCP
    L["stamps"] = a8(L["edge"] + MAX_CONTACTS * EDGE_REC)
    L["workspace"] = L["stamps"] + (128 if timing else 0)
    return L
SN_FC = 16 + 13 * MAX_CONTACTS + 12 * MAX_LCP  # NIMBLE_SNAPSHOT_FC: clamping impulses f_c
ST_CONTACT_OVERFLOW, ST_UNSUPPORTED_SHAPE, ST_DROPPED_OVERFLOW, ST_REDUCED, ST_LCP_TOO_LARGE = 1, 2, 4, 8, 16
ST_PROTOCOL = 64  # a wait between a world's two waves hit the kernel's deadlock guard
ST_DIVERGES = ST_CONTACT_OVERFLOW | ST_UNSUPPORTED_SHAPE | ST_DROPPED_OVERFLOW | ST_LCP_TOO_LARGE | ST_PROTOCOL
SN_PIVOTS, SN_SWEEPS, SN_SOLVER_FLOPS = 9, 10, 11  # the LCP solvers' executed work (include/nimble_amd.h)
MAX_SOLVED_LCP = 128  # include/nimble_amd.h NIMBLE_MAX_SOLVED_LCP (two rows per lane above 64)


class ContactCapacityError(RuntimeError):
    """A world's contact set does not fit the batched path (more contacts than
    NIMBLE_MAX_CONTACTS, a shape pair without a collider, or an overflowing
    dropped-contact list): its step would differ from the reference's."""


def status_message(bits: int) -> str:
    why = []
    if bits & ST_CONTACT_OVERFLOW:
        why.append("more contacts than NIMBLE_MAX_CONTACTS")
    if bits & ST_UNSUPPORTED_SHAPE:
        why.append("a shape pair without a collider on this path")
    if bits & ST_DROPPED_OVERFLOW:
        why.append("dropped-contact list overflow")
    if bits & ST_LCP_TOO_LARGE:
        why.append(f"more than {MAX_SOLVED_LCP} LCP rows")
    if bits & ST_PROTOCOL:
        why.append("the kernel's two-wave deadlock guard expired (step finished on one wave)")
    return ", ".join(why)


class DeviceWorld:
    """A world model uploaded to one device (nimble_world_create)."""

    def __init__(self, world, device_index: int = 0):
        L = lib()
        desc, keep = world.desc()
        self._keep = keep
        h = C.c_void_p()
        _check(L.nimble_world_create(C.byref(desc), C.byref(h)))
        self.h = h
        self.device_index = int(device_index)
        self.n = world.getNumDofs()
        self.nb = int(desc.num_bodies)
        self.snapshot_doubles = int(L.nimble_snapshot_doubles(h))
        self.cache_doubles = int(L.nimble_lcp_cache_doubles(h))
        self.num_pairs = int(L.nimble_num_collision_pairs(h))

    def close(self):
        if self.h:
            lib().nimble_world_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _on_my_device(self, *tensors):
        for t in tensors:
            if t is not None and t.device.index != self.device_index:
                raise RuntimeError(f"tensor on {t.device}, world model uploaded to cuda:{self.device_index}")

    def _shapes(self, B, state=None, forces=None, snapshot=None, cache=None):
        n = self.n
        if state is not None and tuple(state.shape) != (B, 2 * n):
            raise ValueError(f"state shape {tuple(state.shape)} != ({B}, {2 * n})")
        if forces is not None and tuple(forces.shape) != (B, n):
            raise ValueError(f"forces shape {tuple(forces.shape)} != ({B}, {n})")
        if snapshot is not None and (snapshot.shape[0] < B or snapshot.shape[1] != self.snapshot_doubles):
            raise ValueError(f"snapshot shape {tuple(snapshot.shape)}: this world needs [{B}, {self.snapshot_doubles}]")
        if cache is not None and (cache.shape[0] < B or cache.shape[1] != self.cache_doubles):
            raise ValueError(f"LCP cache shape {tuple(cache.shape)}: this world needs [{B}, {self.cache_doubles}]")
        for t in (state, forces, snapshot, cache):
            if t is not None and not t.is_contiguous():
                raise ValueError("nimblephysics_amd buffers must be contiguous")

    def status(self, snapshot):
        """Status bits per world ([B] int32, device) of the forward that wrote
        `snapshot`; zeros for models without collision pairs."""
        import torch
        if self.num_pairs == 0:
            return torch.zeros(snapshot.shape[0], dtype=torch.int32, device=snapshot.device)
        return snapshot[:, SN_STATUS].to(torch.int32)

    def forward(self, state, forces, lcp_cache, next_state, snapshot, stream_ptr: int):
        _require_device(state, forces, lcp_cache, next_state, snapshot)
        B = state.shape[0]
        self._on_my_device(state, forces, lcp_cache, next_state, snapshot)
        self._shapes(B, state, forces, snapshot, lcp_cache)
        _check(lib().nimble_forward(self.h, B, _ptr(state), _ptr(forces), _ptr(lcp_cache), _ptr(next_state),
                                    _ptr(snapshot), C.c_void_p(stream_ptr)))

    def backward(self, state, forces, snapshot, grad_next, grad_state, grad_forces, stream_ptr: int):
        _require_device(state, forces, snapshot, grad_next, grad_state, grad_forces)
        B = state.shape[0]
        self._on_my_device(state, forces, snapshot, grad_next, grad_state, grad_forces)
        self._shapes(B, state, forces, snapshot)
        self._shapes(B, grad_next, grad_forces)
        self._shapes(B, grad_state)
        _check(lib().nimble_backward(self.h, B, _ptr(state), _ptr(forces), _ptr(snapshot), _ptr(grad_next),
                                     _ptr(grad_state), _ptr(grad_forces), C.c_void_p(stream_ptr)))

    def backward_masses(self, state, forces, snapshot, grad_next, grad_state, grad_forces, grad_masses,
                        stream_ptr: int):
        """backward() plus dL/d(body masses) [B, num_bodies] (nimble_backward_masses)."""
        _require_device(state, forces, snapshot, grad_next, grad_state, grad_forces, grad_masses)
        B = state.shape[0]
        self._on_my_device(state, forces, snapshot, grad_next, grad_state, grad_forces, grad_masses)
        self._shapes(B, state, forces, snapshot)
        self._shapes(B, grad_next, grad_forces)
        self._shapes(B, grad_state)
        if tuple(grad_masses.shape) != (B, self.nb) or not grad_masses.is_contiguous():
            raise ValueError(f"grad_masses shape {tuple(grad_masses.shape)} != ({B}, {self.nb})")
        _check(lib().nimble_backward_masses(self.h, B, _ptr(state), _ptr(forces), _ptr(snapshot), _ptr(grad_next),
                                            _ptr(grad_state), _ptr(grad_forces), _ptr(grad_masses),
                                            C.c_void_p(stream_ptr)))

    def backward_inertia(self, state, forces, snapshot, grad_next, grad_state, grad_forces, grad_inertia,
                         stream_ptr: int):
        """backward() plus dL/d(body inertia parameters) [B, num_bodies, 10] in
        INERTIA_FULL order (mass, COM xyz, Ixx Iyy Izz Ixy Ixz Iyz;
        nimble_backward_inertia)."""
        _require_device(state, forces, snapshot, grad_next, grad_state, grad_forces, grad_inertia)
        B = state.shape[0]
        self._on_my_device(state, forces, snapshot, grad_next, grad_state, grad_forces, grad_inertia)
        self._shapes(B, state, forces, snapshot)
        self._shapes(B, grad_next, grad_forces)
        self._shapes(B, grad_state)
        if tuple(grad_inertia.shape) != (B, self.nb, 10) or not grad_inertia.is_contiguous():
            raise ValueError(f"grad_inertia shape {tuple(grad_inertia.shape)} != ({B}, {self.nb}, 10)")
        _check(lib().nimble_backward_inertia(self.h, B, _ptr(state), _ptr(forces), _ptr(snapshot), _ptr(grad_next),
                                             _ptr(grad_state), _ptr(grad_forces), _ptr(grad_inertia),
                                             C.c_void_p(stream_ptr)))

    def jacobians(self, state, forces, snapshot, stream_ptr: int):
        """(d next_state / d state [B, 2n, 2n], d next_state / d forces
        [B, 2n, n]) of the forward that wrote `snapshot` (nimble_jacobians)."""
        import torch
        _require_device(state, forces, snapshot)
        B = state.shape[0]
        self._on_my_device(state, forces, snapshot)
        self._shapes(B, state, forces, snapshot)
        n = self.n
        J = torch.empty((B, 2 * n, 2 * n), dtype=torch.float64, device=state.device)
        F = torch.empty((B, 2 * n, n), dtype=torch.float64, device=state.device)
        wsd = int(lib().nimble_jacobian_workspace_doubles(self.h, B))
        ws = torch.empty(wsd, dtype=torch.float64, device=state.device) if wsd > 0 else None
        _check(lib().nimble_jacobians(self.h, B, _ptr(state), _ptr(forces), _ptr(snapshot), _ptr(J), _ptr(F),
                                      _ptr(ws), C.c_void_p(stream_ptr)))
        return J, F

    def constraint_force_jacobians(self, state, forces, snapshot, stream_ptr: int):
        """(d f_c / d state [B, MAX_LCP, 2n], d f_c / d forces [B, MAX_LCP, n])
        of the forward that wrote `snapshot` (nimble_constraint_force_jacobians;
        rows past each world's clamping count are zero)."""
        import torch
        _require_device(state, forces, snapshot)
        B = state.shape[0]
        self._on_my_device(state, forces, snapshot)
        self._shapes(B, state, forces, snapshot)
        n = self.n
        Js = torch.empty((B, MAX_LCP, 2 * n), dtype=torch.float64, device=state.device)
        Jf = torch.empty((B, MAX_LCP, n), dtype=torch.float64, device=state.device)
        wsd = int(lib().nimble_jacobian_workspace_doubles(self.h, B))
        ws = torch.empty(wsd, dtype=torch.float64, device=state.device) if wsd > 0 else None
        _check(lib().nimble_constraint_force_jacobians(self.h, B, _ptr(state), _ptr(forces), _ptr(snapshot),
                                                       _ptr(Js), _ptr(Jf), _ptr(ws), C.c_void_p(stream_ptr)))
        return Js, Jf


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
    ndof = [{0: 0, 1: 1, 2: 1, 3: 6, 4: 3, 5: 3}[int(t)] for t in jt]
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
