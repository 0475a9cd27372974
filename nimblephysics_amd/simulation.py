"""World: the reference's dart.simulation.World surface for the timestep.

Mirrors dart/simulation/World.hpp/.cpp: construction defaults (World.cpp:70:
gravity (0,0,-9.81), dt 0.001, parallel pos/vel updates on, fallback CFM 1e-4,
contact clipping depth 0.03, penetration correction off), skeleton loading,
state/action accessors (World.cpp:2024-2130).  A World describes ONE model;
its state vectors are the single-world state.  The batched device path
(``timestep`` with a 2-D state) advances many independent copies of the same
model at once; the per-copy LCP warm-start caches live in ``BatchState``.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np

from . import dynamics as dyn
from . import urdf as _urdf
from ._desc import NIMBLE_MAX_BODIES, NIMBLE_MAX_DOFS, NIMBLE_MAX_SHAPES, build_desc


class World:
    def __init__(self, name: str = "world"):
        self.name = name
        self.skeletons: List[dyn.Skeleton] = []
        self.gravity = np.array([0.0, 0.0, -9.81])
        self.dt = 0.001
        self.penetration_correction = False
        self.parallel_pos_vel = True
        self.fallback_cfm = 1e-4
        self.clipping_depth = 0.03
        self.action_space: Optional[List[int]] = None
        self._forces: Optional[np.ndarray] = None
        self._version = 0
        self._mass_tuned = []  # (body node, entry type, upper bounds, lower bounds) per tuneMass entry
        self._native_by_dev = {}  # device index -> (version, DeviceWorld)

    # --- model ------------------------------------------------------------------
    def addSkeleton(self, skel: dyn.Skeleton):
        skel.world = self
        self.skeletons.append(skel)
        self._touch()
        return skel

    def loadSkeleton(self, path: str, ignore_mesh_collisions: bool = False):
        skel = _urdf.load_urdf(path, ignore_mesh_collisions=ignore_mesh_collisions)
        return self.addSkeleton(skel)

    @staticmethod
    def loadFrom(path: str) -> "World":
        """World::loadFrom (python binding of dart/utils/UniversalLoader):
        .skel files through SkelParser::readWorld (nimblephysics_amd/skel.py)."""
        if path.endswith(".skel"):
            from . import skel as _skel
            return _skel.read_world(path)
        w = World()
        w.loadSkeleton(path)
        return w

    def getSkeleton(self, key):
        if isinstance(key, int):
            return self.skeletons[key]
        for s in self.skeletons:
            if s.name == key:
                return s
        raise KeyError(key)

    def getNumSkeletons(self):
        return len(self.skeletons)

    def getNumDofs(self) -> int:
        return sum(s.getNumDofs() for s in self.skeletons)

    def _touch(self):
        self._version += 1
        n = self.getNumDofs()
        if self._forces is None or len(self._forces) != n:
            self._forces = np.zeros(n)
        if self.action_space is not None and any(a >= n for a in self.action_space):
            self.action_space = None

    # --- parameters -----------------------------------------------------------------
    def setGravity(self, g):
        self.gravity = np.asarray(g, dtype=np.float64).copy()
        self._version += 1

    def getGravity(self):
        return self.gravity.copy()

    def setTimeStep(self, dt):
        self.dt = float(dt)
        self._version += 1

    def getTimeStep(self):
        return self.dt

    def setPenetrationCorrectionEnabled(self, enable: bool):
        self.penetration_correction = bool(enable)
        self._version += 1

    def getPenetrationCorrectionEnabled(self):
        return self.penetration_correction

    def setParallelVelocityAndPositionUpdates(self, enable: bool):
        self.parallel_pos_vel = bool(enable)
        self._version += 1

    def setFallbackConstraintForceMixingConstant(self, c):
        self.fallback_cfm = float(c)
        self._version += 1

    def setContactClippingDepth(self, d):
        self.clipping_depth = float(d)
        self._version += 1

    # --- state (World.cpp:2024 setState / :2040 getState) --------------------------
    def getPositions(self):
        return np.concatenate([s.getPositions() for s in self.skeletons]) if self.skeletons else np.zeros(0)

    def getVelocities(self):
        return np.concatenate([s.getVelocities() for s in self.skeletons]) if self.skeletons else np.zeros(0)

    def setPositions(self, q):
        q = np.asarray(q, dtype=np.float64)
        c = 0
        for s in self.skeletons:
            n = s.getNumDofs()
            s.setPositions(q[c:c + n])
            c += n

    def setVelocities(self, v):
        v = np.asarray(v, dtype=np.float64)
        c = 0
        for s in self.skeletons:
            n = s.getNumDofs()
            s.setVelocities(v[c:c + n])
            c += n

    def getState(self):
        return np.concatenate([self.getPositions(), self.getVelocities()])

    def setState(self, state):
        n = self.getNumDofs()
        state = np.asarray(state, dtype=np.float64)
        if state.size != 2 * n:
            raise ValueError(f"World::setState() expects {2 * n} values, got {state.size}")
        self.setPositions(state[:n])
        self.setVelocities(state[n:])

    def getStateSize(self):
        return 2 * self.getNumDofs()

    def setControlForces(self, f):
        self._forces = np.asarray(f, dtype=np.float64).copy()

    def getControlForces(self):
        return self._forces.copy()

    # --- action space (World.cpp:2061-2130) ------------------------------------------
    def getActionSpace(self) -> List[int]:
        if self.action_space is None:
            return list(range(self.getNumDofs()))
        return list(self.action_space)

    def setActionSpace(self, mapping):
        n = self.getNumDofs()
        mapping = [int(m) for m in mapping]
        for m in mapping:
            if m < 0 or m >= n:
                raise ValueError(f"action mapping index {m} out of bounds [0,{n})")
        self.action_space = mapping

    def removeDofFromActionSpace(self, dof: int):
        self.setActionSpace([a for a in self.getActionSpace() if a != dof])

    def getActionSize(self):
        return len(self.getActionSpace())

    def setAction(self, action):
        action = np.asarray(action, dtype=np.float64)
        f = np.zeros(self.getNumDofs())
        for i, m in enumerate(self.getActionSpace()):
            f[m] = action[i]
        self.setControlForces(f)

    def getAction(self):
        f = self.getControlForces()
        return np.array([f[m] for m in self.getActionSpace()])

    # --- tunable inertia (World::tuneMass / getMassDims / getMasses / setMasses,
    # dart/simulation/World.cpp:1013-1060, :1821; WithRespectToMass,
    # dart/neural/WithRespectToMass.cpp:35-181).  Every WrtMassBodyNodeEntryType
    # is tunable: INERTIA_MASS (1), INERTIA_COM (3, local COM), INERTIA_COM_MU
    # (1, the COM along the body's beta direction), INERTIA_DIAGONAL (3, Ixx
    # Iyy Izz), INERTIA_OFF_DIAGONAL (3, Ixy Ixz Iyz), INERTIA_FULL (10).  The
    # mass vector holds the entries in registration order; setMasses writes
    # them into the bodies (the device model is rebuilt on the next step);
    # lossWrtMass comes from nimble_backward_masses (masses only) or
    # nimble_backward_inertia (all ten parameters per body) through
    # _mass_selection().
    MASS_ENTRY_DIMS = {"INERTIA_MASS": 1, "INERTIA_COM": 3, "INERTIA_COM_MU": 1, "INERTIA_DIAGONAL": 3,
                       "INERTIA_OFF_DIAGONAL": 3, "INERTIA_FULL": 10}

    def tuneMass(self, node, type="INERTIA_MASS", upperBound=None, lowerBound=None):
        kind = getattr(type, "name", type)
        if kind not in self.MASS_ENTRY_DIMS:
            raise ValueError(f"tuneMass: unknown WrtMassBodyNodeEntryType {kind}")
        if not any(node is b for s in self.skeletons for b in s.bodies):
            raise ValueError("tuneMass: the body node is not in this world")
        if any(node is e[0] and kind == e[1] for e in self._mass_tuned):
            raise ValueError("tuneMass: entry already registered")
        dims = self.MASS_ENTRY_DIMS[kind]
        up = np.broadcast_to(np.asarray(upperBound if upperBound is not None else np.inf, dtype=np.float64).reshape(-1),
                             (dims,)).copy()
        lo = np.broadcast_to(np.asarray(lowerBound if lowerBound is not None else
                                        (0.0 if kind == "INERTIA_MASS" else -np.inf), dtype=np.float64).reshape(-1),
                             (dims,)).copy()
        self._mass_tuned.append((node, kind, up, lo))

    def getMassDims(self) -> int:
        return sum(self.MASS_ENTRY_DIMS[k] for _, k, _, _ in self._mass_tuned)

    @staticmethod
    def _entry_get(b, kind):
        """WrtMassBodyNodyEntry::get (WithRespectToMass.cpp:136)."""
        I = b.moment  # Ixx Iyy Izz Ixy Ixz Iyz
        if kind == "INERTIA_MASS":
            return np.array([b.mass])
        if kind == "INERTIA_COM":
            return np.array(b.com, dtype=np.float64)
        if kind == "INERTIA_COM_MU":
            beta = b.getBeta()
            k = 0 if beta[0] != 0 else (1 if beta[1] != 0 else 2)
            return np.array([b.com[k] / beta[k]])
        if kind == "INERTIA_DIAGONAL":
            return np.array(I[:3], dtype=np.float64)
        if kind == "INERTIA_OFF_DIAGONAL":
            return np.array(I[3:], dtype=np.float64)
        return np.concatenate([[b.mass], b.com, I])

    def getMasses(self):
        if not self._mass_tuned:
            return np.zeros(0)
        return np.concatenate([self._entry_get(b, k) for b, k, _, _ in self._mass_tuned]).astype(np.float64)

    def getMassUpperBound(self):
        return np.concatenate([u for _, _, u, _ in self._mass_tuned]) if self._mass_tuned else np.zeros(0)

    def getMassLowerBound(self):
        return np.concatenate([l for _, _, _, l in self._mass_tuned]) if self._mass_tuned else np.zeros(0)

    def setMasses(self, masses):
        """WrtMassBodyNodyEntry::set (WithRespectToMass.cpp:45) per entry; an
        unchanged value keeps the device model."""
        masses = np.asarray(masses, dtype=np.float64).reshape(-1)
        if masses.shape[0] != self.getMassDims():
            raise ValueError(f"setMasses: {masses.shape[0]} values, the world has {self.getMassDims()} mass dims")
        o = 0
        for b, kind, _, _ in self._mass_tuned:
            d = self.MASS_ENTRY_DIMS[kind]
            v = masses[o:o + d]
            o += d
            if np.array_equal(v, self._entry_get(b, kind)):
                continue
            if kind == "INERTIA_MASS":
                b.setMass(float(v[0]))
            elif kind == "INERTIA_COM":
                b.setLocalCOM(v)
            elif kind == "INERTIA_COM_MU":
                b.setLocalCOM(b.getBeta() * float(v[0]))
            elif kind == "INERTIA_DIAGONAL":
                b.setMomentOfInertia(v[0], v[1], v[2], *b.moment[3:])
            elif kind == "INERTIA_OFF_DIAGONAL":
                b.setMomentOfInertia(*b.moment[:3], v[0], v[1], v[2])
            else:
                b.setMass(float(v[0]))
                b.setLocalCOM(v[1:4])
                b.setMomentOfInertia(*v[4:10])

    def _mass_selection(self):
        """(masses_only, index / matrix): with only INERTIA_MASS entries, the
        global body index of each (columns of nimble_backward_masses' [B,
        num_bodies]); otherwise a [num_bodies * 10, getMassDims()] matrix
        taking nimble_backward_inertia's INERTIA_FULL-ordered parameters to
        the mass vector (COM_MU: the beta-weighted COM components)."""
        order = [e[2] for e in self._model_bodies()]
        idx = [next(i for i, o in enumerate(order) if o is b) for b, _, _, _ in self._mass_tuned]
        if all(k == "INERTIA_MASS" for _, k, _, _ in self._mass_tuned):
            return True, idx
        S = np.zeros((len(order) * 10, self.getMassDims()))
        col = 0
        for (b, kind, _, _), bi in zip(self._mass_tuned, idx):
            base = 10 * bi
            comps = {"INERTIA_MASS": [0], "INERTIA_COM": [1, 2, 3], "INERTIA_DIAGONAL": [4, 5, 6],
                     "INERTIA_OFF_DIAGONAL": [7, 8, 9], "INERTIA_FULL": list(range(10))}.get(kind)
            if comps is not None:
                for c in comps:
                    S[base + c, col] = 1.0
                    col += 1
            else:  # INERTIA_COM_MU: d com / d mu = beta
                S[base + 1:base + 4, col] = b.getBeta()
                col += 1
        return False, S

    def _model_bodies(self):
        """The device model's bodies in order: (skeleton index, skeleton,
        BodyNode or None, owning BodyNode, chain element): every BodyNode, a
        UniversalJoint / EulerJoint / PlanarJoint child preceded by the
        massless frames of its 1-dof chain (dynamics.Joint.chain; None in the
        third field), the chain's last element on the BodyNode itself."""
        out = []
        for si, s in enumerate(self.skeletons):
            for b in s.bodies:
                ch = b.joint.chain()
                for k, e in enumerate(ch):
                    out.append((si, s, b if k == len(ch) - 1 else None, b, e))
        return out

    def _mass_body_indices(self):
        """Global body index (device model order) of each tuned mass entry."""
        order = [e[2] for e in self._model_bodies()]
        return [next(i for i, o in enumerate(order) if o is b) for b, _, _, _ in self._mass_tuned]

    # --- flattening -----------------------------------------------------------------------
    def desc_arrays(self) -> Dict[str, np.ndarray]:
        model = self._model_bodies()
        nb = len(model)
        n = self.getNumDofs()
        if nb > NIMBLE_MAX_BODIES or n > NIMBLE_MAX_DOFS:
            raise ValueError(f"model too large: {nb} bodies / {n} dofs (max {NIMBLE_MAX_BODIES}/{NIMBLE_MAX_DOFS})")
        index = {}
        for k, (si, s, b, owner, _) in enumerate(model):
            if b is not None:
                index[id(b)] = k
        dof_base = {}
        c = 0
        for s in self.skeletons:
            dof_base[id(s)] = c
            c += s.getNumDofs()

        def t12(T):
            return np.asarray(T, dtype=np.float64)[:3, :4].reshape(12)

        A: Dict[str, list] = {k: [] for k in (
            "parent", "skeleton", "joint_type", "dof_offset", "skeleton_mobile", "T_parent_joint",
            "T_child_joint", "axis", "mass", "com", "moment", "friction", "restitution")}
        prev = None
        for k, (si, s, b, owner, (kind, axis, Tp, Tc)) in enumerate(model):
            j = owner.joint
            first = prev is None or prev[3] is not owner
            pos = 0 if first else pos + 1
            # (a chain's first element hangs from the owner's parent, the
            # others from the previous element's massless frame)
            A["parent"].append((index[id(owner.parent)] if owner.parent is not None else -1) if first else k - 1)
            A["skeleton"].append(si)
            A["joint_type"].append(kind)
            A["dof_offset"].append(dof_base[id(s)] + j.dof_offset + pos)
            A["skeleton_mobile"].append(1 if s.mobile else 0)
            A["T_parent_joint"].append(t12(Tp))
            A["T_child_joint"].append(t12(Tc))
            A["axis"].append(axis)
            A["mass"].append(b.mass if b is not None else 0.0)
            A["com"].append(b.com if b is not None else np.zeros(3))
            A["moment"].append(b.moment if b is not None else np.zeros(6))
            A["friction"].append(owner.friction)
            A["restitution"].append(owner.restitution)
            prev = (si, s, b, owner)
        per_dof = {k: [] for k in ("damping", "spring", "rest_position", "pos_lower", "pos_upper", "vel_lower",
                                    "vel_upper", "force_lower", "force_upper")}
        attr = {"damping": "damping", "spring": "spring", "rest_position": "rest", "pos_lower": "pos_lo",
                "pos_upper": "pos_hi", "vel_lower": "vel_lo", "vel_upper": "vel_hi", "force_lower": "force_lo",
                "force_upper": "force_hi"}
        for s in self.skeletons:
            for b in s.bodies:
                for k, a in attr.items():
                    per_dof[k].extend(list(getattr(b.joint, a)))
        shapes = []
        for si, s, b, _, _ in model:
            if b is None:
                continue
            for node in b.shape_nodes:
                if node.collision:
                    shapes.append((index[id(b)], node))
        if len(shapes) > NIMBLE_MAX_SHAPES:
            raise ValueError("too many collision shapes")
        out = {
            "num_bodies": nb, "num_dofs": n, "num_shapes": len(shapes), "dt": self.dt,
            "gravity": self.gravity, "contact_clipping_depth": self.clipping_depth,
            "fallback_cfm": self.fallback_cfm, "penetration_correction": int(self.penetration_correction),
            "parallel_pos_vel": int(self.parallel_pos_vel),
            "parent": np.array(A["parent"], np.int32), "skeleton": np.array(A["skeleton"], np.int32),
            "joint_type": np.array(A["joint_type"], np.int32), "dof_offset": np.array(A["dof_offset"], np.int32),
            "skeleton_mobile": np.array(A["skeleton_mobile"], np.int32),
            "T_parent_joint": np.array(A["T_parent_joint"]).reshape(-1),
            "T_child_joint": np.array(A["T_child_joint"]).reshape(-1),
            "axis": np.array(A["axis"]).reshape(-1), "mass": np.array(A["mass"]),
            "com": np.array(A["com"]).reshape(-1), "moment": np.array(A["moment"]).reshape(-1),
            "friction": np.array(A["friction"]), "restitution": np.array(A["restitution"]),
            "shape_body": np.array([s[0] for s in shapes], np.int32),
            "shape_type": np.array([s[1].shape.kind for s in shapes], np.int32),
            "shape_size": np.array([s[1].shape.size for s in shapes]).reshape(-1),
            "shape_T": np.array([t12(s[1].T) for s in shapes]).reshape(-1),
        }
        # mesh colliders: vertex lists concatenated in shape order
        first, count, verts, cand = [], [], [], []
        nv = 0
        for _, node in shapes:
            sh = node.shape
            if sh.kind == dyn.SHAPE_MESH:
                first.append(nv)
                count.append(sh.vertices.shape[0])
                verts.append(sh.vertices)
                cand.append(sh.candidate())
                nv += sh.vertices.shape[0]
            else:
                first.append(0)
                count.append(0)
        out["shape_mesh_first"] = np.array(first, np.int32)
        out["shape_mesh_count"] = np.array(count, np.int32)
        out["mesh_vertices"] = np.concatenate(verts).reshape(-1) if verts else np.zeros(0)
        out["mesh_vertex_candidate"] = np.concatenate(cand).astype(np.int32) if cand else np.zeros(0, np.int32)
        for k, v in per_dof.items():
            out[k] = np.array(v, dtype=np.float64)
        return out

    def desc(self):
        return build_desc(self.desc_arrays())

    def native(self, device=None):
        """Device-side world handle for `device` (a torch device or index;
        default: the current HIP device), created lazily and rebuilt whenever
        the model changed (World setters, and every dynamics setter through
        ``dynamics._model_changed``).  One handle per device: the model lives
        in that device's HBM and its kernels launch there."""
        from . import _native
        import torch
        if device is None:
            idx = torch.cuda.current_device()
        else:
            idx = device.index if isinstance(device, torch.device) else int(device)
            if idx is None:
                idx = torch.cuda.current_device()
        handles = self.__dict__.setdefault("_native_by_dev", {})
        cur = handles.get(idx)
        if cur is None or cur[0] != self._version:
            # a superseded handle is not closed here: autograd graphs and
            # BackpropSnapshots of earlier steps may still hold it, and
            # DeviceWorld.__del__ releases it once nothing does
            with torch.cuda.device(idx):
                handles[idx] = (self._version, _native.DeviceWorld(self, idx))
        return handles[idx][1]

    # --- step Jacobians at the current state (World.cpp:2190-2245) -------------
    def getCachedBackpropSnapshot(self):
        """neural.forwardPass(self, idempotent=True), re-run only when the
        positions, velocities or control forces changed (World.cpp:2190)."""
        from . import neural
        key = (self.getPositions().tobytes(), self.getVelocities().tobytes(), self.getControlForces().tobytes(),
               self._version)
        cached = getattr(self, "_cached_snapshot_key", None)
        if cached is None or cached[0] != key:
            self._cached_snapshot_key = (key, neural.forwardPass(self, idempotent=True))
        return self._cached_snapshot_key[1]

    def getStateJacobian(self):
        """d(next state)/d(state) [2n, 2n] at the current state (World.cpp:2210)."""
        return self.getCachedBackpropSnapshot().getStateJacobian(self)

    def getActionJacobian(self):
        """d(next state)/d(action) [2n, |A|] at the current state (World.cpp:2227)."""
        return self.getCachedBackpropSnapshot().getActionJacobian(self)

    # --- LCP warm start (BoxedLcpConstraintSolver::mX) ------------------------
    def setCachedLCPSolution(self, x):
        """World::setCachedLCPSolution (World.cpp): the warm start of the next
        step's LCP, used only when its size equals that LCP's row count (else
        ignored, as BoxedLcpConstraintSolver does).  `x` is one vector (every
        world of the next batch) or a list with one vector (or None: empty)
        per world."""
        per_world = (isinstance(x, (list, tuple)) and len(x) > 0 and (x[0] is None or np.ndim(x[0]) == 1)) \
            or (x is not None and np.ndim(x) == 2)
        if per_world:
            rows = [None if r is None else np.asarray(r, dtype=np.float64) for r in x]
        else:
            rows = [None if x is None else np.asarray(x, dtype=np.float64)]
        for r in rows:
            if r is not None and r.ndim != 1:
                raise ValueError("setCachedLCPSolution: one 1-D vector per world")
        self._pending_lcp_cache = rows

    def getCachedLCPSolution(self, world_index: int = 0):
        """The LCP solution of world `world_index` of the last batched step
        (the next step's warm start; empty when it had no LCP)."""
        # a value set since the last step is the one the next step will use
        # (World::getCachedLCPSolution returns what setCachedLCPSolution set)
        rows = getattr(self, "_pending_lcp_cache", None)
        bs = getattr(self, "_batch_state", None)
        if rows is not None or bs is None:
            rows = rows or [None]
            r = rows[world_index if len(rows) > 1 else 0]
            return np.zeros(0) if r is None else r.copy()
        row = bs.cache[world_index].cpu().numpy()
        m = int(row[0])
        return row[1:1 + m].copy() if m > 0 else np.zeros(0)

    # --- per-world status of the last batched step (see timestep.py) ----------
    def getLastStatus(self):
        """Status bits of each world of the last ``timestep`` call (a device
        int32 tensor [B], 0 = the step is the reference's): 1 contact
        overflow, 2 unsupported shape pair, 4 dropped-contact list overflow
        (these three mean the physics differs from the reference's), 8 the
        LCP was reduced (LCPUtils::reduce merged duplicate columns; the
        reference's own behaviour, informational)."""
        return getattr(self, "_last_status", None)

    def setStatusPolicy(self, policy: str):
        """'raise' (default): ``timestep`` raises ContactCapacityError when a
        world's step cannot match the reference (status bits 1, 2, 4);
        'record': only record them in getLastStatus() (no host sync)."""
        if policy not in ("raise", "record"):
            raise ValueError(policy)
        self._status_policy = policy

    def getStatusPolicy(self) -> str:
        return getattr(self, "_status_policy", "raise")
