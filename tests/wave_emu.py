"""Drive the host emulation of the product kernels (tests/cpp/wave_emu:
timestep.hip + capi.cpp compiled for the CPU against an emulated wavefront,
with AddressSanitizer).  Test infrastructure: build() compiles the driver,
step() runs one forward + backward of a world through the emulated C-ABI."""
from __future__ import annotations

import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "wave_emu")
CLANG = "/opt/rocm/llvm/bin/clang++"


def build(name="step_emu", out=None):
    """Compile tests/cpp/wave_emu/<name>.cpp with ASan; returns the binary."""
    out = out or os.path.join("/tmp", f"nimble_{name}_{os.getuid()}")
    src = os.path.join(SRC, f"{name}.cpp")
    deps = [src, os.path.join(SRC, "hip", "hip_runtime.h")]
    csrc = os.path.join(ROOT, "nimblephysics_amd", "csrc")
    deps += [os.path.join(csrc, f) for f in os.listdir(csrc)]
    inc = os.path.join(ROOT, "include")
    deps += [os.path.join(inc, f) for f in os.listdir(inc)]
    if os.path.exists(out) and os.path.getmtime(out) > max(os.path.getmtime(d) for d in deps):
        return out
    subprocess.check_call([CLANG, "-std=c++20", "-O0", "-g", "-mavx512f", "-fsanitize=address",
                           "-fno-omit-frame-pointer", *os.environ.get("WAVE_EMU_FLAGS", "").split(), "-I", SRC, "-Wno-everything", "-x", "c++", "-o", out, src,
                           "-lpthread"])
    return out


def _fmt(v, ints=False):
    v = np.asarray(v).ravel()
    if ints:
        return " ".join(str(int(x)) for x in v)
    return " ".join("inf" if x == np.inf else "-inf" if x == -np.inf else repr(float(x)) for x in v)


def step(world, st, f, g, env=None, timeout=1800):
    """(next_state, grad_state, grad_forces, snapshot headers [B, 16])."""
    exe = build()
    d = world.desc_arrays()
    cand = np.asarray(d.get("mesh_vertex_candidate", []))
    nmv = len(np.asarray(d["mesh_vertices"])) // 3
    lines = [_fmt([d["num_bodies"], d["num_dofs"], d["num_shapes"], nmv, d["penetration_correction"],
                   d["parallel_pos_vel"], 1 if len(cand) else 0], True),
             _fmt([d["dt"], *d["gravity"], d["contact_clipping_depth"], d["fallback_cfm"]])]
    for k in ("parent", "skeleton", "joint_type", "dof_offset", "skeleton_mobile"):
        lines.append(_fmt(d[k], True))
    for k in ("T_parent_joint", "T_child_joint", "axis", "mass", "com", "moment", "friction", "restitution",
              "damping", "spring", "rest_position", "pos_lower", "pos_upper", "vel_lower", "vel_upper",
              "force_lower", "force_upper"):
        lines.append(_fmt(d[k]))
    lines += [_fmt(d["shape_body"], True), _fmt(d["shape_type"], True), _fmt(d["shape_size"]), _fmt(d["shape_T"]),
              _fmt(d["shape_mesh_first"], True), _fmt(d["shape_mesh_count"], True), _fmt(d["mesh_vertices"])]
    if len(cand):
        lines.append(_fmt(cand, True))
    lines += [str(st.shape[0]), _fmt(st), _fmt(f), _fmt(g)]
    e = dict(os.environ)
    e.update(env or {})
    e["ASAN_OPTIONS"] = "detect_leaks=0"
    if os.environ.get("WAVE_EMU_DUMP"):
        with open(os.environ["WAVE_EMU_DUMP"], "w") as fh:
            fh.write("\n".join(lines))
    r = subprocess.run([exe], input="\n".join(lines), capture_output=True, text=True, timeout=timeout, env=e)
    with open(os.path.join("/tmp", f"nimble_wave_emu_{os.getuid()}.stderr"), "w") as fh:
        fh.write(r.stderr)
    if r.returncode != 0:
        raise RuntimeError(f"emulated step failed ({r.returncode}):\n{r.stderr[-6000:]}")
    out = {}
    for ln in r.stdout.splitlines():
        t = ln.split()
        out[t[0]] = np.array([float(x) for x in t[1:]])
    B, n = st.shape[0], world.getNumDofs()
    return (out["next"].reshape(B, 2 * n), out["gs"].reshape(B, 2 * n), out["gf"].reshape(B, n),
            out["head"].reshape(B, 16))


def lds_bytes(world):
    """(forward, backward) LDS bytes per workgroup the C-ABI sizes for
    `world` (NIMBLE_AMD_VERBOSE report of nimble_world_create, through the
    emulated step of one world at rest)."""
    import re
    n = world.getNumDofs()
    st = np.zeros((1, 2 * n))
    f = np.zeros((1, n))
    step(world, st, f, np.zeros_like(st), {"NIMBLE_AMD_VERBOSE": "1"})
    txt = open(os.path.join("/tmp", f"nimble_wave_emu_{os.getuid()}.stderr")).read()
    m = re.search(r"LDS forward (\d+) B .* backward (\d+) B", txt)
    return int(m.group(1)), int(m.group(2))
