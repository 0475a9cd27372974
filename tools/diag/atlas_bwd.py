"""Worst gradient elements of the box Atlas bench batch vs the oracle
(diagnostic for the per-element tolerance)."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from nimblephysics_amd import workloads
from oracle import oracle as O
from test_gpu_contact_parity import SN_M, SN_NCON, _device_backward, _device_step

world = workloads.atlas_world(True)
st, f = workloads.random_states(world, 1024, seed=1000, q_scale=0.02, v_scale=0.05, f_scale=1.0)
ow = O.OracleWorld(world)
ref = ow.forward(st, f)
nxt, tsnap, cache, ts, tf = _device_step(world, st, f)
g = np.random.default_rng(11).standard_normal(st.shape)
ggs, ggf = _device_backward(world, ts, tf, tsnap, g)
rgs, rgf = ow.backward(g)
snap = tsnap.cpu().numpy()
n = world.getNumDofs()
for name, a, b in (("gs_q", ggs[:, :n], rgs[:, :n]), ("gs_v", ggs[:, n:], rgs[:, n:]), ("gf", ggf, rgf)):
    scale = np.maximum(np.abs(b), 1e-5 * np.abs(b).max())
    r = np.abs(a - b) / scale
    idx = np.argsort(r.ravel())[::-1][:6]
    for k in idx:
        w, j = divmod(int(k), b.shape[1])
        print(name, "world", w, "elem", j, "rel %.3e" % r.ravel()[k], "got %.12e ref %.12e" % (a[w, j], b[w, j]),
              "world max %.3e batch max %.3e" % (np.abs(b[w]).max(), np.abs(b).max()),
              "nc", int(snap[w, SN_NCON]), "m", int(snap[w, SN_M]),
              "world normwise %.3e" % (np.abs(a[w] - b[w]).max() / np.abs(b[w]).max()))
