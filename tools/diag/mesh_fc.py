"""Mesh Atlas: for worlds whose state gradient differs from the oracle's,
compare the LCP solutions / clamping impulses and the clamping block's rank
(is the LCP solution unique?).  Diagnostic."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from nimblephysics_amd import _native, workloads
from oracle import oracle as O
from test_gpu_contact_parity import SN_M, SN_NC, SN_STATUS, _device_backward, _device_step, _same_path

FC = _native.SNAPSHOT_FC if hasattr(_native, "SNAPSHOT_FC") else 16 + 13 * _native.MAX_CONTACTS + 12 * _native.MAX_LCP
B = 256
world = workloads.atlas_mesh_world(True)
world.setStatusPolicy("record")
st, f = workloads.random_states(world, B, seed=1000, q_scale=0.02, v_scale=0.05)
ow = O.OracleWorld(world)
ref = ow.forward(st, f)
nxt, tsnap, cache, ts, tf = _device_step(world, st, f)
g = np.random.default_rng(1000).standard_normal(st.shape)
ggs, ggf = _device_backward(world, ts, tf, tsnap, g)
rgs, rgf = ow.backward(g)
snap = tsnap.cpu().numpy()
cache = cache.cpu().numpy()
n = world.getNumDofs()
for b in range(B):
    sn = snap[b]
    m = int(sn[SN_M])
    if int(sn[SN_STATUS]) & _native.ST_LCP_TOO_LARGE or m == 0 or not _same_path(ow, sn, b):
        continue
    e = np.abs(ggs[b] - rgs[b]).max() / np.abs(rgs[b]).max()
    mapping, xr = O.lcp_debug(ow, b)
    xd = cache[b, 1:1 + m]
    fcr = O.lcp_fc(ow, b)
    ncl = int(sn[SN_NC])
    fcd = sn[FC:FC + ncl]
    A, bb, lo, hi, fi = O.lcp_problem(ow, b)
    cl = np.where(mapping >= 0)[0] if (mapping >= 0).any() else np.arange(0)
    J = O.lcp_cols(ow, b)
    rank = np.linalg.matrix_rank(J[:, :m]) if m else 0
    print("world %3d m %2d rank(J) %2d clamping %2d  grad_s err %.2e  |dx| %.2e (|x| %.2e)  |dfc| %.2e  |J(xd-xr)| %.2e"
          % (b, m, rank, ncl, e, np.abs(xd - xr).max(initial=0), np.abs(xr).max(initial=0),
             np.abs(fcd - fcr).max(initial=0) if len(fcd) == len(fcr) else -1, np.abs(J[:, :m] @ (xd - xr)).max(initial=0)))
