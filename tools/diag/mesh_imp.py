"""Mesh Atlas: for every solved world, the device's rank-deficiency flag
(SN_IMP), the clamping matrix Q's singular values and the pivoted-QR
diagonal ratios near the COD rank threshold.  Diagnostic."""
import sys
import numpy as np
import scipy.linalg as sl
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from nimblephysics_amd import _native, workloads
from oracle import oracle as O
from test_gpu_contact_parity import SN_M, SN_NC, SN_STATUS, _device_backward, _device_step, _same_path

MAXL = _native.MAX_LCP
B = 256
world = workloads.atlas_mesh_world(True)
world.setStatusPolicy("record")
n = world.getNumDofs()
st, f = workloads.random_states(world, B, seed=1000, q_scale=0.02, v_scale=0.05)
ow = O.OracleWorld(world)
ow.forward(st, f)
nxt, tsnap, cache, ts, tf = _device_step(world, st, f)
g = np.random.default_rng(1000).standard_normal(st.shape)
ggs, ggf = _device_backward(world, ts, tf, tsnap, g)
rgs, rgf = ow.backward(g)
snap = tsnap.cpu().numpy()
LAY = _native.snapshot_layout(n)
snPT, snQ = LAY["pt"], LAY["q"]
for b in range(B):
    sn = snap[b]
    m = int(sn[SN_M])
    if int(sn[SN_STATUS]) & _native.ST_LCP_TOO_LARGE or m == 0 or not _same_path(ow, sn, b):
        continue
    nc = int(sn[SN_NC])
    e = np.abs(ggs[b] - rgs[b]).max() / np.abs(rgs[b]).max()
    if nc == 0:
        continue
    Q = sn[snQ:snQ + nc * nc].reshape(nc, nc)
    PT = sn[snPT:snPT + nc * nc].reshape(nc, nc)
    impd = np.sum((np.eye(nc) - Q @ PT.T) ** 2)
    s = np.linalg.svd(Q, compute_uv=False)
    R = sl.qr(Q, pivoting=True, mode="r")[0]
    d = np.abs(np.diag(R))
    print("world %3d m %2d nc %2d err %.2e SN_IMP %d impNorm(dev) %.2e  smin/smax %.2e  |R| ratios %s"
          % (b, m, nc, e, int(sn[8]), impd, s[-1] / s[0], " ".join("%.1e" % (x / d[0]) for x in d[-3:])))
