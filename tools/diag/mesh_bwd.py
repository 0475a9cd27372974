"""Per-world gradient error of the mesh Atlas vs the oracle, with contact
count, LCP rows and contact types of the worst worlds (diagnostic)."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from nimblephysics_amd import _native, workloads
from oracle import oracle as O
from test_gpu_contact_parity import CREC, SN_CONTACTS, SN_M, SN_NCON, SN_STATUS, _device_backward, _device_step, _same_path

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
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
rows = []
for b in range(B):
    sn = snap[b]
    nc = int(sn[SN_NCON]); m = int(sn[SN_M]); status = int(sn[SN_STATUS])
    if status & _native.ST_LCP_TOO_LARGE:
        continue
    same = m == 0 or _same_path(ow, sn, b)
    e = np.abs(ggs[b] - rgs[b]).max() / max(np.abs(rgs[b]).max(), 1e-300)
    ef = np.abs(ggf[b] - rgf[b]).max() / max(np.abs(rgf[b]).max(), 1e-300)
    types = np.bincount(sn[SN_CONTACTS:SN_CONTACTS + CREC * nc].reshape(nc, CREC)[:, 7].astype(int) & 15, minlength=4) if nc else []
    rows.append((e, ef, b, nc, m, same, list(types)))
rows.sort(reverse=True)
for r in rows[:25]:
    print("err_s %.3e err_f %.3e world %d nc %d m %d same %s types %s" % r)
bad = [r for r in rows if r[0] > 1e-6]
print("bad", len(bad), "of", len(rows), "min m among bad", min([r[4] for r in bad], default=-1),
      "max m among good", max([r[4] for r in rows if r[0] <= 1e-6], default=-1))
