"""Mesh Atlas bench rollout (bench.py --workload atlas_mesh, rank 0's
sampler): per step, the worlds with each status bit and the contact / row
counts (the device's own rollout, fresh LCP cache per step).  Diagnostic."""
import sys

import numpy as np

sys.path[:0] = ["tests", "."]
from nimblephysics_amd import _native, workloads  # noqa: E402
from test_gpu_contact_parity import SN_M, SN_NCON, SN_STATUS, _device_step  # noqa: E402

B = 1024
world = workloads.atlas_mesh_world(True)
world.setStatusPolicy("record")
st, f = workloads.atlas_states(world, B, 1000)
for step in range(25):
    nxt, tsnap, cache, ts, tf = _device_step(world, st, f)
    sn = tsnap[:, :16].cpu().numpy()
    stat = sn[:, SN_STATUS].astype(np.int64)
    bits = {b: int(((stat & b) != 0).sum()) for b in (1, 2, 4, 8, 16, 32)}
    ncon = sn[:, SN_NCON]
    m = sn[:, SN_M]
    print(f"step {step}: bits {bits} contacts max {ncon.max():.0f} mean {ncon.mean():.1f} rows max {m.max():.0f} "
          f"worlds>64 rows {(m > 64).sum()}", flush=True)
    bad = np.where((stat & _native.ST_DIVERGES) != 0)[0]
    if len(bad):
        print("   first bad worlds", bad[:8].tolist(), "ncon", ncon[bad[:8]].tolist(), "stat", stat[bad[:8]].tolist())
    st = nxt.cpu().numpy() if hasattr(nxt, "cpu") else nxt
