"""Per-stage shader-clock breakdown of the backward kernel (debug build)."""
import sys

import numpy as np
import torch

sys.path[:0] = ["tests", "."]
import models  # noqa: E402

B = 1024
w = models.atlas_world(True)
st, f = models.random_states(w, B, seed=1000, q_scale=0.02, v_scale=0.05)
d = torch.device("cuda:0")
state, action = torch.tensor(st, device=d), torch.tensor(f, device=d)
dev = w.native()
cache = torch.zeros((B, dev.cache_doubles), dtype=torch.float64, device=d)
cache[:, 0] = -1
snap = torch.zeros((B, dev.snapshot_doubles), dtype=torch.float64, device=d)
nxt = torch.empty_like(state)
s = torch.cuda.current_stream().cuda_stream
n = w.getNumDofs()
from nimblephysics_amd import _native  # noqa: E402
ws = _native.snapshot_layout(n, timing=True)["stamps"]  # csrc/pool_sizes.h snStamps(n)
g = torch.tensor(np.random.default_rng(0).standard_normal(st.shape), device=d)
gs, gf = torch.empty_like(state), torch.empty_like(action)
dev.forward(state, action, cache, nxt, snap, s)
snap[:, ws + 20:ws + 40] = 0
snap[:, ws + 80:ws + 90] = 0
dev.backward(state, action, snap, g, gs, gf, s)
torch.cuda.synchronize()
T = snap[:, ws:ws + 90].cpu().numpy()
hd = snap[:, :8].cpu().numpy()
names = [((20, 21), "load+coreDynamics"), ((21, 22), "contact prep / plain solves"), ((30, 31), " prep: Ac/AcubE"),
         ((31, 32), " prep: MA + yf,w solves"), ((32, 33), " prep: Q, delta, u"), ((33, 34), " prep: COD factor"),
         ((34, 35), " prep: pinv columns"), ((35, 36), " prep: vectors, imp"), ((36, 37), " prep: 4 chol solves"),
         ((37, 38), " prep: gRows, TAB"), ((22, 23), "kinematics(a*) + deriv composites"),
         ((23, 24), "per-direction ID columns"), ((24, 25), "M-fields + G terms"), ((25, 26), "FD free + write")]
print("clamping worlds", int((hd[:, 2] > 0).sum()))
for (a, b), nm in names:
    # (worlds whose LCP uses the HBM workspace overwrite the stamp slots)
    m = (T[:, a] > 0) & (T[:, b] > 0) & (T[:, b] - T[:, a] > 0) & (T[:, b] - T[:, a] < 1e8)
    if m.any():
        dtk = T[m, b] - T[m, a]
        print(f"  {nm:36s} worlds {m.sum():5d}  mean {dtk.mean():10.0f}  max {dtk.max():10.0f}")
for k, nm in [(80, "G terms total"), (81, "M fields"), (82, " G: omega/vertex sums"), (83, " G: P chain + contraction"),
              (84, " G: face side"), (85, " G: contact bodies (count)")]:
    v = T[:, k]
    print(f"  {nm:36s} worlds {(v > 0).sum():5d}  mean {v[v > 0].mean() if (v > 0).any() else 0:10.0f}  max {v.max():10.0f}")
