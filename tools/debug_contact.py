"""Debug helper: compare the GPU snapshot of one world with the oracle's LCP
path (run on a GPU box)."""
import sys

import numpy as np
import torch

sys.path[:0] = ["tests", "."]
import models  # noqa: E402
from oracle import oracle as O  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "rest"
envs = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
w = models.box_world()
st, f = models.box_states(kind, 64, seed=5)
ow = O.OracleWorld(w)
ref = ow.forward(st, f)
dev = w.native()
d = torch.device("cuda:0")
ts, tf = torch.tensor(st, device=d), torch.tensor(f, device=d)
cache = torch.zeros((64, dev.cache_doubles), dtype=torch.float64, device=d)
cache[:, 0] = -1
nxt = torch.empty_like(ts)
snap = torch.zeros((64, dev.snapshot_doubles), dtype=torch.float64, device=d)
dev.forward(ts, tf, cache, nxt, snap, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
sn = snap.cpu().numpy()
np.set_printoptions(precision=10, linewidth=220)
for b in envs:
    m = int(sn[b, 1])
    rows = sn[b, 176:176 + 12 * m].reshape(m, 12)
    print("env", b, "GPU  sc/ign/cfm/nc/nu", sn[b, 6], sn[b, 7], sn[b, 4], sn[b, 2], sn[b, 3], "status", sn[b, 5])
    print("  GPU map", rows[:, 7].astype(int))
    print("  GPU X  ", rows[:, 6])
    print("  GPU b  ", rows[:, 5])
    mp, x = O.lcp_debug(ow, b)
    print("  ORA flags", O.lcp_flags(ow, b))
    print("  ORA map", mp)
    print("  ORA X  ", x)
    print("  next rel err", np.abs(nxt.cpu().numpy()[b] - ref[b]).max() / np.abs(ref[b]).max())
