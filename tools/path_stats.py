"""Per-regime LCP path agreement between the GPU and the oracle (GPU box)."""
import sys

import numpy as np
import torch

sys.path[:0] = ["tests", "."]
import models  # noqa: E402
from oracle import oracle as O  # noqa: E402


def run(world, st, f):
    ow = O.OracleWorld(world)
    ref = ow.forward(st, f)
    dev = world.native()
    d = torch.device("cuda:0")
    B = st.shape[0]
    ts, tf = torch.tensor(st, device=d), torch.tensor(f, device=d)
    cache = torch.zeros((B, dev.cache_doubles), dtype=torch.float64, device=d)
    cache[:, 0] = -1
    nxt = torch.empty_like(ts)
    snap = torch.zeros((B, dev.snapshot_doubles), dtype=torch.float64, device=d)
    dev.forward(ts, tf, cache, nxt, snap, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    sn = snap.cpu().numpy()
    got = nxt.cpu().numpy()
    same, errs_same, errs_diff, dantzig_o, dantzig_g = 0, [], [], 0, 0
    for b in range(B):
        fl = O.lcp_flags(ow, b)
        m = int(sn[b, 1])
        mp, _ = O.lcp_debug(ow, b)
        gm = sn[b, 176:176 + 12 * m].reshape(m, 12)[:, 7].astype(int) if m else np.zeros(0, int)
        gfl = np.array([sn[b, 6], sn[b, 7], sn[b, 4], sn[b, 2], sn[b, 3]])
        e = np.abs(got[b] - ref[b]).max() / np.abs(ref[b]).max()
        if m and fl[0] == 0 and fl[2] == 0:
            dantzig_o += 1
        if m and gfl[0] == 0 and gfl[2] == 0:
            dantzig_g += 1
        if np.array_equal(fl, gfl) and np.array_equal(mp, gm):
            same += 1
            errs_same.append(e)
        else:
            errs_diff.append(e)
    return same, B, max(errs_same, default=0), max(errs_diff, default=0), dantzig_o, dantzig_g


for kind in ["rest", "slide", "tilt", "lift"]:
    w = models.box_world()
    st, f = models.box_states(kind, 256, seed=5)
    print(kind, "same/B %d/%d  maxerr same %.2e diff %.2e  dantzig-ok oracle %d gpu %d" % run(w, st, f))
w = models.atlas_world(True)
for seed in (3, 4):
    st, f = models.random_states(w, 256, seed=seed, q_scale=0.01, v_scale=0.02)
    print("atlas", seed, "same/B %d/%d  maxerr same %.2e diff %.2e  dantzig-ok oracle %d gpu %d" % run(w, st, f))
