"""Per-world forward latency of the STL-mesh Atlas by LCP size (debug build
with -DNIMBLE_STAGE_TIMING; GPU box, NIMBLE_AMD_LIB=dbg/libnimble_dbg.so).

Steps the bench sampler's 1024 worlds a few times and, per step, buckets the
worlds by LCP rows m: which kernel stepped them (the one-row kernel with the
pool on chip, the one-row kernel with the pool in HBM, or the wide kernel)
and their latency (shader clocks from loadState to integratePositions), with
the contact-stage split of the slowest world of each bucket.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path[:0] = ["tests", "."]
from nimblephysics_amd import _native, workloads  # noqa: E402

B = 1024
w = workloads.atlas_mesh_world(True)
st, f = workloads.atlas_states(w, B, 1000)
d = torch.device("cuda:0")
state, action = torch.tensor(st, device=d), torch.tensor(f, device=d)
dev = w.native()
n = w.getNumDofs()
cache = torch.zeros((B, dev.cache_doubles), dtype=torch.float64, device=d)
cache[:, 0] = -1
snap = torch.zeros((B, dev.snapshot_doubles), dtype=torch.float64, device=d)
ws = _native.snapshot_layout(n, timing=True)["stamps"]
s = torch.cuda.current_stream().cuda_stream
out = {"workload": "atlas_mesh, bench sampler seed 1000, 1024 worlds", "steps": []}
for it in range(int(os.environ.get("STEPS", "4"))):
    snap[:, ws:ws + 128] = 0
    nxt = torch.empty_like(state)
    dev.forward(state, action, cache, nxt, snap, s)
    torch.cuda.synchronize()
    T = snap[:, ws:ws + 128].cpu().numpy()
    hd = snap[:, :8].cpu().numpy()
    m = hd[:, 1].astype(int)
    tot = np.where((T[:, 10] > 0) & (T[:, 13] > 0), T[:, 13] - T[:, 10], 0)
    edges = [0, 1, 13, 25, 37, 49, 65, 81, 97, 129]
    rows = []
    for a, b in zip(edges[:-1], edges[1:]):
        sel = (m >= a) & (m < b)
        if not sel.any():
            continue
        v = tot[sel]
        wi = np.flatnonzero(sel)[np.argmax(v)]
        rows.append({"rows": f"{a}-{b - 1}", "worlds": int(sel.sum()), "mean_clk": float(v.mean()),
                     "max_clk": float(v.max()), "sum_clk": float(v.sum()),
                     "slowest": {"world": int(wi), "m": int(m[wi]), "clamping": int(hd[wi, 2]),
                                 "short_circuit": int(hd[wi, 6]),
                                 "stages": {nm: float(T[wi, y] - T[wi, x]) for nm, (x, y) in
                                            {"collide": (0, 1), "rows+A": (1, 3), "guess": (3, 4), "construct1": (4, 5),
                                             "dantzig": (5, 6), "fallbacks": (6, 7), "construct2": (7, 8),
                                             "impulses+precompute": (8, 9)}.items()
                                            if T[wi, x] > 0 and T[wi, y] > 0}}})
    out["steps"].append({"step": it, "buckets": rows})
    print(f"--- step {it}")
    for r in rows:
        print(f"  m {r['rows']:>7s}: worlds {r['worlds']:4d} mean {r['mean_clk']:10.0f} max {r['max_clk']:10.0f} "
              f"| slowest m={r['slowest']['m']} nc={r['slowest']['clamping']} sc={r['slowest']['short_circuit']} "
              + " ".join(f"{k}={v:.0f}" for k, v in r["slowest"]["stages"].items()))
    state = nxt
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open(os.path.join("gpurun_out", os.environ.get("BUCKETS_OUT", "mesh_buckets.json")), "w"), indent=1)
