"""Per-stage shader-clock breakdown of the forward kernel (debug build with
-DNIMBLE_STAGE_TIMING; run on a GPU box with NIMBLE_AMD_LIB pointing at it)."""
import glob
import re
import sys

import numpy as np
import torch

sys.path[:0] = ["tests", "."]
import models  # noqa: E402
import nimblephysics_amd as nimble  # noqa: E402


def check_slot_map(csrc="nimblephysics_amd/csrc"):
    """Static check of the stamp slot map: every multi-slot debug block
    (SLOT_* in stamp.cuh, with its width) is disjoint from the others and from
    every single stamp / accumulator slot the sources write, and all fit in
    SLOT_COUNT.  Returns the block table; raises on a collision."""
    src = "".join(open(f).read() for f in sorted(glob.glob(csrc + "/*.cuh") + glob.glob(csrc + "/*.hip")))
    stamp = open(csrc + "/stamp.cuh").read()
    count = int(re.search(r"#define SLOT_COUNT (\d+)", stamp).group(1))
    widths = {"SLOT_PGS": 5, "SLOT_COD": 3, "SLOT_DANTZIG": 10}
    blocks = {k: (int(v), int(v) + widths[k]) for k, v in re.findall(r"#define (SLOT_\w+) (\d+)", stamp) if k in widths}
    singles = set(int(k) for k in re.findall(r"STAMP\((\d+)\)", src))
    singles |= set(int(k) for k in re.findall(r"TACC_END\((\d+)", src))
    singles |= set(int(k) for k in re.findall(r"g_stamp\[(\d+)\]", src))
    if re.search(r"g_stamp \+ \d", src):
        raise AssertionError("raw g_stamp + <number> offset: use a SLOT_* block")
    for k, (a, b) in blocks.items():
        assert b <= count, (k, a, b, count)
        hit = sorted(x for x in singles if a <= x < b)
        assert not hit, f"{k} [{a},{b}) overlaps single slots {hit}"
        for k2, (a2, b2) in blocks.items():
            assert k == k2 or b <= a2 or b2 <= a, f"{k} overlaps {k2}"
    assert max(singles) < count, max(singles)
    return blocks


SLOTS = check_slot_map()
SD = SLOTS["SLOT_DANTZIG"][0]
B = 1024
import os  # noqa: E402
if os.environ.get("STAGE_WORKLOAD") == "atlas_mesh":
    from nimblephysics_amd import workloads  # noqa: E402
    w = workloads.atlas_mesh_world(True)
else:
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
for it in range(4):
    snap[:, ws:ws + 128] = 0
    prev_state, prev_cache = state.clone(), cache.clone()
    dev.forward(state, action, cache, nxt, snap, s)
    torch.cuda.synchronize()
    state = nxt.clone()
    T = snap[:, ws:ws + 128].cpu().numpy()
    hd = snap[:, :8].cpu().numpy()
    names = {(10, 14): " kinematics", (14, 15): " composites", (15, 16): " CRBA + bias", (16, 17): " cholesky", (17, 11): " dynamics cache store",
             (70, 71): "  kin: local transforms", (71, 72): "  kin: tree compose", (72, 73): "  kin: motion subspace",
             (73, 74): "  kin: twists", (74, 75): "  kin: accelerations",
             (10, 11): "load+coreDynamics", (40, 41): " c1: Q build", (41, 42): " c1: COD factor",
             (42, 43): " c1: COD solve", (43, 44): " c1: nx + valid", (45, 46): " pre: Ac/AcubE",
             (46, 47): " pre: MA/MAc backsub", (47, 48): " pre: Q", (48, 49): " pre: COD", (49, 50): " pre: pinv",
             (50, 51): " pre: imp", (11, 12): "solve v1", (0, 1): "collide", (1, 2): "rows",
             (2, 3): "cols/massed/A/b", (2, 86): " b = -J v1", (86, 87): " Y = L^-1 J^T", (87, 88): " A = Y^T Y (MFMA)",
             (88, 3): " pen / aCol", (3, 4): "warm start/guess", (4, 5): "construct 1",
             (5, 6): "dantzig", (6, 7): "pgs/fallbacks", (7, 8): "construct 2", (8, 9): "impulses/snapshot",
             (12, 13): "contact stage total+integrate",
             (104, 105): "wide: reload dynamics", (105, 106): "wide: solve v1",
             (106, 107): "wide: contact stage total+integrate"}
    print(f"--- step {it}: contact worlds {int((hd[:,0]>0).sum())}, short-circuit {int(hd[:,6].sum())}, "
          f"cfm worlds {int((hd[:,4]>0).sum())}")
    for (a, b), nm in names.items():
        m = (T[:, a] > 0) & (T[:, b] > 0)
        if m.any():
            dtk = T[m, b] - T[m, a]
            print(f"  {nm:32s} worlds {m.sum():5d}  mean {dtk.mean():10.0f}  max {dtk.max():10.0f}")
    # the slowest worlds set the kernel time: their per-stage split (a
    # deferred world's contact stage ran in the wide kernel: 106..107)
    wide = (T[:, 106] > 0) & (T[:, 107] > 0)
    tot = np.where(wide, T[:, 107] - T[:, 106], np.where((T[:, 12] > 0) & (T[:, 13] > 0), T[:, 13] - T[:, 12], 0))
    # every interval is between stamps of one launch: none may be negative
    for (a, b), nm in names.items():
        m = (T[:, a] > 0) & (T[:, b] > 0)
        assert not (m & (T[:, b] < T[:, a])).any(), f"negative interval {nm.strip()}: stamps of two launches"
    # the one-row kernel's own tail (its launch time is its slowest world's)
    one = np.where(~wide & (T[:, 12] > 0) & (T[:, 13] > 0), T[:, 13] - T[:, 10], 0)
    for wi in np.argsort(-one)[:3]:
        parts = [f"{nm.strip()}={int(T[wi, b] - T[wi, a])}" for (a, b), nm in names.items()
                 if T[wi, a] > 0 and T[wi, b] > 0 and b < 100 and (a, b) not in ((10, 11), (12, 13))]
        print(f"  one-row world {wi}: total {int(one[wi])} rows {int(hd[wi, 1])} clamp {int(hd[wi, 2])} contacts {int(hd[wi, 0])} "
              f"narrow phase {int(T[wi, 76])} post-process {int(T[wi, 77])} mesh pairs {int(T[wi, 120])} MPR {int(T[wi, 121])} "
              f"witness {int(T[wi, 122])} contacts {int(T[wi, 123])} (hulls {int(T[wi, 124])} sort {int(T[wi, 125])} "
              f"contain {int(T[wi, 126])} edges {int(T[wi, 127])}) | " + " ".join(parts))
    for wi in np.argsort(-tot)[:6]:
        parts = []
        for (a, b), nm in names.items():
            if T[wi, a] > 0 and T[wi, b] > 0 and (a, b) not in ((10, 11), (12, 13), (106, 107)):
                parts.append(f"{nm.strip()}={int(T[wi, b] - T[wi, a])}")
        print("      collide: narrow phase %d  post-process %d" % (T[wi, 76], T[wi, 77]))
        print("      construct acc: iters %d cls %d Q %d codF %d codS %d nx %d valid %d | codF qr %d rz %d rank %d" % tuple(T[wi, 60:70]))
        if T[wi, 94] > 0:
            a0 = T[wi, 3]
            who = {0: "-", 1: "wave0", 2: "helper"}
            rel = lambda k: int(T[wi, k] - a0) if T[wi, k] > 0 else -1  # noqa: E731
            print("      board (clk from A built): construct done %d, helper Dantzig %d..%d (%d pivots, %s), answer at %d; "
                  "PGS fallback %s %d..%d, frictionless %s %d..%d"
                  % (T[wi, 5] - a0, T[wi, 94] - a0, T[wi, 95] - a0, T[wi, SD], {1: "ok", 2: "failed"}.get(int(T[wi, 96]), "?"),
                     T[wi, 6] - a0, who.get(int(T[wi, 97]), "?"), rel(100), rel(101), who.get(int(T[wi, 98]), "?"),
                     rel(102), rel(103)))
        print(f"  world {wi}: pivots {int(T[wi,SD])} at row {int(T[wi,SD+1])} pgs-sweeps {int(T[wi,54])} ign {hd[wi,7]:.0f} total {int(tot[wi])} rows {int(hd[wi,1])} clamp {int(hd[wi,2])} flag {hd[wi,4]:.0f} | " + " ".join(parts))

# the slowest world of the last step re-run alone (one wave on the GPU): how
# much of its time is contention with the other worlds' waves
wi = int(np.argsort(-tot)[0])
st1, ca1, ac1 = prev_state[wi:wi + 1].clone(), prev_cache[wi:wi + 1].clone(), action[wi:wi + 1].clone()
sn1 = torch.zeros((1, dev.snapshot_doubles), dtype=torch.float64, device=d)
nx1 = torch.empty_like(st1)
for rep in range(2):
    sn1[:, ws:ws + 128] = 0
    c1 = ca1.clone()
    dev.forward(st1, ac1, c1, nx1, sn1, s)
    torch.cuda.synchronize()
T1 = sn1[:, ws:ws + 128].cpu().numpy()[0]
parts = []
for (a, b), nm in names.items():
    if T1[a] > 0 and T1[b] > 0 and (a, b) not in ((10, 11),):
        parts.append(f"{nm.strip()}={int(T1[b] - T1[a])} (batch {int(T[wi, b] - T[wi, a])})")
print(f"solo world {wi}: " + " ".join(parts))
print("      construct acc solo: iters %d cls %d Q %d codF %d codS %d nx %d valid %d | codF qr %d rz %d rank %d" % tuple(T1[60:70]))

# per-world forward latency histogram of the last batch step (the kernel's
# time is the slowest world's): written as JSON next to the log
import json, os  # noqa: E402
out = os.environ.get("STAGE_HIST_OUT")
if out:
    tot_all = np.where((T[:, 10] > 0) & (T[:, 13] > 0), T[:, 13] - T[:, 10], 0).astype(np.float64)
    ok = tot_all > 0
    v = tot_all[ok]
    edges = np.linspace(0, v.max() * 1.0001, 21)
    h, _ = np.histogram(v, bins=edges)
    path = hd[:, 6]
    res = {"worlds": int(ok.sum()), "unit": "shader clocks (s_memtime) per world, loadState..integratePositions",
           "mean": float(v.mean()), "p50": float(np.percentile(v, 50)), "p90": float(np.percentile(v, 90)),
           "p99": float(np.percentile(v, 99)), "max": float(v.max()), "max_over_mean": float(v.max() / v.mean()),
           "bins_clk": [float(e) for e in edges], "counts": [int(c) for c in h],
           "by_class": {
               "no_contact": float(v[(hd[ok, 0] == 0)].mean()) if (hd[ok, 0] == 0).any() else None,
               "short_circuit": float(v[(hd[ok, 0] > 0) & (path[ok] > 0)].mean()) if ((hd[ok, 0] > 0) & (path[ok] > 0)).any() else None,
               "fallback": float(v[(hd[ok, 0] > 0) & (path[ok] == 0)].mean()) if ((hd[ok, 0] > 0) & (path[ok] == 0)).any() else None},
           "slowest": [{"world": int(wi), "clk": float(tot_all[wi]), "rows": int(hd[wi, 1]), "clamping": int(hd[wi, 2]),
                        "short_circuit": int(hd[wi, 6]), "dantzig_pivots": int(T[wi, SD]), "pgs_sweeps": int(T[wi, 54])}
                       for wi in np.argsort(-tot_all)[:10]]}
    json.dump(res, open(out, "w"), indent=1)
    print("histogram ->", out, json.dumps({k: res[k] for k in ("mean", "p50", "p99", "max", "max_over_mean")}))

# placement of each world's two waves (HW_ID: SIMD bits 5:4, CU 11:8, SE
# 15:13; XCC_ID bits 3:0), from the last batch step
hw0, hw1 = T[:, 90].astype(np.int64), T[:, 92].astype(np.int64)
xcc0 = T[:, 91].astype(np.int64) & 15
have = (hw0 > 0) | (hw1 > 0)
if have.any():
    simd0, simd1 = (hw0 >> 4) & 3, (hw1 >> 4) & 3
    cu0, cu1 = (hw0 >> 8) & 15, (hw1 >> 8) & 15
    same_simd = (simd0 == simd1) & (cu0 == cu1)
    tot_all = np.where((T[:, 10] > 0) & (T[:, 13] > 0), T[:, 13] - T[:, 10], 0).astype(np.float64)
    ok = have & (tot_all > 0)
    print(f"placement: worlds {int(have.sum())}, helper on wave 0's SIMD {int(same_simd[have].sum())}, "
          f"XCC histogram {np.bincount(xcc0[have], minlength=8).tolist()}")
    for name, msk in (("same SIMD", ok & same_simd), ("other SIMD", ok & ~same_simd)):
        if msk.any():
            print(f"  {name:10s}: worlds {int(msk.sum())} mean {tot_all[msk].mean():.0f} clk, max {tot_all[msk].max():.0f}")
    if out:
        res = json.load(open(out))
        res["placement"] = {"helper_on_same_simd": int(same_simd[have].sum()), "worlds": int(have.sum()),
                            "xcc_histogram": np.bincount(xcc0[have], minlength=8).tolist(),
                            "mean_clk_same_simd": float(tot_all[ok & same_simd].mean()) if (ok & same_simd).any() else None,
                            "mean_clk_other_simd": float(tot_all[ok & ~same_simd].mean()) if (ok & ~same_simd).any() else None}
        json.dump(res, open(out, "w"), indent=1)
