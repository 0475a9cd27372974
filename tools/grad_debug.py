"""Per-world / per-dof gradient error structure, GPU vs oracle (GPU box)."""
import sys

import numpy as np
import torch

sys.path[:0] = ["tests", "."]
import models  # noqa: E402
from oracle import oracle as O  # noqa: E402

w = models.atlas_world(True)
B = 64
st, f = models.random_states(w, B, seed=3, q_scale=0.01, v_scale=0.02)
ow = O.OracleWorld(w)
ref = ow.forward(st, f)
dev = w.native()
d = torch.device("cuda:0")
ts, tf = torch.tensor(st, device=d), torch.tensor(f, device=d)
cache = torch.zeros((B, dev.cache_doubles), dtype=torch.float64, device=d)
cache[:, 0] = -1
nxt = torch.empty_like(ts)
snap = torch.zeros((B, dev.snapshot_doubles), dtype=torch.float64, device=d)
s = torch.cuda.current_stream().cuda_stream
dev.forward(ts, tf, cache, nxt, snap, s)
n = w.getNumDofs()
np.set_printoptions(precision=3, linewidth=200)
for mode in ("pos", "vel", "rand"):
    g = np.zeros(st.shape)
    if mode == "pos":
        g[:, :n] = np.random.default_rng(1).standard_normal((B, n))
    elif mode == "vel":
        g[:, n:] = np.random.default_rng(1).standard_normal((B, n))
    else:
        g = np.random.default_rng(1).standard_normal(st.shape)
    rgs, rgf = ow.backward(g)
    gs, gf = torch.empty_like(ts), torch.empty_like(tf)
    dev.backward(ts, tf, snap, torch.tensor(g, device=d), gs, gf, s)
    torch.cuda.synchronize()
    gs, gf = gs.cpu().numpy(), gf.cpu().numpy()
    sn = snap.cpu().numpy()
    print("== grad mode", mode)
    for b in range(B):
        eq = np.abs(gs[b, :n] - rgs[b, :n]).max() / np.abs(rgs[b]).max()
        ev = np.abs(gs[b, n:] - rgs[b, n:]).max() / np.abs(rgs[b]).max()
        et = np.abs(gf[b] - rgf[b]).max() / np.abs(rgf[b]).max()
        if max(eq, ev, et) > 1e-6:
            fl = O.lcp_flags(ow, b)
            print(f"world {b}: eq {eq:.2e} ev {ev:.2e} et {et:.2e} ncon {int(sn[b,0])} nc {int(sn[b,2])} nu {int(sn[b,3])} "
                  f"flags {fl}")
            print("   dq err dofs", np.argsort(-np.abs(gs[b, :n] - rgs[b, :n]))[:8],
                  (gs[b, :n] - rgs[b, :n])[np.argsort(-np.abs(gs[b, :n] - rgs[b, :n]))[:8]])
for b in (32, 55):
    m = int(sn[b, 1])
    rows = sn[b, 176:176 + 12 * m].reshape(m, 12)
    print("world", b, "GPU flags", sn[b, [6, 7, 4, 2, 3]], "map", rows[:, 7], "X", rows[:, 6])
    print("   GPU fc", sn[b, 752:752 + int(sn[b, 2])], "Eval", rows[:, 10], "bounce", rows[:, 11])
    mp, x = O.lcp_debug(ow, b)
    print("   ORA flags", O.lcp_flags(ow, b), "map", mp, "X", x)
    print("   ORA fc", O.lcp_fc(ow, b))
# numpy restatement of grad_tau = dt (w - nu) for the failing worlds, from
# the oracle's own matrices
gv_only = np.zeros(st.shape)
gv_only[:, n:] = np.random.default_rng(1).standard_normal((B, n))
rgs, rgf = ow.backward(gv_only)
gs, gf = torch.empty_like(ts), torch.empty_like(tf)
dev.backward(ts, tf, snap, torch.tensor(gv_only, device=d), gs, gf, s)
torch.cuda.synchronize()
gf = gf.cpu().numpy()
dt = w.getTimeStep()
for b in (32, 55):
    q = st[b, :n]
    M = ow.mass_matrix(q)
    Minv = np.linalg.inv(M)
    cols = O.lcp_cols(ow, b)
    mp, x = O.lcp_debug(ow, b)
    fl = O.lcp_flags(ow, b)
    cl = [j for j in range(len(mp)) if mp[j] == -1]
    Ac = cols[:, cl]
    AcubE = Ac.copy()
    for j in range(len(mp)):
        if mp[j] >= 0:
            c = cl.index(mp[j])
            fp = mp[j]
            up, lo_ = x[fp] * 1.0, -x[fp] * 1.0
            e = 1.0 if abs(x[j] - up) < abs(x[j] - lo_) else -1.0
            AcubE[:, c] += e * cols[:, j]
    Q = Ac.T @ Minv @ AcubE + fl[2] * np.eye(len(cl))
    wv = Minv @ gv_only[b, n:]
    u = AcubE.T @ wv
    lam = np.linalg.pinv(Q).T @ u
    nu = Minv @ (Ac @ lam)
    gt_np = dt * (wv - nu)
    print("world", b, "numpy vs oracle", np.abs(gt_np - rgf[b]).max() / np.abs(rgf[b]).max(),
          "numpy vs gpu", np.abs(gt_np - gf[b]).max() / np.abs(gf[b]).max(), "Q", Q)
snp = snap.cpu().numpy()
for b in (32, 55):
    ws = ((752 + 48 + n + 7) // 8) * 8
    dbg = snp[b, ws:]
    nc = int(dbg[0])
    o = 2
    Qg = dbg[o:o + nc * nc].reshape(nc, nc); o += nc * nc
    ug = dbg[o:o + nc]; o += nc
    lg = dbg[o:o + nc]; o += nc
    PT = dbg[o:o + nc * nc].reshape(nc, nc); o += nc * nc
    AcubEg = dbg[o:o + n * nc].reshape(n, nc); o += n * nc
    Acg = dbg[o:o + n * nc].reshape(n, nc); o += n * nc
    print("world", b, "imp", dbg[1], "Q gpu", Qg, "P^T", PT)
    print("   u", ug, "lam", lg)
    q = st[b, :n]
    Minv = np.linalg.inv(ow.mass_matrix(q))
    cols = O.lcp_cols(ow, b)
    mp, x = O.lcp_debug(ow, b)
    cl = [j for j in range(len(mp)) if mp[j] == -1]
    print("   Ac diff", np.abs(Acg - cols[:, cl]).max(), "AcubE-Ac gpu", np.abs(AcubEg - Acg).max())
print("---- intermediates vs numpy")
for b in (32, 55):
    ws = ((752 + 48 + n + 7) // 8) * 8
    dbg = snp[b, ws:]
    nc = int(dbg[0]); o = 2
    Qg = dbg[o:o + nc * nc].reshape(nc, nc); o += nc * nc
    ug = dbg[o:o + nc]; o += nc
    lg = dbg[o:o + nc]; o += nc
    o += nc * nc
    AcubEg = dbg[o:o + n * nc].reshape(n, nc); o += n * nc
    q = st[b, :n]
    Minv = np.linalg.inv(ow.mass_matrix(q))
    cols = O.lcp_cols(ow, b)
    mp, x = O.lcp_debug(ow, b)
    cl = [j for j in range(len(mp)) if mp[j] == -1]
    AcubE = cols[:, cl].copy()
    for j in range(len(mp)):
        if mp[j] >= 0:
            c = cl.index(mp[j]); fp = mp[j]
            e = 1.0 if abs(x[j] - x[fp]) < abs(x[j] + x[fp]) else -1.0
            AcubE[:, c] += e * cols[:, j]
    wv = Minv @ gv_only[b, n:]
    print("world", b, "AcubE diff", np.abs(AcubEg - AcubE).max(), "u gpu", ug, "u np", AcubE.T @ wv,
          "x", x, "mp", mp)
print("---- NV columns")
for b in (32, 55):
    ws = ((752 + 48 + n + 7) // 8) * 8
    dbg = snp[b, ws:]
    nc = int(dbg[0]); o = 2 + 2 * nc * nc + 2 * nc + 2 * n * nc
    NV = dbg[o:o + n * 16].reshape(n, 16); o += n * 16
    w2 = dbg[o:o + n]
    q = st[b, :n]
    Minv = np.linalg.inv(ow.mass_matrix(q))
    cols = O.lcp_cols(ow, b)
    mp, x = O.lcp_debug(ow, b)
    cl = [j for j in range(len(mp)) if mp[j] == -1]
    Ac = cols[:, cl]
    lg = dbg[2 + nc * nc + nc: 2 + nc * nc + 2 * nc]
    mu = Ac @ lg
    print("world", b, "w diff", np.abs(NV[:, 9] - Minv @ gv_only[b, n:]).max(), "mu diff", np.abs(NV[:, 11] - mu).max(),
          "nu diff", np.abs(NV[:, 1] - Minv @ mu).max(), "w2 diff", np.abs(w2 - (NV[:, 9] - NV[:, 1])).max(),
          "gt vs dt*w2", np.abs(gf[b] - dt * w2).max(), "|gt|", np.abs(gf[b]).max())
