"""LCP solver micro-benchmark on the bench workload's own LCPs.

  python tools/lcp_bench.py gen     # CPU: oracle forward on the bench batch,
                                    # dump every world's LCP to dbg/lcp_problems.npz
  python tools/lcp_bench.py run     # GPU: waveDantzig + wavePgs per problem,
                                    # clocks + per-phase split, checked vs oracle

The harness (tools/lcp_bench.hip -> dbg/liblcp_bench.so) is built by `build`
(hipcc, here) and shipped to the GPU box with the snapshot.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
PROB = os.path.join(ROOT, "dbg", "lcp_problems.npz")
LIB = os.environ.get("LCP_BENCH_LIB", os.path.join(ROOT, "tests", "cpp", "liblcp_bench.so"))
NMAX = 48
REC = 128


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-DLCP_PROFILE", "-o", LIB, os.path.join(ROOT, "tools", "lcp_bench.hip")])


def gen(steps=3, batch=1024):
    import models
    from oracle.oracle import OracleWorld, lcp_problem, dantzig
    w = models.atlas_world(True)
    st, f = models.random_states(w, batch, seed=1000, q_scale=0.02, v_scale=0.05, f_scale=1.0)
    o = OracleWorld(w)
    rows = []
    for step in range(steps):
        nxt = o.forward(st, f)
        for b in range(batch):
            A, bb, lo, hi, fi = lcp_problem(o, b)
            if len(bb) > 0:
                rows.append((len(bb), A, bb, lo, hi, fi))
        st = nxt
    P = len(rows)
    n = np.array([r[0] for r in rows], dtype=np.int32)
    A = np.zeros((P, NMAX * NMAX))
    b = np.zeros((P, NMAX)); lo = np.zeros((P, NMAX)); hi = np.zeros((P, NMAX))
    fi = -np.ones((P, NMAX), dtype=np.int32)
    okD = np.zeros(P, dtype=np.int32); xD = np.zeros((P, NMAX))
    for k, (m, Am, bm, lom, him, fim) in enumerate(rows):
        A[k, :m * m] = np.asarray(Am).reshape(-1)[:m * m]
        b[k, :m] = bm; lo[k, :m] = lom; hi[k, :m] = him; fi[k, :m] = fim
        ok, x = dantzig(np.asarray(Am).reshape(m, m), bm, lom, him, fim, early=True)
        okD[k] = int(ok); xD[k, :m] = x
    os.makedirs(os.path.dirname(PROB), exist_ok=True)
    np.savez_compressed(PROB, n=n, A=A, b=b, lo=lo, hi=hi, fi=fi, okD=okD, xD=xD)
    print(f"{P} problems, n histogram {np.bincount(n)}, oracle dantzig ok {okD.mean():.3f}")


def run(reps=3):
    import torch
    d = np.load(PROB)
    P = len(d["n"])
    dev = torch.device("cuda:0")
    T = {k: torch.tensor(d[k], device=dev) for k in ("n", "A", "b", "lo", "hi", "fi")}
    x0 = torch.zeros_like(T["b"])
    out = torch.zeros((P, REC), dtype=torch.float64, device=dev)
    lib = C.CDLL(LIB)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(reps):
        rc = lib.lcp_bench_launch(C.c_int(P), C.c_int(NMAX), C.c_int(int(d["n"].max())), *[C.c_void_p(T[k].data_ptr()) for k in
                                                              ("n", "A", "b", "lo", "hi", "fi")],
                                  C.c_void_p(x0.data_ptr()), C.c_void_p(out.data_ptr()), C.c_void_p(s))
        assert rc == 0
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    n = d["n"]
    okD = o[:, 0] > 0
    agree = (okD == (d["okD"] > 0))
    err = 0.0
    for k in np.nonzero(okD & (d["okD"] > 0))[0]:
        m = n[k]
        e = np.abs(o[k, 16:16 + m] - d["xD"][k, :m]).max() / max(1.0, np.abs(d["xD"][k, :m]).max())
        err = max(err, e)
    # (the RAW success flags: not the step's outcome, which is success AND
    # isLCPSolutionValid -- tools/dantzig_reconcile.py classify compares that
    # with the reference's compiled dSolveLCP)
    print(f"{P} problems: raw dantzig flag same as the oracle's on {agree.mean():.4f} (effective outcomes: "
          f"tools/dantzig_reconcile.py classify), max rel x err where both raw-succeed {err:.2e}")
    # regression check against a previous GPU run (dbg/lcp_baseline.npz, copied
    # from gpurun_out/lcp_out.npz): solver outputs should be unchanged
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(ROOT, "gpurun_out", "lcp_out.npy"), o)
    base = os.path.join(ROOT, "dbg", "lcp_baseline.npy")
    if os.path.exists(base):
        ob = np.load(base)
        same_ok = (ob[:, 0] == o[:, 0]).mean(), (ob[:, 2] == o[:, 2]).mean()
        a, c = np.nan_to_num(ob[:, 16:112], nan=1e300), np.nan_to_num(o[:, 16:112], nan=1e300)
        dx = np.abs(a - c).max(axis=1) / np.maximum(1.0, np.abs(a).max(axis=1))
        print(f"vs baseline: dantzig ok same {same_ok[0]:.4f}, pgs ok same {same_ok[1]:.4f}, "
              f"bit-identical x {np.mean(dx == 0):.4f}, max rel dx {dx.max():.2e}, "
              f"dantzig clocks {o[:, 1].sum() / ob[:, 1].sum():.3f}x, pgs clocks {o[:, 3].sum() / ob[:, 3].sum():.3f}x")
    names = ["swap", "solveL1", "solveL1T", "ldltRemove", "w_i", "pivot body", "(matvec)", "(transfers)"]
    for m in sorted(set(n.tolist())):
        sel = n == m
        cd, cp = o[sel, 1], o[sel, 3]
        print(f" n={m:2d} x{sel.sum():4d}: dantzig mean {cd.mean():8.0f} max {cd.max():8.0f} "
              f"(ok {okD[sel].mean():.2f}, pivots mean {o[sel, 4].mean():.1f})  "
              f"pgs mean {cp.mean():8.0f} max {cp.max():8.0f} (sweeps mean {o[sel, 6].mean():.1f})")
        worst = np.argmax(np.where(sel, o[:, 1], -1))
        prof = o[worst, 8:14]
        print("      worst dantzig split: " + " ".join(f"{nm}={int(v)}" for nm, v in zip(names, o[worst, 8:16])))


PROB_WIDE = os.path.join(ROOT, "dbg", "lcp_wide.npz")
NMAX_WIDE = 128


def gen_wide(steps=2, batch=1024):
    """The STL-mesh Atlas' LCPs with more than 64 rows (the wide kernels')."""
    from nimblephysics_amd import workloads
    from oracle.oracle import OracleWorld, lcp_problem, dantzig
    w = workloads.atlas_mesh_world(True)
    st, f = workloads.atlas_states(w, batch, 1000)
    o = OracleWorld(w)
    rows = []
    for step in range(steps):
        nxt = o.forward(st, f)
        for b in range(batch):
            A, bb, lo, hi, fi = lcp_problem(o, b)
            if len(bb) > 64:
                rows.append((len(bb), A, bb, lo, hi, fi))
        st = nxt
    P = len(rows)
    N = NMAX_WIDE
    n = np.array([r[0] for r in rows], dtype=np.int32)
    A = np.zeros((P, N * N)); b = np.zeros((P, N)); lo = np.zeros((P, N)); hi = np.zeros((P, N))
    fi = -np.ones((P, N), dtype=np.int32)
    okD = np.zeros(P, dtype=np.int32)
    for k, (m, Am, bm, lom, him, fim) in enumerate(rows):
        A[k, :m * m] = np.asarray(Am).reshape(-1)
        b[k, :m] = bm; lo[k, :m] = lom; hi[k, :m] = him; fi[k, :m] = fim
        okD[k] = int(dantzig(np.asarray(Am).reshape(m, m), bm, lom, him, fim, early=True)[0])
    np.savez_compressed(PROB_WIDE, n=n, A=A, b=b, lo=lo, hi=hi, fi=fi, okD=okD)
    print(f"{P} wide problems, n {n.min()}..{n.max()}, oracle dantzig ok {okD.mean():.3f}")


def run_wide(limit=512):
    import torch
    d = np.load(PROB_WIDE)
    P = min(len(d["n"]), limit)
    dev = torch.device("cuda:0")
    T = {k: torch.tensor(d[k][:P], device=dev) for k in ("n", "A", "b", "lo", "hi", "fi")}
    out = torch.zeros((P, REC), dtype=torch.float64, device=dev)
    lib = C.CDLL(LIB)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(2):
        rc = lib.lcp_bench_wide_launch(C.c_int(P), C.c_int(NMAX_WIDE), C.c_int(int(d["n"][:P].max())),
                                       *[C.c_void_p(T[k].data_ptr()) for k in ("n", "A", "b", "lo", "hi", "fi")],
                                       C.c_void_p(out.data_ptr()), C.c_void_p(s))
        assert rc == 0
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    names = ["swap", "solveL1", "solveL1T", "ldltRemove", "w_i", "pivot body", "(matvec)", "(transfers)"]
    piv = np.maximum(o[:, 4], 1)
    print(f"{P} wide problems (raw flag same as the oracle's {np.mean((o[:, 0] > 0) == (d['okD'][:P] > 0)):.3f}; "
          "effective outcomes vs the reference: tools/dantzig_reconcile.py classify_wide); "
          f"clocks mean {o[:, 1].mean():.0f} max {o[:, 1].max():.0f}; pivots mean {o[:, 4].mean():.1f} max {o[:, 4].max():.0f}; "
          f"clocks per pivot mean {np.mean(o[:, 1] / piv):.0f}")
    worst = np.argsort(-o[:, 1])[:5]
    for k in worst:
        print(f"  problem {k} n={d['n'][k]} clocks {o[k, 1]:.0f} pivots {o[k, 4]:.0f} | "
              + " ".join(f"{nm}={int(v)}" for nm, v in zip(names, o[k, 8:16])))
    packed = os.environ.get("LCP_WIDE_PACKED", "0") not in ("", "0")
    np.save(os.path.join(ROOT, "gpurun_out", "lcp_wide_out_packed.npy" if packed else "lcp_wide_out.npy"), o)
    base = os.path.join(ROOT, "dbg", "lcp_wide_baseline.npy")
    if os.path.exists(base):
        ob = np.load(base)[:P]
        a, c = np.nan_to_num(ob[:, 16:128], nan=1e300), np.nan_to_num(o[:, 16:128], nan=1e300)
        dx = np.abs(a - c).max(axis=1) / np.maximum(1.0, np.abs(a).max(axis=1))
        print(f"vs baseline: ok same {(ob[:, 0] == o[:, 0]).mean():.4f}, pivots same {(ob[:, 4] == o[:, 4]).mean():.4f}, "
              f"bit-identical x {np.mean(dx == 0):.4f}, max rel dx {dx.max():.2e}, clocks {o[:, 1].sum() / ob[:, 1].sum():.3f}x")


def solo(count=6):
    """The slowest n=24 problems, each launched alone (one wave on the GPU):
    uncontended latency of the solvers."""
    import torch
    d = np.load(PROB)
    base = np.load(os.path.join(ROOT, "gpurun_out", "lcp_out.npy"))
    order = np.argsort(-(base[:, 1] + base[:, 3]))[:count]
    dev = torch.device("cuda:0")
    lib = C.CDLL(LIB)
    s = torch.cuda.current_stream().cuda_stream
    for k in order:
        T = {key: torch.tensor(d[key][k:k + 1], device=dev) for key in ("n", "A", "b", "lo", "hi", "fi")}
        x0 = torch.zeros_like(T["b"])
        out = torch.zeros((1, REC), dtype=torch.float64, device=dev)
        for _ in range(2):
            lib.lcp_bench_launch(C.c_int(1), C.c_int(NMAX), C.c_int(int(d["n"][k])),
                                 *[C.c_void_p(T[key].data_ptr()) for key in ("n", "A", "b", "lo", "hi", "fi")],
                                 C.c_void_p(x0.data_ptr()), C.c_void_p(out.data_ptr()), C.c_void_p(s))
        torch.cuda.synchronize()
        o = out.cpu().numpy()[0]
        print(f" problem {k} n={d['n'][k]}: solo dantzig {o[1]:8.0f} (batch {base[k, 1]:8.0f}, pivots {o[4]:.0f}) "
              f"pgs {o[3]:8.0f} (batch {base[k, 3]:8.0f}, sweeps {o[6]:.0f}, fast {o[7]:.0f}) | "
              + " ".join(f"{v:.0f}" for v in o[8:14]) + f" | cod factor {o[115]:.0f} solve {o[116]:.0f}")


if __name__ == "__main__":
    cmd = sys.argv[1] if len(sys.argv) > 1 else "run"
    if cmd == "build":
        build()
    elif cmd == "gen":
        gen()
    elif cmd == "solo":
        solo()
    elif cmd == "gen_wide":
        gen_wide()
    elif cmd == "run_wide":
        run_wide()
    else:
        run()
