"""COD micro-benchmark: register-resident QR vs the LDS factorisation on
construct-like matrices (Q = Y^T Y of rank r <= n, and full-rank ones).

  python tools/micro/cod_bench.py build   # here: dbg/libcod_{reg,lds}.so
  python tools/micro/cod_bench.py run     # GPU box: clocks, rank, solution
  python tools/micro/cod_bench.py mfma    # GPU box: QR phase split + MFMA rank-4 update
  python tools/micro/cod_bench.py wide    # GPU box: the two-slot LDS factorisation at 64..100
  python tools/micro/cod_bench.py ab      # GPU box: register QR vs dbg/libcod_reg_old.so (a previous build)
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "tools", "micro", "cod_bench.hip")
LIBS = {"reg": os.path.join(ROOT, "dbg", "libcod_reg.so"), "lds": os.path.join(ROOT, "dbg", "libcod_lds.so")}
PROF_LIB = os.path.join(ROOT, "dbg", "libcod_prof.so")
MFMA_SRC = os.path.join(ROOT, "tools", "micro", "cod_mfma.hip")
MFMA_EXE = os.path.join(ROOT, "dbg", "cod_mfma")
NMAX, REC = 24, 64


def build():
    os.makedirs(os.path.join(ROOT, "dbg"), exist_ok=True)
    for k, lib in LIBS.items():
        extra = ["-DNIMBLE_COD_LDS_ONLY"] if k == "lds" else []
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared"] + extra +
                              ["-o", lib, SRC])
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-DNIMBLE_COD_PROFILE", "-o", PROF_LIB, SRC])
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-o", MFMA_EXE, MFMA_SRC])


def problems(P=2048, seed=0):
    rng = np.random.default_rng(seed)
    n = rng.integers(2, NMAX + 1, size=P).astype(np.int32)
    n[: P // 4] = 24
    A = np.zeros((P, NMAX * NMAX))
    b = np.zeros((P, NMAX))
    for p in range(P):
        k = n[p]
        r = k if p % 3 == 0 else max(1, k // 2)
        Y = rng.standard_normal((33, k))
        if r < k:
            Y = Y[:, :r] @ rng.standard_normal((r, k))
        Q = Y.T @ Y
        A[p, : k * k] = Q.ravel()
        b[p, :k] = rng.standard_normal(k)
    return n, A, b


def run():
    import torch
    n, A, b = problems()
    P = len(n)
    dev = torch.device("cuda:0")
    T = [torch.tensor(x, device=dev) for x in (n, A, b)]
    s = torch.cuda.current_stream().cuda_stream
    res = {}
    for k, lib in LIBS.items():
        L = C.CDLL(lib)
        out = torch.zeros((P, REC), dtype=torch.float64, device=dev)
        for _ in range(3):
            assert L.cod_bench_launch(C.c_int(P), C.c_int(NMAX), *[C.c_void_p(t.data_ptr()) for t in T],
                                      C.c_void_p(out.data_ptr()), C.c_int(REC), C.c_void_p(s)) == 0
        torch.cuda.synchronize()
        res[k] = out.cpu().numpy()
    # uncontended latency: the first 200 (n = 24) problems alone, < 1 wave per CU
    for k, lib in LIBS.items():
        L = C.CDLL(lib)
        out = torch.zeros((200, REC), dtype=torch.float64, device=dev)
        for _ in range(3):
            L.cod_bench_launch(C.c_int(200), C.c_int(NMAX), *[C.c_void_p(t.data_ptr()) for t in T],
                               C.c_void_p(out.data_ptr()), C.c_int(REC), C.c_void_p(s))
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        print(f" solo n=24 {k}: factor clocks mean {o[:, 0].mean():8.0f} solve {o[:, 1].mean():7.0f}")
    # numpy min-norm least squares with the same rank as the check
    worst = {"reg": 0.0, "lds": 0.0}
    rank_same = (res["reg"][:, 2] == res["lds"][:, 2]).mean()
    for p in range(P):
        k = n[p]
        Q = A[p, : k * k].reshape(k, k)
        r = int(res["lds"][p, 2])
        U, S, Vt = np.linalg.svd(Q)
        xr = Vt[:r].T @ ((U[:, :r].T @ b[p, :k]) / S[:r])
        for key in worst:
            e = np.abs(res[key][p, 8:8 + k] - xr).max() / max(1.0, np.abs(xr).max())
            worst[key] = max(worst[key], e)
    print(f"{P} problems: rank agrees {rank_same:.4f}; max rel err vs SVD min-norm: reg {worst['reg']:.2e} lds {worst['lds']:.2e}")
    for m in (8, 12, 16, 24):
        sel = n == m
        if sel.any():
            print(f" n={m:2d} x{sel.sum():4d}: factor clocks reg {res['reg'][sel, 0].mean():8.0f} lds {res['lds'][sel, 0].mean():8.0f}"
                  f" | solve reg {res['reg'][sel, 1].mean():7.0f} lds {res['lds'][sel, 1].mean():7.0f}")


def mfma():
    """The register QR's per-step phase split (24 x 24 problems, solo and at
    1024 waves) and the rank-4 trailing-update micro-benchmark; JSON to stdout."""
    import json
    import torch
    n, A, b = problems()
    sel = np.where(n == 24)[0]
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    L = C.CDLL(PROF_LIB)
    res = {}
    for name, idx in (("solo_200", sel[:200]), ("batch_1024", np.resize(sel, 1024))):
        T = [torch.tensor(x[idx], device=dev) for x in (n, A, b)]
        out = torch.zeros((len(idx), REC), dtype=torch.float64, device=dev)
        for _ in range(2):
            assert L.cod_bench_launch(C.c_int(len(idx)), C.c_int(NMAX), *[C.c_void_p(t.data_ptr()) for t in T],
                                      C.c_void_p(out.data_ptr()), C.c_int(REC), C.c_void_p(s)) == 0
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        res[name] = {"factor_clk": float(o[:, 0].mean()), "qr_pivot_clk": float(o[:, 3].mean()),
                     "qr_broadcast_clk": float(o[:, 4].mean()), "qr_update_norms_clk": float(o[:, 5].mean()),
                     "qr_writeback_clk": float(o[:, 6].mean())}
    r = subprocess.run([MFMA_EXE], capture_output=True, text=True, timeout=120)
    res["rank4_update"] = json.loads(r.stdout.strip().splitlines()[-1])
    print(json.dumps(res, indent=1))


def wide(P=512, seed=1):
    """codFactorR<true, 2> on n x n Gram matrices, n in 64..100 (the wide
    forward kernel's staged classification factorisations): clocks of the
    factorisation and the solve, the per-step phase split (pivot + swap,
    reflector + |v|^2, trailing update + norms, write-back) and the error of
    the min-norm solution against numpy."""
    import json
    import torch
    NM = 100
    rng = np.random.default_rng(seed)
    n = rng.integers(64, NM + 1, size=P).astype(np.int32)
    n[: P // 4] = 96
    A = np.zeros((P, NM * NM))
    b = np.zeros((P, NM))
    for p in range(P):
        k = n[p]
        r = k if p % 3 == 0 else max(1, (2 * k) // 3)
        Y = rng.standard_normal((k + 8, r)) @ rng.standard_normal((r, k))
        A[p, : k * k] = (Y.T @ Y).ravel()
        b[p, :k] = rng.standard_normal(k)
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    res = {}
    for name, lib in (("plain", LIBS["reg"]), ("prof", PROF_LIB)):
        L = C.CDLL(lib)
        for label, cnt in (("solo_200", 200), ("batch", P)):
            T = [torch.tensor(x[:cnt], device=dev) for x in (n, A, b)]
            out = torch.zeros((cnt, 8 + 128), dtype=torch.float64, device=dev)
            for _ in range(2):
                assert L.cod_bench_wide_launch(C.c_int(cnt), C.c_int(NM), *[C.c_void_p(t.data_ptr()) for t in T],
                                               C.c_void_p(out.data_ptr()), C.c_int(8 + 128), C.c_void_p(s)) == 0
            torch.cuda.synchronize()
            o = out.cpu().numpy()
            sel = n[:cnt] == 96
            r = {"factor_clk_n96": float(o[sel, 0].mean()), "solve_clk_n96": float(o[sel, 1].mean())}
            if name == "prof":
                r.update({k: float(o[sel, 3 + i].mean()) for i, k in
                          enumerate(("pivot_swap", "reflector", "update_norms", "writeback", "dot"))})
            else:
                worst = 0.0
                for p in range(min(cnt, 64)):
                    k = n[p]
                    Q = A[p, : k * k].reshape(k, k)
                    rk = int(o[p, 2])
                    U, S, Vt = np.linalg.svd(Q)
                    xr = Vt[:rk].T @ ((U[:, :rk].T @ b[p, :k]) / S[:rk])
                    worst = max(worst, np.abs(o[p, 8:8 + k] - xr).max() / max(1.0, np.abs(xr).max()))
                r["max_rel_err_vs_svd"] = worst
            res[f"{name}_{label}"] = r
    print(json.dumps(res, indent=1))


def ab(old=os.path.join(ROOT, "dbg", "libcod_reg_old.so")):
    """A/B of the register QR against a previous build of it (same problems):
    clocks at n = 24 and whether factor outputs (solution, rank) are
    bit-identical."""
    import torch
    n, A, b = problems()
    P = len(n)
    dev = torch.device("cuda:0")
    T = [torch.tensor(x, device=dev) for x in (n, A, b)]
    s = torch.cuda.current_stream().cuda_stream
    res = {}
    for k, lib in (("old", old), ("new", LIBS["reg"])):
        L = C.CDLL(lib)
        out = torch.zeros((P, REC), dtype=torch.float64, device=dev)
        for _ in range(3):
            assert L.cod_bench_launch(C.c_int(P), C.c_int(NMAX), *[C.c_void_p(t.data_ptr()) for t in T],
                                      C.c_void_p(out.data_ptr()), C.c_int(REC), C.c_void_p(s)) == 0
        torch.cuda.synchronize()
        res[k] = out.cpu().numpy()
        sel = n == 24
        print(f"{k}: n=24 factor clocks {res[k][sel, 0].mean():.0f}, solve {res[k][sel, 1].mean():.0f}")
    same = np.array_equal(np.nan_to_num(res["old"][:, 8:]), np.nan_to_num(res["new"][:, 8:])) and \
        np.array_equal(res["old"][:, 2], res["new"][:, 2])
    print(f"bit-identical solutions and ranks: {same}")


if __name__ == "__main__":
    {"build": build, "run": run, "mfma": mfma, "wide": wide, "ab": ab}[sys.argv[1] if len(sys.argv) > 1 else "run"]()
