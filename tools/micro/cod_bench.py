"""COD micro-benchmark: register-resident QR vs the LDS factorisation on
construct-like matrices (Q = Y^T Y of rank r <= n, and full-rank ones).

  python tools/micro/cod_bench.py build   # here: dbg/libcod_{reg,lds}.so
  python tools/micro/cod_bench.py run     # GPU box: clocks, rank, solution
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "tools", "micro", "cod_bench.hip")
LIBS = {"reg": os.path.join(ROOT, "dbg", "libcod_reg.so"), "lds": os.path.join(ROOT, "dbg", "libcod_lds.so")}
NMAX, REC = 24, 64


def build():
    os.makedirs(os.path.join(ROOT, "dbg"), exist_ok=True)
    for k, lib in LIBS.items():
        extra = ["-DNIMBLE_COD_LDS_ONLY"] if k == "lds" else []
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared"] + extra +
                              ["-o", lib, SRC])


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


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1] if len(sys.argv) > 1 else "run"]()
