"""The device Dantzig solver (waveDantzigR, lcp_wave.cuh) on the LCPs where
the device, the oracle's restatement and the reference's own compiled
dSolveLCP (oracle/_ref, dart/external/odelcpsolver/lcp.cpp:780) do not all
agree (tests/golden/dantzig_disagreements.npz, tools/dantzig_reconcile.py
over the bench Atlas' LCPs).

What reaches the step is the effective outcome, dSolveLCP's success AND
LCPUtils::isLCPSolutionValid (BoxedLcpConstraintSolver.cpp:466-521).  Per
problem: the device's effective outcome equals the reference's, and then x
agrees to 1e-9 where both are valid, or both are solutions of a degenerate
LCP (rank-deficient A, x_device - x_ref in its null space; the step's
re-standardisation then maps either to the same x); or the reference itself
gives both outcomes under 1e-15-relative perturbations of A (ambiguous:
rank-deficient A, both feet flat).  Run through the stand-alone harness
tests/cpp/liblcp_bench.so (tools/lcp_bench.hip: the product's lcp_wave.cuh,
A in LDS as in the forward kernel).
"""
import ctypes as C
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "golden", "dantzig_disagreements.npz")
HARNESS = os.path.join(ROOT, "tests", "cpp", "liblcp_bench.so")
REC, X_D = 128, 16


def classify(k, m, A, b, lo, hi, fi, ok, x, d):
    """'agree' (same effective outcome, x within 1e-9 when valid) or
    'ambiguous' (outcomes differ, the fixture's reference outcome flips
    under perturbation); raises otherwise."""
    eff = bool(ok) and bool(O.lcp_valid(A, x, b, hi, lo, fi))
    ref_eff = bool(d["ref_valid"][k])
    if eff == ref_eff:
        if eff:
            rx = d["ref_x"][k, :m]
            err = np.abs(x - rx).max() / max(1.0, np.abs(rx).max())
            if err > 1e-9:
                # both valid yet apart: a rank-deficient A whose LCP has a set of
                # solutions; the difference must lie in A's null space (same w)
                res = np.abs(A @ (x - rx)).max() / max(1.0, np.abs(A).max() * np.abs(rx).max())
                assert res <= 1e-12 and np.linalg.matrix_rank(A) < m, (k, err, res)
                return "nonunique"
        return "agree"
    amb = int(d["ref_ambiguous"][k])
    if amb < 0 and O.ref_lib() is not None:
        # (not classified when the fixture was made: the device at that time
        # agreed) -- check with the reference's own solver now
        amb = int(O.ref_dantzig_ambiguous(A, b, lo, hi, fi, seed=int(d["problem"][k])))
    assert amb == 1, (k, "effective outcome differs from the reference's on an unambiguous problem")
    return "ambiguous"


def test_dantzig_disagreements_on_device():
    if not os.path.exists(HARNESS):
        pytest.fail(f"{HARNESS} missing: __graft_entry__.build() compiles it")
    d = np.load(FIXTURE)
    P = len(d["n"])
    assert P > 0
    nmax = int(round(np.sqrt(d["A"].shape[1])))
    dev = torch.device("cuda:0")
    T = {k: torch.tensor(d[k], device=dev) for k in ("n", "A", "b", "lo", "hi")}
    T["fi"] = torch.tensor(d["fi"].astype(np.int32), device=dev)
    T["n"] = T["n"].to(torch.int32)
    x0 = torch.zeros_like(T["b"])
    out = torch.zeros((P, REC), dtype=torch.float64, device=dev)
    lib = C.CDLL(HARNESS)
    rc = lib.lcp_bench_launch(C.c_int(P), C.c_int(nmax), C.c_int(int(d["n"].max())),
                              *[C.c_void_p(T[k].data_ptr()) for k in ("n", "A", "b", "lo", "hi", "fi")],
                              C.c_void_p(x0.data_ptr()), C.c_void_p(out.data_ptr()),
                              C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    kinds = {"agree": 0, "ambiguous": 0, "nonunique": 0}
    for k in range(P):
        m = int(d["n"][k])
        A = d["A"][k, :m * m].reshape(m, m)
        kinds[classify(k, m, A, d["b"][k, :m], d["lo"][k, :m], d["hi"][k, :m], d["fi"][k, :m], o[k, 0] > 0,
                       o[k, X_D:X_D + m], d)] += 1
    print(kinds)


FIXTURE_WIDE = os.path.join(ROOT, "tests", "golden", "dantzig_wide_disagreements.npz")


@pytest.mark.parametrize("packed", [0, 1])
def test_dantzig_wide_disagreements_on_device(packed, monkeypatch):
    """The two-rows-per-lane Dantzig of the wide forward kernel (waveDantzigR
    R = 2, L unpacked or in the packed panels of the wide kernel's LDS stage)
    on the STL-mesh Atlas' > 64-row LCPs where the device, the oracle and the
    reference's compiled dSolveLCP do not all give the same raw outcome
    (tests/golden/dantzig_wide_disagreements.npz: tools/dantzig_reconcile.py
    classify_wide over 512 problems, profiles/r06_dantzig_wide_reconcile.json:
    effective outcomes equal on all 512).  Each problem's effective outcome
    must equal the reference's, or the reference's must flip under 1e-15
    perturbations."""
    if not os.path.exists(HARNESS):
        pytest.fail(f"{HARNESS} missing: __graft_entry__.build() compiles it")
    monkeypatch.setenv("LCP_WIDE_PACKED", str(packed))
    d = np.load(FIXTURE_WIDE)
    P = len(d["n"])
    assert P > 0
    nmax = int(round(np.sqrt(d["A"].shape[1])))
    dev = torch.device("cuda:0")
    T = {k: torch.tensor(d[k], device=dev) for k in ("A", "b", "lo", "hi")}
    T["fi"] = torch.tensor(d["fi"].astype(np.int32), device=dev)
    T["n"] = torch.tensor(d["n"].astype(np.int32), device=dev)
    assert int(d["n"].max()) <= 112  # the harness record holds x of up to 112 rows
    out = torch.zeros((P, REC), dtype=torch.float64, device=dev)
    lib = C.CDLL(HARNESS)
    rc = lib.lcp_bench_wide_launch(C.c_int(P), C.c_int(nmax), C.c_int(int(d["n"].max())),
                                   *[C.c_void_p(T[k].data_ptr()) for k in ("n", "A", "b", "lo", "hi", "fi")],
                                   C.c_void_p(out.data_ptr()), C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    kinds = {"agree": 0, "ambiguous": 0, "nonunique": 0}
    for k in range(P):
        m = int(d["n"][k])
        A = d["A"][k, :m * m].reshape(m, m)
        kinds[classify(k, m, A, d["b"][k, :m], d["lo"][k, :m], d["hi"][k, :m], d["fi"][k, :m], o[k, 0] > 0,
                       o[k, X_D:X_D + m], d)] += 1
    print(packed, kinds)
