"""Reconcile the Dantzig micro-benchmark (tools/lcp_bench.py) with the
reference's own dSolveLCP (oracle/_ref, dart/external/odelcpsolver/lcp.cpp:780).

The r02/r03 micro logs printed "dantzig success agrees with oracle on 0.927,
max rel x err 1.04".  That compared the device solver's RAW success flag and x
with the oracle's restatement.  On these problems (the bench Atlas' LCPs, most
of them rank-deficient: both feet flat) two things make that comparison
meaningless:

* a raw "success" is not the solver's answer: BoxedLcpConstraintSolver keeps
  a Dantzig solution only if LCPUtils::isLCPSolutionValid accepts it
  (BoxedLcpConstraintSolver.cpp:466-521), so the outcome that reaches the step
  is success AND valid;
* on rank-deficient A, dSolveLCP's pivoting flips under 1e-16-level rounding:
  the oracle's restatement and the reference's own compiled solver disagree
  with each other on ~5 % of these problems, every one ambiguous under 1e-15
  perturbations.

Usage (CPU here, after a GPU `python tools/lcp_bench.py run` has written
gpurun_out/lcp_out.npy for dbg/lcp_problems.npz):

  python tools/dantzig_reconcile.py classify   # summary -> profiles/r04_dantzig_reconcile.json
                                               # fixture -> tests/golden/dantzig_disagreements.npz

The fixture keeps every problem on which the device, the oracle and the
reference do not all give the same effective outcome, with the reference's
outcome and its ambiguity; tests/test_wave_emu.py runs them through the host
emulation of waveDantzigR, tests/test_gpu_lcp.py through the device (the
harness tools/lcp_bench.hip built to tests/cpp/liblcp_bench.so).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
PROB = os.path.join(ROOT, "dbg", "lcp_problems.npz")
OUT = os.path.join(ROOT, "gpurun_out", "lcp_out.npy")
FIXTURE = os.path.join(ROOT, "tests", "golden", "dantzig_disagreements.npz")
SUMMARY = os.path.join(ROOT, "profiles", "r04_dantzig_reconcile.json")
X_D = 16  # tools/lcp_bench.hip Rec::X_D


def ref_ambiguous(A, b, lo, hi, fi, seed, trials=512):
    """Both effective outcomes of the reference's compiled dSolveLCP occur
    under 1e-15-relative symmetric perturbations of A."""
    from oracle import oracle as O
    return bool(O.ref_dantzig_ambiguous(A, b, lo, hi, fi, seed, trials))


def effective(ok, x, A, b, lo, hi, fi):
    from oracle import oracle as O
    return bool(ok) and bool(O.lcp_valid(A, x, b, hi, lo, fi))


def classify():
    from oracle import oracle as O
    d = np.load(PROB)
    g = np.load(OUT)
    P = len(d["n"])
    rows = []
    keep = []
    tally = {"problems": P, "raw_gpu_vs_oracle_agree": 0, "raw_gpu_vs_ref_agree": 0, "raw_oracle_vs_ref_agree": 0,
             "eff_gpu_vs_ref_agree": 0, "eff_oracle_vs_ref_agree": 0, "eff_gpu_vs_ref_disagree_ambiguous": 0,
             "eff_gpu_vs_ref_disagree_unambiguous": 0, "both_valid_x_max_rel_err": 0.0,
             "raw_success_invalid_gpu": 0, "raw_success_invalid_ref": 0}
    for k in range(P):
        m = int(d["n"][k])
        A = d["A"][k, :m * m].reshape(m, m)
        b, lo, hi, fi = d["b"][k, :m], d["lo"][k, :m], d["hi"][k, :m], d["fi"][k, :m]
        gok, gx = bool(g[k, 0] > 0), g[k, X_D:X_D + m]
        ook, ox = O.dantzig(A, b, lo, hi, fi, True)
        rok, rx = O.ref_dantzig(A, b, lo, hi, fi, True)
        ge, oe, re_ = effective(gok, gx, A, b, lo, hi, fi), effective(ook, ox, A, b, lo, hi, fi), \
            effective(rok, rx, A, b, lo, hi, fi)
        tally["raw_gpu_vs_oracle_agree"] += int(gok == ook)
        tally["raw_gpu_vs_ref_agree"] += int(gok == rok)
        tally["raw_oracle_vs_ref_agree"] += int(ook == rok)
        tally["eff_gpu_vs_ref_agree"] += int(ge == re_)
        tally["eff_oracle_vs_ref_agree"] += int(oe == re_)
        tally["raw_success_invalid_gpu"] += int(gok and not ge)
        tally["raw_success_invalid_ref"] += int(rok and not re_)
        amb = None
        if not (ge == oe == re_):
            amb = ref_ambiguous(A, b, lo, hi, fi, seed=k)
        if ge != re_:
            tally["eff_gpu_vs_ref_disagree_ambiguous" if amb else "eff_gpu_vs_ref_disagree_unambiguous"] += 1
        xdiff = False
        if ge and re_:
            e = float(np.abs(gx - rx).max() / max(1.0, np.abs(rx).max()))
            tally["both_valid_x_max_rel_err"] = max(tally["both_valid_x_max_rel_err"], e)
            if e > 1e-9:
                # both solve the LCP: on a rank-deficient A the solution set is
                # not a point -- x_gpu - x_ref lies in A's null space
                xdiff = True
                tally["both_valid_x_differ"] = tally.get("both_valid_x_differ", 0) + 1
                res = float(np.abs(A @ (gx - rx)).max() / max(1.0, np.abs(A).max() * np.abs(rx).max()))
                tally["both_valid_x_differ_null_residual"] = max(tally.get("both_valid_x_differ_null_residual", 0.0), res)
        if not (gok == ook == rok) or not (ge == oe == re_) or xdiff:
            keep.append(k)
            rows.append({"problem": k, "m": m, "rank": int(np.linalg.matrix_rank(A)), "gpu_ok": gok, "gpu_valid": ge,
                         "oracle_ok": bool(ook), "oracle_valid": oe, "ref_ok": bool(rok), "ref_valid": re_,
                         "ref_ambiguous": amb})
    for key in list(tally):
        if key.endswith("_agree"):
            tally[key + "_frac"] = tally[key] / P
    out = {"source": "tools/dantzig_reconcile.py classify over dbg/lcp_problems.npz (tools/lcp_bench.py gen: the "
                     "bench Atlas, 1024 worlds x 3 steps, seed 1000) and the device run gpurun_out/lcp_out.npy",
           "effective_outcome": "dSolveLCP success AND LCPUtils::isLCPSolutionValid (what the step keeps)",
           "tally": tally, "kept": rows}
    os.makedirs(os.path.dirname(SUMMARY), exist_ok=True)
    json.dump(out, open(SUMMARY, "w"), indent=1)
    # the fixture: inputs of the kept problems and the reference's outcome
    ks = np.array(keep, dtype=np.int64)
    nmax = int(round(np.sqrt(d["A"].shape[1])))
    ref_x = np.zeros((len(ks), nmax))
    for i, k in enumerate(ks):
        m = int(d["n"][k])
        ref_x[i, :m] = O.ref_dantzig(d["A"][k, :m * m].reshape(m, m), d["b"][k, :m], d["lo"][k, :m],
                                     d["hi"][k, :m], d["fi"][k, :m], True)[1]
    np.savez_compressed(FIXTURE, problem=ks, n=d["n"][ks], A=d["A"][ks], b=d["b"][ks], lo=d["lo"][ks],
                        hi=d["hi"][ks], fi=d["fi"][ks], ref_x=ref_x,
                        ref_ok=np.array([r["ref_ok"] for r in rows], dtype=np.int32),
                        ref_valid=np.array([r["ref_valid"] for r in rows], dtype=np.int32),
                        ref_ambiguous=np.array([-1 if r["ref_ambiguous"] is None else int(r["ref_ambiguous"])
                                                for r in rows], dtype=np.int32))
    print(json.dumps(tally, indent=1))
    print(f"{len(keep)} problems kept -> {FIXTURE}")


if __name__ == "__main__":
    cmd = sys.argv[1] if len(sys.argv) > 1 else "classify"
    if cmd == "classify":
        classify()
