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
  python tools/dantzig_reconcile.py classify_wide [TAG]
      # the R = 2 (wide) Dantzig on the STL-mesh Atlas' > 64-row LCPs
      # (tools/lcp_bench.py gen_wide / run_wide: gpurun_out/lcp_wide_out.npy,
      # gpurun_out/lcp_wide_out_packed.npy with LCP_WIDE_PACKED=1)
      #   summary -> profiles/r06_dantzig_wide_reconcile.json
      #   fixture -> tests/golden/dantzig_wide_disagreements.npz

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


def classify(prob=PROB, outs=((None, OUT),), summary=SUMMARY, fixture=FIXTURE, limit=None, source=None):
    """Per problem: the device's, the oracle's and the reference's raw and
    effective outcomes; every problem on which they do not all agree (for
    any of the device runs in `outs`, (label, path) pairs) is kept, with the
    reference's outcome and its ambiguity."""
    from oracle import oracle as O
    d = np.load(prob)
    gs = [(lab, np.load(path)) for lab, path in outs]
    P = len(d["n"]) if limit is None else min(limit, len(d["n"]))
    out = {"source": source or ("tools/dantzig_reconcile.py classify over dbg/lcp_problems.npz (tools/lcp_bench.py "
                                "gen: the bench Atlas, 1024 worlds x 3 steps, seed 1000) and the device run "
                                "gpurun_out/lcp_out.npy"),
           "effective_outcome": "dSolveLCP success AND LCPUtils::isLCPSolutionValid (what the step keeps)"}
    keep = set()
    refs = {}
    for lab, g in gs:
        tally, rows = _classify_run(O, d, g, P, refs)
        out["tally" if lab is None else f"tally_{lab}"] = tally
        out["kept" if lab is None else f"kept_{lab}"] = rows
        keep |= {r["problem"] for r in rows}
        print(lab, json.dumps(tally, indent=1))
    os.makedirs(os.path.dirname(summary), exist_ok=True)
    json.dump(out, open(summary, "w"), indent=1)
    _write_fixture(O, d, sorted(keep), refs, fixture)
    print(f"{len(keep)} problems kept -> {fixture}")


def _ref_outcome(O, d, k, refs):
    """(raw ok, x, effective, ambiguous-or-None) of the reference's dSolveLCP on problem k (cached)."""
    if k not in refs:
        m = int(d["n"][k])
        A = d["A"][k, :m * m].reshape(m, m)
        b, lo, hi, fi = d["b"][k, :m], d["lo"][k, :m], d["hi"][k, :m], d["fi"][k, :m]
        rok, rx = O.ref_dantzig(A, b, lo, hi, fi, True)
        refs[k] = [bool(rok), rx, effective(rok, rx, A, b, lo, hi, fi), None]
    return refs[k]


def _classify_run(O, d, g, P, refs):
    rows = []
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
        ref = _ref_outcome(O, d, k, refs)
        rok, rx, re_ = ref[0], ref[1], ref[2]
        ge, oe = effective(gok, gx, A, b, lo, hi, fi), effective(ook, ox, A, b, lo, hi, fi)
        tally["raw_gpu_vs_oracle_agree"] += int(gok == ook)
        tally["raw_gpu_vs_ref_agree"] += int(gok == rok)
        tally["raw_oracle_vs_ref_agree"] += int(ook == rok)
        tally["eff_gpu_vs_ref_agree"] += int(ge == re_)
        tally["eff_oracle_vs_ref_agree"] += int(oe == re_)
        tally["raw_success_invalid_gpu"] += int(gok and not ge)
        tally["raw_success_invalid_ref"] += int(rok and not re_)
        amb = None
        if not (ge == oe == re_):
            if ref[3] is None:
                ref[3] = ref_ambiguous(A, b, lo, hi, fi, seed=k)
            amb = ref[3]
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
            rows.append({"problem": k, "m": m, "rank": int(np.linalg.matrix_rank(A)), "gpu_ok": gok, "gpu_valid": ge,
                         "oracle_ok": bool(ook), "oracle_valid": oe, "ref_ok": bool(rok), "ref_valid": re_,
                         "ref_ambiguous": amb})
    for key in list(tally):
        if key.endswith("_agree"):
            tally[key + "_frac"] = tally[key] / P
    return tally, rows


def _write_fixture(O, d, keep, refs, fixture):
    """The fixture: inputs of the kept problems (A cut to the largest kept
    row count) and the reference's outcome."""
    ks = np.array(keep, dtype=np.int64)
    nmax = int(round(np.sqrt(d["A"].shape[1])))
    nk = int(d["n"][ks].max()) if len(ks) else 1
    A = np.zeros((len(ks), nk * nk))
    ref_x = np.zeros((len(ks), nk))
    amb = np.zeros(len(ks), dtype=np.int32)
    for i, k in enumerate(ks):
        m = int(d["n"][k])
        A[i, :m * m] = d["A"][k, :m * m]
        r = _ref_outcome(O, d, k, refs)
        ref_x[i, :m] = r[1]
        amb[i] = -1 if r[3] is None else int(r[3])
    vec = {key: d[key][ks][:, :nk] for key in ("b", "lo", "hi", "fi")}
    np.savez_compressed(fixture, problem=ks, n=d["n"][ks], A=A, ref_x=ref_x, **vec,
                        ref_ok=np.array([int(refs[k][0]) for k in ks], dtype=np.int32),
                        ref_valid=np.array([int(refs[k][2]) for k in ks], dtype=np.int32),
                        ref_ambiguous=amb, nmax_source=np.int32(nmax))


PROB_WIDE = os.path.join(ROOT, "dbg", "lcp_wide.npz")
SUMMARY_WIDE = os.path.join(ROOT, "profiles", "r06_dantzig_wide_reconcile.json")
FIXTURE_WIDE = os.path.join(ROOT, "tests", "golden", "dantzig_wide_disagreements.npz")


def classify_wide(tag="r06"):
    outs = [("stage_unpacked", os.path.join(ROOT, "gpurun_out", "lcp_wide_out.npy")),
            ("stage_packed", os.path.join(ROOT, "gpurun_out", "lcp_wide_out_packed.npy"))]
    outs = [(lab, p) for lab, p in outs if os.path.exists(p)]
    classify(PROB_WIDE, outs, SUMMARY_WIDE.replace("r06", tag), FIXTURE_WIDE, limit=512,
             source="tools/dantzig_reconcile.py classify_wide over the first 512 problems of dbg/lcp_wide.npz "
                    "(tools/lcp_bench.py gen_wide: the STL-mesh Atlas' LCPs of more than 64 rows, 1024 worlds x 2 "
                    "steps, seed 1000) and the device runs of the R = 2 Dantzig (tools/lcp_bench.hip "
                    "lcp_bench_wide_kernel, L unpacked / in the wide forward kernel's packed panels)")


if __name__ == "__main__":
    cmd = sys.argv[1] if len(sys.argv) > 1 else "classify"
    if cmd == "classify":
        classify()
    elif cmd == "classify_wide":
        classify_wide(*sys.argv[2:3])
