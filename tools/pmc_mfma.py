"""Summarise the rocprofv3 fp64 MFMA PMC pass (tools/gpu_measure.sh:
SQ_INSTS_VALU_MFMA_F64, SQ_INSTS_VALU_MFMA_MOPS_F64, SQ_VALU_MFMA_BUSY_CYCLES,
GRBM_GUI_ACTIVE) into profiles/pmc_mfma.json: per launch of each nimble
kernel, the fp64 MFMA instructions, their FLOPs (MOPS x 512, rocprofv3's
MfmaFlopsF64) and the MFMA utilisation rocprofv3 defines as MfmaUtil =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x SIMDs) (256 CUs x 4 SIMDs).

  python tools/pmc_mfma.py <pmc_dir> [workload] [out.json]
"""
import csv
import collections
import glob
import json
import os
import sys

SIMDS = 256 * 4
# rocprofv3 reports GRBM_GUI_ACTIVE summed over the 8 XCDs (6.75M for a
# 349.5 us launch = 8 x 2.4 GHz); MfmaUtil takes the per-XCD (max) value
XCDS = 8
PEAK_FP64_MFMA_TFLOPS = 78.6  # MI355X dense fp64 matrix rate (MI355X_MICROARCH.md)


def main():
    d = sys.argv[1]
    wl = sys.argv[2] if len(sys.argv) > 2 else "atlas"
    out = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_mfma.json"
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    dur = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if not k.startswith("nimble_"):
                continue
            per[k][r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[(k, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    res = {}
    for k, disp in per.items():
        n = len(disp)
        mean = lambda c: sum(v.get(c, 0.0) for v in disp.values()) / n  # noqa: E731
        ns = sum(dur[(k, i)] for i in disp) / n
        gui = mean("GRBM_GUI_ACTIVE")
        busy = mean("SQ_VALU_MFMA_BUSY_CYCLES")
        flops = mean("SQ_INSTS_VALU_MFMA_MOPS_F64") * 512
        e = {"launches": n, "mfma_f64_insts": mean("SQ_INSTS_VALU_MFMA_F64"), "mfma_f64_flops": flops,
             "mfma_busy_cycles": busy, "duration_ns": ns,
             "mfma_tflops": flops / (ns * 1e-9) / 1e12 if ns else None}
        e["mfma_frac_of_fp64_matrix_peak"] = e["mfma_tflops"] / PEAK_FP64_MFMA_TFLOPS if ns else None
        if gui > 0:
            e["grbm_gui_active_per_xcd"] = gui / XCDS
            e["mfma_util"] = busy / (gui / XCDS * SIMDS)
        res[k] = e
    allw = json.load(open(out)) if os.path.exists(out) else {}
    allw[wl] = res
    json.dump(allw, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
