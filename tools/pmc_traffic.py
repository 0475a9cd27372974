"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate passes as
gfx950's TCC slots require) into profiles/pmc_traffic.json: HBM-side bytes
per launch and per world for each nimble kernel.

  python tools/pmc_traffic.py <fetch_dir> <write_dir> <worlds_per_launch> [workload] [out.json]

The summary is stored under the workload's key (bench.py --workload).

FETCH_SIZE/WRITE_SIZE are reported by rocprofv3 in KiB.  Per
MI355X_MICROARCH.md (HBM section) FETCH_SIZE counts half of the bytes of wide
coalesced streaming reads on gfx950.  The per-world rows this path reads are
8-byte-per-lane wave-contiguous accesses; tools/micro/bytes_calib.hip
calibrates that width on a 512 MiB buffer (profiles/r02c_calib_*.csv):
FETCH_SIZE = exactly 1/2 of the bytes for 8 B/lane reads as for 16 B/lane,
WRITE_SIZE = exactly the bytes for 8 B/lane stores.  So `bytes_per_world`
= 2 x FETCH_SIZE + WRITE_SIZE."""
import csv
import glob
import json
import os
import sys


def load(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") == counter:
                    rows.append((r["Kernel_Name"], float(r["Counter_Value"])))
    return rows


def main():
    fdir, wdir, worlds = sys.argv[1], sys.argv[2], int(sys.argv[3])
    wl = sys.argv[4] if len(sys.argv) > 4 else "atlas"
    out = sys.argv[5] if len(sys.argv) > 5 else "profiles/pmc_traffic.json"
    res = {}
    for k in ("nimble_forward_kernel", "nimble_forward_mesh_kernel", "nimble_backward_kernel",
              "nimble_forward_wide_kernel", "nimble_backward_wide_kernel"):
        fe = [v for n, v in load(fdir, "FETCH_SIZE") if k in n]
        wr = [v for n, v in load(wdir, "WRITE_SIZE") if k in n]
        if not fe or not wr:
            continue
        fkb = sum(fe) / len(fe)
        wkb = sum(wr) / len(wr)
        per_launch = 2.0 * fkb * 1024 + wkb * 1024
        res[k] = {"fetch_kib_raw": fkb, "write_kib": wkb, "launches": len(fe),
                  "bytes_per_launch": per_launch, "bytes_per_world": per_launch / worlds,
                  "worlds_per_launch": worlds, "fetch_correction": "x2 (gfx950 FETCH_SIZE)"}
    allw = json.load(open(out)) if os.path.exists(out) else {}
    allw[wl] = res
    json.dump(allw, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
