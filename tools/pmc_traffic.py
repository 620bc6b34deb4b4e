"""Summarise rocprofv3 PMC passes for one kernel into profiles/traffic_<tag>.json (and
traffic_latest.json, which bench.py reads). Each counter set comes from a run of its own.

HBM traffic (MI355X_MICROARCH.md §HBM): rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KB
(bytes = value * 1024). On gfx950 FETCH_SIZE counts exactly half the bytes of a wide
coalesced streaming read, so the guide's correction doubles it; WRITE_SIZE is exact for
16-B-per-lane streaming stores. Our kernels' accesses are 4-8 B wide (uncalibrated widths):
both the raw and the corrected sums are kept, `hbm_bytes_per_launch` is the corrected one.

usage: pmc_traffic.py <tag> <fetch.csv> <write.csv> <workload> <scale> [kernel] [sq.csv]
"""
import csv
import json
import sys


def per_dispatch(path, kernel, counter):
    vals = []
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    return vals


def mean(v):
    return sum(v) / len(v) if v else None


def main(tag, fetch_csv, write_csv, workload, scale, kernel="dense_big_kernel", sq_csv=None):
    f = per_dispatch(fetch_csv, kernel, "FETCH_SIZE")
    w = per_dispatch(write_csv, kernel, "WRITE_SIZE")
    fb = mean(f) * 1024
    wb = mean(w) * 1024
    out = {"workload": workload, "scale": float(scale), "kernel": kernel,
           "fetch_bytes_per_launch_raw": fb, "write_bytes_per_launch": wb,
           "hbm_bytes_per_launch_raw": fb + wb,
           "hbm_bytes_per_launch": 2 * fb + wb, "dispatches": [len(f), len(w)],
           "note": "hbm = 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024; MI355X_MICROARCH.md §HBM "
                   "gfx950 correction for streaming reads); separate --pmc passes"}
    if sq_csv:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES", "SQ_BUSY_CYCLES",
                  "SQ_WAVE_CYCLES"):
            v = mean(per_dispatch(sq_csv, kernel, c))
            if v is not None:
                out[c.lower() + "_per_launch"] = v
        if "sq_insts_valu_per_launch" in out:
            out["valu_insts_per_launch"] = out["sq_insts_valu_per_launch"]
    # the headline (C3) keeps profiles/traffic_latest.json; other workloads get one file each
    latest = "profiles/traffic_latest.json" if workload == "c3" else f"profiles/traffic_latest_{workload}.json"
    for name in (f"profiles/traffic_{tag}.json", latest):
        json.dump(out, open(name, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
