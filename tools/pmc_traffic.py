"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) for one kernel into
profiles/traffic_<tag>.json (+ traffic_latest.json, read by bench.py). Units: rocprofv3 reports
both counters in KB; bytes = value * 1024 (MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of a
wide coalesced stream on gfx950; other access widths are uncalibrated — reported raw)."""
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


def main(tag, fetch_csv, write_csv, workload, scale, kernel="dense_big_kernel"):
    f = per_dispatch(fetch_csv, kernel, "FETCH_SIZE")
    w = per_dispatch(write_csv, kernel, "WRITE_SIZE")
    fb = sum(f) / len(f) * 1024
    wb = sum(w) / len(w) * 1024
    out = {"workload": workload, "scale": float(scale), "kernel": kernel,
           "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
           "hbm_bytes_per_launch": fb + wb, "dispatches": [len(f), len(w)],
           "note": "raw (FETCH_SIZE+WRITE_SIZE)*1024 from separate --pmc passes; 8-byte sc1 "
                   "stores are counted as 64-byte write requests"}
    for name in (f"profiles/traffic_{tag}.json", "profiles/traffic_latest.json"):
        json.dump(out, open(name, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
