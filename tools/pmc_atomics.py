"""Atomic throughput of the partitioned-frontier kernels (BASELINE north_star:
"atomic throughput ... from rocprof"). Joins a rocprofv3 --pmc pass (TCC_ATOMIC_sum: atomic
requests the L2 served, TCC_EA0_ATOMIC_sum: those sent on to memory, TCP_TCC_ATOMIC_*_REQ_sum:
atomic requests from the CUs, with / without return) with a --kernel-trace pass of the same
command (durations), per kernel name.

usage: pmc_atomics.py <tag> <counter_collection.csv> <kernel_trace.csv> [kernel-substring ...]
writes profiles/<tag>/atomics.json
"""
import csv
import json
import os
import sys
from collections import defaultdict


def main(tag, pmc_csv, trace_csv, *kernels):
    kernels = kernels or ("part_flow_kernel", "part_step_kernel", "part_absorb", "part_expand")
    cnt = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    with open(pmc_csv) as fh:
        for row in csv.DictReader(fh):
            for k in kernels:
                if k in row["Kernel_Name"]:
                    cnt[k][row["Counter_Name"]] += float(row["Counter_Value"])
                    disp[k].add(row["Dispatch_Id"])
    dur = defaultdict(float)
    ndur = defaultdict(int)
    with open(trace_csv) as fh:
        for row in csv.DictReader(fh):
            for k in kernels:
                if k in row["Kernel_Name"]:
                    dur[k] += (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
                    ndur[k] += 1
    out = {"note": "counters summed over every dispatch of the PMC run; durations from the kernel-trace "
                   "run of the same command; rate = TCC_ATOMIC_sum / total kernel time (atomic requests "
                   "per second the L2 served)"}
    for k in kernels:
        c = dict(cnt[k])
        t = dur[k] if ndur[k] == len(disp[k]) or not disp[k] else dur[k] * len(disp[k]) / max(1, ndur[k])
        out[k] = {"dispatches": len(disp[k]), "kernel_s": t, "counters": c,
                  "tcc_atomics_per_s": c.get("TCC_ATOMIC_sum", 0.0) / t if t > 0 else None,
                  "cu_atomic_requests_per_s": (c.get("TCP_TCC_ATOMIC_WITH_RET_REQ_sum", 0.0) +
                                               c.get("TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum", 0.0)) / t
                  if t > 0 else None}
    os.makedirs(f"profiles/{tag}", exist_ok=True)
    json.dump(out, open(f"profiles/{tag}/atomics.json", "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
