import json, sys
for f in sys.argv[1:]:
    print("==", f)
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print(" value %.4g ops/s  ms/step %.1f  kernel_ms %.1f  cfg/s %.4g  verdicts %s" % (
                d["value"], d["ms_per_step"], d["kernel_ms_per_step"], d["configs_explored_per_s"], d["verdicts"]))
            print(" roofline", {k: d["roofline"][k] for k in ("achieved", "frac", "traffic", "grid_phases", "ret_steps", "candidates", "spill_inserts")})
            if d.get("cpu_baseline"): print(" cpu", d["cpu_baseline"], "parity", d.get("parity_sample"))
        else:
            print(" ", line.rstrip()[:300])
