#!/usr/bin/env python3
"""Benchmark of the MI355X linearizability checker (BASELINE.json metric: history ops
verified/sec + configs explored/sec, % of the HBM roofline).

One "step" = one full check of the workload's histories by the HIP search (lc_plan_run on
HBM-resident encoded histories). Default workload: C3 (jepsen.independent cas-register,
1k keys x 1k ops, 5 clients/key, p_info 0.01), the north_star's headline config; under
`torchrun --nproc-per-node N` the 1k keys are split over the ranks (strong scaling, as
BASELINE configs[2] says; no data-path collective: keys are independent, SURVEY §8(e) axis
1). `end_to_end` times lc_check from host arrays (encode + H2D + search + D2H).

Prints ONE JSON line on rank 0 (driver contract) with `roofline` and `cpu_baseline`.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "jepsen-jgroups-raft_amd"))

from lincheck import _lib, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak (spec)
# MI355X_MICROARCH.md §LDS: ds_read_b64 moves 256 B/clk/CU; 256 CUs at 2.4 GHz
LDS_PEAK_GBS = 256 * 256 * 2.4
MODEL_OF = {"c1": "cas-register", "c2": "cas-register", "c3": "cas-register",
            "c4": "cas-register", "c5": "counter", "c2c": "counter", "c5x": "counter"}


# one process per GPU over RCCL ("nccl"); LC_BENCH_BACKEND=gloo and LC_BENCH_DEVICE=<index> are
# test hooks that run several ranks on one GPU (the rank protocol, not the interconnect)
BACKEND = os.environ.get("LC_BENCH_BACKEND", "nccl")


def gpu_index() -> int:
    d = os.environ.get("LC_BENCH_DEVICE")
    return int(d) if d is not None else int(os.environ.get("LOCAL_RANK", 0))


def coll_device() -> str:
    return "cuda" if BACKEND == "nccl" else "cpu"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(h, model: str, budget_s: float, threads: int, full: bool = True, reps: int = 1):
    """Time the CPU oracle (a C restatement of knossos.linear, test infrastructure) on the
    same workload in the same run; returns (cpu dict, oracle results, checked keys, checked
    history).

    Many keys (r4): EVERY key by default — the whole workload, checked by
    `threads` POSIX threads that take keys in key order from a shared counter (dynamic
    scheduling), as Knossos would check them; on C3 that is ~50 s on the GPU box's 16 threads
    (~200 s of CPU work; the wall is the slowest key's single-thread search plus the work
    dequeued before it). The work is a fixed set of deterministic searches, so two runs differ
    only by the machine. `value` is the wall figure; `per_key_sum` beside it is the throughput
    if the per-key times packed perfectly onto the threads (sum / threads). full=False: every
    20th key (a quick sample whose wall is one key's time; not a baseline to quote). One
    history: the longest prefix that fits the budget (the oracle is single-threaded per
    history, as Knossos is)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402  (bench cpu_baseline leg only)
    n = h.n_hist
    if n > 1:
        stride = max(1, n // 50)
        sample = list(range(n)) if full else list(range(0, n, stride))
        hs = h.select(sample)
        walls = []
        for rep in range(max(1, reps)):  # the same deterministic searches: keep the fastest pass
            t0 = time.perf_counter()
            r_rep = oracle.check_many(model, hs, n_threads=threads)
            walls.append(time.perf_counter() - t0)
            log(f"[cpu baseline] pass {rep}: {walls[-1]:.2f}s")
            if walls[-1] == min(walls):
                res = r_rep
        wall = min(walls)
        per = np.array([r["wall_ns"] for r in res], np.float64) / 1e9
        desc = (f"the whole workload: all {n} keys" if full or stride == 1 else
                f"every {stride}th key ({len(sample)} of {n}: 0, {stride}, ...; a quick sample)") + \
            f", {threads} threads taking keys in key order from a shared counter" + \
            (f"; the fastest of {len(walls)} passes" if len(walls) > 1 else "")
        used = threads
        keys = {"min_s": round(float(per.min()), 5), "median_s": round(float(np.median(per)), 5),
                "max_s": round(float(per.max()), 4), "sum_s": round(float(per.sum()), 4),
                "slowest_key": int(sample[int(per.argmax())]),
                "ops_per_s_if_perfectly_packed": ops_of(hs) / max(float(per.sum()) / threads, 1e-9),
                "wall_bound_s": round(max(float(per.sum()) / threads, float(per.max())), 3)}
    else:
        # one history: the oracle is single-threaded like Knossos's per-history search;
        # time the longest prefix that fits the budget, growing from a short one (a wide
        # history's search cost grows much faster than its length)
        m = min(h.n, 2000)
        while True:
            hs = synth.truncate(h, m) if m < h.n else h
            t0 = time.perf_counter()
            res = oracle.check_many(model, hs, n_threads=1, max_configs=0)
            wall = time.perf_counter() - t0
            log(f"[cpu baseline] prefix of {m} entries: {wall:.2f}s")
            if m >= h.n or wall >= budget_s / 4:
                break
            m = min(h.n, int(m * min(4.0, max(1.5, budget_s / 4 / max(wall, 1e-3)))))
        sample = [0]
        desc = f"first {hs.n} of {h.n} entries of the single history, 1 thread"
        used = 1
        keys = None
    ops = hs.n_ops()
    out = {"value": ops / wall, "unit": "history ops/s", "cores": used, "kind": "port",
           "sample": desc, "wall_s": round(wall, 3),
           "configs_per_s": sum(r["explored"] for r in res) / wall}
    if keys is not None:
        # the sample's wall is max(sum / threads, slowest key): a key's search is one thread
        out["per_key"] = keys
        out["pass_walls_s"] = [round(w, 3) for w in walls]
    return out, res, sample, hs


def golden_fixture(workload):
    """The oracle-pinned whole-history fixture of a single-history workload, if committed."""
    name = {"c4": "c4_oracle.json"}.get(workload, f"counter_{workload}_oracle.json")
    path = os.path.join(ROOT, "tests", "golden", name)
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        return json.load(fh)


def ops_of(h):
    return h.n_ops()


def bench_c5(args, rank, world, dist, barrier_sync):
    """C5: the counter bounds scan (BASELINE configs[4]) over one 1M-op history. The history's
    entries are split over the ranks (strong scaling); each step is ONE exchange of five int64
    sums per rank (all-gather over RCCL) + the rank's scan + an all-reduce MIN of the verdict
    (SURVEY §8(e) axis 3). Inputs are HBM-resident (lc_bounds_plan)."""
    from lincheck import shard
    tdist = dist[1] if dist else None
    h = synth.gen_config("c5", scale=args.scale)
    n = int(h.off[1] - h.off[0])
    own = shard.bounds_shard(n, rank, world)
    t0 = time.perf_counter()
    plan = _lib.BoundsPlan(0, h, own=own, device=gpu_index())
    log(f"[rank {rank}] c5: {n} entries, {h.n_ops()} ops, shard {own}; "
        f"plan {time.perf_counter() - t0:.2f}s")

    def step():
        excl = shard.exclusive_sums(plan.sums(), tdist) if world > 1 else None
        ok, bad, ms = plan.run(excl)
        return shard.first_bad(bad, tdist), ms

    for _ in range(args.warmup):
        step()
    barrier_sync()
    kms = 0.0
    bad = -1
    t0 = time.perf_counter()
    for _ in range(args.steps):
        bad, ms = step()
        kms += ms
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if dist:
        torch, td = dist
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_device())
        td.all_reduce(t, op=td.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank != 0:
        plan.close()
        return None
    # algorithmic HBM bytes of rank 0's scan per step: the two delta arrays
    # read by the reduce (16 B/entry) and by the prefix pass (16 B + the 4-B observation map),
    # per observation its five prefixes written (40 B) and read back with its record (40 + 32
    # B); plus the block-sum pass before the exchange when sharded (16 B/entry)
    n_own = own[1] - own[0]
    is_obs = (h.type == 1) & (((h.f == 0) & (h.vflags == 1)) |
                              (((h.f == 5) | (h.f == 6)) & (h.vflags == 2)))
    n_obs = int(is_obs[own[0]:own[1]].sum())
    alg = 36 * n_own + 112 * n_obs + (16 * n_own if world > 1 else 0)
    k_s = kms / args.steps / 1e3
    achieved = alg / k_s / 1e9 if k_s > 0 else 0.0
    traffic = None
    if os.path.exists(args.traffic):
        try:
            tr = json.load(open(args.traffic))
            if tr.get("workload") == "c5" and abs(tr.get("scale", 1.0) - args.scale) < 1e-9:
                traffic = tr.get("hbm_bytes_per_launch")
        except Exception:  # noqa: BLE001
            traffic = None
    cpu = None
    if not args.no_cpu and world == 1:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # noqa: E402  (bench cpu_baseline leg only)
        reps, t0 = 0, time.perf_counter()
        while True:
            eok, ebad = oracle.counter_bounds(h)
            reps += 1
            if time.perf_counter() - t0 > min(args.cpu_budget, 10.0):
                break
        wall = (time.perf_counter() - t0) / reps
        cpu = {"value": h.n_ops() / wall, "unit": "history ops/s", "cores": 1, "kind": "port",
               "sample": f"the whole {h.n_ops()}-op history, {reps} scan(s), 1 thread",
               "wall_s": round(wall, 4),
               "parity": {"ok": bool(eok) == (bad < 0), "bad_idx": int(ebad) == bad}}
    out = {
        "metric": "history ops verified/sec (+ configs explored/sec, % HBM roofline)",
        "value": h.n_ops() * args.steps / elapsed,
        "unit": "history ops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (simulated linearizable counter SUT, SURVEY §8(d) seeds)",
        "config": {"workload": "c5: counter 1M ops, 16 clients, p_info 0.01: bounds prefix scan",
                   "ops": h.n_ops(), "entries": n, "scale": args.scale,
                   "parallelism": f"entries split over {world} GPU(s), one 5 x int64 all-gather "
                                  "per step"},
        "verdict": {"bounds_ok": bad < 0, "bad_idx": bad},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "lc::bounds_{reduce,scan_partials,prefix,check}",
                     "kernel_ms": k_s * 1e3, "alg_bytes_per_launch": alg},
        "cpu_baseline": cpu,
    }
    plan.close()
    return out


def bench_partition(args, rank, world, dist, barrier_sync):
    """Axis 2: ONE cas-register history (c2 or c4) searched by all ranks at once,
    its frontier partitioned by config hash, one all-to-all of candidates per BFS level (RCCL
    over xGMI). Strong scaling: every rank works on the same history."""
    from lincheck import partition
    tdist = dist[1] if dist else None
    h = synth.gen_config(args.workload, scale=args.scale)
    local = gpu_index()
    if args.in_process:
        return bench_part_check(args, h, world)
    # per-rank lists of 2^cap configs; C4's widest closures need 2^25 on one rank
    cap = args.capacity_log2 or (25 if args.workload == "c4" else 22)
    runs = []
    for i in range(args.warmup + args.steps):
        if i == args.warmup:
            barrier_sync()
            t0 = time.perf_counter()
        r = partition.check_partitioned(h, tdist=tdist, device_index=local, capacity_log2=cap,
                                        device_loop=not args.level_protocol)
        if i >= args.warmup:
            runs.append(r)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if dist:
        torch, td = dist
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_device())
        td.all_reduce(t, op=td.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank != 0:
        return None
    r = runs[-1]
    dev_loop = world == 1 and not args.level_protocol
    k_s = sum(x["kernel_ms"] for x in runs) / len(runs) / 1e3
    achieved = r["alg_bytes"] / k_s / 1e9 if k_s > 0 else 0.0
    return {
        "metric": "history ops verified/sec (+ configs explored/sec, % HBM roofline)",
        "value": h.n_ops() * args.steps / elapsed,
        "unit": "history ops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (simulated linearizable SUT, SURVEY §8(d) seeds)",
        "config": {"workload": f"{args.workload}: one register history, frontier partitioned "
                               f"by config hash over {world} rank(s)",
                   "ops": h.n_ops(), "scale": args.scale,
                   "parallelism": f"axis 2: {world} GPU(s), " + (
                       "device-resident level loop (lc_part_run)" if dev_loop else
                       "one all-to-all per BFS level")},
        "configs_explored_per_s": r["explored"] * args.steps / elapsed,
        "verdict": {"valid": r["valid"], "explored": r["explored"], "steps": r["steps"],
                    "levels": r["levels"], "exchanged_bytes": r["exchanged_bytes"]},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": "lc::part_step_kernel" if dev_loop else
                               "lc::part_expand + lc::part_absorb (rank 0)",
                     "kernel_ms": k_s * 1e3, "alg_bytes_per_launch": r["alg_bytes"],
                     "note": "per check (all levels); " + (
                         "GPU time from the first step's launch to the last one's end" if dev_loop
                         else "the wall time is dominated by the per-level host round trip "
                              "(count exchange + all-to-all), see DESIGN.md §6")},
        "cpu_baseline": None,
    }


def bench_part_check(args, h, world):
    """Axis 2 through lc_part_check: ONE history, its frontier partitioned over --in-process N
    ranks that are threads of this process (rank r on device r mod visible devices; on a 1-GPU
    box they share it: this measures the in-process exchange, not xGMI)."""
    n = args.in_process
    cap = args.capacity_log2 or (25 if args.workload == "c4" else 22)
    times, g = [], None
    for i in range(args.warmup + args.steps):
        t0 = time.perf_counter()
        g = _lib.part_check(h, n_ranks=n, capacity_log2=cap)
        if i >= args.warmup:
            times.append(time.perf_counter() - t0)
    el = sum(times)
    return {
        "metric": "history ops verified/sec (+ configs explored/sec, % HBM roofline)",
        "value": h.n_ops() * args.steps / el, "unit": "history ops/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (simulated linearizable SUT, SURVEY §8(d) seeds)",
        "config": {"workload": f"{args.workload}: one register history, frontier partitioned by "
                               f"config hash over {n} in-process rank(s) (lc_part_check)",
                   "ops": h.n_ops(), "scale": args.scale,
                   "parallelism": f"axis 2: {n} rank threads, peer copies; "
                                  f"{lc_devices()} visible device(s)"},
        "configs_explored_per_s": int(g["explored"][0]) * args.steps / el,
        "verdict": {"valid": int(g["valid"][0]), "explored": int(g["explored"][0]),
                    "err": int(g["err"][0])},
        "roofline": None, "cpu_baseline": None}


def lc_devices():
    return int(_lib.load().lc_device_count())


def cpu_info():
    """Host CPU facts for cpu_baseline: model name, nproc, the affinity set, and the thread
    count used = the box's CPU share per GPU (OMP_NUM_THREADS, 16 on the GPU box) or, when
    unset, every CPU this process may run on."""
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    omp = os.environ.get("OMP_NUM_THREADS", "")
    threads = min(aff, int(omp)) if omp.isdigit() and int(omp) > 0 else aff
    return {"cpu_model": model, "nproc": nproc, "affinity": aff, "threads": max(1, threads),
            "share": "OMP_NUM_THREADS" if omp.isdigit() else "affinity"}


def read_profile(path, workload, scale, kname):
    """Per-launch PMC figures committed under profiles/ (tools/pmc_traffic.py) for this
    workload and kernel, or None."""
    if not os.path.exists(path):
        return None
    try:
        tr = json.load(open(path))
    except Exception:  # noqa: BLE001
        return None
    if tr.get("workload") != workload or abs(tr.get("scale", 1.0) - scale) > 1e-9:
        return None
    if tr.get("kernel", "") not in kname:
        return None
    return tr


def spawn_ranks(n: int) -> int:
    """Run this same command as n ranks under torch.distributed.run (127.0.0.1, a free port) and
    relay rank 0's JSON line; returns the launcher's exit code. The parent never touches the GPU."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] --gpus {n}: launching {n} ranks: {' '.join(cmd)}")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=dict(os.environ))
    n_json = 0
    for line in p.stdout:  # rank 0 prints the one JSON line; anything else goes to stderr
        if line.startswith("{"):
            n_json += 1
            print(line, end="", flush=True)
        else:
            log(line.rstrip("\n"))
    rc = p.wait()
    if rc == 0 and n_json != 1:
        log(f"[bench] expected one JSON line from rank 0, got {n_json}")
        return 1
    return rc


def protocol_only(args, rank, world, dist):
    """The rank protocol without GPU work: warmup, barrier, K timed no-op steps, barrier, MAX of
    the elapsed time over ranks, one JSON line from rank 0 (LC_BENCH_PROTOCOL_ONLY test hook)."""
    def barrier():
        if dist:
            dist[1].barrier()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        torch, td = dist
        t = torch.tensor([elapsed], dtype=torch.float64)
        td.all_reduce(t, op=td.ReduceOp.MAX)
        elapsed = float(t.item())
        r = torch.tensor([1], dtype=torch.int64)
        td.all_reduce(r)
        ranks_seen = int(r.item())
    else:
        ranks_seen = 1
    if rank == 0:
        print(json.dumps({"metric": "protocol-only (test hook)", "value": 0.0, "n_gpus": world,
                          "ranks_seen": ranks_seen, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": elapsed / max(1, args.steps) * 1e3}), flush=True)
    if dist:
        dist[1].destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--workload", default="c3", choices=sorted(MODEL_OF))
    ap.add_argument("--scale", type=float, default=1.0, help="shrink the workload (tests)")
    ap.add_argument("--cpu-budget", type=float, default=6.0,
                    help="CPU baseline sizing (the 16-key probe underestimates the sample ~2.5x: ~15 s)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-sample", action="store_true",
                    help="cpu_baseline on every 20th key only (quick; the default is every key)")
    ap.add_argument("--cpu-reps", type=int, default=2,
                    help="whole-workload CPU passes; the fastest is quoted (r4u: one pass of two "
                         "ran 31 %% slow, its slowest key 53 s against 39 s in every other pass)")
    ap.add_argument("--e2e-reps", type=int, default=5,
                    help="lc_check calls from host arrays timed after the run (0: skip)")
    ap.add_argument("--e2e-shards", type=int, default=8,
                    help="also time lc_check(n_gpus=S) from host arrays (0/1: skip)")
    ap.add_argument("--emulate", default="",
                    help="r/N: check rank r's share of an N-rank split on this one GPU")
    ap.add_argument("--partition", action="store_true",
                    help="axis 2: one history (c2/c4) with its frontier partitioned over ranks")
    ap.add_argument("--capacity-log2", type=int, default=0, help="--partition: per-rank capacity")
    ap.add_argument("--in-process", type=int, default=0,
                    help="--partition: N ranks as threads of this process (lc_part_check)")
    ap.add_argument("--level-protocol", action="store_true",
                    help="--partition at 1 GPU: the host-driven level protocol, not lc_part_run")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="per-launch HBM bytes measured by rocprofv3 PMC passes (or absent)")
    args = ap.parse_args()
    if os.environ.get("LC_MAPS_DUMP"):
        # diagnosis of exit-time faults: the process's mappings as the interpreter exits (before
        # the C exit handlers run), so a faulting PC can be mapped to a library and offset
        import atexit
        import shutil
        atexit.register(lambda: shutil.copy("/proc/self/maps", os.environ["LC_MAPS_DUMP"]))

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python3 bench.py --gpus N` (the driver's scaling command) launches its N ranks itself:
        # one child process per GPU under torch.distributed.run, started before this process
        # makes any HIP call (never an exec); rank 0's JSON line is relayed
        raise SystemExit(spawn_ranks(args.gpus))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to "
                         "report a different GPU count than was asked for")
    global BACKEND
    local = gpu_index()
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        if os.environ.get("LC_BENCH_PROTOCOL_ONLY"):
            BACKEND = "gloo"
        else:
            ndev = torch.cuda.device_count()
            if ndev < 1:
                raise SystemExit("bench.py: no GPU visible")
            if "LC_BENCH_DEVICE" not in os.environ and ndev < world:
                # more ranks than GPUs (a 1-GPU box): ranks share devices, which RCCL refuses,
                # so the bench's own collectives (MAX of the time, SUM of explored) go over gloo
                local = local % ndev
                os.environ["LC_BENCH_DEVICE"] = str(local)
                BACKEND = "gloo"
            torch.cuda.set_device(local)
        tdist.init_process_group(BACKEND)
        dist = (torch, tdist)
    if os.environ.get("LC_BENCH_PROTOCOL_ONLY"):
        # test hook (tests/test_bench_cpu.py): the launch / barrier / max-over-ranks protocol of
        # this script with no GPU work, so the rank launcher is testable on a CPU-only host
        return protocol_only(args, rank, world, dist)

    def barrier_sync():
        if dist:
            dist[0].cuda.synchronize()
            dist[1].barrier()
            dist[0].cuda.synchronize()

    if args.workload == "c5" or args.partition:
        if args.partition and args.workload not in ("c2", "c4"):
            raise SystemExit("--partition runs one history: --workload c2 or c4")
        out = (bench_partition if args.partition else bench_c5)(args, rank, world, dist, barrier_sync)
        if out is not None:
            print(json.dumps(out), flush=True)
        if dist:
            dist[1].destroy_process_group()
        return

    model = MODEL_OF[args.workload]
    kind = _lib.MODEL_KIND[model]
    cfg = synth.CONFIGS[args.workload]
    # strong scaling (BASELINE configs[2]: 1k keys sharded across the GPUs): every rank builds
    # the same key set and keeps its share of lc_shard_histories' LPT split, the split
    # lc_check(n_gpus) uses; keys are independent, so no data-path collective
    t0 = time.perf_counter()
    h_all = synth.gen_config(args.workload, scale=args.scale)
    shard_rank, shard_world = rank, world
    if args.emulate:
        shard_rank, shard_world = (int(x) for x in args.emulate.split("/"))
    if shard_world > 1 and h_all.n_hist > 1:
        mine = np.flatnonzero(_lib.shard_histories_by_cost(kind, 0, h_all, shard_world)[0] == shard_rank)
        h = h_all.select(mine.tolist())
    else:
        h = h_all
    gen_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    plan = _lib.Plan(kind, 0, h, device=local)
    plan_s = time.perf_counter() - t0
    log(f"[rank {rank}] {args.workload}: {h.n_hist} of {h_all.n_hist} histories, {h.n} entries, "
        f"{h.n_ops()} ops; gen {gen_s:.2f}s, plan create (encode+upload) {plan_s:.2f}s")

    for _ in range(args.warmup):
        plan.run()
    barrier_sync()
    kernel_ms = 0.0
    t0 = time.perf_counter()
    step_stats = []
    for _ in range(args.steps):
        plan.run()
        step_stats.append(plan.stats())
        kernel_ms += step_stats[-1]["kernel_ms"]
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if dist:
        torch, tdist = dist
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_device())
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
    res = plan.results()
    st = plan.stats()
    phases = {k[len("create_"):]: round(st[k], 3) for k in st if k.startswith("create_")}
    log(f"[rank {rank}] plan create phases (ms): {phases}")
    explored_rank = int(res["explored"].sum())
    total_ops = h_all.n_ops() * args.steps if not args.emulate else h.n_ops() * args.steps
    value = total_ops / elapsed
    vcount = {int(v): int((res["valid"] == v).sum()) for v in (0, 1, 2)}
    plan.close()

    # end to end through the C-ABI as a JVM caller uses it (lc_check: host arrays -> encode
    # (a4/a8) -> H2D -> search -> D2H), rank 0's share; PCIe-inclusive, so never `value`
    e2e = None
    if args.e2e_reps > 0 and rank == 0:
        _lib.check(kind, 0, h)  # (untimed: lc_check's cached per-device plan is created here)
        ts = []
        for _ in range(args.e2e_reps):
            t0 = time.perf_counter()
            _lib.check(kind, 0, h)
            ts.append(time.perf_counter() - t0)
        ts.sort()
        med = ts[len(ts) // 2]
        # lc_check keeps one plan per device: the last call's setup split (lc_check_stats)
        cs = _lib.check_stats(local)
        e2e = {"ms_per_check": med * 1e3, "value": h.n_ops() / med, "unit": "history ops/s",
               "reps": args.e2e_reps, "what": "lc_check from host arrays (encode + H2D + search "
               "+ D2H), this rank's histories",
               "last_call_phases_ms": {k[len("create_"):]: round(cs[k], 3) for k in cs
                                       if k.startswith("create_")} | {
                                           "search_kernels": round(cs["kernel_ms"], 3)},
               "first_plan_create_phases_ms": phases}
        if h.n_hist > 1 and args.e2e_shards > 1:
            # lc_check(n_gpus = S) as a JVM caller spreads one independent history over S GPUs
            # (register.clj:106): the batch is encoded once, split by modeled cost, each shard's
            # plan copies its histories' encoded arrays; here the S shards are multiplexed on
            # the visible device(s), so this is the host path plus S serialised searches
            ref = _lib.check(kind, 0, h)
            _lib.check(kind, 0, h, n_gpus=args.e2e_shards)  # (untimed: the shards' plans)
            ts = []
            for _ in range(args.e2e_reps):
                t0 = time.perf_counter()
                g = _lib.check(kind, 0, h, n_gpus=args.e2e_shards)
                ts.append(time.perf_counter() - t0)
            ts.sort()
            same = all(np.array_equal(g[k], ref[k]) for k in ("valid", "fail_idx", "explored"))
            e2e["sharded"] = {"n_gpus": args.e2e_shards, "devices": lc_devices(),
                              "ms_per_check": ts[len(ts) // 2] * 1e3, "same_answers": bool(same),
                              "what": "lc_check(n_gpus) multiplexed over the visible devices: one "
                                      "encode, the cost split, per shard a copy of its encoded "
                                      "histories + upload + search"}

    if dist:
        # every rank's explored configs (the whole job's configs/s)
        t = dist[0].tensor([explored_rank], dtype=dist[0].int64, device=coll_device())
        dist[1].all_reduce(t)
        explored_all = int(t.item())
    else:
        explored_all = explored_rank
    if rank != 0:
        if dist:
            dist[1].destroy_process_group()
        return

    # dominant kernel: the dense closure-table kernels when they decided histories (events on
    # each kernel's own stream), else the grid search kernel
    acc = {}
    for s_ in step_stats:
        for k, v in s_.items():
            acc[k] = acc.get(k, 0.0) + v
    avg = {k: v / args.steps for k, v in acc.items()}
    if st.get("ctab_histories", 0) > 0:
        kname = "lc::ctab_kernel"
        k_ms = avg["ctab_ms"]
        fin, fout, expl = avg["ctab_frontier_in"], avg["ctab_frontier_out"], avg["ctab_explored"]
        table_hbm = lds_bytes = None
    elif st["dense_histories"] > 0:
        which = "big" if avg["dense_big_ms"] >= avg["dense_wave_ms"] else "wave"
        kname = f"lc::dense_{which}_kernel"
        k_ms = avg[f"dense_{which}_ms"]
        fin, fout, expl = (avg[f"dense_{which}_{q}"] for q in ("frontier_in", "frontier_out",
                                                                "explored"))
        table_hbm = avg[f"dense_{which}_hbm_bytes"]
        lds_bytes = avg[f"dense_{which}_lds_bytes"]
    else:
        kname = "lc::search_kernel"
        k_ms = kernel_ms / args.steps
        fin, fout, expl = st["frontier_in"], st["frontier_out"], st["candidates"]
        table_hbm = lds_bytes = None
    # bytes_alg = F_in*C + N_cand*(C+8) + F_out*C (C = 8 B per register config);
    # the dense kernels do not enumerate candidates, so N_cand is taken as the configs they
    # produced (every new config is at least one consistent candidate): a lower bound
    C = st["config_bytes"] or 8.0
    alg = fin * C + expl * (C + 8) + fout * C
    k_s = k_ms / 1e3
    achieved = alg / k_s / 1e9 if k_s > 0 else 0.0
    tpath = args.traffic  # the other workloads' PMC summaries: profiles/traffic_latest_<workload>.json
    alt = tpath.replace("traffic_latest.json", f"traffic_latest_{args.workload}.json")
    if args.workload != "c3" and alt != tpath and os.path.exists(alt):
        tpath = alt
    prof = read_profile(tpath, args.workload, args.scale, kname)
    traffic = prof.get("hbm_bytes_per_launch") if prof else None
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kname,
            "kernel_ms": k_ms, "alg_bytes_per_launch": alg,
            "alg_model": "SURVEY 8(d): F_in*C + N_cand*(C+8) + F_out*C, C=8; N_cand >= "
                         "configs explored (lower bound)" if table_hbm is not None else
                         "SURVEY 8(d): F_in*C + N_cand*(C+8) + F_out*C",
            "terms": {"frontier_in": fin, "n_cand": expl, "frontier_out": fout}}
    if avg.get("slowest_history_us", 0) > 0 and k_ms > 0:
        # how much of the launch is ONE history's dependent chain of steps
        # (its dequeue-to-end time on the device clock): near 1, the kernel is chain-bound and
        # the nominal §8(d) frac says little about it
        sh_ms = avg["slowest_history_us"] / 1e3
        roof["chain"] = {"slowest_history_ms": sh_ms, "steps": int(st["slowest_history_steps"]),
                         "width": int(st["slowest_history_width"]),
                         "us_per_step": avg["slowest_history_us"] / max(1.0, st["slowest_history_steps"]),
                         "frac_of_kernel": sh_ms / k_ms}
    if table_hbm is not None:
        lds_ach = lds_bytes / k_s / 1e9 if k_s > 0 else 0.0
        roof["table"] = {"hbm_bytes_per_launch": table_hbm, "lds_bytes_per_launch": lds_bytes,
                         "lds_achieved": lds_ach, "lds_peak": LDS_PEAK_GBS, "unit": "GB/s",
                         "lds_frac": lds_ach / LDS_PEAK_GBS,
                         "note": "what the closure tables really move: step streams + tile "
                                 "mirrors in HBM, the tables themselves in LDS"}
        if prof and prof.get("valu_insts_per_launch"):
            # MI355X_MICROARCH.md: a wave issues one VALU instruction per 2 cycles per SIMD
            cap = 1024 * 2.4e9 / 2 * k_s
            roof["valu"] = {"insts_per_launch": prof["valu_insts_per_launch"],
                            "issue_frac": prof["valu_insts_per_launch"] / cap}
        roof["note"] = ("the kernel's time is the longest history's dependent chain of popcount "
                        "layers (VALU issue and LDS latency), see DESIGN.md §3.1")
    else:
        roof.update({"grid_phases": st["phases"], "ret_steps": st["steps"],
                     "spill_inserts": st["spill_inserts"]})

    cpu = None
    parity = None
    if not args.no_cpu and world == 1 and not args.emulate:
        ci = cpu_info()
        cpu, ores, sample, hs = cpu_baseline(h, model, args.cpu_budget, ci["threads"], not args.cpu_sample,
                                             args.cpu_reps if not args.cpu_sample else 1)
        cpu.update({k: ci[k] for k in ("cpu_model", "nproc", "affinity")})
        cpu["cores_from"] = ci["share"]
        if h.n_hist > 1:
            # the GPU/CPU ratio from the same run, over the same keys
            cpu["gpu_over_cpu"] = value / cpu["value"]
            pk = cpu.get("per_key") or {}
            if pk.get("sum_s"):
                cpu["per_key_sum"] = {"value": pk["ops_per_s_if_perfectly_packed"],
                                      "gpu_over_cpu": value / pk["ops_per_s_if_perfectly_packed"],
                                      "note": "history ops / (sum of per-key times / threads): the "
                                              "CPU throughput if the keys packed perfectly"}
                # every core this process may use (affinity), from the measured per-key times:
                # the wall is at least max(sum / cores, the slowest key) (projection)
                cpu["projected_all_affinity"] = {
                    "cores": ci["affinity"],
                    "value": hs.n_ops() / max(pk["sum_s"] / ci["affinity"], pk["max_s"]),
                    "note": "projection from per-key times, not measured (the box's CPU share is "
                            f"{ci['threads']} threads)"}
        if h.n_hist > 1:
            mism = [k for i, k in enumerate(sample)
                    if int(res["valid"][k]) != ores[i]["valid"] or
                    int(res["fail_idx"][k]) != ores[i]["fail_idx"] or
                    int(res["explored"][k]) != ores[i]["explored"]]
            parity = {"keys_compared": len(sample), "mismatches": len(mism)}
        else:
            g = _lib.check(kind, 0, hs)
            parity = {"keys_compared": 1,
                      "mismatches": int(int(g["valid"][0]) != ores[0]["valid"] or
                                        int(g["explored"][0]) != ores[0]["explored"])}
            # a prefix overstates the CPU where the frontier grows along the history (crashed ops
            # stay pending): quote the committed whole-history oracle run beside it (tests/golden,
            # one thread in the build container; its explored count is the GPU's)
            fx = golden_fixture(args.workload)
            if fx and fx.get("provenance", {}).get("wall_s"):
                w = float(fx["provenance"]["wall_s"])
                cpu["whole_history"] = {
                    "value": fx["n_ops"] / w, "configs_per_s": fx["explored"] / w, "wall_s": w,
                    # this box's GPU rate over an oracle wall time from ANOTHER machine: a
                    # cross-machine ratio, never to be read as a same-run speedup
                    "gpu_over_cpu_cross_machine": value / (fx["n_ops"] / w),
                    "same_explored": int(res["explored"][0]) == fx["explored"],
                    "source": f"tests/golden ({fx['provenance'].get('checker', 'oracle')}, build container, "
                              f"{fx['provenance'].get('date', '')}): the whole history, not measured in this run"}

    desc = {"c1": "register 10 keys x 200 ops, 5 clients",
            "c2": "register 1 key x 5k ops, 16 clients",
            "c3": "jepsen.independent cas-register 1k keys x 1k ops, 5 clients/key",
            "c4": "register 1 key x 100k ops, 16 clients, crashed :info ops",
            "c2c": "counter 1 key x 5k ops, 16 clients (C2's shape), one whole-history search",
            "c5x": "counter 1M ops, 16 clients, 4 crashed ops (C5's exact-search variant)"}[args.workload]
    out = {
        "metric": "history ops verified/sec (+ configs explored/sec, % HBM roofline)",
        "value": value,
        "unit": "history ops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (simulated linearizable SUT, SURVEY §8(d) seeds)",
        "config": {"workload": f"{args.workload}: {desc}",
                   "histories": h_all.n_hist, "ops": h_all.n_ops(), "p_info": cfg["p_info"],
                   "scale": args.scale,
                   "parallelism": f"keys split over {world} GPU(s) by LPT (lc_shard_histories)",
                   "timed": "lc_plan_run: the search on encoded histories resident in HBM"},
        "configs_explored_per_s": explored_all * args.steps / elapsed,
        "kernel_ms_per_step": kernel_ms / args.steps,
        "verdicts": vcount,
        "end_to_end": e2e,
        "roofline": roof,
        "cpu_baseline": cpu,
        "parity_sample": parity,
    }
    if args.emulate:
        out["config"]["emulated"] = (f"rank {shard_rank} of {shard_world}: {h.n_hist} histories, "
                                     f"{h.n_ops()} ops on this GPU; value counts them only")
    print(json.dumps(out), flush=True)
    if dist:
        dist[1].destroy_process_group()


if __name__ == "__main__":
    main()
