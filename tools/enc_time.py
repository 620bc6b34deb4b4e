"""Dump a synthetic workload's history arrays and time the host encoder on them (C++ harness
tools/enc_time.cpp, built here with g++). usage: python tools/enc_time.py [workload] [reps]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jepsen-jgroups-raft_amd"))

from lincheck import synth  # noqa: E402


def main(workload="c3", reps="5"):
    d = f"/tmp/enc_{workload}"
    os.makedirs(d, exist_ok=True)
    h = synth.gen_config(workload)
    for name, arr in zip(("off", "index", "process", "type", "f", "v0", "v1", "vflags"),
                         h.arrays()):
        arr.tofile(f"{d}/{name}.bin")
    exe = "/tmp/enc_time"
    subprocess.check_call(["g++", "-O3", "-march=native", "-std=c++17", "-pthread", "-o", exe,
                           os.path.join(ROOT, "tools/enc_time.cpp"),
                           os.path.join(ROOT, "jepsen-jgroups-raft_amd/csrc/encode.cpp")])
    subprocess.check_call([exe, d, reps])


if __name__ == "__main__":
    main(*sys.argv[1:])
