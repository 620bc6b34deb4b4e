"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer: the product's
history encoder (csrc/encode.cpp) and the C oracle, fed seeded random well-formed and malformed
histories by tests/sanitize/fuzz_main.cpp. GPU code is not sanitized (not available on this
pool); this covers the host side of the boundary."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="no host compiler")
def test_encoder_and_oracle_under_asan_ubsan(tmp_path):
    obj = tmp_path / "oracle.o"
    exe = tmp_path / "fuzz"
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-g", "-O1"]
    subprocess.run(["gcc", *san, "-c", "-o", str(obj), os.path.join(ROOT, "oracle", "lincheck_oracle.c")],
                   check=True)
    subprocess.run(["g++", *san, "-std=c++17", "-o", str(exe),
                    os.path.join(ROOT, "tests", "sanitize", "fuzz_main.cpp"),
                    os.path.join(ROOT, "jepsen-jgroups-raft_amd", "csrc", "encode.cpp"), str(obj), "-lpthread"],
                   check=True)
    # verify_asan_link_order=0: the environment may preload a library ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "sanitize ok" in r.stdout
