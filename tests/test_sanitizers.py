"""Race / memory-error detection presets for the host C++ runtime (SURVEY
§5.2; reference: Bazel --config=tsan/asan, .bazelrc:103-136): the shm ring /
trace / seqlock stress test built with -fsanitize=thread and with
-fsanitize=address,undefined must run clean.  ``RDB_SANITIZE=thread python -m
ray_dynamic_batching_amd._build --only runtime`` builds the whole runtime
extension with the same flags."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "ray_dynamic_batching_amd", "runtime", "csrc", "tests", "ring_stress.cpp")


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_ring_stress_under_sanitizer(tmp_path, san):
    cxx = shutil.which(os.environ.get("CXX", "g++"))
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "ring_stress")
    build = subprocess.run([cxx, "-O1", "-g", "-std=c++17", f"-fsanitize={san}", "-fno-omit-frame-pointer", SRC,
                            "-o", exe, "-lrt", "-pthread"], capture_output=True, text=True, timeout=300)
    assert build.returncode == 0, build.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    run = subprocess.run([exe, "4", "5000"], capture_output=True, text=True, timeout=300, env=env)
    assert run.returncode == 0 and "OK" in run.stdout, (run.stdout + run.stderr)[-4000:]
