"""Race / memory-error detection for the threaded host C++ (SURVEY §5.2;
reference: the Bazel tsan / asan configs the Python suites run under in CI,
.bazelrc:103-136, .buildkite/core.rayci.yml:196-203).

* the shm ring / trace / seqlock stress binary, built with -fsanitize=thread and
  -fsanitize=address,undefined;
* the WHOLE host runtime extension (router Client / LoadGen / Consumer threads,
  node agent supervisor + monitor + control server, TP broadcast ring) built as
  an instrumented copy under ``_variants/san-<preset>/`` (never over the
  production ``_rdb_runtime``), loaded with RDB_RUNTIME_SO by a CPython
  launcher linked with the same sanitizer, running the runtime / agent / router
  / Serve-process / TP test files.  Child processes (agent-spawned replicas,
  multiprocessing ranks) start from the same launcher, so they are checked too.
A report anywhere fails the test."""
import os
import shutil
import subprocess

import pytest

from ray_dynamic_batching_amd import _build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "ray_dynamic_batching_amd", "runtime", "csrc", "tests", "ring_stress.cpp")
SUITES = ["tests/test_runtime_shm.py", "tests/test_router_native.py", "tests/test_node_agent.py",
          "tests/test_tp_bcast.py", "tests/test_serve_tp.py"]
REPORTS = ("WARNING: ThreadSanitizer", "ERROR: AddressSanitizer", "runtime error:", "ERROR: LeakSanitizer")


def _san_env(san: str) -> dict:
    env = dict(os.environ)
    supp = os.path.join(ROOT, "tests", "tsan.supp")
    # report_mutex_bugs=0: the uninstrumented gloo process group's condition
    # variables look like "unlock of an unlocked mutex" to TSan (false positive in
    # libtorch); data races -- what the instrumented runtime is checked for -- stay on
    env.update(TSAN_OPTIONS=f"halt_on_error=1:second_deadlock_stack=1:report_mutex_bugs=0:suppressions={supp}",
               # the interpreter itself leaks by design (interned objects at exit)
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    return env


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_ring_stress_under_sanitizer(tmp_path, san):
    cxx = shutil.which(_build._san_cxx())
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "ring_stress")
    build = subprocess.run([cxx, "-O1", "-g", "-std=c++17", f"-fsanitize={san}", "-fno-omit-frame-pointer", SRC,
                            "-o", exe, "-lrt", "-pthread"], capture_output=True, text=True, timeout=300)
    assert build.returncode == 0, build.stderr[-3000:]
    run = subprocess.run([exe, "4", "5000"], capture_output=True, text=True, timeout=300, env=_san_env(san))
    assert run.returncode == 0 and "OK" in run.stdout, (run.stdout + run.stderr)[-4000:]


@pytest.mark.slow
@pytest.mark.timeout(1500)
@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_runtime_suites_under_sanitizer(san):
    try:
        so = _build.build_runtime(sanitize=san)
        py = _build.build_sanitized_python(san)
    except Exception as e:  # noqa: BLE001 -- no sanitizer toolchain on this host
        pytest.skip(f"sanitizer build unavailable: {e}")
    env = _san_env(san)
    env.update(RDB_RUNTIME_SO=str(so), RDB_NO_AUTOBUILD="1", PYTHONHOME=os.environ.get("PYTHONHOME", "/usr"),
               PYTHONPATH=ROOT)
    r = subprocess.run([str(py), "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu and not slow"]
                       + SUITES, cwd=ROOT, capture_output=True, text=True, timeout=1400, env=env)
    out = r.stdout + r.stderr
    hits = [m for m in REPORTS if m in out]
    assert r.returncode == 0 and not hits, (hits, out[-6000:])
    assert " passed" in out


@pytest.mark.timeout(600)
def test_launcher_reports_a_race_in_an_instrumented_extension(tmp_path):
    """Canary: a deliberately racy instrumented .so, loaded through ctypes by
    the TSan launcher, must make TSan fire (exit code 66) -- so the clean suite
    runs above are evidence, not a mis-wired setup."""
    try:
        py = _build.build_sanitized_python("thread")
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"sanitizer build unavailable: {e}")
    so = tmp_path / "canary.so"
    src = os.path.join(ROOT, "ray_dynamic_batching_amd", "runtime", "csrc", "tests", "tsan_canary.cpp")
    b = subprocess.run([_build._san_cxx(), "-O1", "-g", "-fsanitize=thread", "-fPIC", "-shared", src, "-o", str(so),
                        "-pthread"], capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr[-2000:]
    env = _san_env("thread")
    env["PYTHONHOME"] = os.environ.get("PYTHONHOME", "/usr")
    r = subprocess.run([str(py), "-c", f"import ctypes; print(ctypes.CDLL({str(so)!r}).rdb_tsan_canary(100000))"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 66 and "WARNING: ThreadSanitizer: data race" in r.stderr, (r.returncode, r.stderr[-2000:])
