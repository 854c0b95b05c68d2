"""In-tree build of the native extensions (no setuptools / hipify involved).

* ``_rdb_ops``     -- gfx950 HIP kernels (MFMA GEMM / implicit-GEMM conv, norms,
                      attention, softmax-top-k, gather) + the replica Engine.
                      Built with ``hipcc --offload-arch=gfx950``.
* ``_rdb_runtime`` -- host runtime (shm rings, router, load generator,
                      consumer).  Pure C++, built with g++ so it works on
                      CPU-only hosts.

Both land next to this file so they travel with the repository snapshot.
Usage: ``python -m ray_dynamic_batching_amd._build [--force] [--only ops|runtime]``;
``--sanitize thread`` builds an instrumented runtime + Python launcher under
``_variants/san-thread/`` (tests/test_sanitizers.py).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import re
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
OPS_SRC = PKG / "ops" / "csrc"
RT_SRC = PKG / "runtime" / "csrc"
BUILD = PKG.parent / "build" / "native"
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("RDB_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _pybind_includes() -> list[str]:
    import pybind11

    return [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]


def ops_target() -> Path:
    return PKG / f"_rdb_ops{EXT}"


def runtime_target() -> Path:
    return PKG / f"_rdb_runtime{EXT}"


def _ops_sources() -> list[Path]:
    # largest translation units first (the GEMM template instantiations), so the
    # longest compiles start at once on the job pool
    srcs = sorted(OPS_SRC.glob("*.hip")) + sorted(OPS_SRC.glob("*.cpp"))
    return sorted(srcs, key=lambda p: (not p.name.startswith(("conv", "gemm_bf16", "gemm_f16", "gemm_ln", "qkv")), p.name))


def _deps(srcs: list[Path], extra_dirs: list[Path]) -> list[Path]:
    deps = list(srcs)
    for d in extra_dirs:
        deps += list(d.glob("*.h"))
    return deps


_INC = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _local_includes(src: Path, seen: set | None = None) -> list[Path]:
    """Transitive quoted includes of ``src`` that resolve inside the source
    trees: an object is rebuilt only when a header it actually includes changed."""
    seen = set() if seen is None else seen
    out = []
    for name in _INC.findall(src.read_text(errors="ignore")):
        for base in (src.parent, OPS_SRC, RT_SRC):
            p = (base / name).resolve()
            if p.exists():
                if p not in seen:
                    seen.add(p)
                    out.append(p)
                    out += _local_includes(p, seen)
                break
    return out


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(p.stat().st_mtime > t for p in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}")


def hipcc() -> str:
    p = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    if not os.path.exists(p):
        raise RuntimeError("hipcc not found; set ROCM_PATH")
    return p


# per-source compiler flags: gemm_v4.hip's one-block-per-CU kernels keep their
# MFMA accumulators in VGPR form (the default heuristic picks AGPRs and copies
# them after every MFMA: profiles/gemm_lab_r5_v4.txt)
SRC_FLAGS = {"gemm_v4.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}


def variant_target(name: str) -> Path:
    """Where ``build_ops(variant=name)`` puts an A/B build of the kernels
    (loaded instead of the default one when ``RDB_OPS_SO`` points at it)."""
    return PKG / "_variants" / name / f"_rdb_ops{EXT}"


def build_ops(force: bool = False, jobs: int | None = None, verbose: bool = False, variant: str = "",
              defines: tuple = ()) -> Path:
    """Build _rdb_ops; ``variant`` + ``defines`` (e.g. ("RDB_GEMM_GROUPED",)) build
    an A/B copy under ``_variants/<variant>/`` from separate objects."""
    target = variant_target(variant) if variant else ops_target()
    bdir = BUILD / ("variant-" + variant) if variant else BUILD
    srcs = _ops_sources()
    if not force and not _stale(target, _deps(srcs, [OPS_SRC, RT_SRC])):
        return target
    bdir.mkdir(parents=True, exist_ok=True)
    target.parent.mkdir(parents=True, exist_ok=True)
    cc = hipcc()
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result",
              f"-I{OPS_SRC}", f"-I{RT_SRC}"] + _pybind_includes() + [f"-D{d}" for d in defines]
    if variant:
        # A/B builds may add compiler flags (e.g. "-mllvm -amdgpu-mfma-vgpr-form=1")
        common += os.environ.get("RDB_VARIANT_HIPFLAGS", "").split()
    objs = []
    cmds = []
    for s in srcs:
        o = bdir / (s.name + ".o")
        objs.append(o)
        newest = max(p.stat().st_mtime for p in [s] + _local_includes(s))
        if not force and o.exists() and o.stat().st_mtime >= newest:
            continue  # object up to date
        lang = ["-x", "hip"] if s.suffix == ".hip" else []
        cmds.append([cc] + common + SRC_FLAGS.get(s.name, []) + lang + ["-c", str(s), "-o", str(o)])
    jobs = jobs or min(8, os.cpu_count() or 4, 16)
    with cf.ThreadPoolExecutor(jobs) as ex:
        for c in cmds:
            if verbose:
                print(" ".join(c))
        list(ex.map(_run, cmds))
    tmp = target.with_suffix(".tmp.so")
    _run([cc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(tmp)] + [str(o) for o in objs]
         + [f"-L{ROCM}/lib", "-lamdhip64", "-lrocprofiler-sdk-roctx", f"-Wl,-rpath,{ROCM}/lib"])
    os.replace(tmp, target)
    return target


def sanitizer_dir(san: str) -> Path:
    """Where the sanitizer build of the host runtime and its launcher live:
    ``_variants/san-<preset>/`` -- never the production extension's path."""
    return PKG / "_variants" / ("san-" + san.replace(",", "-"))


def build_runtime(force: bool = False, sanitize: str = "") -> Path:
    """Build _rdb_runtime.  ``sanitize`` ("thread", "address,undefined", ...;
    default from RDB_SANITIZE) builds an instrumented copy under
    ``sanitizer_dir(preset)`` instead (load it with RDB_RUNTIME_SO; the
    production ``_rdb_runtime`` is never replaced by a sanitizer build)."""
    san = sanitize or os.environ.get("RDB_SANITIZE", "")
    target = (sanitizer_dir(san) / f"_rdb_runtime{EXT}") if san else runtime_target()
    srcs = [RT_SRC / "runtime.cpp", RT_SRC / "node_agent.cpp"]
    if not force and not _stale(target, _deps(srcs, [RT_SRC])):
        return target
    target.parent.mkdir(parents=True, exist_ok=True)
    cxx = _san_cxx() if san else os.environ.get("CXX", "g++")
    tmp = target.with_suffix(".tmp.so")
    flags = ["-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={san}"] if san else ["-O2"]
    _run([cxx] + flags + ["-std=c++17", "-fPIC", "-shared", "-Wall", "-Wno-unused-function",
          "-fvisibility=hidden", f"-I{RT_SRC}"] + _pybind_includes() + [str(s) for s in srcs]
         + ["-o", str(tmp), "-lrt", "-pthread"])
    os.replace(tmp, target)
    return target


def _san_cxx() -> str:
    """Compiler of the sanitizer builds: ROCm's clang++ (its compiler-rt links the
    sanitizer runtime into the launcher only; the instrumented extension resolves
    it from there -- with GCC 11's shared libtsan, any fork after dlopen-ing the
    instrumented extension hung), else $CXX / g++."""
    if os.environ.get("RDB_SAN_CXX"):
        return os.environ["RDB_SAN_CXX"]
    clang = Path(ROCM) / "lib" / "llvm" / "bin" / "clang++"
    return str(clang) if clang.exists() else os.environ.get("CXX", "g++")


def build_sanitized_python(san: str, force: bool = False) -> Path:
    """A CPython launcher (Py_BytesMain) linked with -fsanitize=<san>, so the
    sanitizer runtime is initialised before the interpreter and every
    extension it loads -- how the Python test suites run against the
    instrumented runtime (reference: the Bazel tsan / asan configs, .bazelrc)."""
    out = sanitizer_dir(san) / "python"
    src = RT_SRC / "tests" / "sanitized_python.cpp"
    if not force and out.exists() and out.stat().st_mtime >= src.stat().st_mtime:
        return out
    out.parent.mkdir(parents=True, exist_ok=True)
    inc = sysconfig.get_paths()["include"]
    libdir = sysconfig.get_config_var("LIBDIR") or "/usr/lib/x86_64-linux-gnu"
    ver = sysconfig.get_config_var("LDVERSION") or sysconfig.get_python_version()
    _run([_san_cxx(), "-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={san}", "-fPIE", "-pie",
          f"-I{inc}", str(src), "-o", str(out), f"-L{libdir}", f"-lpython{ver}", f"-Wl,-rpath,{libdir}",
          "-ldl", "-lm", "-pthread"])
    return out


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_runtime(force)
    build_ops(force, verbose=verbose)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["ops", "runtime"])
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--variant", default="", help="A/B build name (kernels only), with -D defines")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--sanitize", default="", help="host runtime only: build an instrumented copy + launcher under "
                    "_variants/san-<preset>/ (e.g. thread, address,undefined)")
    a = ap.parse_args(argv)
    if a.sanitize:
        print("built", build_runtime(a.force, sanitize=a.sanitize), build_sanitized_python(a.sanitize, a.force))
        return 0
    if a.variant:
        print("built", build_ops(a.force, verbose=a.verbose, variant=a.variant, defines=tuple(a.defines)))
        return 0
    if a.only in (None, "runtime"):
        print("built", build_runtime(a.force))
    if a.only in (None, "ops"):
        print("built", build_ops(a.force, verbose=a.verbose))
    return 0


if __name__ == "__main__":
    sys.exit(main())
