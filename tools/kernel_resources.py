#!/usr/bin/env python3
"""Per-kernel register / LDS / spill report of the built gfx950 extension,
read from the code objects' AMDHSA metadata (no GPU needed):

    python tools/kernel_resources.py [--so ray_dynamic_batching_amd/_rdb_ops*.so] [--spills-only]

The linked extension carries one clang offload bundle per translation unit in
its ``.hip_fatbin`` section; each bundle's gfx950 entry is an ELF code object
whose NT_AMDGPU_METADATA note lists every kernel with ``.vgpr_count``,
``.agpr_count``, ``.vgpr_spill_count``, ``.sgpr_spill_count`` and
``.group_segment_fixed_size`` (static LDS).  Exit status 1 if any kernel spills
VGPRs or uses scratch (the check every hot kernel should pass); SGPR spills go
to VGPR lanes and are only listed.
"""
from __future__ import annotations

import argparse
import glob
import os
import re
import struct
import subprocess
import sys
import tempfile

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
DEMANGLE = "c++filt"


def bundles(blob: bytes):
    """(triple, code object bytes) of every entry of every bundle in the fatbin."""
    for m in re.finditer(re.escape(MAGIC), blob):
        base = m.start()
        off = base + len(MAGIC)
        (n,) = struct.unpack_from("<Q", blob, off)
        off += 8
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", blob, off)
            off += 24
            triple = blob[off:off + tlen].decode()
            off += tlen
            yield triple, blob[base + eoff: base + eoff + esize]


def kernels(code: bytes):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(code)
        f.flush()
        out = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True).stdout
    cur = None
    for line in out.splitlines():
        line = line.strip()
        m = re.match(r"^- \.agpr_count:\s+(\d+)", line) or re.match(r"^\.agpr_count:\s+(\d+)", line)
        if m:
            cur = {"agpr": int(m.group(1))}
            continue
        if cur is None:
            continue
        for key, name in ((".name:", "name"), (".vgpr_count:", "vgpr"), (".vgpr_spill_count:", "vspill"),
                          (".sgpr_spill_count:", "sspill"), (".group_segment_fixed_size:", "lds"),
                          (".private_segment_fixed_size:", "scratch")):
            if line.startswith(key):
                v = line.split(":", 1)[1].strip()
                cur[name] = v if name == "name" else int(v)
        if "name" in cur and "vgpr" in cur and "vspill" in cur and "lds" in cur:
            yield cur
            cur = None


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ap.add_argument("--so", default=(glob.glob(os.path.join(root, "ray_dynamic_batching_amd", "_rdb_ops*.so")) or [""])[0])
    ap.add_argument("--spills-only", action="store_true")
    ap.add_argument("--filter", default="", help="substring of the demangled kernel name")
    a = ap.parse_args(argv)
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin")
        subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fb}", a.so, os.path.join(td, "x.so")], check=True)
        blob = open(fb, "rb").read()
    rows = []
    for triple, code in bundles(blob):
        if "gfx950" not in triple:
            continue
        rows.extend(kernels(code))
    names = [r["name"] for r in rows]
    dem = subprocess.run([DEMANGLE], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    for r, d in zip(rows, dem):
        r["demangled"] = d
    # VGPR spills / scratch go to memory; SGPR spills land in VGPR lanes (cheap) and are only listed
    spilling = [r for r in rows if r.get("vspill", 0) or r.get("scratch", 0)]
    shown = spilling if a.spills_only else rows
    if a.filter:
        shown = [r for r in shown if a.filter in r["demangled"]]
    for r in sorted(shown, key=lambda r: (-r.get("vspill", 0), r["demangled"])):
        print(f"regs {r['vgpr']:3d} (agpr {r['agpr']:3d}) spill v{r.get('vspill', 0):4d} s{r.get('sspill', 0):3d} "
              f"scratch {r.get('scratch', 0):5d} lds {r['lds']:6d}  {r['demangled'][:150]}")
    print(f"{len(rows)} gfx950 kernels, {len(spilling)} with VGPR spills or scratch "
          f"(regs = unified VGPR + AGPR count)", file=sys.stderr)
    return 1 if spilling else 0


if __name__ == "__main__":
    sys.exit(main())
