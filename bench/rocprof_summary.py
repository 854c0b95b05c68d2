"""Summarize a rocprofv3 output directory (rocpd SQLite ``*_results.db`` or
``*kernel_stats.csv``) into a small JSON that is committed under profiles/.

    python bench/rocprof_summary.py gpurun_out/prof7 -o profiles/rocprof_bench.json [--top 25]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import sqlite3


def _short(name: str) -> str:
    m = re.match(r"_ZN3rdb\d+(\w+?)I", name)
    if m:
        tmpl = re.findall(r"Li(\d+)E", name)[:2] + re.findall(r"Lb([01])E", name)
        return f"rdb::{m.group(1)}<{','.join(tmpl)}>" if tmpl else f"rdb::{m.group(1)}"
    return name if len(name) < 90 else name[:87] + "..."


def summarize(path: str, top: int = 25):
    dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    rows = []
    if dbs:
        c = sqlite3.connect(dbs[0])
        # the rocpd ``top_kernels`` view reports durations in microseconds
        rows = [dict(name=r[0], calls=r[1], total_ms=r[2] / 1e3, avg_us=r[3], pct=r[4])
                for r in c.execute("select name,total_calls,total_duration,average,percentage from top_kernels")]
    else:
        for f in glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    rows.append(dict(name=r["Name"], calls=int(r["Calls"]), total_ms=float(r["TotalDurationNs"]) / 1e6,
                                     avg_us=float(r["AverageNs"]) / 1e3, pct=float(r["Percentage"])))
    rows.sort(key=lambda r: -r["total_ms"])
    total = sum(r["total_ms"] for r in rows)
    out = dict(total_kernel_ms=round(total, 3), kernels=len(rows),
               top=[dict(kernel=_short(r["name"]), calls=r["calls"], total_ms=round(r["total_ms"], 3),
                         avg_us=round(r["avg_us"], 2), pct=round(100 * r["total_ms"] / total, 2)) for r in rows[:top]])
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("-o", "--out", default="")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args(argv)
    s = summarize(a.path, a.top)
    txt = json.dumps(s, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
