"""Per-forward kernel table from a rocprofv3 kernel trace (steady-state tail).

    python bench/trace_table.py gpurun_out/bd/bd_kernel_trace.csv [--tail 0.3] [--marker embed_ln]

Takes the last ``--tail`` fraction of the trace window (past tuning / capture),
counts forwards by the kernel named by ``--marker`` (one launch per forward) and
prints, per kernel name, launches per forward, mean duration and time per
forward, plus the wall time per forward in that window.
"""
from __future__ import annotations

import argparse
import collections
import csv


def table(path: str, tail: float = 0.3, marker: str = "embed_ln", width: int = 90):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t0, t1 = int(rows[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in rows)
    cut = t1 - int(tail * (t1 - t0))
    sel = [r for r in rows if int(r["Start_Timestamp"]) >= cut]
    nf = max(1, sum(1 for r in sel if marker in r["Kernel_Name"]))
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        a = agg[r["Kernel_Name"][:width]]
        a[0] += 1
        a[1] += d
    out = []
    for name, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1]):
        out.append(dict(kernel=name, per_fwd=round(c / nf, 2), avg_us=round(d / c, 2), us_per_fwd=round(d / nf, 1)))
    wall_us = (t1 - int(sel[0]["Start_Timestamp"])) / 1e3 / nf
    return dict(forwards=nf, wall_us_per_fwd=round(wall_us, 1),
                kernel_us_per_fwd=round(sum(d for _, d in agg.values()) / nf, 1), kernels=out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--tail", type=float, default=0.3)
    ap.add_argument("--marker", default="embed_ln")
    a = ap.parse_args()
    t = table(a.trace, a.tail, a.marker)
    print(f"forwards {t['forwards']}  wall {t['wall_us_per_fwd']} us/fwd  kernel sum {t['kernel_us_per_fwd']} us/fwd")
    for k in t["kernels"]:
        print(f"{k['per_fwd']:6.2f}/fwd {k['avg_us']:8.2f} us {k['us_per_fwd']:8.1f} us/fwd  {k['kernel']}")


if __name__ == "__main__":
    main()
