"""Summarize rocprofv3 ``--pmc`` CSV passes of one program into per-kernel
hardware-counter metrics (committed under profiles/).

    python bench/pmc_summary.py gpurun_out/pmc_sq gpurun_out/pmc_fetch gpurun_out/pmc_write \
        -o profiles/pmc_bert_forward.json

Each directory is one counter pass (``rocprofv3 --pmc ... --output-format csv``);
rows are (dispatch, counter) pairs.  Counters are averaged per dispatch and per
kernel, then the derived metrics are computed:

* ``mfma_tflops`` = SQ_INSTS_MFMA x 16384 FLOP / kernel time (every GEMM MFMA here is
  v_mfma_f32_16x16x32_{bf16,f16}), ``mfma_frac_of_peak`` = that / 2.5 PFLOP/s dense bf16;
* ``lds_bank_conflict_frac`` = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles / all LDS-array cycles);
* ``fetch_bytes`` = 2 x FETCH_SIZE x 1024 (gfx950 FETCH_SIZE counts half of a wide coalesced read,
  MI355X_MICROARCH.md §HBM), ``write_bytes`` = WRITE_SIZE x 1024; both include Infinity-Cache hits;
* ``clock_ghz``   = GRBM_GUI_ACTIVE / 8 / kernel time (reads high below ~0.3 ms dispatches).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re


def _short(name: str, grid: str = "", wg: str = "") -> str:
    """rdb::<kernel><tile ints> [grid/wg]: rocprofv3 demangles some names only
    partly, so the tile shape comes from the mangled ``Li<int>E`` arguments and
    the launch geometry tells the per-shape dispatches of one template apart."""
    m = re.match(r"_ZN3rdb\d+(\w+?)I", name) or re.match(r"(?:void )?rdb::(\w+)", name)
    if m:
        tmpl = re.findall(r"Li(\d+)E", name)[:2]
        base = f"rdb::{m.group(1)}" + (f"<{','.join(tmpl)}>" if tmpl else "")
    else:
        base = name if len(name) < 60 else name[:57] + "..."
    return f"{base} grid={grid} wg={wg}" if grid else base


def _rows(path: str):
    files = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        with open(f, newline="") as fh:
            yield from csv.DictReader(fh)


def _window(rows, marker, forwards):
    """Keep the dispatches from the ``forwards``-th last dispatch of ``marker`` on
    (the steady-state graph replays at the end of the program)."""
    if not marker:
        return rows
    starts = sorted({int(r["Dispatch_Id"]) for r in rows if marker in r.get("Kernel_Name", "")})
    if not starts:
        return rows
    first = starts[-forwards] if len(starts) >= forwards else starts[0]
    return [r for r in rows if int(r["Dispatch_Id"]) >= first]


def load(paths, marker="", forwards=1):
    # kernel -> counter -> list of per-dispatch values; kernel -> durations
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    dur = collections.defaultdict(dict)
    for p in paths:
        for r in _window(list(_rows(p)), marker, forwards):
            k = _short(r.get("Kernel_Name", "?"), r.get("Grid_Size", ""), r.get("Workgroup_Size", ""))
            did = (p, r.get("Dispatch_Id", r.get("Correlation_Id", "")))
            cname = r.get("Counter_Name", "")
            try:
                v = float(r.get("Counter_Value", "nan"))
            except ValueError:
                continue
            per[k][cname][did] = per[k][cname].get(did, 0.0) + v
            s, e = r.get("Start_Timestamp"), r.get("End_Timestamp")
            if s and e:
                dur[k][did] = (int(e) - int(s)) * 1e-9
    return per, dur


def summarize(paths, top=30, marker="", forwards=1):
    per, dur = load(paths, marker, forwards)
    out = []
    for k, cs in per.items():
        avg = {c: sum(v.values()) / len(v) for c, v in cs.items() if v}
        dids = {d for v in cs.values() for d in v}
        n = len(dids) // max(1, len({d[0] for d in dids}))   # dispatches per counter pass
        d = list(dur[k].values())
        t = sum(d) / len(d) if d else None
        row = {"kernel": k, "dispatches": n, "avg_us": round(t * 1e6, 2) if t else None}
        row.update({c: round(v, 1) for c, v in sorted(avg.items())})
        gui = avg.get("GRBM_GUI_ACTIVE")
        if t and avg.get("SQ_INSTS_MFMA"):
            row["mfma_tflops"] = round(avg["SQ_INSTS_MFMA"] * 16384 / t / 1e12, 1)
            row["mfma_frac_of_peak"] = round(row["mfma_tflops"] / 2500.0, 3)
        if avg.get("SQ_LDS_IDX_ACTIVE"):
            row["lds_bank_conflict_frac"] = round(avg.get("SQ_LDS_BANK_CONFLICT", 0.0) / avg["SQ_LDS_IDX_ACTIVE"], 4)
        if "FETCH_SIZE" in avg:
            row["fetch_bytes"] = round(2 * avg["FETCH_SIZE"] * 1024)
        if "WRITE_SIZE" in avg:
            row["write_bytes"] = round(avg["WRITE_SIZE"] * 1024)
        if gui and t:
            row["clock_ghz"] = round(gui / 8 / t / 1e9, 3)
        out.append(row)
    out.sort(key=lambda r: -(r["avg_us"] or 0) * r["dispatches"])
    return out[:top]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("-o", "--out", default="")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--note", default="")
    ap.add_argument("--marker", default="", help="kernel that starts one forward (keep the last --forwards of them)")
    ap.add_argument("--forwards", type=int, default=1)
    a = ap.parse_args()
    ks = summarize(a.dirs, a.top, a.marker, a.forwards)
    tot = sum((r["avg_us"] or 0) * r["dispatches"] for r in ks) / max(1, a.forwards)
    res = {"note": a.note, "formulae": __doc__.split("* ", 1)[1].strip(),
           "kernel_us_per_forward_profiled": round(tot, 1) if a.marker else None, "kernels": ks}
    s = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s)
    print(s)


if __name__ == "__main__":
    main()
