"""Per-block timeline of the UNPROFILED bench, from in-kernel stamps.

The diagnostic kernel build (``python -m ray_dynamic_batching_amd._build
--variant stamps -D RDB_BLOCK_STAMPS``; ops/csrc/common.h ``RDB_STAMP_*``)
makes one thread of every block of the GEMM / attention / norm kernels write
one record to a device buffer: block start and end (``s_memrealtime``, the
100 MHz constant clock), the kernel family and tile, the grid size, the
dispatch packet it belongs to and the hardware CU it ran on (XCC_ID + HW_ID).
No profiler is attached, so the concurrency of the two compute streams is the
real one -- rocprofv3's traced runs serialise dispatches and stretch the
forward (1,396 us traced vs 982 us per batch un-profiled in round 4).

This module turns the records into:

* launches: records grouped by dispatch packet (split at gaps, packets are
  reused): span = first block start -> last block end;
* per kernel (family, tile, grid): launches, mean span, block-time, CU-time
  (each block's duration divided among the blocks co-resident on its CU at
  every instant -- the share of the machine the kernel really held), and the
  co-residency fraction (block-time during which a block of ANOTHER launch
  ran on the same CU);
* the whole window: wall (union of spans), kernel sum (sum of spans), overlap
  1 - wall / sum, and machine utilisation = CU-busy time / (CUs x wall).

    python bench/stamp_timeline.py gpurun_out/stamps.npy -o profiles/stamp_timeline_r5.json
"""
from __future__ import annotations

import argparse
import collections
import json
from typing import Dict, List, Tuple

import numpy as np

TICK_NS = 10.0       # s_memrealtime runs at 100 MHz

FAMILIES = {1: "gemm_pp", 2: "mfma_gemm", 3: "qkv_attn", 4: "norm16", 5: "skinny_gemm", 6: "embed16",
            7: "attention", 8: "conv", 9: "gemm_pp_ln"}


def decode(rec: np.ndarray) -> Dict[str, np.ndarray]:
    """rec: [N, 4] uint64 -> columns (see common.h RDB_STAMP_END)."""
    rec = np.asarray(rec, dtype=np.uint64).reshape(-1, 4)
    rec = rec[(rec[:, 0] != 0) & (rec[:, 1] >= rec[:, 0])]
    meta, hw = rec[:, 2], rec[:, 3]
    return dict(
        t0=rec[:, 0].astype(np.int64), t1=rec[:, 1].astype(np.int64),
        family=((meta >> np.uint64(56)) & np.uint64(0xFF)).astype(np.int64),
        tile=((meta >> np.uint64(40)) & np.uint64(0xFFFF)).astype(np.int64),
        grid=(meta & np.uint64(0xFFFFFFFFFF)).astype(np.int64),
        packet=(hw >> np.uint64(32)).astype(np.int64),
        cu=(hw & np.uint64(0xFFFFFFFF)).astype(np.int64),
    )


def cu_key(hw: int) -> int:
    """XCC id (bits 16-19 of the packed word) + SE / SH / CU fields of HW_ID:
    one integer per physical CU (wave / SIMD bits masked off)."""
    xcc = (hw >> 16) & 0xF
    hwid = hw & 0xFFFF
    return (xcc << 16) | (hwid & 0xFF00)


def launches(d: Dict[str, np.ndarray], gap_ticks: int = 50) -> List[Dict]:
    """Group records by (packet, family, tile, grid); a packet slot is reused
    by later dispatches, so split a group where its blocks' start times jump
    by more than ``gap_ticks`` past the running end of the group."""
    order = np.lexsort((d["t0"], d["grid"], d["tile"], d["family"], d["packet"]))
    out, cur, key, end = [], [], None, -1
    for i in order:
        k = (d["packet"][i], d["family"][i], d["tile"][i], d["grid"][i])
        if k != key or d["t0"][i] > end + gap_ticks:
            if cur:
                out.append(cur)
            cur, key, end = [], k, -1
        cur.append(i)
        end = max(end, d["t1"][i])
    if cur:
        out.append(cur)
    res = []
    for idx in out:
        idx = np.asarray(idx)
        res.append(dict(family=int(d["family"][idx[0]]), tile=int(d["tile"][idx[0]]), grid=int(d["grid"][idx[0]]),
                        start=int(d["t0"][idx].min()), end=int(d["t1"][idx].max()), blocks=idx))
    return res


def _union(intervals: List[Tuple[int, int]]) -> int:
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(intervals):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def cu_shares(d: Dict[str, np.ndarray], launch_of: np.ndarray):
    """Per block: CU-share time (duration split among co-resident blocks) and
    co-resident time with blocks of OTHER launches on the same CU."""
    n = len(d["t0"])
    share = np.zeros(n)
    co = np.zeros(n)
    by_cu = collections.defaultdict(list)
    for i in range(n):
        by_cu[cu_key(int(d["cu"][i]))].append(i)
    busy = 0
    for cu, idx in by_cu.items():
        ev = []
        for i in idx:
            ev.append((int(d["t0"][i]), 1, i))
            ev.append((int(d["t1"][i]), -1, i))
        ev.sort(key=lambda x: (x[0], x[1]))
        active = set()
        last = None
        for t, kind, i in ev:
            if last is not None and active and t > last:
                dt = t - last
                busy += dt
                k = len(active)
                launches_here = {launch_of[j] for j in active}
                for j in active:
                    share[j] += dt / k
                    if len(launches_here) > 1 and any(launch_of[x] != launch_of[j] for x in active):
                        co[j] += dt
            last = t
            if kind == 1:
                active.add(i)
            else:
                active.discard(i)
    return share, co, busy, len(by_cu)


def summarize(rec: np.ndarray, n_cus: int = 256) -> Dict:
    d = decode(rec)
    if not len(d["t0"]):
        return dict(records=0)
    ls = launches(d)
    launch_of = np.zeros(len(d["t0"]), dtype=np.int64)
    for k, l in enumerate(ls):
        launch_of[l["blocks"]] = k
    share, co, busy, cus_seen = cu_shares(d, launch_of)
    dur = (d["t1"] - d["t0"]).astype(np.float64)
    spans = [(l["start"], l["end"]) for l in ls]
    wall = _union(spans)
    ksum = sum(e - s for s, e in spans)
    per = collections.defaultdict(lambda: dict(launches=0, span_ticks=0, block_ticks=0.0, cu_ticks=0.0,
                                               co_ticks=0.0, blocks=0))
    for l in ls:
        name = (FAMILIES.get(l["family"], f"family{l['family']}"), l["tile"], l["grid"])
        p = per[name]
        p["launches"] += 1
        p["span_ticks"] += l["end"] - l["start"]
        p["blocks"] += len(l["blocks"])
        p["block_ticks"] += float(dur[l["blocks"]].sum())
        p["cu_ticks"] += float(share[l["blocks"]].sum())
        p["co_ticks"] += float(co[l["blocks"]].sum())
    us = TICK_NS / 1e3
    kernels = []
    for (fam, tile, grid), p in per.items():
        kernels.append(dict(
            kernel=f"{fam}[tile {tile}] grid={grid}", launches=p["launches"],
            mean_span_us=round(p["span_ticks"] / p["launches"] * us, 2),
            mean_block_us=round(p["block_ticks"] / max(1, p["blocks"]) * us, 2),
            cu_us_per_launch=round(p["cu_ticks"] / p["launches"] * us, 1),
            co_resident_frac=round(p["co_ticks"] / max(1e-9, p["block_ticks"]), 3),
            total_cu_us=round(p["cu_ticks"] * us, 1),
        ))
    kernels.sort(key=lambda k: -k["total_cu_us"])
    return dict(
        records=int(len(d["t0"])), launches=len(ls), cus_seen=cus_seen,
        wall_us=round(wall * us, 1), kernel_sum_us=round(ksum * us, 1),
        overlap=round(1 - wall / ksum, 4) if ksum else 0.0,
        cu_busy_us=round(busy * us, 1), machine_util=round(busy / (n_cus * wall), 4) if wall else 0.0,
        kernels=kernels,
    )


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("records", help=".npy file of [N, 4] uint64 stamp records")
    ap.add_argument("-o", "--out", default="")
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--note", default="")
    a = ap.parse_args(argv)
    s = summarize(np.load(a.records), a.cus)
    if a.note:
        s = dict(note=a.note, **s)
    txt = json.dumps(s, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
