"""Steady-state GPU occupancy from a rocprofv3 kernel trace: per-queue busy
fraction, union busy fraction (any kernel running), and the gaps between
consecutive kernels of one queue, over the last `--tail` fraction of the
trace (the timed serving region of bench.py).

    python bench/trace_gaps.py gpurun_out/prof_bench/p_kernel_trace.csv
"""
import argparse
import csv
import collections


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--tail", type=float, default=0.5, help="fraction of the trace (by time) to analyse")
    ap.add_argument("--timeline", default="", help="write a 3 ms kernel timeline (start end queue name) here")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]) for r in rows)
    t_end = max(e[1] for e in ev)
    t0 = ev[0][0] + (t_end - ev[0][0]) * (1 - a.tail)
    ev = [e for e in ev if e[0] >= t0]
    span = t_end - ev[0][0]
    per_q = collections.defaultdict(list)
    for e in ev:
        per_q[e[2]].append(e)
    print(f"window {span / 1e6:.2f} ms, {len(ev)} kernels")
    for q, es in sorted(per_q.items()):
        busy = sum(e[1] - e[0] for e in es)
        gaps = [b[0] - a_[1] for a_, b in zip(es, es[1:]) if b[0] > a_[1]]
        gaps.sort()
        med = gaps[len(gaps) // 2] if gaps else 0
        small = sum(g for g in gaps if g < 20000)
        print(f"queue {q}: {len(es)} kernels, busy {busy / span:.1%}, gaps<20us total {small / span:.1%} "
              f"(median gap {med / 1e3:.2f} us)")
    # union busy
    cur_s, cur_e, union = None, None, 0
    for s, e, *_ in ev:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    union += cur_e - cur_s
    print(f"union busy (any kernel running): {union / span:.1%}")
    # overlap: time with >= 2 kernels running
    pts = sorted([(s, 1) for s, e, *_ in ev] + [(e, -1) for s, e, *_ in ev])
    depth, last, two = 0, None, 0
    for t, d in pts:
        if depth >= 2 and last is not None:
            two += t - last
        depth += d
        last = t
    print(f">=2 kernels concurrently: {two / span:.1%}")
    # per kernel name: how much of its time another queue's kernel ran beside it
    other = collections.defaultdict(list)     # queue -> sorted (s, e) of every OTHER queue's kernels
    for q in per_q:
        other[q] = sorted((e[0], e[1]) for e in ev if e[2] != q)
    import bisect

    by_name = collections.defaultdict(lambda: [0, 0, 0])   # name -> [count, dur, overlapped]
    for q, es in per_q.items():
        o = other[q]
        starts = [x[0] for x in o]
        for s, e, _q, name in es:
            ov = 0
            i = max(0, bisect.bisect_left(starts, s) - 8)
            while i < len(o) and o[i][0] < e:
                ov += max(0, min(e, o[i][1]) - max(s, o[i][0]))
                i += 1
            rec = by_name[_short(name)]
            rec[0] += 1
            rec[1] += e - s
            rec[2] += min(ov, e - s)
    print("per kernel: share of its time with another queue's kernel running")
    for name, (n, d, ov) in sorted(by_name.items(), key=lambda kv: -kv[1][1])[:16]:
        print(f"  {d / span:6.1%} of window  {n:6d} x {d / n / 1e3:7.2f} us  overlapped {ov / d:5.1%}  {name}")
    if a.timeline:
        t_mid = ev[len(ev) // 2][0]
        with open(a.timeline, "w") as f:
            for s, e, q, name in ev:
                if t_mid <= s < t_mid + 3_000_000:
                    f.write(f"{(s - t_mid) / 1e3:9.2f} {(e - t_mid) / 1e3:9.2f} q{q} {_short(name)}\n")


def _short(name: str) -> str:
    n = name.split("(")[0]
    for pre in ("void ", "rdb::"):
        n = n.replace(pre, "")
    return n[:90]


if __name__ == "__main__":
    main()
