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


if __name__ == "__main__":
    main()
