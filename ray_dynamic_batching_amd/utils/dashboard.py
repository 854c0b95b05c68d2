"""TTY SLO dashboard over a metrics.json file (reference:
293-project/src/metrics_display.py, status thresholds at :64-65).

    python -m ray_dynamic_batching_amd.utils.dashboard [--file metrics.json] [--simple] [--once]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

QUEUE_WARN = 1600       # queue size below this is OK (metrics_display.py:64)
SLO_GOOD, SLO_WARN = 98.0, 95.0


def render(metrics: dict, simple: bool = False) -> str:
    out = []
    hdr = f"{'model':<14}{'queue':>7}{'total':>9}{'dropped':>9}{'viol':>7}{'SLO %':>8}{'rate':>9}" \
          f"{'last':>9}{'avg':>9}{'p95':>9}{'p99':>9}  status"
    out.append(hdr)
    out.append("-" * len(hdr))
    for m, s in sorted(metrics.items()):
        total = s.get("total_requests", 0)
        viol = s.get("slo_violations", 0)
        comp = (total - viol) / total * 100 if total else 100.0
        status = "OK" if (s.get("queue_size", 0) < QUEUE_WARN and comp >= SLO_GOOD) else \
            ("WARN" if comp >= SLO_WARN else "CRITICAL")
        out.append(f"{m:<14}{s.get('queue_size', 0):>7}{total:>9}{s.get('dropped_requests', 0):>9}{viol:>7}"
                   f"{comp:>8.2f}{s.get('request_rate', 0):>9.1f}{s.get('last_latency', 0):>9.1f}"
                   f"{s.get('avg_latency', 0):>9.1f}{s.get('p95_latency', 0):>9.1f}{s.get('p99_latency', 0):>9.1f}"
                   f"  {status}")
    return "\n".join(out)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--file", default="metrics.json")
    ap.add_argument("--simple", action="store_true")
    ap.add_argument("--once", action="store_true")
    ap.add_argument("--interval", type=float, default=1.0)
    a = ap.parse_args(argv)
    while True:
        try:
            with open(a.file) as f:
                m = json.load(f)
            text = render(m, a.simple)
        except (OSError, ValueError) as e:
            text = f"waiting for {a.file} ({e})"
        if not a.once and not a.simple:
            sys.stdout.write("\x1b[2J\x1b[H")
        print(time.strftime("%H:%M:%S"), "SLO dashboard")
        print(text, flush=True)
        if a.once:
            return 0
        time.sleep(a.interval)


if __name__ == "__main__":
    sys.exit(main())
