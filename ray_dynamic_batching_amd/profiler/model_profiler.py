"""Batch-size sweep profiler producing the planner's CSV contract.

Reference: 293-project/profiling/ModelProfiler.py:14-392 (+ run_profiler.py,
results_formatter.py).  Same behaviour and outputs:
  * sweep range(min_batch, max_batch + 1, step); per point reset allocator
    stats, warmup runs, timed runs, mean/std/min/max, throughput
    (B*1000/avg), peak memory, memory per sample; OOM -> status "OOM"; stop
    after 3 consecutive failures;
  * save_results -> <name>_<ts>_report.txt / _detailed.json / _summary.csv.
MI355X-native additions:
  * ``mode="graph"`` (default on GPU) times the hipGraph-captured forward --
    what the replica engine actually replays -- instead of an eager forward;
    ``mode="eager"`` reproduces the reference measurement;
  * ``include_h2d=True`` adds the serving-path input copy (pinned H2D) so the
    profile can be quoted both ways (BASELINE.md "How we will compare");
  * a CPU mode (wall clock) for tests and CPU deployments.
"""
from __future__ import annotations

import gc
import json
import math
import os
import time
from datetime import datetime, timedelta
from typing import Callable, List, Optional

import torch

from ..planner.profiles import CSV_FIELDS, write_profile_csv


class ModelProfiler:
    def __init__(self, model, input_shapes: List[tuple], min_batch_size: int = 1, max_batch_size: int = 512,
                 batch_size_step: int = 1, warmup_runs: int = 3, num_runs: int = 10,
                 output_dir: str = "profiling_results", mode: Optional[str] = None, include_h2d: bool = False,
                 input_dtype: Optional[torch.dtype] = None, device: Optional[str] = None, batch_sizes=None,
                 sleep_interval: float = 0.0, input_fn: Optional[Callable[[int], List[torch.Tensor]]] = None):
        if min_batch_size < 1:
            raise ValueError("min_batch_size must be at least 1")
        if max_batch_size < min_batch_size:
            raise ValueError("max_batch_size must be greater than or equal to min_batch_size")
        if batch_size_step < 1:
            raise ValueError("batch_size_step must be at least 1")
        if warmup_runs < 0:
            raise ValueError("warmup_runs must be non-negative")
        if num_runs < 1:
            raise ValueError("num_runs must be at least 1")
        self.model = model
        self.input_shapes = [tuple(s) for s in input_shapes]
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.gpu = self.device.type == "cuda"
        self.mode = mode or ("graph" if self.gpu else "eager")
        if self.mode == "graph" and not self.gpu:
            raise ValueError("graph mode needs a GPU")
        self.include_h2d = include_h2d
        self.input_dtype = input_dtype or getattr(model, "input_dtype", torch.float32)
        self.warmup_runs = warmup_runs
        self.num_runs = num_runs
        self.output_dir = output_dir
        self.sleep_interval = sleep_interval
        self.input_fn = input_fn
        self.batch_sizes = list(batch_sizes) if batch_sizes is not None else \
            list(range(min_batch_size, max_batch_size + 1, batch_size_step))
        os.makedirs(output_dir, exist_ok=True)
        self.gpu_info = self._device_info()

    # ---------------------------------------------------------------- helpers
    def _device_info(self) -> dict:
        if self.gpu:
            p = torch.cuda.get_device_properties(self.device)
            return dict(name=p.name, total_memory=p.total_memory / 1024 ** 2,
                        arch=getattr(p, "gcnArchName", ""), hip_version=torch.version.hip,
                        compute_units=p.multi_processor_count)
        return dict(name="cpu", total_memory=0.0, arch="x86_64", hip_version=None, compute_units=os.cpu_count())

    def _reset(self) -> None:
        gc.collect()
        if self.gpu:
            torch.cuda.synchronize(self.device)
            torch.cuda.empty_cache()
            torch.cuda.reset_peak_memory_stats(self.device)

    def _inputs(self, b: int) -> List[torch.Tensor]:
        if self.input_fn is not None:
            return self.input_fn(b)
        out = []
        for s in self.input_shapes:
            if self.input_dtype in (torch.int32, torch.int64):
                hi = getattr(getattr(self.model, "cfg", None), "vocab_size", 1000)
                t = torch.randint(1, hi, (b,) + s, dtype=self.input_dtype)
            else:
                t = torch.randn((b,) + s).to(self.input_dtype)
            out.append(t)
        return out

    def _forward(self, xs):
        f = getattr(self.model, "forward", self.model)
        return f(*xs)

    def _time_once(self, fn) -> float:
        if self.gpu:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(self.device)
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize(self.device)
            return s.elapsed_time(e)
        t = time.perf_counter()
        fn()
        return (time.perf_counter() - t) * 1e3

    # ------------------------------------------------------------- profiling
    def profile_batch_size(self, b: int) -> dict:
        res = dict(batch_size=b, status="initialized", error=None)
        graph = None
        try:
            self._reset()
            host = self._inputs(b)
            if self.gpu:
                dev = [h.to(self.device) for h in host]
                pinned = [h.pin_memory() for h in host] if self.include_h2d else None
            else:
                dev, pinned = host, None
            with torch.no_grad():
                if self.mode == "graph":
                    side = torch.cuda.Stream(self.device)
                    side.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(side):
                        for _ in range(max(1, self.warmup_runs)):
                            self._forward(dev)
                    torch.cuda.current_stream().wait_stream(side)
                    graph = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(graph):
                        self._forward(dev)

                    def step():
                        if pinned is not None:
                            for d, p in zip(dev, pinned):
                                d.copy_(p, non_blocking=True)
                        graph.replay()
                else:
                    def step():
                        if pinned is not None:
                            for d, p in zip(dev, pinned):
                                d.copy_(p, non_blocking=True)
                        self._forward(dev)
                    for _ in range(self.warmup_runs):
                        step()
                lat = [self._time_once(step) for _ in range(self.num_runs)]
            mean = sum(lat) / len(lat)
            std = math.sqrt(sum((x - mean) ** 2 for x in lat) / len(lat))
            if self.gpu:
                cur = torch.cuda.memory_allocated(self.device) / 1024 ** 2
                peak = torch.cuda.max_memory_allocated(self.device) / 1024 ** 2
            else:
                cur = peak = 0.0
            thr = b * 1000.0 / mean
            total = self.gpu_info["total_memory"] or 1.0
            res.update(status="success", avg_latency_ms=mean, std_latency_ms=std, min_latency_ms=min(lat),
                       max_latency_ms=max(lat), throughput=thr, throughput_efficiency=thr / b,
                       current_memory_mb=cur, peak_memory_mb=peak, available_memory_mb=total - cur,
                       memory_per_sample_mb=peak / b, raw_latencies=lat, memory_utilization=peak / total * 100.0)
        except torch.cuda.OutOfMemoryError:
            res.update(status="OOM", error="Out of memory error")
        except Exception as e:  # noqa: BLE001
            res.update(status="error", error=f"{type(e).__name__}: {e}")
        finally:
            graph = None
            self._reset()
        return res

    def profile_all(self) -> List[dict]:
        results = []
        consecutive = 0
        t0 = time.time()
        for i, b in enumerate(self.batch_sizes, 1):
            r = self.profile_batch_size(b)
            results.append(r)
            eta = (time.time() - t0) / i * (len(self.batch_sizes) - i)
            if r["status"] == "success":
                consecutive = 0
                print(f"batch {b}: {r['avg_latency_ms']:.3f} ms, {r['throughput']:.1f}/s "
                      f"(eta {timedelta(seconds=int(eta))})", flush=True)
            else:
                consecutive += 1
                print(f"batch {b}: {r['status']} {r.get('error')}", flush=True)
                if consecutive >= 3:
                    print("stopping after 3 consecutive failures")
                    break
            if self.sleep_interval:
                time.sleep(self.sleep_interval)
        return results

    def save_results(self, results: List[dict], model_name: str = "unnamed_model", model_info: dict = None,
                     dataset_info: dict = None, plot: bool = True) -> dict:
        ts = datetime.now().strftime("%Y%m%d_%H%M%S")
        base = os.path.join(self.output_dir, f"{model_name}_{ts}")
        paths = dict(report=base + "_report.txt", json=base + "_detailed.json", csv=base + "_summary.csv")
        if plot and plot_results(results, base + "_plot.png", title=model_name):
            paths["plot"] = base + "_plot.png"
        write_profile_csv(paths["csv"], results)
        full = dict(model_name=model_name, timestamp=ts, device=self.gpu_info, model_info=model_info or {},
                    dataset_info=dataset_info or {}, mode=self.mode, include_h2d=self.include_h2d,
                    profiling_config=dict(batch_sizes=self.batch_sizes, warmup_runs=self.warmup_runs,
                                          num_runs=self.num_runs), results=results)
        with open(paths["json"], "w") as f:
            json.dump(full, f, indent=2, default=str)
        with open(paths["report"], "w") as f:
            f.write(ResultsFormatter.format(full))
        return paths


def plot_results(results: List[dict], path: str, title: str = "") -> bool:
    """The reference's 4-panel figure (293-project/profiling/run_profiler.py:
    110-156): throughput, latency, peak memory and per-item efficiency vs batch
    size.  Returns False when matplotlib is unavailable or nothing succeeded."""
    ok = [r for r in results if r.get("status") == "success"]
    if not ok:
        return False
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        return False
    bs = [r["batch_size"] for r in ok]
    thr = [r["throughput"] for r in ok]
    panels = [("Throughput vs Batch Size", "Throughput (samples/sec)", thr, "b-"),
              ("Latency vs Batch Size", "Latency (ms)", [r["avg_latency_ms"] for r in ok], "r-"),
              ("Memory Usage vs Batch Size", "Peak Memory (MB)", [r["peak_memory_mb"] for r in ok], "g-"),
              ("Efficiency vs Batch Size", "Throughput per Batch Item", [t / b for t, b in zip(thr, bs)], "m-")]
    fig, axes = plt.subplots(2, 2, figsize=(15, 10))
    for ax, (ttl, ylab, ys, style) in zip(axes.flat, panels):
        ax.plot(bs, ys, style)
        ax.set_title(ttl)
        ax.set_xlabel("Batch Size")
        ax.set_ylabel(ylab)
        ax.grid(True)
    if title:
        fig.suptitle(title)
    fig.tight_layout()
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    fig.savefig(path)
    plt.close(fig)
    return True


class ResultsFormatter:
    """Text report with best-throughput point and coefficient-of-variation
    analysis (reference: profiling/results_formatter.py)."""

    @staticmethod
    def format(full: dict) -> str:
        ok = [r for r in full["results"] if r["status"] == "success"]
        dev = full["device"]
        lines = [f"Profiling report: {full['model_name']} ({full['timestamp']})", "=" * 72,
                 f"Device: {dev['name']} arch={dev.get('arch')} memory={dev['total_memory']:.1f} MB",
                 f"Mode: {full['mode']} (include_h2d={full['include_h2d']}); warmup "
                 f"{full['profiling_config']['warmup_runs']}, runs {full['profiling_config']['num_runs']}", ""]
        lines.append(f"{'batch':>6} {'lat ms':>10} {'std':>8} {'cv %':>6} {'thr/s':>12} {'peak MB':>10}")
        for r in ok:
            cv = r["std_latency_ms"] / r["avg_latency_ms"] * 100 if r["avg_latency_ms"] else 0
            lines.append(f"{r['batch_size']:>6} {r['avg_latency_ms']:>10.3f} {r['std_latency_ms']:>8.3f} {cv:>6.1f} "
                         f"{r['throughput']:>12.1f} {r['peak_memory_mb']:>10.1f}")
        failed = [r for r in full["results"] if r["status"] != "success"]
        if ok:
            best = max(ok, key=lambda r: r["throughput"])
            lines += ["", f"Best throughput: {best['throughput']:.1f} samples/s at batch {best['batch_size']} "
                          f"({best['avg_latency_ms']:.2f} ms)"]
            high_cv = [r["batch_size"] for r in ok if r["std_latency_ms"] > 0.1 * r["avg_latency_ms"]]
            if high_cv:
                lines.append(f"High variance (cv > 10%) at batch sizes: {high_cv[:20]}")
        if failed:
            lines.append(f"Failed points: {[(r['batch_size'], r['status']) for r in failed]}")
        return "\n".join(lines) + "\n"
