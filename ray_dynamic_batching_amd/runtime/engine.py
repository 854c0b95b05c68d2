"""GPU replica engine driver: captures one hipGraph per (batch bucket, pipeline
slot) for a servable model and hands them to the native Engine, which then runs
the whole batching / H2D / replay / D2H / completion loop without Python.

A *servable model* exposes ``input_shape``, ``input_dtype``, ``output_shape``,
``output_dtype`` (per request) and ``forward(x[B, *input_shape])``.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch

from ..utils.native import require_gpu_ops


TUNED_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ops", "tuned")


def shipped_tile_table(model, max_batch: int, compute_streams: int, pipeline_depth: int) -> str:
    """Path of the MI355X tile table shipped for this replica configuration
    (``ops/tuned/mi355x_<signature>_B<max_batch>_cs<streams>_d<depth>.json``,
    signature = ``model.tile_signature``, e.g. ``bert_L12_S128`` / ``resnet50``),
    or "" when none was tuned for it.  ``bench.py``, ``bench/serve_bench.py`` and
    Serve-deployed replicas (``EngineConfig.tile_table="auto"``) all resolve their
    table here, so the deployed replica replays what the benchmark replays."""
    sig = getattr(model, "tile_signature", None)
    if not sig:
        return ""
    names = [f"mi355x_{sig}_B{max_batch}_cs{compute_streams}_d{pipeline_depth}.json"]
    if compute_streams == 1:
        names.append(f"mi355x_{sig}_B{max_batch}_d{pipeline_depth}.json")    # round-3 single-stream name
    for n in names:
        p = os.path.join(TUNED_DIR, n)
        if os.path.exists(p):
            return p
    # same stream count, another pipeline depth: the tiles were picked for as many
    # overlapped batches, which the depth (slots waiting for a stream) does not change
    import glob

    same_cs = sorted(glob.glob(os.path.join(TUNED_DIR, f"mi355x_{sig}_B{max_batch}_cs{compute_streams}_d*.json")))
    return same_cs[0] if same_cs else ""


def resolve_tile_table(choice: str, model, max_batch: int, compute_streams: int, pipeline_depth: int) -> str:
    """EngineConfig.tile_table / bench ``--tile-table`` -> a path to replay or ""
    (= tune at start-up): "auto" = the shipped table when there is one, "none" =
    tune, anything else = that file."""
    if not choice or choice == "none":
        return ""
    if choice == "auto":
        return shipped_tile_table(model, max_batch, compute_streams, pipeline_depth)
    return choice


def default_buckets(max_batch: int) -> List[int]:
    b, out = 1, []
    while b < max_batch:
        out.append(b)
        b *= 2
    out.append(max_batch)
    # finer buckets near the top where padding waste costs the most
    extra = [max_batch * 3 // 4] if max_batch >= 8 else []
    return sorted(set(out + [e for e in extra if e > 0]))


@dataclass
class SessionSpec:
    model: object
    queue: int
    max_batch: int = 32
    max_wait_s: float = 0.005
    buckets: Optional[Sequence[int]] = None
    priority: int = 0
    slo_ms: float = 0.0
    drop_stale: bool = False
    name: str = ""
    # filled by the runner
    sid: int = -1
    capture_s: float = 0.0
    pools: list = field(default_factory=list)
    graphs: list = field(default_factory=list)
    inputs: list = field(default_factory=list)
    outputs: list = field(default_factory=list)


class EngineRunner:
    POLICY_PRIORITY_EDF = 0
    POLICY_DUTY_CYCLE = 1

    def __init__(self, job_name: str, replica: int, sessions: Sequence[SessionSpec], pipeline_depth: int = 2,
                 zero_copy: bool = True, device: Optional[int] = None, warmup_iters: int = 2, policy: int = 0,
                 compute_streams: int = 1, batch_policy: str = "timeout", stagger_us: Optional[int] = None,
                 tile_table: Optional[str] = None):
        """``policy``: 0 = priority then earliest-deadline-first across sessions
        (co-located models, config 5); 1 = Nexus duty cycle (``set_duty_cycle`` +
        per-session ``set_duty_share``).  ``compute_streams`` > 1 runs that many
        batches concurrently (one hipGraph per pipeline slot, slot i on stream
        i % n, separate graph memory pools per stream so they never alias).
        ``batch_policy``: "timeout" (default, ``@serve.batch`` semantics: a batch
        closes when full or ``max_wait`` after its first request) or "idle" (a
        partial batch is also dispatched as soon as a compute stream has no batch
        running -- lower latency at low load, same batches under saturation).
        ``stagger_us``: hold a batch starting on an idle stream that long behind
        the other stream's idle start (None: RDB_ENGINE_STAGGER_US).
        ``tile_table``: a tile-table file to replay instead of tuning at start-up
        (None: RDB_TUNE_FILE; resolve "auto" with ``resolve_tile_table``)."""
        if batch_policy not in ("timeout", "idle"):
            raise ValueError(f"batch_policy must be 'timeout' or 'idle', got {batch_policy!r}")
        self.ops = require_gpu_ops()
        self.device = torch.cuda.current_device() if device is None else device
        self.job_name = job_name
        self.replica = replica
        self.depth = pipeline_depth
        self.sessions = list(sessions)
        self.compute_streams = max(1, min(compute_streams, pipeline_depth))
        from .queues import check_hw_queues

        check_hw_queues(self.compute_streams)     # streams sharing a HIP hardware queue serialise
        self.engine = self.ops.Engine(job_name, replica, pipeline_depth, zero_copy, self.device, policy,
                                      self.compute_streams)
        self.batch_policy = batch_policy
        if batch_policy == "idle":
            self.engine.set_idle_dispatch(True)
        if stagger_us is not None:
            self.engine.set_stagger_us(int(stagger_us))
        self.stagger_us = self.engine.stagger_us()
        # per-shape tile tuning ranks candidates by throughput with this many
        # concurrent launches (ops._tuned_cfg), i.e. the replica's own regime
        os.environ.setdefault("RDB_TUNE_STREAMS", str(self.compute_streams))
        self.pools = []
        self.capture_s = 0.0
        self.warmup_iters = warmup_iters
        # whole-forward selection among near-tied GEMM tiles for the largest bucket
        # (ops.tune_in_context); RDB_TUNE_IN_CONTEXT=0 turns it off
        self.tune_in_context = os.environ.get("RDB_TUNE_IN_CONTEXT", "1") == "1"
        self.tuning_changes = {}
        # RDB_TUNE_FILE: replay a saved tile table (A/B runs, profiling passes) instead
        # of tuning; written after tuning when the file does not exist yet
        self.tune_file = tile_table if tile_table is not None else os.environ.get("RDB_TUNE_FILE", "")
        self._tune_loaded = False
        if self.tune_file and os.path.exists(self.tune_file):
            from .. import ops

            ops.load_tuning(self.tune_file)
            self._tune_loaded = True

    def _bytes(self, shape, dtype) -> int:
        n = 1
        for s in shape:
            n *= s
        return n * torch.empty((), dtype=dtype).element_size()

    def build(self, warm_s: Optional[float] = None) -> "EngineRunner":
        """Capture every session's graphs, then warm the device: ``warm_s``
        seconds (default RDB_ENGINE_WARM_S, 0.25) of back-to-back replays of the
        largest bucket on every compute stream, so the first served batches do not
        run at idle clocks / cold caches (what a production replica does before it
        reports ready).  The replays write only the sessions' own output slots."""
        import os

        t0 = time.perf_counter()
        self.pools = [torch.cuda.graph_pool_handle() for _ in range(self.compute_streams)]
        for s in self.sessions:
            self._capture(s, live=False)
        torch.cuda.synchronize()
        if self.tune_file and not self._tune_loaded:
            from .. import ops

            ops.save_tuning(self.tune_file)
        self.capture_s = time.perf_counter() - t0
        self.warm_device(float(os.environ.get("RDB_ENGINE_WARM_S", "0.25")) if warm_s is None else warm_s)
        return self

    def warm_device(self, seconds: float) -> int:
        """Replay the largest bucket's graphs of every session on the compute
        streams for ``seconds``; returns the number of replays (before start()).
        A model whose captured forward has side effects (state it updates per
        call) opts out with ``warm_replay = False``."""
        if seconds <= 0:
            return 0
        streams = [torch.cuda.Stream(device=self.device) for _ in range(self.compute_streams)]
        cur = torch.cuda.current_stream()
        n = 0
        t_end = time.perf_counter() + seconds
        while time.perf_counter() < t_end:
            for st in streams:
                st.wait_stream(cur)
            for s in self.sessions:
                if not s.graphs or not getattr(s.model, "warm_replay", True):
                    continue
                for slot, g in enumerate(s.graphs[-1]):
                    with torch.cuda.stream(streams[slot % self.compute_streams]):
                        g.replay()
                    n += 1
            for st in streams:
                cur.wait_stream(st)
            torch.cuda.synchronize(self.device)
            if n == 0:          # nothing to replay (no graphs, or every model opted out)
                break
        return n

    def _capture(self, s: SessionSpec, live: bool) -> None:
        """Warm up, (tune,) capture and register one session's graphs.  ``live``:
        the engine is already serving other sessions -- the session gets its own
        graph memory pools (so unloading frees them), captures in thread-local
        mode (the engine's threads keep launching meanwhile) and is registered
        inactive; ``add_session`` activates it once every graph is in place."""
        import os

        dev = torch.device("cuda", self.device)
        m = s.model
        if getattr(m, "fold_ln_auto", False):
            # deferred LayerNorm (models/bert.py) shortens ONE batch's forward
            # (-3.5 % at bs32) but its heavier GEMM epilogues cost throughput
            # when batches overlap on several compute streams, where the
            # LayerNorm kernels already hide under the other stream's GEMMs
            # (profiles/bert_fold_ln_ab.json)
            m.fold_ln = m.auto_fold_ln(self.compute_streams) if hasattr(m, "auto_fold_ln") \
                else self.compute_streams == 1
            if os.environ.get("RDB_FOLD_LN") in ("0", "1"):      # A/B override
                m.fold_ln = os.environ["RDB_FOLD_LN"] == "1"
        if getattr(m, "fuse_residual_ln", False) and self.compute_streams > 1:
            # the LayerNorm GEMM epilogue's row-panel wait assumes the whole grid
            # is resident; a second compute stream sharing the CUs breaks that
            # (a timed-out wait would give a wrong LayerNorm): refuse it here
            import warnings

            warnings.warn("RDB_BERT_LNOUT needs compute_streams == 1; using the LayerNorm kernels")
            m.fuse_residual_ln = False
        if hasattr(m, "refresh_folded_weights"):
            m.refresh_folded_weights()   # graphs capture weights derived from the CURRENT ones
        buckets = sorted(set(s.buckets or default_buckets(s.max_batch)))
        if buckets[-1] != s.max_batch:
            buckets.append(s.max_batch)
        s.buckets = buckets
        in_bytes = self._bytes(m.input_shape, m.input_dtype)
        out_bytes = self._bytes(m.output_shape, m.output_dtype)
        add = self.engine.readd_session if live else self.engine.add_session
        s.sid = add(s.queue, s.max_batch, s.max_wait_s, buckets, in_bytes, out_bytes, s.priority, s.slo_ms,
                    s.drop_stale)
        pools = [torch.cuda.graph_pool_handle() for _ in range(self.compute_streams)] if live else self.pools
        s.pools = pools
        s.inputs = []
        for slot in range(self.depth):
            x = torch.zeros((s.max_batch,) + tuple(m.input_shape), dtype=m.input_dtype, device=dev)
            if hasattr(m, "example_input") and m.input_dtype in (torch.int32, torch.int64):
                x.copy_(m.example_input(s.max_batch, seed=slot, device=dev))
            s.inputs.append(x)
            self.engine.set_input(s.sid, slot, x.data_ptr())
        # warm up every bucket eagerly on a side stream (lazy init, caches,
        # per-shape kernel autotuning)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for b in buckets:
                for _ in range(self.warmup_iters):
                    m.forward(s.inputs[0][:b])
        side.synchronize()
        self.check_model_errors(m)
        if self.tune_in_context and not self._tune_loaded and not live:
            ctx_streams = int(os.environ.get("RDB_TUNE_CONTEXT_STREAMS", self.compute_streams))
            self.tuning_changes.update(self._tune_in_context(m, s.inputs[0][:buckets[-1]], dev, ctx_streams))
        s.graphs = [[None] * self.depth for _ in buckets]
        s.outputs = [[None] * self.depth for _ in buckets]
        mode = "thread_local" if live else "global"
        from .. import ops

        # one split-K workspace per compute stream, shared by every graph replayed
        # on that stream (they run in stream order): no memset node per split-K launch
        if not getattr(self, "_stream_ws", None):
            self._stream_ws = [ops.splitk_workspace(dev) for _ in range(self.compute_streams)]
        for bi, b in enumerate(buckets):
            for slot in range(self.depth):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pools[slot % self.compute_streams], stream=side,
                                      capture_error_mode=mode), \
                        ops.capture_splitk_workspace(self._stream_ws[slot % self.compute_streams]):
                    y = m.forward(s.inputs[slot][:b])
                if not y.is_contiguous():
                    raise RuntimeError("servable model output must be contiguous")
                s.graphs[bi][slot] = g
                s.outputs[bi][slot] = y
                self.engine.set_graph(s.sid, bi, slot, g.raw_cuda_graph_exec(), y.data_ptr())
        # first launch of a graph exec uploads it (kernel-arg buffers, AQL
        # packet templates); do that here for every (bucket, slot) so no
        # served batch pays it
        with torch.cuda.stream(side):
            for row in s.graphs:
                for g in row:
                    g.replay()
        side.synchronize()
        # latency estimates per bucket (used for stale-request dropping)
        for bi, b in enumerate(buckets):
            g = s.graphs[bi][0]
            with torch.cuda.stream(side):
                g.replay()
            side.synchronize()
            t = time.perf_counter()
            with torch.cuda.stream(side):
                for _ in range(3):
                    g.replay()
            side.synchronize()
            # timed while the engine may be serving other sessions (live add):
            # only a seed -- the first batch that runs alone replaces it
            self.engine.set_latency_estimate(s.sid, bi, (time.perf_counter() - t) / 3 * 1e3, live)
        self.check_model_errors(m)

    def check_model_errors(self, m=None) -> None:
        """Raise if a kernel reported a silent-wrong-result condition: the
        LayerNorm GEMM epilogue's bounded row-panel wait timed out (its output
        is then wrong, ops.ln_out_error).  Run after warm-up, after the latency
        replays, and periodically by the replica process."""
        models = [m] if m is not None else [s.model for s in self.sessions if s.model is not None]
        if any(getattr(x, "fuse_residual_ln", False) for x in models):
            from .. import ops

            if ops.ln_out_error(self.device):
                raise RuntimeError("LayerNorm GEMM epilogue: a row-panel wait timed out (wrong LayerNorm); "
                                   "run without RDB_BERT_LNOUT")

    def add_session(self, spec: SessionSpec, activate: bool = True) -> int:
        """Load a model into the RUNNING engine (planner placement): capture its
        graphs beside the live sessions, then activate it at the launcher's next
        batch boundary.  Returns the index into ``self.sessions``."""
        t0 = time.perf_counter()
        self._capture(spec, live=True)
        spec.capture_s = time.perf_counter() - t0
        self.sessions.append(spec)
        if activate:
            self.engine.set_session_active(spec.sid, True)
        return len(self.sessions) - 1

    def retire_session(self, index: int, timeout_s: float = 10.0) -> bool:
        """Unload: stop the session at a batch boundary, wait for its in-flight
        batches, then drop its graphs, buffers and (our reference to) the model,
        so its HBM -- weights and private graph pools -- returns to the allocator
        (``torch.cuda.empty_cache`` releases it to the device)."""
        s = self.sessions[index]
        if s.sid < 0 or s.graphs is None:
            return True
        if not self.engine.retire_session(s.sid, timeout_s):
            return False
        s.graphs = None
        s.outputs = None
        s.inputs = None
        s.pools = None
        s.model = None
        torch.cuda.synchronize(self.device)
        torch.cuda.empty_cache()
        return True

    @staticmethod
    def _tune_in_context(m, x, dev, streams: int = 1) -> dict:
        """Coordinate-descent tile choice on the WHOLE forward, timed the way the
        engine runs it: ``streams`` captured forwards replayed concurrently on
        ``streams`` streams (the throughput regime of a multi-stream replica),
        so tiles that trade single-batch latency for CU efficiency can win."""
        from .. import ops

        with ops.record_tuning_keys() as keys:
            with torch.no_grad():
                m.forward(x)
        torch.cuda.synchronize()
        if not keys:
            return {}
        streams = max(1, streams)
        pools = [torch.cuda.graph_pool_handle() for _ in range(streams)]
        sts = [torch.cuda.Stream(device=dev) for _ in range(streams)]
        sk_ws = [ops.splitk_workspace(dev) for _ in range(streams)]     # as the engine's graphs get them

        def time_forward() -> float:
            gs = []
            for i in range(streams):
                g = torch.cuda.CUDAGraph()
                sts[i].wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(sts[i]):
                    with torch.cuda.graph(g, pool=pools[i], stream=sts[i]), ops.capture_splitk_workspace(sk_ws[i]):
                        m.forward(x)
                gs.append(g)
            torch.cuda.synchronize()
            cur = torch.cuda.current_stream()

            def burst(n):
                for st in sts:
                    st.wait_stream(cur)
                for _ in range(n):
                    for g, st in zip(gs, sts):
                        with torch.cuda.stream(st):
                            g.replay()
                for st in sts:
                    cur.wait_stream(st)

            burst(3)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            best = float("inf")
            for _ in range(3):
                e0.record()
                burst(10)
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) / (10 * streams))
            del gs
            return best

        return ops.tune_in_context(time_forward, keys=list(keys), min_gain=0.02)

    def start(self):
        self.engine.start()
        return self

    def set_duty_cycle(self, cycle_ms: float, shares_ms: Optional[Sequence[float]] = None):
        """Nexus plan -> engine: duty cycle and per-session GPU-time shares (ms)."""
        self.engine.set_duty_cycle(cycle_ms)
        for s, share in zip(self.sessions, shares_ms or []):
            self.engine.set_duty_share(s.sid, share)

    def set_active(self, session: int, on: bool):
        """Load/unload a model at a batch boundary (planner re-placement)."""
        self.engine.set_session_active(self.sessions[session].sid, on)

    def stop(self):
        self.engine.stop()

    def stats(self):
        return self.engine.stats()

    def latency_estimates(self, session: int = 0) -> dict:
        """Per bucket size: (solo ms, overlapped-span ms).  The solo estimate
        (latency replays, then batches that overlapped no other batch) charges
        duty-cycle shares and gates backfill; the overlapped span EMA predicts
        completion for stale-request dropping (engine.cpp Session::est_ns)."""
        s = self.sessions[session]
        return {b: tuple(self.engine.latency_estimate(s.sid, bi)) for bi, b in enumerate(s.buckets)}

    def error(self) -> str:
        return self.engine.error()
