"""Entry point of a replica PROCESS (one per GPU slot), spawned by the controller.

    python -m ray_dynamic_batching_amd.serve.replica_main --spec S --replica R --gpu G

* servable-model deployments -> the native replica engine (no Python on the
  request path);
* any other deployment -> a Python worker: a reader thread pops requests from
  the shm ring (GIL released while waiting), the user-code event loop runs the
  calls (``@serve.batch`` batches them), results go back through the
  completion ring.  Streaming methods send one completion per item.
* a heartbeat thread refreshes the replica's shm heartbeat; the user's
  ``check_health`` runs every ``health_check_period_s``; SIGTERM drains.
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import os
import signal
import sys
import threading
import time
import traceback

logger = logging.getLogger("ray_dynamic_batching_amd.replica")

KIND_TENSOR, KIND_PICKLE, KIND_STREAM_ITEM, KIND_STREAM_END = 0, 1, 2, 3
ST_OK, ST_DROPPED, ST_ERROR = 0, 1, 2


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--spec", required=True)
    ap.add_argument("--replica", type=int, required=True)
    ap.add_argument("--gpu", default="")
    a = ap.parse_args(argv)
    logging.basicConfig(level=os.environ.get("RDB_LOG_LEVEL", "INFO"),
                        format=f"%(asctime)s replica{a.replica} %(levelname)s %(message)s")
    import cloudpickle

    with open(a.spec, "rb") as f:
        spec = cloudpickle.load(f)
    from ..runtime import job as rjob
    from .config import DeploymentConfig
    from .context import ReplicaContext, _set_replica_context

    cfg = DeploymentConfig(**spec["config"])
    job = rjob.Job(spec["job"], create=False)
    r = a.replica
    gpu = int(a.gpu.split(",")[0]) if a.gpu else -1
    from ..parallel.rendezvous import TPEnv

    tp = TPEnv.from_env()
    follower = tp is not None and tp.rank > 0     # TP ranks 1..N-1: no replica slot of their own
    stop = threading.Event()
    if follower:
        # a follower blocks inside collectives: let SIGTERM end it at once (the
        # agent stops / restarts the whole group together)
        signal.signal(signal.SIGTERM, signal.SIG_DFL)
    else:
        job.set_replica_status(r, 1, gpu, os.getpid())

        def _term(*_):
            stop.set()
        signal.signal(signal.SIGTERM, _term)
    if not follower and os.environ.get("RDB_AGENT_SOCKET") and os.environ.get("RDB_METRICS_KEY"):
        from ..utils import user_metrics

        user_metrics.start_publisher(os.environ["RDB_AGENT_SOCKET"], os.environ["RDB_METRICS_KEY"])

    parent = os.getppid()

    def heartbeat():
        while not stop.is_set():
            if not follower:
                job.heartbeat(r)
            # orphaned (the controller / node agent process died without
            # terminating us): leave instead of serving a job nobody supervises;
            # a recovering controller starts its own replicas
            if os.getppid() != parent:
                logger.warning("node agent (pid %d) is gone: replica exits", parent)
                stop.set()
                os._exit(3)
            time.sleep(0.25)
    threading.Thread(target=heartbeat, daemon=True).start()

    ctx = ReplicaContext(spec["app_name"], spec["deployment"], f"{spec['app_name']}#{spec['deployment']}#{r}", r,
                         None, cfg.max_ongoing_requests, gpu)
    _set_replica_context(ctx)
    from .logging_utils import configure_replica_logger

    lcfg = cfg.get_logging_config()
    ctx.logger = configure_replica_logger(spec["app_name"], spec["deployment"], r, ctx.replica_id, lcfg,
                                          capture_user_logs=True)
    ctx.logger.info("replica starting (pid %d, gpu %s)", os.getpid(), gpu)
    try:
        if tp is not None:
            return _run_tp(spec, cfg, r, stop, tp, gpu)
        if spec.get("servable"):
            return _run_engine(spec, cfg, job, r, stop)
        return _run_python(spec, cfg, job, r, stop, ctx)
    except Exception:
        logger.error("replica failed:\n%s", traceback.format_exc())
        if not follower:
            job.set_replica_status(r, 4, gpu, os.getpid())
        return 1


def _run_tp(spec, cfg, r, stop, tp, gpu) -> int:
    """One rank of a tensor-parallel replica (the agent gang-spawned every rank
    of the group).  Ranks meet through the agent's KV, build their model shard
    and run the TPReplica loop: rank 0 pops batches from the replica's queue and
    broadcasts them, every rank runs its shard's forward (collectives inside),
    rank 0 answers.  Any rank failing ends the process, and the agent restarts
    the whole group."""
    import torch

    from ..parallel import collective as col
    from ..parallel.rendezvous import init_tp_group
    from ..runtime.tp_replica import TPReplica, bcast_name

    sv = spec.get("servable")
    if not sv:
        raise RuntimeError("tensor_parallel_size > 1 needs a servable model deployment (serve.model_deployment)")
    use_gpu = gpu >= 0 and not os.environ.get("RDB_NO_GPU") and torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(0)
    backend = cfg.tp_backend or ("nccl" if use_gpu else "gloo")
    t0 = time.time()
    init_tp_group(backend, "tp", tp)
    logger.info("TP rank %d/%d joined group %s epoch %d over %s in %.2fs", tp.rank, tp.world, tp.group, tp.epoch,
                backend, time.time() - t0)
    if use_gpu and os.environ.get("RDB_TP_XGMI", "0") == "1":
        # the custom xGMI all-reduce (fused residual + RMSNorm), over RCCL or -- a TP
        # group rehearsed on ONE GPU, where RCCL refuses two ranks per device -- gloo
        # host groups (IPC handles exchanged over either)
        col.enable_xgmi("tp")
    factory = sv["factory"]
    model = factory(device="cuda" if use_gpu else "cpu", tp_rank=tp.rank, tp_size=tp.world, group_name="tp")
    if use_gpu and tp.world > 1 and os.environ.get("RDB_TP_LINE_UP", "0") == "1" and hasattr(model, "pre_collective"):
        # rehearsal of a TP group on ONE GPU: every rank drains its stream and
        # meets the others before each all-reduce (a rank spinning in the xGMI
        # kernel would hold the CU slots a peer's GEMM needs); never on a node
        # where each rank has its own GPU
        def _line_up():
            torch.cuda.synchronize()
            col.barrier("tp")
        model.pre_collective = _line_up
    eng = cfg.engine
    buckets = eng.buckets or [1, 2, 4, 8, 16, 32][: max(1, sv["max_batch_size"].bit_length())]
    buckets = sorted({min(b, sv["max_batch_size"]) for b in buckets} | {sv["max_batch_size"]})
    ring = bcast_name(tp.group, tp.epoch)
    use_graphs = use_gpu and os.environ.get("RDB_TP_GRAPHS", "1") == "1"
    if use_graphs and os.environ.get("RDB_TP_NATIVE", "1") == "1":
        return _run_tp_native(spec, cfg, r, stop, tp, model, buckets, ring)
    rep = TPReplica(model, spec["job"] if tp.rank == 0 else None, r, r, buckets, group="tp",
                    max_wait_s=sv["batch_wait_timeout_s"], use_graphs=use_graphs, gpu_index=gpu, ring=ring)
    rep.capture()                      # rank 0 marks the replica READY
    while True:
        if tp.rank == 0 and stop.is_set():
            rep.stop_all()
            break
        if rep.step(0.05) < 0:
            break
    logger.info("TP rank %d leaves after %d batches / %d requests", tp.rank, rep.batches, rep.requests)
    return 0


def _run_tp_native(spec, cfg, r, stop, tp, model, buckets, ring) -> int:
    """GPU ranks of a TP replica on the native engine (runtime/tp_replica.py
    NativeTP): rank 0 a leader engine on the replica's queue, the others
    followers of its broadcast ring; no Python per batch on any rank."""
    from ..runtime.tp_replica import NativeTP

    sv = spec["servable"]
    eng = cfg.engine
    ntp = NativeTP(model, spec["job"], r, buckets, tp.rank, tp.world, "tp", ring, sv["max_batch_size"],
                   sv["batch_wait_timeout_s"], pipeline_depth=min(eng.pipeline_depth, 2),
                   batch_policy=eng.batch_policy)
    ntp.start()
    logger.info("TP rank %d/%d: native engine (%s), ring %s", tp.rank, tp.world,
                "leader" if tp.rank == 0 else "follower", ring)
    code = 0
    while not (tp.rank == 0 and stop.is_set()):
        why = ntp.check()
        if why:
            if why != "stopped":
                logger.error("TP rank %d: %s", tp.rank, why)
                code = 2
            break
        stop.wait(0.2)
    ntp.stop()
    st = ntp.stats()
    logger.info("TP rank %d leaves after %d batches / %d requests", tp.rank, st["batches"], st["requests"])
    return code


def _run_engine(spec, cfg, job, r, stop) -> int:
    import torch

    sv = spec["servable"]
    torch.cuda.set_device(0)
    factory = sv["factory"]
    try:
        model = factory(device="cuda")
    except TypeError:
        model = factory()
    runner = build_engine_runner(spec, cfg, r, model)
    logger.info("engine: %d compute streams, depth %d, policy %s, stagger %d us, tile table %s",
                runner.compute_streams, runner.depth, runner.batch_policy, runner.stagger_us,
                os.path.basename(runner.tune_file) or "tuned at start-up")
    runner.start()   # sets the replica READY in shm
    while not stop.is_set():
        err = runner.error()
        if not err:
            try:
                runner.check_model_errors()
            except RuntimeError as e:
                err = str(e)
        if err:
            logger.error("engine error: %s", err)
            return 2
        stop.wait(0.2)
    runner.stop()
    return 0


def build_engine_runner(spec, cfg, r, model, runner_cls=None):
    """The replica's native engine, configured from the deployment's
    ``EngineConfig`` -- the same knobs ``bench.py`` runs the headline replica
    with (compute streams, pipeline depth, batch policy, stagger, the shipped
    tile table resolved by model signature, device warm-up)."""
    from ..runtime.engine import EngineRunner, SessionSpec, resolve_tile_table

    sv = spec["servable"]
    eng = cfg.engine
    s = SessionSpec(model=model, queue=r, max_batch=sv["max_batch_size"], max_wait_s=sv["batch_wait_timeout_s"],
                    buckets=eng.buckets, priority=cfg.priority, slo_ms=float(cfg.slo_ms or 0.0),
                    drop_stale=cfg.drop_stale)
    table = resolve_tile_table(eng.tile_table, model, sv["max_batch_size"], eng.compute_streams, eng.pipeline_depth)
    runner = (runner_cls or EngineRunner)(spec["job"], r, [s], pipeline_depth=eng.pipeline_depth,
                                          zero_copy=eng.zero_copy, compute_streams=eng.compute_streams,
                                          batch_policy=eng.batch_policy, stagger_us=eng.stagger_us,
                                          tile_table=table)
    return runner.build(warm_s=eng.warm_s)


def _run_python(spec, cfg, job, r, stop, ctx) -> int:
    import cloudpickle

    from ..runtime import job as rjob
    from . import tensor_wire
    from .handle import RequestMeta
    from .replica import UserCallable

    loop = asyncio.new_event_loop()
    asyncio.set_event_loop(loop)
    from .logging_utils import AccessLog

    lcfg = cfg.get_logging_config()
    user = UserCallable(spec["func_or_class"], spec["init_args"], spec["init_kwargs"], cfg.user_config,
                        AccessLog(ctx.logger, lcfg is None or lcfg.enable_access_log))
    ctx.servable_object = user.obj
    cons = rjob.Consumer(job, [r])
    inflight = [0]
    from . import multiplex
    from .router import mux_hash

    multiplex.set_publisher(lambda ids: job.set_queue_models(r, [mux_hash(i) for i in ids]))
    from ..utils.faults import injector

    faults = injector()

    async def handle(req):
        rid, q, client, kind, t_sub, dl, payload = req
        if faults.drop_request():   # injected message loss: the router re-dispatches
            cons.complete(client, rid, q, int(rjob.Status.REPLICA_DIED), t_sub, b"", KIND_PICKLE)
            inflight[0] -= 1
            return
        try:
            if kind == tensor_wire.KIND_TENSOR_CALL or (kind == KIND_TENSOR and payload[:4] == tensor_wire.MAGIC):
                # one array argument as raw bytes in the ring slot (no unpickling): a view of the payload
                # (kind 0 + the wire magic: a native client -- LoadGen -- submitting encoded calls)
                method, arg, mux, user_rid, stream = tensor_wire.decode_call(payload)
                args, kwargs = (arg,), {}
            else:
                method, args, kwargs, mux, stream, user_rid = cloudpickle.loads(payload)
            meta = RequestMeta(user_rid, method, mux, stream, spec["app_name"], spec["deployment"])
            if stream:
                items = []

                def emit(k, v):
                    if k == "item":
                        cons.complete(client, rid, q, ST_OK, t_sub, cloudpickle.dumps(v), KIND_STREAM_ITEM)
                    elif k == "end":
                        cons.complete(client, rid, q, ST_OK, t_sub, b"", KIND_STREAM_END)
                    else:
                        cons.complete(client, rid, q, ST_ERROR, t_sub, _dump_exc(v), KIND_PICKLE)
                await user.call_stream(meta, args, kwargs, emit)
            else:
                res = await user.call(meta, args, kwargs)
                if tensor_wire.result_encodable(res):
                    out, okind = tensor_wire.encode_result(res), tensor_wire.KIND_TENSOR_RESULT
                else:
                    out, okind = cloudpickle.dumps(res), KIND_PICKLE
                if not cons.complete(client, rid, q, ST_OK, t_sub, out, okind):
                    logger.error("result of request %d too large for the completion slot", rid)
        except Exception as e:
            cons.complete(client, rid, q, ST_ERROR, t_sub, _dump_exc(e), KIND_PICKLE)
        finally:
            inflight[0] -= 1

    def reader():
        while not stop.is_set():
            try:
                reqs = cons.pop(256, 50_000_000)
            except Exception:  # pragma: no cover
                break
            if reqs:
                faults.before_batch()
                inflight[0] += len(reqs)
                for req in reqs:
                    asyncio.run_coroutine_threadsafe(handle(req), loop)
        loop.call_soon_threadsafe(loop.stop)

    async def health():
        fails = 0
        while not stop.is_set():
            await asyncio.sleep(cfg.health_check_period_s)
            try:
                await asyncio.wait_for(user.check_health(), cfg.health_check_timeout_s)
                fails = 0
            except Exception:
                fails += 1
                logger.warning("check_health failed (%d):\n%s", fails, traceback.format_exc())
                if fails >= cfg.health_check_failure_threshold:
                    job.set_replica_status(r, 4, ctx.gpu if ctx.gpu is not None else -1, os.getpid())
                    stop.set()

    t = threading.Thread(target=reader, daemon=True)
    job.set_replica_status(r, 2, ctx.gpu if ctx.gpu is not None else -1, os.getpid())
    t.start()
    loop.create_task(health())
    loop.run_forever()
    t.join(5)
    # graceful drain of in-flight requests
    deadline = time.time() + cfg.graceful_shutdown_timeout_s
    while inflight[0] > 0 and time.time() < deadline:
        loop.run_until_complete(asyncio.sleep(0.01))
    user.destroy()
    return 0


def _dump_exc(e: BaseException) -> bytes:
    import cloudpickle

    try:
        return cloudpickle.dumps(e)
    except Exception:
        from .exceptions import RayServeException

        return cloudpickle.dumps(RayServeException(f"{type(e).__name__}: {e}"))


if __name__ == "__main__":
    sys.exit(main())
