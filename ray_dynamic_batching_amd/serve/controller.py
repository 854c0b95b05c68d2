"""Serve controller + node agent (single node, in the driver process).

Reference parity:
* ServeController control loop every 0.1 s (serve/_private/controller.py:370-471):
  deployment state update, health checks, autoscaling;
* DeploymentState replica state machine (deployment_state.py): start, health-check,
  restart dead replicas, scale up/down, graceful drain;
* raylet worker pool + GPU allocation + GCS health checks / actor restarts
  (node_manager / worker_pool / resource_instance_set.cc /
  gcs_health_check_manager.cc / gcs_actor_manager.cc) are the NATIVE node agent
  (runtime/csrc/node_agent.cpp): it owns the GPU slots, spawns the replica
  PROCESSES pinned with HIP_VISIBLE_DEVICES, watches exit status + shm
  heartbeats, fails a dead replica's pending requests, bumps its generation and
  restarts it with exponential back-off;
* config checkpoint (controller.py:510-563 KV): the last applied application
  config is written to the agent's persistent KV (and a JSON file for the CLI);
  the agent also answers PING/STATUS/KV_* on a Unix socket.
"""
from __future__ import annotations

import atexit
import json
import logging
import os
import sys
import tempfile
import threading
import time
import traceback
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

from .api import Application, Deployment
from .autoscaling_policy import AutoscalingMetrics, AutoscalingState
from .config import CONTROL_LOOP_INTERVAL_S, DeploymentConfig
from .exceptions import RayServeException
from .handle import DeploymentHandle
from .router import LocalRouter, ShmRouter
from .replica import LocalReplica

logger = logging.getLogger("ray_dynamic_batching_amd.serve")

_CONTROLLER: Optional["ServeController"] = None
_CTRL_LOCK = threading.Lock()


def discovery_file() -> str:
    return os.environ.get("RDB_SERVE_DISCOVERY", os.path.join(tempfile.gettempdir(), f"rdb_serve_{os.getuid()}.json"))


def get_controller(create: bool = True) -> Optional["ServeController"]:
    global _CONTROLLER
    with _CTRL_LOCK:
        if _CONTROLLER is None and create:
            _CONTROLLER = ServeController()
        return _CONTROLLER


_ROUTE_JOBS: Dict[str, Any] = {}


def _read_routes(job_name: Optional[str], table: Optional[str]) -> Dict[str, Any]:
    """Latest routing table: the seqlock snapshot the controller publishes in the
    job segment (live updates), else the file written at spawn time."""
    if job_name:
        from ..runtime import job as rjob

        j = _ROUTE_JOBS.get(job_name)
        if j is None:
            j = _ROUTE_JOBS[job_name] = rjob.Job(job_name, create=False)
        version, blob = j.read_snapshot()
        if version:
            return json.loads(blob)
    with open(table) as f:
        return json.load(f)


def lookup_router(app_name: str, deployment: str):
    """Router for a handle: the controller in the driver, the routing table in
    a replica process (handles shipped for composition)."""
    table = os.environ.get("RDB_ROUTING_TABLE")
    job_name = os.environ.get("RDB_JOB")
    if (table or job_name) and _CONTROLLER is None:
        routes = _read_routes(job_name, table)
        r = routes.get(f"{app_name}/{deployment}")
        if r is None:
            raise RayServeException(f"no route for {app_name}/{deployment}")
        codec = None
        if r.get("codec"):
            from .servable import TensorCodec
            import torch

            c = r["codec"]
            codec = TensorCodec(c["input_shape"], getattr(torch, c["input_dtype"]), c["output_shape"],
                                getattr(torch, c["output_dtype"]))
        return ShmRouter(r["job"], r["model_id"], deployment, r.get("max_queued", -1), codec,
                         retry_timeout_s=r.get("retry_timeout_s", 60.0), max_retries=r.get("max_retries", 3))
    ctrl = get_controller(create=False)
    if ctrl is None:
        raise RayServeException("serve is not running; call serve.run() first")
    return ctrl.router_for(app_name, deployment)


@dataclass
class ProcReplica:
    slot: int                 # replica index in the job segment (== queue id)
    proc_id: int = -1         # node-agent process handle (rank 0's, for a TP replica)
    group_id: int = -1        # node-agent gang of a tensor-parallel replica
    alloc: Any = None
    started_at: float = 0.0
    ready: bool = False
    restarts: int = 0
    next_restart_at: float = 0.0
    health_failures: int = 0
    draining: bool = False


@dataclass
class DeploymentState:
    app_name: str
    name: str
    deployment: Deployment
    app: Application
    config: DeploymentConfig
    mode: str
    model_id: int = 0
    router: Any = None
    target: int = 1
    local_replicas: List[LocalReplica] = field(default_factory=list)
    proc_replicas: List[ProcReplica] = field(default_factory=list)
    autoscaler: Optional[AutoscalingState] = None
    as_metrics: Optional[AutoscalingMetrics] = None   # look-back averaged replica ongoing counts
    init_args: tuple = ()
    init_kwargs: dict = field(default_factory=dict)
    next_index: int = 0
    codec: Any = None
    spec_path: str = ""
    slots: List[int] = field(default_factory=list)   # job replica slots reserved for this deployment


class ServeController:
    def __init__(self):
        from ..runtime import agent as ragent
        from ..runtime.resources import detect_num_gpus

        self.apps: Dict[str, Dict[str, DeploymentState]] = {}
        self.ingress: Dict[str, str] = {}
        self.route_prefixes: Dict[str, Optional[str]] = {}
        self.proxy = None
        self.grpc_proxy = None
        self.jobs: Dict[str, Any] = {}            # app -> job segment handle (process mode)
        self._rings_ready: Dict[str, set] = {}    # job name -> request rings initialised (NUMA-bound)
        self.lock = threading.RLock()
        self._clock = time.monotonic          # autoscaling look-back windows (tests may fake it)
        self.workdir = tempfile.mkdtemp(prefix="rdb_serve_")
        # RDB_SERVE_KV names a STABLE checkpoint location (the GCS-KV role): the
        # JSON document for the CLI and, beside it, the agent's persistent KV --
        # a controller started later on the same path recovers from them
        self.kv_path = os.environ.get("RDB_SERVE_KV", os.path.join(self.workdir, "serve_kv.json"))
        agent_kv = (self.kv_path + ".agent.bin") if os.environ.get("RDB_SERVE_KV") else \
            os.path.join(self.workdir, "agent_kv.bin")
        self.agent = ragent.NodeAgent(detect_num_gpus(), 0.0, agent_kv)
        self.app_modes: Dict[str, str] = {}
        self.app_blobs: Dict[str, Dict[str, Any]] = {}     # app -> how to rebuild it (checkpoint)
        self.recovered: List[str] = []
        self.agent_socket = os.path.join(self.workdir, "agent.sock")
        try:
            self.agent.serve(self.agent_socket)
            with open(discovery_file(), "w") as f:   # lets `serve status` find the live agent
                json.dump(dict(pid=os.getpid(), socket=self.agent_socket, kv=self.kv_path), f)
        except (RuntimeError, OSError):  # pragma: no cover - control RPC is optional
            self.agent_socket = ""
        self.default_mode = os.environ.get("RDB_SERVE_MODE", "auto")
        self.shutdown_requested = threading.Event()   # set by a remote `serve shutdown`
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._control_loop, name="rdb-serve-controller", daemon=True)
        self._thread.start()
        atexit.register(self.shutdown)
        if os.environ.get("RDB_SERVE_KV") and os.environ.get("RDB_SERVE_RECOVER", "1") != "0":
            try:
                self.recover()
            except Exception:  # pragma: no cover - a bad checkpoint must not block start-up
                logger.error("serve: recovery from %s failed:\n%s", self.kv_path, traceback.format_exc())

    def configure(self, mode: str = None, http_options: Optional[Dict[str, Any]] = None,
                  grpc_options: Optional[Dict[str, Any]] = None, **_):
        if mode:
            self.default_mode = mode
        if http_options is not None and self.proxy is None:
            from .http_proxy import HTTPProxy

            self.proxy = HTTPProxy(self, http_options.get("host", "127.0.0.1"),
                                   int(http_options.get("port", 8000))).start()
        if grpc_options is not None and self.grpc_proxy is None:
            from .grpc_proxy import GRPCProxy

            o = dict(grpc_options)
            self.grpc_proxy = GRPCProxy(self, o.get("host", "127.0.0.1"), int(o.get("port", 9000)),
                                        request_types=o.get("request_types"),
                                        streaming_methods=o.get("streaming_methods", ()),
                                        timeout_s=float(o.get("request_timeout_s", 600.0))).start()

    # ------------------------------------------------------------------ deploy
    def _resolve_mode(self, app: Application, mode: Optional[str]) -> str:
        mode = mode or self.default_mode
        if mode in ("local", "process"):
            return mode
        wants_gpu = any(a.deployment.config.num_gpus > 0 for a in app.walk())
        return "process" if wants_gpu else "local"

    def deploy_application(self, app: Application, name: str = "default", route_prefix: Optional[str] = "/",
                           mode: Optional[str] = None) -> DeploymentHandle:
        with self.lock:
            if name in self.apps:
                self.delete_application(name)
            mode = self._resolve_mode(app, mode)
            graph = app.walk()
            names = [a.deployment.name for a in graph]
            if len(set(names)) != len(names):
                raise RayServeException(f"duplicate deployment names in application {name!r}: {names}")
            states: Dict[str, DeploymentState] = {}
            self.apps[name] = states
            self.ingress[name] = app.deployment.name
            self.route_prefixes[name] = route_prefix
            if mode == "process":
                self._create_job(name, graph)
            for mid, a in enumerate(graph):
                d = a.deployment
                cfg = d.config
                st = DeploymentState(name, d.name, d, a, cfg, mode, model_id=mid)
                st.target = cfg.initial_num_replicas()
                if cfg.autoscaling_config is not None:
                    st.autoscaler = AutoscalingState(cfg.autoscaling_config)
                    st.as_metrics = AutoscalingMetrics(cfg.autoscaling_config)
                # composition: bound Applications become handles
                st.init_args = tuple(self._to_handle(name, x) for x in a.init_args)
                st.init_kwargs = {k: self._to_handle(name, v) for k, v in a.init_kwargs.items()}
                sv = getattr(d, "servable", None)
                if sv is not None and mode == "local" and not st.init_args:
                    # local mode runs the servable eagerly behind @serve.batch
                    st.init_args = (sv["factory"], sv["max_batch_size"], sv["batch_wait_timeout_s"])
                    st.init_kwargs = dict(device="cuda" if cfg.num_gpus > 0 else "cpu")
                if mode == "local":
                    st.router = LocalRouter(d.name, cfg.max_queued_requests)
                else:
                    self._prepare_process_deployment(st)
                states[d.name] = st
            if mode == "process":
                self._write_routing_table(name)
            for st in states.values():
                self._reconcile(st, wait=True)
            self.app_modes[name] = mode
            self.app_blobs[name] = self._rebuild_recipe(app)
            self._checkpoint()
            return DeploymentHandle(app.deployment.name, name)

    def _to_handle(self, app_name: str, x):
        if isinstance(x, Application):
            return DeploymentHandle(x.deployment.name, app_name)
        return x

    # --- process mode plumbing ------------------------------------------------
    def _max_replicas(self, cfg: DeploymentConfig) -> int:
        if cfg.autoscaling_config is not None:
            return cfg.autoscaling_config.max_replicas
        return max(1, int(cfg.num_replicas or 1))

    def _create_job(self, app_name: str, graph: List[Application]) -> None:
        from ..runtime import job as rjob

        n = sum(self._max_replicas(a.deployment.config) for a in graph)
        req_bytes, cmp_bytes = 64 * 1024, 64 * 1024
        for a in graph:
            sv = getattr(a.deployment, "servable", None)
            if a.deployment.config.engine.request_slot_bytes:
                req_bytes = max(req_bytes, a.deployment.config.engine.request_slot_bytes)
        jname = f"serve_{os.getpid()}_{app_name}_{int(time.time() * 1000) % 10**8}"
        # request rings are initialised per replica slot at its first spawn, bound
        # to the NUMA node of the GPU it lands on (_init_ring)
        job = rjob.Job(jname, create=True, n_replicas=n, n_queues=n, n_clients=16 + n, req_capacity=1024,
                       req_slot_bytes=req_bytes, cmp_capacity=4096, cmp_slot_bytes=cmp_bytes, defer_req_rings=True)
        self.jobs[app_name] = job
        self._rings_ready[jname] = set()

    def _prepare_process_deployment(self, st: DeploymentState) -> None:
        import cloudpickle

        job = self.jobs[st.app_name]
        used = sum(len(s.slots) for s in self.apps[st.app_name].values())
        st.slots = list(range(used, used + self._max_replicas(st.config)))
        sv = getattr(st.deployment, "servable", None)
        spec = dict(app_name=st.app_name, deployment=st.name, func_or_class=st.deployment.func_or_class,
                    init_args=st.init_args, init_kwargs=st.init_kwargs, config=st.config.model_dump(),
                    job=job.info()["name"], model_id=st.model_id, servable=sv)
        st.spec_path = os.path.join(self.workdir, f"{st.app_name}.{st.name}.spec.pkl")
        with open(st.spec_path, "wb") as f:
            cloudpickle.dump(spec, f)
        if sv is not None:
            st.codec = _codec_for_servable(sv)
        st.router = ShmRouter(job.info()["name"], st.model_id, st.name, st.config.max_queued_requests, st.codec,
                              retry_timeout_s=st.config.request_retry_timeout_s,
                              max_retries=st.config.max_request_retries)

    def _write_routing_table(self, app_name: str) -> None:
        routes = {}
        for st in self.apps[app_name].values():
            r = dict(job=self.jobs[app_name].info()["name"], model_id=st.model_id,
                     max_queued=st.config.max_queued_requests, max_retries=st.config.max_request_retries,
                     retry_timeout_s=st.config.request_retry_timeout_s)
            if st.codec is not None:
                c = st.codec
                r["codec"] = dict(input_shape=list(c.input_shape), output_shape=list(c.output_shape),
                                  input_dtype=str(_torch_dtype_name(c.in_np)), output_dtype=str(_torch_dtype_name(c.out_np)))
            routes[f"{app_name}/{st.name}"] = r
        path = os.path.join(self.workdir, f"{app_name}.routes.json")
        with open(path, "w") as f:
            json.dump(routes, f)
        self._routes_path = path
        self.jobs[app_name].publish(json.dumps(routes).encode())   # live copy for replicas

    def _replica_env(self, st: DeploymentState, rep: ProcReplica, job) -> Dict[str, str]:
        env = {"RDB_ROUTING_TABLE": self._routes_path, "RDB_JOB": job.info()["name"]}
        if self.agent_socket:   # user metrics (utils.user_metrics) are published through the agent KV
            env["RDB_AGENT_SOCKET"] = self.agent_socket
            env["RDB_METRICS_KEY"] = f"{st.app_name}/{st.name}/{rep.slot}"
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        if getattr(st.deployment, "servable", None) is not None:
            # one HIP hardware queue per engine stream, in place before the replica's HIP starts
            from ..runtime.queues import ensure_hw_queues

            env["GPU_MAX_HW_QUEUES"] = os.environ.get("GPU_MAX_HW_QUEUES", "")
            if not env["GPU_MAX_HW_QUEUES"]:
                del env["GPU_MAX_HW_QUEUES"]
            ensure_hw_queues(st.config.engine.compute_streams, env)
        pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = pkg_root + os.pathsep + os.environ.get("PYTHONPATH", "")
        return env

    def _placement(self, st: DeploymentState, gpu: int) -> Dict[str, Any]:
        """NUMA placement of a replica (rank) on physical GPU ``gpu``: the node
        agent starts the process pinned to the GPU's share of its NUMA node's CPUs
        (the same split bench.py's ranks use, runtime/numa.py gpu_placement)."""
        if not st.config.engine.numa_pin or gpu < 0:
            return dict(numa_node=-1, cpus=[], cpulist="")
        from ..runtime import numa

        try:
            return numa.gpu_placement(gpu)
        except Exception as e:  # noqa: BLE001 -- placement is an optimisation, never a failure
            logger.warning("NUMA placement of GPU %d failed: %s", gpu, e)
            return dict(numa_node=-1, cpus=[], cpulist="")

    def _init_ring(self, job, slot: int, numa_node: int) -> None:
        """First use of a replica slot: bind its request ring's pages to the NUMA
        node of the replica's GPU (a shared-memory policy: it holds for every
        process that touches the pages) and write the slot sequence numbers.
        Runs before the slot's queue is configured, so no producer can pick it
        earlier; a restarted replica keeps its live ring."""
        ready = self._rings_ready.setdefault(job.info()["name"], set())
        if slot in ready:
            return
        rc = job.init_req_ring(slot, numa_node)
        if rc != 0:
            logger.info("request ring %d: mbind to node %d returned %d (left to first touch)", slot, numa_node, rc)
        ready.add(slot)

    def _spawn_tp(self, st: DeploymentState, rep: ProcReplica, owner: str) -> bool:
        """A tensor-parallel replica: one placement bundle per rank, gang-reserved;
        the agent spawns the ranks as one group (each pinned to its bundle's
        GPUs), they rendezvous through the agent KV (parallel/rendezvous.py),
        rank 0 owns the replica slot and the group restarts as one.  Reference:
        placement_group_bundles (python/ray/serve/api.py:240-259)."""
        from ..runtime.resources import visible_devices_env

        if not self.agent_socket:
            raise RayServeException("tensor-parallel replicas need the node agent's control socket (KV rendezvous)")
        n = st.config.tensor_parallel_size
        alloc = self.agent.allocate_bundles(owner, st.config.tp_bundles(),
                                            st.config.placement_group_strategy or "PACK")
        if alloc is None:
            logger.warning("no GPU capacity for TP replica %s (%d ranks)", owner, n)
            return False
        rep.alloc = alloc
        try:
            job = self.jobs[st.app_name]
            gpus = list(alloc["gpus"])
            places = [self._placement(st, int(g[0]) if len(g) else -1) for g in alloc["bundle_gpus"]]
            self._init_ring(job, rep.slot, places[0]["numa_node"] if places else -1)
            job.configure_queue(rep.slot, rep.slot, st.model_id, st.config.max_ongoing_requests,
                                float(st.config.slo_ms or 0.0), True)
            job.set_replica_status(rep.slot, 1, gpus[0] if gpus else -1, 0)
            base = self._replica_env(st, rep, job)
            argvs, envs, logs = [], [], []
            for i, g in enumerate(alloc["bundle_gpus"]):
                env = dict(base)
                env.update(visible_devices_env(list(g)))
                env["RDB_NUMA_NODE"] = str(places[i]["numa_node"])
                envs.append(env)
                argvs.append([sys.executable, "-m", "ray_dynamic_batching_amd.serve.replica_main", "--spec",
                              st.spec_path, "--replica", str(rep.slot), "--gpu", ",".join(map(str, g))])
                logs.append(os.path.join(self.workdir, f"{owner.replace('#', '.')}.rank{i}.log"))
            cpus = [list(p["cpus"]) for p in places] if any(p["cpus"] for p in places) else []
            rep.group_id = self.agent.spawn_group(owner, argvs, envs, logs, job.info()["name"], rep.slot,
                                                  [rep.slot], float(st.config.health_check_timeout_s), -1, 0.5,
                                                  30.0, cpus)
            rep.proc_id = self.agent.group_info(rep.group_id)["members"][0]
        except Exception:
            # never leak the gang reservation of a replica that did not start
            self.agent.release(owner)
            rep.alloc = None
            raise
        rep.started_at = time.time()
        rep.ready = False
        rep.health_failures = 0
        return True

    def _stop_replica_procs(self, rep: ProcReplica, grace_s: float) -> None:
        if rep.group_id >= 0:
            members = self.agent.group_info(rep.group_id)["members"]
            self.agent.terminate_group(rep.group_id, grace_s)
            if not self.agent.forget_group(rep.group_id):   # the Group entry and its members
                for m in members:
                    self.agent.forget(m)
            rep.group_id = -1
        elif rep.proc_id >= 0:
            self.agent.terminate(rep.proc_id, grace_s)
            self.agent.forget(rep.proc_id)

    def _spawn(self, st: DeploymentState, rep: ProcReplica) -> bool:
        from ..runtime.resources import visible_devices_env

        owner = f"{st.app_name}#{st.name}#{rep.slot}"
        self.agent.release(owner)
        if st.config.tensor_parallel_size > 1:
            return self._spawn_tp(st, rep, owner)
        bundles = st.config.placement_bundles()
        if bundles is not None:
            # gang reservation of every bundle (placement group); the replica
            # process sees all of the group's GPUs (e.g. a TP replica's ranks)
            alloc = self.agent.allocate_bundles(owner, bundles, st.config.placement_group_strategy or "PACK")
        else:
            alloc = self.agent.allocate(owner, float(st.config.num_gpus), float(st.config.hbm_gb or 0.0))
        if alloc is None:
            logger.warning("no GPU capacity for %s (num_gpus=%s, bundles=%s)", owner, st.config.num_gpus, bundles)
            return False
        rep.alloc = alloc
        gpus = list(alloc["gpus"])
        job = self.jobs[st.app_name]
        place = self._placement(st, int(gpus[0]) if gpus and float(st.config.num_gpus) > 0 else -1)
        self._init_ring(job, rep.slot, place["numa_node"])
        job.configure_queue(rep.slot, rep.slot, st.model_id, st.config.max_ongoing_requests,
                            float(st.config.slo_ms or 0.0), True)
        job.set_replica_status(rep.slot, 1, gpus[0] if gpus else -1, 0)
        env = dict(visible_devices_env(gpus))
        env.update(self._replica_env(st, rep, job))
        env["RDB_NUMA_NODE"] = str(place["numa_node"])
        cmd = [sys.executable, "-m", "ray_dynamic_batching_amd.serve.replica_main", "--spec", st.spec_path,
               "--replica", str(rep.slot), "--gpu", ",".join(map(str, gpus))]
        log = os.path.join(self.workdir, f"{owner.replace('#', '.')}.log")
        rep.proc_id = self.agent.spawn(owner, cmd, env, log, job.info()["name"], rep.slot, [rep.slot],
                                       float(st.config.health_check_timeout_s), -1, 0.5, 30.0,
                                       list(place["cpus"]))
        rep.started_at = time.time()
        rep.ready = False
        rep.health_failures = 0
        return True

    # ------------------------------------------------------------- reconcile
    def _reconcile(self, st: DeploymentState, wait: bool = False) -> None:
        if st.mode == "local":
            self._reconcile_local(st)
        else:
            self._reconcile_process(st, wait)

    def _reconcile_local(self, st: DeploymentState) -> None:
        alive = [r for r in st.local_replicas if not r.dead]
        changed = False
        while len(alive) < st.target:
            idx = st.next_index
            st.next_index += 1
            r = LocalReplica(st.app_name, st.name, idx, st.deployment.func_or_class, st.init_args, st.init_kwargs,
                             st.config)
            alive.append(r)
            changed = True
        while len(alive) > st.target:
            victim = min(alive, key=lambda r: r.ongoing)
            alive.remove(victim)
            threading.Thread(target=victim.shutdown, args=(st.config.graceful_shutdown_timeout_s,), daemon=True).start()
            changed = True
        st.local_replicas = alive
        if changed:
            st.router.update_replicas(alive)

    def _reconcile_process(self, st: DeploymentState, wait: bool) -> None:
        job = self.jobs[st.app_name]
        live = [r for r in st.proc_replicas if not r.draining]
        now = time.time()
        while len(live) < st.target:
            used = {r.slot for r in st.proc_replicas}
            free = [s for s in st.slots if s not in used]
            if not free:
                break
            rep = ProcReplica(free[0])
            st.proc_replicas.append(rep)
            live.append(rep)
            self._spawn(st, rep)
        while len(live) > st.target:
            victim = live.pop()
            self._drain(st, victim)
        if wait:
            deadline = now + float(os.environ.get("RDB_REPLICA_START_TIMEOUT_S", "900"))
            for rep in live:
                while time.time() < deadline:
                    if job.replica_status(rep.slot) == 2:
                        rep.ready = True
                        break
                    if rep.proc_id >= 0:
                        info = self.agent.info(rep.proc_id)
                        if info["restarts"] > 0 or info["state"] in ("EXITED", "STOPPED"):
                            raise RayServeException(f"replica {st.name}#{rep.slot} exited during startup "
                                                    f"({info['last_exit']}); log: {self.workdir}")
                    time.sleep(0.02)
                else:
                    raise RayServeException(f"replica {st.name}#{rep.slot} did not become ready")
        st.router.update_replicas(None)

    def _drain(self, st: DeploymentState, rep: ProcReplica) -> None:
        """Graceful drain: stop routing (queue inactive), let in-flight finish, SIGTERM."""
        job = self.jobs[st.app_name]
        rep.draining = True
        job.configure_queue(rep.slot, rep.slot, st.model_id, st.config.max_ongoing_requests, 0.0, False)

        def _finish():
            deadline = time.time() + st.config.graceful_shutdown_timeout_s
            while time.time() < deadline and job.queue_depth(rep.slot) > 0:
                time.sleep(st.config.graceful_shutdown_wait_loop_s / 20)
            self._stop_replica_procs(rep, 5.0)
            job.fail_queue(rep.slot, 6)
            job.set_replica_status(rep.slot, 4, -1, 0)
            self.agent.release(f"{st.app_name}#{st.name}#{rep.slot}")
            with self.lock:
                if rep in st.proc_replicas:
                    st.proc_replicas.remove(rep)
        threading.Thread(target=_finish, daemon=True).start()

    # ------------------------------------------------------------ control loop
    def _control_loop(self) -> None:
        last_health: Dict[Tuple[str, str], float] = {}
        ticks = 0
        while not self._stop.wait(CONTROL_LOOP_INTERVAL_S):
            try:
                with self.lock:
                    for app_name, states in list(self.apps.items()):
                        for st in states.values():
                            self._health_tick(st, last_health)
                            self._autoscale_tick(st)
                ticks += 1
                if ticks % 5 == 0:
                    self._remote_requests()
            except Exception:  # pragma: no cover
                logger.error("controller loop error:\n%s", traceback.format_exc())

    # ------------------------------------------------------------ remote control
    # `serve deploy` / `serve shutdown` from another process (reference: the CLI
    # talks to the running controller, serve/scripts.py:320,779): the request is
    # a key in the node agent's KV (written over the agent's control socket) and
    # this loop picks it up within ~0.5 s.
    SHUTDOWN_KEY = "serve/request/shutdown"
    DEPLOY_KEY = "serve/request/deploy"

    def _remote_requests(self) -> None:
        dep = self.agent.kv_get(self.DEPLOY_KEY)
        if dep:
            self.agent.kv_delete(self.DEPLOY_KEY)
            try:
                from .schema import ServeDeploySchema, deploy_config

                deploy_config(ServeDeploySchema.model_validate(json.loads(bytes(dep).decode())))
                self.agent.kv_put("serve/request/deploy_result", b"OK")
            except Exception as e:  # report back to the CLI instead of killing the loop
                logger.error("remote deploy failed:\n%s", traceback.format_exc())
                self.agent.kv_put("serve/request/deploy_result", f"ERROR {e}".encode())
        if self.agent.kv_get(self.SHUTDOWN_KEY):
            self.agent.kv_delete(self.SHUTDOWN_KEY)
            logger.info("shutdown requested over the control socket")
            self.shutdown_requested.set()
            threading.Thread(target=self.shutdown, name="rdb-serve-shutdown", daemon=True).start()

    def _health_tick(self, st: DeploymentState, last: Dict) -> None:
        now = time.time()
        if st.mode == "local":
            changed = False
            for r in list(st.local_replicas):
                ok = r.poll_health(now, st.config.health_check_period_s, st.config.health_check_timeout_s)
                if ok is None:
                    continue                      # no check finished this tick
                if not ok:
                    r.health_failures = getattr(r, "health_failures", 0) + 1
                    if r.health_failures >= st.config.health_check_failure_threshold:
                        logger.warning("replica %s unhealthy; replacing", r.replica_id)
                        r.shutdown(0)
                        st.local_replicas.remove(r)
                        changed = True
                else:
                    r.health_failures = 0
            if changed:
                self._reconcile_local(st)
            return
        job = self.jobs.get(st.app_name)
        if job is None:
            return
        # the native agent restarts dead / silent replicas itself; here we only
        # track readiness and surface its events in the log
        for rep in list(st.proc_replicas):
            if rep.draining or rep.proc_id < 0:
                continue
            info = self.agent.info(rep.proc_id)
            rep.restarts = info["restarts"]
            rep.ready = job.replica_status(rep.slot) == 2 and info["state"] in ("STARTING", "RUNNING")
        for pid, kind, msg in self.agent.events():
            if kind in ("died", "exited", "spawn_failed"):
                logger.warning("replica process %d %s: %s", pid, kind, msg)

    def _autoscale_tick(self, st: DeploymentState) -> None:
        if st.autoscaler is None:
            return
        # replica ongoing counts are sampled and look-back averaged
        # (AutoscalingMetrics), not fed to the policy one raw sample per tick
        if st.mode == "local":
            ongoing = {r.replica_id: r.ongoing for r in st.local_replicas}
            running_ids = list(ongoing)
        else:
            job = self.jobs[st.app_name]
            live = [r for r in st.proc_replicas if not r.draining]
            ongoing = {r.slot: job.queue_depth(r.slot) for r in live}
            running_ids = [r.slot for r in live if r.ready]
        if st.as_metrics is None:
            st.as_metrics = AutoscalingMetrics(st.autoscaler.cfg)
        st.as_metrics.tick(self._clock(), ongoing)
        total = st.as_metrics.total_num_requests(running_ids, st.router.num_queued())
        running = len(running_ids)
        new_target = st.config.cap_replicas(st.autoscaler.step(total, running, st.target))
        if new_target != st.target:
            logger.info("autoscaling %s: %d -> %d (ongoing=%s)", st.name, st.target, new_target, total)
            st.target = new_target
            self._reconcile(st, wait=False)

    # ------------------------------------------------------------ queries
    def router_for(self, app_name: str, deployment: str):
        with self.lock:
            states = self.apps.get(app_name)
            if not states or deployment not in states:
                raise RayServeException(f"deployment {deployment!r} not found in application {app_name!r}")
            return states[deployment].router

    def get_app_handle(self, name: str) -> DeploymentHandle:
        if name not in self.ingress:
            raise RayServeException(f"application {name!r} not found")
        return DeploymentHandle(self.ingress[name], name)

    def get_deployment_handle(self, deployment: str, app_name: Optional[str] = None) -> DeploymentHandle:
        if app_name is None:
            matches = [a for a, s in self.apps.items() if deployment in s]
            if len(matches) != 1:
                raise RayServeException(f"deployment {deployment!r} is ambiguous or missing; pass app_name")
            app_name = matches[0]
        self.router_for(app_name, deployment)
        return DeploymentHandle(deployment, app_name)

    def metrics_text(self) -> str:
        """Prometheus exposition of the whole instance: user metrics of this
        process and of every replica process (snapshots in the agent KV) plus
        the native per-replica serving counters of every process-mode app."""
        from ..utils import metrics as shm_metrics
        from ..utils import user_metrics as um

        snaps = [({"process": "controller"}, um.registry_snapshot())]
        for k in self.agent.kv_keys(um.KV_PREFIX):
            blob = self.agent.kv_get(k)
            parts = k[len(um.KV_PREFIX):].split("/")
            if not blob or len(parts) != 3:
                continue
            try:
                snaps.append((dict(application=parts[0], deployment=parts[1], replica=parts[2]),
                              json.loads(bytes(blob).decode())))
            except ValueError:
                continue
        text = um.render_prometheus(snaps)
        with self.lock:
            for app_name, states in self.apps.items():
                job = self.jobs.get(app_name)
                if job is None:
                    continue
                deps = {st.model_id: st.name for st in states.values()}
                qmap = {r.slot: r.slot for st in states.values() for r in st.proc_replicas}
                if qmap:
                    text += shm_metrics.prometheus_text(job, deps, qmap)
        return text

    def status(self) -> Dict[str, Any]:
        out = {"applications": {}}
        with self.lock:
            for app_name, states in self.apps.items():
                deps = {}
                for st in states.values():
                    if st.mode == "local":
                        reps = [r.stats() for r in st.local_replicas]
                        healthy = sum(1 for r in st.local_replicas if not r.dead)
                    else:
                        job = self.jobs[app_name]
                        reps = []
                        for r in st.proc_replicas:
                            s = job.replica_stats(r.slot)
                            s.update(slot=r.slot, draining=r.draining, queue=job.queue_stats(r.slot))
                            reps.append(s)
                        healthy = sum(1 for r in st.proc_replicas if r.ready and not r.draining)
                    status = "HEALTHY" if healthy >= st.target else ("UPDATING" if healthy > 0 else "UNHEALTHY")
                    deps[st.name] = dict(status=status, target_replicas=st.target, running_replicas=healthy,
                                         mode=st.mode, replicas=reps)
                out["applications"][app_name] = dict(status="RUNNING", ingress=self.ingress[app_name],
                                                     deployments=deps)
        return out

    # ------------------------------------------------------------ teardown
    def delete_application(self, name: str) -> None:
        with self.lock:
            states = self.apps.pop(name, None)
            self.ingress.pop(name, None)
            self.route_prefixes.pop(name, None)
            self.app_modes.pop(name, None)
            self.app_blobs.pop(name, None)
            if not states:
                return
            for st in states.values():
                for r in st.local_replicas:
                    r.shutdown(st.config.graceful_shutdown_timeout_s)
                for rep in st.proc_replicas:
                    self._stop_replica_procs(rep, 10.0)
                    self.agent.release(f"{st.app_name}#{st.name}#{rep.slot}")
            job = self.jobs.pop(name, None)
            if job is not None:
                from .router import ShmRouter

                hub = ShmRouter._clients.pop(job.info()["name"], None)
                job.set_shutdown(True)
                if hub is not None:
                    hub.close()
                job.close()
            self._checkpoint()

    def shutdown(self) -> None:
        global _CONTROLLER
        for name in list(self.apps):
            try:
                self.delete_application(name)
            except Exception:  # pragma: no cover
                logger.error("error deleting %s:\n%s", name, traceback.format_exc())
        if self.proxy is not None:
            self.proxy.stop()
            self.proxy = None
        if self.grpc_proxy is not None:
            self.grpc_proxy.stop()
            self.grpc_proxy = None
        self._stop.set()
        if self._thread.is_alive() and threading.current_thread() is not self._thread:
            self._thread.join(5.0)
        try:
            self.agent.shutdown(5.0)
        except Exception:  # pragma: no cover
            pass
        try:  # no stale discovery record for `serve status` / `serve shutdown`
            with open(discovery_file()) as f:
                if json.load(f).get("pid") == os.getpid():
                    os.remove(discovery_file())
        except (OSError, ValueError):
            pass
        with _CTRL_LOCK:
            if _CONTROLLER is self:
                _CONTROLLER = None

    # ------------------------------------------------------------ checkpoint
    @staticmethod
    def _rebuild_recipe(app: Application) -> Dict[str, Any]:
        """How a later controller rebuilds this application: its import path when
        it came from a config (reference: the checkpointed deploy schema is
        re-imported), else the application graph itself, cloudpickled (user
        classes by value, as process-mode replicas receive them)."""
        ip = getattr(app, "_import_path", None)
        if ip:
            return dict(import_path=ip, args=getattr(app, "_import_args", None) or {})
        import base64

        import cloudpickle

        try:
            return dict(pickle=base64.b64encode(cloudpickle.dumps(app)).decode())
        except Exception as e:  # noqa: BLE001 - unpicklable app: recorded, not recoverable
            return dict(error=f"not picklable: {e}")

    def _checkpoint(self) -> None:
        """Persist the applied config (reference: controller KV checkpoint,
        serve/_private/controller.py:510-563): per application its route prefix,
        mode, ingress, every deployment's config and a rebuild recipe."""
        data = {}
        for app_name, states in self.apps.items():
            data[app_name] = dict(ingress=self.ingress.get(app_name),
                                  route_prefix=self.route_prefixes.get(app_name),
                                  mode=self.app_modes.get(app_name),
                                  app=self.app_blobs.get(app_name, {}),
                                  deployments={n: st.config.model_dump(mode="json") for n, st in states.items()})
        blob = json.dumps(dict(version=1, time=time.time(), applications=data), default=str)
        try:
            self.agent.kv_put("serve/checkpoint", blob.encode())
            tmp = self.kv_path + ".tmp"
            with open(tmp, "w") as f:
                f.write(blob)
            os.replace(tmp, self.kv_path)
        except OSError:  # pragma: no cover
            pass

    def read_checkpoint(self) -> Optional[Dict[str, Any]]:
        """The last checkpoint: the agent's persistent KV first (the GCS KV of
        the reference), else the JSON document."""
        blob = None
        try:
            blob = self.agent.kv_get("serve/checkpoint")
        except Exception:  # noqa: BLE001
            blob = None
        if not blob:
            try:
                with open(self.kv_path, "rb") as f:
                    blob = f.read()
            except OSError:
                return None
        try:
            doc = json.loads(blob)
        except ValueError:
            return None
        return doc if doc.get("version") == 1 else None

    def recover(self) -> List[str]:
        """Redeploy every application of the last checkpoint that is not running
        (controller restart, reference serve/_private/controller.py:510-563):
        rebuilt from its import path or pickled graph, with the checkpointed
        deployment configs re-applied (autoscaled replica counts and later
        ``options()`` included), route prefix and mode.  Returns the names."""
        doc = self.read_checkpoint()
        if not doc:
            return []
        out = []
        for name, a in doc.get("applications", {}).items():
            if name in self.apps:
                continue
            recipe = a.get("app") or {}
            try:
                if recipe.get("import_path"):
                    from .schema import ServeApplicationSchema, build_application

                    app = build_application(ServeApplicationSchema(import_path=recipe["import_path"], name=name,
                                                                   args=recipe.get("args") or {}))
                    app._import_path = recipe["import_path"]
                elif recipe.get("pickle"):
                    import base64

                    import cloudpickle

                    app = cloudpickle.loads(base64.b64decode(recipe["pickle"]))
                else:
                    logger.warning("serve: application %r has no rebuild recipe (%s)", name, recipe.get("error"))
                    continue
                cfgs = a.get("deployments", {})
                for node in app.walk():
                    c = cfgs.get(node.deployment.name)
                    if c:
                        node.deployment = node.deployment._with_config(DeploymentConfig(**c))
                self.deploy_application(app, name=name, route_prefix=a.get("route_prefix", "/"), mode=a.get("mode"))
                out.append(name)
            except Exception:  # noqa: BLE001 - one bad app must not stop the others
                logger.error("serve: could not recover application %r:\n%s", name, traceback.format_exc())
        self.recovered = out
        return out


def _codec_for_servable(sv) -> Any:
    """Build the tensor codec from the model's declared I/O (cheap: metadata only)."""
    from .servable import TensorCodec

    spec = getattr(sv["factory"], "io_spec", None)
    if spec is None:
        return None
    return TensorCodec(*spec)


def _torch_dtype_name(np_dtype) -> str:
    import numpy as np

    return {np.int32: "int32", np.int64: "int64", np.float32: "float32", np.float16: "float16",
            np.uint8: "uint8"}[np_dtype]
