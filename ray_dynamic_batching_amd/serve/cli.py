"""``serve`` command line (reference: serve/scripts.py:139-886).

    python -m ray_dynamic_batching_amd.serve.cli start [--http-port P] [--duration S]   # long-running instance
    python -m ray_dynamic_batching_amd.serve.cli run my_module:app [--mode local|process] [--duration S]
    python -m ray_dynamic_batching_amd.serve.cli deploy config.yaml [--duration S] [--in-process]
    python -m ray_dynamic_batching_amd.serve.cli build my_module:app -o config.yaml
    python -m ray_dynamic_batching_amd.serve.cli config config.yaml      # validate + print
    python -m ray_dynamic_batching_amd.serve.cli status [--kv serve_kv.json]
    python -m ray_dynamic_batching_amd.serve.cli shutdown [-y]

The controller lives in the process that runs ``start``/``run``/``deploy``
(single-node design).  ``deploy`` hands the config to an instance that is
already running (found through its discovery file, talked to over the node
agent's control socket) unless ``--in-process``; ``shutdown`` stops it.
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import yaml


def _serve_until(duration: float) -> None:
    """Keep this (controller) process serving until --duration ends, Ctrl-C, or
    a `serve shutdown` from another shell."""
    from . import api
    from .controller import get_controller

    ctrl = get_controller()
    end = time.time() + duration if duration > 0 else float("inf")
    try:
        while time.time() < end and not ctrl.shutdown_requested.is_set():
            ctrl.shutdown_requested.wait(min(0.2, max(0.0, end - time.time())))
    except KeyboardInterrupt:  # pragma: no cover
        pass
    finally:
        if not ctrl.shutdown_requested.is_set():
            print(json.dumps(api.status(), default=str, indent=1))
        api.shutdown()


def _live_socket(sock: str = "") -> str:
    """Control socket of a running serve instance (discovery file), or ''."""
    import os

    from .controller import discovery_file

    if not sock:
        try:
            with open(discovery_file()) as f:
                rec = json.load(f)
            os.kill(int(rec.get("pid", -1)), 0)        # the instance is alive
            sock = rec.get("socket", "")
        except (OSError, ValueError):
            return ""
    return sock if sock and os.path.exists(sock) else ""


def _remote_deploy(sock: str, schema, timeout_s: float) -> str:
    from ..runtime import agent as ragent
    from .controller import ServeController

    ragent.request(sock, "KV_DEL serve/request/deploy_result")
    ragent.request(sock, f"KV_PUT {ServeController.DEPLOY_KEY} {json.dumps(schema.model_dump(mode='json'))}")
    end = time.time() + timeout_s
    while time.time() < end:
        r = ragent.request(sock, "KV_GET serve/request/deploy_result")
        if r.startswith("OK "):
            return r[3:]
        time.sleep(0.1)
    return "ERROR timed out waiting for the running instance"


def _remote_shutdown(sock: str, timeout_s: float) -> bool:
    import os

    from ..runtime import agent as ragent
    from .controller import ServeController, discovery_file

    ragent.request(sock, f"KV_PUT {ServeController.SHUTDOWN_KEY} 1")
    end = time.time() + timeout_s
    while time.time() < end:
        if not os.path.exists(sock) or not os.path.exists(discovery_file()):
            return True
        time.sleep(0.1)
    return False


def _status(sock: str, kv: str) -> dict:
    """Live status from the node agent's control socket (processes, GPU slots,
    last checkpointed config); falls back to a checkpoint file."""
    import os

    from .controller import discovery_file

    if not sock and not kv:
        try:
            with open(discovery_file()) as f:
                sock = json.load(f).get("socket", "")
        except (OSError, ValueError):
            sock = ""
    if sock and os.path.exists(sock):
        from ..runtime import agent as ragent

        try:
            st = ragent.status(sock)
            ck = ragent.request(sock, "KV_GET serve/checkpoint")
            st["checkpoint"] = json.loads(ck[3:]) if ck.startswith("OK ") else None
            return st
        except (RuntimeError, ValueError):
            pass
    try:
        with open(kv or "serve_kv.json") as f:
            return json.load(f)
    except (OSError, ValueError):
        return {"applications": {}}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="serve")
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("import_path")
    r.add_argument("--name", default="default")
    r.add_argument("--mode", default=None)
    r.add_argument("--duration", type=float, default=0)
    r.add_argument("--http-port", type=int, default=-1, help="start the HTTP proxy on this port (-1 = off)")
    r.add_argument("--grpc-port", type=int, default=-1, help="start the gRPC proxy on this port (-1 = off)")
    d = sub.add_parser("deploy")
    d.add_argument("config")
    d.add_argument("--duration", type=float, default=0)
    d.add_argument("--http-port", type=int, default=-1)
    d.add_argument("--grpc-port", type=int, default=-1)
    b = sub.add_parser("build")
    b.add_argument("import_path")
    b.add_argument("-o", "--output", default="-")
    c = sub.add_parser("config")
    c.add_argument("config")
    s = sub.add_parser("status")
    s.add_argument("--kv", default="", help="checkpoint file (default: ask the running node agent)")
    s.add_argument("--socket", default="", help="node agent control socket (default: discovered)")
    st = sub.add_parser("start")
    st.add_argument("--http-port", type=int, default=-1)
    st.add_argument("--grpc-port", type=int, default=-1)
    st.add_argument("--duration", type=float, default=0)
    sh = sub.add_parser("shutdown")
    sh.add_argument("--socket", default="")
    sh.add_argument("-y", "--yes", action="store_true")
    sh.add_argument("--timeout", type=float, default=30.0)
    d.add_argument("--in-process", action="store_true", help="never hand the config to a running instance")
    d.add_argument("--socket", default="")
    d.add_argument("--timeout", type=float, default=120.0)
    a = ap.parse_args(argv)

    from .schema import ServeApplicationSchema, ServeDeploySchema, build_application, deploy_config, import_attr

    if a.cmd == "deploy" and not a.in_process:
        sock = _live_socket(a.socket)
        if sock:
            res = _remote_deploy(sock, ServeDeploySchema.from_yaml(a.config), a.timeout)
            print("deployed to the running instance" if res == "OK" else res, flush=True)
            return 0 if res == "OK" else 1
    if a.cmd == "shutdown":
        sock = _live_socket(a.socket)
        if not sock:
            print("no running serve instance found", flush=True)
            return 0
        ok = _remote_shutdown(sock, a.timeout)
        print("shut down" if ok else "shutdown timed out", flush=True)
        return 0 if ok else 1
    if a.cmd in ("run", "deploy", "start"):
        from .api import start

        http = {"host": "127.0.0.1", "port": a.http_port} if a.http_port >= 0 else None
        grpc_ = {"host": "127.0.0.1", "port": a.grpc_port} if a.grpc_port >= 0 else None
        if a.cmd == "deploy":   # proxies named in the config file (port flags win)
            sch = ServeDeploySchema.from_yaml(a.config)
            http = http or sch.http_options
            grpc_ = grpc_ or sch.grpc_options
        if http or grpc_:
            start(http_options=http, grpc_options=grpc_)
    if a.cmd == "start":
        from .controller import get_controller

        get_controller()
        print("serve instance started", flush=True)
        _serve_until(a.duration)
    elif a.cmd == "run":
        from .api import run

        app = build_application(ServeApplicationSchema(import_path=a.import_path, name=a.name))
        run(app, name=a.name, mode=a.mode)
        print(f"application {a.name!r} running", flush=True)
        _serve_until(a.duration)
    elif a.cmd == "deploy":
        deploy_config(ServeDeploySchema.from_yaml(a.config))
        print("deployed", flush=True)
        _serve_until(a.duration)
    elif a.cmd == "build":
        app = build_application(ServeApplicationSchema(import_path=a.import_path))
        deps = []
        for node in app.walk():
            cfg = node.deployment.config.model_dump(mode="json", exclude_defaults=True)
            cfg.pop("name", None)
            deps.append(dict(name=node.deployment.name, **cfg))
        out = dict(applications=[dict(name="default", route_prefix="/", import_path=a.import_path, deployments=deps)])
        text = yaml.safe_dump(out, sort_keys=False)
        if a.output == "-":
            print(text)
        else:
            open(a.output, "w").write(text)
    elif a.cmd == "config":
        sch = ServeDeploySchema.from_yaml(a.config)
        print(yaml.safe_dump(sch.model_dump(mode="json"), sort_keys=False))
    elif a.cmd == "status":
        print(json.dumps(_status(a.socket, a.kv), indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
