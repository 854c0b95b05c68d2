"""``serve`` command line (reference: serve/scripts.py:139-886).

    python -m ray_dynamic_batching_amd.serve.cli run my_module:app [--mode local|process] [--duration S]
    python -m ray_dynamic_batching_amd.serve.cli deploy config.yaml [--duration S]
    python -m ray_dynamic_batching_amd.serve.cli build my_module:app -o config.yaml
    python -m ray_dynamic_batching_amd.serve.cli config config.yaml      # validate + print
    python -m ray_dynamic_batching_amd.serve.cli status --kv serve_kv.json

The controller lives in the process that runs ``run``/``deploy`` (single-node
design), so those commands keep serving until interrupted or --duration ends.
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import yaml


def _serve_until(duration: float) -> None:
    from . import api

    try:
        if duration > 0:
            time.sleep(duration)
        else:  # pragma: no cover - interactive
            while True:
                time.sleep(1)
    except KeyboardInterrupt:  # pragma: no cover
        pass
    finally:
        print(json.dumps(api.status(), default=str, indent=1))
        api.shutdown()


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
    d = sub.add_parser("deploy")
    d.add_argument("config")
    d.add_argument("--duration", type=float, default=0)
    d.add_argument("--http-port", type=int, default=-1)
    b = sub.add_parser("build")
    b.add_argument("import_path")
    b.add_argument("-o", "--output", default="-")
    c = sub.add_parser("config")
    c.add_argument("config")
    s = sub.add_parser("status")
    s.add_argument("--kv", default="", help="checkpoint file (default: ask the running node agent)")
    s.add_argument("--socket", default="", help="node agent control socket (default: discovered)")
    a = ap.parse_args(argv)

    from .schema import ServeApplicationSchema, ServeDeploySchema, build_application, deploy_config, import_attr

    if a.cmd in ("run", "deploy") and a.http_port >= 0:
        from .api import start

        start(http_options={"host": "127.0.0.1", "port": a.http_port})
    if a.cmd == "run":
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
