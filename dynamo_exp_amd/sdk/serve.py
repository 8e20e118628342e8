"""`serve` CLI + process supervisor (reference `dynamo serve`, cli/serve.py +
cli/serving.py with circus watchers).

    python -m dynamo_exp_amd.sdk.serve graphs.agg:Frontend -f configs/agg.yaml [--Svc.key=val ...]
        [--dry-run] [--service-name X] [--enable-local-planner] [--control-plane host:port]

* resolves YAML + CLI overrides into DYNAMO_SERVICE_CONFIG;
* starts the in-tree control plane if none is reachable;
* one watcher per service (`workers` processes, HIP_VISIBLE_DEVICES from the
  allocator), restarted on crash with backoff;
* watchers can be added/removed at runtime through the control plane
  (subject `supervisor.{ns}`) -- the planner's LocalConnector uses this;
* state file ~/.dynamo/state/{ns}.json lists watchers, GPUs and pids.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import signal
import subprocess
import sys
import time
from dataclasses import dataclass, field

from ..runtime import configure_logging
from ..runtime.control_plane import (ControlPlaneClient, ControlPlaneServer, NativeServerProcess, default_address,
                                     use_native_server)
from .allocator import ResourceAllocator
from .config import ENV, ServiceConfig, resolve
from .state import locked_state

log = logging.getLogger("dynamo_exp_amd.serve")


@dataclass
class Watcher:
    name: str
    service: str
    cmd: list[str]
    env: dict
    numprocesses: int = 1
    gpus: list[int] = field(default_factory=list)
    procs: list[subprocess.Popen] = field(default_factory=list)  # index = process slot
    restarts: int = 0
    stopping: bool = False
    slot_envs: list[dict] = field(default_factory=list)  # per-process env (own GPU slice)


def slot_gpu_envs(alloc: ResourceAllocator, numprocesses: int, gpus_per_worker: float) -> tuple[list, list]:
    """GPUs for `numprocesses` workers of `gpus_per_worker` GPUs each and the
    env update of every process slot: its own whole GPUs
    (HIP_VISIBLE_DEVICES), or a shared GPU for a fractional request.  Used by
    the launch and by `--dry-run` (which prints the placement it would make)."""
    gpus: list[int] = []
    per_slot: list[dict] = [{} for _ in range(numprocesses)]
    shared = False
    if gpus_per_worker:
        if gpus_per_worker >= 1:
            per = int(gpus_per_worker)
            gpus = alloc.assign_gpus(per * numprocesses)
            for i, e in enumerate(per_slot):
                e.update(ResourceAllocator.env_for(gpus[i * per:(i + 1) * per]))
            shared = not gpus and numprocesses > 1  # allocation disabled: all on the default GPU
        else:
            gpus = alloc.assign_gpus(gpus_per_worker)
            for e in per_slot:
                e.update(ResourceAllocator.env_for(gpus))
            shared = True
    if shared:
        # several processes on one GPU: with 4 HW queues each, the GPU's
        # queue scheduler time-slices them and a step can stall for tens
        # of seconds (tools/prefix_stress.py, two processes: 14-52 s
        # steps at 4 queues, none at 2)
        for e in per_slot:
            e["GPU_MAX_HW_QUEUES"] = str(min(2, int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)))
    return gpus, per_slot


def plan_placement(graph, alloc: ResourceAllocator | None = None) -> list[dict]:
    """The placement a launch of `graph` makes, in launch order (dependencies
    first): per service its workers and each worker's device env."""
    alloc = alloc or ResourceAllocator()
    out = []
    for s in reversed(graph):
        g = float(s.resources.get("gpu", 0) or 0)
        _, per_slot = slot_gpu_envs(alloc, s.workers, g)
        out.append({"service": s.name, "workers": s.workers, "gpus_per_worker": g, "slots": per_slot})
    return out


class Supervisor:
    def __init__(self, namespace: str, target: str, config: dict, control_plane: str,
                 allocator: ResourceAllocator | None = None):
        self.ns = namespace
        self.target = target
        self.config = config
        self.cp_addr = control_plane
        self.alloc = allocator or ResourceAllocator()
        self.watchers: dict[str, Watcher] = {}
        self.service_gpus: dict[str, float] = {}  # configured resources.gpu per service (planner adds)
        self._stop = False

    def _base_env(self) -> dict:
        env = dict(os.environ)
        env[ENV] = json.dumps(self.config)
        env["DX_CONTROL_PLANE"] = self.cp_addr
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        return env

    def gpus_for_add(self, cmd: dict) -> float:
        """GPU share of a runtime `add`: the command's, else the service's configured one."""
        g = cmd.get("gpus")
        return self.service_gpus.get(cmd["service"], 0.0) if g is None else float(g)

    def add_watcher(self, name: str, service: str, numprocesses: int = 1, gpus_per_worker: float = 0,
                    extra_env: dict | None = None) -> Watcher:
        """`numprocesses` workers of `service`; each process gets its own
        `gpus_per_worker` GPUs (HIP_VISIBLE_DEVICES), or a shared GPU for a
        fractional request."""
        env = self._base_env()
        env.update(extra_env or {})
        gpus, per_slot = slot_gpu_envs(self.alloc, numprocesses, gpus_per_worker)
        slot_envs = [dict(env, **u) for u in per_slot]
        cmd = [sys.executable, "-m", "dynamo_exp_amd.sdk.worker", self.target, "--service-name", service]
        w = Watcher(name, service, cmd, env, numprocesses, gpus, slot_envs=slot_envs)
        self.watchers[name] = w
        for i in range(numprocesses):
            self._spawn(w, i)
        self._save()
        log.info("watcher %s: %d x %s gpus=%s", name, numprocesses, service, gpus)
        return w

    def _spawn(self, w: Watcher, slot: int) -> None:
        env = w.slot_envs[slot] if slot < len(w.slot_envs) else w.env
        p = subprocess.Popen(w.cmd, env=env, start_new_session=True)
        if slot < len(w.procs):
            w.procs[slot] = p
        else:
            w.procs.append(p)

    def remove_watcher(self, name: str, graceful_timeout: float = 30.0) -> bool:
        w = self.watchers.pop(name, None)
        if w is None:
            return False
        w.stopping = True
        for p in w.procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        end = time.time() + graceful_timeout
        for p in w.procs:
            try:
                p.wait(max(0.1, end - time.time()))
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
        self.alloc.release(w.gpus)
        self._save()
        return True

    def poll(self) -> None:
        """Restart crashed workers (circus respawn)."""
        for w in list(self.watchers.values()):
            for i, p in enumerate(list(w.procs)):
                rc = p.poll()
                if rc is not None and not w.stopping and not self._stop:
                    log.warning("%s worker pid %d exited rc=%s; restarting", w.name, p.pid, rc)
                    w.restarts += 1
                    time.sleep(min(5.0, 0.2 * w.restarts))
                    self._spawn(w, i)  # same slot, same GPUs
                    self._save()

    def _save(self) -> None:
        with locked_state(self.ns) as st:
            st["watchers"] = {n: {"service": w.service, "numprocesses": w.numprocesses, "gpus": w.gpus,
                                  "pids": [p.pid for p in w.procs]} for n, w in self.watchers.items()}
            st["gpus"] = {"all": self.alloc.gpus, "free": self.alloc.free_gpus()}
            st["target"] = self.target
            st["control_plane"] = self.cp_addr

    def shutdown(self) -> None:
        self._stop = True
        for n in list(self.watchers):
            self.remove_watcher(n, graceful_timeout=10)

    async def command_loop(self) -> None:
        """Runtime add/remove requests: publish {op, name, service, gpus} on supervisor.{ns}."""
        cp = await ControlPlaneClient(self.cp_addr).connect()
        sub = await cp.subscribe(f"supervisor.{self.ns}")
        async for msg in sub:
            try:
                cmd = json.loads(msg["data"])
                op = cmd.get("op")
                if op == "add":
                    # no explicit share: the service's configured resources.gpu (a planner scale-up adds a
                    # worker as the graph configures it, e.g. a fractional GPU share)
                    w = self.add_watcher(cmd["name"], cmd["service"], int(cmd.get("numprocesses", 1)),
                                         self.gpus_for_add(cmd))
                    res = {"ok": True, "gpus": w.gpus, "pids": [p.pid for p in w.procs]}
                elif op == "retire":  # stop respawning its workers (they are about to drain and exit)
                    w = self.watchers.get(cmd["name"])
                    if w is not None:
                        w.stopping = True
                    res = {"ok": w is not None, "pids": [p.pid for p in w.procs] if w is not None else []}
                elif op == "remove":
                    res = {"ok": await asyncio.to_thread(self.remove_watcher, cmd["name"],
                                                         float(cmd.get("timeout", 30)))}
                elif op == "list":
                    res = {"ok": True, "watchers": {n: w.service for n, w in self.watchers.items()},
                           "free_gpus": self.alloc.free_gpus()}
                else:
                    res = {"ok": False, "error": f"unknown op {op}"}
            except Exception as e:  # noqa: BLE001
                res = {"ok": False, "error": str(e)}
            if cmd.get("reply"):
                await cp.put(cmd["reply"], json.dumps(res).encode())


async def _ensure_control_plane(addr: str):
    try:
        c = await ControlPlaneClient(addr).connect(timeout=0.5)
        await c.close()
        return None
    except Exception:
        host, port = addr.rsplit(":", 1)
        bind = "0.0.0.0" if host in ("127.0.0.1", "localhost") else host
        if use_native_server():
            s = NativeServerProcess(bind, int(port)).start()
            log.info("started native control plane (dx-ctrld) on %s", addr)
        else:
            s = await ControlPlaneServer(bind, int(port)).start()
            log.info("started control plane on %s", addr)
        return s


def main(argv=None):
    ap = argparse.ArgumentParser(prog="serve")
    ap.add_argument("target", help="module:EntryService")
    ap.add_argument("-f", "--config-file", default=None)
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("--service-name", default=None, help="run only this service (standalone)")
    ap.add_argument("--enable-local-planner", action="store_true")
    ap.add_argument("--control-plane", default=None)
    ap.add_argument("--working-dir", default=None)
    a, overrides = ap.parse_known_args(argv)
    configure_logging()
    if a.working_dir:
        os.chdir(a.working_dir)
    cfg = resolve(a.config_file, overrides)
    os.environ[ENV] = json.dumps(cfg)
    ServiceConfig.reset()
    from .worker import load_service

    entry = load_service(a.target)
    graph = entry.graph()
    for s in graph:
        s.apply_overrides(cfg)
    if a.service_name:
        graph = [s for s in graph if s.name == a.service_name]
    if a.dry_run:
        try:
            placement = plan_placement(graph)
        except RuntimeError as e:  # more GPUs asked for than this node has
            placement = {"error": str(e)}
        print(json.dumps({"config": cfg, "services": [s.config_dict() for s in graph], "placement": placement},
                         indent=2))
        return
    addr = a.control_plane or default_address()

    async def run():
        server = await _ensure_control_plane(addr)
        sup = Supervisor(entry.dynamo.namespace, a.target, cfg, addr)
        # dependencies first so workers are discoverable before frontends
        for s in reversed(graph):
            sup.service_gpus[s.name] = float(s.resources.get("gpu", 0) or 0)
            sup.add_watcher(f"{s.dynamo.namespace}_{s.name}", s.name, s.workers, sup.service_gpus[s.name])
        if a.enable_local_planner:
            from ..planner.planner import spawn_local_planner

            planner = spawn_local_planner(entry.dynamo.namespace, addr, cfg)
        else:
            planner = None
        cmd_task = asyncio.create_task(sup.command_loop())
        loop = asyncio.get_running_loop()
        stop = asyncio.Event()
        for sig in (signal.SIGINT, signal.SIGTERM):
            loop.add_signal_handler(sig, stop.set)
        while not stop.is_set():
            sup.poll()
            try:
                await asyncio.wait_for(stop.wait(), 0.5)
            except asyncio.TimeoutError:
                pass
        cmd_task.cancel()
        if planner is not None and planner.poll() is None:
            planner.terminate()
        await asyncio.to_thread(sup.shutdown)
        if isinstance(server, NativeServerProcess):
            server.stop()
        elif server is not None:
            await server.stop()

    asyncio.run(run())


if __name__ == "__main__":
    main()
