"""Process supervisor for the full stack — the docker-compose.yml equivalent (reference
docker-compose.yml:45-128: postgres, nats, redis, gateway, parser x2, analysis x2, query).

``python -m docagents_amd.deploy [--env deploy/env.example] [--gpus N] [--parsers 2] [--analyzers 2]
[--base-port 8080] [--log-dir ./logs]``

Starts, in dependency order with a health check after each (compose ``depends_on`` + healthchecks):
the native broker (QUEUE_URL) and KV cache (REDIS_ADDR) binaries, the MI355X engine server
(torchrun over N GPUs when N > 1; skipped unless LLM_PROVIDER / EMBEDDER_PROVIDER is ``engine``),
the query service, the gateway, then the parser and analysis workers (their /healthz). Ports follow
the reference: gateway = base, query = base + 1, parser i = base + 2 + 10 i, analysis i =
base + 3 + 10 i. A crashed process is restarted with exponential backoff (``restart: unless-stopped``);
SIGINT / SIGTERM stops everything in reverse order (engine last, so it can checkpoint its shards).
``LOG_DIR/status.json`` lists every process with its pid and restart count.

Every child is a plain ``subprocess`` (the native servers run their own binaries directly): nothing
here replaces a process image, and the supervisor itself never touches the GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time
from dataclasses import dataclass, field


def load_env_file(path: str) -> dict:
    env = {}
    if path and os.path.exists(path):
        for line in open(path):
            line = line.strip()
            if not line or line.startswith("#") or "=" not in line:
                continue
            k, v = line.split("=", 1)
            env[k.strip()] = v.strip().strip('"').strip("'")
    return env


def _wait_tcp(host: str, port: int, timeout: float, proc: subprocess.Popen | None = None) -> bool:
    t0 = time.time()
    while time.time() - t0 < timeout:
        if proc is not None and proc.poll() is not None:
            return False
        try:
            socket.create_connection((host, port), 0.5).close()
            return True
        except OSError:
            time.sleep(0.2)
    return False


def _hostport(addr: str, default_port: int):
    a = addr.split("://")[-1]
    h, _, p = a.rpartition(":")
    return (h or "127.0.0.1").replace("0.0.0.0", "127.0.0.1"), int(p or default_port)


@dataclass
class Proc:
    name: str
    cmd: list
    env: dict
    wait: tuple | None = None  # (host, port) to health-check after start
    timeout: float = 60.0
    proc: subprocess.Popen | None = None
    restarts: int = 0
    next_start: float = 0.0
    extra: dict = field(default_factory=dict)

    def start(self, log_dir):
        out = open(os.path.join(log_dir, f"{self.name}.log"), "ab")
        self.proc = subprocess.Popen(self.cmd, env=self.env, stdout=out, stderr=subprocess.STDOUT,
                                     start_new_session=True)
        out.close()


def plan(env: dict, gpus: int = 1, parsers: int = 2, analyzers: int = 2, base_port: int = 8080,
         engine: bool = True) -> list[Proc]:
    """The process table (compose services) for ``env``; defaults fill the reference's addresses."""
    from .native import binary
    env = dict(env)
    env.setdefault("QUEUE_PROVIDER", "broker")
    env.setdefault("QUEUE_URL", "nats://127.0.0.1:4222")
    env.setdefault("CACHE_PROVIDER", "kv")
    env.setdefault("REDIS_ADDR", "127.0.0.1:6379")
    env.setdefault("LLM_PROVIDER", "engine")
    env.setdefault("ENGINE_URL", "tcp://127.0.0.1:9090")
    env.setdefault("QUERY_SERVICE_URL", f"http://127.0.0.1:{base_port + 1}/api/query")
    py = sys.executable
    procs: list[Proc] = []
    bh, bp = _hostport(env["QUEUE_URL"], 4222)
    kh, kp = _hostport(env["REDIS_ADDR"], 6379)
    procs.append(Proc("broker", [str(binary("da-broker")), "--listen", f"0.0.0.0:{bp}"], env, (bh, bp)))
    kv = [str(binary("da-kvserver")), "--listen", f"0.0.0.0:{kp}"]
    if env.get("REDIS_PASSWORD"):
        kv += ["--requirepass", env["REDIS_PASSWORD"]]
    procs.append(Proc("kvcache", kv, env, (kh, kp)))
    uses_engine = (env["LLM_PROVIDER"] in ("engine", "openai")
                   or env.get("EMBEDDER_PROVIDER", "") in ("engine", "openai"))
    if uses_engine and engine:
        eh, ep = _hostport(env["ENGINE_URL"], 9090)
        if gpus > 1:
            cmd = [py, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
                   "--master-addr", "127.0.0.1", "--master-port", env.get("ENGINE_MASTER_PORT", "29600"),
                   "-m", "docagents_amd.services", "engine", "--listen", f"tcp://0.0.0.0:{ep}"]
        else:
            cmd = [py, "-m", "docagents_amd.services", "engine", "--listen", f"tcp://0.0.0.0:{ep}"]
        procs.append(Proc("engine", cmd, env, (eh, ep), timeout=900.0))
    procs.append(Proc("query", [py, "-m", "docagents_amd.services", "query"], dict(env, PORT=str(base_port + 1)),
                      ("127.0.0.1", base_port + 1)))
    procs.append(Proc("gateway", [py, "-m", "docagents_amd.services", "gateway"], dict(env, PORT=str(base_port)),
                      ("127.0.0.1", base_port)))
    for i in range(parsers):
        port = base_port + 2 + 10 * i
        procs.append(Proc(f"parser-{i}", [py, "-m", "docagents_amd.services", "parser"], dict(env, PORT=str(port)),
                          ("127.0.0.1", port)))
    for i in range(analyzers):
        port = base_port + 3 + 10 * i
        procs.append(Proc(f"analysis-{i}", [py, "-m", "docagents_amd.services", "analysis"],
                          dict(env, PORT=str(port)), ("127.0.0.1", port)))
    return procs


class Supervisor:
    def __init__(self, procs: list[Proc], log_dir: str, max_backoff: float = 30.0):
        self.procs, self.log_dir, self.max_backoff = procs, log_dir, max_backoff
        self.stopping = False
        self.ready = False  # every process started and healthy (clients wait for this, not the gateway)
        os.makedirs(log_dir, exist_ok=True)

    def _status(self):
        st = [{"name": p.name, "pid": p.proc.pid if p.proc is not None and p.proc.poll() is None else None,
               "restarts": p.restarts} for p in self.procs]
        tmp = os.path.join(self.log_dir, "status.json.tmp")
        with open(tmp, "w") as f:
            json.dump({"supervisor": os.getpid(), "ready": self.ready, "procs": st}, f)
        os.replace(tmp, os.path.join(self.log_dir, "status.json"))

    def start_all(self) -> bool:
        for p in self.procs:
            if self.stopping:
                return False
            p.start(self.log_dir)
            if p.wait and not _wait_tcp(*p.wait, timeout=p.timeout, proc=p.proc):
                print(f"[deploy] {p.name} did not become healthy; see {self.log_dir}/{p.name}.log", file=sys.stderr)
                return False
            print(f"[deploy] {p.name} up", file=sys.stderr, flush=True)
            self._status()
        self.ready = True
        self._status()
        return True

    def tick(self):
        """Restart exited processes with exponential backoff (0.5 s doubling, capped)."""
        changed = False
        for p in self.procs:
            if p.proc is not None and p.proc.poll() is not None:
                p.restarts += 1
                delay = min(self.max_backoff, 0.5 * 2 ** min(p.restarts - 1, 6))
                print(f"[deploy] {p.name} exited ({p.proc.returncode}); restart #{p.restarts} in {delay:.1f}s",
                      file=sys.stderr, flush=True)
                p.next_start = time.time() + delay
                p.proc = None
                changed = True
            elif p.proc is None and time.time() >= p.next_start:
                p.start(self.log_dir)
                changed = True
        if changed:
            self._status()

    def stop_all(self, timeout: float = 30.0):
        for p in reversed(self.procs):
            if p.proc is not None and p.proc.poll() is None:
                os.killpg(p.proc.pid, signal.SIGTERM)
                try:
                    p.proc.wait(timeout)
                except subprocess.TimeoutExpired:
                    os.killpg(p.proc.pid, signal.SIGKILL)
                    p.proc.wait(5)
        self._status()

    def run(self) -> int:
        def on_sig(*_):
            self.stopping = True
        signal.signal(signal.SIGINT, on_sig)
        signal.signal(signal.SIGTERM, on_sig)
        ok = self.start_all()
        while ok and not self.stopping:
            time.sleep(0.25)
            self.tick()
        self.stop_all()
        return 0 if ok else 1


def main(argv=None):
    ap = argparse.ArgumentParser("deploy")
    ap.add_argument("--env", default="")
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("ENGINE_GPUS", "1")))
    ap.add_argument("--parsers", type=int, default=2)
    ap.add_argument("--analyzers", type=int, default=2)
    ap.add_argument("--base-port", type=int, default=8080)
    ap.add_argument("--log-dir", default="./logs")
    ap.add_argument("--no-engine", action="store_true")
    a = ap.parse_args(argv)
    env = dict(os.environ)
    env.update(load_env_file(a.env))
    procs = plan(env, a.gpus, a.parsers, a.analyzers, a.base_port, engine=not a.no_engine)
    return Supervisor(procs, a.log_dir).run()


if __name__ == "__main__":
    sys.exit(main())
