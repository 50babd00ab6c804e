"""Process supervisor for the full stack — the docker-compose.yml equivalent (reference
docker-compose.yml:1-131: postgres, nats, redis, gateway, parser x2, analysis x2, query).

``python -m docagents_amd.deploy [--env deploy/env.example] [--gpus N] [--parsers 2] [--analyzers 2]``

Starts: native broker (QUEUE_URL), native KV cache (REDIS_ADDR), the MI355X engine server
(torchrun over N GPUs when N > 1; skipped with LLM_PROVIDER=stub), then the agents with the
reference's ports (gateway 8080, query 8081, parser 8082+, analysis 8083+). Dependencies start in
order with health checks (compose ``depends_on`` + healthchecks); a crashed agent is restarted
with exponential backoff; SIGINT/SIGTERM stops everything (engine last, so it can snapshot).
"""
from __future__ import annotations

import argparse
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


def _wait_tcp(host: str, port: int, timeout: float) -> bool:
    t0 = time.time()
    while time.time() - t0 < timeout:
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
    proc: subprocess.Popen | None = None
    restarts: int = 0
    next_start: float = 0.0
    critical: bool = False
    extra: dict = field(default_factory=dict)

    def start(self, log_dir):
        out = open(os.path.join(log_dir, f"{self.name}.log"), "ab")
        self.proc = subprocess.Popen(self.cmd, env=self.env, stdout=out, stderr=subprocess.STDOUT,
                                     start_new_session=True)
        out.close()


def main(argv=None):
    ap = argparse.ArgumentParser("deploy")
    ap.add_argument("--env", default="")
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("ENGINE_GPUS", "1")))
    ap.add_argument("--parsers", type=int, default=2)
    ap.add_argument("--analyzers", type=int, default=2)
    ap.add_argument("--log-dir", default="./logs")
    ap.add_argument("--no-engine", action="store_true")
    a = ap.parse_args(argv)
    env = dict(os.environ)
    env.update(load_env_file(a.env))
    env.setdefault("QUEUE_PROVIDER", "broker")
    env.setdefault("QUEUE_URL", "nats://127.0.0.1:4222")
    env.setdefault("CACHE_PROVIDER", "kv")
    env.setdefault("REDIS_ADDR", "127.0.0.1:6379")
    env.setdefault("LLM_PROVIDER", "engine")
    env.setdefault("ENGINE_URL", "tcp://127.0.0.1:9090")
    env.setdefault("QUERY_SERVICE_URL", "http://127.0.0.1:8081/api/query")
    os.makedirs(a.log_dir, exist_ok=True)
    py = sys.executable
    procs: list[Proc] = []
    bh, bp = _hostport(env["QUEUE_URL"], 4222)
    kh, kp = _hostport(env["REDIS_ADDR"], 6379)
    procs.append(Proc("broker", [py, "-m", "docagents_amd.services", "broker", "--listen", f"0.0.0.0:{bp}"], env,
                      (bh, bp), critical=True))
    kv_cmd = [py, "-m", "docagents_amd.services", "kvcache", "--listen", f"0.0.0.0:{kp}"]
    procs.append(Proc("kvcache", kv_cmd, env, (kh, kp), critical=True))
    if env["LLM_PROVIDER"] in ("engine", "openai") and not a.no_engine:
        eh, ep = _hostport(env["ENGINE_URL"], 9090)
        if a.gpus > 1:
            cmd = [py, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
                   "--master-addr", "127.0.0.1", "--master-port", env.get("ENGINE_MASTER_PORT", "29600"),
                   "-m", "docagents_amd.services", "engine", "--listen", f"tcp://0.0.0.0:{ep}"]
        else:
            cmd = [py, "-m", "docagents_amd.services", "engine", "--listen", f"tcp://0.0.0.0:{ep}"]
        procs.append(Proc("engine", cmd, env, (eh, ep), critical=True))
    procs.append(Proc("query", [py, "-m", "docagents_amd.services", "query"], dict(env, PORT="8081"), ("127.0.0.1", 8081)))
    procs.append(Proc("gateway", [py, "-m", "docagents_amd.services", "gateway"], dict(env, PORT="8080"),
                      ("127.0.0.1", 8080)))
    for i in range(a.parsers):
        procs.append(Proc(f"parser-{i}", [py, "-m", "docagents_amd.services", "parser"], dict(env, PORT=str(8082 + 10 * i))))
    for i in range(a.analyzers):
        procs.append(Proc(f"analysis-{i}", [py, "-m", "docagents_amd.services", "analysis"],
                          dict(env, PORT=str(8083 + 10 * i))))
    stop = {"flag": False}

    def on_sig(*_):
        stop["flag"] = True
    signal.signal(signal.SIGINT, on_sig)
    signal.signal(signal.SIGTERM, on_sig)
    for p in procs:
        p.start(a.log_dir)
        if p.wait and not _wait_tcp(*p.wait, timeout=600 if p.name == "engine" else 60):
            print(f"[deploy] {p.name} did not become healthy; see {a.log_dir}/{p.name}.log", file=sys.stderr)
            stop["flag"] = True
            break
        print(f"[deploy] {p.name} up", file=sys.stderr)
    while not stop["flag"]:
        time.sleep(0.5)
        for p in procs:
            if p.proc is not None and p.proc.poll() is not None and time.time() >= p.next_start:
                p.restarts += 1
                delay = min(30.0, 0.5 * 2 ** min(p.restarts, 6))
                print(f"[deploy] {p.name} exited ({p.proc.returncode}); restart #{p.restarts} in {delay:.1f}s",
                      file=sys.stderr)
                p.next_start = time.time() + delay
                p.proc = None
            elif p.proc is None and time.time() >= p.next_start:
                p.start(a.log_dir)
    for p in reversed(procs):
        if p.proc is not None and p.proc.poll() is None:
            os.killpg(p.proc.pid, signal.SIGTERM)
    for p in reversed(procs):
        if p.proc is not None:
            try:
                p.proc.wait(30)
            except subprocess.TimeoutExpired:
                os.killpg(p.proc.pid, signal.SIGKILL)
    return 0


if __name__ == "__main__":
    sys.exit(main())
