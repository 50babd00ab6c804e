"""Engine observability: step watchdog, rank liveness, torch.profiler capture.

The reference has no engine (compute is a remote API call with a 30 s client timeout,
internal/llm/openai.go:20-23) and no tracing or watchdog (README.md:706-722). Here:

* ``Watchdog`` — every GPU command runs between ``begin``/``end``. A monitor thread flags the
  engine unhealthy when one command exceeds ``soft_s`` (the ``health`` RPC then reports it, and
  the query/analysis agents' engine client fails fast instead of queueing behind a hung GPU),
  and, when ``hard_s`` > 0, terminates the process so the supervisor (``deploy.py``) restarts it.
  A hung collective on one rank shows up here on rank 0 as a stuck command.
* ``liveness`` — the C7 all-reduce run periodically on idle engines (``EngineServer``).
* ``StepProfiler`` — ``DA_TORCH_PROFILE=<dir>[:<n>]`` wraps the next ``n`` engine commands in
  ``torch.profiler`` and writes a Chrome trace plus a kernel summary table per command.
"""
from __future__ import annotations

import os
import sys
import threading
import time

from ..utils import metrics


class Watchdog:
    def __init__(self, soft_s: float = 120.0, hard_s: float = 0.0, log=None, poll_s: float = 1.0,
                 on_hard=None):
        self.soft_s, self.hard_s, self.log, self.poll_s = soft_s, hard_s, log, poll_s
        self.on_hard = on_hard or self._die
        self._lock = threading.Lock()
        self._cur: tuple[str, float] | None = None
        self.stuck: str | None = None
        self.steps = 0
        self.last_ok = time.time()
        self._stop = threading.Event()
        self._thr = None
        metrics.ENGINE_HEALTHY.set(1)

    def start(self):
        if self._thr is None:
            self._thr = threading.Thread(target=self._run, name="engine-watchdog", daemon=True)
            self._thr.start()
        return self

    def stop(self):
        self._stop.set()

    def begin(self, cmd: str):
        with self._lock:
            self._cur = (cmd, time.monotonic())

    def end(self):
        with self._lock:
            self._cur = None
            self.steps += 1
            self.last_ok = time.time()
            if self.stuck is not None:
                if self.log:
                    self.log.warn("engine step recovered", "cmd", self.stuck)
                self.stuck = None
                metrics.ENGINE_HEALTHY.set(1)

    def check(self, now: float | None = None):
        """One monitor tick (also called directly by tests)."""
        now = time.monotonic() if now is None else now
        with self._lock:
            cur = self._cur
        if cur is None:
            return
        cmd, t0 = cur
        el = now - t0
        if el > self.soft_s and self.stuck is None:
            self.stuck = cmd
            metrics.ENGINE_HEALTHY.set(0)
            if self.log:
                self.log.error("engine step exceeded watchdog timeout", "cmd", cmd, "elapsed_s", round(el, 1))
        if self.hard_s > 0 and el > self.hard_s:
            if self.log:
                self.log.error("engine step hung; terminating for restart", "cmd", cmd, "elapsed_s", round(el, 1))
            self.on_hard(cmd, el)

    @property
    def healthy(self) -> bool:
        return self.stuck is None

    def state(self) -> dict:
        with self._lock:
            cur = self._cur
        return {"ok": self.healthy, "stuck": self.stuck, "steps": self.steps, "last_ok": self.last_ok,
                "running": None if cur is None else {"cmd": cur[0], "elapsed_s": time.monotonic() - cur[1]}}

    def _run(self):
        while not self._stop.wait(self.poll_s):
            self.check()

    @staticmethod
    def _die(cmd, el):
        sys.stderr.flush()
        os._exit(70)  # EX_SOFTWARE; the supervisor restarts the engine (deploy.py)


class StepProfiler:
    """torch.profiler around engine commands, enabled by ``DA_TORCH_PROFILE=<dir>[:<n>]``."""

    def __init__(self, spec: str | None = None, rank: int = 0):
        spec = os.environ.get("DA_TORCH_PROFILE", "") if spec is None else spec
        self.dir, self.left, self.rank, self.n = "", 0, rank, 0
        if spec:
            d, _, n = spec.partition(":")
            self.dir, self.left = d, int(n or 8)
            os.makedirs(self.dir, exist_ok=True)

    @property
    def active(self) -> bool:
        return self.left > 0

    def run(self, cmd: str, fn, *a):
        if not self.active:
            return fn(*a)
        import torch
        acts = [torch.profiler.ProfilerActivity.CPU]
        if torch.cuda.is_available():
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        with torch.profiler.profile(activities=acts, record_shapes=False) as prof:
            with torch.profiler.record_function(f"engine.{cmd}"):
                out = fn(*a)
            if torch.cuda.is_available():
                torch.cuda.synchronize()
        self.n += 1
        self.left -= 1
        base = os.path.join(self.dir, f"rank{self.rank}_{self.n:03d}_{cmd}")
        prof.export_chrome_trace(base + ".json")
        key = "self_cuda_time_total" if torch.cuda.is_available() else "self_cpu_time_total"
        with open(base + ".txt", "w") as f:
            f.write(prof.key_averages().table(sort_by=key, row_limit=40))
        return out


def device_memory(dev) -> dict:
    import torch
    if getattr(dev, "type", "cpu") != "cuda":
        return {}
    return {"allocated": torch.cuda.memory_allocated(dev), "reserved": torch.cuda.memory_reserved(dev)}
