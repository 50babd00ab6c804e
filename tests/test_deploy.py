"""deploy.py — the docker-compose.yml equivalent (reference docker-compose.yml:45-128) — brought up as
real separate processes: native broker + native KV cache (+ the engine server) + query + gateway +
2 parsers + 2 analyzers. Drives upload -> summary -> query -> cached query through the gateway,
checks that a killed worker is restarted, and that SIGTERM takes the whole tree down."""
import json
import os
import signal
import socket
import subprocess
import sys
import time

import httpx

from docagents_amd.text import multipart

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_block(n=40):
    """A base port with [base, base + n) free."""
    for _ in range(50):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        base = s.getsockname()[1]
        s.close()
        if base + n >= 65000:
            continue
        ok = True
        for p in range(base, base + n):
            t = socket.socket()
            try:
                t.bind(("127.0.0.1", p))
            except OSError:
                ok = False
            finally:
                t.close()
            if not ok:
                break
        if ok:
            return base
    raise RuntimeError("no free port block")


def _status(log_dir):
    with open(os.path.join(log_dir, "status.json")) as f:
        return {p["name"]: p for p in json.load(f)["procs"]}


def _wait(pred, timeout, what):
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            v = pred()
            if v:
                return v
        except Exception:  # noqa: BLE001
            pass
        time.sleep(0.2)
    raise TimeoutError(what)


def _bring_up(tmp_path, extra_env, n_expected):
    base = _free_block()
    log_dir = str(tmp_path / "logs")
    env = dict(os.environ, PYTHONPATH=ROOT, STORE_PROVIDER="sqlite", DB_PATH=str(tmp_path / "meta.sqlite3"),
               DATA_DIR=str(tmp_path), QUEUE_URL=f"nats://127.0.0.1:{base + 30}",
               REDIS_ADDR=f"127.0.0.1:{base + 31}", REDIS_PASSWORD="pw", ENGINE_URL=f"tcp://127.0.0.1:{base + 32}",
               MIN_SIMILARITY="-1", LOG_LEVEL="warn", **extra_env)
    sup = subprocess.Popen([sys.executable, "-m", "docagents_amd.deploy", "--base-port", str(base), "--log-dir", log_dir],
                           env=env, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=open(tmp_path / "deploy.err", "w"),
                           start_new_session=True)
    gw = f"http://127.0.0.1:{base}"
    try:
        _wait(lambda: len([p for p in _status(log_dir).values() if p["pid"]]) == n_expected, 600,
              "every service up")
    except TimeoutError:
        sup.kill()
        raise AssertionError(open(tmp_path / "deploy.err").read()[-3000:])
    return sup, gw, log_dir


def _down(sup, log_dir):
    pids = [p["pid"] for p in _status(log_dir).values() if p["pid"]]
    sup.send_signal(signal.SIGTERM)
    try:
        sup.wait(timeout=90)
    except subprocess.TimeoutExpired:
        for pid in pids + [sup.pid]:  # never leave the tree behind, then fail
            try:
                os.killpg(pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
        raise
    time.sleep(0.2)
    for pid in pids:  # every child gone (no orphans)
        try:
            os.kill(pid, 0)
            alive = True
        except ProcessLookupError:
            alive = False
        assert not alive, f"pid {pid} survived the supervisor"


def _upload(gw, name, text):
    body, ctype = multipart.build({}, {"file": (name, text.encode(), "text/plain")})
    r = httpx.post(gw + "/api/documents/upload", content=body, headers={"content-type": ctype}, timeout=30)
    assert r.status_code == 202, r.text
    return r.json()["document_id"]


def _flow(gw, docs_text, question):
    ids = [_upload(gw, f"doc{i}.txt", t) for i, t in enumerate(docs_text)]
    for d in ids:
        s = _wait(lambda: httpx.get(f"{gw}/api/documents/{d}/summary", timeout=10).status_code == 200 and
                  httpx.get(f"{gw}/api/documents/{d}/summary", timeout=10).json(), 300, "summary")
        assert s["documentId"] == d
    body = {"question": question, "document_ids": ids, "top_k": 3}
    # embeddings land after the summary: probe with distinct questions until sources appear
    _wait(lambda: httpx.post(gw + "/api/query", json=dict(body, question=f"{question} {time.time()}"),
                             timeout=120).json()["sources"], 300, "sources")
    q = httpx.post(gw + "/api/query", json=body, timeout=120)
    assert q.status_code == 200, q.text
    j = q.json()
    assert j["cached"] is False and len(j["sources"]) == 3
    q2 = httpx.post(gw + "/api/query", json=body, timeout=60)
    assert q2.json()["cached"] is True and q2.json()["answer"] == j["answer"]
    return ids, j


def test_deploy_stub_stack_end_to_end_and_restart(tmp_path):
    sup, gw, log_dir = _bring_up(tmp_path, {"LLM_PROVIDER": "stub", "EMBED_DIM": "64"}, 8)
    try:
        text = ("The MI355X accelerator has 256 compute units and 288 GB of HBM3E memory. " * 60).strip()
        _, j = _flow(gw, [text, "A second document about xGMI links and RCCL collectives. " * 40],
                     "How much memory does the MI355X have?")
        assert j["answer"].startswith("According to the documentation")
        # kill one worker: the supervisor restarts it (compose restart policy)
        st = _status(log_dir)
        victim = st["parser-0"]["pid"]
        os.killpg(victim, signal.SIGKILL)
        _wait(lambda: _status(log_dir)["parser-0"]["pid"] not in (None, victim) and
              _status(log_dir)["parser-0"]["restarts"] == 1, 60, "parser restart")
        d = _upload(gw, "after.txt", "Text uploaded after the restart of a parser worker. " * 30)
        _wait(lambda: httpx.get(f"{gw}/api/documents/{d}/summary", timeout=10).status_code == 200, 120,
              "summary after restart")
    finally:
        _down(sup, log_dir)


def test_deploy_engine_stack_on_cpu_direct_ingest(tmp_path):
    """The GPU topology with the engine server running tiny models on the CPU: analysis ingests through
    ``embed_index`` (vectors written into the engine shard, durably logged) and the query service
    answers from the engine."""
    env = {"LLM_PROVIDER": "engine", "EMBED_ARCH": "tiny-enc", "LLM_ARCH": "tiny-dec", "CUDA_VISIBLE_DEVICES": "",
           "HIP_VISIBLE_DEVICES": "", "MAX_NEW_TOKENS": "8", "SUMMARY_MAX_NEW_TOKENS": "8", "ENGINE_MAX_BATCH": "8",
           "INDEX_DIR": str(tmp_path / "index")}
    sup, gw, log_dir = _bring_up(tmp_path, env, 9)
    try:
        docs = ["Alpha document about compute units and wavefronts. " * 50,
                "Beta document about HBM bandwidth and the Infinity Cache. " * 50]
        ids, j = _flow(gw, docs, "What is the Infinity Cache?")
        assert isinstance(j["answer"], str) and 0.0 <= j["confidence"] <= 1.0
        # the vectors went through the engine's durable shard log, not through the agents
        wal = [f for f in os.listdir(tmp_path / "index") if f.startswith("shard0.wal.")]
        assert wal and os.path.getsize(tmp_path / "index" / wal[0]) > 0
    finally:
        _down(sup, log_dir)
