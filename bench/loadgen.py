"""HTTP load generator for the full agent stack (SURVEY.md §7.1 "bench/").

Drives the public API exactly like a client of the reference would (README.md of the reference:
upload -> poll summary -> query), through the gateway:

  1. ingest: upload ``--docs`` synthetic documents (``--concurrency`` in flight), poll each
     summary until it is ready -> docs/min from the first upload to the last ready summary;
  1b. unloaded ingest latency: ``--serial-docs`` more documents uploaded one at a time, each
     polled (every 10 ms) until its summary reads 200 -> p50 / p90 upload -> summary readable, the
     reference's only ingest number ("wait 2-3 seconds", README.md:346);
  2. unloaded cache-miss latency: ``--serial-queries`` unique questions sent one at a time
     (concurrency 1) -> p50 / p90 / p99 through gateway proxy -> query service -> engine, the
     number the reference publishes ("~2-3 seconds", README.md:590);
  3. cache-miss queries: ``--queries`` unique questions over the ingested documents -> QPS and
     p50/p99 latency (embed + search + answer inside the stack) at ``--concurrency`` in flight;
  4. cache-hit queries: the same questions again -> p50/p99 (served from the query cache; the
     reference promises "sub-millisecond" server-side, README.md:588).

``--spawn`` starts the multi-process deploy.py stack (``--topology deploy``, default) or the all-in-one
process (``--topology all``) on free ports
with the current environment (``LLM_PROVIDER=stub`` on CPU, ``engine`` with ``ENGINE_URL`` set for
the GPU engine); otherwise ``--gateway URL`` targets a running deployment. Prints one JSON line.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import socket
import statistics
import subprocess
import sys
import threading
import time

import httpx

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from docagents_amd.text import multipart  # noqa: E402
from docagents_amd.text.synthetic import TextGen  # noqa: E402
from docagents_amd.utils import timeline as req_timeline  # noqa: E402


def _tenths(done_at: list[float], span: float) -> list[float] | None:
    """Completions per tenth of a run of ``span`` seconds, as q/s (done_at: seconds from its start)."""
    if span <= 0:
        return None
    n = [0] * 10
    for x in done_at:
        n[min(9, max(0, int(x * 10 / span)))] += 1
    return [round(c / (span / 10), 1) for c in n]


def _cpu_sampler(stop, out: dict, every: float = 0.5):
    """Sample the CPU use (cores) of this process and its descendants until ``stop``; ``out`` gets
    {"<name>#<pid>": {"mean": m, "max": x}} keyed by the service name from the command line."""
    import psutil
    me = psutil.Process()
    seen: dict = {}
    samples: dict = {}
    while not stop.is_set():
        for p in [me] + me.children(recursive=True):
            try:
                if p.pid not in seen:
                    seen[p.pid] = p
                    p.cpu_percent(None)  # prime
                    continue
                v = seen[p.pid].cpu_percent(None) / 100.0
                cmd = p.cmdline()
                name = next((c for c in reversed(cmd) if c in ("gateway", "query", "engine", "parser", "analysis",
                                                              "broker", "kvcache", "all")), os.path.basename(cmd[-1]) if cmd else "?")
                samples.setdefault(f"{name}#{p.pid}", []).append(v)
            except (psutil.NoSuchProcess, psutil.AccessDenied, IndexError):
                pass
        stop.wait(every)
    for k, xs in samples.items():
        if xs and max(xs) > 0.05:
            out[k] = {"mean": round(sum(xs) / len(xs), 2), "max": round(max(xs), 2)}


def _pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(round(q / 100.0 * (len(xs) - 1))))]


def _ephemeral_range() -> tuple[int, int]:
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            lo, hi = (int(x) for x in f.read().split())
        return lo, hi
    except (OSError, ValueError):
        return 32768, 60999


def _free_block(n: int = 40) -> int:
    """A base port with [base, base + n) free on every interface (the deploy topology's port plan),
    BELOW the kernel's ephemeral range: the services' own outgoing connections take local ports from
    that range, and one of them holding a planned port made a service fail to bind (a GPU-box stack
    run whose query service restarted three times on 'address already in use')."""
    import random
    lo, hi = _ephemeral_range()
    top = lo - n - 1 if lo - n - 1 > 10000 else 65000 - n
    bottom = 10000 if top == lo - n - 1 else hi + 1
    rng = random.Random(os.getpid() ^ int(time.time() * 1000))
    for _ in range(200):
        base = rng.randrange(bottom, top)
        ok = True
        for p in range(base, base + n):
            t = socket.socket()
            try:
                t.bind(("0.0.0.0", p))
            except OSError:
                ok = False
            finally:
                t.close()
            if not ok:
                break
        if ok:
            return base
    raise RuntimeError("no free port block")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


async def _wait_ready(client, url, timeout=120.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            if (await client.get(url, timeout=2.0)).status_code == 200:
                return
        except Exception:  # noqa: BLE001
            pass
        await asyncio.sleep(0.2)
    raise TimeoutError(url)


def _raw_hits(url: str, bodies: list[str]) -> list[float]:
    """Sequential POST /api/query over one keep-alive socket with no client library in the way:
    the latency a cache hit costs the stack itself (the httpx client adds ~1 ms per request)."""
    import socket
    from urllib.parse import urlsplit
    u = urlsplit(url)
    s = socket.create_connection((u.hostname, u.port))
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    out = []
    try:
        for b in bodies:
            data = b.encode()
            req = (f"POST /api/query HTTP/1.1\r\nHost: {u.hostname}\r\nContent-Type: application/json\r\n"
                   f"Content-Length: {len(data)}\r\n\r\n").encode() + data
            t = time.perf_counter()
            s.sendall(req)
            buf = b""
            while True:
                buf += s.recv(65536)
                head, sep, rest = buf.partition(b"\r\n\r\n")
                if not sep:
                    continue
                n = next(int(ln.split(b":")[1]) for ln in head.split(b"\r\n") if ln.lower().startswith(b"content-length"))
                if len(rest) >= n:
                    break
            out.append((time.perf_counter() - t) * 1000.0)
    finally:
        s.close()
    return out


async def run(gw: str, docs: int, words: int, queries: int, concurrency: int, top_k: int, seed: int,
              poll_s: float = 0.05, ingest_timeout: float = 600.0, query_url: str = "", serial: int = 50,
              serial_docs: int = 10, partial: int = 20) -> dict:
    tg = TextGen(seed=seed)
    texts = [tg.document(words) for _ in range(docs)]
    sem = asyncio.Semaphore(concurrency)
    limits = httpx.Limits(max_connections=concurrency * 2, max_keepalive_connections=concurrency * 2)
    # queries: the pooled keep-alive client the gateway itself uses (api/proxy.py). At 128 in flight
    # httpx saturated this process's core and queued requests ~1.3-2.4 s before they reached the
    # gateway (bench/timeline_report.py: loadgen_to_gateway; a stub LLM with fixed 2 s answers
    # showed it without any GPU), which is the harness, not the stack
    from docagents_amd.api.proxy import PooledHTTPClient
    qclient = PooledHTTPClient(timeout=120.0, max_idle=concurrency * 2)
    async with httpx.AsyncClient(timeout=120.0, limits=limits) as client:
        await _wait_ready(client, gw + "/healthz")

        # ---- ingest ----
        ids: list[str] = []
        ready_at: dict[str, float] = {}

        async def upload(i):
            body, ctype = multipart.build({}, {"file": (f"doc{i}.txt", texts[i].encode(), "text/plain")})
            async with sem:
                r = await client.post(gw + "/api/documents/upload", content=body, headers={"content-type": ctype})
            r.raise_for_status()
            return r.json()["document_id"]

        t0 = time.perf_counter()
        ids = list(await asyncio.gather(*[upload(i) for i in range(docs)]))
        t_up = time.perf_counter()

        async def poll(doc_id):
            while time.perf_counter() - t0 < ingest_timeout:
                r = await client.get(f"{gw}/api/documents/{doc_id}/summary")
                if r.status_code == 200:
                    ready_at[doc_id] = time.perf_counter()
                    return True
                await asyncio.sleep(poll_s)
            return False

        ok = await asyncio.gather(*[poll(d) for d in ids])
        t_ingest = (max(ready_at.values()) - t0) if ready_at else None
        ready = [d for d, o in zip(ids, ok) if o]
        # ingest timeline: when the uploads were all accepted and how the summaries trickled in
        rt = sorted(v - t0 for v in ready_at.values())
        timeline = {"uploads_accepted_s": _r(t_up - t0), "first_ready_s": _r(rt[0]) if rt else None,
                    "median_ready_s": _r(statistics.median(rt)) if rt else None,
                    "last_ready_s": _r(rt[-1]) if rt else None}

        # ---- unloaded ingest latency: one document at a time, upload -> summary readable ----
        serial_ingest = []
        for i in range(serial_docs):
            t_s = time.perf_counter()
            body, ctype = multipart.build({}, {"file": (f"serial{i}.txt", tg.document(words).encode(), "text/plain")})
            r = await client.post(gw + "/api/documents/upload", content=body, headers={"content-type": ctype})
            r.raise_for_status()
            did = r.json()["document_id"]
            while time.perf_counter() - t_s < 120:
                if (await client.get(f"{gw}/api/documents/{did}/summary")).status_code == 200:
                    serial_ingest.append((time.perf_counter() - t_s) * 1000.0)
                    break
                await asyncio.sleep(0.01)

        # ---- queries ----
        qs = [f"What does {tg.word()} say about {tg.word()} and {tg.word()}?" for _ in range(queries)]
        bodies = []
        for i, q in enumerate(qs):
            pick = [ready[(i + j) % len(ready)] for j in range(min(3, len(ready)))] if ready else []
            bodies.append(json.dumps({"question": q, "document_ids": pick, "top_k": top_k}))

        async def ask(body):
            async with sem:
                if req_timeline.enabled():
                    req_timeline.mark("l_send", q=json.loads(body)["question"])
                t = time.perf_counter()
                try:
                    status, _ = await qclient.post(gw + "/api/query", body.encode(), {"Content-Type": "application/json"})
                except Exception:  # noqa: BLE001 - counted as an error, like a failed response
                    status = 599
                dt = (time.perf_counter() - t) * 1000.0
                if req_timeline.enabled():
                    req_timeline.mark("l_recv", q=json.loads(body)["question"], status=status)
            return status, dt

        # ---- unloaded cache misses: one request in flight ----
        sq = [json.dumps({"question": f"Serial question {i}: what about {tg.word()} and {tg.word()}?",
                          "document_ids": [ready[(7 * i + j) % len(ready)] for j in range(min(3, len(ready)))],
                          "top_k": top_k}) for i in range(serial)] if ready else []
        for b in sq[:2]:  # warm the batch-1 paths (graph capture) before timing
            await ask(b.replace("Serial question", "Warm-up question"))
        mbase = query_url.rsplit("/api/", 1)[0] + "/metrics" if query_url else ""
        before = _stage_sums(mbase) if mbase else {}
        serial_res = [await ask(b) for b in sq]
        serial_stages = _stage_delta(before, _stage_sums(mbase)) if mbase else {}
        # partial hits (the reference's "~2-2.5 s", README.md:589): the same questions with another
        # top_k — a new query-cache key, so search + answer run, but the question's embedding comes
        # from the embedding cache (no encoder pass)
        pq = []
        for b in sq[:max(0, partial)]:
            d = json.loads(b)
            d["top_k"] = top_k + 1 if top_k < 20 else top_k - 1
            pq.append(json.dumps(d))
        partial_res = [await ask(b) for b in pq]

        t1 = time.perf_counter()
        cpu_stop = threading.Event()
        cpu_out: dict = {}
        cpu_thr = threading.Thread(target=_cpu_sampler, args=(cpu_stop, cpu_out), daemon=True)
        cpu_thr.start()
        miss_done: list[float] = []

        async def ask_loaded(b):
            r = await ask(b)
            miss_done.append(time.perf_counter() - t1)
            return r

        async def progress():  # a long (soak) run reports every 30 s
            while True:
                await asyncio.sleep(30)
                print(f"[loadgen] {len(miss_done)}/{len(bodies)} queries done, "
                      f"{time.perf_counter() - t1:.0f} s", file=sys.stderr, flush=True)
        prog = asyncio.ensure_future(progress())
        miss = await asyncio.gather(*[ask_loaded(b) for b in bodies])
        prog.cancel()
        t_miss = time.perf_counter() - t1
        cpu_stop.set()
        cpu_thr.join(5)
        hit = []
        for b in bodies:  # sequential: per-request latency of a cache hit, not throughput
            hit.append(await ask(b))
        raw_gw = await asyncio.to_thread(_raw_hits, gw, bodies)
        raw_q = await asyncio.to_thread(_raw_hits, query_url, bodies) if query_url else []
        handler_ms = None
        if query_url:
            m = (await client.get(query_url.rsplit("/api/", 1)[0] + "/metrics")).text
            vals = {ln.split("{")[0]: float(ln.split()[-1]) for ln in m.splitlines()
                    if ln.startswith("da_query_stage_seconds_") and 'stage="cache_hit"' in ln}
            if vals.get("da_query_stage_seconds_count"):
                handler_ms = vals["da_query_stage_seconds_sum"] / vals["da_query_stage_seconds_count"] * 1000.0

    miss_ok = [dt for st, dt in miss if st == 200]
    serial_ok = [dt for st, dt in serial_res if st == 200]
    hit_ok = [dt for st, dt in hit if st == 200]
    return {
        "metric": "http_stack", "docs": docs, "docs_ready": len(ready), "words_per_doc": words,
        "ingest_docs_per_min": round(len(ready) / t_ingest * 60.0, 1) if t_ingest else None,
        "serial_ingest_docs": len(serial_ingest),
        "serial_ingest_p50_ms": _r(statistics.median(serial_ingest) if serial_ingest else None),
        "serial_ingest_p90_ms": _r(_pct(serial_ingest, 90)),
        "reference_ingest_ms": "2000-3000 (README.md:346, 'wait 2-3 seconds')",
        "serial_queries": len(serial_res), "serial_errors": sum(1 for st, _ in serial_res if st != 200),
        "serial_cache_miss_p50_ms": _r(statistics.median(serial_ok) if serial_ok else None),
        "serial_cache_miss_p90_ms": _r(_pct(serial_ok, 90)),
        "serial_cache_miss_p99_ms": _r(_pct(serial_ok, 99)),
        "serial_partial_hit_queries": len(partial_res),
        "serial_partial_hit_p50_ms": _r(statistics.median([dt for st, dt in partial_res if st == 200]) if any(
            st == 200 for st, _ in partial_res) else None),
        "reference_partial_hit_ms": "2000-2500 (README.md:589)",
        "serial_stage_mean_ms": serial_stages,
        "queries": queries, "query_errors": sum(1 for st, _ in miss if st != 200),
        "qa_qps": round(len(miss_ok) / t_miss, 2) if t_miss > 0 else None,
        # completions per tenth of the loaded run (q/s): flat = steady state (a soak shows no drift)
        "qa_qps_tenths": _tenths(miss_done, t_miss),
        "cache_miss_p50_ms": _r(statistics.median(miss_ok) if miss_ok else None),
        "cache_miss_p99_ms": _r(_pct(miss_ok, 99)),
        "cache_hit_p50_ms": _r(statistics.median(hit_ok) if hit_ok else None),
        "cache_hit_p99_ms": _r(_pct(hit_ok, 99)),
        "cache_hit_gateway_raw_p50_ms": _r(statistics.median(raw_gw) if raw_gw else None),
        "cache_hit_query_service_raw_p50_ms": _r(statistics.median(raw_q) if raw_q else None),
        "cache_hit_handler_mean_ms": _r(handler_ms),
        "concurrency": concurrency, "top_k": top_k, "ingest_timeline": timeline,
        # CPU use of every process of the stack (and this one) while the concurrent queries ran,
        # in cores (1.0 = one core busy): a saturated single-threaded front end shows as ~1.0
        "cpu_cores_during_queries": cpu_out,
    }


def _stage_sums(url: str) -> dict:
    """{stage: (sum_s, count)} of the query service's da_query_stage_seconds histogram."""
    out = {}
    try:
        text = httpx.get(url, timeout=5.0).text
    except Exception:  # noqa: BLE001
        return out
    for ln in text.splitlines():
        for suf, i in (("_sum", 0), ("_count", 1)):
            pre = "da_query_stage_seconds" + suf + "{"
            if ln.startswith(pre):
                st = ln.split('stage="', 1)[1].split('"', 1)[0]
                out.setdefault(st, [0.0, 0.0])[i] = float(ln.split()[-1])
    return out


def _stage_delta(a: dict, b: dict) -> dict:
    res = {}
    for st, (s1, c1) in b.items():
        s0, c0 = a.get(st, (0.0, 0.0))
        if c1 > c0:
            res[st] = round((s1 - s0) / (c1 - c0) * 1000.0, 3)
    return res


def _scrape(url: str, names: tuple[str, ...]) -> dict:
    """Mean of each Prometheus histogram ``name{label}`` (sum / count) at a /metrics URL."""
    try:
        text = httpx.get(url, timeout=5.0).text
    except Exception as e:  # noqa: BLE001
        return {"error": repr(e)}
    acc: dict = {}
    for ln in text.splitlines():
        for n in names:
            for suf in ("_sum", "_count"):
                if ln.startswith(n + suf):
                    lab = ln[len(n + suf):].split(" ")[0]
                    acc.setdefault(n + lab, {})[suf] = float(ln.split()[-1])
    return {k: {"n": int(v.get("_count", 0)), "mean_ms": _r(v["_sum"] / v["_count"] * 1000.0)}
            for k, v in acc.items() if v.get("_count")}


async def _engine_stats(url: str) -> dict:
    from docagents_amd.engine.rpc import EngineCluster
    c = EngineCluster(url, timeout=30.0)
    try:
        await c.connect(retries=2)
        st = await c.call("stats")
    finally:
        await c.close()
    if "replicas" in st:  # several replicas: report replica 0's view (plus the count)
        st = dict(st["replicas"][0], replicas=len(st["replicas"]))
    r0 = st["ranks"][0] if st.get("ranks") else {}
    return {"exec": st.get("exec"), "batching": st.get("batching"), "gen": r0.get("gen"), "embed": r0.get("embed"),
            "sched": r0.get("sched"), "rpc_mean_ms": st.get("rpc_mean_ms")}


def diagnostics(base: int, parsers: int = 2, analyzers: int = 2, engine_url: str = "") -> dict:
    """Where the time went inside the deploy stack: per-service handler latencies (worker /metrics),
    query stages, and the engine's batching + generator counters."""
    out = {"query": _scrape(f"http://127.0.0.1:{base + 1}/metrics", ("da_query_stage_seconds",))}
    for i in range(parsers):
        out[f"parser-{i}"] = _scrape(f"http://127.0.0.1:{base + 2 + 10 * i}/metrics", ("da_task_seconds",))
    for i in range(analyzers):
        out[f"analysis-{i}"] = _scrape(f"http://127.0.0.1:{base + 3 + 10 * i}/metrics", ("da_task_seconds",))
    if engine_url:
        try:
            out["engine"] = asyncio.run(_engine_stats(engine_url))
        except Exception as e:  # noqa: BLE001
            out["engine"] = {"error": repr(e)}
    return out


def _r(x):
    return None if x is None else round(x, 3)


def main(argv=None):
    ap = argparse.ArgumentParser("loadgen")
    ap.add_argument("--gateway", default="")
    ap.add_argument("--spawn", action="store_true", help="start a stack for the run (see --topology)")
    ap.add_argument("--topology", default="deploy", choices=["deploy", "all"],
                    help="deploy: the compose-equivalent multi-process stack (native broker + KV cache, engine "
                         "server when LLM_PROVIDER=engine, query, gateway, 2 parsers, 2 analyzers); all: every "
                         "agent in one process with the in-process bus")
    ap.add_argument("--docs", type=int, default=32)
    ap.add_argument("--words", type=int, default=2000)
    ap.add_argument("--queries", type=int, default=64)
    ap.add_argument("--serial-queries", type=int, default=50, help="unloaded (concurrency 1) cache-miss queries")
    ap.add_argument("--serial-docs", type=int, default=10, help="unloaded single-document uploads (upload -> summary)")
    ap.add_argument("--partial-queries", type=int, default=20,
                    help="unloaded partial hits: serial questions again with another top_k (embedding cached)")
    ap.add_argument("--concurrency", type=int, default=16)
    ap.add_argument("--top-k", type=int, default=5)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--query-url", default="", help="query service URL (direct cache-hit timing)")
    a = ap.parse_args(argv)
    proc = None
    gw = a.gateway
    sup_log = None
    if a.spawn or not gw:
        port = _free_port() if a.topology == "all" else _free_block()
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env = dict(os.environ, PORT=str(port),
                   PYTHONPATH=os.pathsep.join(x for x in (root, os.environ.get("PYTHONPATH", "")) if x))
        env.setdefault("MIN_SIMILARITY", "-1")
        tmp = os.environ.get("TMPDIR", "/tmp")
        env.setdefault("DB_PATH", os.path.join(tmp, f"loadgen-{port}.sqlite3"))
        if a.topology == "all":
            proc = subprocess.Popen([sys.executable, "-m", "docagents_amd.services", "all"], env=env,
                                    stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        else:
            env.setdefault("QUEUE_URL", f"nats://127.0.0.1:{port + 30}")
            env.setdefault("REDIS_ADDR", f"127.0.0.1:{port + 31}")
            env.setdefault("ENGINE_URL", f"tcp://127.0.0.1:{port + 32}")
            env.setdefault("DATA_DIR", os.path.join(tmp, f"loadgen-{port}"))
            sup_log = os.path.join(tmp, f"loadgen-{port}-logs")
            proc = subprocess.Popen([sys.executable, "-m", "docagents_amd.deploy", "--base-port", str(port),
                                     "--log-dir", sup_log], env=env, stdout=subprocess.DEVNULL,
                                    stderr=subprocess.DEVNULL, start_new_session=True)
        gw = f"http://127.0.0.1:{port}"
        if sup_log:  # the whole stack, not just the gateway (workers start after it)
            t0 = time.time()
            while True:
                try:
                    with open(os.path.join(sup_log, "status.json")) as f:
                        if json.load(f).get("ready"):
                            break
                except (OSError, ValueError):
                    pass
                if time.time() - t0 > 900 or proc.poll() is not None:
                    raise RuntimeError(f"deploy stack did not come up; see {sup_log}")
                time.sleep(0.25)
    try:
        qurl = f"http://127.0.0.1:{int(gw.rsplit(':', 1)[1]) + 1}/api/query" if proc is not None else a.query_url
        out = asyncio.run(run(gw, a.docs, a.words, a.queries, a.concurrency, a.top_k, a.seed, query_url=qurl,
                              serial=a.serial_queries, serial_docs=a.serial_docs, partial=a.partial_queries))
        out["topology"] = a.topology if proc is not None else "external"
        if proc is not None and a.topology == "deploy":
            eng = env.get("ENGINE_URL", "") if env.get("LLM_PROVIDER") == "engine" else ""
            out["diag"] = diagnostics(port, engine_url=eng)
    finally:
        if proc is not None:
            proc.terminate()
            try:
                proc.wait(120 if sup_log else 10)
            except subprocess.TimeoutExpired:
                proc.kill()
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
