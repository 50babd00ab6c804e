"""Engine server: owns the GPU(s); serves embed / summarize / answer / index RPCs to the agents.

Micro-batching: every method has a queue; while the GPU executes one batch, newly arriving
requests accumulate and are run together as the next batch (one encoder launch for all queued
embeddings, one ``Generator.generate`` for all queued answers/summaries). This is the cross-request
batching the reference cannot do (it issues one OpenAI call per request).

Multi-GPU (``torchrun --nproc-per-node N``): rank 0 serves RPCs and drives the group; ranks 1..N-1
run ``follower_loop``. A command is broadcast as a small object over a gloo group; bulk work is
split data-parallel (each rank embeds / generates a slice, results gathered to rank 0); the vector
index is sharded (documents routed to rank = hash(doc_id) % N, inserts stay local to the owner's
HBM, searches fan out with the query matrix broadcast over RCCL and top-k merged on rank 0).
"""
from __future__ import annotations

import asyncio
import concurrent.futures as cf
import hashlib
import time
import traceback

import numpy as np
import torch

from ..text.preprocess import extract_summary
from ..utils import faults, metrics
from .observe import StepProfiler, Watchdog, device_memory
from .rpc import pack, parse_url, read_frame


def owner_of(doc_id: str, world: int) -> int:
    return int.from_bytes(hashlib.blake2b(doc_id.encode(), digest_size=8).digest(), "little") % max(1, world)


class EngineGroup:
    """Executes engine commands on one rank or on all ranks of a torch.distributed group."""

    def __init__(self, engine, rank: int = 0, world: int = 1, ctrl_group=None, data_group=None, shard_log=None):
        self.engine, self.rank, self.world = engine, rank, world
        self.ctrl_group, self.data_group = ctrl_group, data_group
        # durable shard (index/wal.py): every mutation of this rank's rows is logged before it is
        # applied; None = HBM only (tests, benchmarks)
        self.shard_log = shard_log

    def _put(self, doc_id, keys, vecs):
        """Replace ``doc_id``'s rows in this rank's shard (logged first when durable)."""
        idx = self.engine.index
        if self.shard_log is not None:
            self.shard_log.put(idx, doc_id, keys, vecs)
        else:
            idx.remove_doc(doc_id)
            idx.add(doc_id, keys, vecs)

    def _upsert(self, doc_id, keys, vecs):
        """Per-chunk upsert of ``doc_id``'s rows (index_add = the reference's SaveEmbeddings,
        ``ON CONFLICT (chunk_id)``, postgres.go:197): rows of other chunks of the document stay."""
        idx = self.engine.index
        if self.shard_log is not None:
            self.shard_log.upsert(idx, doc_id, keys, vecs)
        else:
            from ..index.wal import validate
            validate(idx, keys, vecs)
            idx.remove_keys(doc_id, keys)
            idx.add(doc_id, keys, vecs)

    # ---------------------------------------------------------------- collectives (control plane)
    def _bcast(self, obj):
        if self.world == 1:
            return obj
        import torch.distributed as dist
        lst = [obj]
        dist.broadcast_object_list(lst, src=0, group=self.ctrl_group)
        return lst[0]

    def _gather(self, obj):
        """Every rank's ``obj`` (msgpack-encoded) gathered as tensors over the data group (RCCL on GPU
        ranks): answers, summaries, stats. Embeddings and search results use typed tensor gathers."""
        if self.world == 1:
            return [obj]
        from ..parallel.dist import all_gather_bytes
        from .rpc import dumps, loads
        t0 = time.perf_counter()
        parts = all_gather_bytes(dumps(obj), self.engine.device, self.data_group)
        metrics.ENGINE_COLLECTIVE.labels("all_gather_bytes").inc(time.perf_counter() - t0)
        return [loads(p) for p in parts]

    def run(self, cmd: str, args: dict):
        """Rank 0: broadcast the command, execute collectively, return rank 0's result."""
        if self.world > 1:
            self._bcast((cmd, args))
        return self.execute(cmd, args)

    def follower_loop(self):
        while True:
            cmd, args = self._bcast(None)
            if cmd == "shutdown":
                return
            try:
                self.execute(cmd, args)
            except Exception:  # noqa: BLE001 - keep the group alive; rank 0 reports errors
                traceback.print_exc()

    # ---------------------------------------------------------------- commands
    def _slice(self, n: int):
        per = (n + self.world - 1) // self.world
        a = min(n, self.rank * per)
        return a, min(n, a + per)

    def execute(self, cmd: str, a: dict):
        e = self.engine
        if cmd == "embed":
            texts = a["texts"]
            lo, hi = self._slice(len(texts))
            faults.maybe_fail("engine.embed")
            v = e.embed(texts[lo:hi], a.get("preprocess", True), out_dtype=torch.float32)
            if self.world > 1:  # the slices as one tensor all-gather (RCCL on GPU ranks)
                from ..parallel.dist import all_gather_padded_rows
                t0 = time.perf_counter()
                v = all_gather_padded_rows(v, len(texts), self.data_group)
                metrics.ENGINE_COLLECTIVE.labels("embed_all_gather").inc(time.perf_counter() - t0)
            return v.cpu().numpy()
        if cmd in ("answer", "summarize"):
            items = a["items"]
            # tensor-parallel decoder: every rank runs every generation on its weight shard
            lo, hi = (0, len(items)) if getattr(self, "tensor_parallel", False) else self._slice(len(items))
            faults.maybe_fail("engine.generate")
            mine = items[lo:hi]
            if cmd == "summarize":
                res = e.summarize_many(mine) if mine else []
            else:
                batch = [self._answer_item(it) for it in mine]
                res = e.answer_many(batch) if batch else []
            if getattr(self, "tensor_parallel", False):
                return res
            out = []
            for r in self._gather(res):
                out.extend(r)
            return out
        if cmd == "cb_tick":
            # continuous batching: TP ranks all run every sequence (identical schedulers); DP
            # ranks take the new items round-robin by tag and run their own schedulers
            tp = getattr(self, "tensor_parallel", False)
            mine = [(t, it if "ids" in it else self._answer_item(it)) for t, it in a["items"]
                    if tp or t % self.world == self.rank]
            if mine:
                faults.maybe_fail("engine.generate")
            done, busy = e.cb_tick(mine, a.get("steps"))
            if tp or self.world == 1:
                return done, busy
            parts = self._gather((done, busy))
            return [d for p in parts for d in p[0]], any(p[1] for p in parts)
        if cmd == "index_add":
            if owner_of(a["doc_id"], self.world) == self.rank:
                self._upsert(a["doc_id"], np.asarray(a["keys"], dtype=np.int64),
                             torch.from_numpy(np.ascontiguousarray(a["vecs"], dtype=np.float32)))
            return True
        if cmd == "embed_index":
            # ingest without a vector round trip: the owner rank of each document
            # embeds its chunks and writes the unit-norm rows straight into its HBM shard; only the
            # row counts travel back
            mine = [it for it in a["items"] if owner_of(it[0], self.world) == self.rank]
            counts = {}
            if mine:
                faults.maybe_fail("engine.embed")
                texts = [t for _, _, ts in mine for t in ts]
                v = e.embed(texts, True)
                o = 0
                for doc_id, keys, ts in mine:
                    self._put(doc_id, np.asarray(keys, dtype=np.int64), v[o:o + len(ts)])
                    counts[doc_id] = len(ts)
                    o += len(ts)
            n = torch.tensor([counts.get(it[0], 0) for it in a["items"]], dtype=torch.int64)
            if self.world > 1:  # each document has one owner: the sum is its row count
                import torch.distributed as dist
                dev = e.device if dist.get_backend(self.data_group) != "gloo" else torch.device("cpu")
                n = n.to(dev)
                dist.all_reduce(n, group=self.data_group)
            return [int(x) for x in n.cpu().tolist()]
        if cmd == "index_remove":
            if self.shard_log is not None:
                n = self.shard_log.remove(e.index, a["doc_id"])
            else:
                n = e.index.remove_doc(a["doc_id"])
            return sum(self._gather(n))
        if cmd == "index_docs":
            rows = {d: en.rows for d, en in e.index.docs.items() if en.rows}
            merged = {}
            for part in self._gather(rows):
                for d, n in part.items():
                    merged[d] = merged.get(d, 0) + n
            return merged
        if cmd == "checkpoint":
            if self.shard_log is not None:
                self.shard_log.checkpoint(e.index)
            return sum(self._gather(len(e.index)))
        if cmd == "search":
            return self._search(a)
        if cmd == "stats":
            return self._gather(e.describe())
        if cmd == "snapshot":
            from ..index.snapshot import save_index
            save_index(e.index, f"{a['path']}.shard{self.rank}")
            return True
        if cmd == "restore":
            from ..index.snapshot import load_index
            load_index(e.index, f"{a['path']}.shard{self.rank}")
            return len(e.index)
        if cmd == "ping":
            return self._gather(self.rank)
        raise ValueError(f"unknown engine command {cmd!r}")

    def _answer_item(self, it):
        e = self.engine
        if it.get("chunks") is not None:
            ids = [(c["tokens"].tolist() if c.get("tokens") is not None else e._ids(c["text"]))
                   for c in it["chunks"]]
        else:
            ids = [e._ids(it.get("context", ""))] if it.get("context") else []
        return it["question"], ids, it.get("quality", 0.0)

    def _search(self, a):
        e = self.engine
        k, thr, filters = int(a["k"]), float(a["min_sim"]), a.get("filters")
        if self.world == 1:
            q = torch.from_numpy(np.ascontiguousarray(a["vecs"], dtype=np.float32))
            s, rows = e.index.search(q, k, thr, filters)
            ids = e.index.gather_ids(rows)
            return s.cpu().numpy(), ids.cpu().numpy()
        import torch.distributed as dist
        dev = e.device
        Q = self._bcast(a["vecs"].shape[0] if self.rank == 0 else None)
        d = e.dim
        q = (torch.from_numpy(np.ascontiguousarray(a["vecs"], dtype=np.float32)).to(dev) if self.rank == 0
             else torch.empty((Q, d), dtype=torch.float32, device=dev))
        dist.broadcast(q, src=0, group=self.data_group)                     # C2 (broadcast form)
        s, rows = e.index.search(q, k, thr, filters)
        gid = e.index.gather_ids(rows)
        # C1: scores (fp32 bits) and ids packed into ONE int64 buffer -> one all-gather per search
        from ..parallel.dist import all_gather_rows, pack_scores_ids, unpack_scores_ids
        t1 = time.perf_counter()
        P = all_gather_rows(pack_scores_ids(s, gid), self.data_group)
        metrics.ENGINE_COLLECTIVE.labels("search_all_gather").inc(time.perf_counter() - t1)
        S, G = unpack_scores_ids(P)
        flatS = S.view(self.world, Q, k).permute(1, 0, 2).reshape(Q, -1)
        flatG = G.view(self.world, Q, k).permute(1, 0, 2).reshape(Q, -1)
        flatS = torch.where(flatG >= 0, flatS, torch.full_like(flatS, float("-inf")))
        ms, mi = torch.sort(flatS, dim=1, descending=True, stable=True)
        ms, mi = ms[:, :k], mi[:, :k]
        mid = torch.where(torch.isfinite(ms), flatG.gather(1, mi), torch.full_like(mi, -1))
        return ms.cpu().numpy(), mid.cpu().numpy()


class EngineServer:
    """asyncio RPC front end with per-method micro-batch queues."""

    BATCHED = ("embed", "answer", "summarize", "embed_index")

    def __init__(self, group: EngineGroup, log, max_batch_items: int = 256, step_timeout_s: float = 300.0,
                 hard_timeout_s: float = 0.0, liveness_s: float = 30.0, profiler: StepProfiler | None = None,
                 continuous: bool = False, cb_steps: int = 1, checkpoint_s: float = 0.0,
                 cb_window_s: float = 0.02):
        self.group, self.log = group, log
        self.checkpoint_s = checkpoint_s  # periodic shard snapshots when the shard is durable (0 = off)
        self.gpu = cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="gpu")
        self.queues: dict[str, asyncio.Queue] = {}
        self.max_batch_items = max_batch_items
        self.stats = {m: {"batches": 0, "items": 0, "busy_s": 0.0} for m in self.BATCHED}
        self.exec_stats: dict[str, list] = {}
        self.server = None
        self.watchdog = Watchdog(step_timeout_s, hard_timeout_s, log)
        self.profiler = profiler or StepProfiler(rank=group.rank)
        self.liveness_s = liveness_s
        self.live_ranks = group.world
        self._busy = 0
        self._tok = {"prefill": 0, "decode": 0}
        # continuous batching of answers (a decode tick loop instead of whole-batch waves)
        self.continuous = continuous and getattr(group.engine, "gen", None) is not None
        self.cb_steps = cb_steps
        self.cb_window_s = cb_window_s
        self._cb_new: list = []
        self._cb_futs: dict = {}
        self._cb_tag = 0
        self._cb_wake = asyncio.Event()
        self._search_q: list = []
        self._search_wake = asyncio.Event()
        # CPU-side work of a request (prompt tokenization) stays off the GPU thread
        self.cpu = cf.ThreadPoolExecutor(max_workers=2, thread_name_prefix="engine-cpu")

    def _run_step(self, cmd, args):
        """Executed on the GPU thread: watchdog + optional torch.profiler + step metrics."""
        self.watchdog.begin(cmd)
        t0 = time.perf_counter()
        try:
            return self.profiler.run(cmd, self.group.run, cmd, args)
        finally:
            dt = time.perf_counter() - t0
            metrics.ENGINE_STEP.labels(cmd).observe(dt)
            ex = self.exec_stats.setdefault(cmd, [0, 0.0])  # time ON the GPU thread (no queueing)
            ex[0] += 1
            ex[1] += dt
            self.watchdog.end()
            self._account(cmd)

    def _account(self, cmd):
        e = self.group.engine
        if cmd in ("answer", "summarize") and getattr(e, "gen", None) is not None:
            st = e.gen.stats
            for ph, key in (("prefill", "prefill_tokens"), ("decode", "decode_tokens")):
                v = int(st.get(key, 0))
                if v > self._tok[ph]:
                    metrics.ENGINE_TOKENS.labels(ph).inc(v - self._tok[ph])
                    self._tok[ph] = v
        elif cmd in ("index_add", "index_remove", "restore", "stats"):
            metrics.ENGINE_INDEX_ROWS.labels(str(self.group.rank)).set(len(e.index))
            for k, v in device_memory(getattr(e, "device", None)).items():
                metrics.ENGINE_HBM.labels(str(self.group.rank), k).set(v)

    async def _gpu(self, cmd, args):
        if not self.watchdog.healthy and cmd not in ("stats", "ping"):
            raise RuntimeError(f"engine unhealthy: step {self.watchdog.stuck!r} exceeded the watchdog timeout")
        loop = asyncio.get_running_loop()
        self._busy += 1
        try:
            return await loop.run_in_executor(self.gpu, self._run_step, cmd, args)
        finally:
            self._busy -= 1

    async def _cb_submit(self, items):
        futs = []
        loop = asyncio.get_running_loop()
        for it in items:
            self._cb_tag += 1
            f = loop.create_future()
            self._cb_futs[self._cb_tag] = f
            self._cb_new.append((self._cb_tag, it))
            futs.append(f)
        self._cb_wake.set()
        return await asyncio.gather(*futs)

    async def _cb_summarize(self, texts):
        """Summaries through the continuous scheduler (map windows, then reduce prompts for texts
        longer than the context): a document arriving while others are being summarized or answers
        are decoding joins the running batch at the next tick instead of waiting for it to drain.
        Tokenization runs on a CPU thread, not on the GPU thread."""
        e = self.group.engine
        loop = asyncio.get_running_loop()
        windows, owner = await loop.run_in_executor(self.cpu, e.summary_windows, texts)
        res = await self._cb_submit([{"ids": w, "max_new": e.summary_max_new} for w in windows])
        partial, final = {}, {}
        for (i, is_part), (txt, _) in zip(owner, res):
            if is_part:
                partial.setdefault(i, []).append(txt)
            else:
                final[i] = txt
        if partial:
            red = await loop.run_in_executor(self.cpu, e.summary_reduce_prompts, partial)
            rres = await self._cb_submit([{"ids": p, "max_new": e.summary_max_new} for _, p in red])
            for (i, _), (txt, _) in zip(red, rres):
                final[i] = txt
        metrics.ENGINE_ITEMS.labels("summarize").inc(len(texts))
        return [extract_summary(final[i]) for i in range(len(texts))]

    async def _search_enqueue(self, args):
        fut = asyncio.get_running_loop().create_future()
        self._search_q.append((args, fut))
        self._search_wake.set()
        return await fut

    async def _search_loop(self):
        """Search micro-batching: the queries that queued while the GPU thread was busy run as ONE
        index scan per (k, min_sim) group, with per-query document filters (the index takes a
        filter list per query row)."""
        while True:
            if not self._search_q:
                self._search_wake.clear()
                await self._search_wake.wait()
            reqs, self._search_q = self._search_q, []
            groups: dict = {}
            for a, f in reqs:
                groups.setdefault((int(a["k"]), float(a["min_sim"]), a.get("filters") is None), []).append((a, f))
            for (k, thr, nof), g in groups.items():
                t0 = time.perf_counter()
                try:  # a malformed request fails its group, never the loop (later searches would hang)
                    vecs = [np.asarray(a["vecs"], dtype=np.float32).reshape(-1, self.group.engine.dim)
                            for a, _ in g]
                    filters = None
                    if not nof:
                        filters = [flt for (a, _), v in zip(g, vecs) for flt in (a["filters"] * v.shape[0]
                                                                                 if len(a["filters"]) == 1
                                                                                 else a["filters"])]
                        if len(filters) != sum(v.shape[0] for v in vecs):
                            raise ValueError("search: one document filter per query row (or one for all rows)")
                    s, ids = await self._gpu("search", {"vecs": np.concatenate(vecs), "k": k, "min_sim": thr,
                                                        "filters": filters})
                except Exception as e:  # noqa: BLE001
                    for _, f in g:
                        if not f.done():
                            f.set_exception(e)
                    continue
                st = self.stats.setdefault("search", {"batches": 0, "items": 0, "busy_s": 0.0})
                st["batches"] += 1
                st["items"] += len(g)
                st["busy_s"] += time.perf_counter() - t0
                metrics.ENGINE_BATCH_SIZE.labels("search").observe(len(g))
                o = 0
                for (_, f), v in zip(g, vecs):
                    if not f.done():
                        f.set_result((s[o:o + v.shape[0]], ids[o:o + v.shape[0]]))
                    o += v.shape[0]

    async def _cb_loop(self):
        """Tick the decode scheduler while it has work; new answers join at the next tick."""
        busy = False
        while True:
            if not busy and not self._cb_new:
                self._cb_wake.clear()
                await self._cb_wake.wait()
                if self.cb_window_s > 0:
                    # idle -> busy: let the rest of a burst arrive so it is admitted (prefilled) in
                    # one tick and decodes in lockstep, instead of the first request's tick delaying
                    # everyone else's start by a whole tick
                    await asyncio.sleep(self.cb_window_s)
            new, self._cb_new = self._cb_new, []
            t0 = time.perf_counter()
            try:
                done, busy = await self._gpu("cb_tick", {"items": new, "steps": self.cb_steps})
            except Exception as e:  # noqa: BLE001 - fail the requests of this tick, keep serving
                for tag, _ in new:
                    f = self._cb_futs.pop(tag, None)
                    if f is not None and not f.done():
                        f.set_exception(e)
                busy = False
                continue
            st = self.stats.setdefault("answer_cb", {"ticks": 0, "items": 0, "busy_s": 0.0})
            st["ticks"] += 1
            st["items"] += len(done)
            st["busy_s"] += time.perf_counter() - t0
            if new:
                metrics.ENGINE_BATCH_SIZE.labels("answer_cb_admit").observe(len(new))
            for tag, ans, conf in done:
                f = self._cb_futs.pop(tag, None)
                if f is not None and not f.done():
                    f.set_result((ans, conf))
            metrics.ENGINE_ITEMS.labels("answer").inc(len(done))

    async def _checkpoint_loop(self):
        """Periodic shard snapshot + log rotation (bounds replay time after a crash)."""
        while True:
            await asyncio.sleep(self.checkpoint_s)
            if self.group.shard_log.stats["rows_since_ckpt"] == 0:
                continue
            try:
                await self._gpu("checkpoint", {})
            except Exception as e:  # noqa: BLE001
                self.log.error("index checkpoint failed", "err", repr(e))

    async def _liveness_loop(self):
        """C7: periodic rank-liveness all-reduce while idle (a dead follower hangs it -> watchdog)."""
        while True:
            await asyncio.sleep(self.liveness_s)
            if self._busy or self.group.world == 1:
                continue
            try:
                ranks = await self._gpu("ping", {})
                self.live_ranks = len(ranks)
                metrics.ENGINE_LIVE_RANKS.set(self.live_ranks)
            except Exception as e:  # noqa: BLE001
                self.log.error("engine liveness check failed", "err", repr(e))

    async def _batcher(self, method: str):
        q = self.queues[method]
        while True:
            first = await q.get()
            reqs = [first]
            n = len(first[0])
            while not q.empty() and n < self.max_batch_items:
                r = q.get_nowait()
                reqs.append(r)
                n += len(r[0])
            items = [x for r in reqs for x in r[0]]
            t0 = time.perf_counter()
            try:
                if method == "embed":
                    pre = reqs[0][2]
                    res = await self._gpu("embed", {"texts": items, "preprocess": pre})
                else:
                    res = await self._gpu(method, {"items": items})
                st = self.stats[method]
                st["batches"] += 1
                st["items"] += len(items)
                st["busy_s"] += time.perf_counter() - t0
                metrics.ENGINE_BATCHES.labels(method).inc()
                metrics.ENGINE_ITEMS.labels(method).inc(len(items))
                metrics.ENGINE_BATCH_SIZE.labels(method).observe(len(items))
                o = 0
                for its, fut, _ in reqs:
                    if not fut.done():
                        fut.set_result(res[o:o + len(its)])
                    o += len(its)
            except Exception as e:  # noqa: BLE001
                for _, fut, _ in reqs:
                    if not fut.done():
                        fut.set_exception(e)

    async def _enqueue(self, method, items, extra=None):
        fut = asyncio.get_running_loop().create_future()
        await self.queues[method].put((items, fut, extra))
        return await fut

    async def dispatch(self, method: str, args: dict):
        if method == "embed":
            # batches of the same preprocess flag only
            key = "embed" if args.get("preprocess", True) else "embed_raw"
            vecs = await self._enqueue(key, list(args["texts"]), args.get("preprocess", True))
            return {"vecs": np.asarray(vecs, dtype=np.float32)}
        if method == "summarize":
            if self.continuous:
                res = await self._cb_summarize(list(args["texts"]))
            else:
                res = await self._enqueue("summarize", list(args["texts"]))
            return {"results": [[s, list(kp)] for s, kp in res]}
        if method == "answer":
            if self.continuous:
                res = await self._cb_submit(list(args["items"]))
            else:
                res = await self._enqueue("answer", list(args["items"]))
            return {"results": [[a, float(c)] for a, c in res]}
        if method == "search":
            s, ids = await self._search_enqueue(args)
            return {"scores": s, "keys": ids}
        if method == "embed_index":
            res = await self._enqueue("embed_index", [(str(args["doc_id"]), np.asarray(args["keys"], dtype=np.int64),
                                                       list(args["texts"]))])
            return {"rows": int(res[0]), "dim": int(self.group.engine.dim)}
        if method in ("index_add", "index_remove", "snapshot", "restore", "ping", "index_docs", "checkpoint"):
            return await self._gpu(method, args)
        if method == "stats":
            st = await self._gpu("stats", {})
            return {"ranks": st, "batching": self.stats,
                    "exec": {k: {"n": n, "s": round(t, 4)} for k, (n, t) in self.exec_stats.items()}}
        if method == "health":
            return dict(self.watchdog.state(), live_ranks=self.live_ranks, world=self.group.world)
        raise ValueError(f"unknown method {method!r}")

    async def _client(self, reader, writer):
        lock = asyncio.Lock()

        async def handle(msg):
            rid = msg.get("id")
            try:
                res = await self.dispatch(msg.get("method"), msg.get("args") or {})
                out = {"id": rid, "result": res}
            except Exception as e:  # noqa: BLE001
                self.log.error("engine rpc failed", "method", msg.get("method"), "err", repr(e),
                               "trace_id", msg.get("trace", ""))
                out = {"id": rid, "error": f"{type(e).__name__}: {e}"}
            async with lock:
                writer.write(pack(out))
                await writer.drain()

        try:
            while True:
                msg = await read_frame(reader)
                asyncio.ensure_future(handle(msg))
        except (asyncio.IncompleteReadError, ConnectionError):
            pass
        finally:
            writer.close()

    async def start(self, url: str):
        for m in ("embed", "embed_raw", "answer", "summarize", "embed_index"):
            self.queues[m] = asyncio.Queue()
        for m in ("embed", "answer", "summarize", "embed_index"):
            asyncio.ensure_future(self._batcher(m))
        if self.checkpoint_s > 0 and self.group.shard_log is not None:
            self.checkpoint_task = asyncio.ensure_future(self._checkpoint_loop())
        self.queues_raw_task = asyncio.ensure_future(self._batcher_raw())
        self.watchdog.start()
        if self.continuous:
            self.cb_task = asyncio.ensure_future(self._cb_loop())
        self.search_task = asyncio.ensure_future(self._search_loop())
        if self.liveness_s > 0 and self.group.world > 1:
            self.liveness_task = asyncio.ensure_future(self._liveness_loop())
        kind, addr = parse_url(url)
        if kind == "unix":
            self.server = await asyncio.start_unix_server(self._client, path=addr)
        else:
            self.server = await asyncio.start_server(self._client, addr[0], addr[1])
        return self.server

    async def _batcher_raw(self):
        # raw (already preprocessed) embeddings share the embed batcher logic
        self.stats.setdefault("embed_raw", {"batches": 0, "items": 0, "busy_s": 0.0})
        self.BATCHED = self.BATCHED + ("embed_raw",)
        q = self.queues["embed_raw"]
        while True:
            first = await q.get()
            reqs = [first]
            while not q.empty():
                reqs.append(q.get_nowait())
            items = [x for r in reqs for x in r[0]]
            try:
                res = await self._gpu("embed", {"texts": items, "preprocess": False})
                o = 0
                for its, fut, _ in reqs:
                    if not fut.done():
                        fut.set_result(res[o:o + len(its)])
                    o += len(its)
            except Exception as e:  # noqa: BLE001
                for _, fut, _ in reqs:
                    if not fut.done():
                        fut.set_exception(e)
