"""Engine server: owns the GPU(s); serves embed / summarize / answer / search / index RPCs.

Micro-batching: every method has a queue; while the GPU executes one batch, newly arriving
requests accumulate and are run together as the next batch (one encoder launch for all queued
embeddings; answers and summaries join a continuous decode scheduler). This is the cross-request
batching the reference cannot do (it issues one OpenAI call per request).

Three lanes per replica, each a thread with its own HIP stream, so latency-critical work never
queues behind a decode tick or an admission prefill:
  * the GPU thread: the continuous scheduler's ticks, summaries, ingest embeds, index mutations;
  * the fast lane: query-sized embeds (the question of ``embed`` / ``embed_search``), on a
    high-priority stream with its own kernel workspace;
  * the search plane (parallel/search_plane.py): a scan worker with its own stream serving this
    rank's shard to every replica; searches are routed to the shards that own their documents.

Multi-GPU (``torchrun --nproc-per-node N``, TP_SIZE = t): N / t independent replicas, replica r =
ranks [r t, (r + 1) t) served by its leader on port base + r (``EngineGroup``); the vector index is
sharded over all N ranks (documents routed to rank = hash(doc_id) % N).
"""
from __future__ import annotations

import asyncio
import concurrent.futures as cf
import time
import traceback

import numpy as np
import torch

from ..text.preprocess import extract_summary
from ..utils import faults, metrics, timeline
from .observe import StepProfiler, Watchdog, device_memory
from ..parallel.search_plane import owner_of  # noqa: F401 - re-exported (clients route by it)
from .rpc import pack, parse_url, read_frame


class EngineGroup:
    """The ranks of ONE engine replica (a tensor-parallel group of ``tp_size`` ranks; one rank when
    the decoder is not sharded) executing engine commands.

    Replicas are independent, like the reference's agent replicas (docker-compose.yml:84-85,105-106):
    each leader serves its own RPC endpoint with its own micro-batchers and continuous scheduler, and
    no command crosses replicas — decode ticks, admissions, embeds and ingest never wait for another
    replica. Within a replica the leader broadcasts each command to its TP followers over a gloo
    group (the TP ranks step one decoder together). The only cross-replica traffic is the sharded
    search (parallel/search_plane.py: point-to-point requests to the shards that own a search's
    documents, served by a scan thread and stream of their own on every rank) and ingest routing:
    a document's vectors live on rank ``owner_of(doc_id, world)``, and clients send its index
    mutations to that rank's replica (``EngineCluster.call``). Index mutations order themselves
    against concurrent scans on the device (index/flat.py ``writing`` / ``reading``)."""

    def __init__(self, engine, rank: int = 0, world: int = 1, ctrl_group=None, data_group=None, shard_log=None,
                 tp_size: int = 1, plane=None):
        self.engine, self.rank, self.world = engine, rank, world
        self.ctrl_group, self.data_group = ctrl_group, data_group
        self.tp_size = max(1, int(tp_size))
        if world % self.tp_size:
            raise ValueError(f"TP size {self.tp_size} must divide the world size {world}")
        self.replica, self.replicas = rank // self.tp_size, world // self.tp_size
        self.leader = self.replica * self.tp_size
        self.is_leader = rank == self.leader
        self.plane = plane
        # durable shard (index/wal.py): every mutation of this rank's rows is logged before it is
        # applied; None = HBM only (tests, benchmarks)
        self.shard_log = shard_log
        self.ckpt_at = time.monotonic()
        self.tick_stop = None  # set by the server: "requests are waiting for admission"

    @property
    def tensor_parallel(self) -> bool:
        return self.tp_size > 1

    def _put(self, doc_id, keys, vecs):
        """Replace ``doc_id``'s rows in this rank's shard (logged first when durable)."""
        idx = self.engine.index
        if self.shard_log is not None:
            self.shard_log.put(idx, doc_id, keys, vecs)
        else:
            with idx.writing():  # one committed mutation: a scan sees the old rows or the new ones
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
            with idx.writing():
                idx.remove_keys(doc_id, keys)
                idx.add(doc_id, keys, vecs)

    def owner(self, doc_id: str) -> int:
        return owner_of(doc_id, self.world)

    def _check_routed(self, doc_id: str) -> int:
        o = self.owner(doc_id)
        if o // self.tp_size != self.replica:
            raise ValueError(f"document {doc_id} lives on rank {o} (replica {o // self.tp_size}); "
                             f"this is replica {self.replica}: route index calls by owner (EngineCluster)")
        return o

    # ---------------------------------------------------------------- replica control plane
    def _bcast(self, obj):
        if self.tp_size == 1:
            return obj
        import torch.distributed as dist
        lst = [obj]
        dist.broadcast_object_list(lst, src=self.leader, group=self.ctrl_group)
        return lst[0]

    def _gather(self, obj):
        """Every replica rank's ``obj`` (msgpack-encoded) gathered as tensors over the replica's data
        group (RCCL on GPU ranks): stats, row counts."""
        if self.tp_size == 1:
            return [obj]
        from ..parallel.dist import all_gather_bytes
        from .rpc import dumps, loads
        t0 = time.perf_counter()
        parts = all_gather_bytes(dumps(obj), self.engine.device, self.data_group)
        metrics.ENGINE_COLLECTIVE.labels("all_gather_bytes").inc(time.perf_counter() - t0)
        return [loads(p) for p in parts]

    LOCAL = ("embed",)  # leader-only commands (the encoder is not sharded)

    def run(self, cmd: str, args: dict):
        """Leader: broadcast the command to the replica's TP followers (when it needs them), execute."""
        if self.tp_size > 1 and cmd not in self.LOCAL:
            self._bcast((cmd, args))
        return self.execute(cmd, args)

    def follower_loop(self, on_idle=None):
        while True:
            cmd, args = self._bcast(None)
            if cmd == "shutdown":
                return
            try:
                self.execute(cmd, args)
            except Exception:  # noqa: BLE001 - keep the replica alive; the leader reports errors
                traceback.print_exc()

    # ---------------------------------------------------------------- commands
    def execute(self, cmd: str, a: dict):
        e = self.engine
        if cmd == "embed":
            faults.maybe_fail("engine.embed")
            return e.embed(a["texts"], a.get("preprocess", True), out_dtype=torch.float32).cpu().numpy()
        if cmd in ("answer", "summarize"):
            # every TP rank of the replica runs every generation on its weight shard; the leader's
            # result is the replica's (identical on all TP ranks)
            items = a["items"]
            faults.maybe_fail("engine.generate")
            if cmd == "summarize":
                return e.summarize_many(items) if items else []
            batch = [self._answer_item(it) for it in items]
            return e.answer_many(batch) if batch else []
        if cmd == "cb_tick":
            faults.maybe_delay("engine.tick")
            mine = [(t, it if "ids" in it else self._answer_item(it)) for t, it in a["items"]]
            if mine:
                faults.maybe_fail("engine.generate")
            # an early stop decided by the leader alone would desynchronise the TP ranks' decode
            # steps: only a one-rank replica stops a tick when new work arrives
            stop = self.tick_stop if self.tp_size == 1 else None
            return e.cb_tick(mine, a.get("steps"), stop)
        if cmd == "index_add":
            if self._check_routed(a["doc_id"]) == self.rank:
                self._upsert(a["doc_id"], np.asarray(a["keys"], dtype=np.int64),
                             torch.from_numpy(np.ascontiguousarray(a["vecs"], dtype=np.float32)))
            return True
        if cmd == "embed_index":
            # ingest without a vector round trip: the owner rank of each document
            # embeds its chunks and writes the unit-norm rows straight into its HBM shard; only the
            # row counts travel back (routing was checked per request in EngineServer.dispatch, so a
            # misrouted document fails alone, not the co-batched ingests of other clients)
            mine = [it for it in a["items"] if self.owner(it[0]) == self.rank]
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
            merged = {}
            for part in self._gather(counts):
                merged.update(part)
            return [int(merged.get(it[0], 0)) for it in a["items"]]
        if cmd == "index_remove":
            n = 0
            if self._check_routed(a["doc_id"]) == self.rank:
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
            # each rank checkpoints its own shard when its log has anything since the last one
            if self.shard_log is not None and (a.get("force") or self.shard_log.stats["rows_since_ckpt"] > 0):
                self.shard_log.checkpoint(e.index)
                self.ckpt_at = time.monotonic()
            return sum(self._gather(len(e.index)))
        if cmd == "stats":
            d = e.describe()
            d["rank"], d["replica"] = self.rank, self.replica
            if self.plane is not None:
                d["search_plane"] = dict(self.plane.stats, **self.plane.health())
            return self._gather(d)
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


class EngineServer:
    """asyncio RPC front end with per-method micro-batch queues."""

    BATCHED = ("embed", "answer", "summarize", "embed_index")

    def __init__(self, group: EngineGroup, log, max_batch_items: int = 256, step_timeout_s: float = 300.0,
                 hard_timeout_s: float = 0.0, liveness_s: float = 30.0, profiler: StepProfiler | None = None,
                 continuous: bool = False, cb_steps: int = 1, checkpoint_s: float = 0.0,
                 cb_window_s: float = 0.003, fast_embed_max: int = 8, urls: list[str] | None = None,
                 cb_max_steps: int = 16, lanes=None, fast_yield: bool = False, admit_min: int = 16,
                 admit_wait_s: float = 0.15, admit_hold_frac: float = 0.25):
        self.group, self.log = group, log
        self.urls = urls or []  # every replica's listen URL (topology RPC), replica order
        # the fast lane: query-sized embeds on their own thread / high-priority stream / workspace
        self.fast_embed_max = fast_embed_max
        # lanes = (main, fast) streams of a CU partition (ops/streams.py serving_lanes), or None
        main_stream, fast_stream = (lanes or (None, None))[:2]
        self.fast = cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="fast-embed")
        self._fast_q: list = []
        self._fast_wake = asyncio.Event()
        self._fast_stream = fast_stream
        # fast_yield: decode ticks end after the current step while question embeds are queued or
        # running, and the next tick waits (bounded) for the lane to go idle
        self.fast_yield = fast_yield
        self._fast_running = 0
        self._fast_idle = asyncio.Event()
        self._fast_idle.set()
        self.rpc_ms: dict[str, list] = {}  # method -> [calls, total ms] (engine side)
        self.checkpoint_s = checkpoint_s  # periodic shard snapshots when the shard is durable (0 = off)
        init = (lambda: torch.cuda.set_stream(main_stream)) if main_stream is not None else None
        self.gpu = cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="gpu", initializer=init)
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
        # decode steps per scheduler tick: cb_steps while requests wait for admission, up to
        # cb_max_steps otherwise (a one-rank replica also ends a long tick as soon as one arrives)
        self.cb_steps, self.cb_max_steps = cb_steps, max(cb_steps, cb_max_steps)
        # grouped admission under load: while at least admit_hold_frac of the decode rows are busy,
        # arrivals are held until admit_min of them (or as many as there are free rows) are waiting,
        # or the oldest has waited admit_wait_s, and then prefill together. One admission per
        # arrival (a 1-prompt prefill, a tick cut short and a reap sync each) is what made a
        # 128-row batch lose to a 64-row one in the deploy stack (profiles/r5/rejected_r5.txt)
        self.admit_min, self.admit_wait_s, self.admit_hold_frac = max(1, admit_min), admit_wait_s, admit_hold_frac
        self._cb_oldest = 0.0  # arrival time of the oldest held request
        group.tick_stop = lambda: self._admit_ready() or (self.fast_yield and bool(self._fast_q or self._fast_running))
        self.cb_window_s = cb_window_s
        self._cb_new: list = []
        self._cb_futs: dict = {}
        self._cb_tag = 0
        self._cb_wake = asyncio.Event()
        if group.plane is None:  # a replica always searches through a plane (one rank: a local one)
            from ..parallel.search_plane import SearchPlane
            group.plane = SearchPlane(group.engine.index, 0, 1, device=group.engine.device).start()
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
        if not self._cb_new:
            self._cb_oldest = time.monotonic()
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
        plan = e.summary_plan(texts, e.summary_max_new)
        kind, val = await loop.run_in_executor(self.cpu, e.summary_step, plan)
        while kind == "prompts":  # map windows, then every reduce level (engine.summary_plan)
            res = await self._cb_submit([{"ids": p, "max_new": getattr(val, "max_new", e.summary_max_new)} for p in val])
            kind, val = await loop.run_in_executor(self.cpu, e.summary_step, plan, [t for t, _ in res])
        metrics.ENGINE_ITEMS.labels("summarize").inc(len(texts))
        return [extract_summary(t) for t in val]

    def _fast_embed(self, texts, preprocess: bool) -> np.ndarray:
        """Runs on the fast-lane thread: the encoder on a high-priority stream with its own kernel
        workspace, so it co-runs with the GPU thread's decode tick instead of queueing behind it."""
        e = self.group.engine
        faults.maybe_fail("engine.embed")
        if e.device.type != "cuda":
            return e.embed(texts, preprocess, out_dtype=torch.float32).cpu().numpy()
        from ..ops import kernels as K
        if self._fast_stream is None:
            torch.cuda.set_device(e.device)
            self._fast_stream = torch.cuda.Stream(device=e.device, priority=-1)
        with torch.cuda.stream(self._fast_stream), K.workspace_role("fast"):
            return e.embed(texts, preprocess, out_dtype=torch.float32).cpu().numpy()

    async def _embed_fast(self, texts, preprocess: bool):
        """Queue query-sized texts for the fast lane; the lane runs every text queued while its
        previous encoder call was in flight as ONE call (micro-batching), so under load the lane's
        throughput scales with the burst instead of one encoder pass per question."""
        fut = asyncio.get_running_loop().create_future()
        self._fast_q.append((list(texts), bool(preprocess), fut))
        self._fast_idle.clear()
        self._fast_wake.set()
        return await fut

    async def _fast_loop(self):
        loop = asyncio.get_running_loop()
        while True:
            if not self._fast_q:
                self._fast_idle.set()
                self._fast_wake.clear()
                await self._fast_wake.wait()
            pre = self._fast_q[0][1]
            take = [r for r in self._fast_q if r[1] == pre][:64]
            self._fast_q = [r for r in self._fast_q if all(r is not t for t in take)]
            texts = [t for r in take for t in r[0]]
            t0 = time.perf_counter()
            self._fast_running += 1
            try:
                v = await loop.run_in_executor(self.fast, self._fast_embed, texts, pre)
            except Exception as e:  # noqa: BLE001 - fail this batch, keep the lane serving
                for _, _, f in take:
                    if not f.done():
                        f.set_exception(e)
                continue
            finally:
                self._fast_running -= 1
            st = self.stats.setdefault("embed_fast", {"batches": 0, "items": 0, "busy_s": 0.0})
            st["batches"] += 1
            st["items"] += len(texts)
            st["busy_s"] += time.perf_counter() - t0
            metrics.ENGINE_ITEMS.labels("embed").inc(len(texts))
            metrics.ENGINE_BATCH_SIZE.labels("embed_fast").observe(len(texts))
            o = 0
            for ts, _, f in take:
                if not f.done():
                    f.set_result(v[o:o + len(ts)])
                o += len(ts)

    async def _search(self, vecs, k, min_sim, filters):
        """Sharded top-k through the search plane (its own thread + stream on every rank)."""
        t0 = time.perf_counter()
        fut = self.group.plane.submit(np.asarray(vecs, dtype=np.float32), int(k), float(min_sim), filters)
        s, ids = await asyncio.wrap_future(fut)
        st = self.stats.setdefault("search", {"batches": 0, "items": 0, "busy_s": 0.0})
        st["batches"] += 1
        st["items"] += int(np.asarray(vecs).reshape(-1, self.group.engine.dim).shape[0])
        st["busy_s"] += time.perf_counter() - t0
        return s, ids

    def _admit_ready(self) -> bool:
        """Whether the held arrivals go to the scheduler now (the grouped-admission rule above).
        Called on the event loop and, as the tick's stop callback, on the GPU thread between decode
        steps (plain reads of counters the GPU thread itself updates)."""
        n = len(self._cb_new)
        if n == 0:
            return False
        sched = getattr(self.group.engine, "_sched", None)
        if self.admit_min <= 1 or sched is None:
            return True
        active = sched.n_active
        if active < self.admit_hold_frac * sched.B:
            return True  # light load: latency first
        free = sched.B - active - len(sched.pending)
        if free <= 0:
            return False  # no row to seat them: the tick runs until rows free (steps_to_free)
        return n >= min(self.admit_min, free) or time.monotonic() - self._cb_oldest >= self.admit_wait_s

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
            if self.fast_yield and not self._fast_idle.is_set():
                try:  # question embeds first: they take ~2 ms on an uncontended GPU
                    await asyncio.wait_for(self._fast_idle.wait(), 0.02)
                except asyncio.TimeoutError:
                    pass
            # short ticks while anything waits for admission (the requests taken now, or earlier ones
            # the scheduler could not seat yet), long ticks otherwise; arrivals during a long tick
            # end it through group.tick_stop (checked between steps, at most 2 steps queued ahead)
            sched = getattr(self.group.engine, "scheduler", None)
            if self._admit_ready():
                new, self._cb_new = self._cb_new, []
                if timeline.enabled() and new:
                    timeline.mark("e_admit", q=[it.get("question") for _, it in new], n_active=getattr(sched, "n_active", 0))
            else:
                new = []
            held = bool(self._cb_new)
            waiting = bool(new) or bool(getattr(sched, "pending", None))
            if held or (waiting and sched is not None and sched.n_active >= sched.B):
                # requests wait for rows (or for their group): run until the first rows free up, or
                # until the held group is ready (tick_stop), not one step at a time
                steps = max(self.cb_steps, min(self.cb_max_steps, sched.steps_to_free()))
            else:
                steps = self.cb_steps if waiting else self.cb_max_steps
            t0 = time.perf_counter()
            try:
                done, busy = await self._gpu("cb_tick", {"items": new, "steps": steps})
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
            if timeline.enabled():
                timeline.mark("e_tick", steps=steps, admitted=len(new), done=len(done), dt=time.perf_counter() - t0,
                              n_active=getattr(sched, "n_active", 0))
            for tag, ans, conf in done:
                f = self._cb_futs.pop(tag, None)
                if f is not None and not f.done():
                    f.set_result((ans, conf))
            metrics.ENGINE_ITEMS.labels("answer").inc(len(done))

    async def _checkpoint_loop(self):
        """Periodic shard snapshot + log rotation (bounds replay time after a crash). Every rank of
        the replica checkpoints its own shard when its log has records since the last checkpoint
        (removes count), whichever rank the documents hashed to."""
        while True:
            await asyncio.sleep(self.checkpoint_s)
            try:
                await self._gpu("checkpoint", {})
            except Exception as e:  # noqa: BLE001
                self.log.error("index checkpoint failed", "err", repr(e))

    async def _liveness_loop(self):
        """C7: periodic replica-liveness gather while idle (a dead TP follower hangs it -> watchdog);
        cross-replica liveness is the search plane's round (health: ``search_plane``)."""
        while True:
            await asyncio.sleep(self.liveness_s)
            if self._busy or self.group.tp_size == 1:
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
        if method == "topology":
            g = self.group
            return {"replica": g.replica, "replicas": g.replicas, "tp": g.tp_size, "world": g.world,
                    "urls": list(self.urls), "dim": int(g.engine.dim)}
        if method == "embed":
            texts = list(args["texts"])
            pre = args.get("preprocess", True)
            if len(texts) <= self.fast_embed_max:  # the query path: the fast lane
                return {"vecs": np.asarray(await self._embed_fast(texts, pre), dtype=np.float32)}
            # batches of the same preprocess flag only
            vecs = await self._enqueue("embed" if pre else "embed_raw", texts, pre)
            return {"vecs": np.asarray(vecs, dtype=np.float32)}
        if method == "embed_search":
            tl = timeline.enabled()
            if tl:
                timeline.mark("e_es_rx", t_text=args["texts"][0] if args.get("texts") else None)
            # the query path in one call (cmd/query/main.go:87-105): embed the question on the fast
            # lane, search every shard through the plane; the vector comes back for the embedding
            # cache. texts: already preprocessed (the client checked they are non-empty).
            try:
                v = await self._embed_fast(list(args["texts"]), bool(args.get("preprocess", False)))
            except Exception as e:  # noqa: BLE001 - the client maps the tag to the reference's message
                raise RuntimeError(f"embed_search/embed: {e}") from e
            if tl:
                timeline.mark("e_es_embedded", t_text=args["texts"][0] if args.get("texts") else None)
            try:
                s, ids = await self._search(v, args["k"], args["min_sim"], args.get("filters"))
            except Exception as e:  # noqa: BLE001
                raise RuntimeError(f"embed_search/search: {e}") from e
            if tl:
                timeline.mark("e_es_tx", t_text=args["texts"][0] if args.get("texts") else None)
            return {"vecs": np.asarray(v, dtype=np.float32), "scores": s, "keys": ids}
        if method == "summarize":
            if self.continuous:
                res = await self._cb_summarize(list(args["texts"]))
            else:
                res = await self._enqueue("summarize", list(args["texts"]))
            return {"results": [[s, list(kp)] for s, kp in res]}
        if method == "answer":
            if timeline.enabled():
                for it in args["items"]:
                    timeline.mark("e_answer_rx", q=it.get("question"))
            if self.continuous:
                res = await self._cb_submit(list(args["items"]))
            else:
                res = await self._enqueue("answer", list(args["items"]))
            if timeline.enabled():
                for it in args["items"]:
                    timeline.mark("e_answer_tx", q=it.get("question"))
            return {"results": [[a, float(c)] for a, c in res]}
        if method == "search":
            s, ids = await self._search(args["vecs"], args["k"], args["min_sim"], args.get("filters"))
            return {"scores": s, "keys": ids}
        if method == "embed_index":
            self.group._check_routed(str(args["doc_id"]))  # a misrouted document fails alone
            res = await self._enqueue("embed_index", [(str(args["doc_id"]), np.asarray(args["keys"], dtype=np.int64),
                                                       list(args["texts"]))])
            return {"rows": int(res[0]), "dim": int(self.group.engine.dim)}
        if method in ("index_add", "index_remove", "snapshot", "restore", "ping", "index_docs", "checkpoint"):
            return await self._gpu(method, args)
        if method == "stats":
            st = await self._gpu("stats", {})
            return {"ranks": st, "batching": self.stats,
                    "exec": {k: {"n": n, "s": round(t, 4)} for k, (n, t) in self.exec_stats.items()},
                    "rpc_mean_ms": {k: round(t / max(1, n), 3) for k, (n, t) in self.rpc_ms.items()}}
        if method == "health":
            pl = self.group.plane
            ph = pl.health() if pl is not None else {"ok": True, "shards_down": []}
            return dict(self.watchdog.state(), live_ranks=self.live_ranks, world=self.group.world,
                        replica=self.group.replica, search_plane=bool(ph["ok"]),
                        shards_down=list(ph["shards_down"]))
        raise ValueError(f"unknown method {method!r}")

    async def _client(self, reader, writer):
        lock = asyncio.Lock()

        async def handle(msg):
            rid = msg.get("id")
            method = msg.get("method")
            t0 = time.perf_counter()
            try:
                res = await self.dispatch(method, msg.get("args") or {})
                out = {"id": rid, "result": res}
                if method in ("embed", "embed_search", "search"):
                    # engine-side latency of the query-path calls (receipt -> reply ready): with the
                    # client's stage time it splits a slow query between the engine and the RPC hop
                    r = self.rpc_ms.setdefault(method, [0, 0.0])
                    r[0] += 1
                    r[1] += (time.perf_counter() - t0) * 1000
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
        self.fast_task = asyncio.ensure_future(self._fast_loop())
        if self.liveness_s > 0 and self.group.tp_size > 1:
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
