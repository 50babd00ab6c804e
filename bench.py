"""Headline benchmark: RAG QA queries/sec (+ p50 cache-miss latency, ingest docs/min) on MI355X.

Metric / config from BASELINE.json: "QA queries/sec + p50 cache-miss latency; docs/min ingest at
1/2/4/8 MI355X" on config 2: "BGE-base embedder + Phi-3-mini QA on 1xMI355X, 100k-chunk brute-force
cosine in HBM" — here 100k chunks PER GPU (weak scaling: the index grows with N; a query's
documents are spread over all shards, so at N > 1 most searches read several ranks' shards).

One timed step = every GPU serves B cache-miss queries end to end (the reference's query path,
cmd/query/main.go:44-136, minus the cache hit): tokenize -> BGE-base encode (HIP kernels) ->
search (N = 1: the local shard through the search plane; N > 1: the lock-step RCCL sharded search,
C2 all-gather of the query rows, every shard scans them, C1 all-gather of the per-shard top-k,
device merge; ``--search plane`` keeps the point-to-point plane) -> fused cosine + doc-filter +
threshold + top-k on each shard (vecsearch.hip) -> build the Answer prompt from the top-k chunks
(pre-tokenized at ingest) -> Phi-3-mini prefill (~2.9k tokens/query) + decode MAX_NEW tokens at
T=0.2 (HIP kernels, HIP graphs) -> confidence = avg similarity x mean token probability ->
detokenize. After the timed steps at N > 1, the multi-GPU blocks (parallel/collective_bench.py)
time the fabric mechanisms into the same JSON line.

Synthetic data (no network): random-init weights of the named architectures, random unit vectors
for the 100k background chunks per GPU (their token ids drawn from the locally trained BPE vocab),
synthetic questions; each query filters on `--docs-per-query` random documents spread over all
shards. MIN_SIMILARITY is set to -1 so every query retrieves exactly top_k chunks (random weights
make the reference's 0.7 floor meaningless; -1 is the MOST work per query, never less).

Launch: python bench.py [--gpus N --steps K --warmup W]. With N > 1 and no WORLD_SIZE in the
environment, this process launches N ranks itself (python -m torch.distributed.run, one rank per GPU)
before anything touches the GPU, relays their output and exits with their status; under an external
torchrun (WORLD_SIZE set) it is one rank, and WORLD_SIZE != --gpus is an error. Every rank is an
independent replica (its own engine) and the index is sharded one shard per rank; the JSON line
reports the process-group backend and the number of ranks that joined (ranks_seen, an all-reduce of
ones).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time


def _launch_ranks(argv: list[str]) -> int | None:
    """Parent side of ``--gpus N``: None = run the bench in this process (we are a rank, or N = 1);
    otherwise the exit status of N child ranks launched here. Imports nothing GPU-related and never
    exec()s: the children are fresh processes (torch.distributed.run), this one only waits."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    a, _ = ap.parse_known_args(argv)
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != a.gpus:
            print(f"[bench] WORLD_SIZE={ws} but --gpus {a.gpus}: refusing to report a different world",
                  file=sys.stderr, flush=True)
            return 2
        return None
    if a.gpus <= 1:
        return None
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    print(f"[bench] launching {a.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


if __name__ == "__main__":
    _rc = _launch_ranks(sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc)

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from docagents_amd.engine.engine import Engine  # noqa: E402
from docagents_amd.parallel.dist import (all_reduce_max, all_reduce_sum, barrier, init_from_env,  # noqa: E402
                                         shutdown)
from docagents_amd.parallel.search_plane import SearchPlane, owner_of  # noqa: E402
from docagents_amd.parallel.sharded_index import ShardedIndex  # noqa: E402
from docagents_amd.engine.prompts import concatenate_chunks, dedup_overlap  # noqa: E402
from docagents_amd.text.chunker import Options, chunk_text  # noqa: E402
from docagents_amd.text.synthetic import TextGen  # noqa: E402

METRIC = "QA queries/sec + p50 cache-miss latency; docs/min ingest at 1/2/4/8 MI355X"
REFERENCE_CACHE_MISS_MS = 2500.0  # README.md:590 "~2-3 seconds" (midpoint); no QPS is published


def log(info, *a):
    if info.rank == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


class ChunkTokens:
    """Token ids of the synthetic background chunks (what ingest would have cached per chunk)."""

    def __init__(self, vocab_lo: int, vocab_hi: int, seed: int = 1234, pool: int = 1 << 20):
        rng = np.random.default_rng(seed)
        self.pool = rng.integers(vocab_lo, vocab_hi, size=pool, dtype=np.int32)
        self.lens = rng.integers(500, 561, size=4096)

    def get(self, cid: int) -> list[int]:
        n = int(self.lens[cid % 4096])
        o = (cid * 7919) % (len(self.pool) - n)
        return self.pool[o:o + n].tolist()


def shard_vectors(rank: int, rows: int, d: int, dev) -> torch.Tensor:
    """Rank ``rank``'s synthetic background chunks: seeded random unit vectors [rows, d] bf16
    (bench/sharded_recall.py regenerates every shard from the same seeds)."""
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    X = torch.randn((rows, d), device=dev, generator=g)
    return torch.nn.functional.normalize(X, dim=-1).to(torch.bfloat16)


def doc_names(world: int, ndocs: int) -> list[list[str]]:
    """Per rank, ``ndocs`` document names that production routing (owner_of: hash(doc) % N) places
    on that rank's shard, so the plane routes every query row to the shards that hold its documents.
    Document j of a rank owns rows [j * chunks_per_doc, (j + 1) * chunks_per_doc) of its shard."""
    names = [[] for _ in range(world)]
    i = 0
    while min(len(n) for n in names) < ndocs:
        for r in range(world):
            nm = f"d{r}-{i}"
            if len(names[r]) < ndocs and owner_of(nm, world) == r:
                names[r].append(nm)
        i += 1
    return names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=128,
                    help="cache-miss queries per GPU per step (128: the decode weights are read once per 128 "
                         "rows; the KV cache of 132 x 4096-token slots is 213 GB of the 288 GB HBM. Same box: "
                         "34.09 q/s vs 33.09 at 64, profiles/r5/batch128/)")
    ap.add_argument("--index-rows", type=int, default=100_000, help="chunks per GPU shard")
    ap.add_argument("--chunks-per-doc", type=int, default=10)
    ap.add_argument("--docs-per-query", type=int, default=8)
    ap.add_argument("--top-k", type=int, default=5)
    ap.add_argument("--max-new", type=int, default=64)
    ap.add_argument("--min-sim", type=float, default=-1.0)
    ap.add_argument("--enc", default="bge-base")
    ap.add_argument("--llm", default="phi3-mini")
    ap.add_argument("--latency-reps", type=int, default=24, help="batch-1 cache-miss queries for p50 / p90")
    ap.add_argument("--ingest-docs", type=int, default=None,
                    help="docs per GPU per ingest batch (default: one engine batch, the QA --batch)")
    ap.add_argument("--ingest-batches", type=int, default=3,
                    help="timed ingest batches (distinct documents); docs/min is their median")
    ap.add_argument("--ingest-words", type=int, default=2000)
    ap.add_argument("--pdf-ingest", action="store_true",
                    help="ingest synthetic PDFs (gateway PDF extraction in the timed path; BASELINE config 3)")
    ap.add_argument("--tp", type=int, default=1,
                    help="tensor-parallel degree of the QA decoder (BASELINE config 5: Llama-3-70B TP=8); "
                         "the world splits into world/tp data-parallel groups, the index stays world-way sharded")
    ap.add_argument("--index-kind", default="flat", choices=["flat", "ivfflat"])
    ap.add_argument("--ivf-lists", type=int, default=1024)
    ap.add_argument("--ivf-probes", type=int, default=16)
    ap.add_argument("--enc-dtype", default="bf16", choices=["bf16", "fp16", "fp8"],
                    help="encoder dtype: fp16 = the whole encoder on fp16 MFMA (BASELINE config 4), "
                         "fp8 = OCP e4m3 MFMA GEMMs (BASELINE config 5)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--breakdown", type=int, default=1, help="1: one extra untimed QA step with per-phase timing")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--overlap", type=int, default=0,
                    help="1: QA waves pipelined — the decode of step i on half of the CUs beside the prefill "
                         "of step i + 1 (Engine.answer_overlapped); 0 (default): one wave after the other. "
                         "Same box: 30.2 vs 32.3 q/s (profiles/r3/overlap/): the co-run loses to the clock "
                         "and HBM interference what the partition gains")
    ap.add_argument("--overlap-frac", type=float, default=0.5, help="decode lane's share of the CUs")
    ap.add_argument("--cpu-rehearsal", action="store_true",
                    help="tests only: run on CPU ranks (gloo) with tiny configs to pin the JSON schema; "
                         "the numbers are not a benchmark")
    ap.add_argument("--search", default="auto", choices=["auto", "rccl", "plane"],
                    help="QA-step search transport at N > 1: rccl = the lock-step sharded search (C2 all-gather "
                         "of the query rows, every shard scans them, C1 all-gather of the per-shard top-k over "
                         "RCCL / xGMI, device merge); plane = the serving search plane (owner-routed, host TCP); "
                         "auto = rccl without TP, plane with TP (TP ranks share their queries)")
    ap.add_argument("--multi-iters", type=int, default=24,
                    help="N > 1: timed sharded searches of the rccl_search block (C1 + C2 over RCCL)")
    ap.add_argument("--serving-requests", type=int, default=256,
                    help="N > 1: single-question searches per rank of the serving_search block (the owner-routed "
                         "plane vs SEARCH_TRANSPORT=rccl lock-step rounds); 0 skips it")
    ap.add_argument("--ingest-latency-reps", type=int, default=10,
                    help="single-document ingest latency reps (upload -> summary readable, engine level)")
    ap.add_argument("--tp70b", default="auto", choices=["auto", "on", "off"],
                    help="N > 1: the tp_decode_70b block (BASELINE config 5's QA model, Llama-3-70B, built "
                         "directly as TP = N shards: xGMI graph vs RCCL graph decode); auto = at N = 8")
    ap.add_argument("--tp70b-batches", default="1,16", help="tp_decode_70b: decode batches timed")
    ap.add_argument("--tp70b-arch", default="llama3-70b",
                    help="tp_decode_70b's decoder (tests: a miniature of the same TP = 8 layout on CPU ranks)")
    ap.add_argument("--block-budget-s", type=float, default=360.0,
                    help="N > 1: wall budget of each multi-GPU block; past it every rank ends the run and rank 0 "
                         "prints the JSON line with the blocks done so far (a hung collective cannot eat the headline)")
    a = ap.parse_args()

    if a.ingest_docs is None:
        a.ingest_docs = a.batch
    info = init_from_env()
    W, R = info.world, info.rank
    if any(k.startswith("DA_") for k in os.environ):  # A/B arms (bench/ab_arms.py): only when asked
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench"))
        from ab_arms import apply_env_overrides
        ab = apply_env_overrides()
        if ab:
            log(info, f"A/B overrides: {ab}")
    dev = info.device
    if dev.type != "cuda" and not a.cpu_rehearsal:
        raise SystemExit("bench.py needs a GPU (run it through gpurun)")
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    t_setup = time.perf_counter()
    TP = a.tp
    if TP < 1 or W % TP:
        raise SystemExit(f"--tp {TP} must divide the world size {W}")
    DP, dp_rank = W // TP, R // TP
    tp_ctx = None
    if TP > 1:
        import torch.distributed as dist
        from docagents_amd.models.llama import TPContext
        groups = [dist.new_group(list(range(g * TP, (g + 1) * TP))) for g in range(DP)]  # every rank creates every group
        tp_ctx = TPContext(R % TP, TP, groups[dp_rank])
    overlap = bool(a.overlap) and TP == 1 and not a.no_graphs
    import torch.distributed as tdist
    ctrl = tdist.new_group(backend="gloo") if W > 1 else None  # the search plane's address exchange
    eng = Engine(a.enc, a.llm, dev, seed=a.seed, tp=tp_ctx, max_batch=a.batch, max_seq=4096, temperature=0.2,
                 max_new_tokens=a.max_new, summary_max_new=128, use_graphs=not a.no_graphs,
                 index_kind=a.index_kind, ivf_lists=a.ivf_lists, ivf_probes=a.ivf_probes, enc_dtype=a.enc_dtype,
                 overlap_waves=overlap)
    shard = ShardedIndex(eng.index, R, W)  # IVF only: the k-means statistics all-reduce (C6)
    d = eng.dim

    # ---- synthetic 100k-chunk shard in HBM ----
    rows = a.index_rows
    X = shard_vectors(R, rows, d, dev)
    ndocs = rows // a.chunks_per_doc
    names = doc_names(W, ndocs)
    doc_ids = names[R]
    ids = (np.int64(R) * 1_000_000_000 + np.arange(rows, dtype=np.int64))
    eng.index.add_bulk(doc_ids, [a.chunks_per_doc] * ndocs, ids, X)
    del X
    if a.index_kind == "ivfflat":
        shard.train(iters=10, sample=min(rows, 1 << 20))  # shared centroids: k-means stats all-reduced (C6)
    plane = SearchPlane.start_world(eng.index, R, W, ctrl, device=dev, timeout_s=120.0)
    vocab_hi = eng.dec_tok.get_vocab_size()
    chunks = ChunkTokens(300, vocab_hi)
    tg = TextGen(seed=77 + dp_rank)  # the ranks of one TP group serve the same queries

    def make_filters(step: int):
        """This rank's B query filters: docs_per_query random documents on random shards (the ranks
        of one TP group serve the same queries)."""
        rng = np.random.default_rng(10_000 + 7919 * step + dp_rank)
        fs = []
        for _ in range(B_cur):
            rr = rng.integers(0, W, size=a.docs_per_query)
            ii = rng.integers(0, ndocs, size=a.docs_per_query)
            fs.append([names[x][y] for x, y in zip(rr, ii)])
        return fs

    use_rccl = W > 1 and (a.search == "rccl" or (a.search == "auto" and TP == 1))

    def search(qv, filters):
        """The QA step's sharded search. rccl: every rank calls it with the same B at the same point of
        the bench (the QA, latency and breakdown loops run in lock-step), so it is one collective
        round — filters exchanged on the gloo control group, then ShardedIndex.search (C2 + local
        scan + C1 over RCCL). plane: submit to this rank's search plane (routed to the owner shards)."""
        if use_rccl:
            flt_all = [None] * W
            tdist.all_gather_object(flt_all, filters, group=ctrl)
            sc, gid = shard.search(qv, a.top_k, a.min_sim, [f for fs in flt_all for f in fs])
            return sc.float().cpu().numpy(), gid.cpu().numpy()
        return plane.submit(qv.float().cpu().numpy(), a.top_k, a.min_sim, filters).result()

    def qa_items(step: int, B: int):
        """A QA step up to the answers: embed the questions, sharded search, context chunks."""
        qs = [tg.question() for _ in range(B)]
        filters = make_filters(step)
        qv = eng.embed(qs)
        s_h, id_h = search(qv, filters)
        items = []
        for b in range(B):
            valid = id_h[b] >= 0
            sc = s_h[b][valid]
            quality = float(sc.mean()) if len(sc) else 0.0
            items.append((qs[b], [chunks.get(int(c)) for c in id_h[b][valid]], quality))
        return items

    def qa_step(step: int, B: int):
        items = qa_items(step, B)
        res = eng.answer_many(items, a.max_new)
        return res, items

    def qa_steps_overlapped(step0: int, n: int, B: int):
        """n QA steps as pipelined waves: step i's embed + search + prefill run while step i - 1
        decodes (every step's answers are complete when this returns)."""
        waves = []

        def next_items(i):
            if i >= n:
                return None
            waves.append(qa_items(step0 + i, B))
            return waves[-1]
        res = eng.answer_overlapped(next_items, a.max_new, a.overlap_frac)
        return res, waves

    # ---- QA throughput ----
    B_cur = a.batch
    log(info, f"setup {time.perf_counter() - t_setup:.1f}s; warmup {a.warmup} steps (B={a.batch}/GPU, W={W})")
    for i in range(a.warmup):
        qa_step(i, a.batch)
        log(info, f"warmup step {i + 1}/{a.warmup} done")
    if overlap:  # both decode states of the pipelined path captured before the timed steps
        qa_steps_overlapped(50, 2, a.batch)
        log(info, "overlapped warmup done")
    barrier(); sync()
    t0 = time.perf_counter()
    plen = []
    if overlap:
        eng.gen.stats.pop("overlap_moves", None); eng.gen.stats.pop("overlap_decode_join_s", None)
        _, waves = qa_steps_overlapped(100, a.steps, a.batch)
        log(info, f"overlap: prefill moved to the full chip at (layer, s) {eng.gen.stats.get('overlap_moves')}, "
                  f"decode joined after {eng.gen.stats.get('overlap_decode_join_s')} s")
        for items in waves:
            plen.extend(len(eng.answer_prompt_ids(q, ch, a.max_new)) for q, ch, _ in items[:4])
    else:
        for i in range(a.steps):
            res, items = qa_step(100 + i, a.batch)
            plen.extend(len(eng.answer_prompt_ids(q, ch, a.max_new)) for q, ch, _ in items[:4])
    sync(); barrier()
    dt = time.perf_counter() - t0
    dt_max = all_reduce_max(dt, dev)
    qps = DP * a.batch * a.steps / dt_max

    # ---- phase breakdown of one extra (untimed) QA step, device-synchronized at phase boundaries ----
    def breakdown(B: int, seed: int) -> dict:
        sy = sync
        ph = {}
        qs = [tg.question() for _ in range(B)]
        filters = make_filters(seed)
        sy(); t = time.perf_counter()
        qv = eng.embed(qs); sy(); ph["embed"] = time.perf_counter() - t; t = time.perf_counter()
        s_h, id_h = search(qv, filters); ph["search"] = time.perf_counter() - t
        t = time.perf_counter()
        items = [(qs[b], [chunks.get(int(c)) for c in id_h[b][id_h[b] >= 0]], 0.5) for b in range(B)]
        prompts = [eng.answer_prompt_ids(q, ch, a.max_new) for q, ch, _ in items]
        ph["prompt_build"] = time.perf_counter() - t
        g_ = eng.gen
        g_.sync_phases = True
        pw0, d0, st0 = g_.stats.get("prefill_wall_s", 0.0), g_.stats["decode_s"], g_.stats["decode_steps"]
        t = time.perf_counter()
        res = g_.generate(prompts, a.max_new)
        sy(); tot = time.perf_counter() - t
        g_.sync_phases = False
        ph["prefill"] = g_.stats["prefill_wall_s"] - pw0
        ph["decode"] = g_.stats["decode_s"] - d0
        t = time.perf_counter()
        _ = [eng.chat.decode(r.tokens) for r in res]
        ph["detokenize"] = time.perf_counter() - t
        ph["generate_other"] = tot - ph["prefill"] - ph["decode"]
        out = {k: round(v * 1000, 2) for k, v in ph.items()}
        steps = g_.stats["decode_steps"] - st0
        out["decode_ms_per_step"] = round(ph["decode"] * 1000 / max(1, steps), 3)
        out["prompt_tokens_mean"] = round(float(np.mean([len(p) for p in prompts])), 1)
        return out

    phases, lat_phases = {}, {}
    if a.breakdown:
        phases = breakdown(a.batch, 777)
        log(info, f"QA step phases (ms): {phases}")

    # ---- p50 cache-miss latency (one query per GPU, end to end) ----
    lat = []
    if a.latency_reps > 0:
        B_cur = 1
        qa_step(900, 1)  # warm the batch-1 graph
        for i in range(a.latency_reps):
            barrier(); sync()
            t1 = time.perf_counter()
            qa_step(1000 + i, 1)
            sync()
            lat.append(all_reduce_max(time.perf_counter() - t1, dev) * 1000)
    p50 = statistics.median(lat) if lat else None
    p90 = sorted(lat)[min(len(lat) - 1, int(round(0.9 * (len(lat) - 1))))] if lat else None
    if a.breakdown and a.latency_reps > 0:  # after the timed reps: the batch-1 graph is captured
        lat_phases = breakdown(1, 778)
        log(info, f"latency query phases (ms): {lat_phases}")

    # ---- ingest docs/min: chunk -> enrich+embed -> summarize -> index (per GPU, batched) ----
    docs_per_min = None
    ingest_runs, ingest_lat = [], []
    ingest_phases: dict = {}
    if a.ingest_docs > 0:
        dg = TextGen(seed=500 + dp_rank)
        batches = [[dg.document(a.ingest_words) for _ in range(a.ingest_docs)] for _ in range(max(1, a.ingest_batches))]
        if a.pdf_ingest:
            from docagents_amd.text.pdf import extract_text as pdf_text
            from docagents_amd.text.pdf import make_pdf

            def _pages(t, per=400):
                w = t.split()
                return [" ".join(w[i:i + per]) for i in range(0, len(w), per)]
            batches = [[make_pdf(_pages(t)) for t in texts] for texts in batches]

        def ingest(texts, tag, ph=None):
            # ph: dict -> per-phase wall time (ms), device-synchronized at each boundary (untimed run)
            tp = [time.perf_counter()]

            def mark(name):
                if ph is not None:
                    sync()
                    tp.append(time.perf_counter())
                    ph[name] = round((tp[-1] - tp[-2]) * 1000, 2)
            if a.pdf_ingest:
                texts = [pdf_text(b) for b in texts]  # the gateway's PDF extraction (cmd/gateway/main.go:223-249)
                mark("pdf_extract")
            all_chunks, owners, summ_in = [], [], []
            for j, t in enumerate(texts):
                cs = chunk_text(t, Options(400, 80))
                all_chunks.extend(f"Document: doc{j}.txt\n\n{c.text}" for c in cs)
                owners.append(len(cs))
                # the analysis agent's summary input: ord-ordered chunks, overlaps removed (§5.7)
                summ_in.append(concatenate_chunks(dedup_overlap([c.text for c in cs], 80)))
            mark("chunk")
            vec = eng.embed(all_chunks)
            mark("embed")
            summaries = eng.summarize_many(summ_in)
            mark("summarize")
            o = 0
            for j, n in enumerate(owners):
                eng.index.add(f"ing{tag}-{R}-{j}", np.arange(n) + 5_000_000_000 + o, vec[o:o + n])
                o += n
            mark("index_add")
            return summaries

        ingest(batches[0][:2], "w")
        for bi, texts in enumerate(batches):
            barrier(); sync()
            t2 = time.perf_counter()
            ingest(texts, f"t{bi}")
            sync(); barrier()
            di = all_reduce_max(time.perf_counter() - t2, dev)
            ingest_runs.append(DP * a.ingest_docs / di * 60.0)
        docs_per_min = statistics.median(ingest_runs)
        if a.ingest_latency_reps > 0:
            # the reference's only ingest number is per-document latency: "upload -> summary
            # available: wait 2-3 seconds" (README.md:346). One document at a time, end to end
            # (chunk -> embed -> summarize -> index), after a warm single-document pass
            single = [dg.document(a.ingest_words) for _ in range(a.ingest_latency_reps + 1)]
            if a.pdf_ingest:
                single = [make_pdf(_pages(t)) for t in single]
            ingest(single[:1], "lw")
            for i, doc in enumerate(single[1:]):
                barrier(); sync()
                t3 = time.perf_counter()
                ingest([doc], f"l{i}")
                sync()
                ingest_lat.append(all_reduce_max(time.perf_counter() - t3, dev) * 1000)
            log(info, f"single-document ingest ms: {[round(x, 1) for x in ingest_lat]}")
        if a.breakdown:
            ingest(batches[0], "b", ph=ingest_phases)
            log(info, f"ingest batch phases (ms): {ingest_phases}")

    # ---- the headline's JSON (the N > 1 blocks below add to it) ----
    # physical GPUs behind the ranks (a 1-GPU rehearsal of N ranks must not read as N GPUs)
    import socket
    where = [None] * W
    if W > 1:
        tdist.all_gather_object(where, (socket.gethostname(), dev.index), group=ctrl)
    else:
        where = [(socket.gethostname(), dev.index)]
    n_phys = len(set(map(tuple, where)))
    is_cuda = dev.type == "cuda"
    gen = dict(eng.gen.stats)
    from docagents_amd.parallel import hbm_plan as HP
    plan = HP.bench_plan(HP.BenchArgs(enc=a.enc, llm=a.llm, batch=a.batch, max_new=a.max_new, index_rows=a.index_rows,
                                      enc_dtype=a.enc_dtype, tp=TP, overlap=overlap,
                                      tp70b={"on": True, "off": False}.get(a.tp70b), ingest=a.ingest_docs > 0), W)
    out = {
        "metric": METRIC, "value": round(qps, 3), "unit": "queries/s", "n_gpus": n_phys, "world_size": W,
        "oversubscribed": n_phys < W, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(dt_max / a.steps * 1000, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dist_backend": info.backend, "ranks_seen": None,
        "dtype": {"bf16": "bf16", "fp16": "bf16 (fp16 encoder)", "fp8": "bf16 (fp8 e4m3 encoder GEMMs)"}[a.enc_dtype],
        "data": "synthetic (random-init weights; random unit vectors for the background chunks; synthetic questions)",
        "config": {"model": f"{a.enc} embedder + {a.llm} QA", "global_batch": DP * a.batch,
                   "seq_len": int(np.mean(plen)) if plen else None,
                   "parallelism": (f"tp{TP} x dp{DP}" if TP > 1 else f"dp{W}") + f" + {W}-way sharded index",
                   "qa_waves": f"pipelined (decode beside the next prefill, decode lane {a.overlap_frac:.2f} of the CUs)"
                   if overlap else "sequential",
                   "index_kind": a.index_kind if a.index_kind == "flat" else
                   f"ivfflat(lists={a.ivf_lists}, probes={a.ivf_probes})",
                   "index_rows_per_gpu": a.index_rows, "top_k": a.top_k, "max_new_tokens": a.max_new,
                   "temperature": 0.2, "min_similarity": a.min_sim, "docs_per_query": a.docs_per_query,
                   "search_transport": "rccl all-gather (C2 query rows + C1 per-shard top-k), device merge"
                   if use_rccl else ("search plane (owner-routed, host TCP)" if W > 1 else "local shard")},
        "p50_cache_miss_ms": round(p50, 2) if p50 else None,
        "p90_cache_miss_ms": round(p90, 2) if p90 else None, "latency_reps": len(lat),
        "reference_cache_miss_ms": REFERENCE_CACHE_MISS_MS,
        "cache_miss_speedup_vs_reference": round(REFERENCE_CACHE_MISS_MS / p50, 2) if p50 else None,
        "ingest_docs_per_min": round(docs_per_min, 1) if docs_per_min else None,
        "ingest_docs_per_min_runs": [round(x, 1) for x in ingest_runs],
        "ingest_format": "pdf" if a.pdf_ingest else "txt",
        "ingest_single_doc_p50_ms": round(statistics.median(ingest_lat), 1) if ingest_lat else None,
        "ingest_single_doc_p90_ms": round(sorted(ingest_lat)[min(len(ingest_lat) - 1, int(round(0.9 * (len(ingest_lat) - 1))))], 1)
        if ingest_lat else None,
        "ingest_single_doc_reps": len(ingest_lat), "ingest_single_doc_words": a.ingest_words,
        "reference_ingest_single_doc_ms": "2000-3000 (README.md:346: upload -> summary, 'wait 2-3 seconds')",
        "prefill_tokens": gen["prefill_tokens"], "decode_steps": gen["decode_steps"],
        "qa_step_phase_ms": phases or None,
        "latency_phase_ms": lat_phases or None,
        "ingest_phase_ms": ingest_phases or None,
        # per-rank HBM: the plan (parallel/hbm_plan.py, per phase) and what the caching allocator peaked at
        "hbm_plan_gb": HP.plan_gb(plan),
        "hbm_peak_gb": {"headline": round(torch.cuda.max_memory_allocated(dev) / 1e9, 1)} if is_cuda else None,
    }
    out["search_plane"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in plane.stats.items()}

    # ---- the multi-GPU mechanisms, timed (N > 1; after the headline, every rank together) ----
    # parallel/collective_bench.py: C1 + C2 as RCCL collectives (>= 20 sharded searches of B rows per
    # rank), the decoder at TP = N (xGMI all-reduce vs torch.distributed, eager and graph-captured, batch
    # 1 and B) with the per-decision TP verdict, Llama-3-70B at TP = 8 (BASELINE config 5's QA model),
    # and the xGMI all-reduce vs RCCL per call at 16 KB / 384 KB / 6 MB. Each block reports its own
    # error instead of the bench failing; a watchdog ends the run with the blocks done so far if a
    # block overruns --block-budget-s (a hung collective). The graph-captured RCCL arms (the served
    # TP fallback) run last, in blocks of their own: the one form that has never run on a node.
    multi: dict = {}
    if W > 1:
        from docagents_amd.parallel import collective_bench as CB
        B_cur = a.batch

        def tp_prompts(B, salt):
            rng = np.random.default_rng(4242 + salt)  # the same prompts on every rank
            tq = TextGen(seed=4242 + salt)
            return [eng.answer_prompt_ids(tq.question(), [chunks.get(int(c)) for c in rng.integers(0, 1 << 30, a.top_k)],
                                          a.max_new) for _ in range(B)]
        tp70_batches = sorted({int(x) for x in a.tp70b_batches.split(",") if x.strip()})
        run70 = TP == 1 and (a.tp70b == "on" or (a.tp70b == "auto" and W == HP.TP70B_WORLD))
        td_prompts = {1: tp_prompts(1, 1), a.batch: tp_prompts(a.batch, 2)} if TP == 1 else {}
        p70 = {b: tp_prompts(b, 10 + b) for b in tp70_batches} if run70 else {}
        # the headline's decoder KV cache (213 GB at the default size) and graphs go before the TP
        # decoders are built: both would not fit one GPU (parallel/hbm_plan.py)
        eng.release_decoder()
        import threading
        current = {"block": None, "t0": time.monotonic()}

        def watchdog():
            while not done_ev.wait(1.0):
                if time.monotonic() - current["t0"] <= a.block_budget_s:
                    continue
                out.update(multi)
                out["multi_timeout"] = {"block": current["block"], "budget_s": a.block_budget_s}
                if R == 0:
                    try:
                        line = json.dumps(out)
                    except Exception:  # noqa: BLE001 - a dict the main thread was writing: the headline keys
                        line = json.dumps({k: out[k] for k in list(out) if k not in multi} |
                                          {"multi_timeout": out["multi_timeout"]}, default=str)
                    print(line, flush=True)
                print(f"[bench] rank {R}: block {current['block']} overran {a.block_budget_s:.0f} s; ending the run",
                      file=sys.stderr, flush=True)
                os._exit(0)
        done_ev = threading.Event()
        threading.Thread(target=watchdog, daemon=True, name="bench-watchdog").start()

        def block(name, fn):
            current["block"], current["t0"] = name, time.monotonic()
            if is_cuda:
                torch.cuda.synchronize(dev)
                torch.cuda.reset_peak_memory_stats(dev)
                base = torch.cuda.memory_allocated(dev)
            t_b = time.perf_counter()
            hang = os.environ.get("DA_BENCH_HANG_BLOCK", "")  # tests: a block that never returns
            if hang == name:
                time.sleep(3600)
            try:
                multi[name] = fn()
            except Exception as e:  # noqa: BLE001 - reported in the JSON line, the headline stands
                multi[name] = {"ok": False, "error": repr(e)[:1000]}
            multi[name]["wall_s"] = round(time.perf_counter() - t_b, 1)
            if is_cuda:
                multi[name]["hbm_peak_gb"] = round(torch.cuda.max_memory_allocated(dev) / 1e9, 1)
                multi[name]["hbm_held_before_gb"] = round(base / 1e9, 1)
                out["hbm_peak_gb"][name] = multi[name]["hbm_peak_gb"]
                torch.cuda.empty_cache()
            log(info, f"{name}: {multi[name]}")

        block("rccl_search", lambda: CB.rccl_search(
            shard, search, eng.embed, lambda i: ([tg.question() for _ in range(a.batch)], make_filters(5000 + i)),
            a.top_k, a.min_sim, a.multi_iters, ctrl, dev))

        # ranks sharing one GPU (a rehearsal) make every IPC all-reduce wait for the card's other
        # contexts (~23 ms per call at 8 ranks): a few decode steps there, the full budget on a node
        tp_new = a.max_new if n_phys == W else min(a.max_new, 6)
        if TP == 1:  # (--tp > 1: the headline itself decodes tensor-parallel)
            block("tp_decode", lambda: CB.tp_decode(
                eng.dec_cfg, eng.decoder.w, R, W, dev, td_prompts, tp_new, rccl_graphs=False,
                log=lambda m: log(info, m)))
        if run70:
            # BASELINE config 5's QA model on the fabric: Llama-3-70B built directly as TP = N shards
            # (seeded per shard), the served form (xGMI all-reduce, graph-replayed) vs the collective
            # library eager; the graph-captured RCCL fallback in the last block
            from docagents_amd.models.configs import decoder_config
            coll = "rccl" if info.backend == "nccl" else info.backend
            arms70 = ("xgmi_graph", f"{coll}_eager")
            block("tp_decode_70b", lambda: CB.tp_decode(
                decoder_config(a.tp70b_arch), None, R, W, dev, p70, tp_new, verdict=False, seed=a.seed + 70,
                arms=arms70, log=lambda m: log(info, m)))
        if is_cuda:
            from docagents_amd.parallel.xgmi_allreduce import verify_and_time
            block("xgmi_allreduce", lambda: verify_and_time(None, dev))

        # last: on ranks sharing one GPU (a rehearsal) the search streams' high-priority queues,
        # once used, slowed every later block 2-3x (profiles/r5/rank8_gloo/serving_search_order/)
        def serving_search():
            """The serving transports side by side: the owner-routed plane (host TCP, the default) and
            SEARCH_TRANSPORT=rccl (lock-step rounds of RCCL all-gathers; parallel/collective_plane.py)."""
            import datetime

            from docagents_amd.parallel.collective_plane import CollectiveSearchPlane
            cctrl = tdist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=120))
            cdata = tdist.new_group(backend=info.backend)
            # the plane's scan stream, not a new one: ranks sharing one GPU (a rehearsal) each add a
            # hardware queue per stream, and oversubscribed queues are time-sliced
            cplane = CollectiveSearchPlane(eng.index, R, W, cdata, cctrl, device=dev, stream=plane.stream,
                                           timeout_s=120.0).start()
            try:
                qv = eng.embed([tg.question() for _ in range(a.serving_requests)]).float().cpu().numpy()
                flt = []
                while len(flt) < len(qv):
                    flt.extend(make_filters(9000 + len(flt)))
                reqs = [(qv[i:i + 1], flt[i]) for i in range(len(qv))]
                res = CB.serving_search({"plane": plane, "rccl": cplane}, reqs, a.top_k, a.min_sim, ctrl, dev)
                res["rounds"] = cplane.stats["rounds"]
                res["idle_gathers"] = cplane.stats.get("idle_gathers")
                res["rccl_transport"] = cplane.stats["transport"]
                return res
            finally:
                tdist.barrier(group=ctrl)  # every rank done submitting before the rounds stop
                cplane.stop(timeout=10.0)
        if a.serving_requests > 0:
            block("serving_search", serving_search)
        if info.backend == "nccl" and TP == 1:
            # the served TP fallback when the xGMI probe fails (models/llama.py TPContext.all_reduce_:
            # torch.distributed captured in the decode graph), Phi-3 and, at N = 8, Llama-3-70B
            block("tp_decode_rccl_graph", lambda: CB.tp_decode(
                eng.dec_cfg, eng.decoder.w, R, W, dev, td_prompts, tp_new, rccl_graphs=True, verdict=False,
                arms=("rccl_graph",), log=lambda m: log(info, m)))
            if run70:
                block("tp_decode_70b_rccl_graph", lambda: CB.tp_decode(
                    decoder_config(a.tp70b_arch), None, R, W, dev, p70, tp_new, rccl_graphs=True, verdict=False,
                    seed=a.seed + 70, arms=("rccl_graph",), log=lambda m: log(info, m)))
        done_ev.set()

    out["ranks_seen"] = int(round(all_reduce_sum(1.0, dev)))  # every rank that reached the end of the run
    out.update(multi)
    if R == 0:
        print(json.dumps(out), flush=True)
    barrier()
    plane.stop(timeout=2.0)
    if W == 1:
        shutdown()
        return
    # N > 1: every rank is done and past the barrier; end without the interpreter's teardown. An
    # 8-rank run on the box aborted one rank AFTER the JSON line with "terminate called without an
    # active exception" (a native thread destroyed joinable at exit: profiles/r6/
    # rehearsal_config5_llama70b_tp8_fp8enc_ivf_8rank_1gpu.err.txt), which turns the launcher's
    # status into a failure for a run whose every result is in
    barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(0)


if __name__ == "__main__":
    main()
