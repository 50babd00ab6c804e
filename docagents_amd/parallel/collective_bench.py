"""The multi-GPU mechanisms of the north star, timed (``bench.py`` at N > 1, after the headline).

The headline (QA q/s with N data-parallel replicas) scales by replicas, as the reference does
(docker-compose.yml:84-85,105-106), so on its own it says nothing about the fabric. These blocks
time the collectives the north star names, each on all N ranks together:

  rccl_search   C2 + C1 as RCCL collectives: ``ShardedIndex.search`` (all-gather of every rank's
                query rows, local fused scan + filter + floor + top-k, ONE packed all-gather of the
                per-shard top-k, topk_merge kernel) at B rows per rank, >= 20 timed calls; q/s over
                the whole world, p50 / p90 ms per call, and the rows checked identical to the
                serving plane's owner-routed answer for the same batch
  tp_decode     the bench's decoder at TP = N over every rank (column / row-parallel layers,
                vocab-parallel sampler): decode ms per step at batch 1 and batch B with the xGMI
                IPC all-reduce (graph-replayed, as served) and with torch.distributed (RCCL on
                GPUs) in its place, plus the per-decision agreement verdict of a TP = N decoder
                with the unsharded one (parallel/tp_verify.py)
  tp_decode_70b the same timing for Llama-3-70B at TP = 8 (BASELINE config 5's QA model), each rank
                building only its shard from a per-shard seed (``tp_decode(..., full_weights=None)``)
  *_rccl_graph  the served TP fallback: torch.distributed all-reduces captured in the decode graph
  xgmi          the IPC all-reduce vs RCCL per call at 16 KB / 384 KB / 6 MB (xgmi_allreduce.py)

Every block is collective: all ranks call it in the same order with the same shapes.
"""
from __future__ import annotations

import statistics
import time

import numpy as np
import torch
import torch.distributed as dist

from .dist import all_reduce_max, barrier


def _sync(dev):
    if torch.device(dev).type == "cuda":
        torch.cuda.synchronize(dev)


def _pct(xs, q):
    s = sorted(xs)
    return s[min(len(s) - 1, int(round(q * (len(s) - 1))))]


def rccl_search(shard, plane_search, embed, make_batch, k: int, min_sim: float, iters: int, ctrl, dev) -> dict:
    """make_batch(i) -> (questions, this rank's per-row document filters). plane_search(qv, filters)
    -> (scores, ids) through the serving plane. Returns the rccl_search block."""
    W = shard.world
    batches = []
    for i in range(iters + 2):
        qs, mine = make_batch(i)
        qv = embed(qs)
        every = [None] * W
        dist.all_gather_object(every, mine, group=ctrl)
        batches.append((qv, mine, [f for r in range(W) for f in every[r]]))
    B = batches[0][0].shape[0]
    qv, mine, flt_all = batches[0]
    s_r, id_r = shard.search(qv, k, min_sim, flt_all)
    s_r, id_r = s_r.float().cpu().numpy(), id_r.cpu().numpy()
    shard.search(*batches[1][:1], k, min_sim, batches[1][2])  # warm
    # throughput: back to back
    _sync(dev); barrier()
    t0 = time.perf_counter()
    for qv, _, flt in batches[2:]:
        shard.search(qv, k, min_sim, flt)
    _sync(dev)
    dt = all_reduce_max(time.perf_counter() - t0, dev)
    # latency: one call at a time (every rank enters together: the call is collective)
    lat = []
    for qv, _, flt in batches[2:]:
        _sync(dev)
        t1 = time.perf_counter()
        shard.search(qv, k, min_sim, flt)
        _sync(dev)
        lat.append(all_reduce_max(time.perf_counter() - t1, dev) * 1000)
    # identity with the serving plane's owner-routed answer for batch 0, after every collective of
    # the block (a rank-local plane failure cannot desynchronise the ranks' collective sequence)
    try:
        s_p, id_p = plane_search(batches[0][0], batches[0][1])
        agree = int(sum(1 for b in range(B) if np.array_equal(id_r[b], id_p[b])))
        close = bool(np.allclose(np.where(id_r >= 0, s_r, 0), np.where(id_p >= 0, s_p, 0), atol=1e-3))
    except Exception as e:  # noqa: BLE001
        agree, close = -1, repr(e)[:200]
    return {"rows_per_rank": B, "iters": iters, "world": W, "qps": round(W * B * iters / dt, 1),
            "ms_per_call_mean": round(dt / iters * 1000, 3), "p50_ms": round(statistics.median(lat), 3),
            "p90_ms": round(_pct(lat, 0.9), 3), "rows_identical_to_plane": agree, "rows_checked": B,
            "scores_close": close}


def serving_search(planes: dict, reqs: list, k: int, min_sim: float, ctrl, dev, inflight: int = 64) -> dict:
    """The two serving search transports under a serving load. planes: {name: plane} — "plane" (the
    owner-routed point-to-point SearchPlane) and "rccl" (CollectiveSearchPlane: lock-step rounds of
    RCCL all-gathers); reqs: this rank's single-question searches [(vec [1, d], document filter)].
    Every rank submits its requests ``inflight`` at a time through one transport, then the next.
    Per transport: aggregate searches/s over the ranks (wall = max over ranks), p50 / p90 of a
    search's submit -> result time; and whether both transports returned the same ids for every
    request. The barriers run on the gloo ``ctrl`` group: the collective transport's round thread
    drives RCCL meanwhile, and no second thread may (two communicators from two threads)."""
    W = dist.get_world_size()
    out, ids = {}, {}
    for name, pl in planes.items():
        pl.submit(reqs[0][0], k, min_sim, [reqs[0][1]]).result(120)  # warm (connections / first round)
        dist.barrier(group=ctrl)
        lat, got = [], []
        t0 = time.perf_counter()
        for w0 in range(0, len(reqs), inflight):
            wave = []
            for v, f in reqs[w0:w0 + inflight]:
                done = {}
                fut = pl.submit(v, k, min_sim, [f])
                fut.add_done_callback(lambda _f, d=done: d.setdefault("t", time.perf_counter()))
                wave.append((time.perf_counter(), fut, done))
            for ts, fut, done in wave:
                _, g = fut.result(120)
                lat.append((done.get("t", time.perf_counter()) - ts) * 1000)
                got.append(np.asarray(g).reshape(-1))
        dt = all_reduce_max(time.perf_counter() - t0, dev)
        ids[name] = got
        out[name] = {"searches_per_s": round(W * len(reqs) / dt, 1), "p50_ms": round(statistics.median(lat), 3),
                     "p90_ms": round(_pct(lat, 0.9), 3)}
    if len(ids) == 2:
        a, b = ids.values()
        out["ids_identical"] = int(all_reduce_max(float(sum(1 for x, y in zip(a, b) if not np.array_equal(x, y))),
                                                  dev)) == 0
    out.update({"requests_per_rank": len(reqs), "inflight_per_rank": inflight, "world": W})
    return out


def _round_up(x: int, m: int) -> int:
    return -(-x // m) * m


def hbm_check(need: int, what: str, dev, margin: int = 8 << 30) -> None:
    """Refuse an allocation of ``need`` bytes that would not fit the device's free memory (less a
    margin for the runtime and RCCL): the block then reports a clear error instead of an OOM
    half-way through its collectives. Collective: every rank refuses if any rank must (a rank that
    raised alone would leave its peers inside the next collective)."""
    short = ""
    if torch.device(dev).type == "cuda":
        free, total = torch.cuda.mem_get_info(dev)
        if need + margin > free:
            short = (f"{what}: needs {need / 1e9:.1f} GB + {margin / 1e9:.0f} GB margin, "
                     f"{free / 1e9:.1f} of {total / 1e9:.1f} GB free")
    if dist.is_initialized() and dist.get_world_size() > 1:
        if all_reduce_max(1.0 if short else 0.0, dev) > 0 and not short:
            short = f"{what}: another rank lacks the memory"
    if short:
        raise MemoryError(short)


def tp_decode(dec_cfg, full_weights, rank: int, world: int, dev, prompts_by_b: dict, max_new: int,
              rccl_graphs: bool | None = None, verdict: bool = True, log=None, seed: int = 0,
              arms: tuple | None = None) -> dict:
    """The decoder at TP = world over every rank, timed per decode step. prompts_by_b: {batch:
    prompts} (the same on every rank). full_weights: the unsharded weights (identical on every rank:
    seeded), or None to build this rank's shard directly from ``seed`` (Llama-3-70B: never the
    140 GB unsharded model on a rank). Arms: the xGMI all-reduce graph-replayed (the served form)
    and eager, and torch.distributed in its place, eager and graph-captured (``rccl_graph``: the
    form serving falls back to when the xGMI probe fails, models/llama.py TPContext.all_reduce_;
    on by default with RCCL). ``arms``: only these arm names."""
    from ..engine.generator import Generator
    from ..models.llama import KVCache, LlamaDecoder, TPContext, random_weights, shard_weights
    backend = dist.get_backend()
    if rccl_graphs is None:
        rccl_graphs = backend == "nccl"
    maxB = max(prompts_by_b)
    longest = max(len(p) for ps in prompts_by_b.values() for p in ps)
    max_seq = min(dec_cfg.max_pos, _round_up(longest + max_new + 8, 256))
    from .hbm_plan import decoder_weight_bytes
    hbm_check(KVCache.bytes_for(dec_cfg, maxB + 4, max_seq, world)
              + (decoder_weight_bytes(dec_cfg, world) if full_weights is None else 0),
              f"tp_decode {dec_cfg.name} TP={world} ({maxB + 4} slots x {max_seq})", dev)
    tp = TPContext(rank, world, None)
    w = (random_weights(dec_cfg, dev, seed, rank, world) if full_weights is None
         else shard_weights(dec_cfg, full_weights, rank, world))
    model = LlamaDecoder(dec_cfg, dev, tp=tp, weights=w)
    del w
    model.alloc_cache(maxB + 4, max_seq)
    xg = (tp.xgmi, tp.xgmi_norm)
    run = []
    if xg[0] is not None:
        run += [("xgmi_graph", True, True), ("xgmi_eager", True, False)]
    run.append((f"{'rccl' if backend == 'nccl' else backend}_eager", False, False))
    if rccl_graphs and backend == "nccl":
        run.append(("rccl_graph", False, True))
    if arms is not None:
        run = [r for r in run if r[0] in arms]
    arms = run
    out: dict = {"tp": world, "model": dec_cfg.name, "max_new_tokens": max_new,
                 "weights_gb_per_rank": round(decoder_weight_bytes(dec_cfg, world) / 1e9, 2),
                 "kv_slots": maxB + 4, "kv_max_seq": max_seq,
                 "prompt_tokens_mean": {str(b): round(float(np.mean([len(p) for p in ps])), 1)
                                        for b, ps in prompts_by_b.items()},
                 "xgmi_mapped": xg[0] is not None, "arms": {}}
    xgmi_failed = ""
    for name, use_x, graphs in arms:
        if use_x and xgmi_failed:
            out["arms"][name] = {"skipped": xgmi_failed}
            continue
        tp.xgmi, tp.xgmi_norm = xg if use_x else (None, None)
        gen = Generator(model, max_batch=maxB, max_seq=max_seq, temperature=0.2, seed=0, use_graphs=graphs)
        row = {"graphs": graphs}
        try:
            for b, prompts in sorted(prompts_by_b.items()):
                gen.generate([p[:64] for p in prompts], max_new)  # warm: the decode graph of this bucket
                gen.sync_phases = True
                _sync(dev); barrier()
                s0, n0, p0 = gen.stats["decode_s"], gen.stats["decode_steps"], gen.stats.get("prefill_wall_s", 0.0)
                gen.generate(prompts, max_new)
                gen.sync_phases = False
                steps = max(1, gen.stats["decode_steps"] - n0)
                row[f"b{b}_decode_ms_per_step"] = round(all_reduce_max((gen.stats["decode_s"] - s0) / steps, dev) * 1000, 3)
                row[f"b{b}_prefill_ms"] = round(all_reduce_max(gen.stats["prefill_wall_s"] - p0, dev) * 1000, 2)
        finally:
            gen.close()
        if use_x:  # any barrier timeout on any rank -> every rank skips the remaining xGMI arms
            err = ""
            try:
                for c in xg:
                    if c is not None:
                        c.check()
            except Exception as e:  # noqa: BLE001
                err = repr(e)[:200]
            errs: list = [None] * world
            dist.all_gather_object(errs, err)
            xgmi_failed = next((e for e in errs if e), "")
            if xgmi_failed:
                row["xgmi_error"] = xgmi_failed
        out["arms"][name] = row
        if log is not None:
            log(f"tp_decode arm {name}: {row}")
    tp.xgmi, tp.xgmi_norm = xg
    if xg[0] is not None:
        out["xgmi_calls"] = xg[0].calls + (xg[1].calls if xg[1] is not None else 0)
    tp.close()
    del model
    if verdict:
        from .tp_verify import decision_verdict, verdict_ok
        v = decision_verdict(rank, world, None, dev)
        out["agreement"] = {"ok": verdict_ok(v), "arch": v["arch"], "decisions": v["decisions"],
                            "checked": v["checked"], "checked_agree": v["checked_agree"],
                            "prefix_ok": sum(v["prefix_ok"]), "prompts": len(v["prefix_ok"]),
                            "max_logit_diff": round(v["max_logit_diff"], 5), "xgmi": v["xgmi"]}
    if torch.device(dev).type == "cuda":
        torch.cuda.empty_cache()
    return out
