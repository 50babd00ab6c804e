"""Engine server process: ``python -m docagents_amd.services engine [--listen tcp://0.0.0.0:9090]``.

Multi-GPU: ``python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m
docagents_amd.services engine``. One process per GPU; RCCL ("nccl" backend) carries the data-plane
collectives over xGMI, gloo groups carry the small control messages.

  TP_SIZE=t (divides the world; default 1): world / t independent replicas. Replica r = ranks
  [r t, (r + 1) t), served by its leader on port base + r (unix: path.r<r> for r > 0) with its own
  micro-batchers and continuous scheduler; TP followers step the decoder with their leader. The
  vector index is sharded over every rank; a search goes point to point to the shards that own its
  documents (parallel/search_plane.py), so a dead rank fails only the searches that need its shard.
  SEARCH_TRANSPORT=rccl (TP_SIZE=1): every rank's searches travel instead in lock-step rounds of
  RCCL all-gathers over xGMI (parallel/collective_plane.py; one hung rank then stops search on all).
  Agents connect to the base URL; ``EngineCluster`` discovers the other replicas (topology RPC),
  load-balances generation / embedding over them and routes index calls to the owner's replica.
Durable shards (default): ``--index-dir DIR`` (INDEX_DIR, default DATA_DIR/index) holds each rank's
vector log + snapshot (index/wal.py); a restarted engine recovers every row it acknowledged, after
SIGKILL too. Checkpoints every INDEX_CHECKPOINT_S seconds and on SIGTERM. INDEX_DIR=none: HBM only.
Legacy ``--snapshot PATH``: restore each rank's shard from PATH.shard{rank} on start, save on SIGTERM.
"""
from __future__ import annotations

import argparse
import asyncio
import os
import signal

import torch


def replica_url(base: str, r: int) -> str:
    """Listen URL of replica r: base port + r for tcp, path.r<r> for unix sockets (r > 0)."""
    if r == 0:
        return base
    if base.startswith("unix://"):
        return f"{base}.r{r}"
    from ..engine.rpc import parse_url
    _, (host, port) = parse_url(base)
    return f"tcp://{host}:{port + r}"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser("engine")
    ap.add_argument("--listen", default=os.environ.get("ENGINE_LISTEN", "tcp://0.0.0.0:9090"))
    ap.add_argument("--snapshot", default=os.environ.get("INDEX_SNAPSHOT", ""))
    ap.add_argument("--index-dir", default=None)
    a = ap.parse_args(argv)

    from ..config import load
    from ..engine.engine import Engine
    from ..engine.server import EngineGroup, EngineServer
    from ..models.llama import TPContext
    from ..parallel.dist import init_from_env
    from ..utils.log import new as new_logger

    cfg = load()
    log = new_logger(cfg.log_level)
    try:
        cfg.validate_engine()
    except ValueError as e:  # before any GPU or process-group work: fail at startup, loudly
        log.error("invalid engine configuration", "err", str(e))
        raise SystemExit(f"engine: {e}") from e
    if cfg.engine_switch_interval_ms > 0:
        # the engine's threads (RPC loop, GPU thread, fast embed lane, search plane, tokenizers)
        # hand the GIL back and forth several times per query (a shorter switch interval was
        # measured for the loaded query path: no gain, profiles/r3/stack)
        import sys
        sys.setswitchinterval(cfg.engine_switch_interval_ms / 1000.0)
    info = init_from_env()
    world, rank = info.world, info.rank
    t = max(1, cfg.tp_size)
    if world % t:
        raise SystemExit(f"TP_SIZE={t} must divide the world size {world}")
    replicas, replica = world // t, rank // t
    rep_ctrl = rep_data = plane_ctrl = search_ctrl = search_data = None
    tp = None
    dev = info.device
    if world > 1:
        import datetime

        import torch.distributed as dist
        # every rank creates every group, in the same order
        for r in range(replicas):
            ranks = list(range(r * t, (r + 1) * t))
            c = dist.new_group(ranks, backend="gloo") if t > 1 else None
            d = dist.new_group(ranks) if t > 1 else None
            if r == replica:
                rep_ctrl, rep_data = c, d
        to = datetime.timedelta(seconds=max(60.0, cfg.engine_step_timeout))
        plane_ctrl = dist.new_group(backend="gloo", timeout=to)  # the plane's one address exchange
        if cfg.search_transport == "rccl":
            # the collective transport's round control (gloo; its timeout bounds a round with a hung
            # peer) and data (RCCL over xGMI on GPU ranks) groups
            sto = datetime.timedelta(seconds=max(10.0, min(60.0, cfg.engine_step_timeout)))
            search_ctrl = dist.new_group(backend="gloo", timeout=sto)
            search_data = dist.new_group(backend="nccl" if dev.type == "cuda" else "gloo")
        if t > 1:
            tp = TPContext(rank % t, t, rep_data)
    # CU-masked lanes before any decode graph is captured: the kernels pick launch forms that assume
    # round-robin XCD dispatch only while no masked stream exists (ops/kernels.py decode_xc_ok)
    lanes = (None, None, None)
    if dev.type == "cuda" and cfg.engine_latency_cus > 0:
        from ..ops.streams import serving_lanes
        lanes = serving_lanes(cfg.engine_latency_cus, dev)
        log.info("cu partition", "latency_cus", cfg.engine_latency_cus)
    eng = Engine(cfg.embed_arch, cfg.llm_arch, dev, seed=cfg.seed, tp=tp, max_batch=cfg.max_batch,
                 kv_cache_gb=cfg.kv_cache_gb,
                 temperature=cfg.temperature, max_new_tokens=cfg.max_new_tokens,
                 summary_max_new=cfg.summary_max_new_tokens, index_kind=cfg.index_kind, ivf_lists=cfg.ivf_lists,
                 ivf_probes=cfg.ivf_probes, max_seq=4096 if dev.type == "cuda" else 1024,
                 enc_dtype=cfg.dtype)
    if cfg.engine_admit_tokens > 0:
        eng.admit_tokens = cfg.engine_admit_tokens
    if cfg.engine_continuous and dev.type == "cuda" and eng.gen is not None:
        eng.scheduler.warmup()  # every row bucket's decode graph, before the first request (all TP ranks)
    index_dir = a.index_dir if a.index_dir is not None else cfg.index_dir_path()
    shard_log = None
    if index_dir and index_dir != "none":
        from ..index.wal import ShardLog
        shard_log = ShardLog(index_dir, rank, fsync=cfg.index_fsync)
        rec = shard_log.recover(eng.index)
        log.info("recovered index shard", "rank", rank, "dir", index_dir, **rec)
    if a.snapshot and os.path.exists(f"{a.snapshot}.shard{rank}"):
        from ..index.snapshot import load_index
        n = load_index(eng.index, f"{a.snapshot}.shard{rank}")
        log.info("restored index shard", "rank", rank, "rows", n)
    from ..parallel.search_plane import SearchPlane
    if cfg.search_transport == "rccl" and world > 1:
        from ..parallel.collective_plane import CollectiveSearchPlane
        plane = CollectiveSearchPlane(eng.index, rank, world, search_data, search_ctrl, device=dev, stream=lanes[2],
                                      timeout_s=max(5.0, min(60.0, cfg.engine_step_timeout)),
                                      idle_s=cfg.search_round_idle_ms / 1000.0,
                                      idle_max_s=cfg.search_round_idle_max_ms / 1000.0).start()
    else:
        plane = SearchPlane.start_world(eng.index, rank, world, plane_ctrl, device=dev, stream=lanes[2],
                                        host=os.environ.get("ENGINE_PLANE_HOST", "127.0.0.1"),
                                        timeout_s=max(5.0, min(60.0, cfg.engine_step_timeout)))
    log.info("search transport", "kind", cfg.search_transport if world > 1 else "local")
    grp = EngineGroup(eng, rank, world, rep_ctrl, rep_data, shard_log=shard_log, tp_size=t, plane=plane)
    if not grp.is_leader:
        grp.follower_loop()
        plane.stop()
        if torch.distributed.is_initialized():
            torch.distributed.destroy_process_group()
        return 0
    urls = [replica_url(a.listen, r) for r in range(replicas)]

    async def serve():
        srv = EngineServer(grp, log, max_batch_items=max(1, eng.gen.max_batch if eng.gen is not None else 64) * 4, step_timeout_s=cfg.engine_step_timeout,
                           hard_timeout_s=cfg.engine_hard_timeout, liveness_s=cfg.engine_liveness_s,
                           continuous=cfg.engine_continuous, cb_steps=cfg.engine_cb_steps,
                           cb_max_steps=cfg.engine_cb_max_steps, lanes=lanes, fast_yield=cfg.engine_fast_yield,
                           admit_min=cfg.engine_admit_min, admit_wait_s=cfg.engine_admit_wait_ms / 1000.0,
                           admit_hold_frac=cfg.engine_admit_hold_frac,
                           checkpoint_s=cfg.index_checkpoint_s, urls=urls)
        if cfg.engine_metrics_port:
            import prometheus_client
            prometheus_client.start_http_server(cfg.engine_metrics_port)
            log.info("engine metrics listening", "port", cfg.engine_metrics_port)
        server = await srv.start(urls[replica])
        from ..utils import timeline
        if timeline.enabled():
            from .runner import _loop_lag_monitor
            asyncio.ensure_future(_loop_lag_monitor())
        log.info("engine listening", "addr", urls[replica], "replica", replica, "replicas", replicas,
                 "world", world, "device", str(dev), "encoder", cfg.embed_arch, "decoder", cfg.llm_arch, "tp", t)
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        for sgn in (signal.SIGINT, signal.SIGTERM):
            try:
                loop.add_signal_handler(sgn, stop.set)
            except (NotImplementedError, RuntimeError):
                pass
        await stop.wait()
        server.close()
        if shard_log is not None:
            await srv._gpu("checkpoint", {"force": True})
            log.info("index checkpoint saved", "dir", index_dir)
        if a.snapshot:
            await srv._gpu("snapshot", {"path": a.snapshot})
            log.info("index snapshot saved", "path", a.snapshot)
        if t > 1:
            grp._bcast(("shutdown", {}))
        plane.stop()

    asyncio.run(serve())
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
    return 0
