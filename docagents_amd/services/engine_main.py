"""Engine server process: ``python -m docagents_amd.services engine [--listen tcp://0.0.0.0:9090]``.

Multi-GPU: ``python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m
docagents_amd.services engine``. One process per GPU; RCCL ("nccl" backend) carries the data-plane
collectives over xGMI, a gloo group carries the small control messages. Rank 0 serves the RPCs.

  TP_SIZE=1 (default)  data parallel: embeddings / generations split across ranks, index sharded
  TP_SIZE=world        the decoder is tensor-parallel across all ranks (Llama-3-70B class); every
                       rank runs every generation on its shard, index still sharded
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
    info = init_from_env()
    ctrl = data = None
    tp = None
    if info.world > 1:
        import torch.distributed as dist
        ctrl = dist.new_group(backend="gloo")
        data = dist.group.WORLD
        if cfg.tp_size > 1:
            if cfg.tp_size != info.world:
                raise SystemExit("TP_SIZE must be 1 or the world size")
            tp = TPContext(info.rank, info.world, data)
    dev = info.device
    eng = Engine(cfg.embed_arch, cfg.llm_arch, dev, seed=cfg.seed, tp=tp, max_batch=cfg.max_batch,
                 temperature=cfg.temperature, max_new_tokens=cfg.max_new_tokens,
                 summary_max_new=cfg.summary_max_new_tokens, index_kind=cfg.index_kind, ivf_lists=cfg.ivf_lists,
                 ivf_probes=cfg.ivf_probes, max_seq=4096 if dev.type == "cuda" else 1024,
                 enc_dtype="fp8" if cfg.dtype == "fp8" else "bf16")
    if cfg.engine_admit_tokens > 0:
        eng.admit_tokens = cfg.engine_admit_tokens
    index_dir = a.index_dir if a.index_dir is not None else cfg.index_dir_path()
    shard_log = None
    if index_dir and index_dir != "none":
        from ..index.wal import ShardLog
        shard_log = ShardLog(index_dir, info.rank, fsync=cfg.index_fsync)
        rec = shard_log.recover(eng.index)
        log.info("recovered index shard", "rank", info.rank, "dir", index_dir, **rec)
    grp = EngineGroup(eng, info.rank, info.world, ctrl, data, shard_log=shard_log)
    grp.tensor_parallel = tp is not None
    if a.snapshot and os.path.exists(f"{a.snapshot}.shard{info.rank}"):
        from ..index.snapshot import load_index
        n = load_index(eng.index, f"{a.snapshot}.shard{info.rank}")
        log.info("restored index shard", "rank", info.rank, "rows", n)
    if info.rank != 0:
        grp.follower_loop()
        return 0

    async def serve():
        srv = EngineServer(grp, log, max_batch_items=cfg.max_batch * 4, step_timeout_s=cfg.engine_step_timeout,
                           hard_timeout_s=cfg.engine_hard_timeout, liveness_s=cfg.engine_liveness_s,
                           continuous=cfg.engine_continuous, cb_steps=cfg.engine_cb_steps,
                           checkpoint_s=cfg.index_checkpoint_s)
        if cfg.engine_metrics_port:
            import prometheus_client
            prometheus_client.start_http_server(cfg.engine_metrics_port)
            log.info("engine metrics listening", "port", cfg.engine_metrics_port)
        server = await srv.start(a.listen)
        log.info("engine listening", "addr", a.listen, "world", info.world, "device", str(dev),
                 "encoder", cfg.embed_arch, "decoder", cfg.llm_arch, "tp", cfg.tp_size)
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
            await srv._gpu("checkpoint", {})
            log.info("index checkpoint saved", "dir", index_dir)
        if a.snapshot:
            await srv._gpu("snapshot", {"path": a.snapshot})
            log.info("index snapshot saved", "path", a.snapshot)
        if info.world > 1:
            grp._bcast(("shutdown", {}))

    asyncio.run(serve())
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
    return 0
