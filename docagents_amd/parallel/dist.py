"""Process-group plumbing: one process per GPU, ``torch.distributed`` over RCCL ("nccl" backend on
ROCm) on the GPUs, gloo on CPU (tests). Reads RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from the
environment (torchrun). Collectives used by the framework:

  C1 all-gather of per-shard top-k          -> ``ShardedIndex.search``
  C2 all-gather of query embeddings         -> ``ShardedIndex.search``
  C3 all-reduce of row-parallel outputs     -> ``LlamaDecoder`` (TP)
  C4 all-gather of vocab-parallel logits    -> ``LlamaDecoder`` (TP)
  C6 all-reduce of k-means statistics       -> ``IVFFlatIndex.train``
  C7 barrier / liveness all-reduce          -> ``liveness_check``
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init_from_env(prefer_gpu: bool = True, timeout_s: int = 600) -> DistInfo:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = prefer_gpu and torch.cuda.is_available()
    if use_gpu:
        # one rank per GPU; more ranks than GPUs (a rehearsal of the multi-rank path on a 1-GPU box,
        # DA_DIST_BACKEND=gloo) wrap around
        idx = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(idx)
        device = torch.device("cuda", idx)
    else:
        device = torch.device("cpu")
    backend = "none"
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        backend = os.environ.get("DA_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if use_gpu and backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    elif dist.is_initialized():
        backend = dist.get_backend()
    return DistInfo(rank, world, local, backend, device)


def barrier():
    if dist.is_initialized():
        dist.barrier()


def all_reduce_max(x: float, device) -> float:
    if not dist.is_initialized():
        return x
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_sum(x: float, device) -> float:
    if not dist.is_initialized():
        return x
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t)
    return float(t.item())


def all_gather_rows(t: torch.Tensor, group=None) -> torch.Tensor:
    """[n, ...] per rank (same n on every rank) -> [world * n, ...] in rank order."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return t
    w = dist.get_world_size(group)
    if t.is_cuda and dist.get_backend(group) == "gloo":  # gloo rehearsal of GPU ranks: stage on the host
        return all_gather_rows(t.cpu(), group).to(t.device)
    out = torch.empty((w * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t.contiguous(), group=group)
    return out


def _stage(t: torch.Tensor, group) -> torch.Tensor:
    """gloo cannot all-gather device tensors (1-GPU multi-rank rehearsal): stage on the host."""
    return t.cpu() if t.is_cuda and dist.get_backend(group) == "gloo" else t


def all_gather_padded_rows(t: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """Rank r holds rows [r*per, min(n_total, (r+1)*per)) of an n_total-row result, per =
    ceil(n_total / world) (the engine's data-parallel slicing). One all_gather_into_tensor of the
    zero-padded slices (RCCL on GPU ranks) -> the [n_total, ...] result in rank order, on every rank."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return t
    w = dist.get_world_size(group)
    per = (n_total + w - 1) // w
    pad = torch.zeros((per,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[:t.shape[0]] = t
    src = _stage(pad, group)
    out = torch.empty((w * per,) + tuple(t.shape[1:]), dtype=t.dtype, device=src.device)
    dist.all_gather_into_tensor(out, src, group=group)
    return out[:n_total].to(t.device)


def pack_scores_ids(scores: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    """fp32 scores + int64 ids [Q, k] -> one int64 [Q, k, 2] buffer (scores as their bit pattern), so
    a search's top-k lists travel in ONE collective."""
    bits = scores.float().contiguous().view(torch.int32).to(torch.int64)
    return torch.stack([ids.to(torch.int64), bits], dim=-1).contiguous()


def unpack_scores_ids(p: torch.Tensor):
    return p[..., 1].to(torch.int32).view(torch.float32), p[..., 0]


def all_gather_bytes(payload: bytes, device, group=None) -> list[bytes]:
    """Variable-length byte payloads from every rank, as tensors (RCCL on GPU ranks, gloo on CPU):
    one all-gather of the lengths, one of the zero-padded uint8 payloads. The engine's data plane
    for results that are not plain tensors (answers, summaries) — no pickles."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return [payload]
    w = dist.get_world_size(group)
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if dev.type == "cuda" and dist.get_backend(group) == "gloo":
        dev = torch.device("cpu")
    n = torch.tensor([len(payload)], dtype=torch.int64, device=dev)
    ns = torch.empty(w, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(ns, n, group=group)
    lens = ns.cpu().tolist()
    mx = max(1, max(lens))
    buf = torch.zeros(mx, dtype=torch.uint8, device=dev)
    if payload:
        buf[:len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(dev)
    out = torch.empty(w * mx, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(out, buf, group=group)
    host = out.cpu().numpy()
    return [host[i * mx:i * mx + lens[i]].tobytes() for i in range(w)]


def liveness_check(device, timeout_ok: bool = True) -> int:
    """C7: every rank contributes 1; returns the number of live ranks (== world when healthy)."""
    if not dist.is_initialized():
        return 1
    t = torch.ones(1, dtype=torch.int32, device=device)
    dist.all_reduce(t)
    return int(t.item())


def shutdown():
    if dist.is_initialized():
        try:
            dist.barrier()
        finally:
            dist.destroy_process_group()
