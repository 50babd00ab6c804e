"""Durable vector shard: append-only vector log + periodic snapshots.

The reference persists every embedding in Postgres inside ``SaveEmbeddings``
(internal/store/postgres.go:176-201) and searches the persisted rows (:218-285), so a crash of any
process loses nothing. Here the rows live in HBM; this log makes them survive a crash of the engine
process (SIGKILL, watchdog ``os._exit``, a lost box):

* every index mutation is appended to ``shard{rank}.wal.{gen}`` BEFORE it is applied to the HBM
  index and the file is fsync'ed (``fsync=True``) before the RPC returns — the same point at which
  the reference's INSERT has committed;
* a checkpoint writes ``shard{rank}.snap`` (safetensors, live rows only, the covered log generation
  in its metadata) atomically, then starts generation ``gen + 1`` and deletes the covered logs;
* ``recover`` = load the snapshot + replay every newer generation in order. A torn tail record (a
  crash mid-append) fails its CRC and is cut off; everything before it is kept.

Record framing: ``b"DAVL" | u32 payload_len | u32 crc32(payload) | payload``; payload =
``u8 op | u16 len(doc) | doc utf-8 | u32 n | u32 dim | i64 keys[n] | bf16 vecs[n, dim]`` with
op 1 = replace the document's rows by these (embed_index: the engine sees every chunk of the
document), op 2 = remove the document, op 3 = per-chunk upsert (index_add: drop only the document's
rows whose keys are in the batch, then add — the reference's ``ON CONFLICT (chunk_id)``,
postgres.go:197).

A mutation is validated against the index (vector rank / dim, one key per vector) BEFORE it is
logged, so a bad request is rejected without leaving a record behind; a record that still fails to
apply on replay (a log written by an older build) is skipped and counted (``quarantined``), never
allowed to stop the engine from starting. Checkpoint files and the directory are fsync'ed before
the logs they cover are deleted.
"""
from __future__ import annotations

import glob
import os
import re
import struct
import zlib

import numpy as np
import torch

MAGIC = b"DAVL"
OP_PUT, OP_REMOVE, OP_UPSERT = 1, 2, 3
_HDR = struct.Struct("<4sII")


def _encode(op: int, doc_id: str, keys: np.ndarray | None = None, vecs: torch.Tensor | None = None) -> bytes:
    d = doc_id.encode()
    if op == OP_REMOVE or keys is None:
        body = struct.pack("<BH", op, len(d)) + d + struct.pack("<II", 0, 0)
    else:
        v = vecs.detach().to(device="cpu", dtype=torch.bfloat16).contiguous()
        n, dim = int(v.shape[0]), int(v.shape[1]) if v.dim() == 2 else 0
        k = np.ascontiguousarray(keys, dtype=np.int64)
        if k.shape[0] != n:
            raise ValueError(f"{k.shape[0]} keys for {n} vectors")
        body = (struct.pack("<BH", op, len(d)) + d + struct.pack("<II", n, dim) + k.tobytes()
                + v.view(torch.int16).numpy().tobytes())
    return _HDR.pack(MAGIC, len(body), zlib.crc32(body)) + body


def _decode(body: bytes):
    op, dl = struct.unpack_from("<BH", body, 0)
    o = 3
    doc = body[o:o + dl].decode()
    o += dl
    n, dim = struct.unpack_from("<II", body, o)
    o += 8
    if op == OP_REMOVE:
        return op, doc, None, None
    keys = np.frombuffer(body, dtype=np.int64, count=n, offset=o).copy()
    o += 8 * n
    raw = np.frombuffer(body, dtype=np.int16, count=n * dim, offset=o).copy()
    vecs = torch.from_numpy(raw).view(torch.bfloat16).view(n, dim)
    return op, doc, keys, vecs


def fsync_dir(path: str) -> None:
    """Make a rename / create / unlink inside ``path`` durable."""
    fd = os.open(path, os.O_RDONLY)
    try:
        os.fsync(fd)
    finally:
        os.close(fd)


def validate(index, keys, vecs) -> None:
    """Raise ValueError for a mutation ``index.add`` would reject (checked before it is logged)."""
    if vecs.dim() != 2:
        raise ValueError(f"vectors must be [n, dim], got shape {tuple(vecs.shape)}")
    n, dim = int(vecs.shape[0]), int(vecs.shape[1])
    if n and dim != index.dim:
        raise ValueError(f"vector dim {dim} != index dim {index.dim}")
    if len(np.asarray(keys).reshape(-1)) != n:
        raise ValueError(f"{len(np.asarray(keys).reshape(-1))} keys for {n} vectors")


def read_records(path: str):
    """Yield (op, doc, keys, vecs) of the valid prefix of a log; returns the byte length of that prefix
    through StopIteration.value (callers use ``scan``)."""
    good = 0
    with open(path, "rb") as f:
        data = f.read()
    while good + _HDR.size <= len(data):
        magic, ln, crc = _HDR.unpack_from(data, good)
        end = good + _HDR.size + ln
        if magic != MAGIC or end > len(data):
            break
        body = data[good + _HDR.size:end]
        if zlib.crc32(body) != crc:
            break
        yield _decode(body)
        good = end
    return good


def scan(path: str):
    """(records, valid_bytes, total_bytes) of one log file."""
    recs = []
    gen = read_records(path)
    try:
        while True:
            recs.append(next(gen))
    except StopIteration as s:
        good = s.value or 0
    return recs, good, os.path.getsize(path)


class ShardLog:
    """Write-ahead log + snapshots for one rank's vector shard (an index with ``add`` /
    ``remove_doc`` / the snapshot helpers of ``docagents_amd.index.snapshot``)."""

    def __init__(self, directory: str, rank: int = 0, fsync: bool = True):
        self.dir = os.path.abspath(directory)
        self.rank = rank
        self.fsync = fsync
        os.makedirs(self.dir, exist_ok=True)
        self.snap_path = os.path.join(self.dir, f"shard{rank}.snap")
        self.gen = 0
        self._f = None
        # rows_since_ckpt counts every logged mutation's rows (removes count 1): the periodic
        # checkpoint runs when it is non-zero
        self.stats = {"appended": 0, "replayed": 0, "torn_bytes": 0, "checkpoints": 0, "rows_since_ckpt": 0,
                      "quarantined": 0}
        self.quarantine: list[dict] = []

    # ------------------------------------------------------------------ files
    def _wal(self, gen: int) -> str:
        return os.path.join(self.dir, f"shard{self.rank}.wal.{gen}")

    def _gens(self) -> list[int]:
        out = []
        for p in glob.glob(os.path.join(self.dir, f"shard{self.rank}.wal.*")):
            m = re.search(r"\.wal\.(\d+)$", p)
            if m:
                out.append(int(m.group(1)))
        return sorted(out)

    def _open(self):
        if self._f is not None:
            self._f.close()
        new = not os.path.exists(self._wal(self.gen))
        self._f = open(self._wal(self.gen), "ab")
        if new and self.fsync:
            fsync_dir(self.dir)  # the new generation's directory entry is durable before anything relies on it

    # ------------------------------------------------------------------ recovery
    def recover(self, index) -> dict:
        """Restore ``index`` (assumed empty) from the snapshot + newer logs; open the log for appends."""
        from .snapshot import load_index, snapshot_meta
        snap_gen = -1
        rows = 0
        if os.path.exists(self.snap_path):
            snap_gen = int(snapshot_meta(self.snap_path).get("wal_gen", "-1"))
            rows = load_index(index, self.snap_path)
        replayed = torn = 0
        gens = [g for g in self._gens() if g > snap_gen]
        for g in gens:
            recs, good, total = scan(self._wal(g))
            for op, doc, keys, vecs in recs:
                try:
                    self._apply(index, op, doc, keys, vecs)
                except Exception as e:  # noqa: BLE001 - a record that cannot apply must not block startup
                    self.stats["quarantined"] += 1
                    self.quarantine.append({"gen": g, "op": op, "doc": doc, "err": repr(e)})
                    continue
                replayed += 1
            if good < total:  # torn tail: keep the valid prefix so later appends stay readable
                torn += total - good
                with open(self._wal(g), "r+b") as f:
                    f.truncate(good)
        for g in self._gens():
            if g <= snap_gen:
                os.remove(self._wal(g))
        self.gen = max([snap_gen + 1] + gens)
        self._open()
        self.stats["replayed"] += replayed
        self.stats["torn_bytes"] += torn
        return {"snapshot_rows": rows, "replayed": replayed, "torn_bytes": torn, "gen": self.gen,
                "rows": len(index), "quarantined": self.stats["quarantined"]}

    @staticmethod
    def _apply(index, op, doc, keys, vecs):
        writing = getattr(index, "writing", None)
        if writing is None:
            return ShardLog._apply_ops(index, op, doc, keys, vecs)
        with writing():  # remove + add commit as ONE mutation for concurrent scans (index/flat.py)
            return ShardLog._apply_ops(index, op, doc, keys, vecs)

    @staticmethod
    def _apply_ops(index, op, doc, keys, vecs):
        if op == OP_REMOVE:
            index.remove_doc(doc)
        elif op == OP_UPSERT:
            validate(index, keys, vecs)
            index.remove_keys(doc, keys)
            index.add(doc, keys, vecs)
        elif op == OP_PUT:
            validate(index, keys, vecs)
            index.remove_doc(doc)  # put = replace the document's rows (idempotent re-index)
            index.add(doc, keys, vecs)
        else:
            raise ValueError(f"unknown log op {op}")

    # ------------------------------------------------------------------ mutations
    def _append(self, rec: bytes):
        if self._f is None:
            self._open()
        self._f.write(rec)
        self._f.flush()
        if self.fsync:
            os.fsync(self._f.fileno())
        self.stats["appended"] += 1

    def put(self, index, doc_id: str, keys, vecs: torch.Tensor):
        """Validate, log, then replace ``doc_id``'s rows in ``index`` with ``vecs`` (device or host)."""
        self._mutate(index, OP_PUT, doc_id, keys, vecs)

    def upsert(self, index, doc_id: str, keys, vecs: torch.Tensor):
        """Validate, log, then upsert ``doc_id``'s rows by key (rows with other keys are kept)."""
        self._mutate(index, OP_UPSERT, doc_id, keys, vecs)

    def _mutate(self, index, op, doc_id, keys, vecs):
        keys = np.asarray(keys, dtype=np.int64).reshape(-1)
        validate(index, keys, vecs)
        self._append(_encode(op, doc_id, keys, vecs))
        self._apply(index, op, doc_id, keys, vecs)
        self.stats["rows_since_ckpt"] += max(1, int(vecs.shape[0]))

    def remove(self, index, doc_id: str) -> int:
        self._append(_encode(OP_REMOVE, doc_id))
        self.stats["rows_since_ckpt"] += 1
        return index.remove_doc(doc_id)

    # ------------------------------------------------------------------ checkpoints
    def checkpoint(self, index) -> str:
        """Snapshot covering every record so far, then rotate to a fresh log generation."""
        from .snapshot import save_index
        save_index(index, self.snap_path, extra_meta={"wal_gen": str(self.gen)}, durable=True)
        old = self.gen
        self.gen += 1
        self._open()
        fsync_dir(self.dir)  # snapshot rename + new generation are on disk before the covered logs go
        for g in self._gens():
            if g <= old:
                os.remove(self._wal(g))
        if self.fsync:
            fsync_dir(self.dir)
        self.stats["checkpoints"] += 1
        self.stats["rows_since_ckpt"] = 0
        return self.snap_path

    def close(self):
        if self._f is not None:
            self._f.close()
            self._f = None
