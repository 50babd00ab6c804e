"""Custom all-reduce over xGMI peer memory for tensor-parallel decoding.

Why: the TP=8 Llama-3-70B decode step issues 2 all-reduces per layer x 80 layers, each only
B x 8192 bf16 (16 KB at batch 1). RCCL's ring pays its protocol latency per call and drives one
xGMI link per neighbour; on a full-mesh MI355X node a one-shot kernel that reads all 7 peers'
buffers directly (IPC-mapped, 7 links concurrently) is latency-optimal for such messages, and a
two-shot (reduce-scatter + all-gather through the same buffers) covers prefill-sized ones.

Setup (once per communicator, NOT inside graph capture): every rank allocates a staging buffer
(2 x max_bytes, double-buffered by call parity) and a signal block in UNCACHED device memory
(hipExtMallocWithFlags(..., hipDeviceMallocUncached): peers poll the flags and read the staged rows
across devices, so no GPU may serve them from a stale L2 line), exports the allocations holding
them (hipMemGetAddressRange + hipIpcGetMemHandle; the buffer's offset inside travels with the
handle), exchanges the handles over the process group (all_gather_object), and opens the peers'
handles. Buffers are pooled per process, never freed (see _POOL). After that a call is one kernel launch with constant arguments, so it is
captured into the decode HIP graph like any other kernel. Kernel: ops/csrc/allreduce.hip.

Falls back to ``torch.distributed.all_reduce`` (RCCL) for tensors it does not take (dtype other
than bf16/fp32, size not a multiple of 16 B or above max_bytes) and entirely when the peer
mapping cannot be set up (``XgmiAllReduce.create`` returns None and logs why).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import byref, c_int, c_longlong, c_void_p

import torch
import torch.distributed as dist

from ..ops import kernels as K

_BOUND = False


def _lib():
    global _BOUND
    L = K.lib()
    if not _BOUND:
        sigs = {
            "da_ar_malloc": ([c_longlong, c_int, ctypes.POINTER(c_void_p)], c_int),
            "da_ar_free": ([c_void_p], c_int),
            "da_ar_zero": ([c_void_p, c_longlong], c_int),
            "da_ar_ipc_handle": ([c_void_p, c_void_p], c_int),
            "da_ar_ipc_export": ([c_void_p, c_void_p, ctypes.POINTER(c_longlong)], c_int),
            "da_ar_ipc_open": ([c_void_p, ctypes.POINTER(c_void_p)], c_int),
            "da_ar_ipc_close": ([c_void_p], c_int),
            "da_ar_read_err": ([c_void_p, ctypes.POINTER(ctypes.c_uint)], c_int),
            "da_ar_allreduce": ([c_void_p, c_void_p, c_longlong, c_int, c_int, c_int, c_void_p, c_void_p, c_longlong,
                                 c_int, c_int, c_longlong, c_void_p], c_int),
            "da_ar_allreduce_rmsnorm": ([c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, ctypes.c_float, c_int,
                                         c_int, c_void_p, c_void_p, c_longlong, c_int, c_longlong, c_void_p], c_int),
        }
        for name, (argt, res) in sigs.items():
            fn = getattr(L, name)
            fn.argtypes, fn.restype = argt, res
        for name in ("da_ar_signal_bytes", "da_ar_max_blocks", "da_ar_ipc_handle_bytes"):
            getattr(L, name).restype = c_int
        L.da_ar_clock_khz.restype = c_longlong
        _BOUND = True
    return L


# Exported communicator buffers are pooled per (device, bytes), never freed: an uncached buffer
# allocated after another exported one was freed can land inside the runtime's cached range of the
# old one, and hipIpcGetMemHandle then refuses it (hipErrorInvalidValue on one rank of eight in an
# 8-rank rehearsal that created a communicator after closing two). A pooled buffer keeps its IPC
# handle and is zeroed before reuse.
_POOL: dict = {}
_REFUSED: list = []


def _take(L, dev: torch.device, nbytes: int, hb: int, what: str):
    """(ptr, (handle bytes, offset)) of a zeroed, IPC-exported uncached buffer of nbytes on dev: the
    handle names the allocation containing the buffer, which starts ``offset`` bytes into it."""
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), nbytes)
    if _POOL.get(key):
        p, h = _POOL[key].pop()
        _ok(L.da_ar_zero(p, nbytes), f"zero({what})")
        return p, h
    rc = 0
    for _ in range(4):
        p = c_void_p()
        _ok(L.da_ar_malloc(nbytes, 1, byref(p)), f"hipExtMallocWithFlags({what}, uncached)")
        h, off = ctypes.create_string_buffer(hb), c_longlong(0)
        rc = L.da_ar_ipc_export(p, h, byref(off))
        if rc == 0:
            return p, (h.raw, off.value)
        # an allocation the runtime will not export (seen only with 8 ranks sharing one GPU, on one
        # rank, for a buffer allocated late in the process): keep it (freeing it would hand the same
        # range back) and allocate another
        _REFUSED.append(p)
    _ok(rc, f"hipIpcGetMemHandle({what})")


def _give(dev: torch.device, nbytes: int, item) -> None:
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), nbytes)
    _POOL.setdefault(key, []).append(item)


def _ok(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed: hipError {rc}")


class XgmiAllReduce:
    """One-shot / two-shot all-reduce through IPC-mapped peer buffers (one instance per group)."""

    def __init__(self, group=None, device=None, max_bytes: int = 32 << 20, oneshot_max: int = 512 << 10,
                 grid: int = 0, timeout_ms: int = 5000, probe_ms: int = 2000):
        """Collective over ``group``, and symmetric: every rank takes part in every exchange whether
        or not its own setup worked, and either every rank ends with a working communicator or every
        rank raises (one rank on RCCL while its peers spin on xGMI flags would deadlock the group).
        ``probe_ms`` > 0: one small all-reduce with that bounded wait checks the peers' flags and
        staged rows are really visible across the devices before the communicator is used."""
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if not 2 <= self.world <= 8:
            raise ValueError(f"xGMI all-reduce supports 2..8 ranks, got {self.world}")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.max_bytes = (max_bytes + 15) // 16 * 16
        self.oneshot_max = oneshot_max
        self._own: list = []  # (bytes, (ptr, handle)) taken from the pool
        self._opened: list[c_void_p] = []
        self.calls = 0
        # The probe names the ranks whose staged rows no peer saw (an export that mapped other
        # memory: seen once on an 8-rank rehearsal sharing one GPU); those ranks set their buffers
        # aside and every rank sets up again, up to twice.
        for attempt in range(3):
            self._setup(grid, timeout_ms)  # every peer mapped everywhere, or every rank raises
            if probe_ms <= 0:
                return
            res: list = [None] * self.world
            dist.all_gather_object(res, self._probe(probe_ms), group=self.group)
            if not any(e for e, _ in res):
                return
            unseen = set.intersection(*(set(m) | {r} for r, (_, m) in enumerate(res)))
            if not unseen or attempt == 2:
                self.close()
                raise RuntimeError("; ".join(f"rank {r}: {e}" for r, (e, _) in enumerate(res) if e))
            self.close(quarantine=self.rank in unseen)

    def _setup(self, grid: int, timeout_ms: int) -> None:
        err, payload = "", None
        try:
            L = _lib()
            self.grid = grid or L.da_ar_max_blocks()
            self.khz = L.da_ar_clock_khz()
            self.timeout = int(timeout_ms * self.khz)
            hb = L.da_ar_ipc_handle_bytes()
            with torch.cuda.device(self.device):
                nd, ns = 2 * self.max_bytes, L.da_ar_signal_bytes()
                data, hd = _take(L, self.device, nd, hb, "staging")
                self._own.append((nd, (data, hd)))
                sig, hs = _take(L, self.device, ns, hb, "signal")
                self._own.append((ns, (sig, hs)))
            payload = (hd, hs)
        except Exception as e:  # noqa: BLE001 - reported to every rank below
            err = f"local setup: {e}"
        allh: list = [None] * self.world
        dist.all_gather_object(allh, payload, group=self.group)
        dptr, sptr = [], []
        if not err and any(h is None for h in allh):
            err = "a peer failed its local setup"
        mapped: dict = {}

        def open_once(h: bytes, r: int) -> int:
            if h not in mapped:
                p = c_void_p()
                _ok(L.da_ar_ipc_open(ctypes.create_string_buffer(h, hb), byref(p)), f"hipIpcOpenMemHandle(rank {r})")
                self._opened.append(p)
                mapped[h] = p.value
            return mapped[h]
        if not err:
            try:
                with torch.cuda.device(self.device):
                    for r, (h_d, h_s) in enumerate(allh):
                        if r == self.rank:
                            dptr.append(data.value)
                            sptr.append(sig.value)
                            continue
                        # the peer's buffers inside the mapped allocations (staging and signal
                        # may share one: each allocation is opened once)
                        dptr.append(open_once(h_d[0], r) + h_d[1])
                        sptr.append(open_once(h_s[0], r) + h_s[1])
            except Exception as e:  # noqa: BLE001
                err = f"peer mapping: {e}"
        self._agree(err)  # every peer mapped everywhere, or every rank raises
        self._data = (c_void_p * self.world)(*dptr)
        self._sig = (c_void_p * self.world)(*sptr)
        self._sig_self = sig
        dist.barrier(group=self.group)  # every peer mapped before anyone launches

    def _agree(self, err: str) -> None:
        """All ranks exchange their error string; any error anywhere -> every rank closes and raises."""
        errs: list = [None] * self.world
        dist.all_gather_object(errs, err, group=self.group)
        # the ranks whose own setup failed first (the others only report "a peer failed ...")
        bad = sorted((f"rank {r}: {e}" for r, e in enumerate(errs) if e), key=lambda m: "a peer failed" in m)
        if bad:
            self.close()
            raise RuntimeError("; ".join(bad))

    def _probe(self, probe_ms: int) -> tuple:
        """One all-reduce of rank r's 2^r with a short bounded wait: ('', []) when the exact sum
        arrived and no barrier timed out (flags and staged rows visible across the devices), else
        (why, the ranks whose rows this rank did not see)."""
        saved = self.timeout
        self.timeout = int(probe_ms * self.khz)
        try:
            # every workgroup of the grid takes part when the staging allows (fp32: 4 per 16-B vector)
            n = max(4, min(self.grid * 256 * 4, self.max_bytes // 4) // 4 * 4)
            t = torch.full((n,), float(1 << self.rank), dtype=torch.float32, device=self.device)
            self.all_reduce_(t)
            torch.cuda.synchronize(self.device)
            want = (1 << self.world) - 1
            err = ctypes.c_uint(0)
            _ok(_lib().da_ar_read_err(self._sig_self, byref(err)), "read all-reduce error flag")
            if err.value:
                return "probe: a barrier timed out (peer flags not visible across devices)", []
            if not bool(torch.all(t == want)):
                got = t.cpu()
                seen = want
                for v in got.unique().tolist():  # sums of whole powers of two name the ranks seen
                    seen &= int(v) if float(v).is_integer() and 0 <= v <= want else 0
                missing = [r for r in range(self.world) if not (seen >> r) & 1]
                return f"probe: wrong sum (staged rows of ranks {missing} not visible)", missing
            return "", []
        except Exception as e:  # noqa: BLE001
            return f"probe: {e}", []
        finally:
            self.timeout = saved

    @classmethod
    def create(cls, group=None, device=None, **kw):
        """The communicator, or None on EVERY rank of the group (the reason logged) when peer mapping
        is unavailable or the probe fails: the caller then uses RCCL on every rank."""
        if os.environ.get("DA_XGMI_AR", "1") == "0" or not torch.cuda.is_available():
            return None
        try:
            return cls(group, device, **kw)
        except Exception as e:  # noqa: BLE001 - any setup failure means: use RCCL (symmetric, see __init__)
            import sys
            print(f"[xgmi-allreduce] disabled, using RCCL: {e}", file=sys.stderr, flush=True)
            return None

    def takes(self, t: torch.Tensor) -> bool:
        nb = t.numel() * t.element_size()
        return (t.is_cuda and t.dtype in (torch.bfloat16, torch.float32) and t.is_contiguous()
                and nb % 16 == 0 and 0 < nb <= self.max_bytes and t.data_ptr() % 16 == 0)

    def all_reduce_(self, t: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """Sum over the group (in place unless ``out`` is given). Untakeable tensors go to RCCL."""
        out = t if out is None else out
        if not self.takes(t):
            if out is not t:
                out.copy_(t)
            dist.all_reduce(out, group=self.group)
            return out
        nb = t.numel() * t.element_size()
        twoshot = 1 if nb > self.oneshot_max else 0
        rc = _lib().da_ar_allreduce(t.data_ptr(), out.data_ptr(), nb, 0 if t.dtype == torch.bfloat16 else 1,
                                    self.rank, self.world, self._data, self._sig, self.max_bytes, twoshot,
                                    self.grid, self.timeout, torch.cuda.current_stream(t.device).cuda_stream)
        _ok(rc, "xgmi all-reduce launch")
        self.calls += 1
        return out

    def takes_norm(self, x: torch.Tensor) -> bool:
        """Whether ``all_reduce_rmsnorm_`` runs the fused kernel for x [rows, D] (else: the caller
        falls back to all-reduce + rmsnorm)."""
        if x.dim() != 2:
            return False
        D = x.shape[1]
        ok = (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and D % 8 == 0 and D // 8 <= 2048
              and 0 < x.numel() * 2 <= self.max_bytes and x.data_ptr() % 16 == 0)
        return ok and getattr(self, "norm_width", D) == D

    def all_reduce_rmsnorm_(self, x: torch.Tensor, gamma, eps: float, h_out: torch.Tensor) -> torch.Tensor:
        """x [rows, D] <- sum over the group (in place); h_out <- RMSNorm(x) * gamma, one launch
        (bit-identical to all_reduce_ then the rmsnorm kernel). The fused kernel partitions by whole
        rows, so an instance serves ONE row width D (its staging parity protocol assumes a fixed
        row -> workgroup map); TPContext keeps a dedicated instance for it."""
        if not self.takes_norm(x):
            raise ValueError("all_reduce_rmsnorm_: tensor not takeable (check takes_norm)")
        self.norm_width = x.shape[1]
        if gamma is not None:
            K._bf16_cuda(gamma, "gamma")
            K._req(gamma.is_contiguous() and gamma.numel() == x.shape[1], "gamma must be [D]")
        K._req(h_out.shape == x.shape and h_out.is_contiguous() and h_out.dtype == torch.bfloat16, "bad h_out")
        rc = _lib().da_ar_allreduce_rmsnorm(x.data_ptr(), x.data_ptr(), h_out.data_ptr(),
                                            None if gamma is None else gamma.data_ptr(), x.shape[0], x.shape[1],
                                            float(eps), self.rank, self.world, self._data, self._sig, self.max_bytes,
                                            self.grid, self.timeout, torch.cuda.current_stream(x.device).cuda_stream)
        _ok(rc, "xgmi all-reduce + rmsnorm launch")
        self.calls += 1
        return h_out

    def check(self) -> None:
        """Raise if any barrier of this communicator timed out (a peer stopped participating)."""
        err = ctypes.c_uint(0)
        _ok(_lib().da_ar_read_err(self._sig_self, byref(err)), "read all-reduce error flag")
        if err.value:
            raise RuntimeError("xGMI all-reduce barrier timed out (peer missing or call sequences diverged)")

    def close(self, quarantine: bool = False):
        """Unmap the peers and return this rank's buffers to the pool (quarantine: set them aside,
        never reused — the probe found peers could not see them)."""
        if not self._own and not self._opened:
            return
        L = _lib()
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            L.da_ar_ipc_close(p)
        for nbytes, item in self._own:  # back to the pool (see _POOL)
            if quarantine:
                _REFUSED.append(item[0])
            else:
                _give(self.device, nbytes, item)
        self._opened, self._own = [], []


def _size_name(nb: int) -> str:
    return f"{nb >> 20}MB" if nb >= 1 << 20 and nb % (1 << 20) == 0 else f"{nb >> 10}KB"


def verify_and_time(group=None, device=None, iters: int = 50,
                    sizes: tuple = (16 << 10, 384 << 10, 6 << 20)) -> dict:
    """Cross-device evidence for C3 (run by bench.py on multi-GPU nodes, outside the timed steps):
    the IPC all-reduce against the exact rank-order fp32 sum for decode- and prefill-sized bf16
    messages (one-shot and two-shot), the fused all-reduce + RMSNorm against all-reduce followed by
    the rmsnorm kernel (bit identity), and the time per call at each of ``sizes`` (bytes of bf16)
    through this kernel vs RCCL ``all_reduce`` on the same group (RCCL only on the nccl backend)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    # the TP communicators' sizes (32 MB, 512 KB): the pooled buffers of an earlier TP model are
    # reused rather than a fresh buffer exported late in the process (on an 8-rank rehearsal sharing
    # one GPU a late 32 MB export mapped other memory on one rank: the probe caught it)
    ar = XgmiAllReduce(group, dev)
    res: dict = {"world": world, "ok": True, "cases": [], "export_refusals": len(_REFUSED)}
    for i, n in enumerate((64 * 3072, 1 << 20, 6 << 20)):
        xs = [torch.randn(n, generator=torch.Generator().manual_seed(7000 + 31 * i + r)).bfloat16()
              for r in range(world)]
        ref = torch.zeros(n)
        for x in xs:
            ref += x.float()
        t = xs[rank].to(dev)
        ar.all_reduce_(t)
        torch.cuda.synchronize(dev)
        err = float((t.float().cpu() - ref.bfloat16().float()).abs().max())
        res["cases"].append({"n": n, "twoshot": n * 2 > ar.oneshot_max, "max_err": err})
        res["ok"] &= err == 0.0
    # fused all-reduce + RMSNorm (its own instance: one row width per instance)
    fused = XgmiAllReduce(group, dev, max_bytes=512 << 10)
    xs = [torch.randn(64, 3072, generator=torch.Generator().manual_seed(9100 + r)).bfloat16() for r in range(world)]
    x1, x2 = xs[rank].to(dev), xs[rank].to(dev)
    h1 = torch.empty_like(x1)
    fused.all_reduce_rmsnorm_(x1, None, 1e-5, h1)
    ar.all_reduce_(x2)
    h2 = K.rmsnorm(x2, torch.ones(3072, dtype=torch.bfloat16, device=dev), 1e-5)
    torch.cuda.synchronize(dev)
    same = bool(torch.equal(x1, x2) and torch.equal(h1, h2))
    res["fused_norm_bit_identical"] = same
    res["ok"] &= same
    # time per call: this kernel vs RCCL on the same group, at the TP message sizes (16 KB: a
    # batch-1 Llama-3-70B row; 384 KB: a batch-64 Phi-3 row block, 64 x 3072; 6 MB: a two-shot
    # prefill-sized block)
    def timed(fn):
        for _ in range(5):
            fn()
        torch.cuda.synchronize(dev)
        dist.barrier(group=group)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize(dev)
        return s.elapsed_time(e) * 1000.0 / iters

    rccl = dist.get_backend(group) == "nccl"
    res["us_per_call"] = {}
    for nb in sizes:
        x = torch.randn(nb // 2, device=dev).bfloat16()
        row = {"xgmi": round(timed(lambda: ar.all_reduce_(x)), 2), "twoshot": nb > ar.oneshot_max}
        if rccl:
            row["rccl"] = round(timed(lambda: dist.all_reduce(x, group=group)), 2)
        res["us_per_call"][_size_name(nb)] = row
    res["memory"] = "uncached (hipDeviceMallocUncached) staging + signals"
    ar.check()
    fused.check()
    ar.close()
    fused.close()
    return res
