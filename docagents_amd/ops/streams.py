"""CU-masked HIP streams: spatial partitioning of one MI355X (``hipExtStreamCreateWithCUMask``,
csrc/runtime.hip).

Two uses were measured:
* co-running the MFMA-bound prefill of one wave with the HBM-bound decode of the previous one on
  complementary CU sets (bench/cumask_probe.py, profiles/r3/cumask_probe.jsonl): NOT kept — decode
  attention on a quarter of the CUs runs at half speed (its per-CU memory parallelism, not HBM,
  limits it), and the co-run was never faster than running the two back to back;
* isolating the serving latency lanes (query embeds, search plane) on a few CUs from the
  throughput lane (decode replays, admission prefills): ``serving_lanes``.
Masks are chosen in groups of eight consecutive CU bits, spread evenly over the mask; the
placement probe shows a lane's CUs spread over all eight XCDs (8 of 32 per XCD at a quarter).
"""
from __future__ import annotations

import ctypes

import torch

from . import kernels as K

_STREAMS: dict = {}


def cu_count(device=None) -> int:
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    n = ctypes.c_int(0)
    K._check(K.lib().da_device_cu_count(dev.index or 0, ctypes.byref(n)), "hipDeviceGetAttribute")
    return int(n.value)


def split_groups(n_cus: int, frac: float, group: int = 8) -> tuple[list[int], list[int]]:
    """Split the CU bits into (lane A, lane B) in whole groups of ``group`` consecutive bits:
    lane A gets round(frac * groups) groups spread evenly (Bresenham) over the mask, lane B the
    rest. Both lanes are non-empty when 0 < frac < 1."""
    ng = n_cus // group
    na = min(ng - 1, max(1, round(frac * ng))) if 0.0 < frac < 1.0 else (ng if frac >= 1.0 else 0)
    a_groups = sorted({(i * ng) // na for i in range(na)}) if na else []
    a_bits = [g * group + j for g in a_groups for j in range(group)]
    b_bits = [i for i in range(ng * group) if i not in set(a_bits)]
    return a_bits, b_bits


def mask_words(bits: list[int], n_cus: int) -> list[int]:
    words = [0] * ((n_cus + 31) // 32)
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    return words


def masked_stream(bits: list[int], device=None, tag: str = "") -> torch.cuda.ExternalStream:
    """A stream restricted to the CU bits ``bits`` (cached per (device, bits, tag); never destroyed:
    captured graphs and pending work may still reference it). Different tags give distinct streams
    (hardware queues) on the same CUs."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    key = (dev.index or 0, tuple(sorted(bits)), tag)
    s = _STREAMS.get(key)
    if s is not None:
        return s
    n = cu_count(dev)
    if not bits or max(bits) >= n:
        raise ValueError(f"CU mask bits must be a non-empty subset of 0..{n - 1}")
    words = mask_words(bits, n)
    K.MASKED_STREAMS = True  # no same-XCD decode exchange from now on (kernels.decode_xc_ok)
    arr = (ctypes.c_uint * len(words))(*words)
    p = ctypes.c_void_p()
    with torch.cuda.device(dev):
        K._check(K.lib().da_stream_create_cumask(len(words), arr, ctypes.byref(p)), "hipExtStreamCreateWithCUMask")
    s = torch.cuda.ExternalStream(p.value, device=dev)
    _STREAMS[key] = s
    return s


def lane_streams(frac_a: float, device=None) -> tuple[torch.cuda.ExternalStream, torch.cuda.ExternalStream]:
    """Two complementary CU-masked streams: lane A on ~frac_a of the CUs, lane B on the rest."""
    n = cu_count(device)
    a, b = split_groups(n, frac_a)
    return masked_stream(a, device), masked_stream(b, device)


def serving_lanes(latency_cus: int, device=None):
    """Spatial partition of one GPU for serving: ``latency_cus`` CUs (rounded to groups of 8) for
    the latency lanes — the fast embed lane and the search plane, one stream each — and the rest for
    the GPU thread's decode replays and admission prefills. Big prefill GEMMs occupy every CU they
    can reach for milliseconds; a question's ~100-kernel encoder chain queued behind them on the
    same CUs waits for each kernel's slot (measured: 218 ms per query embed at 128 requests in
    flight). Returns (main, fast, search) streams, or (None, None, None) when latency_cus <= 0."""
    if latency_cus <= 0:
        return None, None, None
    n = cu_count(device)
    a, b = split_groups(n, latency_cus / n)
    return (masked_stream(b, device, "main"), masked_stream(a, device, "fast"), masked_stream(a, device, "search"))


def probe_placement(stream, blocks: int = 512, spin: int = 20000) -> list[tuple[int, int, int, int]]:
    """Run the placement kernel on ``stream``: [(xcc, se, cu, simd-independent hw id)] per workgroup."""
    dev = torch.device("cuda", torch.cuda.current_device())
    out = torch.zeros(blocks * 4, dtype=torch.int32, device=dev)
    with torch.cuda.stream(stream):
        K._check(K.lib().da_placement_probe(ctypes.c_void_p(out.data_ptr()), blocks, spin,
                                            ctypes.c_void_p(stream.cuda_stream)), "placement_probe")
    stream.synchronize()
    r = out.view(blocks, 4).cpu().numpy().astype("int64") & 0xffffffff
    res = []
    for xcc, hw, _, _ in r:
        cu = (hw >> 8) & 0xF
        sh = (hw >> 12) & 0x1
        se = (hw >> 13) & 0x7
        res.append((int(xcc), int(se), int(sh), int(cu)))
    return res
