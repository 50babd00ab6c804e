"""CPU model of the xGMI IPC all-reduce protocol (ops/csrc/allreduce.hip) with one
thread per (rank, workgroup) and genuinely separate per-rank staging buffers and signal blocks — so
it does not lean on the same-device aliasing of the 2-ranks-on-1-GPU GPU test.

Mirrors the kernel step for step: per-workgroup call counter k, staging half chosen by k's parity,
flag barriers with values 2k+1 / 2k+2 (store own value into every peer's flag slot, wait for every
peer's value in the own slot), one-shot (stage -> barrier -> rank-order sum) and two-shot (stage ->
barrier -> reduce own slice in place -> barrier -> gather), and the work partition taken from the
library itself (``da_ar_plan``: rows of 256 vectors, row r on workgroup r % grid, shortened grids for
short messages). Checked over several back-to-back calls of mixed sizes under adversarial delays
(a slow reader rank), plus a negative control: without the parity alternation the same schedule
corrupts a result — the hazard the double buffer exists for."""
import ctypes
import threading
import time

import numpy as np
import pytest

from docagents_amd.ops.build import LIB

TPB = 256


def _plan():
    if not LIB.exists():
        pytest.skip("kernel library not built")
    L = ctypes.CDLL(str(LIB))
    L.da_ar_plan.argtypes = [ctypes.c_longlong, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.POINTER(ctypes.c_longlong)]
    L.da_ar_plan.restype = ctypes.c_int

    def plan(nbytes, world, grid, twoshot):
        o = (ctypes.c_longlong * 4)()
        assert L.da_ar_plan(nbytes, world, grid, twoshot, o) == 0
        return int(o[0]), int(o[1]), int(o[2]), int(o[3])
    return plan


class Model:
    """W ranks x G workgroups; a 'vector' is one float64 (stands for a 16-B vector)."""

    def __init__(self, world, grid, max_vec, parity=True, slow_rank=None, delay=0.0):
        self.W, self.G, self.max_vec = world, grid, max_vec
        self.parity = parity
        self.staging = [np.zeros(2 * max_vec) for _ in range(world)]      # per-rank IPC buffer
        self.flags = [np.zeros((grid, world), dtype=np.int64) for _ in range(world)]
        self.cnt = [np.zeros(grid, dtype=np.int64) for _ in range(world)]
        self.cv = threading.Condition()
        self.slow_rank, self.delay = slow_rank, delay

    def barrier(self, rank, b, val):
        with self.cv:
            for w in range(self.W):
                self.flags[w][b, rank] = val  # release store into every peer's signal block
            self.cv.notify_all()
            ok = self.cv.wait_for(lambda: all(self.flags[rank][b, w] >= val for w in range(self.W)), timeout=20)
        assert ok, "barrier timed out"

    def workgroup(self, rank, b, inp, out, nvec, rows, slc, G, twoshot):
        k = int(self.cnt[rank][b])
        poff = self.max_vec if (self.parity and k & 1) else 0
        mine = self.staging[rank]
        for r in range(b, rows, G):  # phase 1: stage
            lo, hi = r * TPB, min(nvec, (r + 1) * TPB)
            mine[poff + lo:poff + hi] = inp[lo:hi]
        self.barrier(rank, b, 2 * k + 1)
        slow = rank == self.slow_rank

        def rank_sum(lo, hi):
            acc = np.zeros(hi - lo)
            for w in range(self.W):  # rank order, like the kernel
                if slow:
                    time.sleep(self.delay)
                acc += self.staging[w][poff + lo:poff + hi]
            return acc
        if not twoshot:
            for r in range(b, rows, G):
                lo, hi = r * TPB, min(nvec, (r + 1) * TPB)
                out[lo:hi] = rank_sum(lo, hi)
        else:
            s_lo, s_hi = rank * slc, min(nvec, rank * slc + slc)
            for r in range(b, rows, G):  # phase 2: reduce own slice in place
                lo, hi = max(r * TPB, s_lo), min(nvec, (r + 1) * TPB, s_hi)
                if lo < hi:
                    mine[poff + lo:poff + hi] = rank_sum(lo, hi)
            self.barrier(rank, b, 2 * k + 2)
            for r in range(b, rows, G):  # phase 3: gather every slice
                for v in range(r * TPB, min(nvec, (r + 1) * TPB)):
                    out[v] = self.staging[v // slc][poff + v]
        self.cnt[rank][b] = k + 1


def _run_calls(plan, world, grid, sizes, parity=True, slow_rank=None, delay=0.0, seed=0):
    """Back-to-back calls: each rank starts its next call as soon as ITS workgroups finished the
    previous one (as in a stream), so fast ranks run ahead into the next call's staging."""
    rng = np.random.default_rng(seed)
    m = Model(world, grid, max(n for n, _ in sizes), parity, slow_rank, delay)
    inputs = [[np.round(rng.standard_normal(n), 3) for _ in range(world)] for n, _ in sizes]
    results = [[None] * world for _ in sizes]

    def rank_stream(r):
        for c, (n, twoshot) in enumerate(sizes):
            nvec, rows, slc, G = plan(16 * n, world, grid, twoshot)
            out = np.full(nvec, np.nan)
            th = [threading.Thread(target=m.workgroup, args=(r, b, inputs[c][r], out, nvec, rows, slc, G, twoshot))
                  for b in range(G)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            results[c][r] = out
    streams = [threading.Thread(target=rank_stream, args=(r,)) for r in range(world)]
    for t in streams:
        t.start()
    for t in streams:
        t.join(60)
    bad = 0
    for c, (n, _) in enumerate(sizes):
        want = np.zeros(n)
        for r in range(world):
            want += inputs[c][r]
        for r in range(world):
            if results[c][r] is None or not np.array_equal(results[c][r], want):
                bad += 1
    return bad, m


@pytest.mark.parametrize("world", [2, 4, 8])
def test_protocol_back_to_back_calls_with_slow_reader(world):
    plan = _plan()
    # mixed sizes: one-shot, two-shot, a message shorter than the grid (shortened launch), repeated
    sizes = [(3000, 0), (5000, 1), (300, 0), (4096, 1), (2500, 0), (700, 1), (3000, 0)]
    bad, m = _run_calls(plan, world, grid=4, sizes=sizes, slow_rank=world - 1, delay=0.0005)
    assert bad == 0
    # every launched workgroup advanced its counter once per call it took part in; all ranks agree
    assert all(np.array_equal(m.cnt[0], m.cnt[r]) for r in range(world))
    assert int(m.cnt[0][0]) == len(sizes)


def test_double_buffer_parity_is_what_makes_it_safe():
    """Negative control: the same schedule with the parity alternation disabled lets a fast rank
    stage call k+1 over data a slow peer is still summing for call k."""
    plan = _plan()
    sizes = [(2048, 0), (2048, 0), (2048, 0), (2048, 0)]
    bad_ok, _ = _run_calls(plan, 2, grid=2, sizes=sizes, slow_rank=1, delay=0.002)
    bad_noparity, _ = _run_calls(plan, 2, grid=2, sizes=sizes, parity=False, slow_rank=1, delay=0.002)
    assert bad_ok == 0
    assert bad_noparity > 0
