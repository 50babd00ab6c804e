"""Performance lint on the gfx950 ISA of the hot kernels (CPU: hipcc cross-compiles to assembly with
the production flags). Two regressions that cost real time on the MI355X and that no numerics test
sees:
  * register spills (scratch) — the 8-wave batch-1 decode attention that measured 2x slower spilled
    312 B per lane (profiles/r4/rejected_r4.txt 3);
  * loops that wait for each of their loads before the next — the split-K reduces' deferred-norm and
    split sums ran one memory round trip per term (profiles/r4/rejected_r4.txt 7).
"""
import os
import re
import shutil
import subprocess

import pytest

from docagents_amd.ops import build as B

HOT_NO_SCRATCH = {  # mangled-name prefixes of the kernels the flagship bench runs
    "attention.hip": ["_Z18decode_attn_kernelILi96ELi1ELi3EE", "_Z18decode_attn_kernelILi96ELi1ELi7EE",
                      "_Z18decode_attn_kernelILi96ELi1ELi15EE", "_Z24decode_attn_mfma1_kernelILi96E",
                      "_Z22flash_attn_pipe_kernelILi96ELb1ELb1EE",
                      "_Z20flash_attn_v2_kernelILi64ELi4ELi1E", "_Z20flash_attn_v2_kernelILi128ELi8ELi1E"],
    "gemm.hip": ["_Z11gemv_kernel", "_Z16gemm_bf16_kernelILi64ELi128ELi1ELi4ELi5ELi4EE",
                 "_Z16gemm_bf16_kernelILi32ELi128ELi1ELi4ELi5ELi4EE",
                 "_Z16gemm_bf16_kernelILi128ELi64ELi2ELi2ELi5ELi4EE",  # 65..128-row decode (O / down)
                 "_Z18gemm_splitk_reduce", "_Z23splitk_reduce_resid_ssq"],
    "gemm8p.hip": ["_Z13gemm8p_kernelILi6ELi256E", "_Z13gemm8p_kernelILi3ELi256E", "_Z13gemm8p_kernelILi4ELi256E"],
    "gemm_dk.hip": ["_Z14gemm_dk_kernel"],
    "vecsearch.hip": ["_Z24topk_dense_stream_kernel", "_Z20topk_dense_mq_kernel"],  # the shard scans
}
NO_SERIAL_LOAD_LOOPS = {"gemm.hip": ["_Z18gemm_splitk_reduce", "_Z23splitk_reduce_resid_ssq",
                                     "_Z27splitk_reduce_resid_rmsnorm"],
                        "gemm_dk.hip": ["_Z14gemm_dk_kernel"],  # the deferred-norm sums
                        "norm.hip": ["_Z12embed_kernel"]}       # the decode step's first launch


def _asm(name, tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    out = tmp_path / (name + ".s")
    r = subprocess.run([hipcc, *B._flags(False), "--cuda-device-only", "-S", str(B.CSRC / name), "-o", str(out)],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    return out.read_text()


def _kernels(asm):
    """{mangled name: (body text, scratch bytes)} of every kernel in the assembly."""
    meta = {m.group(1): int(m.group(2)) for m in re.finditer(
        r"\.name:\s+(\S+)\n(?:(?!\.name:).)*?\.private_segment_fixed_size:\s+(\d+)", asm, re.S)}
    out = {}
    for m in re.finditer(r"^(_Z\S+):\s*(?:;.*)?$", asm, re.M):
        end = asm.find(".Lfunc_end", m.start())
        out[m.group(1)] = (asm[m.start():end], meta.get(m.group(1), 0))
    return out


def _serial_load_loops(body):
    """Self-looping blocks (the block branches back to its own label) whose one or two global loads
    are waited for (vmcnt(0)) before the next iteration: one memory round trip per iteration."""
    bad = []
    for blk in re.split(r"\n(?=\.LBB\S*:)", body):
        label = blk.split(":", 1)[0].strip()
        lines = [ln.strip() for ln in blk.split("\n")[1:] if ln.strip() and not ln.strip().startswith(";")]
        if not label.startswith(".LBB") or not any(ln.startswith("s_cbranch") and ln.endswith(label) for ln in lines):
            continue
        loads = [ln for ln in lines if ln.startswith("global_load")]
        if 1 <= len(loads) <= 2 and any(ln.startswith("s_waitcnt") and "vmcnt(0)" in ln for ln in lines):
            bad.append(label)
    return bad


@pytest.mark.parametrize("src", sorted(set(HOT_NO_SCRATCH) | set(NO_SERIAL_LOAD_LOOPS)))
def test_hot_kernels_isa(src, tmp_path):
    ks = _kernels(_asm(src, tmp_path))
    for pre in HOT_NO_SCRATCH.get(src, []):
        hits = {n: sc for n, (_, sc) in ks.items() if n.startswith(pre)}
        assert hits, f"{src}: no kernel {pre}* (renamed? update the lint)"
        spilled = {n: sc for n, sc in hits.items() if sc > 0}
        assert not spilled, f"{src}: scratch in hot kernels {spilled}"
    for pre in NO_SERIAL_LOAD_LOOPS.get(src, []):
        hits = {n: body for n, (body, _) in ks.items() if n.startswith(pre)}
        assert hits, f"{src}: no kernel {pre}*"
        for n, body in hits.items():
            assert not _serial_load_loops(body), f"{n}: a loop waits for each load before the next"


def test_serial_load_detector_catches_the_round_trip_loop():
    """The detector flags the shape the split-K reduce's deferred-norm sum compiled to before the fix
    (one load, wait, add, branch back) and passes the fixed shape (all loads, then counted waits)."""
    serial = (".LBB0_10:                               ;   Parent Loop BB0_5 Depth=1\n"
              "\tglobal_load_dword v4, v[4:5], off\n\ts_waitcnt vmcnt(0)\n\tv_add_f32_e32 v3, v3, v4\n"
              "\ts_cbranch_scc0 .LBB0_10\n")
    batched = (".LBB0_10:                               ;   Parent Loop BB0_5 Depth=1\n"
               + "".join(f"\tglobal_load_dword v{4 + i}, v[20:21], off offset:{256 * i}\n" for i in range(8))
               + "".join(f"\ts_waitcnt vmcnt({7 - i})\n\tv_add_f32_e32 v3, v3, v{4 + i}\n" for i in range(8))
               + "\ts_cbranch_scc1 .LBB0_10\n")
    assert _serial_load_loops("_Zk:\n" + serial) == [".LBB0_10"]
    assert _serial_load_loops("_Zk:\n" + batched) == []
