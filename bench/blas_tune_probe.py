"""Probe: hipBLASLt default heuristic vs PyTorch TunableOp (exhaustive hipBLASLt/rocBLAS solution
search) on the prefill GEMM shapes of the flagship (Phi-3-mini, packed chunks of ~32k tokens).
Prints one JSON line per shape; writes the tuned table to gpurun_out/tunableop_probe.csv."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [("qkv", 9216, 3072, "mm"), ("o", 3072, 3072, "addmm_"), ("gu", 16384, 3072, "mm"),
          ("down", 3072, 8192, "addmm_")]


def timed(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def main():
    Ms = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "32768").split(",")]
    import torch.cuda.tunable as tn
    os.makedirs("gpurun_out", exist_ok=True)
    tn.set_filename("gpurun_out/tunableop_probe.csv")
    tn.set_max_tuning_duration(400)
    tn.set_max_tuning_iterations(60)
    for M in Ms:
        for name, N, K, op in SHAPES:
            a = torch.randn(M, K, device="cuda").bfloat16()
            w = (torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16()
            out = torch.randn(M, N, device="cuda").bfloat16()
            fn = (lambda: torch.mm(a, w.t(), out=out)) if op == "mm" else (lambda: out.addmm_(a, w.t()))
            tn.enable(False)
            t_def = timed(fn)
            tn.enable(True)
            tn.tuning_enable(True)
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            t_tune = time.perf_counter() - t0
            tn.tuning_enable(False)
            t_tuned = timed(fn)
            tn.enable(False)
            fl = 2.0 * M * N * K
            print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "op": op, "default_ms": round(t_def, 4),
                              "tuned_ms": round(t_tuned, 4), "default_PF": round(fl / t_def / 1e12, 3),
                              "tuned_PF": round(fl / t_tuned / 1e12, 3), "tune_s": round(t_tune, 1)}), flush=True)
    tn.write_file()


if __name__ == "__main__":
    main()
