"""Mean per-dispatch PMC counters (millions) of the GEMM kernels in gpurun_out/<dir>/p*/ (scripts/gpu_pmc.sh)."""
import csv, glob, sys
for arm in sys.argv[1:]:
    tot = {}
    for f in glob.glob(f"gpurun_out/{arm}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "gemm8p" not in r.get("Kernel_Name", "") and "Cijk" not in r.get("Kernel_Name", ""):
                continue
            tot.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(arm, {k: round(sum(v) / len(v) / 1e6, 2) for k, v in sorted(tot.items())})
