"""Mean per-dispatch PMC counters (millions) of the kernels whose name contains FILTER (default: the
GEMMs) in gpurun_out/<dir>/p*/ (scripts/gpu_pmc.sh). usage: [FILTER=substr] pmc_summary.py dir..."""
import csv, glob, os, sys
filt = os.environ.get("FILTER", "")
for arm in sys.argv[1:]:
    tot = {}
    for f in glob.glob(f"gpurun_out/{arm}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if (filt and filt not in name) or (not filt and "gemm8p" not in name and "Cijk" not in name):
                continue
            tot.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(arm, {k: round(sum(v) / len(v) / 1e6, 2) for k, v in sorted(tot.items())})
