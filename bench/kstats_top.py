"""Top-N kernels of a rocprofv3 --kernel-trace --stats run: share, calls, mean us per call."""
import csv
import glob
import sys

d, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20
f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6:.2f} ms; Cijk kernels: {sum(1 for r in rows if 'Cijk' in r['Name'])}")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    c = int(r["Calls"])
    print(f'{float(r["Percentage"]):6.2f}%  {c:7d}  {float(r["TotalDurationNs"]) / c / 1e3:9.2f} us  {r["Name"][:100]}')
