"""Timeline of one QA step from a rocprofv3 --kernel-trace CSV (bench.py --steps 1 --warmup 1):
finds the last window of big prefill GEMMs (gemm8p EPI_ROPE launches of > 500 us), extends it to the
decode that follows, and prints kernel time by name, the sum of inter-kernel gaps, and the largest
gaps with their neighbours. usage: trace_window.py kernel_trace.csv[.gz]"""
import csv, gzip, sys, collections

f = sys.argv[1]
op = gzip.open if f.endswith(".gz") else open
rows = list(csv.DictReader(op(f, "rt")))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
big = [i for i, (s, e, n) in enumerate(ks) if "gemm8p_kernel<6" in n and e - s > 500_000]
# runs of big ROPE GEMMs whose neighbours are < 50 ms apart; the QA step is the last run with the
# most launches (3 prefill chunks x layers; an ingest summarize call prefills one chunk)
runs, cur = [], [big[0]]
for a, b in zip(big, big[1:]):
    if ks[b][0] - ks[a][0] < 50_000_000:
        cur.append(b)
    else:
        runs.append(cur)
        cur = [b]
runs.append(cur)
mx = max(len(r) for r in runs)
run = [r for r in runs if len(r) == mx][-1]
print("big-GEMM runs:", [len(r) for r in runs])
first = run[0]
# step end: the first gap > 20 ms after the last big GEMM (host work between bench phases)
i = run[-1]
while i + 1 < len(ks) and ks[i + 1][0] - ks[i][1] < 20_000_000:
    i += 1
win = ks[first - 3:i + 1]
t0, t1 = win[0][0], win[-1][1]
print(f"window {len(win)} kernels, {(t1 - t0) / 1e6:.1f} ms")
busy = collections.Counter()
calls = collections.Counter()
for s, e, n in win:
    busy[n[:80]] += e - s
    calls[n[:80]] += 1
tot = sum(busy.values())
print(f"kernel busy {tot / 1e6:.1f} ms")
for n, t in busy.most_common(25):
    print(f"{t / 1e6:9.2f} ms {calls[n]:6d}  {n}")
gaps = [(win[k + 1][0] - win[k][1], k) for k in range(len(win) - 1)]
print(f"sum of gaps {sum(g for g, _ in gaps if g > 0) / 1e6:.1f} ms; overlap {-sum(g for g, _ in gaps if g < 0) / 1e6:.1f} ms")
# split the window at the last big-prefill kernel: prefill part vs decode part
last_pf = max(k for k, (s, e, n) in enumerate(win) if "gemm8p" in n or "flash" in n)
for name, part in (("prefill", win[:last_pf + 1]), ("decode", win[last_pf + 1:])):
    if not part:
        continue
    span = part[-1][1] - part[0][0]
    b = sum(e - s for s, e, n in part)
    print(f"{name}: span {span / 1e6:.1f} ms, kernels {b / 1e6:.1f} ms, n={len(part)}")
for g, k in sorted(gaps, reverse=True)[:15]:
    print(f"gap {g / 1e3:9.1f} us after {win[k][2][:60]} -> {win[k + 1][2][:60]}")
