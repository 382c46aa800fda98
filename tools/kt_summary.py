"""Per-pass kernel time of a rocprofv3 kernel trace of bench.py --mode file (tools/fe_trace_ab.sh):
per kernel, total time / passes, and the synchronisation iterations' per-window durations.
  python tools/kt_summary.py DIR PASSES [WINDOWS [ITERS]]   (ITERS: synchronisation launches per window, 10)"""
import collections
import csv
import statistics
import sys

d, passes = sys.argv[1], int(sys.argv[2])
nwin = int(sys.argv[3]) if len(sys.argv) > 3 else 3
niter = int(sys.argv[4]) if len(sys.argv) > 4 else 10
rows = list(csv.DictReader(open(f"{d}/kt_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tot = collections.defaultdict(float)
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mj423::", "").replace("(anonymous namespace)::", "")
    tot[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"{k[:60]:60s} {v / passes:8.4f} ms/pass")
print(f"{'all kernels':60s} {sum(tot.values()) / passes:8.4f} ms/pass")
seq = [r for r in rows if "entpar_sync" in r["Kernel_Name"]]
durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in seq]
per = collections.defaultdict(list)
for wi in range(len(durs) // niter):
    for it in range(niter):
        per[(wi % nwin, it)].append(durs[wi * niter + it])
for w in range(nwin):
    print("sync win", w, " ".join(f"{statistics.median(per[(w, it)]):6.1f}" for it in range(niter)), "us")
