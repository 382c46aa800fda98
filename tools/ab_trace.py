"""Per-build kernel time of a rocprofv3 kernel trace of tools/ab_file.py (every build runs 5
passes in turn, warm-up included): pass p belongs to build (p // 5) % NBUILDS.  Passes are told
apart by their windows' entpar_map_kernel launches (WINDOWS per pass).  Prints, per build, the
median per-pass time of every kernel and the median span from a pass's first map launch to its
last kernel's end.

  python tools/ab_trace.py TRACE_CSV NBUILDS [WINDOWS]
"""
import collections
import csv
import statistics
import sys

path, nb = sys.argv[1], int(sys.argv[2])
nwin = int(sys.argv[3]) if len(sys.argv) > 3 else 3
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
per = collections.defaultdict(lambda: collections.defaultdict(float))  # pass -> kernel -> ms
span = {}
nmap = -1
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mj423::", "").strip() or "mpg_fused_kernel"
    if "entpar_map_kernel" in name:
        nmap += 1
    if nmap < 0:
        continue
    p = nmap // nwin
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    per[p][name[:40]] += (e - s) / 1e6
    if "entpar_map_kernel" in name and nmap % nwin == 0:
        span[p] = [s, e]
    span[p][1] = max(span[p][1], e)
builds = collections.defaultdict(list)
for p in per:
    builds[(p // 5) % nb].append(p)
names = sorted({k for p in per for k in per[p]}, key=lambda k: -per[0].get(k, 0))
print(f"{'kernel':40s} " + " ".join(f"{'b' + str(b):>8s}" for b in range(nb)))
for k in names:
    print(f"{k:40s} " + " ".join(f"{statistics.median(per[p].get(k, 0) for p in builds[b]):8.4f}" for b in range(nb)))
print(f"{'span first map -> last end (ms)':40s} " +
      " ".join(f"{statistics.median((span[p][1] - span[p][0]) / 1e6 for p in builds[b]):8.4f}" for b in range(nb)))
