"""Timeline of one whole-file GPU pass from a rocprofv3 kernel + memory-copy trace of
bench.py --mode file --frontend gpu (tools/file_trace.sh): per stream, the kernels and copies of
pass PASS with start/end relative to the pass's first upload (measurement only).
  python tools/pass_timeline.py TRACE_DIR [PASS]"""
import csv
import sys


def main():
    d = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    ks = list(csv.DictReader(open(f"{d}/kt_kernel_trace.csv")))
    ms = list(csv.DictReader(open(f"{d}/kt_memory_copy_trace.csv")))
    ev = []
    for r in ks:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mj423::", "")
        name = name.replace("(anonymous namespace)::", "").split("<")[0]
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "q" + r["Queue_Id"], name))
    for r in ms:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy", r["Direction"]))
    ev.sort()
    # a pass ends with the status read-back (a D2H copy on the context's queue: __amd_rocclr_copyBuffer
    # or a memory-copy record); the next one starts after it
    ends = [e[1] for e in ev if "copyBuffer" in e[3] or ("DEVICE_TO_HOST" in e[3])]
    passes = [min(e[0] for e in ev)] + ends[:-1]
    t0 = passes[k]
    t1 = passes[k + 1] if k + 1 < len(passes) else float("inf")
    print(f"{len(passes)} passes; pass {k}: {(t1 - t0) / 1e6:.3f} ms from the previous pass's status read-back to its own")
    for s, e, q, n in ev:
        if t0 <= s <= t1:
            print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {q:8s} {n}")


if __name__ == "__main__":
    main()
