#!/usr/bin/env python3
"""Per-kernel counters of the whole-file GPU decode (tools/fe_pmc.sh output), per pass.

Pass 1 (SQ): waves, VALU / SALU / LDS instructions per wave, wave cycles per wave, the fraction
of a wave's cycles it issued VALU (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES; x waves per SIMD = the
SIMD's VALU occupancy) and waited on an instruction dependency (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES).
Passes 2 and 3: FETCH_SIZE and WRITE_SIZE (KiB per pass).  FETCH_SIZE is printed raw and, for
the kernels whose reads are 16-B/lane streaming reads (copy/fill), x2 per MI355X_MICROARCH.md
§HBM; the walks' and the fused kernel's narrow reads are not calibrated (raw is a lower bound).

  python tools/pmc_file_summary.py DIR PASSES [--json OUT]
      [--traffic-entry KEY --algo-bytes-per-pass N --launches-per-pass L]

--traffic-entry: also write the fused kernel's HBM bytes per launch (raw FETCH_SIZE + WRITE_SIZE,
KiB x 1024, per pass / launches per pass) into profiles/pmc_traffic.json under KEY, stamped with
the digest of mj423.FUSED_SOURCES, the commit and the date (bench.py --mode file reads it).  Its
reads are narrow (dwords of the bitstreams, 2-B lengths, 8-B tile entries, 16-B state rows): no x2
correction; the raw count already covers the known read bytes (bitstreams + index).
"""
import datetime
import os
import subprocess
import collections
import csv
import json
import sys


def load(path):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))  # kernel -> counter -> sum
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mj423::", "").strip() or "mpg_fused_kernel"
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return acc, disp


def main():
    d, passes = sys.argv[1], int(sys.argv[2])
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    sq, disp = load(f"{d}/p1/p_counter_collection.csv")
    fe, _ = load(f"{d}/p2/p_counter_collection.csv")
    wr, _ = load(f"{d}/p3/p_counter_collection.csv")
    rows = {}
    for k in sorted(sq, key=lambda k: -sq[k].get("SQ_WAVE_CYCLES", 0)):
        c = sq[k]
        waves = c.get("SQ_WAVES", 0)
        if waves == 0:
            continue
        cyc = c.get("SQ_WAVE_CYCLES", 0)
        rows[k] = {
            "dispatches_per_pass": round(len(disp[k]) / passes, 2),
            "waves_per_pass": round(waves / passes),
            "valu_per_wave": round(c.get("SQ_INSTS_VALU", 0) / waves),
            "salu_per_wave": round(c.get("SQ_INSTS_SALU", 0) / waves),
            "lds_per_wave": round(c.get("SQ_INSTS_LDS", 0) / waves),
            "wave_cycles_per_wave": round(cyc / waves),
            "active_valu_frac": round(c.get("SQ_ACTIVE_INST_VALU", 0) / cyc, 3) if cyc else None,
            "wait_inst_frac": round(c.get("SQ_WAIT_INST_ANY", 0) / cyc, 3) if cyc else None,
            "fetch_kib_per_pass_raw": round(fe.get(k, {}).get("FETCH_SIZE", 0) / passes),
            "write_kib_per_pass": round(wr.get(k, {}).get("WRITE_SIZE", 0) / passes),
        }
    hdr = ("kernel", "disp", "waves", "valu/w", "salu/w", "lds/w", "cyc/w", "actVALU", "waitI", "fetchKiB", "writeKiB")
    print("%-34s %5s %8s %7s %7s %6s %8s %7s %6s %10s %10s" % hdr)
    for k, r in rows.items():
        print("%-34s %5s %8d %7d %7d %6d %8d %7.3f %6.3f %10d %10d" % (
            k[:34], r["dispatches_per_pass"], r["waves_per_pass"], r["valu_per_wave"], r["salu_per_wave"],
            r["lds_per_wave"], r["wave_cycles_per_wave"], r["active_valu_frac"] or 0, r["wait_inst_frac"] or 0,
            r["fetch_kib_per_pass_raw"], r["write_kib_per_pass"]))
    tf = sum(r["fetch_kib_per_pass_raw"] for r in rows.values())
    tw = sum(r["write_kib_per_pass"] for r in rows.values())
    print(f"all kernels: FETCH_SIZE raw {tf} KiB/pass, WRITE_SIZE {tw} KiB/pass")
    if out:
        json.dump({"passes": passes, "kernels": rows, "fetch_kib_per_pass_raw": tf, "write_kib_per_pass": tw},
                  open(out, "w"), indent=1)
    if "--traffic-entry" in sys.argv:
        arg = lambda k: sys.argv[sys.argv.index(k) + 1]  # noqa: E731
        key, algo, lpp = arg("--traffic-entry"), int(arg("--algo-bytes-per-pass")), int(arg("--launches-per-pass"))
        repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, os.path.join(repo, "mjpeg423-video-decoder-software_amd"))
        import mj423
        r = rows["mpg_fused_kernel"]
        rd, wr_b = r["fetch_kib_per_pass_raw"] * 1024.0 / lpp, r["write_kib_per_pass"] * 1024.0 / lpp
        commit = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True,
                                cwd=repo).stdout.strip()
        path = os.path.join(repo, "profiles", "pmc_traffic.json")
        allt = json.load(open(path))
        allt[key] = {"kernel": "mpg_fused_kernel", "kernel_src_digest": mj423.kernel_source_digest(mj423.FUSED_SOURCES),
                     "git_commit": commit, "date": datetime.date.today().isoformat(),
                     "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr_b,
                     "hbm_bytes_per_launch": rd + wr_b, "algorithmic_bytes_per_launch": algo / lpp,
                     "traffic_over_algorithmic": (rd + wr_b) / (algo / lpp),
                     "correction": "none: narrow reads, raw FETCH_SIZE; WRITE_SIZE exact (16-B stores); KiB x1024; "
                                   "separate --pmc passes (tools/fe_pmc.sh)",
                     "source": d}
        json.dump(allt, open(path, "w"), indent=1, sort_keys=True)
        print(f"{key}: {rd + wr_b:.0f} B per launch = {(rd + wr_b) / (algo / lpp):.4f} x algorithmic")


if __name__ == "__main__":
    main()
