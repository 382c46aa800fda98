#!/usr/bin/env python3
"""Per-kernel counters of the whole-file GPU decode (tools/fe_pmc.sh output), per pass.

Pass 1 (SQ): waves, VALU / SALU / LDS instructions per wave, wave cycles per wave, the fraction
of a wave's cycles it issued VALU (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES; x waves per SIMD = the
SIMD's VALU occupancy) and waited on an instruction dependency (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES).
Passes 2 and 3: FETCH_SIZE and WRITE_SIZE (KiB per pass).  FETCH_SIZE is printed raw and, for
the kernels whose reads are 16-B/lane streaming reads (copy/fill), x2 per MI355X_MICROARCH.md
§HBM; the walks' and the fused kernel's narrow reads are not calibrated (raw is a lower bound).

  python tools/pmc_file_summary.py DIR PASSES [--json OUT]
"""
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


if __name__ == "__main__":
    main()
