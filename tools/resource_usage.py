#!/usr/bin/env python3
"""Per-kernel VGPRs / LDS / occupancy / spills of a HIP source for gfx950 (compile-time only).
   python tools/resource_usage.py mjpeg423-video-decoder-software_amd/csrc/mj423_kernels.hip [name-filter] ["-DFOO -DBAR"]"""
import re, subprocess, sys
src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
extra = sys.argv[3].split() if len(sys.argv) > 3 else []
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-c", src,
                    "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"] + extra,
                   capture_output=True, text=True, cwd="/tmp")
if r.returncode:
    sys.exit(r.stderr[-3000:])
cur, rows = None, []
for line in r.stderr.splitlines():
    m = re.search(r"remark:\s*(Function Name|VGPRs|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]|VGPRs Spill|SGPRs Spill): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for c in rows:
    if flt in c["name"]:
        print(f"{c['name'][:72]:72s} v{c.get('VGPRs')} lds{c.get('LDS Size [bytes/block]')} "
              f"occ{c.get('Occupancy [waves/SIMD]')} spill{c.get('VGPRs Spill')}/{c.get('SGPRs Spill')}")
