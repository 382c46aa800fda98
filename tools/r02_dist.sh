#!/bin/bash
# GPU box: the same bench lines in eight separate processes (eight buffer placements):
# C3 batch, C3 stream, C2 stream, 640x480 4:4:4 stream.
export TMPDIR=/tmp
O=gpurun_out/r02dist; mkdir -p $O
rocm-smi --showserial 2>/dev/null | grep -i "serial number" | head -1
for i in 1 2 3 4 5 6 7 8; do
  for m in "c3:--config c3" "c3s:--config c3 --mode stream" "c2s:--config c2 --mode stream" "c1s:--config c1 --mode stream"; do
    n=${m%%:*}; args=${m#*:}
    timeout -k 10 200 python bench.py $args --steps 20 --no-cpu --verify ends > $O/${n}_$i.json 2> $O/${n}_$i.err || { tail -5 $O/${n}_$i.err; exit 1; }
  done
  python - "$O" "$i" <<'PY'
import json, sys
o, i = sys.argv[1], sys.argv[2]
row = []
for n in ("c3", "c3s", "c2s", "c1s"):
    d = json.loads(open(f"{o}/{n}_{i}.json").read().strip().splitlines()[-1])
    row.append(f"{n} {d['roofline']['frac']:.4f}{'' if d['parity_verified'] else ' PARITY FAIL'}")
print(f"process {i}: " + ", ".join(row), flush=True)
PY
done
