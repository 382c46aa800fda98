#!/bin/bash
# The whole decoder, end to end, against the reference's own (GPU box): a seeded synthetic .mpg
# (tools/mpg_synth) decoded to BMP files by
#   ref:    oracle/_ref/mjref_app decode   -- the reference's mjpeg423_decode() compiled in place
#   blocks: oracle/_ref/mjdrop_blocks      -- the same reference decoder, idct()/ycbcr_to_rgb()/encode_bmp()
#                                             from libmj423gpu.so (zero source changes, deferred default)
#   loop:   oracle/_ref/mjdrop_loop        -- only the reference's frame loop; lossless_decode() from the
#                                             library too
#   lib:    oracle/_ref/mjdrop_file        -- libmj423gpu.so's mjpeg423_decode() (pipelined front end + GPU)
# Wall time of each (median of REPS runs, interleaved; default 3) and whether every BMP is
# byte-identical to the reference's.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/e2e
W=/tmp/mj423_e2e; rm -rf $W; mkdir -p $W
for geo in "640 480 240" "1920 1080 48" "1920 1080 240"; do
  set -- $geo; w=$1; h=$2; n=$3; tag=${w}x${h}x${n}
  python -c "import sys; sys.path.insert(0, 'tools'); import mpg_synth; mpg_synth.build(); mpg_synth.write('$W/$tag.mpg', $w, $h, $n, gop=24)" || exit 1
  for r in $(seq ${REPS:-3}); do
    for v in ref blocks loop lib; do
      case $v in ref) exe="oracle/_ref/mjref_app decode";; blocks) exe=oracle/_ref/mjdrop_blocks;;
                 loop) exe=oracle/_ref/mjdrop_loop;; lib) exe=oracle/_ref/mjdrop_file;; esac
      mkdir -p $W/$tag/$v
      t0=$(date +%s%N)
      timeout -k 10 300 $exe $W/$tag.mpg $W/$tag/$v/dec0000.bmp 2> $W/$tag/$v.err || { echo "STOP $v $tag"; cat $W/$tag/$v.err; exit 1; }
      t1=$(date +%s%N)
      echo "$tag $v $(( (t1 - t0) / 1000 ))" >> gpurun_out/e2e/times.txt   # microseconds
    done
  done
  python - $W/$tag $tag $n $w $h <<'PY' >> gpurun_out/e2e/e2e.jsonl
import hashlib, json, os, sys
d, tag, n, w, h = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
runs = {}
for l in open("gpurun_out/e2e/times.txt"):
    if l.startswith(tag + " "):
        runs.setdefault(l.split()[1], []).append(float(l.split()[2]) / 1e6)
times = {k: sorted(v)[len(v) // 2] for k, v in runs.items()}
sha = lambda v: [hashlib.sha256(open(os.path.join(d, v, f"dec{i:04d}.bmp"), "rb").read()).hexdigest() for i in range(n)]
ref = sha("ref")
res = {"geometry": f"{w}x{h}", "frames": n, "seconds": times, "runs": runs,
       "fps": {k: round(n / t, 1) for k, t in times.items()},
       "speedup_vs_reference": {k: round(times["ref"] / t, 2) for k, t in times.items() if k != "ref"},
       "bmps_identical_to_reference": {v: sha(v) == ref for v in ("blocks", "loop", "lib")},
       "note": "median wall time including process start, file reads and BMP writes to /tmp; one host thread for ref"}
print(json.dumps(res))
PY
  tail -1 gpurun_out/e2e/e2e.jsonl
  rm -rf $W/$tag
done
rm -rf $W
echo "decoder_e2e done"
