#!/bin/bash
# Separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes (MI355X_MICROARCH.md §HBM) of the bench configs in
# PROFILE (a trailing "s" = stream mode), for tools/pmc_summary.py.  GPU box; each pass has its own limit.
mkdir -p gpurun_out && export TMPDIR=/tmp
for pr in ${PROFILE-c3 c3s}; do
  cfg=${pr%s}; args="--config $cfg"; [ "$pr" != "$cfg" ] && args="$args --mode stream"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_${pr}_fetch -o f --output-format csv -- python bench.py $args --steps 3 --warmup 1 --no-cpu --no-verify > gpurun_out/prof_${pr}_fetch.log 2>&1 || { echo "STOP fetch $pr"; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_${pr}_write -o w --output-format csv -- python bench.py $args --steps 3 --warmup 1 --no-cpu --no-verify > gpurun_out/prof_${pr}_write.log 2>&1 || { echo "STOP write $pr"; exit 1; }
  echo "pmc $pr done"
done
echo "pmc_pass done"
