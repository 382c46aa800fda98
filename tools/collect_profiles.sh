#!/bin/bash
# Copies a refresh run's evidence from gpurun_out/ into profiles/<dest>/ (kernel-trace stats,
# bench JSON lines, PMC counter CSVs, SQ counters, test and smoke logs).  Usage: collect_profiles.sh r03/check1
D=profiles/$1; mkdir -p $D
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log $D/ 2>/dev/null
for f in gpurun_out/bench_*.log; do b=$(basename $f .log); b=${b#bench_}; tail -1 $f > $D/${b}_bench.json; done
for d in gpurun_out/prof_*_kt; do p=$(basename $d _kt); p=${p#prof_}; cp $d/kt_kernel_stats.csv $D/${p}_kernel_stats.csv; grep "^{\"metric\"" gpurun_out/prof_${p}_kt.log > $D/${p}_bench_under_rocprof.json; done
for d in gpurun_out/prof_*_fetch; do p=$(basename $d _fetch); p=${p#prof_}; cp $d/f_counter_collection.csv $D/${p}_pmc_fetch_size.csv; done
for d in gpurun_out/prof_*_write; do p=$(basename $d _write); p=${p#prof_}; cp $d/w_counter_collection.csv $D/${p}_pmc_write_size.csv; done
if [ -d gpurun_out/sq ]; then for c in gpurun_out/sq/*/; do n=$(basename $c); cp $c/p_counter_collection.csv $D/${n}_sq_counters.csv; done; fi
cp gpurun_out/dropin_*.json $D/ 2>/dev/null
ls $D | wc -l
