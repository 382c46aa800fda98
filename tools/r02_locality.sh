export TMPDIR=/tmp
O=gpurun_out/loc; mkdir -p $O
for L in none out in inout; do
  if [ $L = none ]; then unset PROBE_LOC; else export PROBE_LOC=$L; fi
  PROBE_GOP=24 timeout -k 10 200 ./tools/probe 420 3840 2160 300 5 > $O/loc_$L.txt 2>&1 || { cat $O/loc_$L.txt; exit 1; }
  echo "== $L"; grep "production\|no prefetch ldsqt static" $O/loc_$L.txt
done
