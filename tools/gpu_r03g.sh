#!/bin/bash
# round 3: FC tail forms in the engine, alternating on one box
mkdir -p gpurun_out
for i in 1 2; do for t in "azg 2,1" "blas 4,2" "azg 4,2" "azg 8,4"; do
  set -- $t
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 6 --fc-tail $1 --fc-kparts $2 > gpurun_out/r03_ab2_$1_${2/,/_}_$i.json 2>/dev/null
  rc=$?; echo "$t $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done; done
