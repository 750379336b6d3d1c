#!/bin/bash
# round 3: A/B of the FC tail (libazg split-K vs hipBLASLt) on one box, alternating
mkdir -p gpurun_out
for i in 1 2; do for t in azg blas; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 6 --fc-tail $t > gpurun_out/r03_ab_${t}_$i.json 2> gpurun_out/r03_ab_${t}_$i.err
  rc=$?; echo "$t $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done; done
