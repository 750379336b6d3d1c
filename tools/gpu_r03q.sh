#!/bin/bash
# round 3: small-batch FC tail on libazg split-K vs the f32 tail
mkdir -p gpurun_out
for B in 256 512; do
  timeout -k 10 300 python -u tools/fc_small_probe.py --batch $B >> gpurun_out/r03_fc_small_probe.json 2> gpurun_out/r03_fc_small_probe_$B.err
  rc=$?; echo "B=$B rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r03_fc_small_probe_$B.err; exit $rc; }
done
cat gpurun_out/r03_fc_small_probe.json
