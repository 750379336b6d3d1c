#!/bin/bash
# round 3: one engine whose leaf batch is evaluated as 2 / 4 parts on their own streams
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/overlap_probe.py --split-net --rounds 4 > gpurun_out/r03_split_net_probe.json 2> gpurun_out/r03_split_net_probe.err
rc=$?; echo "probe rc=$rc"; cat gpurun_out/r03_split_net_probe.json; tail -3 gpurun_out/r03_split_net_probe.err; exit $rc
