#!/bin/bash
# round 3: kernel-trace summary of C2 (256 games x 25 sims)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_prof_C2 -o run -- python3 bench.py --config C2 --steps 8 --generation off --no-cpu-baseline > gpurun_out/r03_prof_C2.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/r03_prof_C2.log; exit $rc
