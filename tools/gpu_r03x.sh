#!/bin/bash
# round 3: kernel stats of the small-batch forward (drop-in, inference form, one game)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/r03_prof_small
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_prof_small -o run -- python3 tools/dropin_bench.py --game inflexion --forms inference-winograd --moves 8 > gpurun_out/r03_prof_small.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
