#!/bin/bash
# round 3: default bench (driver args), kernel-trace profile of the same command
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench_C4.json 2> gpurun_out/r03_bench_C4.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/r03_bench_C4.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_prof_C4 -o run -- python -u bench.py --steps 3 --no-cpu-baseline > gpurun_out/r03_prof_C4.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in C2 C3 C5; do
  timeout -k 10 600 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/r03_bench_$c.json 2> gpurun_out/r03_bench_$c.err
  rc=$?; echo "bench $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
