#!/bin/bash
# round 3 checkpoint: whole GPU suite + smoke (as the driver runs them), default bench, kernel-trace profile
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 400 --timeout-method thread --durations=25 > gpurun_out/r03_pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/r03_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r03_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench_C4.json 2> gpurun_out/r03_bench_C4.err
rc=$?; echo "bench rc=$rc"; tail -c 300 gpurun_out/r03_bench_C4.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/r03_prof_C4
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_prof_C4 -o run -- python -u bench.py --steps 3 --no-cpu-baseline --generation off > gpurun_out/r03_prof_C4.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
