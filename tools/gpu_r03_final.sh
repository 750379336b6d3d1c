#!/bin/bash
# round 3 final pass on the committed tree: GPU suite, smoke, default bench (driver's
# arguments) and its kernel summary; large CSVs summarised on the box and deleted
set -e
O=gpurun_out/${1:-r03_final}
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --durations 10 > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $R/$O/bench_prof.json 2> $R/$O/prof.err
python3 $R/tools/prof_summary.py $R/$O/prof/run_kernel_stats.csv > $R/$O/prof.md
rm -f $R/$O/prof/*trace*.csv
