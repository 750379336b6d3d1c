#!/bin/bash
# round 3: tree-kernel layout (compact edge slots, 16-slot first probe, packed node
# keys) -- GPU suite, smoke, A/B against ./ab_base (tools/gpu_ab_tree.sh), kernel
# stats and the PMC HBM passes of this tree; large CSVs summarised and deleted
set -e
O=gpurun_out/${1:-r03t2}
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --durations 15 > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
bash tools/gpu_ab_tree.sh ${1:-r03t2}/ab
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $R/$O/bench_prof.json 2> $R/$O/prof.err
python3 $R/tools/prof_summary.py $R/$O/prof/run_kernel_stats.csv > $R/$O/prof.md
rm -f $R/$O/prof/*trace*.csv
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --no-cpu-baseline > $R/$O/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_write -o run -- python3 $R/bench.py --steps 2 --no-cpu-baseline > $R/$O/pmc_write.log 2>&1
python3 $R/tools/pmc_summary.py $R/$O/pmc_fetch/run_counter_collection.csv $R/$O/pmc_write/run_counter_collection.csv > $R/$O/pmc_summary.json
rm -f $R/$O/pmc_fetch/*.csv $R/$O/pmc_write/*.csv
du -sh $R/gpurun_out
