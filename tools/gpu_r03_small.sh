#!/bin/bash
# round 3: the one-launch small-path layer (azg_small_layer) -- its tests, the drop-in
# per-call time of the library form against the small form, and the small form's kernels
set -e
O=gpurun_out/${1:-r03_small}
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nn.py -m gpu -x -q -k "small" --timeout 120 --timeout-method thread > $O/pytest_small.log 2>&1
for g in othello6 inflexion; do
  timeout -k 10 300 python -u tools/dropin_bench.py --game $g --forms inference-miopen,inference-small,inference-miopen,inference-small > $O/dropin_$g.json 2> $O/dropin_$g.err
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/tools/dropin_bench.py --game inflexion --forms inference-small --moves 8 > $R/$O/prof.log 2>&1
python3 $R/tools/prof_summary.py $R/$O/prof/run_kernel_stats.csv > $R/$O/prof.md
rm -f $R/$O/prof/*trace*.csv
