# NN tests + default bench + kernel stats (quick network-kernel experiments)
# usage: bash tools/gpu_nn.sh <outdir under gpurun_out>
set -e
O=gpurun_out/${1:-nn}
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nn.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $R/$O/bench_prof.json 2> $R/$O/prof.err
