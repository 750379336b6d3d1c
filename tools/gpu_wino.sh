# Winograd transform tests + default bench + kernel stats (quick transform experiments)
set -e
O=gpurun_out/${1:-wino}
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nn.py -m gpu -x -q -k "winograd or board_sizes or reference or fc1" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $R/$O/bench_prof.json 2> $R/$O/prof.err
