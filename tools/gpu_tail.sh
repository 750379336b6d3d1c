# split GEMM default schedule (tail split): kernel tests, 4096-leaf microbench, C4 bench, kernel stats
set -e
O=gpurun_out/${1:-tail}
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nn.py -m gpu -x -q -k "split_gemm" --timeout 120 --timeout-method thread > $O/pytest_sg.log 2>&1
AZG_SG_VARIANTS=4 timeout -k 10 200 python -u tools/split_gemm_bench.py > $O/sg_bench_4096.json 2> $O/sg_bench_4096.err
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $R/$O/bench_prof.json 2> $R/$O/prof.err
