# full GPU pass on the current build: split GEMM tests, C2 full games, GPU suite, smoke, default bench, C2 kernel stats
set -e
O=gpurun_out/${1:-final}
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nn.py -m gpu -x -q -k "split_gemm" --timeout 120 --timeout-method thread > $O/pytest_sg.log 2>&1
timeout -k 10 300 python -u bench.py --config C2 --full-games --no-cpu-baseline > $O/bench_C2_full.json 2> $O/bench_C2_full.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_C2 -o run -- python3 $R/bench.py --config C2 --no-cpu-baseline > $R/$O/bench_C2_prof.json 2> $R/$O/prof_C2.err
