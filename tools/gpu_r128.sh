# 128-row split GEMM (variant 17): kernel tests, 256/1024-leaf microbench, then the full GPU suite, smoke, bench
set -e
O=gpurun_out/${1:-r128}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nn.py -m gpu -x -q -k "split_gemm_kernel" --timeout 120 --timeout-method thread > $O/pytest_sg.log 2>&1
AZG_SG_LEAVES=256 AZG_SG_VARIANTS=4,17 timeout -k 10 200 python -u tools/split_gemm_bench.py > $O/sg_bench_256.json 2> $O/sg_bench_256.err
AZG_SG_LEAVES=1024 AZG_SG_VARIANTS=4,17 timeout -k 10 200 python -u tools/split_gemm_bench.py > $O/sg_bench_1024.json 2> $O/sg_bench_1024.err
timeout -k 10 300 python -u bench.py --config C2 --full-games --no-cpu-baseline > $O/bench_C2_full.json 2> $O/bench_C2_full.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
