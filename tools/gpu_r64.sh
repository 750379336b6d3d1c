# 64-row split GEMM (variant 18): kernel tests, 256/512-leaf microbench
set -e
O=gpurun_out/${1:-r64}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nn.py -m gpu -x -q -k "split_gemm" --timeout 120 --timeout-method thread > $O/pytest_sg.log 2>&1
AZG_SG_LEAVES=256 AZG_SG_VARIANTS=4,17,18 timeout -k 10 200 python -u tools/split_gemm_bench.py > $O/sg_bench_256.json 2> $O/sg_bench_256.err
AZG_SG_LEAVES=512 AZG_SG_VARIANTS=4,17,18 timeout -k 10 200 python -u tools/split_gemm_bench.py > $O/sg_bench_512.json 2> $O/sg_bench_512.err
AZG_SG_LEAVES=128 AZG_SG_VARIANTS=4,17,18 timeout -k 10 200 python -u tools/split_gemm_bench.py > $O/sg_bench_128.json 2> $O/sg_bench_128.err
