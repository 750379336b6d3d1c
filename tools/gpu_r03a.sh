#!/bin/bash
# round 3: new parity tests, split GEMM variant 19 tests + microbench, DMA probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_realnet.py tests/test_gpu_dist.py tests/test_gpu_dropin.py > gpurun_out/r03_t2.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_nn.py -k "split_gemm" > gpurun_out/r03_gemm_tests.log 2>&1 || { echo "gemm tests failed"; tail -5 gpurun_out/r03_gemm_tests.log; exit 1; }
echo gemm tests ok
AZG_SG_VARIANTS="4,19" timeout -k 10 300 python -u tools/split_gemm_bench.py > gpurun_out/r03_split_gemm_bench.json 2> gpurun_out/r03_split_gemm_bench.err || exit 1
echo bench ok
timeout -k 10 120 tools/dma_probe > gpurun_out/r03_dma_probe.json 2>&1
echo probe rc=$?
