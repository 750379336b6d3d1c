#!/bin/bash
# round 3: split-GEMM ring variants 20/21 (deep DMA prefetch for short launches): parity, then timing at C2 shapes
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nn.py -k split_gemm > gpurun_out/r03_ring_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r03_ring_tests.log; [ $rc -eq 0 ] || exit $rc
for L in 256 512 1024; do
  AZG_SG_LEAVES=$L AZG_SG_VARIANTS=4,17,18,20,21 timeout -k 10 300 python -u tools/split_gemm_bench.py > gpurun_out/r03_ring_bench_$L.json 2> gpurun_out/r03_ring_bench_$L.err
  rc=$?; echo "bench $L rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
