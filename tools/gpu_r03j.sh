#!/bin/bash
# round 3: real-net parity incl. Othello (C1/C5) with flips printed, then the default bench (generation pass)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v -rP --timeout 400 --timeout-method thread tests/test_gpu_realnet.py > gpurun_out/r03_realnet_all.log 2>&1
rc=$?; echo "realnet rc=$rc"; grep -E "NEAR-TIE|identical to the reference|passed|failed|Error" gpurun_out/r03_realnet_all.log | head -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r03_bench_C4_gen.json 2> gpurun_out/r03_bench_C4_gen.err
rc=$?; echo "bench rc=$rc"; exit $rc
