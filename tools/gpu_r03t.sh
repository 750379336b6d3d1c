#!/bin/bash
# round 3: real-net parity with the 8-seed main fixture (engine at 4096 games, both GEMM forms; drop-in)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v -rP --timeout 400 --timeout-method thread tests/test_gpu_realnet.py > gpurun_out/r03_realnet8.log 2>&1
rc=$?; echo "realnet rc=$rc"; grep -E "NEAR-TIE|identical to the reference|passed|failed|Error" gpurun_out/r03_realnet8.log | head -40
exit $rc
