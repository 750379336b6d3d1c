#!/bin/bash
# round 3: real-net parity with the flips printed (-rP), recorded for profiles/
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -v -rP --timeout 400 --timeout-method thread tests/test_gpu_realnet.py > gpurun_out/r03_realnet_rP.log 2>&1
rc=$?; echo "realnet rc=$rc"; grep -E "NEAR-TIE|identical to the reference|passed|failed" gpurun_out/r03_realnet_rP.log; exit $rc
