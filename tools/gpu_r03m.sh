#!/bin/bash
# round 3: side-stream engine test, then two half-batch engines on two streams with a capped
# persistent GEMM grid (overlap probe)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r03_parity_streams.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r03_parity_streams.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/overlap_probe.py --diag > gpurun_out/r03_overlap_diag.json 2>&1
rc=$?; echo "diag rc=$rc"; cat gpurun_out/r03_overlap_diag.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/overlap_probe.py > gpurun_out/r03_overlap_probe.json 2> gpurun_out/r03_overlap_probe.err
rc=$?; echo "probe rc=$rc"; cat gpurun_out/r03_overlap_probe.json; tail -3 gpurun_out/r03_overlap_probe.err; exit $rc
