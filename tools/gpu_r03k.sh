#!/bin/bash
# round 3: drop-in MCTS graph replay (graph vs eager, golden drop-in tests, real-net drop-in)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -rP --durations=15 --timeout 300 --timeout-method thread \
    tests/test_gpu_dropin.py tests/test_gpu_realnet.py -k "dropin or execute_episode" > gpurun_out/r03_dropin_graph.log 2>&1
rc=$?; echo "dropin rc=$rc"; grep -E "getActionProb|NEAR-TIE|passed|failed|Error|s call" gpurun_out/r03_dropin_graph.log | head -40
exit $rc
