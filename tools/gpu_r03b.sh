#!/bin/bash
# round 3: real-net parity failures, with messages; stop at the first abnormal exit
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --tb=short --timeout 300 --timeout-method thread tests/test_gpu_realnet.py > gpurun_out/r03_realnet.log 2>&1
rc=$?
echo "realnet rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u -m pytest -v --tb=long --timeout 200 --timeout-method thread tests/test_gpu_dropin.py -k "replay_form" > gpurun_out/r03_replay.log 2>&1
echo "replay rc=$?"
