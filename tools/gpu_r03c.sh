#!/bin/bash
# round 3: the whole GPU suite (as the driver runs it) + smoke; stop at the first abnormal exit
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 400 --timeout-method thread --durations=40 > gpurun_out/r03_pytest_gpu.log 2>&1
rc=$?
echo "gpu tests rc=$rc"
tail -3 gpurun_out/r03_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/r03_smoke.log
exit $rc
