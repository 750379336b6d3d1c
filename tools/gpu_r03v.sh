#!/bin/bash
# round 3: one engine, games as 1 / 2 / 3 / 4 concurrent stream ranges (alternating A/B, default C4 workload);
# then the range path's parity tests
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_realnet.py -k "streams or side_streams or composition" > gpurun_out/r03_streams_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r03_streams_tests.log; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
rm -f gpurun_out/r03_streams_ab.json
for r in 1 2; do
  for k in 1 2 3 4; do
    timeout -k 10 300 python -u bench.py --steps 6 --no-cpu-baseline --generation off --streams $k > gpurun_out/r03_streams_$k.json 2> gpurun_out/r03_streams_$k.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench streams=$k rc=$rc"; tail -5 gpurun_out/r03_streams_$k.err; exit $rc; }
    python -c "
import json; d=json.loads(open('gpurun_out/r03_streams_$k.json').read().strip().splitlines()[-1])
print(json.dumps({'streams':$k,'round':$r,'value':d['value'],'ms':d['ms_per_step']}))" | tee -a gpurun_out/r03_streams_ab.json
  done
done
