#!/bin/bash
# round 3: small-batch forward on libazg small GEMMs: parity, then C1 drop-in / engine timings
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_nn.py tests/test_gpu_dropin.py -k "small or board_sizes or inference or dropin or graph" > gpurun_out/r03_small_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r03_small_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dropin_bench.py --game othello6 --forms module-graph,inference-miopen,inference-winograd > gpurun_out/r03_small_dropin.json 2> gpurun_out/r03_small_dropin.err
rc=$?; echo "dropin rc=$rc"; cat gpurun_out/r03_small_dropin.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dropin_bench.py --game inflexion --forms inference-miopen,inference-winograd >> gpurun_out/r03_small_dropin.json 2>> gpurun_out/r03_small_dropin.err
rc=$?; echo "dropin2 rc=$rc"; tail -2 gpurun_out/r03_small_dropin.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config C1 --no-cpu-baseline > gpurun_out/r03_bench_C1.json 2> gpurun_out/r03_bench_C1.err
rc=$?; echo "C1 rc=$rc"; python -c "
import json; d=json.loads(open('gpurun_out/r03_bench_C1.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('games_per_s'))"
exit $rc
