#!/bin/bash
# round 3: FC tail on libazg -- kernel tests, network tests, tail variants, default bench
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_nn.py > gpurun_out/r03_nn_tests.log 2>&1
rc=$?; echo "nn tests rc=$rc"; tail -3 gpurun_out/r03_nn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/fc_tail_bench.py > gpurun_out/r03_fc_tail_bench.json 2> gpurun_out/r03_fc_tail_bench.err
rc=$?; echo "fc tail bench rc=$rc"; cat gpurun_out/r03_fc_tail_bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r03_bench_C4_fctail.json 2> gpurun_out/r03_bench_C4_fctail.err
rc=$?; echo "bench rc=$rc"; tail -c 300 gpurun_out/r03_bench_C4_fctail.json; exit $rc
