#!/bin/bash
# round 3: split-K tail of the persistent GEMM: parity, then alternating A/B default bench (split vs plain tail)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nn.py -k "split_gemm or inference_net or fc1" > gpurun_out/r03_tail_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r03_tail_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/r03_tail_ab.json
for r in 1 2; do
  for t in split plain; do
    timeout -k 10 300 python -u bench.py --steps 6 --no-cpu-baseline --generation off --gemm-tail $t > gpurun_out/r03_tail_$t.json 2> gpurun_out/r03_tail_$t.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $t rc=$rc"; tail -5 gpurun_out/r03_tail_$t.err; exit $rc; }
    python -c "
import json,sys; d=json.loads(open('gpurun_out/r03_tail_$t.json').read().strip().splitlines()[-1])
g=d['gemm_layers']; print(json.dumps({'tail':'$t','round':$r,'value':d['value'],'ms':d['ms_per_step'],'frac':d['roofline']['frac'],'gemm_all_frac':d['roofline_gemm_all']['frac'],'layers':{k:round(v['us'],1) for k,v in g.items()}}))" | tee -a gpurun_out/r03_tail_ab.json
  done
done
