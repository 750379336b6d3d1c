#!/bin/bash
# round 3: rehearse bench.py --gpus 2 (self-launched ranks, both on the one GPU, gloo collectives)
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --games 512 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_bench_n2_gloo.json 2> gpurun_out/r03_bench_n2_gloo.err
rc=$?; echo "n2 rc=$rc"; tail -c 400 gpurun_out/r03_bench_n2_gloo.json; tail -5 gpurun_out/r03_bench_n2_gloo.err; exit $rc
