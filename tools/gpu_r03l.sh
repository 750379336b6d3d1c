#!/bin/bash
# round 3: drop-in evaluator forms at one leaf per simulation (C1 arrangement) + kernel stats
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dropin_bench.py --game othello6 > gpurun_out/r03_dropin_forms.json 2> gpurun_out/r03_dropin_forms.err
rc=$?; echo "othello6 rc=$rc"; cat gpurun_out/r03_dropin_forms.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dropin_bench.py --game inflexion >> gpurun_out/r03_dropin_forms.json 2>> gpurun_out/r03_dropin_forms.err
rc=$?; echo "inflexion rc=$rc"; tail -4 gpurun_out/r03_dropin_forms.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_prof_dropin_module -o run -- python3 tools/dropin_bench.py --game othello6 --forms module-graph --moves 8 > gpurun_out/r03_prof_dropin_module.log 2>&1
rc=$?; echo "prof module rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_prof_dropin_inf -o run -- python3 tools/dropin_bench.py --game othello6 --forms inference-miopen --moves 8 > gpurun_out/r03_prof_dropin_inf.log 2>&1
rc=$?; echo "prof inf rc=$rc"; exit $rc
