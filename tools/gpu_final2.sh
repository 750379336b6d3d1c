# full GPU pass: GPU suite, smoke, default bench (driver's arguments), kernel stats, PMC HBM passes
set -e
O=gpurun_out/${1:-final2}
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python -u bench.py --config C2 --full-games --no-cpu-baseline > $O/bench_C2_full.json 2> $O/bench_C2_full.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $R/$O/bench_prof.json 2> $R/$O/prof.err
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --no-cpu-baseline > $R/$O/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_write -o run -- python3 $R/bench.py --steps 2 --no-cpu-baseline > $R/$O/pmc_write.log 2>&1
python3 $R/tools/pmc_summary.py $R/$O/pmc_fetch/run_counter_collection.csv $R/$O/pmc_write/run_counter_collection.csv > $R/$O/pmc_summary.json
