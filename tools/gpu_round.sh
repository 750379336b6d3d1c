# One GPU-box pass: GPU tests, smoke, bench (split + f32 GEMMs), split-GEMM microbench,
# rocprof kernel stats, PMC HBM passes (FETCH_SIZE, WRITE_SIZE in separate runs).
# usage: bash tools/gpu_round.sh <outdir under gpurun_out> [--no-pmc]
set -e
O=gpurun_out/${1:-run}
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python -u bench.py --gemm f32 --no-cpu-baseline > $O/bench_f32.json 2> $O/bench_f32.err
timeout -k 10 200 python -u tools/split_gemm_bench.py > $O/split_gemm_bench.json 2> $O/split_gemm_bench.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $R/$O/bench_prof.json 2> $R/$O/prof.err
if [ "$2" != "--no-pmc" ]; then
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --no-cpu-baseline > $R/$O/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_write -o run -- python3 $R/bench.py --steps 2 --no-cpu-baseline > $R/$O/pmc_write.log 2>&1
fi
