# One GPU-box pass: GPU tests, smoke, bench (split + f32 GEMMs), rocprof kernel stats.
# usage: bash tools/gpu_round.sh <outdir under gpurun_out>
set -e
O=gpurun_out/${1:-run}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python -u bench.py --gemm f32 --no-cpu-baseline > $O/bench_f32.json 2> $O/bench_f32.err
timeout -k 10 300 python -u bench.py --gemm split_blas --no-cpu-baseline > $O/bench_split_blas.json 2> $O/bench_split_blas.err
R=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $R/$O/bench_prof.json 2> $R/$O/prof.err
