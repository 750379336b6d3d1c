# split GEMM microbench + rocprof kernel stats of it and of the default bench
set -e
O=gpurun_out/${1:-gemm}
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/split_gemm_bench.py > $O/split_gemm_bench.json 2> $O/split_gemm_bench.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $R/$O/bench_prof.json 2> $R/$O/prof.err
