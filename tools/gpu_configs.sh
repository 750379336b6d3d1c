set -e
O=gpurun_out/r1s2d
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
for c in C1 C3 C5; do timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err; done
timeout -k 10 300 python -u bench.py --config C2 --full-games --no-cpu-baseline > $O/bench_C2_full.json 2> $O/bench_C2_full.err
timeout -k 10 300 python -u bench.py --config C2 --full-games --graph --no-cpu-baseline > $O/bench_C2_full_graph.json 2> $O/bench_C2_full_graph.err
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --no-cpu-baseline > $R/$O/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_write -o run -- python3 $R/bench.py --steps 2 --no-cpu-baseline > $R/$O/pmc_write.log 2>&1
