# All BASELINE configs through bench.py: C1 (eager and hipGraph replay, full game), C2 full games (eager and
# hipGraph), C3, C5, and C4 (the default) as measured full games.
# usage: bash tools/gpu_configs.sh <outdir under gpurun_out>
set -e
O=gpurun_out/${1:-configs}
mkdir -p $O
export TMPDIR=/tmp
for c in C1 C3 C5; do timeout -k 10 300 python -u bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err; done
timeout -k 10 300 python -u bench.py --config C1 --full-games --graph --no-cpu-baseline > $O/bench_C1_full_graph.json 2> $O/bench_C1_full_graph.err
timeout -k 10 300 python -u bench.py --config C2 --full-games --no-cpu-baseline > $O/bench_C2_full.json 2> $O/bench_C2_full.err
timeout -k 10 300 python -u bench.py --config C2 --full-games --graph --no-cpu-baseline > $O/bench_C2_full_graph.json 2> $O/bench_C2_full_graph.err
timeout -k 10 300 python -u bench.py --full-games --no-cpu-baseline > $O/bench_C4_full.json 2> $O/bench_C4_full.err
