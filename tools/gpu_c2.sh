# C2 (256 games x 25 sims) full games, eager and hipGraph
set -e
O=gpurun_out/${1:-c2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config C2 --full-games --no-cpu-baseline > $O/bench_C2_full.json 2> $O/bench_C2_full.err
timeout -k 10 300 python -u bench.py --config C2 --full-games --graph --no-cpu-baseline > $O/bench_C2_full_graph.json 2> $O/bench_C2_full_graph.err
