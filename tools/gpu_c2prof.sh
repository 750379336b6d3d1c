# kernel stats of the C2 config (256 games x 25 sims)
set -e
O=gpurun_out/${1:-c2prof}
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --config C2 --steps 20 --warmup 2 --no-cpu-baseline --timer-every 1000000 > $R/$O/bench_prof.json 2> $R/$O/prof.err
