set -e
O=gpurun_out/r02i; mkdir -p $O
for e in 1 5 25 100000; do timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --timer-every $e > $O/bench_e$e.json 2> $O/bench_e$e.err; done
R=$PWD; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --timer-every 100000 > $R/$O/bench_prof.json 2> $R/$O/prof.err
