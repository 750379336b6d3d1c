# rocprof kernel stats of the C2, C3 and C5 configs (short runs)
set -e
O=gpurun_out/${1:-cfgprof}
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
cd /tmp
for c in C2 C3 C5; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$c -o run -- python3 $R/bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/bench_prof_$c.json 2> $R/$O/prof_$c.err
done
