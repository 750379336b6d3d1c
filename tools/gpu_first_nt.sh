# winograd_first with / without non-temporal V stores (AZG_FIRST_NT), alternating kernel-stats runs on one box
set -e
O=gpurun_out/${1:-first_nt}
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
cd /tmp
for i in 1 2; do
for nt in 0 1; do
AZG_FIRST_NT=$nt timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p${nt}_$i -o run -- python3 $R/bench.py --steps 3 --no-cpu-baseline > $R/$O/b${nt}_$i.json 2> $R/$O/e${nt}_$i.err
done
done
