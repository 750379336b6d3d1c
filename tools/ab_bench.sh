#!/bin/bash
# A/B of two libazg builds on one box: tools/ab_bench.sh <run> <a.so> <b.so> [bench args, commas for spaces]
# Copies each build over the package's libazg.so in turn (A B A B), one bench.py per turn; restores A.
set -e
R=$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)
O=$R/gpurun_out/$1
mkdir -p "$O"
args=${4//,/ }
for i in 1 2; do
    for v in a b; do
        so=$2; [ "$v" = b ] && so=$3
        cp "$R/$so" "$R/alpha-zero-general-inflexion_amd/libazg.so"
        timeout -k 10 300 python -u "$R/bench.py" $args > "$O/ab_${v}_$i.json" 2> "$O/ab_${v}_$i.err"
    done
done
cp "$R/$2" "$R/alpha-zero-general-inflexion_amd/libazg.so"
