#!/bin/bash
# per-layer microbench of azg_small_layer against torch's library layers at one leaf
set -e
O=gpurun_out/${1:-r03_sl}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/small_layer_bench.py > $O/layers.json 2> $O/layers.err
