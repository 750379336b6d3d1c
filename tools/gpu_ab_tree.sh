#!/bin/bash
# A/B of the tree kernels: this tree (A) against a baseline worktree at ./ab_base (B,
# the previous commit's libazg), alternating on one box; stub evaluator (tree-bound)
# and the default network, generation measurement off.
set -e
O=gpurun_out/${1:-ab_tree}
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  for arm in A B; do
    d=.; [ $arm = B ] && d=ab_base
    (cd $d && timeout -k 10 200 python -u bench.py --evaluator stub --steps 20 --warmup 5 --no-cpu-baseline --generation off) > $O/stub_${arm}_$i.json 2> $O/stub_${arm}_$i.err
  done
done
for i in 1 2; do
  for arm in A B; do
    d=.; [ $arm = B ] && d=ab_base
    (cd $d && timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --generation off) > $O/net_${arm}_$i.json 2> $O/net_${arm}_$i.err
  done
done
