#!/bin/bash
# same-box A/B of the headline bench: the round-start library + bench (ab/old, commit
# 35d9af5) against the current tree, alternating
set -e
export TMPDIR=/tmp
O=$PWD/gpurun_out/oldnew
mkdir -p $O
for r in 1 2 3; do
  (cd ab/old && timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --steps 10 --warmup 3 > $O/old_$r.json 2> $O/old_$r.err)
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --steps 10 --warmup 3 > $O/new_$r.json 2> $O/new_$r.err
done
