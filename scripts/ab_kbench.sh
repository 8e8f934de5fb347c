#!/bin/bash
# A/B of k_encode builds on one box: scripts/kbench.py with each library in
# ab/ (AMBC_LIB), interleaved twice, so box-to-box clock differences cancel.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
MS=${MS:-1,3,4,9}
for r in 1 2; do
  for L in ab/lib_*.so; do
    echo "== $L" >> gpurun_out/ab.log
    AMBC_LIB=$L timeout -k 10 120 python3 scripts/kbench.py --msets "$MS" --reps 5 >> gpurun_out/ab.log 2>&1
  done
done
