#!/bin/bash
# A/B of decode builds: scripts/dbench.py with each library in ab/, interleaved twice
set -e
export TMPDIR=/tmp
M=${M:-1,3,4,5}
for r in 1 2; do
  for L in ab/lib_*.so; do
    echo "== $L" >> gpurun_out/abd.log
    AMBC_LIB=$L timeout -k 10 200 python3 scripts/dbench.py --size 134217728 --methods $M --reps 3 >> gpurun_out/abd.log 2>&1
  done
done
