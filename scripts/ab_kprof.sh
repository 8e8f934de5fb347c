#!/bin/bash
# Per-kernel device times (rocprofv3 --kernel-trace --stats) of scripts/kbench.py
# for every library in ab/ (AMBC_LIB): INPUTS / MS select the case.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in ab/lib_*.so; do
  b=$(basename $L .so)
  AMBC_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/kp_$b -o run -- \
    python3 scripts/kbench.py --inputs "${INPUTS:-ascii}" --msets "${MS:-1,2,3,4}" --reps 3 > gpurun_out/kp_$b.log 2>&1
done
