#!/bin/bash
# SQ counters of k_encode for each library in ab/ (one pmc pass per library)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/abpmc
MS=${MS:-1,3,4,9}
for L in ab/lib_*.so; do
  b=$(basename $L .so)
  AMBC_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_INSTS_VMEM --output-format csv -d gpurun_out/abpmc/$b -o run -- python3 scripts/kbench.py --msets "$MS" --inputs random,ascii,mixed --reps 1 > gpurun_out/abpmc/$b.log 2>&1
done
