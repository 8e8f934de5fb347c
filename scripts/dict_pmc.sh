#!/bin/bash
# SQ counters of k_dict on the ASCII class ({1,2,3,4}), two passes, for ab/lib_*.so
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/dpmc
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
SQ2="SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"
for L in ab/lib_*.so; do
  b=$(basename $L .so)
  AMBC_LIB=$L timeout -s KILL 90 rocprofv3 --pmc $SQ1 --output-format csv -d gpurun_out/dpmc/${b}_1 -o run -- python3 scripts/kbench.py --msets "1,2,3,4" --inputs ascii --reps 1 > gpurun_out/dpmc/${b}_1.log 2>&1
  AMBC_LIB=$L timeout -s KILL 90 rocprofv3 --pmc $SQ2 --output-format csv -d gpurun_out/dpmc/${b}_2 -o run -- python3 scripts/kbench.py --msets "1,2,3,4" --inputs ascii --reps 1 > gpurun_out/dpmc/${b}_2.log 2>&1
done
