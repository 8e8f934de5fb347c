#!/bin/bash
# SQ instruction-mix counters of k_encode per input class (two passes; each pass
# stays within the per-block counter limits), csv under gpurun_out/pmc_sq{1,2}
set -e
export TMPDIR=/tmp
MS=${1:-1,3,4,9}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmc_sq1 -o run -- python3 scripts/kbench.py --msets "$MS" --inputs random,ascii --reps 1 > gpurun_out/pmc_sq1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmc_sq2 -o run -- python3 scripts/kbench.py --msets "$MS" --inputs random,ascii --reps 1 > gpurun_out/pmc_sq2.log 2>&1
