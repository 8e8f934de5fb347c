#!/bin/bash
# round 3: SQ counters of k_encode (8 waves per SIMD, chunks in place) per input class, two passes
set -e
export TMPDIR=/tmp
O=gpurun_out/r3sq
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/sq_enc1 -o run -- python3 scripts/kbench.py --msets "1,3,4,9" --inputs random,ascii,mixed --reps 1 > $O/sq_enc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH --output-format csv -d $O/sq_enc2 -o run -- python3 scripts/kbench.py --msets "1,3,4,9" --inputs random,ascii,mixed --reps 1 > $O/sq_enc2.log 2>&1
