#!/bin/bash
# k_encode phase split (s_memtime stamps, diagnostic library) and SQ counters per
# input class, current code
set -e
export TMPDIR=/tmp
O=gpurun_out/r5ph
mkdir -p $O
AMBC_STAMPS=1 AMBC_LIB=adaptive-compression_amd/ambc/libambc_hip_stamps.so timeout -k 10 200 \
    python3 scripts/kbench.py --msets "9;1,3,4,9" --inputs zero,random,ascii,mixed --reps 1 > $O/stamps.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/sq_enc1 -o run -- python3 scripts/kbench.py --msets "1,3,4,9" --inputs random,ascii,mixed --reps 1 > $O/sq_enc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH --output-format csv -d $O/sq_enc2 -o run -- python3 scripts/kbench.py --msets "1,3,4,9" --inputs random,ascii,mixed --reps 1 > $O/sq_enc2.log 2>&1
echo phases ok
