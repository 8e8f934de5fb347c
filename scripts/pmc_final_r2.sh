#!/bin/bash
# Refresh of k_encode's counters after the last round-2 changes: the two SQ passes
# per input class and the FETCH / WRITE traffic passes of the headline bench,
# each counter set in its own rocprofv3 run.
set -e
export TMPDIR=/tmp
O=gpurun_out/r2f
mkdir -p $O
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
SQ2="SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"
timeout -s KILL 150 rocprofv3 --pmc $SQ1 --output-format csv -d $O/sq_enc1 -o run -- python3 scripts/kbench.py --msets "1,3,4,9" --inputs random,ascii,mixed --reps 1 > $O/sq_enc1.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc $SQ2 --output-format csv -d $O/sq_enc2 -o run -- python3 scripts/kbench.py --msets "1,3,4,9" --inputs random,ascii,mixed --reps 1 > $O/sq_enc2.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 2 --warmup 1 > $O/fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 2 --warmup 1 > $O/write.log 2>&1
