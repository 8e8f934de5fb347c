#!/bin/bash
# zlib-9 id 5 above 8 KiB: kernel times per input class and chunk size
# (rocprofv3 stats of kbench with AMBC_FLAG_ZLIB9), then the reference's walk
# with id 5 as zlib-9's bytes (MS_MODE=reference) on 32 / 256 MiB.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in ${CHUNKS:-16384 65536}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kp_z9b_$C -o run -- \
    python3 scripts/kbench.py --chunk $C --flags 2 --inputs "${INPUTS:-zero,random,ascii,mixed}" --msets "${MS:-5}" --reps 2 > gpurun_out/kp_z9b_$C.log 2>&1
done
MS_MODE=reference MS_SETS="${MSSETS:-mixed:1,2,3,4,5;mixed:1,3,4,5}" timeout -k 10 400 python3 -u scripts/multisize_bench.py ${MSSIZES:-32 256} > gpurun_out/ms_z9.log 2>&1
