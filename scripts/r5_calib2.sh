#!/bin/bash
# TCC read requests by size (32 / 64 / 128 B) against known byte counts, then
# on k_encode per input class (kbench)
set -e
export TMPDIR=/tmp
O=gpurun_out/r5cal2
mkdir -p $O
C1="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum"
C2="TCC_BUBBLE_sum TCC_MISS_sum TCC_HIT_sum"
timeout -k 10 60 ./scripts/pmc_calib > $O/calib_plain.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc $C1 --output-format csv -d $O/cal_req -o run -- ./scripts/pmc_calib > $O/cal_req.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc $C2 --output-format csv -d $O/cal_hit -o run -- ./scripts/pmc_calib > $O/cal_hit.log 2>&1
K="python3 scripts/kbench.py --size 536870912 --reps 1 --inputs zero,random,ascii,mixed --msets 1;9;1,3,4,9"
timeout -s KILL 300 rocprofv3 --pmc $C1 --output-format csv -d $O/kb_req -o run -- $K > $O/kb_req.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc $C2 --output-format csv -d $O/kb_hit -o run -- $K > $O/kb_hit.log 2>&1
echo calib2 done
