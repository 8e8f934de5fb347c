#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration per access width (scripts/pmc_calib.hip),
# then the same two counters on k_encode per input class x method set (kbench)
set -e
export TMPDIR=/tmp
O=gpurun_out/r5cal
mkdir -p $O
timeout -k 10 60 ./scripts/pmc_calib > $O/calib_plain.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/cal_fetch -o run -- ./scripts/pmc_calib > $O/cal_fetch.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/cal_write -o run -- ./scripts/pmc_calib > $O/cal_write.log 2>&1
K="python3 scripts/kbench.py --size 536870912 --reps 2 --inputs zero,random,ascii,mixed --msets 1;9;1,3,4,9"
timeout -k 10 300 $K --out $O/kbench_plain.json > $O/kbench_plain.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/kb_fetch -o run -- $K > $O/kb_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/kb_write -o run -- $K > $O/kb_write.log 2>&1
echo calib done
