#!/bin/bash
# Round-5 evidence pass: the GPU suite, the default bench line, rocprofv3 kernel
# stats of the headline, FETCH / WRITE passes (HBM traffic) and the TCC read
# requests by size (calibration: profiles/r5_pmc_calibration.json), and
# k_encode's SQ counters per input class; each GPU step under its own limit
set -e
export TMPDIR=/tmp
O=gpurun_out/${EV_OUT:-r5f}
mkdir -p $O
H="python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods= --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo tests ok
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stats -o run -- $H --steps 5 --warmup 2 > $O/prof_stats.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $H --no-verify --steps 2 --warmup 1 > $O/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $H --no-verify --steps 2 --warmup 1 > $O/pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d $O/pmc_req -o run -- $H --no-verify --steps 2 --warmup 1 > $O/pmc_req.log 2>&1
echo pmc ok
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/sq_enc1 -o run -- python3 scripts/kbench.py --msets "1,3,4,9" --inputs random,ascii,mixed --reps 1 > $O/sq_enc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH --output-format csv -d $O/sq_enc2 -o run -- python3 scripts/kbench.py --msets "1,3,4,9" --inputs random,ascii,mixed --reps 1 > $O/sq_enc2.log 2>&1
echo sq ok
