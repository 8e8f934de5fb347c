#!/bin/bash
# Round-6 evidence pass: the GPU suite, the default bench line, rocprofv3 kernel
# stats of the headline step and of the headline / {1,3,4} decodes, FETCH / WRITE /
# read-request PMC passes for the headline (profiles/pmc_r6.json), k_encode SQ
# counters; each GPU step under its own limit
set -e
export TMPDIR=/tmp
O=gpurun_out/${EV_OUT:-r6f}
mkdir -p $O
H="python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods= --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo tests ok
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
echo smoke ok
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stats -o run -- $H --steps 5 --warmup 2 > $O/prof_stats.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dec -o run -- python3 scripts/decode_leg.py 2 > $O/prof_dec.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dec134 -o run -- python3 scripts/decode_leg.py 2 --methods 1,3,4 > $O/prof_dec134.log 2>&1
echo prof ok
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $H --no-verify --steps 2 --warmup 1 > $O/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $H --no-verify --steps 2 --warmup 1 > $O/pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d $O/pmc_req -o run -- $H --no-verify --steps 2 --warmup 1 > $O/pmc_req.log 2>&1
echo pmc ok
