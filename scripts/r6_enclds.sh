#!/bin/bash
# same-box A/B: k_encode reading 4 KiB chunks in place (default) vs staged in
# LDS (AMBC_ENC_LDS=1), step time and FETCH_SIZE per k_encode dispatch
set -e
export TMPDIR=/tmp
O=gpurun_out/${EV_OUT:-r6enclds}
mkdir -p $O
H="python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods= --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0"
for r in 1 2; do
  timeout -k 10 200 $H --steps 10 --warmup 3 > $O/gl_$r.json 2> $O/gl_$r.err
  AMBC_ENC_LDS=1 timeout -k 10 200 $H --steps 10 --warmup 3 > $O/lds_$r.json 2> $O/lds_$r.err
done
AMBC_ENC_LDS=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_lds -o run -- $H --no-verify --steps 2 --warmup 1 > $O/fetch_lds.log 2>&1
AMBC_ENC_LDS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_lds -o run -- $H --no-verify --steps 3 --warmup 1 > $O/stats_lds.log 2>&1
echo ok
