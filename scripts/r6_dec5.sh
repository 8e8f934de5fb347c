#!/bin/bash
set -e
O=gpurun_out/r6d5
mkdir -p $O
timeout -k 10 300 python3 -u scripts/decode_leg.py 3 --methods 1,3,4,5 > $O/dec1345.log 2>&1
AMBC_TRACE=1 timeout -k 10 300 python3 -u scripts/decode_leg.py 1 --methods 1,3,4,5 > $O/dec1345_trace.log 2>&1
echo ok
