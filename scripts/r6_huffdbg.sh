#!/bin/bash
set -e
O=gpurun_out/r6hd
mkdir -p $O
timeout -k 10 120 python3 -u scripts/r6_huffdbg.py > $O/route_default.log 2>&1
AMBC_HUFF_ROUTE=8 timeout -k 10 120 python3 -u scripts/r6_huffdbg.py > $O/route_8.log 2>&1
AMBC_HUFF_ROUTE=0 timeout -k 10 120 python3 -u scripts/r6_huffdbg.py > $O/route_0.log 2>&1
echo ok
