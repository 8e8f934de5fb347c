#!/bin/bash
set -e
O=gpurun_out/r6hd
mkdir -p $O
timeout -k 10 120 python3 -u scripts/r6_huffdbg.py > $O/route_default2.log 2>&1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_huffdec.py -x -q --timeout 120 --timeout-method thread > $O/huff_tests2.log 2>&1
echo ok
