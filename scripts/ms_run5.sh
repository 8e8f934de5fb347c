#!/bin/bash
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ms_sweep.log
CFGS="4 1024 262144;5 1024 262144;6 1024 262144;5 2048 131072;6 2048 131072;8 2048 131072" bash scripts/ms_sweep.sh
echo "methods 1,2,3,4,5" >> gpurun_out/ms_sweep.log
MS=1,2,3,4,5 CFGS="1 1024 262144;2 1024 262144;2 2048 131072" bash scripts/ms_sweep.sh
