#!/bin/bash
# step time of the headline bench per pipeline setting (AMBC_NSEG / AMBC_CGRID), interleaved
set -e
export TMPDIR=/tmp
for r in 1 2; do
for cfg in "4 1024 AMBC_ONE_ENC_STREAM=1" "4 1024 X=1" "8 1024 X=1" "6 1024 X=1" "5 1024 X=1"; do
  set -- $cfg
  env AMBC_NSEG=$1 AMBC_CGRID=$2 $3 timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 5 --warmup 2 > gpurun_out/seg.json 2>/dev/null
  echo "nseg=$1 cgrid=$2 $3 $(python3 -c "import json; d=json.load(open('gpurun_out/seg.json')); print(d['ms_per_step'], d['value'])")" >> gpurun_out/seg.log
done
done
