#!/bin/bash
# AMBC_TRACE host breakdown of the walk legs, with and without ENVKV
set -e
export TMPDIR=/tmp
O=gpurun_out/wtab
mkdir -p $O
for v in base knob; do
  if [ $v = knob ]; then export ${ENVKV}; else unset ${ENVKV%%=*}; fi
  AMBC_TRACE=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --no-verify --size 268435456 \
      --alt-methods 1,3,4 --ref-walk-bytes 0 --steps 1 --warmup 1 > $O/$v.json 2> $O/$v.err
  echo "== $v"; grep "multisize walk ms" $O/$v.err
done
