#!/bin/bash
# Same-box A/B of the compaction grid size beside the encoder (AMBC_COMPACT_RESIDENT).
set -e
export TMPDIR=/tmp
O=gpurun_out/res
mkdir -p $O
for r in 1 2; do
  for R in 256 512 1024 2048; do
    AMBC_COMPACT_RESIDENT=$R timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 10 --warmup 2 > $O/r${R}_$r.json 2>/dev/null
  done
done
