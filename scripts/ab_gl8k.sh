#!/bin/bash
# k_encode in place (AMBC_ENC_GL_MIN) vs LDS-staged at 8 KiB (C4's chunk) and 4 KiB, same box, alternating
set -e
export TMPDIR=/tmp
O=gpurun_out/gl8k
mkdir -p $O
for r in 1 2; do
  for c in 8192 4096; do
    timeout -k 10 200 python3 bench.py --chunk $c --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --steps 10 --warmup 3 > $O/lds_${c}_$r.json 2> $O/lds_${c}_$r.err
    AMBC_ENC_GL_MIN=$c timeout -k 10 200 python3 bench.py --chunk $c --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --steps 10 --warmup 3 > $O/gl_${c}_$r.json 2> $O/gl_${c}_$r.err
  done
done
