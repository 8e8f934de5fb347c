#!/bin/bash
# k_encode in place at 1 / 2 KiB (AMBC_ENC_GL_MIN=1024) vs LDS-staged, same box
set -e
export TMPDIR=/tmp
O=gpurun_out/gl1k
mkdir -p $O
for r in 1 2; do
  for c in 1024 2048; do
    timeout -k 10 200 python3 bench.py --chunk $c --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --steps 8 --warmup 2 > $O/lds_${c}_$r.json 2> $O/lds_${c}_$r.err
    AMBC_ENC_GL_MIN=1024 timeout -k 10 200 python3 bench.py --chunk $c --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --steps 8 --warmup 2 > $O/gl_${c}_$r.json 2> $O/gl_${c}_$r.err
  done
done
AMBC_ENC_GL_MIN=1024 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "decisions or bodies or edge or tail or golden" > $O/tests.log 2>&1
