#!/bin/bash
# 4 KiB chunks: LDS-staged vs in place (AMBC_ENC_GL_MIN=4096), the headline sets
export TMPDIR=/tmp
for rep in 1 2; do
  for mode in lds gl; do
    echo "== $mode"
    if [ $mode = gl ]; then export AMBC_ENC_GL_MIN=4096; else unset AMBC_ENC_GL_MIN; fi
    timeout -k 10 150 python3 scripts/kbench.py --chunk 4096 --msets "9;1,3,4,9;1,3,4" --reps 3 2>&1 | grep -v elapsed || exit 1
  done
done
