#!/bin/bash
# In-place (GL) vs LDS-staged k_encode for large chunks, same box, A B A B:
#   scripts/ab_gl.sh > gpurun_out/ab_gl.log
export TMPDIR=/tmp
for rep in 1 2; do
  for mode in lds gl; do
    for c in 16384 65536; do
      echo "== $mode chunk $c"
      if [ $mode = lds ]; then export AMBC_ENC_LDS=1; else unset AMBC_ENC_LDS; fi
      timeout -k 10 150 python3 scripts/kbench.py --chunk $c --msets "9;1,3,4,9" --reps 3 2>&1 | grep -v elapsed || exit 1
    done
  done
done
unset AMBC_ENC_LDS
for mode in lds gl; do
  echo "== multisize $mode"
  if [ $mode = lds ]; then export AMBC_ENC_LDS=1; else unset AMBC_ENC_LDS; fi
  AMBC_TRACE=1 MS_SETS="mixed:1,3,4,9;mixed:1,2,3,4,5" timeout -k 10 300 python3 scripts/multisize_bench.py 256 2>&1 | tail -30 || exit 1
done
