#!/bin/bash
# zlib-9 parse at 4 KiB with 16 waves per chunk (128 walkers, 32 bytes each) against
# 8 (64 walkers): parity of the variant against the system zlib, then a same-box
# kbench A/B at chunk 4096 (the bench's zlib-9 method set).
set -e
export TMPDIR=/tmp
O=gpurun_out/z9nw4k
mkdir -p $O
AMBC_LIB=ab/lib_nw16_4k.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_zlib9.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2; do
  for L in ab/lib_base.so ab/lib_nw16_4k.so; do
    echo "== $L" >> $O/ab.log
    AMBC_LIB=$L timeout -k 10 200 python3 scripts/kbench.py --chunk 4096 --flags 2 --msets "1,3,4,5" --inputs zero,random,ascii,mixed --reps 2 >> $O/ab.log 2>&1
  done
done
