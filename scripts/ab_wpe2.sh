#!/bin/bash
# base library vs the 8-wave / in-place-from-4-KiB default, chunk sweep, same box
set -e
export TMPDIR=/tmp
O=gpurun_out/wpe2
mkdir -p $O
run() {  # tag lib chunk [env...]
  local t=$1 l=$2 c=$3; shift 3
  env AMBC_LIB=$l "$@" timeout -k 10 200 python3 bench.py --chunk $c --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --steps 10 --warmup 3 > $O/$t.json 2> $O/$t.err
}
for r in 1 2; do
  for c in 4096 1024 2048 8192 16384; do
    run base_${c}_$r ab/lib_base.so $c
    run new8_${c}_$r ab/lib_new8.so $c
  done
  run new8_4096_ldspath_$r ab/lib_new8.so 4096 AMBC_ENC_GL_MIN=99999999
  run new8_4096_cr2048_$r ab/lib_new8.so 4096 AMBC_COMPACT_RESIDENT=2048
  run new8_4096_cr512_$r ab/lib_new8.so 4096 AMBC_COMPACT_RESIDENT=512
done
