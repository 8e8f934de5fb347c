#!/bin/bash
# k_encode with the register allocation forced to 6 / 8 waves per SIMD (ab/lib_wpe*.so),
# LDS-staged and in place, against the base library; 4 GiB bench, same box, alternating
set -e
export TMPDIR=/tmp
O=gpurun_out/wpe
mkdir -p $O
run() {  # tag lib chunk glmin
  AMBC_LIB=$2 AMBC_ENC_GL_MIN=$4 timeout -k 10 200 python3 bench.py --chunk $3 --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --steps 10 --warmup 3 > $O/$1.json 2> $O/$1.err
}
for r in 1 2; do
  run base_4k_$r ab/lib_base.so 4096 8192
  run wpe6_4k_lds_$r ab/lib_wpe6.so 4096 8192
  run wpe6_4k_gl_$r ab/lib_wpe6.so 4096 4096
  run wpe8_4k_gl_$r ab/lib_wpe8.so 4096 4096
  run base_8k_$r ab/lib_base.so 8192 8192
  run wpe6_8k_$r ab/lib_wpe6.so 8192 8192
  run wpe8_8k_$r ab/lib_wpe8.so 8192 8192
done
