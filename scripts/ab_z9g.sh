#!/bin/bash
# A/B of the zlib-9 walkers' lanes per walker (G) and waves per 4 KiB chunk:
# parity (test_gpu_zlib9.py) per variant, then the {1,3,4,5z} alt leg's kernel time
# per input class (kbench, 256 MiB, chunk 4096, AMBC_FLAG_ZLIB9), interleaved.
set -e
export TMPDIR=/tmp
O=gpurun_out/ab_z9g
mkdir -p $O
V=${VARIANTS:-"base g4 g2 g4nw4"}
for v in $V; do
  L=adaptive-compression_amd/ambc/libambc_hip.so; [ $v != base ] && L=adaptive-compression_amd/ambc/libambc_hip_$v.so
  AMBC_LIB=$L timeout -k 10 300 python3 -u -m pytest tests/test_gpu_zlib9.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/test_$v.log 2>&1
  tail -1 $O/test_$v.log
done
for rep in 1 2; do
  for v in $V; do
    L=adaptive-compression_amd/ambc/libambc_hip.so; [ $v != base ] && L=adaptive-compression_amd/ambc/libambc_hip_$v.so
    AMBC_LIB=$L timeout -k 10 200 python3 scripts/kbench.py --flags 2 --msets "1,3,4,5" --reps 3 > $O/kb_${v}_$rep.log 2>&1
    echo "$v rep $rep: $(python3 -c "
import json
for l in open('$O/kb_${v}_$rep.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['input'], d['encode_ms'], end='; ')
")"
  done
done
# the big kernels: 64 KiB chunks of the walk's mixed input and the synthetic classes
for rep in 1 2; do
  for v in $V; do
    L=adaptive-compression_amd/ambc/libambc_hip.so; [ $v != base ] && L=adaptive-compression_amd/ambc/libambc_hip_$v.so
    AMBC_LIB=$L Z9_CHUNKS=16384,65536 timeout -k 10 200 python3 scripts/z9_stamps_ms.py > $O/big_${v}_$rep.log 2>&1
    echo "$v big rep $rep: $(grep encode $O/big_${v}_$rep.log | sed 's/: encode / /; s/ ms, ratio.*//' | tr '\n' ';')"
  done
done
