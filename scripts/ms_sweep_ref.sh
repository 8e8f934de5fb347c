#!/bin/bash
# like_reference() walk ({1,2,3,4,5}, id 5 = zlib-9 bytes) on 64 MiB: walks x speculation
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
IFS=';' read -ra LIST <<< "${CFGS:-2 1024 262144;1 1024 262144;0 1024 262144;1 2048 131072;0 4096 65536;1 4096 65536}"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  AMBC_MS_SPEC=$1 AMBC_MS_WALKS=$2 AMBC_MS_SPAN=$3 timeout -k 10 300 python3 -c "
import sys; sys.path[:0]=['scripts','adaptive-compression_amd','.']
import multisize_bench as m, ambc, time, ctypes as C
data=m.mixed(64<<20,7)
comp=ambc.AdaptiveCompressor.like_reference()
comp._adaptive_compress(data[:1<<20]); comp._adaptive_compress(data); t=time.perf_counter(); b=comp._adaptive_compress(data); dt=time.perf_counter()-t
s,e,w,f=C.c_uint32(),C.c_uint64(),C.c_uint64(),C.c_uint64()
ambc._lib.load().ambc_last_multisize_info(ambc._lib.default_context().h,C.byref(s),C.byref(e),C.byref(w),C.byref(f))
print('spec=$1 walks=$2 span=$3', round(dt,4), round(len(data)/dt/1e9,3), 'GB/s rounds', s.value, 'encodes', e.value, 'walk_ms', w.value/1e6, 'emit_ms', f.value/1e6, len(b))
" >> gpurun_out/ms_sweep_ref.log 2>&1
done
