#!/bin/bash
# multi-size walk: speculation depth / walk count sweep on 256 MiB mixed input ({1,3,4,9}); the second call is timed
#   CFGS="2 512;1 1024" scripts/ms_sweep.sh   (appends to gpurun_out/ms_sweep.log)
set -e
export TMPDIR=/tmp
IFS=';' read -ra LIST <<< "${CFGS:-2 512;1 512;0 512;1 1024;0 1024;1 2048;0 2048}"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  AMBC_MS_SPEC=$1 AMBC_MS_WALKS=$2 AMBC_MS_SPAN=${3:-524288} timeout -k 10 200 python3 -c "
import sys; sys.argv=['x','256']
sys.path[:0]=['scripts','adaptive-compression_amd','.']
import multisize_bench as m, numpy as np, ambc, time, ctypes as C
data=m.mixed(256<<20,7)
comp=ambc.AdaptiveCompressor(methods=(${MS:-1,3,4,9})); comp.CHUNK_SIZE_CANDIDATES=list(comp.REFERENCE_CHUNK_SIZE_CANDIDATES)
comp._adaptive_compress(data[:1<<20]); comp._adaptive_compress(data); t=time.perf_counter(); b=comp._adaptive_compress(data); dt=time.perf_counter()-t
s,e,w,f=C.c_uint32(),C.c_uint64(),C.c_uint64(),C.c_uint64()
ambc._lib.load().ambc_last_multisize_info(ambc._lib.default_context().h,C.byref(s),C.byref(e),C.byref(w),C.byref(f))
print('spec=$1 walks=$2 span=${3:-524288}', round(dt,4), 'rounds', s.value, 'encodes', e.value, 'walk_ms', w.value/1e6, 'emit_ms', f.value/1e6, len(b))
" >> gpurun_out/ms_sweep.log 2>&1
done
