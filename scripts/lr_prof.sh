#!/bin/bash
# like_reference() walk ({1,2,3,4,5}, id 5 = zlib-9's bytes, the reference's eight
# candidates) on MIB MiB of multisize_bench's mixed input: timing + walk trace, then
# rocprofv3 kernel stats of the same run.   TAG=r4 MIB=64 scripts/lr_prof.sh
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-lr}
MIB=${MIB:-64}
cat > gpurun_out/lr_one.py <<PYEOF
import sys, time, ctypes as C
sys.path[:0] = ['scripts', 'adaptive-compression_amd', '.']
import multisize_bench as m, ambc
data = m.mixed($MIB << 20, 7)
comp = ambc.AdaptiveCompressor.like_reference()
comp._adaptive_compress(data[:1 << 20])
for _ in range(2):
    t = time.perf_counter(); b = comp._adaptive_compress(data); dt = time.perf_counter() - t
    s, e, w, f = C.c_uint32(), C.c_uint64(), C.c_uint64(), C.c_uint64()
    ambc._lib.load().ambc_last_multisize_info(ambc._lib.default_context().h, C.byref(s), C.byref(e), C.byref(w), C.byref(f))
    print('walk', round(dt, 4), 's', round(len(data) / dt / 1e9, 3), 'GB/s', len(b), 'rounds', s.value,
          'encodes', e.value, 'walk_ms', w.value / 1e6, 'emit_ms', f.value / 1e6, flush=True)
PYEOF
AMBC_TRACE=1 timeout -k 10 300 python3 gpurun_out/lr_one.py > gpurun_out/${TAG}_lr_trace.log 2>&1
[ -n "$NOPROF" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_lr_prof -o run -- \
    python3 gpurun_out/lr_one.py > gpurun_out/${TAG}_lr_prof.log 2>&1
