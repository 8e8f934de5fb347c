#!/bin/bash
# the 8-wave encoder's step: segments x compaction stream priority, same box; plus a kernel trace
set -e
export TMPDIR=/tmp
O=gpurun_out/seg8
mkdir -p $O
run() {  # tag [env...]
  local t=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --steps 10 --warmup 3 > $O/$t.json 2> $O/$t.err
}
for r in 1 2; do
  run d_$r AMBC_X=0
  run prio_$r AMBC_CS_PRIO=1
  run s5_$r AMBC_NSEG=5
  run s6_$r AMBC_NSEG=6
  run s3_$r AMBC_NSEG=3
  run s6prio_$r AMBC_NSEG=6 AMBC_CS_PRIO=1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --walk-bytes 0 --no-verify --steps 3 --warmup 1 > $O/trace.log 2>&1
