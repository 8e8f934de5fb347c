#!/bin/bash
# same-box A/B of the shipped library against one experiment build (AMBC_LIB):
# bench.py legs given in ARGS, REPS interleaved runs each.
#   EXP=noprune ARGS='--alt-methods 1,3,4,5z ...' scripts/ab_lib.sh
set -e
export TMPDIR=/tmp
O=gpurun_out/ab_${EXP}
mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
  for v in base $EXP; do
    L=adaptive-compression_amd/ambc/libambc_hip.so; [ $v != base ] && L=adaptive-compression_amd/ambc/libambc_hip_$v.so
    AMBC_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --no-verify $ARGS > $O/${v}_$rep.json 2> $O/${v}_$rep.err
    python3 -c "
import json,sys
d=json.loads(open('$O/${v}_$rep.json').read().strip().splitlines()[-1])
c=d['config']
print('$v', $rep, 'head', d['value'], 'alts', [(a['methods'], a.get('GBps')) for a in c['alt_method_sets']], 'walks', [w['GBps'] for w in c['multisize_walk']], 'lr', (c.get('like_reference_walk') or {}).get('GBps'))
"
  done
done
