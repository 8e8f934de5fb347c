#!/bin/bash
# same-box A/B of an environment knob on the walk legs of bench.py (like_reference,
# {1,3,4,9}, {1,2,3,4,5}): REPS interleaved runs with and without ENVKV (NAME=value)
set -e
export TMPDIR=/tmp
O=gpurun_out/ab_env
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for v in base knob; do
    if [ $v = knob ]; then export ${ENVKV}; else unset ${ENVKV%%=*}; fi
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --no-verify --alt-methods "" --steps 2 --warmup 1 > $O/${v}_$rep.json 2> $O/${v}_$rep.err
    python3 -c "
import json
d=json.loads(open('$O/${v}_$rep.json').read().strip().splitlines()[-1]); c=d['config']
print('$v', $rep, 'walks', [(w['methods'], w['GBps'], w['walk_ms']) for w in c['multisize_walk']], 'lr', c['like_reference_walk']['GBps'], c['like_reference_walk']['walk_ms'])
"
  done
done
