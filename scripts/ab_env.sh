#!/bin/bash
# same-box A/B of an environment knob on bench.py legs: REPS interleaved runs with
# and without ENVKV (NAME=value); ARGS overrides the legs (default: headline + the
# walk legs, like_reference included)
set -e
export TMPDIR=/tmp
O=gpurun_out/ab_env${TAG:+_$TAG}
mkdir -p $O
A=${ARGS:---no-e2e --no-verify --alt-methods 1,3,4,5z --steps 2 --warmup 1}
for rep in $(seq 1 ${REPS:-2}); do
  for v in base knob; do
    if [ $v = knob ]; then export ${ENVKV}; else unset ${ENVKV%%=*}; fi
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --api-bytes 0 $A > $O/${v}_$rep.json 2> $O/${v}_$rep.err
    python3 -c "
import json
d=json.loads(open('$O/${v}_$rep.json').read().strip().splitlines()[-1]); c=d['config']
print('$v', $rep, 'head', d['value'], d['ms_per_step'], 'alts', [(a['methods'], a.get('GBps')) for a in c['alt_method_sets']], 'walks', [(w['methods'], w['GBps'], w['walk_ms'], w['final_encode_ms']) for w in c['multisize_walk']], 'lr', (c.get('like_reference_walk') or {}).get('GBps'))
"
  done
done
