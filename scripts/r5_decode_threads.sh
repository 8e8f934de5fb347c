#!/bin/bash
# Decode host-API A/B over the staging thread count (AMBC_HOST_THREADS unset / 8 / 12 / 24):
# the headline bench with the other host legs off, twice each, each run under its own limit
set -e
O=gpurun_out/r5dt
mkdir -p $O
H="python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods= --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --steps 3 --warmup 1"
for rep in 1 2; do
  timeout -k 10 240 $H > $O/def_$rep.json 2> $O/def_$rep.err
  for t in 8 12 24; do
    AMBC_HOST_THREADS=$t timeout -k 10 240 $H > $O/t${t}_$rep.json 2> $O/t${t}_$rep.err
  done
  echo rep $rep ok
done
