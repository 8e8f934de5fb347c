#!/bin/bash
# Same-box A/B of the shipped library against the experiment build
# (libambc_hip_exp.so): kbench per input class, alternating A B A B.
#   KB_ARGS="--flags 2 --msets 1,3,4,5" scripts/ab_lib.sh > gpurun_out/ab.log
export TMPDIR=/tmp
for L in libambc_hip libambc_hip_exp libambc_hip libambc_hip_exp; do
  echo "== $L"
  AMBC_LIB=adaptive-compression_amd/ambc/$L.so timeout -k 10 150 python3 scripts/kbench.py $KB_ARGS --reps 3 2>&1 | grep -v elapsed || exit 1
done
