#!/bin/bash
# round 4: SQ counters of the zlib-9 parse kernels (k_z9_parse at 4 KiB, k_z9_parse_big
# at 64 KiB) per input class, two passes each (rocprofv3 does not split passes).
#   TAG=r4 scripts/z9_sq_r4.sh   -> gpurun_out/${TAG}z9sq/{sq4k1,sq4k2,sq64k1,sq64k2}
set -e
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4}z9sq
mkdir -p $O
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"
for C in 4096 65536; do
  MS=$([ $C = 4096 ] && echo "1,3,4,5" || echo "5")
  timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $O/sq${C}_1 -o run -- \
      python3 scripts/kbench.py --size $((64 << 20)) --chunk $C --flags 2 --msets "$MS" --inputs ascii,mixed --reps 1 > $O/sq${C}_1.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $P2 --output-format csv -d $O/sq${C}_2 -o run -- \
      python3 scripts/kbench.py --size $((64 << 20)) --chunk $C --flags 2 --msets "$MS" --inputs ascii,mixed --reps 1 > $O/sq${C}_2.log 2>&1
done
