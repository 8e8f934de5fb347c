#!/bin/bash
# decode host API across the bench's legs: 2 MiB page advice on the output
# (default) vs none (AMBC_NO_HUGEPAGE=1) vs 16 prefault threads, alternating
# processes on one box; the box's THP settings and memory state first
set -e
O=gpurun_out/${EV_OUT:-r6thp}
mkdir -p $O
{ cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag \
      /sys/kernel/mm/transparent_hugepage/khugepaged/defrag 2>&1; grep -E "MemTotal|MemFree|MemAvailable|AnonHugePages|HugePages_|Hugepagesize" /proc/meminfo; nproc; } > $O/sys.txt 2>&1 || true
B="python3 -u bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 --steps 2 --warmup 1 --alt-methods 1,3,4;1,3,4,5;1,2,3,4"
for r in 1 2; do
  timeout -k 10 300 $B > $O/base_$r.json 2> $O/base_$r.err
  AMBC_NO_HUGEPAGE=1 timeout -k 10 300 $B > $O/nohp_$r.json 2> $O/nohp_$r.err
  AMBC_PREP_THREADS=16 timeout -k 10 300 $B > $O/p16_$r.json 2> $O/p16_$r.err
done
grep -E "AnonHugePages|MemFree" /proc/meminfo > $O/mem_after.txt || true
echo ok
