#!/bin/bash
# rocprofv3 kernel stats of this round's large-chunk kernels: k_deflate<32768|65536>
# and k_decode_inflate<65536> (multi-size walk with id 5, its decode), and the
# zlib-9 encoder at 8 KiB chunks (k_z9_*<8192>).
set -e
export TMPDIR=/tmp
O=gpurun_out/big
mkdir -p $O
MS_SETS="mixed:1,3,4,5" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ms5 -o run -- python3 scripts/multisize_bench.py 64 > $O/ms5.jsonl 2> $O/ms5.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/z9 -o run -- python3 scripts/kbench.py --chunk 8192 --flags 2 --msets "1,3,4,5" --inputs zero,random,ascii,mixed --reps 1 > $O/z9.log 2>&1
