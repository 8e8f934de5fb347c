#!/bin/bash
# Round 6: the Huffman decoder rebuild -- its GPU tests, the suite, a bench line
# with the {1,3,4} decode, and a kernel trace of that decode
set -e
export TMPDIR=/tmp
O=gpurun_out/${EV_OUT:-r6h}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_huffdec.py -x -v --timeout 120 --timeout-method thread > $O/huff_tests.log 2>&1
echo huff tests ok
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo suite ok; tail -1 $O/tests.log
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "1,3,4" --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 0 > $O/bench.json 2> $O/bench.err
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dec134 -o run -- python3 scripts/decode_leg.py --methods 1,3,4 > $O/prof_dec134.log 2>&1
echo prof ok
# the reference's full default walk (bz2 / LZMA on host threads): host speculation A/B
FW="python3 bench.py --steps 1 --warmup 0 --no-verify --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods= --walk-bytes 0 --ref-walk-bytes 0 --ref-full-walk-bytes 16777216 --ref-full-walk-check-bytes 1048576"
for hs in 1 0; do
  AMBC_MS_HSPEC=$hs timeout -k 10 300 $FW > $O/fw_hspec$hs.json 2> $O/fw_hspec$hs.err
  echo "fullwalk hspec=$hs ok"
done
