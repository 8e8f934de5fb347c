#!/bin/bash
# end-of-session check: smoke(), the GPU suite, the default bench line
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/final/gputest.log 2>&1
timeout -k 10 500 python3 -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err
