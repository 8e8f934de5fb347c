#!/bin/bash
# Round-2 counter collection (each rocprofv3 --pmc pass its own run, SQ passes
# within the per-block limits):
#   traffic   FETCH_SIZE / WRITE_SIZE of every kernel of the headline bench
#   sq_enc    SQ instruction mix of k_encode per input class ({1,3,4,9})
#   sq_alt    the same for k_deflate / k_dict ({1,3,4,5}, {1,2,3,4})
#   sq_dec    k_decode_inflate / k_decode / k_decode_lz4 from scripts/dbench.py
#   stamps    per-phase s_memtime cycles of k_encode (diagnostic library)
set -e
export TMPDIR=/tmp
O=gpurun_out/r2
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods '' --no-verify --steps 2 --warmup 1"
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
SQ2="SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"
run() {  # name, counters, command...
    local name=$1 ctr=$2; shift 2
    timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d $O/$name -o run -- "$@" > $O/$name.log 2>&1
}
run fetch "FETCH_SIZE" python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 2 --warmup 1
run write "WRITE_SIZE" python3 bench.py --no-cpu-baseline --api-bytes 0 --no-e2e --alt-methods "" --no-verify --steps 2 --warmup 1
run sq_enc1 "$SQ1" python3 scripts/kbench.py --msets "1,3,4,9" --inputs random,ascii,mixed --reps 1
run sq_enc2 "$SQ2" python3 scripts/kbench.py --msets "1,3,4,9" --inputs random,ascii,mixed --reps 1
run sq_alt1 "$SQ1" python3 scripts/kbench.py --msets "1,3,4,5;1,2,3,4" --inputs ascii,mixed --reps 1
run sq_alt2 "$SQ2" python3 scripts/kbench.py --msets "1,3,4,5;1,2,3,4" --inputs ascii,mixed --reps 1
run sq_dec1 "$SQ1" python3 scripts/dbench.py --size 67108864 --methods 1,3,4,5 --reps 1
run sq_dec2 "$SQ2" python3 scripts/dbench.py --size 67108864 --methods 1,3,4,5 --reps 1
run sq_decd1 "$SQ1" python3 scripts/dbench.py --size 67108864 --methods 1,2,3,4 --reps 1
run sq_decd2 "$SQ2" python3 scripts/dbench.py --size 67108864 --methods 1,2,3,4 --reps 1
AMBC_STAMPS=1 AMBC_LIB=adaptive-compression_amd/ambc/libambc_hip_stamps.so timeout -k 10 120 \
    python3 scripts/kbench.py --msets "1,3,4,9" --reps 1 > $O/stamps.log 2>&1
timeout -k 10 120 python3 scripts/kbench.py --reps 3 > $O/kbench.log 2>&1
