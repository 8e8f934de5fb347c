set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rocprofv3 --list-avail > $R/gpurun_out/avail.txt 2>&1 || true
cd $R
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/pmc1 -o run -- python3 scripts/kbench.py --msets 9 --inputs random,ascii --reps 1 > gpurun_out/pmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH -d gpurun_out/pmc2 -o run -- python3 scripts/kbench.py --msets 9 --inputs random,ascii --reps 1 > gpurun_out/pmc2.log 2>&1
