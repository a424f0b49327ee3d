#!/bin/bash
# Bench + rocprofv3 kernel trace + separate PMC passes (HBM bytes, SQ mix) for the headline config.
# Usage (on the GPU box): bash scripts/profile_round.sh <tag> [extra bench args]
set -e
TAG=${1:-r01}
shift || true
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT/sq
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="python bench.py --steps 5 --warmup 1 --cpu-baseline 0 $*"
echo "[1/7] bench" && timeout -k 10 400 python bench.py $* > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
echo "[2/7] kernel trace" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o run -- $B > $OUT/kt.log 2>&1
echo "[3/7] pmc FETCH_SIZE" && timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex step_kernel -f csv -d $OUT/pmc_fetch -o run -- $B > $OUT/pmc_fetch.log 2>&1
echo "[4/7] pmc WRITE_SIZE" && timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex step_kernel -f csv -d $OUT/pmc_write -o run -- $B > $OUT/pmc_write.log 2>&1
echo "[5/7] SQ mix" && timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH --kernel-include-regex step_kernel -f csv -d $OUT/sq/a -o run -- $B > $OUT/sq_a.log 2>&1
echo "[6/7] SQ stalls" && timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex step_kernel -f csv -d $OUT/sq/b -o run -- $B > $OUT/sq_b.log 2>&1
echo "[7/7] SQ misc" && timeout -k 10 400 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex step_kernel -f csv -d $OUT/sq/c -o run -- $B > $OUT/sq_c.log 2>&1
find $OUT -name "*.csv" | head -20
echo done
