#!/bin/bash
# Bench + rocprofv3 kernel trace + separate PMC passes (HBM bytes) for the headline config.
# Usage (on the GPU box): bash scripts/profile_round.sh <tag>
set -e
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
echo "[1/4] bench" && timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
echo "[2/4] kernel trace" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o run -- python bench.py --steps 5 --warmup 1 --cpu-baseline 0 > $OUT/kt.log 2>&1
echo "[3/4] pmc FETCH_SIZE" && timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex prisma_step -f csv -d $OUT/pmc_fetch -o run -- python bench.py --steps 5 --warmup 1 --cpu-baseline 0 > $OUT/pmc_fetch.log 2>&1
echo "[4/4] pmc WRITE_SIZE" && timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex prisma_step -f csv -d $OUT/pmc_write -o run -- python bench.py --steps 5 --warmup 1 --cpu-baseline 0 > $OUT/pmc_write.log 2>&1
find $OUT -name "*.csv" | head -20
echo done
