#!/bin/bash
# Round-5 config-5 experiment: parity of a memory-engine variant (its DQN-buffer tests against the
# oracle) and an A/B of two variants on config 5.  Usage: bash scripts/r05_ab.sh <tag> <candidate> "<A/B libs>" [configs]
set -e
TAG=$1; CAND=$2; LIBS=$3; CFG=${4:-er256_dqn}
mkdir -p gpurun_out/$TAG
export PRISMA_LIB=$PWD/prisma_amd/_ablate/libprisma_amd_$CAND.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_mem_engine.py -x -q -m gpu --timeout 300 --timeout-method thread \
  -k "dqn or mem_table or equals" > gpurun_out/$TAG/mem_tests_$CAND.log 2>&1 || { tail -30 gpurun_out/$TAG/mem_tests_$CAND.log; exit 1; }
tail -2 gpurun_out/$TAG/mem_tests_$CAND.log
if [ -n "$STEADY" ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_steady_state.py -x -q -m gpu --timeout 400 --timeout-method thread \
    -k "$STEADY" > gpurun_out/$TAG/steady_$CAND.log 2>&1 || { tail -30 gpurun_out/$TAG/steady_$CAND.log; exit 1; }
  tail -2 gpurun_out/$TAG/steady_$CAND.log
fi
unset PRISMA_LIB
AB_NO_NEW=1 AB_CONFIGS="$CFG" bash scripts/gpu_ab.sh $TAG "$LIBS" 10 13 2>&1 | tee gpurun_out/$TAG/ab.txt
