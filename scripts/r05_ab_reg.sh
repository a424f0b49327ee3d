#!/bin/bash
# Round-5 register-engine MLP experiment: DQN-buffer parity of a variant (its GPU parity tests and a
# config-4 steady-state run against the oracle), then an A/B on configs 3 and 4.
# Usage: bash scripts/r05_ab_reg.sh <tag> <candidate> "<A/B libs>"
set -e
TAG=$1; CAND=$2; LIBS=$3
mkdir -p gpurun_out/$TAG
export PRISMA_LIB=$PWD/prisma_amd/_ablate/libprisma_amd_$CAND.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_steady_state.py -x -q -m gpu --timeout 400 \
  --timeout-method thread -k "dqn or mlp" > gpurun_out/$TAG/reg_tests_$CAND.log 2>&1 || { tail -30 gpurun_out/$TAG/reg_tests_$CAND.log; exit 1; }
tail -2 gpurun_out/$TAG/reg_tests_$CAND.log
unset PRISMA_LIB
AB_NO_NEW=1 AB_CONFIGS="${CFG:-geant_dqn aog_dqn}" bash scripts/gpu_ab.sh $TAG "$LIBS" 10 2 2>&1 | tee gpurun_out/$TAG/ab.txt
