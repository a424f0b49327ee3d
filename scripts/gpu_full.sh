#!/bin/bash
# One GPU call: the whole GPU test suite, one bench line per BASELINE config, and the
# rocprofv3 kernel-trace + PMC passes for the headline (Abilene) and config 5 (ER-256).
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -20 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
bash scripts/configs.sh > gpurun_out/configs_$TAG.log 2>&1 || { tail -20 gpurun_out/configs_$TAG.log; exit 1; }
tail -14 gpurun_out/configs_$TAG.log
bash scripts/profile_round.sh ${TAG} > gpurun_out/prof_${TAG}.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}.log; exit 1; }
bash scripts/profile_round.sh ${TAG}_er256 --topology er256 --policy dqn_buffer --warmup 13 > gpurun_out/prof_${TAG}_er256.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_er256.log; exit 1; }
echo full-done
