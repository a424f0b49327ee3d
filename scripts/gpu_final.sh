#!/bin/bash
# Round-end GPU evidence on the build in tree, in three calls (each within gpurun's 20 min):
#   bash scripts/gpu_final.sh tests <tag>    smoke, the whole -m gpu suite, one bench line per BASELINE config
#   bash scripts/gpu_final.sh prof1 <tag>    rocprofv3 kernel trace + PMC passes: headline, config 5
#   bash scripts/gpu_final.sh prof2 <tag>    the same for configs 3 and 4
#   bash scripts/gpu_final.sh rehearse <tag> the 8-GPU presets (config 4 sweep, config 5) as 2 ranks on cuda:0
STAGE=$1
TAG=${2:-x}
P="python -u -m pytest -q --timeout 600 --timeout-method thread"
case $STAGE in
tests)
  bash scripts/gpu_steps.sh \
    "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()'" \
    "timeout -k 10 900 $P -s -m gpu tests/test_gpu_steady_state.py > gpurun_out/steady_$TAG.log 2>&1; rc=\$?; grep -E 'steady\\]|passed|failed' gpurun_out/steady_$TAG.log | tail -20; exit \$rc" \
    "timeout -k 10 900 $P -s -m gpu tests --ignore tests/test_gpu_steady_state.py > gpurun_out/tests_$TAG.log 2>&1; rc=\$?; grep -E 'compact\\]|passed|failed' gpurun_out/tests_$TAG.log | tail -6; exit \$rc" \
    "bash scripts/configs.sh > gpurun_out/configs_$TAG.log 2>&1; rc=\$?; tail -14 gpurun_out/configs_$TAG.log; cp gpurun_out/configs.jsonl gpurun_out/configs_$TAG.jsonl; exit \$rc"
  ;;
prof1)
  bash scripts/gpu_steps.sh \
    "timeout -k 10 550 bash scripts/profile_round.sh ${TAG} > gpurun_out/prof_${TAG}.log 2>&1; rc=\$?; tail -4 gpurun_out/prof_${TAG}.log; exit \$rc" \
    "timeout -k 10 550 bash scripts/profile_round.sh ${TAG}_er256 --preset config5 --warmup 4 --cpu-baseline 0 > gpurun_out/prof_${TAG}_er256.log 2>&1; rc=\$?; tail -4 gpurun_out/prof_${TAG}_er256.log; exit \$rc"
  ;;
prof2)
  bash scripts/gpu_steps.sh \
    "timeout -k 10 550 bash scripts/profile_round.sh ${TAG}_aog --preset config3 --cpu-baseline 0 > gpurun_out/prof_${TAG}_aog.log 2>&1; rc=\$?; tail -4 gpurun_out/prof_${TAG}_aog.log; exit \$rc" \
    "timeout -k 10 550 bash scripts/profile_round.sh ${TAG}_geant_mlp --preset config4 --load-factors 1.0 --cpu-baseline 0 > gpurun_out/prof_${TAG}_geant_mlp.log 2>&1; rc=\$?; tail -4 gpurun_out/prof_${TAG}_geant_mlp.log; exit \$rc"
  ;;
rehearse)
  B="python bench.py --gpus 2 --same-device --steps 3 --warmup 1 --cpu-baseline 0"
  bash scripts/gpu_steps.sh \
    "timeout -k 10 400 $B --preset config4 --replicas 256 > gpurun_out/rehearse_${TAG}_config4.jsonl 2> gpurun_out/rehearse_${TAG}_config4.err; rc=\$?; cut -c1-200 gpurun_out/rehearse_${TAG}_config4.jsonl; exit \$rc" \
    "timeout -k 10 400 $B --preset config5 --replicas 128 --warmup 2 > gpurun_out/rehearse_${TAG}_config5.jsonl 2> gpurun_out/rehearse_${TAG}_config5.err; rc=\$?; cut -c1-200 gpurun_out/rehearse_${TAG}_config5.jsonl; exit \$rc"
  ;;
esac
