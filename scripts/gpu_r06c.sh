#!/bin/bash
# Round 6: the trainer's stored generations at 4 096 replicas, and the 8-GPU presets rehearsed as
# 2 ranks on cuda:0 (scripts/gpu_final.sh rehearse) on the build in tree.
TAG=${1:-r06c}
bash scripts/gpu_steps.sh \
  "timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_trainer.py -m gpu > gpurun_out/${TAG}_trainer.log 2>&1; rc=\$?; grep -E 'trainer\\]|passed|failed|Error' gpurun_out/${TAG}_trainer.log | tail -8; exit \$rc" \
  "bash scripts/gpu_final.sh rehearse ${TAG}"
