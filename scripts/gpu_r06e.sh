#!/bin/bash
# Round 6: the GPU suite on the build in tree, then A/B of the previous commit (curall) against
# this build (rwlall) on configs 3, 4 (lf 1.0) and 5.
bash scripts/gpu_steps.sh \
  "timeout -k 10 900 python -u -m pytest -q --timeout 600 --timeout-method thread -s -m gpu tests/test_gpu_steady_state.py > gpurun_out/steady_r06e.log 2>&1; rc=\$?; grep -E 'passed|failed' gpurun_out/steady_r06e.log | tail -3; exit \$rc" \
  "timeout -k 10 900 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests --ignore tests/test_gpu_steady_state.py > gpurun_out/tests_r06e.log 2>&1; rc=\$?; tail -3 gpurun_out/tests_r06e.log; exit \$rc" \
  "bash scripts/ab_libs.sh 'curall rwlall' --preset config3 && bash scripts/ab_libs.sh 'curall rwlall' --preset config4 --load-factors 1.0 && bash scripts/ab_libs.sh 'curall rwlall' --preset config5 --warmup 4"
