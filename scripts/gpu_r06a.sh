#!/bin/bash
# Round 6, first GPU call: smoke, the new episode-end / bench-shape parity tests, the tunnelled-
# overlay tests, then the BASELINE config lines (no CPU baseline) on this build.
bash scripts/gpu_steps.sh \
  "timeout -k 10 300 python -c \"import __graft_entry__ as g; g.smoke()\"" \
  "timeout -k 10 700 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_steady_state.py -k \"bench_shape or episode_end or short_episodes\" > gpurun_out/r06a_steady.log 2>&1; rc=\$?; grep -E \"steady\\]|passed|failed|Error|assert\" gpurun_out/r06a_steady.log | tail -20; exit \$rc" \
  "timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k tunnel > gpurun_out/r06a_tun.log 2>&1; rc=\$?; tail -4 gpurun_out/r06a_tun.log; exit \$rc" \
  "bash scripts/configs.sh > gpurun_out/configs_r06a.log 2>&1; rc=\$?; tail -9 gpurun_out/configs_r06a.log; cp gpurun_out/configs.jsonl gpurun_out/configs_r06a.jsonl; exit \$rc"
