#!/bin/bash
# memory-engine parity on the build in tree, then the config-5 A/B of its weight-issue variants
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash scripts/gpu_steps.sh \
  "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()'" \
  "timeout -k 10 600 $P -m gpu tests/test_gpu_mem_engine.py tests/test_gpu_compact.py -s > gpurun_out/mem_r04g.log 2>&1; rc=\$?; grep -E 'compact\\]|passed|failed|Error' gpurun_out/mem_r04g.log | tail -8; exit \$rc" \
  "timeout -k 10 700 $P -s -m gpu tests/test_gpu_steady_state.py -k 'config5 or mem_engine' > gpurun_out/steady_mem_r04g.log 2>&1; rc=\$?; grep -E 'steady\\]|passed|failed|Error' gpurun_out/steady_mem_r04g.log | tail -10; exit \$rc" \
  "timeout -k 10 600 bash scripts/ab_libs.sh \"r04a a0 a1 a3\" --topology er256 --policy dqn_buffer --warmup 13 --steps 10 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_r04g_dqn.txt" \
  "timeout -k 10 300 bash scripts/ab_libs.sh \"r04a a0\" --topology er256 --policy sp --warmup 13 --steps 10 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_r04g_sp.txt"
