#!/bin/bash
# Round-4 memory-engine check: smoke, memory-engine parity (unit, steady state, compaction), the
# rest of the GPU suite, config-5 phase timing with wait probes, then an A/B of config 5 and the
# headline against a base library (prisma_amd/_ablate/libprisma_amd_<base>.so).
# Usage: bash scripts/gpu_r04_mem.sh <tag> <base>
TAG=${1:-x}
BASE=${2:-r04a}
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash scripts/gpu_steps.sh \
  "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()'" \
  "timeout -k 10 600 $P -m gpu tests/test_gpu_mem_engine.py tests/test_gpu_compact.py -s > gpurun_out/mem_$TAG.log 2>&1; rc=\$?; grep -E 'compact\\]|passed|failed|Error' gpurun_out/mem_$TAG.log | tail -8; exit \$rc" \
  "timeout -k 10 700 $P -s -m gpu tests/test_gpu_steady_state.py -k 'config5 or mem_engine' > gpurun_out/steady_mem_$TAG.log 2>&1; rc=\$?; grep -E 'steady\\]|passed|failed|Error' gpurun_out/steady_mem_$TAG.log | tail -10; exit \$rc" \
  "timeout -k 10 700 $P -m gpu tests --ignore tests/test_gpu_steady_state.py --ignore tests/test_gpu_mem_engine.py --ignore tests/test_gpu_compact.py > gpurun_out/tests_$TAG.log 2>&1; rc=\$?; tail -3 gpurun_out/tests_$TAG.log; exit \$rc" \
  "timeout -k 10 300 python scripts/timing.py run --topology er256 --replicas 1024 --hops 8192 --policy dqn_buffer --warm 13 > gpurun_out/timing_er256_$TAG.txt 2>&1; rc=\$?; cat gpurun_out/timing_er256_$TAG.txt; exit \$rc" \
  "bash scripts/ab_r04.sh $TAG $BASE"
