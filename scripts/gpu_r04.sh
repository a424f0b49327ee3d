#!/bin/bash
# Round-4 GPU check: the memory-engine long-run / episode-end parity tests and the steady-state
# suite (printing "compared up to t = ..."), the whole -m gpu suite, then one bench line per
# BASELINE config (scripts/configs.sh) and an A/B of configs 2/4 against a base library.
# Usage: bash scripts/gpu_r04.sh <tag> [base-variant-name]
TAG=${1:-x}
BASE=${2:-base}
mkdir -p gpurun_out
P="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 900 $P -s tests/test_gpu_steady_state.py > gpurun_out/steady_$TAG.log 2>&1 || { grep -E "steady\]|PASS|FAIL|Error|differs" gpurun_out/steady_$TAG.log | tail -30; exit 1; }
grep -E "steady\]" gpurun_out/steady_$TAG.log
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    --ignore tests/test_gpu_steady_state.py > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
if [ "$3" = tests ]; then
  timeout -k 10 300 python scripts/timing.py run --topology er256 --replicas 1024 --hops 8192 --policy dqn_buffer --warm 13 > gpurun_out/timing_er256_$TAG.txt 2>&1 || { tail -20 gpurun_out/timing_er256_$TAG.txt; exit 1; }
  cat gpurun_out/timing_er256_$TAG.txt
  exit 0
fi
bash scripts/configs.sh > gpurun_out/configs_$TAG.log 2>&1 || { tail -20 gpurun_out/configs_$TAG.log; exit 1; }
tail -14 gpurun_out/configs_$TAG.log
cp gpurun_out/configs.jsonl gpurun_out/configs_$TAG.jsonl
for i in 1 2; do
  for lib in $BASE new; do
    if [ $lib = new ]; then unset PRISMA_LIB; else export PRISMA_LIB=$PWD/prisma_amd/_ablate/libprisma_amd_$lib.so; fi
    for cfg in "" "--topology geant --policy dqn_buffer --ping-as-obs 0 --replicas 2048"; do
      timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 10 --warmup 2 $cfg > gpurun_out/ab.json || exit 1
      python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$lib', '$cfg'[:20], round(d['value']/1e6,1), 'Mhops/s', round(d['roofline']['kernel_ms'],2), 'ms')"
    done
  done
done
