#!/bin/bash
# Round-3 GPU check: steady-state parity + the whole -m gpu suite, then an A/B of the headline
# bench (driver's 20 steps / 5 warmup, which crosses a 60-s episode end) against a base library.
# Usage: bash scripts/gpu_r03.sh <tag> [base-variant-name]
TAG=${1:-x}
BASE=${2:-base}
mkdir -p gpurun_out
P="python -u -m pytest -x -v --timeout 400 --timeout-method thread"
timeout -k 10 700 $P -s tests/test_gpu_steady_state.py "tests/test_gpu_parity.py::test_episode_end_and_auto_reset" \
    > gpurun_out/steady_$TAG.log 2>&1 && \
timeout -k 10 700 $P -q -m gpu tests > gpurun_out/tests_$TAG.log 2>&1 && \
for i in 1 2; do
  for lib in $BASE new; do
    if [ $lib = new ]; then unset PRISMA_LIB; else export PRISMA_LIB=$PWD/prisma_amd/_ablate/libprisma_amd_$lib.so; fi
    timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 20 --warmup 5 > gpurun_out/ab_${TAG}_${lib}_$i.json || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_${lib}_$i.json')); print('$lib', round(d['value']/1e6,1), 'Mhops/s', round(d['roofline']['kernel_ms'],2), 'ms', 'hops/launch', d['roofline']['hops_per_launch'])"
  done
done
rc=$?
grep -E "steady\]|passed|failed|Error" gpurun_out/steady_$TAG.log | tail -20
tail -3 gpurun_out/tests_$TAG.log
exit $rc
