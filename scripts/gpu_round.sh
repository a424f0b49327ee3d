#!/bin/bash
# GPU tests then bench lines (Abilene headline, GEANT, Abilene DQN-buffer); each GPU step bounded, chained with &&.
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q --timeout=300 > gpurun_out/tests_$TAG.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
timeout -k 10 300 python bench.py --cpu-baseline 0 --topology geant > gpurun_out/bench_geant_$TAG.json 2> gpurun_out/bench_geant_$TAG.err && \
timeout -k 10 300 python bench.py --cpu-baseline 0 --policy dqn_buffer > gpurun_out/bench_dqn_$TAG.json 2> gpurun_out/bench_dqn_$TAG.err
rc=$?
tail -5 gpurun_out/tests_$TAG.log
for f in gpurun_out/bench_$TAG.json gpurun_out/bench_geant_$TAG.json gpurun_out/bench_dqn_$TAG.json; do
  python -c "import json,sys; d=json.load(open('$f')); print(d['config']['workload'][:60], round(d['value']/1e6,1), 'Mhops/s', round(d['roofline']['kernel_ms'],2), 'ms')" 2>/dev/null
done
tail -3 gpurun_out/bench_dqn_$TAG.err
exit $rc
