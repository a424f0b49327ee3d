#!/bin/bash
# GPU tests then bench lines (Abilene headline + GEANT); each GPU step bounded, chained with &&.
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q --timeout=300 > gpurun_out/tests_$TAG.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
timeout -k 10 300 python bench.py --cpu-baseline 0 --topology geant > gpurun_out/bench_geant_$TAG.json 2> gpurun_out/bench_geant_$TAG.err
rc=$?
tail -5 gpurun_out/tests_$TAG.log; cat gpurun_out/bench_$TAG.json gpurun_out/bench_geant_$TAG.json; tail -5 gpurun_out/bench_$TAG.err
exit $rc
