#!/bin/bash
# Round-6 evidence on the build in tree: smoke, every BASELINE config with its CPU baseline, the
# driver's default bench line, the headline at 8 192 hops per step (round 4's shape), and the
# 8-GPU presets rehearsed as 2 ranks on cuda:0.
TAG=${1:-r06g}
bash scripts/gpu_steps.sh \
  "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()'" \
  "CPU=1 bash scripts/configs.sh > gpurun_out/configs_${TAG}.log 2>&1; rc=\$?; tail -14 gpurun_out/configs_${TAG}.log | cut -c1-220; cp gpurun_out/configs.jsonl gpurun_out/configs_cpu_${TAG}.jsonl; exit \$rc" \
  "timeout -k 10 600 python bench.py > gpurun_out/bench_default_${TAG}.json 2> gpurun_out/bench_default_${TAG}.err; rc=\$?; cut -c1-300 gpurun_out/bench_default_${TAG}.json; exit \$rc" \
  "timeout -k 10 300 python bench.py --hops 8192 --cpu-baseline 0 > gpurun_out/bench_8192_${TAG}.json 2> gpurun_out/bench_8192_${TAG}.err; rc=\$?; cut -c1-200 gpurun_out/bench_8192_${TAG}.json; exit \$rc" \
  "bash scripts/gpu_final.sh rehearse ${TAG}"
