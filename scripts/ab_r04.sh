#!/bin/bash
# A/B of the library in tree against prisma_amd/_ablate/libprisma_amd_<base>.so on one box:
# config 5 (ER-256 DQN-buffer, 1 024 replicas, warmed past the flow-start transient), config 4
# (GEANT DQN-buffer, 2 048) and the headline (driver's 20 steps / 5 warmup), two rounds.
TAG=${1:-x}
BASE=${2:-base}
for i in 1 2; do
  for lib in $BASE new; do
    if [ $lib = new ]; then unset PRISMA_LIB; else export PRISMA_LIB=$PWD/prisma_amd/_ablate/libprisma_amd_$lib.so; fi
    for cfg in "--topology er256 --policy dqn_buffer --warmup 13 --steps 10" \
               "--topology geant --policy dqn_buffer --ping-as-obs 0 --replicas 2048 --steps 10 --warmup 2" \
               "--steps 20 --warmup 5"; do
      timeout -k 10 300 python bench.py --cpu-baseline 0 $cfg > gpurun_out/ab.json || exit 1
      python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$TAG $lib', '$cfg'[:28], round(d['value']/1e6,2), 'Mhops/s', round(d['roofline']['kernel_ms'],2), 'ms', 'err', d['errors'])" | tee -a gpurun_out/ab_$TAG.txt
    done
  done
done
