#!/bin/bash
# A/B of the working tree's library against prebuilt variants (prisma_amd/_ablate/libprisma_amd_<name>.so),
# alternating on one box, over several bench configurations.  Each line: lib, config, Mhops/s, kernel ms,
# hops per launch.  Usage: bash scripts/gpu_ab.sh <tag> "<variants>" [steps warmup]
TAG=${1:-x}
VARS=${2:-base}
STEPS=${3:-20}
WARM=${4:-5}
mkdir -p gpurun_out
CONFIGS=("headline|" "geant_dqn|--topology geant --policy dqn_buffer --ping-as-obs 0 --replicas 2048"
         "aog_dqn|--topology abilene_on_geant --policy dqn_buffer")
# AB_CONFIGS="name ..." picks a subset; er256_dqn / er256_sp are config 5 (warmed past the transient)
CONFIGS+=("er256_dqn|--topology er256 --policy dqn_buffer --warmup 13" "er256_sp|--topology er256 --policy sp --warmup 13")
if [ -n "$AB_CONFIGS" ]; then
  SEL=()
  for c in "${CONFIGS[@]}"; do for n in $AB_CONFIGS; do [ "${c%%|*}" = "$n" ] && SEL+=("$c"); done; done
  CONFIGS=("${SEL[@]}")
fi
for i in 1 2; do
  for c in "${CONFIGS[@]}"; do
    name=${c%%|*}; args=${c#*|}
    # AB_NO_NEW=1: variants only (the working tree's sources no longer match the in-tree library)
    for lib in $VARS $([ -n "$AB_NO_NEW" ] || echo new); do
      if [ $lib = new ]; then unset PRISMA_LIB; else export PRISMA_LIB=$PWD/prisma_amd/_ablate/libprisma_amd_$lib.so; fi
      out=gpurun_out/ab_${TAG}_${name}_${lib}_$i.json
      timeout -k 10 200 python bench.py --cpu-baseline 0 --steps $STEPS --warmup $WARM $args > $out || exit 1
      python -c "import json; d=json.load(open('$out')); print('$lib', '$name', round(d['value']/1e6,1), 'Mhops/s', round(d['roofline']['kernel_ms'],2), 'ms', 'hops/launch', d['roofline']['hops_per_launch'])"
    done
  done
done
